set -o pipefail
# r03d: image-tile kernel with a deeper ring (runtime slot count), incremental epilogue walk, late
# residual DMA; tk_pad; the reference's own Relay-text models (menangerie) quantized and traced
mkdir -p gpurun_out/r03d
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "img or pad or halo or patch or resid or bn256 or block" --timeout 120 --timeout-method thread > gpurun_out/r03d/ops.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d/ingest.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_block.py "[{}]" "" 3 > gpurun_out/r03d/layers.txt 2>&1 &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03d/bench.json 2> gpurun_out/r03d/bench.err
