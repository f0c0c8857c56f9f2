set -o pipefail
# r03e: image-tile kernel (deeper ring, incremental epilogue walk, late residual DMA), tk_pad, per-channel
# float multiply (rhs_kind 3), the reference's own Relay-text models quantized and traced, O_DIRECT
# trace writer with the file-sink probe, per-layer times and the default bench line
mkdir -p gpurun_out/r03e
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "img or pad or halo or patch or resid or bn256 or block" --timeout 120 --timeout-method thread > gpurun_out/r03e/ops.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_realize.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03e/ingest.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_block.py "[{}]" "" 3 > gpurun_out/r03e/layers.txt 2>&1 &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03e/bench.json 2> gpurun_out/r03e/bench.err &&
timeout -k 10 400 python3 -u bench.py --sink file --steps 3 --warmup 1 --skip-cpu --out-dir /tmp/tk_sink > gpurun_out/r03e/bench_file.json 2> gpurun_out/r03e/bench_file.err
