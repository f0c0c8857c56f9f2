set -o pipefail
# r03c: image-tile conv kernel (tk_conv_img.hip): parity of its cases and of the other block paths,
# ResNet-50 / ResNet-18 model parity, per-layer A/B against the im2col kernel (ablation build), bench
mkdir -p gpurun_out/r03c
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v -k "img" --timeout 120 --timeout-method thread > gpurun_out/r03c/img.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03c/ops.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03c/models.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_block.py "[{}]" "" 3 > gpurun_out/r03c/layers.txt 2>&1 &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03c/bench.json 2> gpurun_out/r03c/bench.err
