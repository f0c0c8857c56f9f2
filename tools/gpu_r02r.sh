set -o pipefail
# r02r: 128-row tiles on the 14x14 3x3 layers: op + model parity, bench
mkdir -p gpurun_out/r02r
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02r/ops.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py -x -q -k "resnet" --timeout 300 --timeout-method thread > gpurun_out/r02r/models.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/r02r/bench.json 2> gpurun_out/r02r/bench.err
