set -o pipefail
# 64-channel K stages for the 3x3 image-tile kernel: every-algo parity, then the bench's find step
export TMPDIR=/tmp
mkdir -p gpurun_out/r03x
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread -k "every_algo or conv_block" > gpurun_out/r03x/ops.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --tune-report gpurun_out/r03x/tune.json > gpurun_out/r03x/bench.json 2> gpurun_out/r03x/bench.err
