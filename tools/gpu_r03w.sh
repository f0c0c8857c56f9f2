set -o pipefail
# r03w: persistent im2col kernel with cross-tile prefetch (algos 3 / 4): every-algo parity, then the
# bench with the find step's per-node report (which layers pick it)
export TMPDIR=/tmp
mkdir -p gpurun_out/r03w
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 300 --timeout-method thread -k "algo" > gpurun_out/r03w/ops.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --tune-report gpurun_out/r03w/tune.json > gpurun_out/r03w/bench.json 2> gpurun_out/r03w/bench.err
