set -o pipefail
# r03j: image-tile epilogue software-pipelined: parity, then the bench's find-step report
export TMPDIR=/tmp
mkdir -p gpurun_out/r03j
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 300 --timeout-method thread -k "algo or img" > gpurun_out/r03j/ops.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --tune-report gpurun_out/r03j/tune.json > gpurun_out/r03j/bench.json 2> gpurun_out/r03j/bench.err
