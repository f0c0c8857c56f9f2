set -o pipefail
# r03o: bench with the submission find step (auto run mode), twice; trace-job suite (uses it too)
export TMPDIR=/tmp
mkdir -p gpurun_out/r03o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_module.py tests/test_gpu_trace_job.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03o/tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --tune-report gpurun_out/r03o/tune.json > gpurun_out/r03o/bench.json 2> gpurun_out/r03o/bench.err
