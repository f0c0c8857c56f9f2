set -o pipefail
# r03t: default graph copies (4 chains): graph-replay parity, trace-job suite, bench
export TMPDIR=/tmp
mkdir -p gpurun_out/r03t
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_module.py tests/test_gpu_trace_job.py tests/test_gpu_models.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03t/tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03t/bench.json 2> gpurun_out/r03t/bench.err
