set -o pipefail
# r03m: module runs as replayed HIP graphs (tk_module_run_graph): parity of traced runs, then the bench
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_module.py tests/test_gpu_models.py tests/test_debug_executor.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03m/tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --tune-report gpurun_out/r03m/tune.json > gpurun_out/r03m/bench.json 2> gpurun_out/r03m/bench.err
