set -o pipefail
# r03h: image-tile plans for 28x28 planes / 64-channel stages / two workgroups per CU, the
# find step (tk_module_tune): every-algo parity, then the bench with the per-node kernel report
export TMPDIR=/tmp
mkdir -p gpurun_out/r03h
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 300 --timeout-method thread -k "algo or img or patch or halo" > gpurun_out/r03h/ops.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --tune-report gpurun_out/r03h/tune.json > gpurun_out/r03h/bench.json 2> gpurun_out/r03h/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03h/net -o run -- python3 -u bench.py --no-trace --skip-cpu --steps 5 --warmup 2 > gpurun_out/r03h/net.log 2>&1
