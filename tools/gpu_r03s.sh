set -o pipefail
# r03s2: graph-mode record copies as memcpy nodes in 1 / 2 / 4 parallel chains, beside host-issued
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_module.py -m gpu -x -v --timeout 200 --timeout-method thread -k graph > gpurun_out/r03s/test.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --skip-cpu --graph-copies 5 > gpurun_out/r03s/chains1.json 2> gpurun_out/r03s/chains1.err &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --skip-cpu --graph-copies 2 > gpurun_out/r03s/chains2.json 2> gpurun_out/r03s/chains2.err &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --skip-cpu --graph-copies 4 > gpurun_out/r03s/chains4.json 2> gpurun_out/r03s/chains4.err &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --skip-cpu --run-mode host > gpurun_out/r03s/host.json 2> gpurun_out/r03s/host.err
