set -o pipefail
# r03n: traced steps as one replayed HIP graph (copy kernels / memcpy nodes) vs host-issued kernels
# + copies, same box, twice each; graph-replay parity first
export TMPDIR=/tmp
mkdir -p gpurun_out/r03n
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_module.py -m gpu -x -v --timeout 300 --timeout-method thread -k "graph or traced" > gpurun_out/r03n/tests.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/r03n/graph_$i.json 2> gpurun_out/r03n/graph_$i.err &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --skip-cpu --graph-memcpy > gpurun_out/r03n/graphmc_$i.json 2> gpurun_out/r03n/graphmc_$i.err &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --skip-cpu --no-graph > gpurun_out/r03n/plain_$i.json 2> gpurun_out/r03n/plain_$i.err || exit 1
done
