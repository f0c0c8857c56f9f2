set -o pipefail
# run-mode comparison at the final library on one box: graph (default) then host-issued steps
export TMPDIR=/tmp
mkdir -p gpurun_out/r03fin7
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu > gpurun_out/r03fin7/bench_graph.json 2> gpurun_out/r03fin7/bench_graph.err &&
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu --run-mode host > gpurun_out/r03fin7/bench_host.json 2> gpurun_out/r03fin7/bench_host.err
