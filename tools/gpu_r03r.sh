set -o pipefail
# r03r: graph vs host-issued traced steps on whatever box this is (slow-host boxes appear ~1 in 3)
export TMPDIR=/tmp
mkdir -p gpurun_out/r03r
T=$(date +%s)
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --skip-cpu --run-mode graph > gpurun_out/r03r/graph_$T.json 2> gpurun_out/r03r/graph_$T.err &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --skip-cpu --run-mode host > gpurun_out/r03r/host_$T.json 2> gpurun_out/r03r/host_$T.err
