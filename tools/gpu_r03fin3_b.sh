set -o pipefail
# round-3 final evidence (at HEAD: persistent-kernel algos, 64-channel 3x3 stages), part 2: the driver's bench line, rocprofv3 kernel trace + stats of the
# default bench command, the PMC HBM-traffic passes
export TMPDIR=/tmp
mkdir -p gpurun_out/r03fin3
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --tune-report gpurun_out/r03fin3/tune.json > gpurun_out/r03fin3/bench.json 2> gpurun_out/r03fin3/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03fin3/prof -o run -- python3 bench.py --skip-cpu > gpurun_out/r03fin3/prof.log 2>&1 &&
bash tools/pmc.sh gpurun_out/r03fin3/pmc gpurun_out/r03fin3/pmc/summary.json > gpurun_out/r03fin3/pmc.log 2>&1
