set -o pipefail
# round-3 final bench line (the driver's command) with the find-step report
export TMPDIR=/tmp
mkdir -p gpurun_out/r03fin2
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --tune-report gpurun_out/r03fin2/tune_c.json > gpurun_out/r03fin2/bench_c.json 2> gpurun_out/r03fin2/bench_c.err
