set -o pipefail
# final bench lines at HEAD: the driver's N=1 command and a 2-rank gloo rehearsal on one GPU
export TMPDIR=/tmp
mkdir -p gpurun_out/r03fin4
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03fin4/bench.json 2> gpurun_out/r03fin4/bench.err &&
timeout -k 10 500 python3 -u bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/r03fin4/bench_2rank.json 2> gpurun_out/r03fin4/bench_2rank.err
