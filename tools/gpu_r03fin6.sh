set -o pipefail
# 4-rank gloo rehearsal of the N>1 bench path on one GPU (the driver runs N = 2/4/8 over RCCL on a whole node)
export TMPDIR=/tmp
mkdir -p gpurun_out/r03fin6
timeout -k 10 600 python3 -u bench.py --gpus 4 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/r03fin6/bench_4rank.json 2> gpurun_out/r03fin6/bench_4rank.err
