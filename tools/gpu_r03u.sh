set -o pipefail
# r03u: the N>1 path at HEAD (find step + graph-mode traced steps) rehearsed with 2 ranks on one GPU
# over gloo, and the file sink in graph mode
export TMPDIR=/tmp
mkdir -p gpurun_out/r03u
timeout -k 10 500 python3 -u bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/r03u/bench_2rank.json 2> gpurun_out/r03u/bench_2rank.err &&
timeout -k 10 500 python3 -u bench.py --sink file --steps 5 --warmup 2 --skip-cpu --out-dir /tmp/tk_r03u > gpurun_out/r03u/bench_file.json 2> gpurun_out/r03u/bench_file.err
