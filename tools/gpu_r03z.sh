set -o pipefail
# find step over 48 candidates per conv block (every image-tile plan of most layers)
export TMPDIR=/tmp
mkdir -p gpurun_out/r03z
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --tune-report gpurun_out/r03z/tune.json > gpurun_out/r03z/bench.json 2> gpurun_out/r03z/bench.err
