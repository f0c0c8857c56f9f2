set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 120 python tools/probe_host.py > gpurun_out/r02a/probe.json 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r02a/bench1.json 2> gpurun_out/r02a/bench1.err &&
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --skip-cpu > gpurun_out/r02a/bench2.json 2> gpurun_out/r02a/bench2.err
