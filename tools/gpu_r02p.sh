set -o pipefail
# r02p: full GPU suite, bench line, rocprofv3 kernel stats and PMC passes of the current kernels
mkdir -p gpurun_out/r02p
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02p/gputest.log 2>&1 &&
bash tools/refresh_profiles.sh r02p
