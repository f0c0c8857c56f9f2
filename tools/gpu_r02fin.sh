set -o pipefail
# r02fin: round-2 final evidence: smoke, full GPU suite, bench line, rocprofv3 kernel stats, PMC passes
mkdir -p gpurun_out/r02fin
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02fin/smoke.log 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02fin/gputest.log 2>&1 &&
bash tools/refresh_profiles.sh r02fin
