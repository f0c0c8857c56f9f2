set -o pipefail
# r03a: round-3 start: smoke, full GPU suite, default bench line at HEAD
mkdir -p gpurun_out/r03a
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a/smoke.log 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03a/gputest.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
