set -o pipefail
# the driver's GPU commands at the final library (64-channel 3x3 stages): smoke() and the whole -m gpu suite
export TMPDIR=/tmp
mkdir -p gpurun_out/r03fin5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03fin5/smoke.log 2>&1 &&
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03fin5/gputest.log 2>&1
