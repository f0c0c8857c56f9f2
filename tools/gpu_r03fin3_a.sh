set -o pipefail
# round-3 final evidence (at HEAD with the persistent-kernel algos), part 1: smoke() and the whole -m gpu suite (the driver's commands)
export TMPDIR=/tmp
mkdir -p gpurun_out/r03fin3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03fin3/smoke.log 2>&1 &&
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03fin3/gputest.log 2>&1
