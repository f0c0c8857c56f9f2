#!/bin/bash
# One GPU call that regenerates the round's evidence: the default bench line, a rocprofv3
# kernel-trace/stats profile of the same command, and the PMC HBM-traffic passes.
# usage: bash tools/refresh_profiles.sh <tag>   (outputs under gpurun_out/<tag>_*)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- \
    python3 bench.py --skip-cpu > gpurun_out/${T}_prof.log 2>&1 || exit 1
bash tools/pmc.sh gpurun_out/${T}_pmc gpurun_out/${T}_pmc/summary.json > gpurun_out/${T}_pmc.log 2>&1 || exit 1
