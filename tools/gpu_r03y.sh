set -o pipefail
# PMC passes at HEAD with the persistent kernel in the counted families, the new 64-channel-stage
# parity cases
export TMPDIR=/tmp
mkdir -p gpurun_out/r03y
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 250 --timeout-method thread -k "every_algo" > gpurun_out/r03y/ops.log 2>&1 &&
bash tools/pmc.sh gpurun_out/r03y/pmc gpurun_out/r03y/pmc/summary.json > gpurun_out/r03y/pmc.log 2>&1
