#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only — no sys/runtime traces)
# for the fused conv/dense block kernel, on `bench.py --no-trace`.
# usage: tools/pmc.sh <outdir> [extra bench args]
set -o pipefail
OUT=${1:-gpurun_out/pmc}
shift
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-trace $*"
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --kernel-include-regex "gemm_i8_kernel" --output-format csv \
      -d $OUT/pass$i -o run -- $BENCH > $OUT/pass$i.log 2>&1 || { echo "pass $i ($group) failed"; tail -5 $OUT/pass$i.log; exit 1; }
done
echo "pmc done"
