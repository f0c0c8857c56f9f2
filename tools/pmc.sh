#!/bin/bash
# HBM-traffic and stall counters for the fused layer-block kernels (gemm_i8_kernel, conv_img_kernel,
# conv_pf_kernel, dense_tile_kernel), one
# counter group per rocprofv3 pass, kernel-trace only (no sys/runtime traces), on the
# compute-only bench step (the block kernels are identical with capture on; the D2H
# copies would only add unrelated TCC traffic).
# usage: tools/pmc.sh <outdir> <summary.json> [extra bench args]
set -o pipefail
OUT=${1:-gpurun_out/pmc}
JSON=${2:-$OUT/summary.json}
shift 2
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --kernel-include-regex "gemm_i8_kernel|conv_img_kernel|conv_pf_kernel|dense_tile_kernel|dense_slices_epilogue_kernel" --output-format csv \
      -d "$OUT/pass$i" -o run -- python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-trace "$@" \
      > "$OUT/pass$i.log" 2>&1 || { echo "pass $i ($group) failed"; tail -5 "$OUT/pass$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" --json "$JSON" --workload "$*"
