#!/bin/bash
# HBM-traffic, stall and MFMA counters for the fused layer-block kernels (gemm_i8_kernel,
# conv_img_kernel, conv_pf_kernel, dense_tile_kernel, and MobileNetV2's dw3x3_kernel /
# direct_conv_kernel), one counter group per rocprofv3 pass, kernel-trace only (no sys/runtime
# traces), on the compute-only bench step (the block kernels are identical with capture on; the
# D2H copies would only add unrelated TCC traffic).
# Pass 6 counts the matrix cores: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over every SIMD),
# SQ_INSTS_VALU_MFMA_I8 (int8 MFMA instructions), SQ_INSTS_VALU_MFMA_MOPS_I8 (int8 matrix ops / 512)
# and GRBM_GUI_ACTIVE (GPU-busy cycles, summed over the 8 XCDs) -- rocprofiler-sdk's MfmaUtil.
# usage: tools/pmc.sh <outdir> <summary.json> [extra bench args]
set -o pipefail
OUT=${1:-gpurun_out/pmc}
JSON=${2:-$OUT/summary.json}
shift 2
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_MFMA_MOPS_I8 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --kernel-include-regex "gemm_i8_kernel|conv_img_kernel|conv_pf_kernel|dense_tile_kernel|dense_slices_epilogue_kernel|dw3x3_kernel|dw_tile_kernel|direct_conv_kernel" --output-format csv \
      -d "$OUT/pass$i" -o run -- python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-trace "$@" \
      > "$OUT/pass$i.log" 2>&1 || { echo "pass $i ($group) failed"; tail -5 "$OUT/pass$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" --json "$JSON" --workload "$*"
