set -o pipefail
# r02i: deeper LDS-DMA rings (wide stages at 1 workgroup per CU), library int8 GEMM reference
mkdir -p gpurun_out/r02i
timeout -k 10 120 python tools/probe_intmm.py > gpurun_out/r02i/intmm.txt 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py \
  '[{}, {"TK_RING": "4"}, {"TK_RING": "5"}, {"TK_RING": "4", "TK_WIDE_MAX_TILES": "1024"}]' "" 6 > gpurun_out/r02i/ring.txt 2>&1
