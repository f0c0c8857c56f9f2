set -o pipefail
# r03l: im2col-kernel variants on the 56x56 / 28x28 layers (ablation build, TK_IMG=0): XCD tile
# order, nontemporal vs plain record stores, ring depth, 128-row tiles, 256-column rows
mkdir -p gpurun_out/r03l
export TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so
timeout -k 10 400 python -u tools/bench_block.py '[{"TK_IMG": "0"}, {"TK_IMG": "0", "TK_XCD": "1"}, {"TK_IMG": "0", "TK_XCD": "2"}, {"TK_IMG": "0", "TK_FASTEPI": "2"}, {"TK_IMG": "0", "TK_FASTEPI": "1"}, {"TK_IMG": "0", "TK_RING": "4"}, {"TK_IMG": "0", "TK_MT2": "1"}, {"TK_IMG": "0", "TK_BN256_ROWS": "1"}]' "stem,1x1 64->256 56,1x1 256->64 56,3x3 64->64 56,3x3 128->128 28,1x1 512->256 s2,res 1x1 64->256 56,res 1x1 128->512 28,1x1 128->512 28" 3 > gpurun_out/r03l/im2col_variants.txt 2>&1
