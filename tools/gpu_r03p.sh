set -o pipefail
# r03p2: stagger the first round of image-tile workgroups (TK_IMG_SKEW) so CUs sit in different
# phases (K loop vs epilogue stores): does the chip-wide store time then overlap the K loops?
mkdir -p gpurun_out/r03p
export TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so
timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_IMG_SKEW": "2"}, {"TK_IMG_SKEW": "4"}, {"TK_IMG_SKEW": "8"}, {"TK_IMG_SKEW": "16"}]' "1x1 128->512 28,res 1x1 128->512 28,1x1 256->1024 14,res 1x1 256->1024 14" 3 > gpurun_out/r03p/stagger.txt 2>&1
