set -o pipefail
# r03p3: two workgroups per CU forced (TK_IMG_TWO=2) with the first round staggered (TK_IMG_SKEW):
# do one workgroup's record stores then overlap the other's K loop?
mkdir -p gpurun_out/r03p
export TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so
timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_IMG_TWO": "2"}, {"TK_IMG_TWO": "2", "TK_IMG_SKEW": "4"}, {"TK_IMG_TWO": "2", "TK_IMG_SKEW": "8"}, {"TK_IMG_TWO": "2", "TK_ABLATE": "2"}]' "1x1 128->512 28,res 1x1 128->512 28,1x1 256->1024 14" 3 > gpurun_out/r03p/two_stagger.txt 2>&1
