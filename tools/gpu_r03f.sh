set -o pipefail
# r03f: where the image-tile kernel's time goes (ablation build): epilogue / stores / MFMAs / loads
# skipped, ring depth, two workgroups per CU, the im2col kernel (TK_IMG=0) beside it
mkdir -p gpurun_out/r03f
export TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so
timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_IMG": "0"}, {"TK_ABLATE": "4"}, {"TK_ABLATE": "2"}, {"TK_ABLATE": "512"}, {"TK_ABLATE": "128"}, {"TK_ABLATE": "644"}]' "3x3 256->256 14,3x3 512->512 7,1x1 1024->256 14,1x1 256->1024 14,1x1 512->2048 7,1x1 2048->512 7,res 1x1 256->1024 14,res 1x1 512->2048 7,ds 1x1 512->1024" 3 > gpurun_out/r03f/ablate.txt 2>&1 &&
timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_IMG_NS": "3"}, {"TK_IMG_NS": "4"}, {"TK_IMG_TWO": "0"}, {"TK_IMG_R": "32"}, {"TK_IMG_R": "64"}, {"TK_IMG_IPT": "1"}]' "3x3 256->256 14,3x3 512->512 7,1x1 1024->256 14,1x1 256->1024 14,1x1 512->2048 7,1x1 2048->512 7,res 1x1 256->1024 14,res 1x1 512->2048 7,ds 1x1 512->1024" 3 > gpurun_out/r03f/plans.txt 2>&1
