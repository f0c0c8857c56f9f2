set -o pipefail
# r02m: where the 14x14 flat epilogue spends its time (store / shadow / group ablations)
mkdir -p gpurun_out/r02m
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_ABLATE": "2"}, {"TK_ABLATE": "3"}, {"TK_ABLATE": "65536"}, {"TK_ABLATE": "65537"}, {"TK_ABLATE": "4"}, {"TK_ABLATE": "24576"}]' "1x1 256->1024 14" 6 > gpurun_out/r02m/ab.txt 2>&1
