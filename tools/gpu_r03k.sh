set -o pipefail
# r03k3: do the waves' epilogues run in lockstep (compute bursts, then store bursts)?  Odd waves
# start the walk late by TK_IMG_SKEW s_sleep units (ablation build)
mkdir -p gpurun_out/r03k
export TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so
timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_IMG_SKEW": "2"}, {"TK_IMG_SKEW": "4"}, {"TK_IMG_SKEW": "8"}, {"TK_IMG_SKEW": "16"}, {"TK_IMG_SKEW": "32"}]' "1x1 128->512 28,1x1 256->1024 14,res 1x1 256->1024 14" 3 > gpurun_out/r03k/skew.txt 2>&1
