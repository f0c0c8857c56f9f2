set -o pipefail
# r03i: the residual-join penalty on both kernels (ablation build): default, the qnn.add LUT
# lookups replaced by a plain add (8192), the add record not stored (16384), the residual
# words not loaded (image tiles, 65536), against the same layers without a join
mkdir -p gpurun_out/r03i
export TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so
timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_ABLATE": "8192"}, {"TK_ABLATE": "16384"}, {"TK_ABLATE": "65536"}, {"TK_ABLATE": "24576"}, {"TK_IMG": "0"}, {"TK_IMG": "0", "TK_ABLATE": "8192"}, {"TK_IMG": "0", "TK_ABLATE": "16384"}, {"TK_IMG": "0", "TK_ABLATE": "24576"}]' "res 1x1 128->512 28,1x1 128->512 28,res 1x1 256->1024 14,1x1 256->1024 14,res 1x1 64->256 56,1x1 64->256 56" 3 > gpurun_out/r03i/res_ablate.txt 2>&1
