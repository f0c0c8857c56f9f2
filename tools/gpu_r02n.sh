set -o pipefail
# r02n: lean flat epilogue: parity, A/B of the 14x14 / 7x7 layers
mkdir -p gpurun_out/r02n
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -k "bn256 or block or resid" --timeout 120 --timeout-method thread > gpurun_out/r02n/ops.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_BN256": "0"}, {"TK_ABLATE": "32768"}, {"TK_ABLATE": "2"}, {"TK_ABLATE": "65536"}]' "14,7" 6 > gpurun_out/r02n/ab.txt 2>&1
