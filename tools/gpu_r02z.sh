set -o pipefail
# r02z: 128-row tiles with 128-byte K stages on the 14x14 3x3 layers: parity (ablation build) and A/B
mkdir -p gpurun_out/r02z
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so TK_WIDE_MT2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "mt2_256" --timeout 120 --timeout-method thread > gpurun_out/r02z/ops.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_WIDE_MT2": "1"}]' "3x3 256" 6 > gpurun_out/r02z/ab.txt 2>&1
