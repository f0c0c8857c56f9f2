set -o pipefail
# r02o: BN=256 for K <= 256 + med3 clamps + degenerate clip bounds: op parity, ResNet parity, A/B, bench
mkdir -p gpurun_out/r02o
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02o/ops.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py -x -q -k "resnet" --timeout 300 --timeout-method thread > gpurun_out/r02o/models.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_BN256": "0"}, {"TK_BN256_KMAX": "512"}]' "14" 6 > gpurun_out/r02o/ab.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/r02o/bench.json 2> gpurun_out/r02o/bench.err
