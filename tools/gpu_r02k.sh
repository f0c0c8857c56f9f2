set -o pipefail
# r02k: 256-column image tiles (14x14 planes): block parity, ResNet parity, A/B vs 128-column tiles, bench
mkdir -p gpurun_out/r02k
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -k "bn256 or block or resid" --timeout 120 --timeout-method thread > gpurun_out/r02k/ops.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py -x -q -k "resnet" --timeout 300 --timeout-method thread > gpurun_out/r02k/models.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_BN256": "0"}]' "14,7" 6 > gpurun_out/r02k/bn256_ab.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/r02k/bench.json 2> gpurun_out/r02k/bench.err
