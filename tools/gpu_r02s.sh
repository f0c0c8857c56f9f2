set -o pipefail
# r02s: 256-column row tiles on the 56x56 / 28x28 short-K layers: op + model parity, A/B, bench
mkdir -p gpurun_out/r02s
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02s/ops.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py -x -q -k "resnet" --timeout 300 --timeout-method thread > gpurun_out/r02s/models.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_BN256_ROWS": "0"}]' "64->256 56,128->512 28" 6 > gpurun_out/r02s/ab.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/r02s/bench.json 2> gpurun_out/r02s/bench.err
