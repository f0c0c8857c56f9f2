set -o pipefail
# r02e: halo-tile 3x3 kernel: op parity, model parity, A/B vs the im2col block kernel, bench
mkdir -p gpurun_out/r02e
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q --timeout 120 --timeout-method thread > gpurun_out/r02e/ops.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02e/models.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_HALO": "0"}]' "3x3" 6 > gpurun_out/r02e/halo_ab.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/r02e/bench.json 2> gpurun_out/r02e/bench.err
