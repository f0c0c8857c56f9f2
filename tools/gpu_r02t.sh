set -o pipefail
# r02t: lean row-crossing flat epilogue (7x7 planes): op + model parity, A/B, bench
mkdir -p gpurun_out/r02t
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02t/ops.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02t/models.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_ABLATE": "131072"}]' " 7" 6 > gpurun_out/r02t/ab.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/r02t/bench.json 2> gpurun_out/r02t/bench.err
