set -o pipefail
# r02g: patch-tile kernel (1x1 + 3x3, sub-tile loop, residual joins): parity, A/B vs im2col kernel, bench
mkdir -p gpurun_out/r02g
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q --timeout 120 --timeout-method thread > gpurun_out/r02g/ops.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py -q -k "resnet" --timeout 300 --timeout-method thread > gpurun_out/r02g/models.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_PATCH": "0"}, {"TK_ABLATE": "4"}]' "" 6 > gpurun_out/r02g/patch_ab.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/r02g/bench.json 2> gpurun_out/r02g/bench.err
