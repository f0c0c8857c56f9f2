set -o pipefail
# r02f: halo kernel with 6-8 weight steps in flight: parity of the conv-block ops, ablation A/B
mkdir -p gpurun_out/r02f
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q -k "halo or block" --timeout 120 --timeout-method thread > gpurun_out/r02f/ops.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_HALO": "0"}, {"TK_ABLATE": "4"}, {"TK_ABLATE": "128"}, {"TK_ABLATE": "256"}, {"TK_ABLATE": "512"}, {"TK_ABLATE": "644"}, {"TK_ABLATE": "900"}]' "3x3" 6 > gpurun_out/r02f/halo_ab.txt 2>&1
