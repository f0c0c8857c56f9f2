set -o pipefail
# r02h: session baseline: launch floor, bench line, per-layer ablations with fresh output buffers
mkdir -p gpurun_out/r02h
timeout -k 10 120 python tools/probe_launch.py > gpurun_out/r02h/launch.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r02h/bench.json 2> gpurun_out/r02h/bench.err &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py \
  '[{}, {"TK_ABLATE": "4"}, {"TK_ABLATE": "2564"}, {"TK_ABLATE": "2948"}, {"TK_ABLATE": "7044"}]' "" 6 > gpurun_out/r02h/ablate.txt 2>&1
