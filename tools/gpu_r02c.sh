set -o pipefail
# r02c: residual-join cost decomposition; new GPU tests (ingest, trace job); file sink bench
mkdir -p gpurun_out/r02c
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py \
  '[{}, {"TK_ABLATE": "8192"}, {"TK_ABLATE": "16384"}, {"TK_ABLATE": "24576"}, {"TK_ABLATE": "4"}]' \
  "1x1 64->256,1x1 128->512,1x1 256->1024,1x1 512->2048" > gpurun_out/r02c/res_ablate.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_trace_job.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02c/newtests.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --sink file --out-dir /tmp/tk_sink --skip-cpu > gpurun_out/r02c/bench_file.json 2> gpurun_out/r02c/bench_file.err
