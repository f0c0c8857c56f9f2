set -o pipefail
# r03b: D2H ceiling probes (1/2/4/8 SDMA streams, chunked, copy kernel into host-mapped memory; with
# and without SDMA), slow-writer trace-job digest test, 2-rank gloo rehearsal of the complete N>1 line
mkdir -p gpurun_out/r03b
timeout -k 10 120 ./tools/probe_d2h 1024 5 > gpurun_out/r03b/probe_d2h.jsonl 2>&1 &&
HSA_ENABLE_SDMA=0 timeout -k 10 120 ./tools/probe_d2h 1024 5 > gpurun_out/r03b/probe_d2h_nosdma.jsonl 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_trace_job.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03b/trace_job.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/r03b/bench_2rank.json 2> gpurun_out/r03b/bench_2rank.err &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err
