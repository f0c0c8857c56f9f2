set -o pipefail
# r03g: true kernel durations (rocprofv3 kernel trace) of the layer microbenchmark and of the
# network's compute-only steps, with launch gaps; per-dispatch PMC of the residual-join layers
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
L="3x3 256->256 14,3x3 512->512 7,1x1 1024->256 14,1x1 256->1024 14,1x1 512->2048 7,1x1 2048->512 7,ds 1x1 512->1024,res 1x1 128->512 28,res 1x1 64->256 56"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03g/blk -o run -- python3 -u tools/bench_block.py '[{}, {"TK_IMG": "0"}]' "$L" 3 > gpurun_out/r03g/blk.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03g/net -o run -- python3 -u bench.py --no-trace --skip-cpu --steps 5 --warmup 2 > gpurun_out/r03g/net.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY --kernel-include-regex "gemm_i8_kernel|conv_img_kernel" --output-format csv -d gpurun_out/r03g/pmc1 -o run -- python3 -u tools/bench_block.py '[{}]' "res 1x1 256->1024 14,1x1 256->1024 14,res 1x1 128->512 28,1x1 64->256 56,res 1x1 64->256 56" 1 > gpurun_out/r03g/pmc1.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_debug_executor.py tests/test_gpu_realize.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03g/debug_tests.log 2>&1
