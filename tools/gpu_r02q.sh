set -o pipefail
# r02q: 128-row tiles on the 14x14 3x3 / reduce layers; LDS conflict counters without the qnn.add LUTs
mkdir -p gpurun_out/r02q
export TMPDIR=/tmp
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 python -u tools/bench_block.py '[{}, {"TK_MT2": "1"}]' "3x3 256,1024->256,3x3 128,512->128" 6 > gpurun_out/r02q/mt2_ab.txt 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so TK_ABLATE=8192 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "gemm_i8_kernel" --output-format csv -d gpurun_out/r02q/pmc_nolut -o run -- python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-trace > gpurun_out/r02q/pmc_nolut.log 2>&1 &&
TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "gemm_i8_kernel" --output-format csv -d gpurun_out/r02q/pmc_lut -o run -- python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-trace > gpurun_out/r02q/pmc_lut.log 2>&1
