set -o pipefail
# r02b: decomposition of the small-grid conv blocks (14x14 / 7x7 stages) by main-loop ablations
mkdir -p gpurun_out/r02b
export TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so
timeout -k 10 300 python -u tools/bench_block.py \
  '[{}, {"TK_ABLATE": "4"}, {"TK_ABLATE": "384"}, {"TK_ABLATE": "512"}, {"TK_ABLATE": "2048"}, {"TK_ABLATE": "4096"}, {"TK_ABLATE": "388"}, {"TK_ABLATE": "2436"}, {"TK_ABLATE": "6532"}, {"TK_ABLATE": "7044"}, {"TK_WIDE": "0"}]' \
  "3x3 256,3x3 512,1x1 1024,1x1 256->1024,1x1 2048,1x1 512->2048,3x3 128,3x3 64" > gpurun_out/r02b/ablate.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02b/kt -o run -- python3 tools/bench_block.py '[{}]' "3x3 256,3x3 512,1x1 1024" > gpurun_out/r02b/kt.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex gemm_i8 --output-format csv -d gpurun_out/r02b/pmc1 -o run -- python3 tools/bench_block.py '[{}]' "3x3 256" > gpurun_out/r02b/pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex gemm_i8 --output-format csv -d gpurun_out/r02b/pmc2 -o run -- python3 tools/bench_block.py '[{}]' "3x3 256" > gpurun_out/r02b/pmc2.log 2>&1
