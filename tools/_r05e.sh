set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
AB=tachikoma_amd/_ab/libtachikoma_ablate.so
step() { local secs=$1 log=$2; shift 2; echo "[$(date +%T)] $*" >> $O/steps.log; timeout -k 10 $secs "$@" > $O/$log 2>&1; local rc=$?; echo "[$(date +%T)] rc=$rc" >> $O/steps.log; return $rc; }
step 200 abl_7.txt env TK_LIB_PATH=$AB python3 -u tools/bench_block.py "$(python3 tools/abl_r05.py 2)" "3x3 512->512 7" &&
step 200 abl_14.txt env TK_LIB_PATH=$AB python3 -u tools/bench_block.py "$(python3 tools/abl_r05.py 1)" "3x3 256->256 14" &&
step 600 ops.log python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_module.py -m gpu -x -q --timeout 300 --timeout-method thread -k "every_algo or conv_img or conv3x3 or image or copy_trace or graph_replay" &&
step 400 bench_find.json python3 -u bench.py --gpus 1 --steps 10 --warmup 3 --skip-cpu --tune-table none --write-tune-table $O/tune_table.json --tune-report $O/find_step.json --copy-trace $O/copy_trace.json &&
step 400 layers.log rocprofv3 --kernel-trace --output-format csv -d $O/layers -o run -- python3 -u bench.py --steps 3 --warmup 1 --skip-cpu --no-trace --tune-table $O/tune_table.json &&
step 300 smoke.log python3 -u -c "import __graft_entry__ as g; g.smoke()" &&
step 300 copytrace_torch.log rocprofv3 --memory-copy-trace --stats --output-format csv -d $O/copy_torch -o run -- python3 -u tools/probe_torch_copies.py
