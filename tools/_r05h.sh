set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
step() { local secs=$1 log=$2; shift 2; echo "[$(date +%T)] $*" >> $O/steps.log; timeout -k 10 $secs "$@" > $O/$log 2>&1; local rc=$?; echo "[$(date +%T)] rc=$rc" >> $O/steps.log; return $rc; }
step 900 suite.log python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
step 300 smoke.log python3 -u -c "import __graft_entry__ as g; g.smoke()" &&
step 400 bench_find.json python3 -u bench.py --gpus 1 --steps 5 --warmup 2 --skip-cpu --tune-table none --write-tune-table $O/tune_table.json --tune-report $O/find_step.json &&
step 400 bench.json python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --tune-table $O/tune_table.json --copy-trace $O/copy_trace.json &&
step 400 prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --skip-cpu --tune-table $O/tune_table.json &&
step 400 layers.log rocprofv3 --kernel-trace --output-format csv -d $O/layers -o run -- python3 -u bench.py --steps 3 --warmup 1 --skip-cpu --no-trace --tune-table $O/tune_table.json &&
step 300 copytrace_torch.log rocprofv3 --memory-copy-trace --stats --output-format csv -d $O/copy_torch -o run -- python3 -u tools/probe_torch_copies.py
