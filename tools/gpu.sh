#!/bin/bash
# One launcher for every GPU-box session (replaces the per-session tools/gpu_r0*.sh scripts).
# usage (through gpurun):  bash tools/gpu.sh <tag> <recipe> [recipe ...]
# Each recipe runs under its own time limit; the first failure ends the call (no retries).
# Outputs go under gpurun_out/<tag>/.
#   suite      pytest -m gpu (one process)          smoke     __graft_entry__.smoke()
#   bench      default bench line (20/5 steps)      host      same, --run-mode host
#   findstep   the find step on this GPU, written as a tune table (commit it as profiles/<tag>_tune_table.json)
#   copytrace  rocprofv3 memory-copy trace of bench.py's traced steps (graph mode), with one HSA
#              runtime in the process (tools/rocprof_one_hsa.sh), summarised per step
#   copytracetorch control: a torch-only process under plain rocprofv3 --memory-copy-trace (two HSA
#              runtimes: the completion callbacks time out after 30 s and no copy is recorded)
#   copytraceprobe  rocprofv3 memory-copy trace of tools/probe_copies (torch-free; bench under it crashes at exit)
#   copyprobe  the step's 233 record copies isolated: host-issued, graph chains, packed chunks (tools/probe_copies)
#   prof       rocprofv3 kernel-trace --stats of the default bench (compute + traced steps)
#   pmc        the PMC HBM-traffic / stall passes (tools/pmc.sh)
#   layers     rocprofv3 kernel trace of compute-only steps (per-layer durations)
#   filesink   bench --sink file, overlapped and serial     filesweep  file sink writer shapes
#   realized   realized relay.quantize ResNet-50 trace rate (tools/realized_times.py)
#   gloo2      2-rank rehearsal on one GPU (gloo collectives; both ranks' records cross one PCIe link)
#   hostmem    host DRAM write / read bandwidth of the GPU's NUMA node, alone and beside a traced bench
#   tests:<k>  pytest -m gpu -k <k>               file:<path>  pytest -m gpu of one test file
# BARGS="..." is appended to every bench.py command line of bench / findstep / prof / pmc / layers
# (e.g. BARGS="--model resnet18 --tune-table <table>" for BASELINE configs 3 and 5).
set -o pipefail
export TMPDIR=/tmp
T=${1:?tag}
shift
O=gpurun_out/$T
mkdir -p "$O"
run() {  # run <seconds> <log> <cmd...>
  local secs=$1 log=$2
  shift 2
  echo "[$(date +%T)] $*" | tee -a "$O/steps.log"
  timeout -k 10 "$secs" "$@" > "$O/$log" 2>&1
  local rc=$?
  echo "[$(date +%T)] rc=$rc" | tee -a "$O/steps.log"
  if [ $rc -ne 0 ]; then tail -30 "$O/$log"; exit $rc; fi
}
for r in "$@"; do
  case "$r" in
    suite) run 900 suite.log python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) run 300 smoke.log python3 -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 400 bench.json python3 -u bench.py --gpus 1 --steps 20 --warmup 5 $BARGS ;;
    findstep) run 400 bench_find.json python3 -u bench.py --gpus 1 --steps 5 --warmup 2 --skip-cpu \
        --tune-table none --write-tune-table "$O/tune_table.json" --tune-report "$O/find_step.json" $BARGS ;;
    host) run 400 bench_host.json python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu --run-mode host ;;
    copytrace)
      run 400 copytrace.log bash tools/rocprof_one_hsa.sh --memory-copy-trace --kernel-trace --stats \
        --output-format csv -d "$O/copy" -o run -- python3 -u bench.py --steps 3 --warmup 1 --skip-cpu \
        --copy-trace "$O/copy_trace.json" &&
      python3 tools/bench_copy_trace.py "$O/copy" "$O/copy_trace.json" "$O/bench_copy_trace.json" > /dev/null ;;
    copytracetorch)  # control: torch alone under plain rocprofv3 (two HSA runtimes in the process)
      run 300 copytrace_torch.log rocprofv3 --memory-copy-trace --stats --output-format csv -d "$O/copy_torch" \
        -o run -- python3 -u tools/probe_torch_copies.py ;;
    copytraceprobe) run 300 copytrace_probe.log rocprofv3 --memory-copy-trace --stats --output-format csv \
        -d "$O/copy_probe" -o run -- ./tools/probe_copies tools/resnet50_b64_record_sizes.txt 1 ;;
    copyprobe) run 300 copyprobe.jsonl ./tools/probe_copies tools/resnet50_b64_record_sizes.txt 3 ;;
    prof) run 400 prof.log rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
        python3 -u bench.py --skip-cpu $BARGS ;;
    pmc) run 900 pmc.log bash tools/pmc.sh "$O/pmc" "$O/pmc/summary.json" $BARGS ;;
    layers) run 400 layers.log rocprofv3 --kernel-trace --output-format csv -d "$O/layers" -o run -- \
        python3 -u bench.py --steps 3 --warmup 1 --skip-cpu --no-trace $BARGS ;;
    filesink)
      (df -hT /tmp . ; cat /proc/mounts) > "$O/mounts.txt" 2>&1
      run 600 bench_file.json python3 -u bench.py --gpus 1 --steps 10 --warmup 3 --skip-cpu --sink file --out-dir /tmp
      run 600 bench_file_overlap.json python3 -u bench.py --gpus 1 --steps 10 --warmup 3 --skip-cpu --sink file \
        --out-dir /tmp --file-overlap on
      run 600 bench_file_serial.json python3 -u bench.py --gpus 1 --steps 10 --warmup 3 --skip-cpu --sink file \
        --out-dir /tmp --file-overlap off ;;
    filesweep)
      # writer shapes with the overlapped sink: threads, piece size, buffered
      for v in "TK_WRITE_THREADS=1" "TK_WRITE_THREADS=2" "TK_WRITE_THREADS=8" "TK_WRITE_PIECE_MB=256" \
               "TK_WRITE_THREADS=2 TK_WRITE_PIECE_MB=256" "TK_WRITE_BUFFERED=1"; do
        tag=$(echo "$v" | tr ' =' '__')
        run 300 "bench_file_$tag.json" env $v python3 -u bench.py --gpus 1 --steps 8 --warmup 2 --skip-cpu \
          --sink file --out-dir /tmp
      done ;;
    realized) run 600 realized.log python3 -u tools/realized_times.py ;;
    splitlayers) run 400 splitlayers.log rocprofv3 --kernel-trace --output-format csv -d "$O/splitlayers" -o run -- \
        python3 -u bench.py --steps 3 --warmup 1 --skip-cpu --no-trace --tune-table profiles/r04_split_probe_table.json ;;
    gloo2) run 600 bench_2rank_gloo.json python3 -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 ;;
    hostmem)
      # host DRAM bandwidth of the GPU's NUMA node, alone and while a traced bench writes its image
      node=$(python3 -c 'import sys; sys.path.insert(0, "."); from tachikoma_amd import shard; print(shard.pci_numa_node(shard.gpu_pci_address(0)))')
      echo "gpu numa node $node" | tee -a "$O/steps.log"
      run 120 hostmem_alone8.jsonl ./tools/probe_hostmem "$node" 8 3 256
      run 120 hostmem_alone14.jsonl ./tools/probe_hostmem "$node" 14 3 256
      # the bench's timed region (250 steps, ~33 s) starts a few seconds after its "trace image" line
      (timeout -k 10 400 python3 -u bench.py --steps 250 --warmup 3 --skip-cpu > "$O/bench_beside_probe.json" \
        2> "$O/bench_beside_probe.err"; echo "bench rc=$?" >> "$O/steps.log") &
      bpid=$!
      for i in $(seq 1 120); do grep -q "trace image" "$O/bench_beside_probe.err" 2>/dev/null && break; sleep 1; done
      sleep 5
      run 120 hostmem_beside_bench.jsonl ./tools/probe_hostmem "$node" 8 6 256
      wait $bpid ;;
    file:*) f=${r#file:}; run 900 "pytest_$(basename "$f" .py).log" python3 -u -m pytest "$f" -m gpu -x -v --timeout 300 \
        --timeout-method thread ;;
    tests:*) run 900 "tests_${r#tests:}.log" python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread -k "${r#tests:}" ;;
    *) echo "unknown recipe $r"; exit 2 ;;
  esac
done
