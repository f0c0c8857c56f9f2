set -o pipefail
# D2H ceiling by host-buffer kind (mapped = torch pin_memory's, noncoherent, coherent, write-combined, registered malloc)
mkdir -p gpurun_out/r03d2h
for k in mapped noncoherent coherent writecombined register; do
  timeout -k 10 120 ./tools/probe_d2h 1024 5 $k 0 >> gpurun_out/r03d2h/probe.jsonl 2>&1 || exit 1
done
