set -o pipefail
# the same probe in another order (is the first probe of a fresh box slow whatever its buffer kind?)
mkdir -p gpurun_out/r03d2h2
for k in register mapped noncoherent mapped; do
  timeout -k 10 120 ./tools/probe_d2h 1024 5 $k 0 >> gpurun_out/r03d2h2/probe.jsonl 2>&1 || exit 1
done
