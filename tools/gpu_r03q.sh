set -o pipefail
# r03q: store-only probe at forced occupancy (dynamic LDS), plain vs nontemporal
mkdir -p gpurun_out/r03q
timeout -k 10 120 ./tools/_probe_store4 > gpurun_out/r03q/probe_store4.txt 2>&1
