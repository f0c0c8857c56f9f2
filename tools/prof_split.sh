#!/bin/bash
# Kernel durations (rocprofv3 kernel trace) of the conv block on selected layer shapes,
# one process per (shape, TK_ABLATE config): tools/bench_block.py's own event timing
# includes the host launch path, which hides kernels shorter than ~12 us.
# Needs the ablation build: python tachikoma_amd/build.py --ablation
# usage: tools/prof_split.sh <outdir> "<shape filters, ;-separated>" "<ablate flags, space-separated>"
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ps}
SHAPES=${2:-"3x3 512;2048->512;3x3 256;1024->256;3x3 128"}
FLAGS=${3:-"0 4 384 512"}
mkdir -p "$OUT"
IFS=';' read -ra SH <<< "$SHAPES"
for sh in "${SH[@]}"; do
  for ab in $FLAGS; do
    tag=$(echo "$sh" | tr -c 'a-zA-Z0-9' '_')_$ab
    TK_LIB_PATH=tachikoma_amd/_ab/libtachikoma_ablate.so TK_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$tag" -o run -- \
        python3 tools/bench_block.py '[{}]' "$sh" > "$OUT/$tag.log" 2>&1 || exit 1
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys
for d in sorted(glob.glob(sys.argv[1] + '/*/')):
    rows = [r for r in csv.DictReader(open(d + 'run_kernel_stats.csv')) if 'gemm_i8' in r['Name']]
    print(d.rstrip('/').split('/')[-1].ljust(24), '  '.join(f"{r['Name'].split('<')[1].split('>')[0]}: {float(r['AverageNs'])/1e3:6.1f}us" for r in rows))
PY
