set -o pipefail
export TMPDIR=/tmp
for pad in 0 45000 90000 120000; do
  for sh in "3x3 256" "3x3 128" "1024->256" "256->1024"; do
    tag=$(echo "$sh" | tr -c 'a-zA-Z0-9' '_')_$pad
    TK_LDS_PAD=$pad timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ps4/$tag -o run -- python3 tools/bench_block.py '[{}]' "$sh" > gpurun_out/ps4/$tag.log 2>&1 || exit 1
  done
done
