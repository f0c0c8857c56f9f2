"""Per-config GPU kernel time of a `tools/bench_block.py ... --marker` run under
`rocprofv3 --kernel-trace --output-format csv`: the launches between consecutive fill-kernel markers
are one config's warm-up call + its timed calls (reps rounds, configs interleaved); a config's time
is the median over its timed calls of the summed durations of the conv-block kernels of one call
(two for split-K plans).  Host launch overhead, which floors bench_block's event timing near 14 us,
is not in these durations.  Usage: python tools/abl_trace.py <kernel_trace.csv> <n_configs> [iters]"""
import csv
import statistics
import sys

FAMS = ("gemm_i8_kernel", "conv_img_kernel", "conv_pf_kernel", "dense_tile_kernel", "dense_slices_epilogue_kernel",
        "direct_conv_kernel", "reduce_kernel", "splitk")


def main(path, n_configs, iters=20):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    groups, cur = [], []
    for r in rows:
        name = r["Kernel_Name"]
        if "FillFunctor" in name or "fill" in name.lower() and "elementwise" in name:
            groups.append(cur)
            cur = []
        elif any(f in name for f in FAMS):
            cur.append(r)
    groups = [g for g in groups if g]  # (setup fills before the first config delimit no launches)
    per = [[] for _ in range(n_configs)]
    names = [set() for _ in range(n_configs)]
    for gi, g in enumerate(groups):
        ci = gi % n_configs
        calls = iters + 1
        if not g or len(g) % calls:
            print(f"group {gi}: {len(g)} kernels, not a multiple of {calls}", file=sys.stderr)
            continue
        k = len(g) // calls
        for c in range(1, calls):  # skip the warm-up call
            d = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in g[c * k:(c + 1) * k]) / 1e3
            per[ci].append(d)
        names[ci].update(r["Kernel_Name"].split("(")[0] for r in g)
    for ci in range(n_configs):
        med = statistics.median(per[ci]) if per[ci] else float("nan")
        print(f"config {ci:2d}: {med:8.2f} us  (n={len(per[ci])})  {sorted(names[ci])}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 20)
