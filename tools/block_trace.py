"""Kernel durations of a `tools/bench_block.py` run under `rocprofv3 --kernel-trace`: the event
timing of bench_block includes host launch time whenever the host is slower than the kernel, the
trace does not.  Launch order is layer -> rep -> config -> (1 + iters) calls.

usage: python tools/block_trace.py <rocprof dir> <n_configs> [reps] [iters]"""
import csv
import glob
import os
import sys

FAMS = ("gemm_i8_kernel", "direct_conv_kernel", "conv_img_kernel", "conv_pf_kernel")


def main(d, ncfg, reps=3, iters=20):
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if any(f in r["Kernel_Name"] for f in FAMS)]
    per_layer = reps * ncfg * (1 + iters)
    nl = len(ks) // per_layer
    print(f"source: {os.path.relpath(path)}; {len(ks)} block launches = {nl} layers x {reps} reps x {ncfg} configs "
          f"x {1 + iters} calls")
    for li in range(nl):
        lay = ks[li * per_layer:(li + 1) * per_layer]
        cols = []
        for c in range(ncfg):
            durs, gaps = [], []
            for rp in range(reps):
                base = (rp * ncfg + c) * (1 + iters)
                seg = lay[base + 1:base + 1 + iters]
                durs += [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seg]
                gaps += [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(seg, seg[1:])]
            durs.sort()
            gaps.sort()
            cols.append(f"{durs[len(durs) // 2]:7.1f} us (gap {gaps[len(gaps) // 2]:5.1f})")
        name = lay[0]["Kernel_Name"].split("(")[0].replace("void tk::", "")
        print(f"layer {li:2d}  " + "  ".join(cols) + f"   {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), *(int(a) for a in sys.argv[3:]))
