"""Split a rocprofv3 kernel trace of ``bench.py`` into its traced and compute-only steps.

rocprofv3 --stats averages every dispatch of a kernel over the whole command.  The
bench runs traced steps (D2H capture concurrent with the kernels) and compute-only
steps (kernels alone; the roofline is measured on these), so this prints per-kernel
average durations per phase from <dir>/run_kernel_trace.csv.  A step = one run of the
node list (block-kernel dispatches per step = all of them / runs); it is "traced" when device copy
kernels ran inside its window.

usage: python tools/prof_phases.py <rocprof dir> [runs]
runs = steps the bench executed: warmup + 3 x steps + 1 (default command: 2 + 15 + 1 = 18)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, runs=18):
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    fams = ("gemm_i8_kernel", "conv_img_kernel", "direct_conv_kernel", "conv_pf_kernel", "dense_tile_kernel",
            "dense_slices_epilogue_kernel")
    gemm = [r for r in rows if any(f in r["Kernel_Name"] for f in fams)]
    # launches per step = the period of the kernel-name sequence (the module's find step launches
    # candidate kernels first: drop everything before the first whole period from the end)
    names = [r["Kernel_Name"] for r in gemm]
    launches = next((p for p in range(8, len(names) // 2 + 1) if names[-p:] == names[-2 * p:-p]), len(gemm) // runs)
    n_steps = 1
    while (n_steps + 1) * launches <= len(names) and \
            names[-(n_steps + 1) * launches:-n_steps * launches] == names[-launches:]:
        n_steps += 1
    gemm = gemm[len(gemm) - n_steps * launches:]
    # traced steps: blit copy kernels (per-record copies under the profiler) or the packed capture's
    # gather kernels (pack_records_kernel, one per image chunk)
    copies = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
              if "copyBuffer" in r["Kernel_Name"] or "pack_records_kernel" in r["Kernel_Name"]]
    phases = defaultdict(lambda: defaultdict(list))
    steps = defaultdict(int)
    for i in range(0, len(gemm) - launches + 1, launches):
        step = gemm[i:i + launches]
        t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
        # a traced step overlaps its ~150 record copies (or its 8 chunk gathers); stray single
        # copies do not count
        traced = sum(1 for s, e in copies if s < t1 and e > t0) >= 4
        ph = "traced" if traced else "compute-only"
        steps[ph] += 1
        for r in step:
            phases[ph][r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"source: {os.path.relpath(path)}; {launches} block-kernel launches per step")
    for ph in ("compute-only", "traced"):
        if ph not in phases:
            continue
        tot = sum(sum(v) for v in phases[ph].values())
        n = sum(len(v) for v in phases[ph].values())
        print(f"[{ph}] {steps[ph]} steps, block kernels {tot / steps[ph] / 1e6:.3f} ms/step, "
              f"average launch {tot / n / 1e3:.2f} us")
        for k, v in sorted(phases[ph].items()):
            print(f"    {k}: calls {len(v)}, avg {sum(v) / len(v) / 1e3:.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 18)
