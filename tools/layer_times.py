"""Per-layer kernel durations from a rocprofv3 kernel-trace CSV of `bench.py --no-trace`
(maps the k-th launch of each kernel family per step onto the plan's exec groups)."""
import csv
import re
import sys
from collections import defaultdict

sys.path.insert(0, ".")
from tachikoma_amd import zoo  # noqa: E402
from tachikoma_amd.relay.build_module import exec_groups, lower  # noqa: E402


def main(path, model="resnet50", batch=64):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    m = zoo.MODELS[model](batch=batch)
    plan = lower(m.mod, m.params)
    groups = exec_groups(plan)
    blocks = [g for g in groups if g.kind in ("conv_block", "dense_block")]
    fams = ("gemm_i8_kernel", "direct_conv_kernel", "dw3x3_kernel", "dw_tile_kernel", "conv_img_kernel", "conv_pf_kernel",
            "dense_tile_kernel", "dense_slices_epilogue_kernel")
    g_rows = [r for r in rows if any(f in r["Kernel_Name"] for f in fams)]
    # idle time before each launch: end of the previous kernel (any) to this start
    prev_end = {}
    last = None
    for r in rows:
        if last is not None:
            prev_end[id(r)] = int(last["End_Timestamp"])
        last = r
    gap = defaultdict(list)
    kname = {}
    n = len(blocks)
    # launches per step: the smallest period >= n of the kernel-name sequence (a split-K block
    # launches its partial tiles, then the reduce that runs the epilogue)
    names = [r["Kernel_Name"] for r in g_rows]
    L = next(p for p in range(n, n + 24) if names[-p:] == names[-2 * p:-p])
    # whole steps from the end (the module's find step launches candidate kernels first)
    k = 1
    while (k + 1) * L <= len(names) and names[-(k + 1) * L:-k * L] == names[-L:]:
        k += 1
    # the bench ends with compute-only steps (2 x --steps): keep the last 5, never a traced one
    # (traced steps run beside the record copies and, under the profiler, ~15x slower)
    k = min(k, 5)
    g_rows = g_rows[len(g_rows) - k * L:]
    dur = defaultdict(list)
    for st in range(len(g_rows) // L):
        step = g_rows[st * L:(st + 1) * L]
        i = 0
        pending = 0.0
        for r in step:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            # split-K partial passes (im2col tiles' partials, image tiles' partial records): their
            # time goes to the block's second launch (the reduce / epilogue pass)
            if L > n and ("true, false, 1," in r["Kernel_Name"] or re.search(r"conv_img_kernel<\d+, \d+, \d+, \d+, 1>",
                                                                             r["Kernel_Name"])
                          or re.search(r"dense_tile_kernel<\d+, true>", r["Kernel_Name"])):
                pending += d
                continue
            dur[i].append(d + pending)
            pending = 0.0
            if id(r) in prev_end:
                gap[i].append((int(r["Start_Timestamp"]) - prev_end[id(r)]) / 1e3)
            kname[i] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("tk::", "")
            i += 1
    print(f"{'layer':34s} {'us':>8s} {'GB/s':>8s} {'TOPS':>7s} {'gap us':>7s}  kernel")
    tot = tgap = 0
    cls = defaultdict(lambda: [0, 0.0, 0.0, 0.0])  # layer class -> [layers, us, bytes, ops]
    for i, g in enumerate(blocks):
        head = g.ops[0]
        w = plan.tensor(head.inputs[1]).shape
        x = plan.tensor(head.inputs[0])
        outb = sum(o.out.nbytes for o in g.ops)
        if head.op == "qnn.conv2d":
            nb, co, oh, ow = head.out.shape
            macs = nb * co * oh * ow * w[1] * w[2] * w[3]
            grp = head.attrs.get("groups", 1)
            desc = f"conv {x.shape[1]}->{co} k{w[2]} s{head.attrs['strides'][0]} {oh}x{ow}" + \
                (" dw" if grp > 1 and grp == co else (f" g{grp}" if grp > 1 else ""))
            kind = "depthwise 3x3" if grp > 1 else (f"{w[2]}x{w[3]} conv")
        else:
            macs = head.out.shape[0] * w[0] * w[1]
            desc = f"dense {w[1]}->{w[0]}"
            kind = "dense"
        b = x.nbytes + int(w[0] * w[1] * w[2] * w[3] if len(w) == 4 else w[0] * w[1]) + outb
        d = sorted(dur[i])[len(dur[i]) // 2]
        gp = sorted(gap[i])[len(gap[i]) // 2] if gap[i] else 0.0
        tot += d
        tgap += gp
        print(f"{desc:34s} {d:8.1f} {b / d / 1e3:8.0f} {2 * macs / d / 1e6:7.1f} {gp:7.1f}  {kname.get(i, '')}")
        c = cls[kind]
        c[0] += 1
        c[1] += d
        c[2] += b
        c[3] += 2 * macs
    print("total us", round(tot, 1), "idle before block launches us", round(tgap, 1))
    # per layer class: summed algorithmic bytes / summed time, as a fraction of the 8 TB/s HBM peak
    print(f"{'class':16s} {'layers':>6s} {'us':>9s} {'GB/s':>8s} {'HBM frac':>8s} {'TOPS':>7s}")
    for kind, (nl, us, b, ops) in sorted(cls.items(), key=lambda kv: -kv[1][1]):
        print(f"{kind:16s} {nl:6d} {us:9.1f} {b / us / 1e3:8.0f} {b / us / 1e3 / 8000:8.3f} {ops / us / 1e6:7.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
