"""Per-layer kernel durations from a rocprofv3 kernel-trace CSV of `bench.py --no-trace`
(maps the k-th launch of each kernel family per step onto the plan's exec groups)."""
import csv
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
    g_rows = [r for r in rows if r["Kernel_Name"].startswith("gemm_i8_kernel") or
              r["Kernel_Name"].startswith("direct_conv_kernel")]
    n = len(blocks)
    dur = defaultdict(list)
    for i, r in enumerate(g_rows[-(len(g_rows) // n) * n:]):
        dur[i % n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'layer':34s} {'us':>8s} {'GB/s':>8s} {'TOPS':>7s}  VGPR/AGPR")
    tot = 0
    for i, g in enumerate(blocks):
        head = g.ops[0]
        w = plan.tensor(head.inputs[1]).shape
        x = plan.tensor(head.inputs[0])
        outb = sum(o.out.nbytes for o in g.ops)
        if head.op == "qnn.conv2d":
            nb, co, oh, ow = head.out.shape
            macs = nb * co * oh * ow * w[1] * w[2] * w[3]
            desc = f"conv {w[1]*(co//w[0]) if False else x.shape[1]}->{co} k{w[2]} s{head.attrs['strides'][0]} {oh}x{ow}"
        else:
            macs = head.out.shape[0] * w[0] * w[1]
            desc = f"dense {w[1]}->{w[0]}"
        b = x.nbytes + int(w[0] * w[1] * w[2] * w[3] if len(w) == 4 else w[0] * w[1]) + outb
        d = sorted(dur[i])[len(dur[i]) // 2]
        tot += d
        print(f"{desc:34s} {d:8.1f} {b / d / 1e3:8.0f} {2 * macs / d / 1e6:7.1f}")
    print("total us", round(tot, 1))


if __name__ == "__main__":
    main(*sys.argv[1:])
