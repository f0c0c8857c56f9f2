"""Per-kernel durations from a rocprofv3 rocpd database (kernels view): consecutive runs of
the same kernel/grid are grouped, with their average duration and the gap between launches.
usage: python tools/rocpd_kernels.py <run_results.db> [name-regex] [--seq N]
  --seq N: instead, list the last N matching launches one by one (duration and the idle gap
  before each), e.g. one compute-only step of the network."""
import re
import sqlite3
import sys


def seq(db, pat, n):
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select name, start, end, grid_x from kernels order by start").fetchall()
    prev = None
    out = []
    for name, s, e, gx in rows:
        if not pat or re.search(pat, name):
            out.append((re.sub(r"\(.*", "", name)[:60], gx // 256, (e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0))
        prev = e
    tot = 0.0
    for i, (nm, g, d, gap) in enumerate(out[-n:]):
        tot += d
        print(f"{i:3d} {nm:60s} wg {g:6d} {d:8.2f} us  gap {gap:6.2f}")
    print(f"sum {tot:.1f} us")


def main(db, pat=None):
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count, "
                       "accum_vgpr_count, sgpr_count from kernels order by start").fetchall()
    groups = []
    prev_end = None
    for name, s, e, gx, gy, gz, wx, lds, vg, ag, sg in rows:
        if pat and not re.search(pat, name):
            prev_end = e
            continue
        key = (name, gx, gy, gz)
        gap = (s - prev_end) if prev_end is not None else 0
        if groups and groups[-1]["key"] == key:
            g = groups[-1]
        else:
            g = {"key": key, "n": 0, "dur": 0, "gap": 0, "lds": lds, "regs": (vg, ag, sg)}
            groups.append(g)
        g["n"] += 1
        g["dur"] += e - s
        g["gap"] += gap
        prev_end = e
    for g in groups:
        name, gx, gy, gz = g["key"]
        short = re.sub(r"\(.*", "", name)[:70]
        print(f"{short:70s} grid {gx // 256 if gx >= 256 else gx:>6}x{gy}x{gz} n={g['n']:3d} avg {g['dur'] / g['n'] / 1e3:8.2f} us"
              f"  gap {g['gap'] / g['n'] / 1e3:6.2f} us  lds {g['lds']} regs {g['regs']}")


if __name__ == "__main__":
    if "--seq" in sys.argv:
        i = sys.argv.index("--seq")
        seq(sys.argv[1], sys.argv[2] if i > 2 else None, int(sys.argv[i + 1]))
    else:
        main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
