"""Per-kernel durations from a rocprofv3 rocpd database (kernels view): consecutive runs of
the same kernel/grid are grouped, with their average duration and the gap between launches.
usage: python tools/rocpd_kernels.py <run_results.db> [name-regex]"""
import re
import sqlite3
import sys


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
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
