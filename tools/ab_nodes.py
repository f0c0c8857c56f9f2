"""A/B per-node device times of two builds of libtachikoma.so on the same box.

usage: python tools/ab_nodes.py LIB_A LIB_B [model] [batch] [rounds]

Runs tools/node_times.py once per build and round, alternating A, B, A, B, ... (each run
a fresh process: one library per process), and prints the per-node median of each build
and the step totals.  Kernel changes that cannot be switched by an environment variable
are compared this way, on one box, because the same kernel measures +-20 % across boxes.
"""
import os
import subprocess
import sys

import numpy as np


def run(lib, model, batch):
    env = dict(os.environ, TK_LIB_PATH=os.path.abspath(lib))
    out = subprocess.run([sys.executable, "tools/node_times.py", model, str(batch), "5"], env=env,
                         capture_output=True, text=True, timeout=300, check=True).stdout
    rows = []
    for line in out.splitlines():
        tok = line.split()
        if tok and tok[0].isdigit():
            rows.append((int(tok[0]), tok[1], " ".join(tok[2:-2]), float(tok[-2])))
    return rows


def main(lib_a, lib_b, model="resnet50", batch=64, rounds=2):
    res = {0: [], 1: []}
    desc = None
    for _ in range(int(rounds)):
        for k, lib in enumerate((lib_a, lib_b)):
            rows = run(lib, model, batch)
            desc = [(r[1], r[2]) for r in rows]
            res[k].append([r[3] for r in rows])
            print(f"ran {lib}: {sum(res[k][-1]):.1f} us", flush=True)
    a = np.median(np.array(res[0]), axis=0)
    b = np.median(np.array(res[1]), axis=0)
    print(f"{'node':5s} {'kind':12s} {'desc':30s} {'A us':>8s} {'B us':>8s} {'B/A':>6s}")
    for i, (kind, d) in enumerate(desc):
        print(f"{i:<5d} {kind[:12]:12s} {d[:30]:30s} {a[i]:8.1f} {b[i]:8.1f} {b[i] / max(a[i], 1e-3):6.2f}")
    print(f"total A {a.sum():.1f} us  B {b.sum():.1f} us  B/A {b.sum() / a.sum():.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
