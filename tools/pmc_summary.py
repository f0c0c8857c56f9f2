"""Summarise rocprofv3 PMC passes (tools/pmc.sh) per dispatch of the block kernel, in launch order.
FETCH_SIZE is doubled (gfx950 reports half the bytes of wide streaming reads, MI355X_MICROARCH.md §HBM);
FETCH_SIZE/WRITE_SIZE are in KiB."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(dict)   # dispatch -> counter -> value
    meta = {}
    for f in glob.glob(os.path.join(d, "pass*/run_counter_collection.csv")):
        p = f.split("/")[-2]
        rows = list(csv.DictReader(open(f)))
        for r in rows:
            key = (p, int(r["Dispatch_Id"]))
            per[key][r["Counter_Name"]] = float(r["Counter_Value"])
            meta[key] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]),
                         int(r["LDS_Block_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return per, meta


def main(d, last_n=54):
    per, meta = load(d)
    passes = sorted({k[0] for k in per})
    out = defaultdict(dict)
    for p in passes:
        keys = sorted(k for k in per if k[0] == p)[-last_n:]
        for i, k in enumerate(keys):
            out[i].update(per[k])
            out[i]["_meta"] = meta[k]
    tot = defaultdict(float)
    for i in sorted(out):
        for c, v in out[i].items():
            if c != "_meta":
                tot[c] += v
    print("per-step totals over", len(out), "dispatches:")
    for c in sorted(tot):
        v = tot[c]
        if c == "FETCH_SIZE":
            print(f"  {c:24s} {v * 2 / 1e6:10.3f} GB (x2 gfx950 correction)")
        elif c == "WRITE_SIZE":
            print(f"  {c:24s} {v / 1e6:10.3f} GB")
        else:
            print(f"  {c:24s} {v:14.0f}")
    m0 = out[0]["_meta"]
    print("example dispatch:", m0)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 54)
