"""Summarise rocprofv3 PMC passes (tools/pmc.sh) for the fused layer-block kernel.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB; on
gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so it
is doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.  The last
``launches`` dispatches of each pass are one step (the bench runs warmup + steps
with the same node list).

usage: python tools/pmc_summary.py <pmc outdir> [launches] [--runs R] [--json out.json]
(`bench.py --steps 2 --warmup 1 --no-trace` runs 1 + 3*2 + 1 = 8 steps)
"""
import argparse
import csv
import glob
import json
import os
import sys
import time
from collections import defaultdict

KIB = 1024
SIMDS = 1024   # gfx950 MI355X: 256 CUs x 4 SIMDs (rocprofiler-sdk SIMD_NUM)
XCDS = 8       # GRBM_GUI_ACTIVE arrives summed over the 8 XCDs: /8 = the busy cycles of one (its max)


def mfma_figures(c):
    """Matrix-core use from pass 6's counters (rocprofiler-sdk counter_defs.yaml, gfx950):
    MfmaUtil = sum(SQ_VALU_MFMA_BUSY_CYCLES) / (max(GRBM_GUI_ACTIVE) x SIMD_NUM).  rocprofv3 hands
    GRBM_GUI_ACTIVE over summed across the XCDs, so max ~= sum / 8 (all XCDs run the grid).
    Also: executed int8 ops (MOPS_I8 x 512) and busy cycles per int8 MFMA instruction (32 for
    v_mfma_i32_32x32x32_i8: 65,536 ops per 32 cycles per SIMD = the 5.0 POPS dense peak at 2.4 GHz)."""
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
    gui = c.get("GRBM_GUI_ACTIVE")
    if busy is None or not gui:
        return None
    insts = c.get("SQ_INSTS_VALU_MFMA_I8", 0.0)
    dur = c.get("_dur_ns")
    out = {"mfma_busy": round(busy / (gui / XCDS * SIMDS), 4),
           "SQ_VALU_MFMA_BUSY_CYCLES": busy, "SQ_INSTS_VALU_MFMA_I8": insts,
           "int8_ops_executed": c.get("SQ_INSTS_VALU_MFMA_MOPS_I8", 0.0) * 512,
           "busy_cycles_per_i8_mfma": round(busy / insts, 2) if insts else None,
           "gui_cycles_per_xcd": gui / XCDS}
    if dur:
        out["implied_clock_ghz"] = round(gui / XCDS / dur, 3)  # GUI-active cycles per ns of the dispatch
    return out


def load(d):
    per = defaultdict(dict)   # (pass, dispatch) -> counter -> value
    meta = {}
    for f in glob.glob(os.path.join(d, "pass*/**/*counter_collection.csv"), recursive=True):
        p = os.path.relpath(f, d).split(os.sep)[0]
        for r in csv.DictReader(open(f)):
            key = (p, int(r["Dispatch_Id"]))
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):  # the dispatch under this pass
                per[key]["_dur_ns"] = float(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            meta[key] = {"kernel": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "vgpr": int(r["VGPR_Count"]),
                         "agpr": int(r.get("Accum_VGPR_Count", 0) or 0), "lds": int(r["LDS_Block_Size"])}
    return per, meta


def step_period(names, lo=8):
    """Block-kernel dispatches per step: the smallest p >= lo whose last two p-long runs of kernel
    names are equal (the module's find step launches candidate kernels before the steps, so the
    dispatch count is not a multiple of the step)."""
    for p in range(lo, len(names) // 2 + 1):
        if names[-p:] == names[-2 * p:-p]:
            return p
    return None


def min_launches(model="resnet50", batch=64):
    """Block nodes of the bench's default workload (tools/layer_times.py's plan walk)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from tachikoma_amd import zoo
    from tachikoma_amd.relay.build_module import exec_groups, lower
    m = zoo.MODELS[model](batch=batch)
    return sum(1 for g in exec_groups(lower(m.mod, m.params)) if g.kind in ("conv_block", "dense_block"))


def summarise(d, launches=None, runs=None, model="resnet50", batch=64):
    """launches: block-kernel dispatches per step (default: the period of the dispatch sequence,
    step_period, from the workload's block-node count up); runs: only used when no period is
    found (launches = dispatches / runs)."""
    per, meta = load(d)
    passes = sorted({k[0] for k in per})
    if launches is None:
        p0 = passes[0]
        names = [meta[k]["kernel"] for k in sorted(k for k in per if k[0] == p0)]
        # a step launches at least one kernel per block node: shorter periods are repeats inside a
        # step (the 14x14 stage's identical bottlenecks), not steps
        launches = step_period(names, lo=min_launches(model, batch))
        if launches is None:
            counts = {p: sum(1 for k in per if k[0] == p) for p in passes}
            launches = min(counts.values()) // runs
    steps = defaultdict(dict)
    for p in passes:
        keys = sorted(k for k in per if k[0] == p)[-launches:]
        for i, k in enumerate(keys):
            steps[i].update(per[k])
            steps[i]["_meta"] = meta[k]
    tot = defaultdict(float)
    for i in steps:
        for c, v in steps[i].items():
            if c != "_meta":
                tot[c] += v
    n = len(steps)
    # per kernel (template instance) and per dispatch of the step: where the LDS bank conflicts,
    # VALU and HBM bytes are (attribute the conflict ratio per kernel)
    fam = defaultdict(lambda: defaultdict(float))
    disp = []
    for i in sorted(steps):
        m = steps[i]["_meta"]
        name = m["kernel"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("tk::", "").strip()
        f = fam[name]
        f["dispatches"] += 1
        for c, v in steps[i].items():
            if c != "_meta":
                f[c] += v
        lds_i = steps[i].get("SQ_INSTS_LDS", 0.0)
        disp.append({"i": i, "kernel": name, "grid": m["grid"], "lds_bytes": m["lds"],
                     "lds_conflict_per_inst": round(steps[i].get("SQ_LDS_BANK_CONFLICT", 0.0) / lds_i, 3) if lds_i else None,
                     "SQ_INSTS_LDS": lds_i, "SQ_LDS_BANK_CONFLICT": steps[i].get("SQ_LDS_BANK_CONFLICT"),
                     "hbm_bytes": steps[i].get("FETCH_SIZE", 0.0) * KIB * 2 + steps[i].get("WRITE_SIZE", 0.0) * KIB,
                     "dur_ns": steps[i].get("_dur_ns"),
                     "mfma": mfma_figures(steps[i]),
                     # share of the waves' cycles spent waiting on counters / on issue / issuing
                     **{k: round(steps[i].get(c, 0.0) / steps[i]["SQ_WAVE_CYCLES"], 3)
                        for k, c in (("wait_any_per_wave_cycle", "SQ_WAIT_ANY"),
                                     ("wait_inst_per_wave_cycle", "SQ_WAIT_INST_ANY"),
                                     ("active_inst_per_wave_cycle", "SQ_ACTIVE_INST_ANY"))
                        if steps[i].get("SQ_WAVE_CYCLES")}})
    per_kernel = {}
    for name, f in sorted(fam.items(), key=lambda kv: -kv[1].get("SQ_LDS_BANK_CONFLICT", 0.0)):
        li = f.get("SQ_INSTS_LDS", 0.0)
        per_kernel[name] = {"dispatches": int(f["dispatches"]), "SQ_INSTS_LDS": li,
                            "SQ_LDS_BANK_CONFLICT": f.get("SQ_LDS_BANK_CONFLICT", 0.0),
                            "conflict_per_lds_inst": round(f.get("SQ_LDS_BANK_CONFLICT", 0.0) / li, 3) if li else None,
                            "share_of_conflicts": round(f.get("SQ_LDS_BANK_CONFLICT", 0.0) /
                                                        max(tot.get("SQ_LDS_BANK_CONFLICT", 0.0), 1.0), 3),
                            "SQ_INSTS_VALU": f.get("SQ_INSTS_VALU", 0.0),
                            "mfma": mfma_figures(f)}
    fetch = tot.get("FETCH_SIZE", 0.0) * KIB * 2
    write = tot.get("WRITE_SIZE", 0.0) * KIB
    out = {"launches_per_step": n,
           "fetch_bytes_per_step": fetch, "write_bytes_per_step": write,
           "hbm_bytes_per_step": fetch + write,
           "hbm_bytes_per_launch": (fetch + write) / max(n, 1),
           "correction": "FETCH_SIZE x2 (gfx950 wide reads), KiB -> bytes",
           "counters_per_step": {c: v for c, v in sorted(tot.items())},
           "example_dispatch": steps[0]["_meta"] if n else None,
           "lds_conflict_per_lds_inst": round(tot.get("SQ_LDS_BANK_CONFLICT", 0.0) / tot["SQ_INSTS_LDS"], 3)
           if tot.get("SQ_INSTS_LDS") else None,
           "mfma": mfma_figures(tot),
           "per_kernel": per_kernel, "per_dispatch": disp}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("launches", type=int, nargs="?", default=None)
    ap.add_argument("--runs", type=int, default=8, help="steps the profiled bench command ran")
    ap.add_argument("--json")
    ap.add_argument("--workload", default="", help="extra bench args the passes ran with")
    a = ap.parse_args()
    wl = a.workload.split()
    model = wl[wl.index("--model") + 1] if "--model" in wl else "resnet50"
    batch = int(wl[wl.index("--batch") + 1]) if "--batch" in wl else 64
    s = summarise(a.dir, a.launches, a.runs, model, batch)
    s["bench_args"] = wl
    s["model"] = model
    s["batch"] = batch
    # which kernels these counters belong to: bench.py takes the traffic from the summary whose
    # library digest equals the loaded library's (else the newest by this UTC stamp)
    s["created_utc"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
    # and which kernel mix: the tune table the passes replayed (bench --tune-table), by digest
    s["tune_table"] = wl[wl.index("--tune-table") + 1] if "--tune-table" in wl else "auto"
    s["tune_table_digest"] = None
    if s["tune_table"] == "auto":  # what bench.py's default resolves to
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        s["tune_table"] = bench.find_tune_table(model, batch)
    if s["tune_table"] and s["tune_table"] != "none":
        try:
            sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            from tachikoma_amd.relay.device_module import tune_table_digest
            with open(s["tune_table"]) as f:
                s["tune_table_digest"] = tune_table_digest(json.load(f)["entries"])
        except Exception as e:  # noqa: BLE001
            print(f"  (tune table digest unavailable: {e})")
    try:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from tachikoma_amd import _lib
        s["library"] = _lib.build_info()
    except Exception as e:  # noqa: BLE001 - a summary without a digest is still a summary
        s["library"] = None
        print(f"  (library digest unavailable: {e})")
    print(f"per-step totals over {s['launches_per_step']} dispatches:")
    print(f"  HBM fetch {s['fetch_bytes_per_step'] / 1e9:.3f} GB (x2 corrected), write "
          f"{s['write_bytes_per_step'] / 1e9:.3f} GB, per launch {s['hbm_bytes_per_launch'] / 1e6:.2f} MB")
    for c, v in s["counters_per_step"].items():
        print(f"  {c:24s} {v:16.0f}")
    if s.get("mfma"):
        print(f"MFMA busy (MfmaUtil, counted): {s['mfma']}")
    print(f"LDS bank conflicts per LDS instruction: {s['lds_conflict_per_lds_inst']}; per kernel:")
    for k, v in s["per_kernel"].items():
        print(f"  {v['share_of_conflicts']:6.3f} of conflicts, {v['conflict_per_lds_inst']} per inst, "
              f"{v['dispatches']:3d} x {k}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(s, f, indent=1)


if __name__ == "__main__":
    main()
