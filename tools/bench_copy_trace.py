"""Summarise a rocprofv3 --memory-copy-trace of bench.py (packed graph mode, run
through tools/rocprof_one_hsa.sh): the traced steps' D2H copies as the profiler saw them.

A traced step is the graph-input copy (< 1 ms) followed by the packed image's chunk copies (>= 1 ms
each, the capture stream); d2h_probe's copies after the timed region are left out.  The trace has
no byte counts: the chunk bytes come from bench.py --copy-trace's in-process record of the same
plan (tk_module_copy_trace), matched by chunk count.  Per step: chunk durations, the idle gaps
between chunk copies, copy-busy time, bytes / busy.  (Where the first chunk starts within
the step is in the in-process record: kernels of consecutive steps interleave with the previous
step's chunk copies, so the kernel trace gives no clean step start.)
usage: python tools/bench_copy_trace.py <rocprof dir> <copy_trace.json> [out.json]"""
import csv
import json
import os
import sys


def main(d, ct_path, out=None):
    copies = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"], r["Stream_Id"])
                     for r in csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv")))))
    ref = json.load(open(ct_path))["steps"][0]["chunks"]
    chunk_bytes = [c["bytes"] for c in ref]
    d2h = [c for c in copies if c[2].endswith("DEVICE_TO_HOST")]
    steps, i = [], 0
    while i < len(d2h):
        s, e, _, sid = d2h[i]
        if e - s < 1_000_000:
            j = i + 1
            while j < len(d2h) and d2h[j][3] == sid and d2h[j][1] - d2h[j][0] >= 1_000_000 and \
                    d2h[j][0] - d2h[j - 1][1] < 5_000_000:
                j += 1
            if j - i - 1 == len(chunk_bytes):
                steps.append((d2h[i], d2h[i + 1:j]))
                i = j
                continue
        i += 1
    out_steps = []
    for inp, ch in steps:
        busy = sum(e - s for s, e, _, _ in ch)
        nb = sum(chunk_bytes)
        out_steps.append({
            "input_copy_ms": round((inp[1] - inp[0]) / 1e6, 3),
            "chunks_ms": [round((e - s) / 1e6, 3) for s, e, _, _ in ch],
            "chunk_GBps": [round(b / (e - s), 2) for b, (s, e, _, _) in zip(chunk_bytes, ch)],
            "gaps_ms": [round((b[0] - a[1]) / 1e6, 4) for a, b in zip(ch, ch[1:])],
            "copy_busy_ms": round(busy / 1e6, 3),
            "first_to_last_ms": round((ch[-1][1] - ch[0][0]) / 1e6, 3),
            "bytes": nb,
            "GBps_while_copying": round(nb / busy, 2),
            "GBps_first_to_last": round(nb / (ch[-1][1] - ch[0][0]), 2),
        })
    doc = {"source": f"rocprofv3 --memory-copy-trace of bench.py ({d}); chunk bytes from {ct_path}",
           "chunks_per_step": len(chunk_bytes), "steps": out_steps}
    text = json.dumps(doc, indent=1)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:])
