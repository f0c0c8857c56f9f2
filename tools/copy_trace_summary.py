"""Summarise a rocprofv3 --memory-copy-trace CSV of tools/probe_copies (per-copy
rate vs inter-copy gaps of the step's 233 record copies).

The trace has no byte counts, so runs of copies are matched against the record sizes the probe
copied (tools/resnet50_b64_record_sizes.txt): a window of 233 consecutive D2H copies whose
durations follow the sizes is one 'per-record' pass (host-issued copies, batch copies); runs of
equal-length copies are whole-image chunk passes (1/8/32/128 chunks of the same total).  For each
pass: bytes / span, the summed copy time, the summed gaps between copies and the per-copy rate.
usage: python tools/copy_trace_summary.py <run_memory_copy_trace.csv> <sizes.txt> [out.json]"""
import csv
import json
import sys


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Direction"].endswith("DEVICE_TO_HOST"):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    return rows


def pass_stats(seg, sizes):
    total = sum(sizes)
    span = (seg[-1][1] - seg[0][0]) * 1e-9
    busy = sum(e - s for s, e in seg) * 1e-9
    gaps = [max(0, seg[i + 1][0] - seg[i][1]) * 1e-9 for i in range(len(seg) - 1)]
    big = [(b, (e - s) * 1e-9) for (s, e), b in zip(seg, sizes) if b >= 64 << 20]
    return {"copies": len(seg), "bytes": total, "span_ms": round(span * 1e3, 3), "GBps": round(total / span / 1e9, 2),
            "copy_ms": round(busy * 1e3, 3), "copy_GBps": round(total / busy / 1e9, 2),
            "gap_ms": round(sum(gaps) * 1e3, 3), "max_gap_us": round(max(gaps, default=0) * 1e6, 1),
            "big_copy_GBps": round(sum(b for b, _ in big) / sum(t for _, t in big) / 1e9, 2) if big else None}


def main():
    rows = load(sys.argv[1])
    sizes = [int(x) for x in open(sys.argv[2]).read().split()]
    n, total = len(sizes), sum(sizes)
    out, i = [], 0
    while i < len(rows):
        if i + n <= len(rows):
            seg = rows[i:i + n]
            rates = [b / max(1, e - s) for (s, e), b in zip(seg, sizes) if b >= 1 << 20]
            rates.sort()
            med = rates[len(rates) // 2] if rates else 0
            # bytes per ns == GB/s; a per-record pass keeps its big copies near one rate
            if 30 < med < 70 and rates[len(rates) // 10] > 0.6 * med:
                out.append(dict(kind="per-record copies", **pass_stats(seg, sizes)))
                i += n
                continue
        # a run of k equal-duration copies covering the image: k whole-image chunks
        for k in (128, 32, 8, 1):
            if i + k <= len(rows):
                seg = rows[i:i + k]
                durs = [e - s for s, e in seg]
                chunk = -(-total // k)
                if min(durs) > 0.7 * max(durs) and 30 < chunk / max(1, durs[0]) < 70:
                    out.append(dict(kind=f"{k} image chunks", **pass_stats(seg, [chunk] * (k - 1) + [total - chunk * (k - 1)])))
                    i += k
                    break
        else:
            i += 1
    doc = {"source": sys.argv[1], "record_sizes": sys.argv[2], "passes": out,
           "note": "rocprofv3 memory-copy trace of tools/probe_copies; rows are D2H copies matched to the record "
                   "sizes by position (the trace carries no byte counts); graph memcpy nodes do not appear"}
    text = json.dumps(doc, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
