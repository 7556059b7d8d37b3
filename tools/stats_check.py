"""Per-config agreement of a bench line with the rocprofv3 kernel trace of the
SAME run (tools/stats_pass.sh: `rocprofv3 --kernel-trace --stats -- python3
bench.py --config C --steps K ...`, the line printed by that process).

The timed region of bench.py runs exactly K decode calls after the warm-up
and the verify pass, so the last K dispatches of each kernel the line names
(roofline.kernel, '+'-joined for a call of several kernels) are the timed
ones; their mean durations, summed, are the call's kernel time. The line's
own clock is HIP events around the whole call (roofline.avg_launch_ms). The
summary is refused (exit 1) when the two differ by more than --tol (3 %):
a committed frac must follow from a committed trace.

usage: python3 tools/stats_check.py <rocprof dir> <bench line json> [--out f.json]
"""
import argparse
import csv
import glob
import json
import os
import sys


def trace_rows(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit("no kernel_trace.csv under %s" % d)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                             int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    return rows


def base_name(k):
    """The kernel's own name: rocprof's demangled names carry the return
    type, namespaces, template and call arguments."""
    k = k.strip().replace("(anonymous namespace)::", "")
    if k.startswith("void "):
        k = k[5:]
    for c in "<(":
        k = k.split(c)[0]
    return k.split("::")[-1].strip()


def summarize(rows, kernels, steps):
    out = {}
    for k in kernels:
        durs = [(e - s) / 1e6 for _, name, s, e in rows if base_name(name) == k]
        if len(durs) < steps:
            raise SystemExit("kernel %s: %d dispatches < %d timed steps" % (k, len(durs), steps))
        timed = durs[-steps:]
        timed_sorted = sorted(timed)
        out[k] = {"dispatches": len(durs), "timed": steps,
                  "mean_ms": sum(timed) / steps,
                  "median_ms": timed_sorted[steps // 2],
                  "min_ms": timed_sorted[0], "max_ms": timed_sorted[-1],
                  "mean_all_ms": sum(durs) / len(durs)}
    return out


MARK = "spin_kernel"  # bench.py trace_mark (torch.cuda._sleep)


def calls(rows, steps):
    """With BENCH_TRACE_MARKS=1 the timed region is M [encode] M [decode] M
    per step: (encode calls, decode calls), each a list of dispatches."""
    marks = [i for i, r in enumerate(rows) if MARK in r[1]]
    if len(marks) < 3 * steps:
        return None
    marks = marks[-3 * steps:]
    enc, dec = [], []
    for k in range(steps):
        a, b, c = marks[3 * k: 3 * k + 3]
        enc.append(rows[a + 1: b])
        dec.append(rows[b + 1: c])
    return enc, dec


def call_summary(cl):
    """Per call: the span from its first kernel's start to its last kernel's
    end (what HIP events around the call see, minus launch gaps at the
    edges), and the sum of its kernels' durations; per kernel name: mean
    time per call."""
    spans = [(c[-1][3] - c[0][2]) / 1e6 for c in cl if c]
    busy = [sum(e - s for _, _, s, e in c) / 1e6 for c in cl]
    per = {}
    for c in cl:
        for _, name, s, e in c:
            per.setdefault(base_name(name), []).append((e - s) / 1e6)
    n = len(cl)
    return {"span_ms": sum(spans) / max(len(spans), 1), "busy_ms": sum(busy) / n,
            "kernels": {k: {"per_call_ms": round(sum(v) / n, 4), "dispatches_per_call": len(v) / n}
                        for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))}}


def check(d, line, tol=0.03):
    rl = line["roofline"]
    steps = int(line["steps"])
    rows = trace_rows(d)
    segs = calls(rows, steps)
    res = {"config": line["config"]["workload"], "steps": steps, "marked": segs is not None}
    for side, blk in (("decode", rl), ("encode", rl.get("encode"))):
        if not blk:
            continue
        kernels = blk["kernel"].split("+")
        ks = summarize(rows, kernels, steps)
        kernel_ms = sum(v["mean_ms"] for v in ks.values())
        event_ms = float(blk["avg_launch_ms"])
        alg = float(blk["algorithmic_bytes_per_launch"])
        peak = float(rl["peak"])
        r = {
            "kernels": ks, "kernel_ms": round(kernel_ms, 4), "event_ms": event_ms,
            "kernel_over_event": round(kernel_ms / event_ms, 4),
            "frac_events": round(alg / (event_ms / 1e3) / 1e9 / peak, 4),
            "frac_kernel": round(alg / (kernel_ms / 1e3) / 1e9 / peak, 4),
        }
        if segs is not None:
            cs = call_summary(segs[0] if side == "encode" else segs[1])
            r["call"] = {"span_ms": round(cs["span_ms"], 4), "busy_ms": round(cs["busy_ms"], 4),
                         "span_over_event": round(cs["span_ms"] / event_ms, 4),
                         "frac_span": round(alg / (cs["span_ms"] / 1e3) / 1e9 / peak, 4),
                         "kernels": cs["kernels"]}
            # the call as the trace sees it against the events around it
            r["agrees"] = abs(cs["span_ms"] / event_ms - 1.0) <= tol
        else:
            r["agrees"] = abs(kernel_ms / event_ms - 1.0) <= tol
        res[side] = r
    res["agrees"] = all(res[s]["agrees"] for s in ("decode", "encode") if s in res)
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("line")
    ap.add_argument("--out")
    ap.add_argument("--tol", type=float, default=0.03)
    a = ap.parse_args(argv)
    with open(a.line) as f:
        line = next(json.loads(l) for l in f if l.startswith("{") and '"metric"' in l)
    res = check(a.dir, line, a.tol)
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    print(txt)
    return 0 if res["agrees"] else 1


if __name__ == "__main__":
    sys.exit(main())
