"""Where a launch-bound tick loop's time goes, from one rocprofv3 --kernel-trace --runtime-trace run
(tools/gpu.sh step `trace`): per kernel, calls and average duration; the GPU-idle gaps between
consecutive dispatches, by the pair of kernels around them; and the HIP API calls by total host time.
The raw per-dispatch CSVs stay on the box (they are large); only this summary is kept.

usage: python tools/trace_gaps.py <rocprofv3 output dir> [ticks | bench log]   (divides the totals per
tick; from a bench log: its trading.ticks x (steps + warmup), every run of the bench being the same run)
"""
import collections
import csv
import glob
import json
import sys


def rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def short(name):
    """The kernel's name without namespaces' '(anonymous namespace)' and its argument list."""
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0][:80]


def main():
    d = sys.argv[1]
    ticks = 0
    if len(sys.argv) > 2:
        if sys.argv[2].isdigit():
            ticks = int(sys.argv[2])
        else:
            for line in open(sys.argv[2]):
                if line.startswith('{"metric"'):
                    b = json.loads(line)
                    ticks = int(b.get("trading", {}).get("ticks", 0)) * (int(b["steps"]) + int(b["warmup"]))
    ks = rows(f"{d}/**/*kernel_trace.csv")
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in ks]
    ks.sort()
    res = {"dispatches": len(ks)}
    if ks:
        span = ks[-1][1] - ks[0][0]
        busy = sum(e - s for s, e, _ in ks)
        per = collections.defaultdict(lambda: [0, 0])
        for s, e, n in ks:
            per[n][0] += 1
            per[n][1] += e - s
        gaps = collections.defaultdict(lambda: [0, 0])
        for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
            g = max(0, s1 - e0)
            gaps[(n0, n1)][0] += 1
            gaps[(n0, n1)][1] += g
        res.update(span_us=span / 1e3, kernel_busy_us=busy / 1e3, idle_us=(span - busy) / 1e3,
                   kernels={n: {"calls": c, "avg_us": round(t / c / 1e3, 3), "total_us": round(t / 1e3, 1)}
                            for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])},
                   gaps_top=[{"after": a, "before": b, "count": c, "avg_gap_us": round(t / c / 1e3, 3),
                              "total_us": round(t / 1e3, 1)}
                             for (a, b), (c, t) in sorted(gaps.items(), key=lambda x: -x[1][1])[:12]])
        if ticks:
            res["per_tick_us"] = {"span": round(span / 1e3 / ticks, 3), "kernel_busy": round(busy / 1e3 / ticks, 3),
                                  "idle": round((span - busy) / 1e3 / ticks, 3),
                                  "dispatches": round(len(ks) / ticks, 2)}
    api = rows(f"{d}/**/*hip_api_trace.csv")
    if api:
        per = collections.defaultdict(lambda: [0, 0])
        for r in api:
            n = r.get("Function") or r.get("Operation") or "?"
            per[n][0] += 1
            per[n][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        res["hip_api_top"] = [{"fn": n, "calls": c, "avg_us": round(t / c / 1e3, 3), "total_us": round(t / 1e3, 1)}
                              for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:15]]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
