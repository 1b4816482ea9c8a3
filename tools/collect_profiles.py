"""Copy the rocprofv3 summaries of one tools/gpu.sh run into profiles/<tag>/ (tracked) and derive
the per-launch HBM traffic of the measured kernel for bench.py's roofline.traffic.

The kernel is matched by its exact rocprofv3 name: MCS_KERNEL if set, else the engine (mcs::) kernel with
the most calls in the kernel-trace stats (in a PMC-only run: the most dispatches in the counter passes) (the bench's production launches; bench.py's single untimed
counting-build launch, e.g. `fifo_asm_kernel<16, true, 4, 8, true>`, is a different name and is
never averaged in).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half the bytes of a wide
coalesced streaming read on gfx950, so it is doubled (the job stream is read 16 B/lane);
WRITE_SIZE (KB) is taken as is.  Counters come from separate --pmc passes, one production launch
(bench --steps 1 --warmup 0) each.

usage: python tools/collect_profiles.py gpurun_out/<run> profiles/<tag> [prof_<name>]
"""
import csv
import glob
import json
import os
import shutil
import sys

run, out = sys.argv[1], sys.argv[2]
prof = sys.argv[3] if len(sys.argv) > 3 else None
os.makedirs(out, exist_ok=True)

summary = {}
stats = sorted(glob.glob(f"{run}/{prof or 'prof*'}/*kernel_stats.csv"))
kernel = os.environ.get("MCS_KERNEL")
if stats:
    shutil.copy(stats[0], f"{out}/kernel_stats.csv")
    rows = list(csv.DictReader(open(stats[0])))
    if kernel is None:  # the production kernel: the engine's kernel with the most launches
        kernel = max((r for r in rows if "mcs::" in r["Name"]), key=lambda r: int(r["Calls"]))["Name"]
    for r in rows:
        if r["Name"] == kernel:
            summary.update(kernel=r["Name"], calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                           min_ns=float(r["MinNs"]), max_ns=float(r["MaxNs"]))
if kernel is None:  # a PMC-only run: the engine kernel with the most dispatches in the counter passes
    seen = {}
    for g in sorted(glob.glob(f"{run}/pmc*_g*/pmc_counter_collection.csv")):
        for r in csv.DictReader(open(g)):
            n = r.get("Kernel_Name", r.get("Name", ""))
            if "mcs::" in n:
                seen.setdefault(n, set()).add(r["Dispatch_Id"])
    bk = None
    if os.path.exists(f"{run}/bench.json"):  # the bench line's kernel (e.g. mcs::delay_asm_kernel)
        with open(f"{run}/bench.json") as f:
            bk = json.loads(f.read().strip().splitlines()[-1])["roofline"].get("kernel", "").split("::")[-1]
    named = {n: v for n, v in seen.items() if bk and bk.split(" ")[0] in n}
    if named or seen:
        kernel = max(named or seen, key=lambda n: len((named or seen)[n]))
if kernel is None:
    sys.exit("no kernel_stats.csv or PMC pass in the run and no MCS_KERNEL: cannot tell which kernel to summarise")

counters = {}
launches = 0
for g in sorted(glob.glob(f"{run}/pmc*_g*/pmc_counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(g)) if r.get("Kernel_Name", r.get("Name", "")) == kernel]
    # a pass may hold more than one launch of the kernel: summed per launch, averaged over launches
    n_launch = max(len({r["Dispatch_Id"] for r in rows}), 1)
    launches = max(launches, n_launch)
    for r in rows:
        counters[r["Counter_Name"]] = counters.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"]) / n_launch
summary["pmc_kernel"] = kernel
summary["pmc_per_launch"] = counters


def short_name(n):
    """The engine's name for a rocprofv3 kernel name (mcs_last_kernel, bench.py's roofline.kernel): no
    'void', no anonymous namespace, no parameter list, no trailing counting-build flag (', false');
    fifo_asm_kernel's lookahead flag (r06) reads ', look' when set and is dropped when not."""
    n = n.replace("void ", "", 1).replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    n = n.replace(", false, false>", ">").replace(", false, true>", ", look>")
    return n.replace(", false>", ">").replace("<false>", "")


summary["kernel_short"] = short_name(kernel)

bench = None
bench_file = f"{run}/bench.json" if os.path.exists(f"{run}/bench.json") else os.environ.get("MCS_BENCH_JSON")
if bench_file and os.path.exists(bench_file):
    with open(bench_file) as f:
        bk = json.loads(f.read().strip().splitlines()[-1])["roofline"].get("kernel", "")
    summary["bench_kernel"] = bk
    summary["kernel_matches_bench"] = summary["kernel_short"] == bk
if os.path.exists(f"{run}/bench.json"):
    shutil.copy(f"{run}/bench.json", f"{out}/bench.json")
    with open(f"{run}/bench.json") as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
if bench and "placements_per_step_per_gpu" not in bench.get("config", {}):
    bench = None  # (a trading line: no per-placement traffic; the raw counters stay in pmc_per_launch)
if bench and "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
    jobs = bench["config"]["placements_per_step_per_gpu"]
    fetch = counters["FETCH_SIZE"] * 1024.0 * 2.0
    write = counters["WRITE_SIZE"] * 1024.0
    traffic = {
        "clusters": bench["config"]["clusters_per_gpu"],
        "nodes": bench["config"]["nodes"],
        "jobs_per_cluster": bench["config"]["jobs_per_cluster"],
        "policy": "delay" if "DELAY" in bench["metric"] else "fifo",
        "gen": bench["config"].get("gen", "stream"),
        "lam": bench["config"].get("lam", 0.0),
        "max_dur": bench["config"].get("max_dur", 600),
        "kernel": kernel,
        "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes_corrected": fetch,
        "write_bytes": write,
        "algorithmic_bytes_per_launch": float(bench["roofline"]["bytes_per_placement"]) * jobs,
        "bytes_per_placement": (fetch + write) / jobs,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH doubled per "
                  "MI355X_MICROARCH.md gfx950 correction",
    }
    summary["traffic"] = traffic
    with open(f"{out}/traffic.json", "w") as f:
        json.dump(traffic, f, indent=1)
    with open("profiles/traffic_latest" + ("_delay" if traffic["policy"] == "delay" else "")
              + ("_fused" if traffic["gen"] == "fused" else "")
              + (f"_lam{traffic['lam']:g}_dur{traffic['max_dur']}" if traffic["lam"] or traffic["max_dur"] != 600 else "")
              + ".json", "w") as f:
        json.dump(traffic, f, indent=1)
if "SQ_INSTS_SALU" in counters and bench:
    jobs = bench["config"]["placements_per_step_per_gpu"]
    summary["per_placement"] = {k: v / jobs for k, v in counters.items() if k.startswith("SQ_")}
with open(f"{out}/summary.json", "w") as f:
    json.dump(summary, f, indent=1)
for log in ("pytest_gpu.log", "smoke.log"):
    if os.path.exists(f"{run}/{log}"):
        shutil.copy(f"{run}/{log}", f"{out}/{log}")
print(json.dumps(summary, indent=1)[:3000])
