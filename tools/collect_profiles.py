"""Copy the rocprofv3 summaries of one tools/gpu_check.sh run into profiles/<tag>/ (tracked) and
derive the per-launch HBM traffic of fifo_kernel for bench.py's roofline.traffic.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half the bytes of a wide
coalesced streaming read on gfx950, so it is doubled (the job stream is read 16 B/lane);
WRITE_SIZE (KB) is taken as is (calibration caveat: our result stores are 4 B/lane).  Counters
come from separate --pmc passes, one launch (bench --steps 1 --warmup 0) each.

usage: python tools/collect_profiles.py gpurun_out/<run> profiles/<tag>
"""
import csv
import glob
import json
import os
import shutil
import sys

run, out = sys.argv[1], sys.argv[2]
os.makedirs(out, exist_ok=True)


KERNEL = os.environ.get("MCS_KERNEL", "fifo_kernel")  # delay_kernel for --policy delay runs


def fifo_rows(path):
    return [r for r in csv.DictReader(open(path)) if KERNEL in r.get("Kernel_Name", r.get("Name", ""))]


summary = {}
stats = glob.glob(f"{run}/prof/*kernel_stats.csv")
if stats:
    shutil.copy(stats[0], f"{out}/kernel_stats.csv")
    for r in csv.DictReader(open(stats[0])):
        if KERNEL in r["Name"]:
            summary["kernel"] = r["Name"]
            summary["calls"] = int(r["Calls"])
            summary["avg_ns"] = float(r["AverageNs"])
            summary["min_ns"] = float(r["MinNs"])
            summary["max_ns"] = float(r["MaxNs"])

counters = {}
launch_ns = []
for g in sorted(glob.glob(f"{run}/pmc*_g*/pmc_counter_collection.csv")):
    rows = fifo_rows(g)
    # a pass may hold more than one launch of the kernel (bench.py's untimed first launch):
    # the counters are summed over each launch's rows and averaged over the launches
    n_launch = max(len({r["Dispatch_Id"] for r in rows}), 1)
    for r in rows:
        counters[r["Counter_Name"]] = counters.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"]) / n_launch
        launch_ns.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
summary["pmc_per_launch"] = counters

bench = None
if os.path.exists(f"{run}/bench.json"):
    shutil.copy(f"{run}/bench.json", f"{out}/bench.json")
    with open(f"{run}/bench.json") as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
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
