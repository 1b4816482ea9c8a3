"""Summarise rocprofv3 PMC csv files of one gpu_check run: per-placement counters of fifo_kernel."""
import collections
import csv
import glob
import sys

run = sys.argv[1]
jobs = float(sys.argv[2]) if len(sys.argv) > 2 else 67108864.0
for g in sorted(glob.glob(f"{run}/pmc*_g*/pmc_counter_collection.csv")):
    agg = collections.defaultdict(float)
    for row in csv.DictReader(open(g)):
        if any(k in row["Kernel_Name"] for k in ("fifo_kernel", "fifo_asm_kernel")):
            agg[row["Counter_Name"]] += float(row["Counter_Value"])
    print(g.split("/")[-2], {k: round(v / jobs, 3) for k, v in agg.items()})
