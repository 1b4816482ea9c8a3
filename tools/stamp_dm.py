"""Tick timeline of dt_mw_kernel (the resident DELAY-trading tick, mcs_dtrade_mw.hip) from an
MCS_STAMPS probe build (tools/variant.sh dm_stamps multi-cluster-simulator_amd/csrc/mcs_dtrade_mw.hip
-DMCS_STAMPS), on the C5-DELAY system (64 cluster_small clusters, jobs per cluster from argv).
usage: python tools/stamp_dm.py variants/libmcs_dm_stamps.so [jobs_per_cluster]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import ctypes as C, json, os, sys
sys.path.insert(0, os.path.join(os.environ["REPO"], "multi-cluster-simulator_amd"))
from mcs_amd import Engine, GenParams, replicate
from mcs_amd.cluster import Cluster
from mcs_amd import _lib as L
J = int(os.environ["JOBS"])
spec = Cluster.load(os.path.join(os.environ["REPO"], "assets", "cluster_small.json"))
eng = Engine(0, policy="DELAY", trader=True)
eng.load_clusters(replicate(spec, 64))
eng.generate_jobs(GenParams(seed=0x4D43535F53494D31), J)
fn = L.lib().mcs_debug_dm_stamps
buf = (C.c_ulonglong * (64 * 6 + 16))()
rows = (C.c_ulonglong * 21)()
fr = L.lib().mcs_debug_dm_rows
eng.run(); assert fn(buf) == 0 and fr(rows) == 0
st = eng.run(); assert fn(buf) == 0 and fr(rows) == 0
ts = eng.trade_stats()
print(json.dumps({"ms": st.kernel_ms, "ticks": int(ts["ticks"]), "loop_form": int(ts["loop_form"]), "s": list(buf),
                  "rows": list(rows)}))
'''
SEG = ["phase_a", "sample", "record+snapshot+contracts+x1_put", "x2_wait", "side_effects"]
US = 10.0 / 1e3  # s_memrealtime ticks (100 MHz) -> us


def main():
    lib = sys.argv[1]
    jobs = sys.argv[2] if len(sys.argv) > 2 else "2000"
    env = dict(os.environ, MCS_LIB=os.path.abspath(lib), REPO=REPO, JOBS=jobs)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode:
        print("FAILED", out.stderr[-2000:])
        sys.exit(1)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    s = d["s"]
    cl = [s[6 * c:6 * c + 6] for c in range(64)]
    tr = s[64 * 6:64 * 6 + 16]
    nt = max(tr[3], 1)
    res = {"jobs_per_cluster": int(jobs), "ticks": d["ticks"], "loop_form": d["loop_form"],
           "us_per_tick": round(d["ms"] * 1e3 / d["ticks"], 3)}
    # the mean over clusters of each segment per tick, and the busiest cluster's
    per = [[x[i] * US / max(x[5], 1) for i in range(5)] for x in cl if x[5]]
    res["cluster_mean_us_per_tick"] = {SEG[i]: round(sum(p[i] for p in per) / len(per), 3) for i in range(5)}
    busy = min(per, key=lambda p: p[3])
    res["busiest_cluster_us_per_tick"] = {SEG[i]: round(busy[i], 3) for i in range(5)}
    res["trader_us_per_tick"] = {"x1_wait": round(tr[0] * US / nt, 3), "rounds": round(tr[1] * US / nt, 3),
                                 "next_clock+x2_put": round(tr[2] * US / nt, 3)}
    TSEG = ["work(side_effects+phase_a+sample+record)", "phase_a", "releases", "arrivals+first_row_loads",
            "level1_pass", "level0_head", "sample", "record+snapshot+contracts+x1_put"]
    res["per_tick_slowest_wave_us"] = {TSEG[i]: round(tr[8 + i] * US / nt, 3) for i in range(8)}
    res["ticks_with_a_round_due"] = tr[6]
    res["exchange_us_per_tick"] = round((tr[0] - tr[8]) * US / nt, 3)
    rw = d["rows"]
    np_ = max(rw[5], 1)
    res["level1"] = {"passes": rw[5], "passes_per_tick": round(rw[5] / nt, 3),
                     "us_per_pass": round(rw[7] * US / np_, 3),
                     "general_rows_per_pass": round(rw[2] / np_, 2), "quiet_rows_per_pass": round(rw[4] / np_, 2),
                     "candidates_per_pass": round(rw[6] / np_, 2), "placements_per_pass": round(rw[3] / np_, 2),
                     "us_per_general_row_tests_and_placements": round(rw[0] * US / max(rw[2], 1), 3),
                     "us_per_general_row_bookkeeping": round(rw[1] * US / max(rw[2], 1), 3),
                     "us_per_pass_setup": round(rw[8] * US / np_, 3), "us_per_pass_row_loop": round(rw[9] * US / np_, 3),
                     "us_per_pass_end": round(rw[10] * US / np_, 3)}
    for i, nm in enumerate(("quiet_pairs_unshifted", "quiet_pairs_shifted", "other_pairs")):
        res["level1"][nm] = {"per_pass": round(rw[12 + 2 * i] / np_, 2),
                             "us_each": round(rw[11 + 2 * i] * US / max(rw[12 + 2 * i], 1), 3)}
    res["trader_steps"] = {"requests": rw[18], "us_per_request": round(rw[17] * US / max(rw[18], 1), 3),
                           "other_steps": rw[20], "us_per_other_step": round(rw[19] * US / max(rw[20], 1), 3)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
