"""Segment times of dt_step_kernel (the DELAY-trading phase A, mcs_dtrade.hip) from an MCS_STAMPS probe
build (OBJ=mcs_dtrade_k tools/variant.sh dt_stamps multi-cluster-simulator_amd/csrc/mcs_dtrade.hip
-DMCS_STAMPS), per dt_step call (one cluster's step of one tick), on the C5-DELAY system (64
cluster_small clusters, jobs per cluster from argv), graph-replayed loop.
usage: python tools/stamp_dt.py variants/libmcs_dt_stamps.so [jobs_per_cluster]"""
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
fn = L.lib().mcs_debug_dt_stamps
fm = L.lib().mcs_debug_dt_maxsum
fr = L.lib().mcs_debug_dt_rows
buf = (C.c_ulonglong * 8)()
mx = (C.c_ulonglong * 10)()
rw = (C.c_ulonglong * 4)()
eng.run(); fn(buf); fm(mx); fr(rw)
st = eng.run(); assert fn(buf) == 0 and fm(mx) == 0 and fr(rw) == 0
ts = eng.trade_stats()
print(json.dumps({"ms": st.kernel_ms, "ticks": int(ts["ticks"]), "loop_form": int(ts["loop_form"]), "s": list(buf),
                  "mx": list(mx), "rw": list(rw)}))
'''
SEG = ["state_in+lds_copies", "releases", "arrivals", "level1_pass", "level0_head", "copies_out+sample",
       "record+snapshot+contracts"]


def main():
    lib = sys.argv[1]
    jobs = sys.argv[2] if len(sys.argv) > 2 else "2000"
    env = dict(os.environ, MCS_LIB=os.path.abspath(lib), REPO=REPO, JOBS=jobs)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode:
        print("FAILED", out.stderr[-2000:])
        sys.exit(1)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    s, calls = d["s"], max(d["s"][7], 1)
    res = {"jobs_per_cluster": int(jobs), "ticks": d["ticks"], "loop_form": d["loop_form"],
           "us_per_tick": round(d["ms"] * 1e3 / d["ticks"], 3), "dt_step_calls": calls,
           "us_per_dt_step_call": {SEG[i]: round(s[i] * 10.0 / 1e3 / calls, 3) for i in range(7)},
           "us_per_dt_step_call_total": round(sum(s[:7]) * 10.0 / 1e3 / calls, 3)}
    mx, nt = d["mx"], max(d["mx"][9], 1)
    res["per_tick_slowest_cluster_us"] = {SEG[i]: round(mx[i] * 10.0 / 1e3 / nt, 3) for i in range(7)}
    res["per_tick_slowest_step_us"] = round(mx[7] * 10.0 / 1e3 / nt, 3)
    res["per_tick_trader_kernel_us"] = round(mx[8] * 10.0 / 1e3 / nt, 3)
    rw = d["rw"]
    nr = max(rw[2], 1)
    res["level1_rows"] = {"rows": rw[2], "placements": rw[3], "rows_per_tick": round(rw[2] / nt, 2),
                          "us_per_row_tests_and_placements": round(rw[0] * 10.0 / 1e3 / nr, 4),
                          "us_per_row_bookkeeping": round(rw[1] * 10.0 / 1e3 / nr, 4)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
