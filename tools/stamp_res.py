"""Segment times of the resident lock-step tick (mcs_trade_res.hip) from an MCS_STAMPS probe build
(tools/variant.sh res_stamps multi-cluster-simulator_amd/csrc/mcs_trade_res.hip -DMCS_STAMPS):
per tick, each wave's time in the phase-A segments (prefetch, releases, arrivals, decisions,
sample + record), phase B, phase C+D and the three barrier waits, on the C5 system (64 clusters x
256 nodes, jobs per cluster from argv).  s_memrealtime stamps wait for outstanding LDS reads: read
the shares.   usage: python tools/stamp_res.py variants/libmcs_res_stamps.so [jobs_per_cluster]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import ctypes as C, json, os, sys
sys.path.insert(0, os.path.join(os.environ["REPO"], "multi-cluster-simulator_amd"))
from mcs_amd import Engine, GenParams, replicate, uniform_cluster
from mcs_amd import _lib as L
from mcs_amd.engine import scaled_lambda
J = int(os.environ["JOBS"])
eng = Engine(0, borrow=True, trader=True)
eng.load_clusters(replicate(uniform_cluster(256), 64))
eng.generate_jobs(GenParams(seed=1, arrival_mode=1, lam=scaled_lambda(256, load=0.9)), J)
fn = L.lib().mcs_debug_res_stamps
buf = (C.c_ulonglong * 160)()
eng.run(); fn(buf)
st = eng.run(); assert fn(buf) == 0
ts = eng.trade_stats()
print(json.dumps({"ms": st.kernel_ms, "ticks": int(ts["ticks"]), "loop_form": int(ts["loop_form"]),
                  "slot_pool": int(st.slot_pool), "s": list(buf)}))
'''
SEG = ["prefetch+sample_check", "releases", "arrivals", "decisions", "sample+record", "barrier_A",
       "phase_B", "barrier_B", "phase_CD", "barrier_CD+loop"]


def main():
    lib = sys.argv[1]
    jobs = sys.argv[2] if len(sys.argv) > 2 else "20000"
    env = dict(os.environ, MCS_LIB=os.path.abspath(lib), REPO=REPO, JOBS=jobs)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode:
        print("FAILED", out.stderr[-2000:])
        sys.exit(1)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    ticks = d["ticks"]
    s = d["s"]
    per_wave = [[s[w * 10 + i] * 10.0 / 1e3 / ticks for i in range(10)] for w in range(16)]  # us per tick
    res = {"jobs_per_cluster": int(jobs), "ticks": ticks, "kernel_ms": round(d["ms"], 3),
           "us_per_tick": round(d["ms"] * 1e3 / ticks, 3), "loop_form": d["loop_form"], "slot_pool": d["slot_pool"],
           "us_per_tick_wave0": {SEG[i]: round(per_wave[0][i], 3) for i in range(10)},
           "us_per_tick_max_over_waves": {SEG[i]: round(max(w[i] for w in per_wave), 3) for i in range(10)},
           "us_per_tick_mean_over_waves": {SEG[i]: round(sum(w[i] for w in per_wave) / 16, 3) for i in range(10)}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
