"""Segment cycles of the hand-scheduled FIFO loop from an MCS_STAMPS probe build of
mcs_fifo_asm.hip (tools/variant.sh stamps csrc/mcs_fifo_asm.hip -DMCS_STAMPS): per placement,
the cycles spent in release scans, failed fits, batch ends and the rest (decisions and arrival
advances), at several cluster counts (waves per CU), with the counting build's pass / release counts.
s_memtime stamps wait for their SMEM read, which also drains LDS: read the shares, not the time.
usage: python tools/stamp_fa.py variants/libmcs_stamps.so [clusters ...]"""
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
nc = int(os.environ["NC"])
eng = Engine(0, policy="FIFO")
eng.load_clusters(replicate(uniform_cluster(256), nc))
eng.generate_jobs(GenParams(arrival_mode=1, lam=scaled_lambda(256, load=0.9)), 16384)
fn = L.lib().mcs_debug_fa_stamps
buf = (C.c_ulonglong * 5)()
eng.run(); fn(buf)
st = eng.run(); assert fn(buf) == 0
cs = eng.cluster_stats()
print(json.dumps({"ms": st.kernel_ms, "kernel": eng.last_kernel, "s": list(buf), "jobs": int(eng.num_jobs),
                  "passes": int(cs["iterations"].sum()), "rel": int(cs["release_scans"].sum())}))
'''
lib = sys.argv[1]
for nc in (sys.argv[2:] or ["256", "512", "1024", "4096"]):
    env = dict(os.environ, MCS_LIB=os.path.abspath(lib), REPO=REPO, NC=nc, MCS_FIFO_DIAG="1")
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    if out.returncode:
        print(nc, "FAILED", out.stderr[-1500:])
        sys.exit(1)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    J = d["jobs"]
    rel, nofit, bend, tot = (x / J for x in d["s"][:4])
    rest = tot - rel - nofit - bend
    print(json.dumps({"clusters": int(nc), "kernel_ms": round(d["ms"], 3), "kernel": d["kernel"],
                      "cycles_per_job": {"total": round(tot, 1), "release": round(rel, 1), "nofit": round(nofit, 1),
                                         "batch_end": round(bend, 1), "decide_and_arrive": round(rest, 1)},
                      "release_scans_per_job": round(d["rel"] / J, 4),
                      "cycles_per_release": round(rel * J / max(d["rel"], 1), 1),
                      "passes_per_job": round(d["passes"] / J, 4),
                      "duo_header_rereads_per_job": round(d["s"][4] / J, 4)}), flush=True)
