"""Segment shares of fifo_kernel's pass loop from an MCS_STAMPS diagnostic build (s_memtime
stamps; read the shares, not the run time).  usage: python tools/stamp_probe.py variants/libmcs_st_*.so"""
import ctypes as C
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
nn, load = int(os.environ.get("AB_NODES", "256")), float(os.environ.get("AB_LOAD", "0.9"))
eng = Engine(0, policy="FIFO")
eng.load_clusters(replicate(uniform_cluster(nn), 4096))
eng.generate_jobs(GenParams(arrival_mode=1, lam=scaled_lambda(nn, load=load)), 16384)
eng.run()
buf = (C.c_ulonglong * 8)()
L.lib().mcs_debug_stamps(buf)
st = eng.run()
assert L.lib().mcs_debug_stamps(buf) == 0
print(json.dumps({"ms": st.kernel_ms, "s": list(buf)}))
'''
for lib in sys.argv[1:]:
    env = dict(os.environ, MCS_LIB=os.path.abspath(lib), REPO=REPO)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True)
    if out.returncode:
        print(lib, out.stderr[-1500:])
        continue
    r = json.loads(out.stdout.strip().splitlines()[-1])
    s = r["s"]
    n = s[4]
    print(f"{os.path.basename(lib)} {r['ms']:.2f} ms passes {n} (deciding {s[6] / n:.3f}, releasing {s[5] / n:.3f})")
    for name, v in zip(("decide", "place", "release", "reload"), s[:4]):
        print(f"   {name:8s} {v / n:8.1f} cyc/pass")
    print(f"   total    {sum(s[:4]) / n:8.1f} cyc/pass")
