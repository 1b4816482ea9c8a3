"""Tiny hand-scheduled-loop cases per form (MCS_FIFO_ASM=16|17|32 vs 0), printed next to the
oracle: a debugging aid for mcs_fifo_asm.hip (one GPU, a few ms)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(os.environ["REPO"], "multi-cluster-simulator_amd"))
sys.path.insert(0, os.path.join(os.environ["REPO"], "tests"))
from mcs_amd import Engine, JobStreams, replicate, uniform_cluster
import oracle_ref as O
cases = []
n = 12
cases.append(("fill", np.zeros(n, np.uint32), np.full(n, 100, np.uint32), np.full(n, 32, np.uint32), np.full(n, 1, np.uint32)))
cases.append(("half", np.zeros(n, np.uint32), np.full(n, 100, np.uint32), np.full(n, 16, np.uint32), np.full(n, 1, np.uint32)))
a = np.arange(n, dtype=np.uint32); cases.append(("release", a, np.full(n, 3, np.uint32), np.full(n, 32, np.uint32), np.full(n, 24000, np.uint32)))
out = {}
for name, arr, dur, c, m in cases:
    arrays = replicate(uniform_cluster(256), 1)
    s = JobStreams(arr, dur, c, m, np.array([0, n], np.uint64))
    with Engine(0) as eng:
        eng.load_clusters(arrays); eng.submit_jobs(s); eng.run()
        node, start, fin = eng.placements()
        k = eng.last_kernel
    on, os_, of, _ = O.fifo_run_batch(arrays, s, n_threads=1)
    out[name] = {"kernel": k, "gpu": node.tolist(), "start": start.tolist(), "oracle": on.tolist(), "ostart": os_.tolist()}
print(json.dumps(out))
'''
for form in sys.argv[1:] or ["0", "32", "16", "1"]:
    env = dict(os.environ, REPO=REPO, MCS_FIFO_ASM=form)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
    print("MCS_FIFO_ASM", form, r.returncode)
    print(r.stdout.strip()[-4000:] or r.stderr[-2000:], flush=True)
