import os, sys
import numpy as np
REPO = "/root/repo"
sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import test_gpu_online as T
import oracle_ref as O
from kat_util import fuzz_workload
arrays, streams = fuzz_workload("w16s", 1, n_clusters=48, J=1200)
b = T.batch(arrays, streams, policy="DELAY")
on, os_, of, osd = O.delay_run_batch(arrays, streams, n_threads=8)
hs = T.horizons_for(streams, 6)
g = T.run_online(arrays, streams, hs, policy="DELAY")
bad = np.flatnonzero(g[4]["t_end"] != osd["t_end"])
print("horizons", hs)
print("batch t_end == oracle:", np.array_equal(b[4]["t_end"], osd["t_end"]))
for c in bad[:6]:
    sl = streams.of(int(c))
    print("cluster", c, "online", g[4][c], "oracle t_end", osd["t_end"][c], "flags", osd["flags"][c],
          "last arrival", int(streams.arrival[sl].max()), "max finish", int(of[sl].max()), "unplaced", int((on[sl] < 0).sum()),
          "l1_left", g[5]["l1_left"][c], osd["l1_left"][c])
