"""Materialise the C4 job stream in both device forms (GenStream wave writer, then the per-thread
scan with MCS_GEN_SERIAL=1) and check they agree; run under rocprofv3 --kernel-trace --stats to
time gen_stream_kernel against gen_attrs_kernel + gen_arrivals_kernel, and the fused stream's
clock-bound scan gen_bound_wave_kernel against gen_bound_kernel."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multi-cluster-simulator_amd"))
from mcs_amd import Engine, GenParams, replicate, uniform_cluster  # noqa: E402

C, N, J = int(os.environ.get("GT_CLUSTERS", 4096)), 256, int(os.environ.get("GT_JOBS", 16384))
eng = Engine()
eng.load_clusters(replicate(uniform_cluster(N), C))
out = []
for serial in ("0", "1"):
    os.environ["MCS_GEN_SERIAL"] = serial
    eng.generate_jobs(GenParams(seed=7), J)
    out.append(eng.read_jobs())
for f in ("arrival", "dur", "cores", "mem"):
    assert np.array_equal(getattr(out[0], f), getattr(out[1], f)), f
print("forms agree:", C, "clusters x", J, "jobs")
for serial in ("0", "1"):  # the fused stream's clock-bound scan in both forms
    os.environ["MCS_GEN_SERIAL"] = serial
    eng.generate_jobs(GenParams(seed=7, fused=True), J)
eng.close()
