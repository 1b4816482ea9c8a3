"""GPU parity of the ClusterState reduction (csrc/mcs_state.hip, mcs_cluster_states; SURVEY §8f
row 4): for every cluster of a FIFO or DELAY run and several simulated seconds t, the record equals
the oracle's GetResourceUtilization (oracle/mcs_oracle.c, cluster.go:46-63, float32 in node order)
over the counters rebuilt on the host from the oracle's placements, bit for bit."""
import numpy as np
import pytest

import oracle_ref as O
from kat_util import seeded_workload
from mcs_amd import ClusterArrays, Engine, JobStreams, MCSError
from mcs_amd import wire as W

pytestmark = pytest.mark.gpu


def concat(parts):
    arrays = ClusterArrays(*(np.concatenate([getattr(a, f) for a, _ in parts]) for f in
                             ("cap_c", "cap_m", "free_c", "free_m")),
                           np.concatenate([parts[0][0].node_off] + [
                               sum(int(p[0].node_off[-1]) for p in parts[:i]) + p[0].node_off[1:]
                               for i, p in enumerate(parts) if i > 0]).astype(np.uint32))
    offs, base = [np.zeros(1, np.uint64)], 0
    for _, s in parts:
        offs.append(base + s.job_off[1:])
        base += int(s.job_off[-1])
    streams = JobStreams(*(np.concatenate([getattr(s, f) for _, s in parts]) for f in ("arrival", "dur", "cores", "mem")),
                         np.concatenate(offs).astype(np.uint64))
    return arrays, streams


def expected_states(arrays, streams, node, start, fin, t):
    out = []
    for c in range(arrays.n_clusters):
        ns, js = arrays.nodes_of(c), streams.of(c)
        n = ns.stop - ns.start
        run = (node[js] >= 0) & (start[js] <= t) & (fin[js] > t)
        k = node[js][run]
        uc = np.bincount(k, weights=streams.cores[js][run].astype(np.float64), minlength=n).astype(np.uint64)
        um = np.bincount(k, weights=streams.mem[js][run].astype(np.float64), minlength=n).astype(np.uint64)
        fc = arrays.free_c[ns].astype(np.uint64) - uc
        fm = arrays.free_m[ns].astype(np.uint64) - um
        cu, mu = O.resource_utilization(arrays.cap_c[ns], arrays.cap_m[ns], fc, fm)
        tc = int(arrays.cap_c[ns].astype(np.uint64).sum()) & 0xFFFFFFFF
        tm = int(arrays.cap_m[ns].astype(np.uint64).sum()) & 0xFFFFFFFF
        out.append((np.float32(cu), np.float32(mu), tc, tm, int(run.sum())))
    return out


@pytest.mark.parametrize("policy", ["FIFO", "DELAY"])
def test_gpu_cluster_states_match_oracle(policy):
    arrays, streams = concat([seeded_workload("small", 5, 700)[:2], seeded_workload("big", 3, 700)[:2],
                              seeded_workload("n256_delay" if policy == "DELAY" else "n256", 4, 1500)[:2]])
    if policy == "FIFO":
        node, start, fin, _ = O.fifo_run_batch(arrays, streams, n_threads=8)
    else:
        node, start, fin, _ = O.delay_run_batch(arrays, streams, n_threads=8)
    with Engine(0, policy=policy) as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(streams)
        eng.run()
        gn, gs, gf = eng.placements()
        np.testing.assert_array_equal(gn, node)
        placed = node >= 0
        for t in (0, int(np.median(start[placed])), int(start[placed].max()), int(fin[placed].max()) + 5):
            got = eng.cluster_states(t)
            want = expected_states(arrays, streams, node, start, fin, t)
            for c, (cu, mu, tc, tm, nrun) in enumerate(want):
                g = got[c]
                assert (g["total_cpu"], g["total_memory"], g["running"], g["t_s"]) == (tc, tm, nrun, t), (c, t)
                assert g["cores_utilization"].tobytes() == cu.tobytes(), (c, t)
                assert g["memory_utilization"].tobytes() == mu.tobytes(), (c, t)
        # the Start-stream record of cluster 0 at the last t (totals on the first message)
        rec = W.cluster_state(got[0]["cores_utilization"], got[0]["memory_utilization"], 0.0,
                              totals=(int(got[0]["total_cpu"]), int(got[0]["total_memory"])))
        back = W.unmarshal(W.ClusterState, W.marshal(rec))
        assert back.total_cpu == int(got[0]["total_cpu"]) and back.cores_utilization == 0.0


def test_gpu_cluster_states_refused_after_trading():
    arrays, streams, _ = seeded_workload("small", 3, 200)
    with Engine(0, policy="DELAY", trader=True) as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(streams)
        eng.run()
        with pytest.raises(MCSError):
            eng.cluster_states(100)
