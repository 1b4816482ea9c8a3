"""The release scans of the C4 workload, from the FIFO oracle's placements (CPU): the clock values
the hand-scheduled loop visits (arrivals, starts, a placed WaitQueue head's next second, the finish
seconds a waiting head sleeps through) and, between consecutive ones, how many distinct finish
seconds a release scan hands back.  Pins two facts the low-occupancy designs rest on:
0.554 scans per job, the counting build's figure on the GPU (profiles/r03_b512/stamps_w16r.txt), and
nearly every scan releasing exactly one finish second."""
import numpy as np

import oracle_ref as O
from mcs_amd import GenParams, gen_streams_host, replicate, uniform_cluster
from mcs_amd.engine import scaled_lambda


def test_c4_release_scans_are_single_second():
    arrays = replicate(uniform_cluster(256), 4)
    gp = GenParams(seed=0x4D43535F53494D31, arrival_mode=1, lam=scaled_lambda(256, load=0.9))
    J = 16384
    streams = gen_streams_host(gp, arrays, J)
    node, start, fin, _ = O.fifo_run_batch(arrays, streams, n_threads=4)
    scans, counts = 0, []
    for k in range(4):
        s = streams.of(k)
        a, st, f, d = streams.arrival[s], start[s], fin[s], streams.dur[s]
        waited = st > a
        fins = np.unique(f[d > 0])
        visit = set(a.tolist()) | set(st.tolist()) | set((st[waited] + 1).tolist())
        for j in np.nonzero(waited)[0]:
            visit |= set(fins[(fins > a[j]) & (fins <= st[j])].tolist())
        v = np.array(sorted(visit))
        c = np.diff(np.searchsorted(fins, v, side="right"))
        c = c[c > 0]
        scans += len(c)
        counts.append(c)
    c = np.concatenate(counts)
    assert abs(scans / (4 * J) - 0.554) < 0.01
    assert (c == 1).mean() > 0.99
