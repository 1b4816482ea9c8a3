"""How often W16L's one-job lookahead can decide a job without a fit test on its
chain, from the oracle's placements of the C4 stream (256 nodes, scaled arrivals at 90 % load).

For each decision k: 'batch' (first job of a 64-record batch: the lookahead is void), 'inval' (a
release happened since decision k - 1: nodes grew), 'cold' (the first fit of job k against the nodes
before commit k - 1 is another node than n(k-1): the L pass decides it), 'hotmiss'/'hothit' (that
first fit IS n(k-1): the F pass re-tests), 'zero_prev' (k - 1 had zero duration: nothing committed).
Also the fraction of consecutive decisions at the same instant.  Test infrastructure (the oracle).
usage: python tools/look_stats.py [clusters]"""
import heapq
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-cluster-simulator_amd"), os.path.join(REPO, "tests")]
import oracle_ref as O  # noqa: E402
from mcs_amd import GenParams  # noqa: E402
from mcs_amd.engine import gen_cluster_host, scaled_lambda  # noqa: E402

N, J = 256, 16384
gp = GenParams(seed=0x4D43535F53494D31, arrival_mode=1, lam=scaled_lambda(N, load=0.9))
tot = dict(dec=0, batch=0, zero_prev=0, inval=0, cold=0, hothit=0, hotmiss=0, nofitpre=0)
same = pairs = 0
for ci in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    a, d, c, m = gen_cluster_host(gp, ci, 32, 24000, J)
    fc0, fm0 = np.full(N, 32, np.int64), np.full(N, 24000, np.int64)
    node, start = O.fifo_run(fc0.astype(np.uint32), fm0.astype(np.uint32), a, d, c, m)[:2]
    fc, fm, heap, prev = fc0.copy(), fm0.copy(), [], None
    for k in range(J):
        if node[k] < 0:
            break
        t, rel = int(start[k]), False
        while heap and heap[0][0] <= t:
            _, n, cc, mm = heapq.heappop(heap)
            fc[n] += cc
            fm[n] += mm
            rel = True
        tot["dec"] += 1
        if k % 64 == 0:
            tot["batch"] += 1
        elif prev is None:
            tot["zero_prev"] += 1
        elif rel:
            tot["inval"] += 1
        else:
            pc, pm = fc.copy(), fm.copy()
            pc[prev[0]] += prev[1]
            pm[prev[0]] += prev[2]
            fit = np.nonzero((pc >= c[k]) & (pm >= m[k]))[0]
            if len(fit) == 0:
                tot["nofitpre"] += 1
            elif fit[0] != prev[0]:
                tot["cold"] += 1
            else:
                tot["hothit" if node[k] == prev[0] else "hotmiss"] += 1
        n = int(node[k])
        if d[k] > 0:
            fc[n] -= c[k]
            fm[n] -= m[k]
            heapq.heappush(heap, (t + int(d[k]), n, int(c[k]), int(m[k])))
            prev = (n, int(c[k]), int(m[k]))
        else:
            prev = None
    st = start.astype(np.int64)
    same += int(np.sum(st[1:] == st[:-1]))
    pairs += J - 1
print({k: (v, round(v / tot["dec"], 4)) for k, v in tot.items()})
print("consecutive decisions at the same instant:", round(same / pairs, 4))
