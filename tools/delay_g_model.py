"""Model of the hand-scheduled DELAY loop's Level1 pass (mcs_delay_asm.hip, r04) in plain Python,
checked against the CPU oracle on randomised clusters: the algorithm, not the asm.

The loop runs a pass only when a node grew since the last pass (a release) or a D6-skipped job
("untested") waits, and tests a Level1 job only against the grown nodes G (their current values):
every other job failed every node at its last test and nodes only shrink between releases.  This
model restates exactly that (grown set against a snapshot taken at the end of each pass and lowered
to the nodes' values at every Level1 move, componentwise, since the moved job was tested then; untested
marks, the D6 skip on list positions, first fit over all nodes, the event fast-forward) and must
give the oracle's placements bit for bit.

usage: python tools/delay_g_model.py [n_cases]      (CPU only; uses tests/oracle_ref.py)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd"))

EMPTY = 0xFFFFFFFF


def model(fc, fm, jobs, max_wait=10):
    """One cluster: fc, fm free vectors (lists), jobs = list of (arrival, dur, cores, mem) sorted by
    arrival.  Returns node, start lists (node -1 / start EMPTY if never placed)."""
    N = len(fc)
    J = len(jobs)
    node = [-1] * J
    start = [EMPTY] * J
    running = []  # (finish, k, c, m)
    l1 = []  # [c, m, row, dur, untested]
    snap = (list(fc), list(fm))
    released = False
    untested = 0
    h = 0
    t = 0
    if J == 0:
        return node, start

    def first_fit(c, m):
        for k in range(N):
            if fc[k] >= c and fm[k] >= m:
                return k
        return -1

    def commit(k, c, m, row, dur):
        node[row] = k
        start[row] = t
        if dur:
            fc[k] -= c
            fm[k] -= m
            running.append((t + dur, k, c, m))

    while True:
        # releases at t (cluster.go:153-157)
        keep = []
        for r in running:
            if r[0] <= t:
                fc[r[1]] += r[2]
                fm[r[1]] += r[3]
                released = True
            else:
                keep.append(r)
        running = keep
        changed = False
        # ---- the Level1 pass ----
        if l1 and (released or untested):
            G = []
            if released:
                G = [k for k in range(N) if fc[k] > snap[0][k] or fm[k] > snap[1][k]]
                released = False
            if G or untested:
                skip = -1
                out = []
                for i, e in enumerate(l1):
                    cand = e[4] or any(fc[k] >= e[0] and fm[k] >= e[1] for k in G)
                    if i == skip:
                        if cand and not e[4]:
                            e[4] = True
                            untested += 1
                        out.append(e)
                        continue
                    if not cand:
                        out.append(e)
                        continue
                    if e[4]:
                        e[4] = False
                        untested -= 1
                    k = first_fit(e[0], e[1])
                    if k < 0:
                        out.append(e)
                        continue
                    commit(k, e[0], e[1], e[2], e[3])
                    skip = i + 1
                    changed = True
                l1 = out
                snap = (list(fc), list(fm))
        # ---- the Level0 head ----
        if h < J and jobs[h][0] <= t:
            a, d, c, m = jobs[h]
            k = first_fit(c, m)
            if k >= 0:
                commit(k, c, m, h, d)
                h += 1
                changed = True
            elif t - a >= max_wait:
                # the moved job failed every node as they are now: the snapshot may not exceed them
                if not l1:
                    snap = (list(fc), list(fm))
                    released = False
                else:
                    snap = ([min(x, y) for x, y in zip(snap[0], fc)], [min(x, y) for x, y in zip(snap[1], fm)])
                l1.append([c, m, h, d, False])
                h += 1
                changed = True
        if h >= J and not l1:
            return node, start
        if changed:
            t += 1
            continue
        nf = min((r[0] for r in running), default=EMPTY)
        ev = nf
        if h < J:
            a = jobs[h][0]
            e2 = a + max_wait if a <= t else a
            ev = min(ev, e2)
        if ev == EMPTY:
            return node, start  # deadlock: Level1 never fits
        t = max(t + 1, ev)


def main():
    import oracle_ref as O
    from kat_util import fuzz_workload
    from mcs_amd import JobStreams, pack_clusters
    from mcs_amd.cluster import Cluster, Node

    n_cases = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    bad = 0
    for seed in range(n_cases):
        rng = np.random.default_rng(seed)
        nn = int(rng.integers(2, 24))
        cap_c, cap_m = int(rng.integers(1, 40)), int(rng.integers(100, 5000))
        fc = [cap_c if rng.random() < 0.7 else int(rng.integers(0, cap_c + 1)) for _ in range(nn)]
        fm = [cap_m if rng.random() < 0.7 else int(rng.integers(0, cap_m + 1)) for _ in range(nn)]
        J = int(rng.integers(50, 600))
        arr = np.cumsum(rng.poisson(rng.uniform(0.2, 2.5), J)).astype(np.uint32)
        dur = rng.integers(0, int(rng.integers(2, 200)), J).astype(np.uint32)
        c = rng.integers(0, cap_c + 1, J).astype(np.uint32)
        m = rng.integers(0, cap_m + 1, J).astype(np.uint32)
        if rng.random() < 0.3:
            c[int(rng.integers(0, J))] = cap_c + 1  # a job that never fits: a Level1 deadlock
        cl = Cluster(Id=1, Nodes=[Node(Id=i + 1, Cores=cap_c, Memory=cap_m, CoresAvailable=fc[i],
                                       MemoryAvailable=fm[i]) for i in range(nn)])
        arrays = pack_clusters([cl])
        s = JobStreams(arr, dur, c, m, np.array([0, J], np.uint64))
        on, os_, _, _ = O.delay_run_batch(arrays, s)
        jobs = list(zip(arr.tolist(), dur.tolist(), c.tolist(), m.tolist()))
        gn, gs = model(list(fc), list(fm), jobs)
        ok = (np.array(gn) == on).all() and (np.array(gs, np.uint32) == os_).all()
        if not ok:
            bad += 1
            i = int(np.nonzero((np.array(gn) != on) | (np.array(gs, np.uint32) != os_))[0][0])
            print(f"seed {seed}: first mismatch at job {i}: model {gn[i]},{gs[i]} oracle {on[i]},{os_[i]}")
    print(f"{n_cases - bad}/{n_cases} cases equal the oracle")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
