"""Model check of the duo loop's release protocol (fifo_duo_kernel, mcs_fa_macros.h MCS_FA_SCAN16D /
MCS_FH_LOOP): the decision wave D posts slots and consumes release packets, the release wave H runs
poll steps at random interleavings (also between D's header read and its delta read).  Asserts that
every packet D applies equals the true payload sum of the slots finishing at its second and that D's
next earliest finish stays exact.   usage: python tools/duo_model.py"""
import random
INF = 0xFFFFFFFF
class H:
    def __init__(s, L):
        s.L = L; s.e1 = INF; s.e2 = INF; s.seq = 0; s.cnt = 0; s.slots = []  # (finish, node, pay)
    def pub(s): s.L['hdr'] = (s.e1, s.e2, s.seq, s.cnt)
    def step(s):
        L = s.L
        ack = L['ack']; done = L['done']; ent = L['ring'][s.seq % 128]
        if ent is not None and ent[3] == s.seq:
            kx, f, pay, _ = ent
            s.seq += 1
            s.slots.append([f, kx, pay])
            if f == s.e1:
                L['delta'][kx] = L['delta'].get(kx, 0) + pay; s.cnt += 1
            elif f < s.e1:
                s.e2 = s.e1; s.e1 = f; L['delta'] = {}; L['delta'][kx] = pay; s.cnt = 1
            else:
                s.e2 = min(s.e2, f)
            s.pub(); return True
        if ack == s.e1 and s.e1 != INF:
            L['delta'] = {}
            s.slots = [x for x in s.slots if x[0] != s.e1]
            s.e1 = s.e2; s.cnt = 0; s.e2 = INF
            if s.e1 != INF:
                for f, kx, pay in s.slots:
                    if f == s.e1:
                        L['delta'][kx] = L['delta'].get(kx, 0) + pay; s.cnt += 1
                later = [f for f, _, _ in s.slots if f > s.e1]
                s.e2 = min(later) if later else INF
            s.pub(); return True
        return False

def run(seed):
    rnd = random.Random(seed)
    L = {'ring': [None] * 128, 'hdr': (INF, INF, 0, 0), 'ack': 0, 'done': 0, 'delta': {}}
    h = H(L)
    def maybe_h():
        for _ in range(rnd.choice([0, 0, 1, 2, 5])):
            h.step()
    running = []  # true slots (finish, kx, pay)
    seqD = 0; s77 = INF; lastf = 0; t = 0; used = 0
    for op in range(3000):
        maybe_h()
        # D: either post a slot at t or advance the clock
        if rnd.random() < 0.55:
            f = t + rnd.randint(1, 30); kx = rnd.randrange(256); pay = rnd.randint(1, 5)
            L['ring'][seqD % 128] = (kx, f, pay, seqD)  # (seq written last: model as atomic)
            seqD += 1; lastf = f; s77 = min(s77, f); running.append((f, kx, pay)); used += 1
            # ring overrun guard (batch-end check analogue)
            while seqD - L['hdr'][2] > 64: h.step()
        else:
            t += rnd.choice([1, 1, 2, 5, 20])
            while t >= s77:
                spins = 0
                while True:
                    hdr = L['hdr']; maybe_h(); delta = dict(L['delta'])   # header read, then delta read
                    e1, e2, sh, cnt = hdr; un = seqD - sh
                    ok = un == 0 or (un == 1 and lastf > e1)
                    if ok and un == 1: e2 = min(e2, lastf)
                    if ok and e1 == s77: break
                    h.step(); spins += 1
                    assert spins < 1000, "D waits forever"
                want = {}
                rel = [x for x in running if x[0] == e1]
                for f, kx, pay in rel: want[kx] = want.get(kx, 0) + pay
                assert delta == want, (seed, op, e1, delta, want)
                assert cnt == len(rel)
                running = [x for x in running if x[0] != e1]; used -= cnt
                L['ack'] = e1
                s77 = e2
                truemin = min([x[0] for x in running], default=INF)
                assert s77 == truemin, (seed, op, s77, truemin)
    return True
for seed in range(300): run(seed)
print("ok")
