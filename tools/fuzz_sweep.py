"""Run the GPU fuzz parity cases over a range of fresh seeds (beyond the ones the test suite pins)
and report every failing (test, shape/policy, seed); exit status 1 if any failed.

    python tools/fuzz_sweep.py BASE COUNT      (SWEEP_BIG=1: larger FIFO and DELAY cases only;
                                                SWEEP_DT=1: the DELAY-trading cases only)
"""
import os
import sys
import time
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import test_gpu_delay as TD  # noqa: E402
import test_gpu_dtrade as TDT  # noqa: E402
import test_gpu_fused as TF  # noqa: E402
import test_gpu_online as TO  # noqa: E402
import test_gpu_parity as TP  # noqa: E402
import test_gpu_trade as TT  # noqa: E402
from mcs_amd import Engine  # noqa: E402



class _MonkeyPatch:
    """The part of pytest's monkeypatch fixture the fuzz tests use (environment variables)."""

    def __init__(self):
        self.saved = {}

    def setenv(self, k, v):
        self.saved.setdefault(k, os.environ.get(k))
        os.environ[k] = v

    def delenv(self, k, raising=True):
        self.saved.setdefault(k, os.environ.get(k))
        os.environ.pop(k, None)

    def undo(self):
        for k, v in self.saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def fifo_fuzz(eng, shape, seed):
    mp = _MonkeyPatch()
    try:
        TP.test_hand_scheduled_fuzz(eng, shape, seed, mp)
    finally:
        mp.undo()


base, count = int(sys.argv[1]), int(sys.argv[2])
fails, runs = [], 0
t0 = time.time()
with Engine(0) as eng, Engine(0, policy="DELAY") as deng:
    for seed in range(base, base + count):
        cases = [(f"fifo/{s}", lambda s=s: fifo_fuzz(eng, s, seed)) for s in ("w16s", "w16r", "duo", "look", "w32")]
        cases += [(f"delay/{s}", lambda s=s: TD.test_gpu_delay_fuzz(deng, s, seed)) for s in ("w16s", "mid", "w16r", "w32")]
        cases += [(f"fused/{p}", lambda p=p: TF.test_fused_fuzz(p, seed)) for p in ("FIFO", "DELAY")]
        cases += [(f"online/{p}/{s}", lambda p=p, s=s: TO.test_online_fuzz_slices_equal_batch_and_oracle(p, s, seed))
                  for p in ("FIFO", "DELAY") for s in ("w16s", "w16r", "w32")]
        cases += [(f"trade/{s}", lambda s=s: TT.test_gpu_trade_fuzz(s, seed)) for s in ("w16s", "mid", "w16r")]
        cases += [(f"dtrade/{s}", lambda s=s: TDT.test_gpu_dtrade_fuzz(s, seed, 600)) for s in ("w16s", "mid")]
        if os.environ.get("SWEEP_BIG"):  # FIFO 600 x 6000, DELAY 400 x 5000 jobs per case
            def big(shape, seed=seed):
                arrays, st = TP.fuzz_workload(shape, seed, n_clusters=600, J=6000)
                node, start, fin, _, cs = TP.run_engine(eng, arrays, st)
                TP.assert_parity(arrays, st, node, start, fin, cs)
            def dbig(shape, seed=seed):
                arrays, st = TP.fuzz_workload(shape, seed, n_clusters=400, J=5000)
                node, start, fin, _, cs, ds = TD.run(deng, arrays, st)
                TD.assert_delay_parity(arrays, st, node, start, fin, cs, ds)
            cases = [(f"fifo-big/{s}", lambda s=s: big(s)) for s in ("w16s", "mid", "w16r", "w32")]
            cases += [(f"delay-big/{s}", lambda s=s: dbig(s)) for s in ("w16s", "mid", "w16r", "w32")]
            if os.environ.get("SWEEP_TRADE"):  # trading systems: 32 clusters x 2000 jobs instead
                def tbig(shape, seed=seed):
                    arrays, st = TP.fuzz_workload(shape, seed, n_clusters=32, J=2000, blocking=False)
                    TT.assert_trade_parity(arrays, st, TT.gpu_trade(arrays, st))
                def dtbig(shape, seed=seed):  # DELAY trading: placements against the oracle
                    arrays, st = TP.fuzz_workload(shape, seed, n_clusters=16, J=800, blocking=False)
                    g, o = TDT.run(arrays, st), TDT.O.dtrade_run(arrays, st)
                    for k in ("node", "start", "finish"):
                        assert (g[k] == o[k]).all(), k
                cases = [(f"trade-big/{s}", lambda s=s: tbig(s)) for s in ("w16s", "mid", "w16r")]
                cases += [(f"dtrade-big/{s}", lambda s=s: dtbig(s)) for s in ("w16s", "mid")]
        if os.environ.get("SWEEP_DT"):  # DELAY trading only: the fuzz cases and 16 x 800-job systems
            def dtsys(shape, seed=seed):
                arrays, st = TP.fuzz_workload(shape, seed, n_clusters=16, J=800, blocking=False)
                g, o = TDT.run(arrays, st), TDT.O.dtrade_run(arrays, st)
                for k in ("node", "start", "finish"):
                    assert (g[k] == o[k]).all(), k
                assert g["ts"]["t_final"] == o["t_final"] and g["ts"]["loop_form"] == 5
            cases = [(f"dtrade/{s}", lambda s=s: TDT.test_gpu_dtrade_fuzz(s, seed, 600)) for s in ("w16s", "mid")]
            cases += [(f"dtrade-sys/{s}", lambda s=s: dtsys(s)) for s in ("w16s", "mid")]
        for name, fn in cases:
            runs += 1
            if os.environ.get("SWEEP_VERBOSE"):
                print(f"  {name} seed {seed} ...", flush=True)
            try:
                fn()
            except Exception:  # noqa: BLE001 - report and continue with the next case
                fails.append((name, seed))
                print(f"FAIL {name} seed {seed}\n{traceback.format_exc(limit=3)}", flush=True)
        print(f"seed {seed}: {runs} cases run, {len(fails)} failed, {time.time() - t0:.0f} s", flush=True)
print("failures:", fails)
sys.exit(1 if fails else 0)
