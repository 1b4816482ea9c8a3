"""Segment times of the one-launch trading tick (mcs_trade_rk.hip) from its probe build
(tools/variant.sh rkst csrc/mcs_trade_rk.hip -DMCS_RK_STAMPS): per tick, averaged over the system's
waves, the time from the launch start to the state loads, to the end of phases B and C/D, to the
applied acceptances, to the end of phase A and to the state stores (s_memrealtime, 100 MHz).
usage: python tools/stamp_rk.py variants/libmcs_rkst.so [jobs_per_cluster]"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MCS_LIB"] = os.path.abspath(sys.argv[1])
os.environ.setdefault("MCS_TRADE_RK", "1")
sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from kat_util import seeded_workload  # noqa: E402
from mcs_amd import Engine  # noqa: E402
from mcs_amd import _lib as L  # noqa: E402

J = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
arrays, streams, _ = seeded_workload("n256", 64, J)
fn = L.lib().mcs_debug_rk_stamps
buf = (C.c_ulonglong * (64 * 14))()
with Engine(0, borrow=True, trader=True, t_max_s=20_000_000) as eng:
    eng.load_clusters(arrays)
    eng.set_shard(0, 1)
    eng.comm_init(Engine.comm_unique_id())
    eng.submit_jobs(streams)
    fn(buf)
    st = eng.run()
    assert fn(buf) == 0
    ts = eng.trade_stats()
ticks = ts["ticks"]
seg = [[buf[w * 14 + i] for i in range(14)] for w in range(64)]
avg = [sum(s[i] for s in seg) / 64 / ticks * 10.0 / 1000.0 for i in range(14)]  # us per tick (100 MHz)
mx = [max(s[i] for s in seg) / ticks * 10.0 / 1000.0 for i in range(14)]
# the launch timeline: per tick, the workgroups' first start, last start and last end
tl = (C.c_ulonglong * (8192 * 16 * 2))()
assert L.lib().mcs_debug_rk_timeline(tl) == 0
nwg = (64 + 3) // 4
lo_t = max(1, ticks - 8192 + 1)
rows = []
for t in range(lo_t, ticks):
    b = (t & 8191) * 16 * 2
    s0 = [tl[b + 2 * w] for w in range(nwg)]
    en = [tl[b + 2 * w + 1] for w in range(nwg)]
    if min(s0) == 0:
        continue
    rows.append((t, min(s0), max(s0), max(en)))
dur = [(r[3] - r[1]) / 100.0 for r in rows]
spread = [(r[2] - r[1]) / 100.0 for r in rows]
gap = [(b[1] - a[3]) / 100.0 for a, b in zip(rows, rows[1:]) if b[0] == a[0] + 1]
timeline = {"ticks_seen": len(rows), "launch_us": round(sum(dur) / max(len(dur), 1), 3),
            "start_spread_us": round(sum(spread) / max(len(spread), 1), 3),
            "gap_to_next_us": round(sum(gap) / max(len(gap), 1), 3),
            "gap_min_us": round(min(gap), 3) if gap else None}
print(json.dumps({"timeline": timeline, "ticks": ticks, "loop_form": ts["loop_form"], "kernel_ms": st.kernel_ms,
                  "us_per_tick": st.kernel_ms * 1e3 / max(ticks, 1),
                  "segments": ["args", "loads_issued", "loads_back_and_barrier", "B_barrier", "apply", "A_record", "state_out", "A_nodes_to_lds", "A_releases", "A_arrivals_decisions", "A_sample_gtable", "lent_log", "CD_wave0", "B"],
                  "avg_us_per_tick": [round(x, 3) for x in avg], "max_wave_us_per_tick": [round(x, 3) for x in mx]}))
