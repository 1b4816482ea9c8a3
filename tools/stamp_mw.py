"""Segment times of the workgroup-resident lock-step tick (mcs_trade_mw.hip) from an MCS_STAMPS probe
build (tools/variant.sh mw_stamps multi-cluster-simulator_amd/csrc/mcs_trade_mw.hip
-DMCS_STAMPS; MW_WAVES = the build's waves per workgroup, default 4): per tick, each wave's time in phase A's segments (prefetch, releases, arrivals,
decisions, sample + record), the X1 exchange (wave 0 sweeps, the others wait), phase B, its barrier,
X2 + C/D (wave 0) and the loop barrier, on the C5 system (64 clusters x 256 nodes, jobs per cluster
from argv).   usage: python tools/stamp_mw.py variants/libmcs_mw_stamps.so [jobs_per_cluster]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import ctypes as C, json, os, sys
sys.path.insert(0, os.path.join(os.environ["REPO"], "multi-cluster-simulator_amd"))
from mcs_amd import Engine, GenParams, replicate, uniform_cluster
from mcs_amd import _lib as L
from mcs_amd.engine import scaled_lambda
J = int(os.environ["JOBS"])
eng = Engine(0, borrow=True, trader=True)
eng.load_clusters(replicate(uniform_cluster(256), 64))
eng.generate_jobs(GenParams(seed=1, arrival_mode=1, lam=scaled_lambda(256, load=0.9)), J)
fn = L.lib().mcs_debug_mw_stamps
buf = (C.c_ulonglong * 768)()
WV = int(os.environ.get("MW_WAVES", "4")); NWG = 64 // WV
tl = (C.c_ulonglong * (1024 * NWG * (2 * WV + 3)))()
eng.run(); fn(buf)
st = eng.run(); assert fn(buf) == 0
assert L.lib().mcs_debug_mw_tlog(tl) == 0
ts = eng.trade_stats()
print(json.dumps({"ms": st.kernel_ms, "ticks": int(ts["ticks"]), "loop_form": int(ts["loop_form"]),
                  "slot_pool": int(st.slot_pool), "s": list(buf), "tl": list(tl), "wv": WV}))
'''
SEG = ["prefetch", "releases", "arrivals", "decisions", "sample+record", "X1_sweep_or_wait",
       "phase_B", "barrier_B", "X2+CD", "barrier_loop"]


def main():
    lib = sys.argv[1]
    jobs = sys.argv[2] if len(sys.argv) > 2 else "20000"
    env = dict(os.environ, MCS_LIB=os.path.abspath(lib), REPO=REPO, JOBS=jobs)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode:
        print("FAILED", out.stderr[-2000:])
        sys.exit(1)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    ticks = d["ticks"]
    s = d["s"]
    wv = d["wv"]
    nwg = 64 // wv
    per_wave = [[s[w * 12 + i] * 10.0 / 1e3 / ticks for i in range(10)] for w in range(64)]  # us per tick
    passes = [(s[w * 12 + 10] / ticks, s[w * 12 + 11] / ticks) for w in range(0, 64, wv)]  # wave 0 of each wg
    res = {"jobs_per_cluster": int(jobs), "ticks": ticks, "kernel_ms": round(d["ms"], 3), "waves_per_workgroup": wv,
           "us_per_tick": round(d["ms"] * 1e3 / ticks, 3), "loop_form": d["loop_form"], "slot_pool": d["slot_pool"],
           "us_per_tick_wg0_wave0": {SEG[i]: round(per_wave[0][i], 3) for i in range(10)},
           "us_per_tick_wg0_wave1": {SEG[i]: round(per_wave[1][i], 3) for i in range(10)},
           "us_per_tick_max_over_waves": {SEG[i]: round(max(w[i] for w in per_wave), 3) for i in range(10)},
           "us_per_tick_mean_over_waves": {SEG[i]: round(sum(w[i] for w in per_wave) / 64, 3) for i in range(10)},
           "sweep_passes_per_tick_x1_x2_by_wg": [[round(a, 2), round(b, 2)] for a, b in passes]}
    # the X1 wait split (absolute times of every 64th tick of the last launch, 10 ns units): skew =
    # the last record's publication after this workgroup's wave 0 stored its own; propagation =
    # wave 0's sweep end after the last publication; first_pass = its first sweep's end after the last
    # publication (negative: the first pass ran before the last record existed).  Slots per workgroup:
    # [0, wv) each wave's publication, [wv, 2 wv) its X1 barrier arrival, 2 wv first sweep pass, 2 wv + 1
    # sweep end, 2 wv + 2 wave 0 past the barrier
    import numpy as np
    ns = 2 * wv + 3
    raw = np.array(d["tl"], dtype=np.int64).reshape(1024, nwg, ns)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(REPO, "gpurun_out", "mw_tlog.npy"), raw)
    tl = raw[(raw[:, :, [0, 2 * wv + 1, 2 * wv + 2]] > 0).all(axis=(1, 2))]
    us = lambda x: x * 10.0 / 1e3  # noqa: E731  (100 MHz ticks)
    pub, arr = tl[:, :, :wv], tl[:, :, wv:2 * wv]
    last_pub = pub.max(axis=(1, 2))
    last_w = pub.reshape(len(tl), -1).argmax(axis=1)
    done, after = tl[:, :, 2 * wv + 1], tl[:, :, 2 * wv + 2]
    res["x1_split_us"] = {
        "ticks_logged": int(len(tl)),
        "wave0_pub_to_sweep_end": round(float(us(done - tl[:, :, 0]).mean()), 3),
        "skew_last_pub_after_wave0_pub": round(float(us(last_pub[:, None] - tl[:, :, 0]).mean()), 3),
        "propagation_sweep_end_after_last_pub": round(float(us(done - last_pub[:, None]).mean()), 3),
        "first_pass_after_last_pub": round(float(us(tl[:, :, 2 * wv] - last_pub[:, None]).mean()), 3),
        "sweep_end_to_past_barrier": round(float(us(after - done).mean()), 3),
        "last_barrier_arrival_after_sweep_end": round(float(us(arr.max(axis=2) - done).mean()), 3),
        "pub_to_barrier_arrival_by_wave_mean": [round(float(x), 3) for x in us(arr - pub).mean(axis=(0, 1))],
        "x1_segment_total_wave0": round(float(us(after - tl[:, :, 0]).mean()), 3),
        "last_publisher_top": [[int(c), int(k)] for c, k in zip(*np.unique(last_w, return_counts=True))
                               if k >= max(1, len(tl) // 50)],
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
