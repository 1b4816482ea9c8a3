"""Per-variant pass accounting on the C4 workload: decision passes, release scans, placements and
kernel time, for each libmcs.so given (one subprocess each, MCS_LIB=<path>).

usage: python tools/pass_stats.py lib_a.so [lib_b.so ...]   (env AB_POLICY, AB_NODES, AB_LOAD)"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
sys.path.insert(0, os.path.join(os.environ["REPO"], "multi-cluster-simulator_amd"))
from mcs_amd import Engine, GenParams, replicate, uniform_cluster
from mcs_amd.engine import scaled_lambda
nn, load = int(os.environ.get("AB_NODES", "256")), float(os.environ.get("AB_LOAD", "0.9"))
eng = Engine(0, policy=os.environ.get("AB_POLICY", "FIFO"))
eng.load_clusters(replicate(uniform_cluster(nn), 4096))
eng.generate_jobs(GenParams(arrival_mode=1, lam=scaled_lambda(nn, load=load)), 16384)
eng.run()
st = eng.run()
cs = eng.cluster_stats()
print(json.dumps({"ms": st.kernel_ms, "placed": int(cs["placed"].sum()), "waited": int(cs["waited"].sum()),
                  "iterations": int(cs["iterations"].astype("u8").sum()),
                  "release_scans": int(cs["release_scans"].astype("u8").sum())}))
'''


def main():
    for lib in sys.argv[1:]:
        env = dict(os.environ, MCS_LIB=os.path.abspath(lib), REPO=REPO)
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True)
        if out.returncode != 0:
            print(lib, "failed:", out.stderr[-2000:])
            sys.exit(out.returncode)
        r = json.loads(out.stdout.strip().splitlines()[-1])
        p = r["placed"]
        print(f"{os.path.basename(lib):24s} {r['ms']:8.3f} ms  passes/job {r['iterations'] / p:.3f}  "
              f"release scans/job {r['release_scans'] / p:.3f}  waited/job {r['waited'] / p:.3f}")


if __name__ == "__main__":
    main()
