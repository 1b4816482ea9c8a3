"""A/B timing of libmcs.so kernel variants on the C4 workload in ONE process per variant,
alternating variants round-robin so box-to-box and thermal drift cancel.

usage: python tools/ab_bench.py lib_a.so lib_b.so[@VAR=value] [...] [--rounds 3] [--steps 5]
(env AB_POLICY=FIFO|DELAY, AB_NODES, AB_LOAD, AB_CLUSTERS, AB_LAM, AB_MAXDUR select the workload;
default C4 FIFO; AB_POLICY=DELAY AB_LAM=0.95 AB_MAXDUR=972 is the Level1-heavy DELAY stream)
Each variant runs in its own subprocess (MCS_LIB=<path>) per round; prints median kernel ms."""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
sys.path.insert(0, os.path.join(os.environ["REPO"], "multi-cluster-simulator_amd"))
from mcs_amd import Engine, GenParams, replicate, uniform_cluster
from mcs_amd.engine import scaled_lambda
steps = int(os.environ["STEPS"])
nn, load = int(os.environ.get("AB_NODES", "256")), float(os.environ.get("AB_LOAD", "0.9"))
eng = Engine(0, policy=os.environ.get("AB_POLICY", "FIFO"))
nc = int(os.environ.get("AB_CLUSTERS", "4096"))
eng.load_clusters(replicate(uniform_cluster(nn), nc))
lam = float(os.environ.get("AB_LAM", "0")) or scaled_lambda(nn, load=load)
eng.generate_jobs(GenParams(arrival_mode=1, lam=lam, max_dur_s=int(os.environ.get("AB_MAXDUR", "600")),
                             fused=os.environ.get("AB_FUSED", "0") == "1"), 16384)
eng.run()
ms = [eng.run().kernel_ms for _ in range(steps)]
print(json.dumps({"ms": ms}))
'''


def main():
    args = sys.argv[1:]
    rounds, steps = 3, 5
    if "--rounds" in args:
        i = args.index("--rounds"); rounds = int(args[i + 1]); del args[i:i + 2]
    if "--steps" in args:
        i = args.index("--steps"); steps = int(args[i + 1]); del args[i:i + 2]
    res = {a: [] for a in args}
    for _ in range(rounds):
        for lib in args:
            path, _, extra = lib.partition("@")  # lib.so@VAR=value: a per-variant environment
            env = dict(os.environ, MCS_LIB=os.path.abspath(path), REPO=REPO, STEPS=str(steps))
            if extra:
                k, _, v = extra.partition("=")
                env[k] = v
            out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                                 timeout=300)
            if out.returncode != 0:
                print(lib, "FAILED", out.stderr[-2000:])
                sys.exit(1)
            res[lib] += json.loads(out.stdout.strip().splitlines()[-1])["ms"]
    for lib, ms in res.items():
        print(f"{os.path.basename(lib):28s} median {statistics.median(ms):8.3f} ms  min {min(ms):8.3f}  "
              f"max {max(ms):8.3f}  ({int(os.environ.get('AB_CLUSTERS', '4096')) * 16384 / statistics.median(ms) / 1e6:.3f}e9 placements/s)")


if __name__ == "__main__":
    main()
