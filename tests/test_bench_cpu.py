"""bench.py's CPU baseline leg (host only): the oracle on a bounded sample of the bench workload.
The sample is sized by a pilot so a Level1-heavy DELAY stream (~100x the oracle's cost per job)
stays within the budget; an explicit --cpu-sample-clusters is taken as given."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(argv, monkeypatch):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd"))
    import bench

    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    return bench, bench.parse()


def test_cpu_baseline_pilot_bounds_the_sample(monkeypatch):
    bench, a = _bench(["--policy", "delay", "--lam", "0.95", "--max-dur", "972", "--clusters", "64",
                       "--jobs-per-cluster", "512"], monkeypatch)
    monkeypatch.setattr(bench, "CPU_BUDGET_S", 1e-4)  # any pilot exceeds it: the sample shrinks
    wl = bench.Workload(a, 1, 0)
    r = bench.cpu_baseline(a, wl, 2)
    assert r["sample_clusters"] == 4  # the pilot's own size (2 clusters per thread)
    assert r["value"] > 0 and r["cores"] == 2 and r["kind"] == "port"


def test_cpu_baseline_explicit_sample(monkeypatch):
    bench, a = _bench(["--clusters", "64", "--jobs-per-cluster", "256", "--cpu-sample-clusters", "6"],
                      monkeypatch)
    monkeypatch.setattr(bench, "CPU_BUDGET_S", 1e-4)
    wl = bench.Workload(a, 1, 0)
    r = bench.cpu_baseline(a, wl, 2)
    assert r["sample_clusters"] == 6
    assert a.traffic_json.endswith("traffic_latest.json")
