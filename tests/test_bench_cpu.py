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


# ---- bench.py --gpus N: one rank per GPU, and refusal when the world cannot be N ---------------
def test_launcher_command_line(monkeypatch):
    bench, _ = _bench([], monkeypatch)
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "20", "--warmup", "5"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "20", "--warmup", "5"]


def test_world_check_cases(monkeypatch):
    bench, _ = _bench([], monkeypatch)
    wc = bench.world_check
    assert wc(1, {}, 0) == ("run", 1)
    assert wc(8, {}, 8) == ("launch", 8)
    assert wc(8, {}, 1)[0] == "refuse"  # --gpus 8 on a 1-GPU box: never a mislabelled 1-GPU line
    assert wc(8, {"WORLD_SIZE": "8", "LOCAL_RANK": "3"}, 8) == ("run", 8)
    assert wc(8, {"WORLD_SIZE": "4", "LOCAL_RANK": "0"}, 8)[0] == "refuse"  # torchrun world != --gpus
    assert wc(1, {"WORLD_SIZE": "2", "LOCAL_RANK": "0"}, 2)[0] == "refuse"
    assert wc(2, {"WORLD_SIZE": "2", "LOCAL_RANK": "1"}, 1)[0] == "refuse"  # rank without a GPU
    assert wc(0, {}, 8)[0] == "refuse"


def test_launch_spawns_torchrun_child(monkeypatch):
    bench, _ = _bench(["--gpus", "4", "--steps", "3"], monkeypatch)
    import subprocess

    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return R()

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "visible_devices", lambda: 4)
    monkeypatch.setattr(subprocess, "run", fake_run)
    assert bench.main() == 7  # the worst rank's status (torchrun's) is the parent's
    assert "--nproc-per-node=4" in seen["cmd"] and seen["cmd"][-3:] == ["--gpus", "4", "--steps", "3"][-3:]


def test_refusal_exits_nonzero_without_gpus():
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "refusing" in r.stderr and r.stdout == ""
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "differs from --gpus" in r.stderr


def _fake_kfd(tmp_path, kinds):
    """A KFD topology tree: one node directory per entry, 'gpu' nodes with SIMDs, 'cpu' without."""
    root = tmp_path / "nodes"
    for i, k in enumerate(kinds):
        d = root / str(i)
        d.mkdir(parents=True)
        simd = 1024 if k == "gpu" else 0
        (d / "properties").write_text(f"cpu_cores_count {0 if k == 'gpu' else 64}\nsimd_count {simd}\n"
                                      f"gfx_target_version {90500 if k == 'gpu' else 0}\n")
    return str(root)


def test_visible_devices_from_kfd_sysfs(tmp_path, monkeypatch):
    """The parent counts GPUs from the KFD topology (nodes with SIMDs) and narrows the count by
    ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES, without HIP or torch."""
    bench, _ = _bench(["--gpus", "2"], monkeypatch)
    root = _fake_kfd(tmp_path, ["cpu", "gpu", "gpu", "gpu", "cpu", "gpu"])
    assert bench.visible_devices({}, root) == 4
    assert bench.visible_devices({"HIP_VISIBLE_DEVICES": "0,2"}, root) == 2
    assert bench.visible_devices({"HIP_VISIBLE_DEVICES": ""}, root) == 0
    assert bench.visible_devices({"CUDA_VISIBLE_DEVICES": "3,7,1"}, root) == 1  # stops at the invalid 7
    assert bench.visible_devices({"ROCR_VISIBLE_DEVICES": "1,2", "HIP_VISIBLE_DEVICES": "0,1,2"}, root) == 2
    assert bench.visible_devices({"ROCR_VISIBLE_DEVICES": "GPU-1234abcd"}, root) == 1
    assert bench.visible_devices({}, str(tmp_path / "absent")) == 0


def test_parent_maps_no_gpu_runtime(tmp_path):
    """`bench.py --gpus 2` as a parent: its /proc/self/maps at the decision (MCS_BENCH_PARENT_MAPS)
    shows neither /dev/kfd nor any HIP or torch library, i.e. the parent cannot have initialised a
    GPU before spawning (or refusing)."""
    import subprocess

    maps = tmp_path / "maps.txt"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MCS_BENCH_PARENT_MAPS"] = str(maps)
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "refusing" in r.stderr
    text = maps.read_text()
    assert "python" in text  # the dump is real
    for bad in ("/dev/kfd", "libamdhip64", "libtorch", "libhsa-runtime"):
        assert bad not in text, bad
