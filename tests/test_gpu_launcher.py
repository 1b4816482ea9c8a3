"""The `bench.py --gpus N` parent on a real 1-GPU box: it must refuse N = 2 (one GPU visible) without
touching the GPU runtime — its /proc/self/maps at the decision never shows /dev/kfd (nor the HIP or
torch libraries), so a parent can never initialise a device before it spawns torchrun's ranks."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_parent_refuses_two_gpus_without_opening_kfd(tmp_path):
    sys.path.insert(0, REPO)
    import bench

    n = bench.visible_devices()
    assert n >= 1, "the KFD topology shows no GPU on a GPU box"
    maps = tmp_path / "maps.txt"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MCS_BENCH_PARENT_MAPS"] = str(maps)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n + 1), "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "refusing" in r.stderr and r.stdout == "", (r.returncode, r.stderr[-500:])
    text = maps.read_text()
    assert "python" in text
    for bad in ("/dev/kfd", "/dev/dri", "libamdhip64", "libtorch", "libhsa-runtime"):
        assert bad not in text, bad
