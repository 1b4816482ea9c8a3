"""The C ABI driven from C (tests/abi_driver.c), as the cgo binding of INTEGRATION.md would drive
it: KAT2 as a batch run, the same jobs online (POST batches + horizons), the single-job mirrors and
the error convention, compiled with gcc against include/mcs.h and libmcs.so and run on the GPU."""
import os
import subprocess

import pytest

from mcs_amd import _lib as L

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def build_driver(out_dir):
    lib_dir = os.path.dirname(L.LIB_PATH)
    exe = os.path.join(str(out_dir), "abi_driver")
    subprocess.run(["gcc", "-std=c99", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
                    os.path.join(HERE, "abi_driver.c"), "-L", lib_dir, "-lmcs", f"-Wl,-rpath,{lib_dir}", "-o", exe],
                   check=True, capture_output=True, text=True)
    return exe


def test_abi_driver_builds(tmp_path):
    """(CPU) the C caller compiles warning-free against the header and links against libmcs.so"""
    assert os.path.exists(build_driver(tmp_path))


@pytest.mark.gpu
def test_abi_driver_runs_kat2_online_and_mirrors(tmp_path):
    exe = build_driver(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ABI-DRIVER OK" in r.stdout
