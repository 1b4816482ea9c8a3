"""The host-side C++ of libmcs.so under AddressSanitizer + UndefinedBehaviorSanitizer (no GPU).

`make -C multi-cluster-simulator_amd asan` rebuilds the ABI's host translation units (mcs_engine,
mcs_trade, mcs_dtrade, mcs_online: argument checks, the host job generator, engine creation and
teardown when no device is usable) with -Xarch_host -fsanitize=address,undefined (the device code
and the kernel objects are the product's) into build_asan/libmcs_asan.so.  A child interpreter
with clang's ASan runtime preloaded runs the CPU ABI suite (tests/test_abi.py: exports, the host
generator's distributions and Weibull table, the null-handle sweep over every entry point, the
engine's refusal without a device) against it through MCS_LIB; any sanitizer report is fatal.
The oracle's own sanitizer legs are in test_oracle_sanitize.py.
"""
import glob
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "multi-cluster-simulator_amd")


def test_abi_host_code_under_sanitizers():
    rts = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    if not rts:
        pytest.skip("clang ASan runtime not present")
    r = subprocess.run(["make", "-C", PKG, "asan", "-j4"], capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lib = os.path.join(PKG, "build_asan", "libmcs_asan.so")
    env = dict(os.environ, LD_PRELOAD=rts[0], MCS_LIB=lib,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:detect_odr_violation=0:exitcode=86",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=87")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        os.path.join(REPO, "tests", "test_abi.py")], capture_output=True, text=True, env=env,
                       timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-4000:]
    assert " passed" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
