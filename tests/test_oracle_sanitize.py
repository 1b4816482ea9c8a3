"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (no GPU).

Every parity claim compares the HIP path with the oracle, so the oracle's own memory and integer
behaviour is checked here: its Go-shaped queues (memmove / realloc growth) and the uint64 wrap
arithmetic it restates (cluster.go:87-125,141-161).  Two legs, both built by `make -C oracle asan`
with every sanitizer report fatal:

* oracle/oracle_selftest.c: a seeded self-test of every oracle entry point against the oracle's
  exact identities (literal == fast-forward for FIFO and DELAY, the trading reductions, the
  single-call mirrors) — it found a float64 -> uint64 conversion of a wrapped counter that was
  undefined behaviour in C (now or_go_f64_to_u64, as Go converts on amd64);
* the oracle test modules (every golden KAT of tests/golden/ and their seeded cases) run in a child
  interpreter against the sanitized library (MCS_ORACLE_SO) with libasan/libubsan preloaded.

The host-side C++ of libmcs.so (ABI argument checks, the host generator, engine-creation failure
without a device) runs under the same sanitizers in test_abi_sanitize.py's leg below.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(REPO, "oracle")
ASAN_DIR = os.path.join(ORACLE, "asan")
SAN_ENV = {
    "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=86",
    "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1:exitcode=87",
}


def _gcc_runtime(name):
    return subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True,
                          check=True).stdout.strip()


@pytest.fixture(scope="module")
def asan_build():
    r = subprocess.run(["make", "-C", ORACLE, "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + r.stdout[-2000:] + r.stderr[-2000:])
    return ASAN_DIR


def _clean(stderr):
    return "runtime error" not in stderr and "AddressSanitizer" not in stderr and "LeakSanitizer" not in stderr


@pytest.mark.parametrize("seed,scale", [("0x4D43535F53454C46", "8"), ("0x5EED0002", "8")])
def test_oracle_selftest_under_sanitizers(asan_build, seed, scale):
    env = dict(os.environ, **SAN_ENV)
    env["ASAN_OPTIONS"] = env["ASAN_OPTIONS"].replace("detect_leaks=0", "detect_leaks=1")
    r = subprocess.run([os.path.join(asan_build, "oracle_selftest"), seed, scale], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "SELFTEST OK" in r.stdout
    assert _clean(r.stderr), r.stderr[-4000:]


def test_oracle_kat_modules_under_sanitizers(asan_build):
    """Every golden KAT (FIFO, DELAY, FIFO trading, DELAY trading, ApproveTrade, heap order,
    AllocateVirtualNodeResources, contract sizing) and the modules' seeded cases, through the
    sanitized oracle library in a child interpreter."""
    pre = ":".join(_gcc_runtime(n) for n in ("libasan.so", "libubsan.so"))
    env = dict(os.environ, **SAN_ENV, LD_PRELOAD=pre,
               MCS_ORACLE_SO=os.path.join(asan_build, "libmcs_oracle_asan.so"))
    mods = [os.path.join(REPO, "tests", m) for m in ("test_oracle.py", "test_delay_oracle.py", "test_trade_oracle.py",
                                                     "test_dtrade_oracle.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu", *mods],
                       capture_output=True, text=True, env=env, timeout=900, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-4000:]
    assert " passed" in r.stdout and "failed" not in r.stdout
    assert _clean(r.stderr), r.stderr[-4000:]
