"""CPU tests of the C-ABI library (no compute calls that need a GPU): it loads, exports exactly
what include/*.h declare, the host generator is deterministic and has the reference
distributions, and the spec loader follows Go's encoding/json rules."""
import os
import re
import subprocess

import numpy as np
import pytest

import mcs_amd
from mcs_amd import Cluster, GenParams, gen_cluster_host, scaled_lambda
from mcs_amd import _lib as L

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h) for h in sorted(os.listdir(os.path.join(REPO, "include")))
           if h.endswith(".h")]


def header_functions():
    names = set()
    for h in HEADERS:
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(mcs_[a-z0-9_]+)\s*\(", txt))
    return sorted(names)


def test_library_loads_and_exports_header_symbols():
    lib = mcs_amd.lib()
    declared = header_functions()
    assert len(declared) >= 33
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (mcs_[a-z0-9_]+)$", out.stdout, flags=re.M))
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    # every declared function has a ctypes signature in the binding
    bound = {name for name, _, _ in L.SIGNATURES}
    assert set(declared) == bound
    assert lib.mcs_abi_version() == 7


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", L.LIB_PATH], capture_output=True, text=True)
    blob = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_engine_create_without_device_fails_loudly():
    # In this container there is no GPU: the engine must refuse, not fall back to the CPU.
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(mcs_amd.MCSError):
        mcs_amd.Engine(0)


def test_generator_deterministic_and_seeded():
    gp = GenParams(seed=7)
    a1 = gen_cluster_host(gp, 3, 32, 24000, 5000)
    a2 = gen_cluster_host(gp, 3, 32, 24000, 5000)
    for x, y in zip(a1, a2):
        np.testing.assert_array_equal(x, y)
    b = gen_cluster_host(gp, 4, 32, 24000, 5000)
    assert not np.array_equal(a1[2], b[2])
    # prefix property of the counter-based attributes
    p = gen_cluster_host(gp, 3, 32, 24000, 1000)
    for x, y in zip(p, a1):
        np.testing.assert_array_equal(x, y[:1000])


def test_generator_distributions_ref_mode():
    a, d, c, m = gen_cluster_host(GenParams(seed=11), 0, 32, 24000, 200_000)
    assert (np.diff(a.astype(np.int64)) >= 0).all()
    assert c.max() <= 31 and m.max() <= 23999 and d.max() <= 599
    # Beta(2,2): mean 1/2, variance 1/20
    u = c / 32.0
    assert abs(u.mean() - 0.5 + 1 / 64) < 0.01
    v = m / 24000.0
    assert abs(v.var() - 0.05) < 0.003
    assert abs(d.mean() - 299.5) < 2.0
    # Poisson(10) per minute with floor(60/n) spacing: ~ 10 jobs per <= 60 s minute
    jobs_per_s = len(a) / (a[-1] + 1)
    assert 0.16 < jobs_per_s < 0.20


def test_generator_scaled_mode_rate():
    lam = scaled_lambda(256, load=0.9)
    assert 1.5 < lam < 1.6
    a, d, c, m = gen_cluster_host(GenParams(seed=3, arrival_mode=1, lam=lam), 0, 32, 24000, 100_000)
    rate = len(a) / (a[-1] + 1)
    assert abs(rate - lam) / lam < 0.02


def test_generator_weibull_mode_gaps():
    """MCS_ARRIVAL_WEIBULL (client.go:131-145): gaps are floor(X), X ~ Weibull(scale 10, shape 3):
    P(gap = n) = exp(-(n/10)^3) - exp(-((n+1)/10)^3); job 0 arrives at t = 0."""
    a, d, c, m = gen_cluster_host(GenParams(seed=21, arrival_mode=2, lam=10.0), 0, 32, 24000, 300_000)
    assert a[0] == 0 and (np.diff(a.astype(np.int64)) >= 0).all()
    g = np.diff(a.astype(np.int64))
    n = np.arange(0, 40)
    pmf = np.exp(-(n / 10.0) ** 3) - np.exp(-((n + 1) / 10.0) ** 3)
    emp = np.bincount(g, minlength=40)[:40] / len(g)
    assert np.abs(emp - pmf).max() < 0.003
    assert abs(g.mean() - (pmf * n).sum()) < 0.03
    # the shape parameter is honoured, and a scale whose gap table would not vanish is refused
    a2 = gen_cluster_host(GenParams(seed=21, arrival_mode=2, lam=10.0, weibull_k=1.5), 0, 32, 24000, 100_000)[0]
    n2 = np.arange(1, 200)
    assert abs(np.diff(a2.astype(np.int64)).mean() - np.exp(-(n2 / 10.0) ** 1.5).sum()) < 0.1  # E[floor X]
    with pytest.raises(mcs_amd.MCSError):
        gen_cluster_host(GenParams(arrival_mode=2, lam=1000.0), 0, 32, 24000, 10)


def test_generator_rejects_bad_params():
    with pytest.raises(mcs_amd.MCSError):
        gen_cluster_host(GenParams(lam=0.0), 0, 32, 24000, 10)


def test_cluster_json_go_rules(tmp_path):
    cl = Cluster.load(os.path.join(REPO, "assets", "cluster_big.json"))
    assert len(cl.Nodes) == 10 and cl.GetTotalResources() == (320, 240000)
    # case-insensitive keys, unknown keys ignored, missing keys zero (encoding/json)
    c2 = Cluster.from_json('{"id": 4, "nodes": [{"CORES": 8, "memory": 100, "coresavailable": 3, "x": 1}]}')
    assert c2.Id == 4 and c2.Nodes[0].Cores == 8 and c2.Nodes[0].CoresAvailable == 3
    assert c2.Nodes[0].MemoryAvailable == 0
    with pytest.raises(ValueError):
        Cluster.from_json('{"Id": 1, "Nodes": [{"Cores": -1}]}')


def test_struct_layouts_match_headers(tmp_path):
    """The ctypes mirrors have the C layout of include/*.h (sizes and every field offset)."""
    import ctypes as C

    structs = [L.mcs_config, L.mcs_gen_params, L.mcs_stats, L.mcs_cluster_stats, L.mcs_lent_rec,
               L.mcs_trade_rec, L.mcs_trade_stats, L.mcs_comm_id, L.mcs_delay_cluster_stats,
               L.mcs_contract_rec, L.mcs_foreign_rec, L.mcs_cluster_state, L.mcs_approve_query]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mcs_trade.h"', "int main(void) {"]
    for s in structs:
        n = s.__name__
        lines.append(f'printf("{n} %zu\\n", sizeof({n}));')
        for f, _ in s._fields_:
            cf = f.rstrip("_")  # ctypes name lambda_ -> C member lambda
            lines.append(f'printf("{n}.{f} %zu\\n", offsetof({n}, {cf}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(REPO, "include"), "-o", str(exe), str(src)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                          check=True).stdout.split("\n") if l)
    for s in structs:
        n = s.__name__
        assert int(out[n]) == C.sizeof(s), n
        for f, _ in s._fields_:
            assert int(out[f"{n}.{f}"]) == getattr(s, f).offset, f"{n}.{f}"


def test_trading_engine_without_device_fails_loudly():
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(mcs_amd.MCSError):
        mcs_amd.Engine(0, borrow=True, trader=True)


def test_every_engine_entry_point_refuses_a_null_handle():
    """Every entry point that takes an engine handle returns MCS_E_INVALID (or its neutral value) for
    a null handle with null/zero arguments instead of touching memory (no device needed; the same
    sweep runs against the AddressSanitizer build in test_abi_sanitize.py)."""
    import ctypes as C

    lib = mcs_amd.lib()
    n = 0
    for name, res, args in L.SIGNATURES:
        if not args or args[0] is not L.vp or not hasattr(lib, name):
            continue
        vals = [None if (a is L.vp or hasattr(a, "contents") or a is C.c_char_p) else 0 for a in args]
        got = getattr(lib, name)(*vals)
        if res is C.c_int:
            assert got == L.MCS_E_INVALID, (name, got)
        elif res is C.c_char_p:
            assert isinstance(got, bytes), name
        else:
            assert got == 0, (name, got)
        n += 1
    assert n >= 35, n
