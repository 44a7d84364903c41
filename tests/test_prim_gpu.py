"""The hand-written device primitives of the grouping / quantile paths (deequ_amd/csrc/dq_prim.hip) against numpy.

GPU (`-m gpu`): the stable LSD radix sort (keys only, 4- and 8-byte values, bit ranges, descending, ragged sizes,
all-equal and few-distinct keys), the prefix sums (wrapping) and the runs of equal keys (unique keys, starts,
lengths, per-position run ids, per-run sums and firsts), each compared element for element with numpy's stable sort / cumsum / unique,
through the test harness tests/prim_check.cpp (deequ_amd/build/libdqprimcheck.so).  CPU: the harness exports load.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "deequ_amd", "build", "libdqprimcheck.so")


def _lib():
    # torch first: its HIP runtime is then the one the harness binds to (deequ_amd/_lib.py loads libdqscan.so the
    # same way; the other order gives the harness a second runtime instance that sees no device)
    import torch  # noqa: F401

    lib = ctypes.CDLL(LIB)
    p, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.prim_sort_pairs.argtypes = [p, p, p, p, i32, i64, i32, i32, i32]
    lib.prim_exclusive_sum_i64.argtypes = [p, p, i64]
    lib.prim_inclusive_sum_u32.argtypes = [p, p, i64]
    lib.prim_runs.argtypes = [p, i64, p, p, p, p, p, p, p, ctypes.POINTER(ctypes.c_int64), p]
    for f in (lib.prim_sort_pairs, lib.prim_exclusive_sum_i64, lib.prim_inclusive_sum_u32, lib.prim_runs):
        f.restype = ctypes.c_int
    return lib


def test_harness_exports():
    lib = _lib()
    for name in ("prim_sort_pairs", "prim_exclusive_sum_i64", "prim_inclusive_sum_u32", "prim_runs"):
        assert hasattr(lib, name)


def _dev(a: np.ndarray):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _host(t, dtype):
    return t.cpu().numpy().view(dtype)


def _empty(n, itemsize):
    import torch

    return torch.zeros(max(1, n), dtype=torch.int64 if itemsize == 8 else torch.int32, device="cuda")


def _sort(keys: np.ndarray, vals, vb: int, begin: int, end: int, desc: bool):
    lib = _lib()
    n = len(keys)
    kin = _dev(keys.view(np.int64))
    kout = _empty(n, 8)
    vin = vout = None
    if vb:
        vin = _dev(vals.view(np.int64 if vb == 8 else np.int32))
        vout = _empty(n, vb)
    rc = lib.prim_sort_pairs(kin.data_ptr(), kout.data_ptr(), vin.data_ptr() if vb else None,
                             vout.data_ptr() if vb else None, vb, n, begin, end, int(desc))
    assert rc == 0, rc
    ko = _host(kout, np.uint64)[:n]
    vo = _host(vout, np.uint64 if vb == 8 else np.uint32)[:n] if vb else None
    # the input must be untouched
    assert np.array_equal(_host(kin, np.uint64), keys)
    return ko, vo


def _want_order(keys: np.ndarray, begin: int, end: int, desc: bool):
    width = end - begin
    dig = (keys >> np.uint64(begin)) & np.uint64((1 << width) - 1 if width < 64 else 0xFFFFFFFFFFFFFFFF)
    if desc:
        dig = np.uint64((1 << width) - 1 if width < 64 else 0xFFFFFFFFFFFFFFFF) - dig
    return np.argsort(dig, kind="stable")


CASES = [
    # n, key generator, begin, end, desc
    (1, "full", 0, 64, False),
    (7, "full", 0, 64, False),
    (2047, "full", 0, 64, False),
    (2048, "full", 0, 64, False),
    (2049, "few", 0, 64, False),
    (100_003, "full", 0, 64, False),
    (100_003, "few", 0, 64, True),
    (250_000, "small20", 0, 20, False),   # partial last digit (4 bits)
    (250_000, "small20", 0, 20, True),
    (300_001, "full", 8, 24, False),      # a bit range inside the key
    (65_536, "equal", 0, 64, False),
    (3_000_017, "full", 0, 64, False),    # many tiles per workgroup
    (3_000_017, "few", 0, 33, True),
]


def _keys(kind: str, n: int, rng):
    if kind == "full":
        return rng.integers(0, 2**64 - 1, size=n, dtype=np.uint64, endpoint=True)
    if kind == "few":
        base = rng.integers(0, 2**64 - 1, size=17, dtype=np.uint64, endpoint=True)
        return base[rng.integers(0, 17, size=n)]
    if kind == "small20":
        return rng.integers(0, 1 << 20, size=n, dtype=np.uint64)
    if kind == "equal":
        return np.full(n, 0x0123456789ABCDEF, dtype=np.uint64)
    raise ValueError(kind)


@pytest.mark.gpu
@pytest.mark.parametrize("vb", [0, 4, 8])
@pytest.mark.parametrize("n,kind,begin,end,desc", CASES)
def test_sort_pairs(n, kind, begin, end, desc, vb):
    """One-sweep passes (below 2^30 keys: digit totals up front, tile offsets by decoupled look-back)."""
    rng = np.random.default_rng(n * 31 + vb + (7 if desc else 0))
    keys = _keys(kind, n, rng)
    vals = None
    if vb == 8:
        vals = rng.integers(0, 2**64 - 1, size=n, dtype=np.uint64, endpoint=True)
    elif vb == 4:
        vals = np.arange(n, dtype=np.uint32)
    ko, vo = _sort(keys, vals, vb, begin, end, desc)
    order = _want_order(keys, begin, end, desc)
    assert np.array_equal(ko, keys[order])
    if vb:
        assert np.array_equal(vo, vals[order])  # stable: equal keys keep their input order


SEGMENTED_CASES = [(2049, "few", 0, 64, False), (300_001, "full", 8, 24, False), (3_000_017, "full", 0, 64, False),
                   (3_000_017, "few", 0, 33, True)]


@pytest.mark.gpu
@pytest.mark.parametrize("vb", [0, 8])
@pytest.mark.parametrize("n,kind,begin,end,desc", SEGMENTED_CASES)
def test_sort_pairs_segmented(n, kind, begin, end, desc, vb):
    """The segmented reduce-then-scan passes (the form above 2^30 keys), forced by DQ_SORT_SEGMENTED in a child process
    (the knob is read once per process)."""
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, %r); import test_prim_gpu as T; "
            "T.test_sort_pairs(%d, %r, %d, %d, %r, %d); print('ok')" % (os.path.join(ROOT, "tests"), n, kind, begin, end,
                                                                        desc, vb))
    env = dict(os.environ, DQ_SORT_SEGMENTED="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


@pytest.mark.gpu
def test_sort_empty_range_copies():
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 2**64 - 1, size=5000, dtype=np.uint64, endpoint=True)
    vals = np.arange(5000, dtype=np.uint64)
    ko, vo = _sort(keys, vals, 8, 5, 5, False)
    assert np.array_equal(ko, keys) and np.array_equal(vo, vals)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1023, 1024, 1025, 262_144, 2_500_001])
def test_scans(n):
    lib = _lib()
    rng = np.random.default_rng(n)
    v = rng.integers(-2**62, 2**62, size=n, dtype=np.int64)  # partial sums wrap
    a = _dev(v)
    out = _empty(n, 8)
    assert lib.prim_exclusive_sum_i64(a.data_ptr(), out.data_ptr(), n) == 0
    want = np.concatenate([[0], np.cumsum(v)[:-1]]).astype(np.int64)
    assert np.array_equal(_host(out, np.int64)[:n], want)
    # in place
    assert lib.prim_exclusive_sum_i64(a.data_ptr(), a.data_ptr(), n) == 0
    assert np.array_equal(_host(a, np.int64)[:n], want)
    u = rng.integers(0, 2**32 - 1, size=n, dtype=np.uint32, endpoint=True)
    b = _dev(u.view(np.int32))
    outu = _empty(n, 4)
    assert lib.prim_inclusive_sum_u32(b.data_ptr(), outu.data_ptr(), n) == 0
    assert np.array_equal(_host(outu, np.uint32)[:n], np.cumsum(u, dtype=np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("n,distinct", [(1, 1), (5, 5), (1024, 3), (1025, 1025), (777_777, 50_000), (2_000_003, 7)])
def test_runs(n, distinct):
    lib = _lib()
    rng = np.random.default_rng(n + distinct)
    pool = rng.integers(0, 2**64 - 1, size=distinct, dtype=np.uint64, endpoint=True)
    keys = np.sort(pool[rng.integers(0, distinct, size=n)])
    vals = rng.integers(-2**40, 2**40, size=n, dtype=np.int64)
    fv = rng.integers(0, 2**64 - 1, size=n, dtype=np.uint64, endpoint=True)
    k, sv, f = _dev(keys.view(np.int64)), _dev(vals), _dev(fv.view(np.int64))
    uq, st, ln, sm, fs = (_empty(n, 8) for _ in range(5))
    ro = _empty(n, 4)
    nr = ctypes.c_int64(-1)
    rc = lib.prim_runs(k.data_ptr(), n, uq.data_ptr(), st.data_ptr(), ln.data_ptr(), sv.data_ptr(), sm.data_ptr(),
                       f.data_ptr(), fs.data_ptr(), ctypes.byref(nr), ro.data_ptr())
    assert rc == 0
    wu, ws, wl = np.unique(keys, return_index=True, return_counts=True)
    R = len(wu)
    assert nr.value == R
    assert np.array_equal(_host(uq, np.uint64)[:R], wu)
    assert np.array_equal(_host(st, np.int64)[:R], ws)
    assert np.array_equal(_host(ln, np.int64)[:R], wl)
    assert np.array_equal(_host(sm, np.int64)[:R], np.add.reduceat(vals, ws))
    assert np.array_equal(_host(fs, np.uint64)[:R], fv[ws])
    assert np.array_equal(_host(ro, np.int32)[:n], np.repeat(np.arange(R, dtype=np.int32), wl))  # run of each position


@pytest.mark.gpu
def test_runs_unsorted_neighbours():
    """A run is a maximal stretch of equal neighbours (the same key may start several runs)."""
    lib = _lib()
    keys = np.array([5, 5, 1, 1, 1, 5, 9, 9, 5], dtype=np.uint64)
    n = len(keys)
    k = _dev(keys.view(np.int64))
    uq, st, ln = (_empty(n, 8) for _ in range(3))
    nr = ctypes.c_int64(-1)
    assert lib.prim_runs(k.data_ptr(), n, uq.data_ptr(), st.data_ptr(), ln.data_ptr(), None, None, None, None,
                         ctypes.byref(nr), None) == 0
    assert nr.value == 5
    assert _host(uq, np.uint64)[:5].tolist() == [5, 1, 5, 9, 5]
    assert _host(st, np.int64)[:5].tolist() == [0, 2, 5, 6, 8]
    assert _host(ln, np.int64)[:5].tolist() == [2, 3, 1, 2, 1]
