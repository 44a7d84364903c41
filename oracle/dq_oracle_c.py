"""ctypes binding of oracle/c/dq_oracle.c (TEST INFRASTRUCTURE ONLY; see dq_oracle.py header)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libdqoracle.so")
KINDS = {"f64": 1, "i64": 2, "i32": 3, "utf8": 4, "large_utf8": 5, "f32": 6, "i16": 7, "i8": 8, "bool": 9,
         "date32": 3, "timestamp": 2}


class ColStats(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int64), ("sum_f64", ctypes.c_double), ("sum_i64", ctypes.c_int64),
                ("n", ctypes.c_double), ("avg", ctypes.c_double), ("m2", ctypes.c_double),
                ("min", ctypes.c_double), ("max", ctypes.c_double),
                ("imin", ctypes.c_int64), ("imax", ctypes.c_int64)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, u8p = ctypes.c_void_p, ctypes.c_void_p
        L.dqo_xxh64_long.restype = ctypes.c_uint64
        L.dqo_xxh64_long.argtypes = [ctypes.c_int64, ctypes.c_uint64]
        L.dqo_xxh64_int.restype = ctypes.c_uint64
        L.dqo_xxh64_int.argtypes = [ctypes.c_int32, ctypes.c_uint64]
        L.dqo_xxh64_bytes.restype = ctypes.c_uint64
        L.dqo_xxh64_bytes.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_uint64]
        L.dqo_column_stats.argtypes = [ctypes.c_int, vp, u8p, u8p, ctypes.c_int64, ctypes.c_int,
                                       ctypes.POINTER(ColStats)]
        L.dqo_corr.argtypes = [ctypes.c_int, vp, u8p, ctypes.c_int, vp, u8p, u8p, ctypes.c_int64,
                               ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.dqo_hll_registers.argtypes = [ctypes.c_int, vp, vp, u8p, u8p, ctypes.c_int64, vp]
        L.dqo_hll_registers_mt.argtypes = [ctypes.c_int, vp, vp, u8p, u8p, ctypes.c_int64, ctypes.c_int, vp, vp]
        L.dqo_count_bits.restype = ctypes.c_int64
        L.dqo_count_bits.argtypes = [u8p, u8p, ctypes.c_int64]
        L.dqo_profile_scan.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_int64, ctypes.c_int,
                                       ctypes.c_int, ctypes.POINTER(ColStats), vp]
        L.dqo_column_stats_partials.argtypes = [ctypes.c_int, vp, u8p, u8p, ctypes.c_int64, ctypes.c_int,
                                                ctypes.c_int, ctypes.POINTER(ColStats)]
        L.dqo_stats_merge.argtypes = [ctypes.c_int, ctypes.POINTER(ColStats), ctypes.POINTER(ColStats)]
        L.dqo_stats_finish.argtypes = [ctypes.c_int, ctypes.POINTER(ColStats)]
        L.dqo_corr_partials.argtypes = [ctypes.c_int, vp, u8p, ctypes.c_int, vp, u8p, u8p, ctypes.c_int64,
                                        ctypes.c_int, ctypes.c_int, vp]
        L.dqo_corr_merge.argtypes = [vp, vp]
        L.dqo_exact_moments.argtypes = [ctypes.c_int, vp, u8p, u8p, ctypes.c_int64, ctypes.c_double, ctypes.c_int, vp]
        L.dqo_exact_comoments.argtypes = [ctypes.c_int, vp, u8p, ctypes.c_int, vp, u8p, u8p, ctypes.c_int64,
                                          ctypes.c_double, ctypes.c_double, ctypes.c_int, vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def column_stats(kind: str, values: np.ndarray, validity, mask=None, nparts: int = 1) -> ColStats:
    out = ColStats()
    lib().dqo_column_stats(KINDS[kind], _p(values), _p(validity), _p(mask), len(values), nparts,
                           ctypes.byref(out))
    return out


def corr(kx, x, vx, ky, y, vy, mask=None, nparts: int = 1):
    out = (ctypes.c_double * 6)()
    lib().dqo_corr(KINDS[kx], _p(x), _p(vx), KINDS[ky], _p(y), _p(vy), _p(mask), len(x), nparts, out)
    return tuple(out)


def hll_registers(kind, values, offsets, validity, mask, n) -> np.ndarray:
    regs = np.zeros(512, dtype=np.uint8)
    lib().dqo_hll_registers(KINDS[kind], _p(values), _p(offsets), _p(validity), _p(mask), n, _p(regs))
    return regs


def hll_registers_mt(kind, values, offsets, validity, mask, n, nthreads, regs=None):
    """(registers accumulated into `regs`, {redo, long, window}: rows reaching the kernels' rare paths)."""
    if regs is None:
        regs = np.zeros(512, dtype=np.uint8)
    paths = np.zeros(3, dtype=np.int64)
    lib().dqo_hll_registers_mt(KINDS[kind], _p(values), _p(offsets), _p(validity), _p(mask), n, nthreads, _p(regs),
                               _p(paths))
    return regs, {"redo": int(paths[0]), "long": int(paths[1]), "window": int(paths[2])}


def profile_scan(cols, n, nparts, nthreads):
    """cols: list of (kind, values, offsets|None, validity|None). Returns (stats list, regs [ncols,512])."""
    nc = len(cols)
    kinds = np.array([KINDS[c[0]] for c in cols], dtype=np.int32)
    vals = (ctypes.c_void_p * nc)(*[_p(c[1]) for c in cols])
    offs = (ctypes.c_void_p * nc)(*[_p(c[2]) for c in cols])
    vals_v = (ctypes.c_void_p * nc)(*[_p(c[3]) for c in cols])
    stats = (ColStats * nc)()
    regs = np.zeros((nc, 512), dtype=np.uint8)
    lib().dqo_profile_scan(nc, kinds.ctypes.data, ctypes.addressof(vals), ctypes.addressof(offs),
                           ctypes.addressof(vals_v), n, nparts, nthreads, stats, _p(regs))
    return list(stats), regs


# ---- full-scale parity helpers (Spark partition order over many chunks; double-double references) ----
def column_stats_partials(kind, values, validity, nparts, nthreads, mask=None):
    """Spark partial aggregates of nparts row partitions of this array (one per partition, in order)."""
    out = (ColStats * nparts)()
    lib().dqo_column_stats_partials(KINDS[kind], _p(values), _p(validity), _p(mask), len(values), nparts, nthreads,
                                    out)
    return list(out)


def stats_fold(kind, partials):
    """The final aggregate: merge partition partials in order from the zero buffer, then cast."""
    acc = ColStats()
    for p in partials:
        lib().dqo_stats_merge(KINDS[kind], ctypes.byref(acc), ctypes.byref(p))
    lib().dqo_stats_finish(KINDS[kind], ctypes.byref(acc))
    return acc


def corr_partials(kx, x, vx, ky, y, vy, nparts, nthreads, mask=None):
    out = np.zeros((nparts, 6), dtype=np.float64)
    lib().dqo_corr_partials(KINDS[kx], _p(x), _p(vx), KINDS[ky], _p(y), _p(vy), _p(mask), len(x), nparts, nthreads,
                            _p(out))
    return [tuple(r) for r in out]


def corr_fold(partials):
    acc = np.zeros(6, dtype=np.float64)
    for p in partials:
        b = np.array(p, dtype=np.float64)
        lib().dqo_corr_merge(_p(acc), _p(b))
    return tuple(acc)


def exact_moments(kind, values, validity, pivot, nthreads, mask=None):
    """(count, S1, S2) of the finite selected values around `pivot`, each S as a double-double (hi, lo)."""
    out = np.zeros(5, dtype=np.float64)
    lib().dqo_exact_moments(KINDS[kind], _p(values), _p(validity), _p(mask), len(values), float(pivot), nthreads,
                            _p(out))
    return int(out[0]), (out[1], out[2]), (out[3], out[4])


def exact_comoments(kx, x, vx, ky, y, vy, px, py, nthreads, mask=None):
    """(count, Sx, Sy, Sxy, Sxx, Syy) around (px, py) over rows valid in both, as double-doubles."""
    out = np.zeros(11, dtype=np.float64)
    lib().dqo_exact_comoments(KINDS[kx], _p(x), _p(vx), KINDS[ky], _p(y), _p(vy), _p(mask), len(x), float(px),
                              float(py), nthreads, _p(out))
    return (int(out[0]),) + tuple((out[1 + 2 * k], out[2 + 2 * k]) for k in range(5))
