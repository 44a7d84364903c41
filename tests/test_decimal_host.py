"""DecimalType arithmetic of the kernels (deequ_amd/csrc/dq_decimal.h), built for the host, against the oracle's
exact restatement: Decimal.toDouble (the correctly rounded double of unscaled / 10^scale, here Python's
Fraction -> float), Spark 2.2's XxHash64 of a decimal (hashLong of the unscaled long for precision <= 18, else
hashUnsafeBytes of BigInteger.toByteArray -- the `xxhash` package's digest of those bytes checks the byte
form independently) and the DataType class of BigDecimal.toString.

The cases: every scale 0..38 at random magnitudes, the extremes (0, +-1, 2^53 +- 1, 2^64, 10^38 - 1, +-(2^127 - 1)),
and the conversion's hard cases -- exact rounding ties (a decimal equal to the midpoint of two adjacent doubles,
e.g. 9007199254740992.5) and their neighbours one unit of the last decimal place away, which the kernels settle by
the exact integer comparison (dq_settle)."""
import os
import struct
import subprocess
from fractions import Fraction

import numpy as np
import pytest

from oracle import dq_oracle as O
from tests.conftest import ROOT


CLANG = "/opt/rocm/llvm/bin/clang++"


def _build(tmp_path, fused=False):
    """g++ -O2; fused: clang with FMA contraction on (the device default), which the conversion must switch off."""
    exe = tmp_path / ("decimal_check_fma" if fused else "decimal_check")
    cc = [CLANG, "-mfma", "-ffp-contract=fast"] if fused else ["g++"]
    subprocess.run(cc + ["-O2", "-std=c++17", "-I", os.path.join(ROOT, "deequ_amd", "csrc"), "-o", str(exe),
                         os.path.join(ROOT, "tests", "decimal_check.cpp")], check=True)
    return exe


def _cases():
    rng = np.random.default_rng(38)
    out = []
    for s in range(39):
        for p in sorted({max(1, s), min(38, s + 5), 18 if s <= 18 else s, 38}):
            for _ in range(12):
                nd = int(rng.integers(1, p + 1))
                u = int(rng.integers(0, 10 ** min(nd, 18))) * 10 ** max(0, nd - 18) + int(rng.integers(0, 10 ** max(0, min(nd - 18, 18)) or 1))
                u = min(u, 10 ** p - 1)
                out.append((-u if rng.random() < 0.4 else u, s, p))
    for u in (0, 1, -1, (1 << 53) - 1, 1 << 53, (1 << 53) + 1, 1 << 64, (1 << 64) - 1, 10 ** 38 - 1, -(10 ** 38 - 1),
              (1 << 127) - 1, -((1 << 127) - 1), 127, 128, -128, -129, 255, 256, 32767, 32768):
        for s in (0, 1, 6, 7, 18, 30, 38):
            out.append((u, s, 38))
    # exact ties: the midpoint m = (y + succ(y)) / 2 of doubles y in [2^22, 2^60), written at the smallest scale that
    # makes it a decimal, and the decimals one unit in the last place either side
    for _ in range(400):
        e = int(rng.integers(22, 60))
        y = float(rng.integers(1 << 52, 1 << 53)) * 2.0 ** (e - 52)
        succ = struct.unpack("<d", struct.pack("<q", struct.unpack("<q", struct.pack("<d", y))[0] + 1))[0]
        m = (Fraction(y) + Fraction(succ)) / 2
        s = 0
        while (m * 10 ** s).denominator != 1:
            s += 1
        u = int(m * 10 ** s)
        if abs(u) + 1 >= 10 ** 38:
            continue
        for d in (0, -1, 1):
            out.append((u + d, s, 38))
            out.append((-(u + d), s, 38))
            if s < 38 and abs(u) * 10 < 10 ** 38:
                out.append((10 * u + d, s + 1, 38))  # the same value one scale up, and its neighbours
    return out


@pytest.mark.parametrize("fused", [False, True])
def test_decimal_formulation(tmp_path, fused):
    import xxhash

    if fused and not os.path.exists(CLANG):
        pytest.skip("no clang++ for the contraction check")
    exe = _build(tmp_path, fused)
    cases = _cases()
    mask = (1 << 64) - 1
    inp = "".join(f"{u & mask} {(u >> 64) & mask} {s} {p}\n" for u, s, p in cases)
    out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    assert len(out) == len(cases)
    ties = 0
    for (u, s, p), line in zip(cases, out):
        bits, h, cls = line.split()
        want = O.decimal_to_double(u, s)
        got = struct.unpack("<d", struct.pack("<Q", int(bits, 16)))[0]
        assert got == want and (got != 0.0 or bits == "0000000000000000"), (u, s, got, want)
        d = abs(Fraction(u, 10 ** s) - Fraction(got))
        ties += d != 0 and d in (abs(Fraction(float(np.nextafter(got, np.inf))) - Fraction(got)) / 2,
                                 abs(Fraction(float(np.nextafter(got, -np.inf))) - Fraction(got)) / 2)
        hv = int(h, 16)
        assert hv == O.decimal_hash(u, p) & mask, (u, p)
        kind, v = O.decimal_hash_input(u, p)
        if kind == "bytes":
            assert hv == xxhash.xxh64_intdigest(v, seed=42), (u, p)
        assert int(cls) == O.datatype_class(O.decimal_to_string(u, s).encode()), (u, s)
    assert ties > 300  # exact ties were exercised (each rounded to the even neighbour: got == want above)


def test_decimal_to_string_forms():
    """BigDecimal.toString's plain / scientific switch (adjusted exponent -6) as the oracle restates it."""
    assert O.decimal_to_string(12345, 2) == "123.45"
    assert O.decimal_to_string(5, 2) == "0.05"
    assert O.decimal_to_string(10, 7) == "0.0000010"
    assert O.decimal_to_string(1, 7) == "1E-7"
    assert O.decimal_to_string(-15, 8) == "-1.5E-7"
    assert O.decimal_to_string(0, 18) == "0E-18"
    assert O.decimal_to_string(0, 6) == "0.000000"
    assert O.decimal_to_string(-99, 0) == "-99"
    assert O.decimal_to_string(123450000000000000000, 18) == "123.450000000000000000"
