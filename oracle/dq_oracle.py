"""CPU restatement of Deequ's fused scan semantics -- TEST INFRASTRUCTURE ONLY.

This module is the *checker* for the MI355X path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it; the product (``deequ_amd``) never does, and must fail loudly when its HIP
library is missing instead of falling back to anything in here.

What it restates (reference = malcolmgreaves/deequ, paths relative to
``src/main/scala/com/amazon/deequ/``):

* analyzer aggregation semantics: ``analyzers/{Size,Completeness,Compliance,Sum,
  Mean,StandardDeviation,Minimum,Maximum,Correlation,ApproxCountDistinct}.scala``
  and ``analyzers/Analyzer.scala:220-234, 337-443`` (conditionalSelection /
  conditionalCount / ifNoNullsIn / merge / metricFromEmpty);
* state algebra (``State.sum``) of every hot-path state type;
* HLL++ register update / pack / merge / estimate
  (``analyzers/catalyst/StatefulHyperloglogPlus.scala:89-297``, constants
  ``analyzers/catalyst/HLLConstants.scala:27-37,51,84``);
* ``HdfsStateProvider`` byte formats and file identifiers
  (``analyzers/StateProvider.scala:81-83, 176-294``);
* ``DataType`` (``analyzers/DataType.scala:40-183``) and its UDAF
  ``analyzers/catalyst/StatefulDataType.scala:26-83``: Scala ``Regex`` extractors
  (``Matcher.matches``, whole-value) over the value's Java string -- the UDAF's
  input is ``StringType``, so Spark casts numeric columns with
  ``Long/Integer.toString`` / ``Double.toString`` first.

Spark 2.2.2 itself is not vendored in the reference (pom.xml:79-83), so the
following are restated from Spark's published source and pinned by the
reference's own known-answer tests (see tests/golden/reference_kats.json) and,
for the hash, by the independent ``xxhash`` 3.8.1 Python package:

* ``CentralMomentAgg`` update/merge (StandardDeviation; call site
  ``analyzers/catalyst/StatefulStdDevPop.scala:24``),
* ``Corr`` update/merge (Correlation; ``analyzers/catalyst/StatefulCorrelation.scala:24``),
* ``XxHash64Function`` / ``XXH64.hashLong|hashInt|hashUnsafeBytes`` with seed 42
  (``analyzers/catalyst/StatefulHyperloglogPlus.scala:93``),
* SQL ``sum``/``count``/``min``/``max`` null semantics and three-valued logic.

Spark's partial/final aggregation is simulated exactly: rows are split into
``n_partitions`` contiguous partitions, each partition is folded sequentially
with the update expressions, and the final aggregate folds the partition
buffers in order into the zero buffer with the merge expressions.
"""
from __future__ import annotations

import math
import re
import struct
from dataclasses import dataclass
from fractions import Fraction
from typing import List, Optional, Sequence, Tuple

import numpy as np

MASK64 = (1 << 64) - 1

# --------------------------------------------------------------------------------------
# Java numeric helpers
# --------------------------------------------------------------------------------------


def to_i64(x: int) -> int:
    x &= MASK64
    return x - (1 << 64) if x >> 63 else x


def to_i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def java_math_round(a: float) -> int:
    """java.lang.Math.round(double) (JDK 8 bit algorithm; = floor(a + 1/2) exactly)."""
    if math.isnan(a):
        return 0
    bits = struct.unpack("<q", struct.pack("<d", a))[0]
    biased_exp = (bits & 0x7FF0000000000000) >> 52
    shift = (52 - 1 + 1023) - biased_exp
    if (shift & -64) == 0:
        r = (bits & 0x000FFFFFFFFFFFFF) | 0x0010000000000000
        if bits < 0:
            r = -r
        return ((r >> shift) + 1) >> 1
    # |a| >= 2^52 or tiny: (long) a  (saturating cast)
    if a >= 9.223372036854776e18:
        return (1 << 63) - 1
    if a <= -9.223372036854776e18:
        return -(1 << 63)
    return int(a)


def java_min(a: float, b: float) -> float:
    """java.lang.Math.min(double,double): NaN propagates, -0.0 < 0.0."""
    if a != a:
        return a
    if b != b:
        return b
    if a == 0.0 and b == 0.0:
        return a if math.copysign(1.0, a) < 0 else b
    return a if a <= b else b


def java_max(a: float, b: float) -> float:
    if a != a:
        return a
    if b != b:
        return b
    if a == 0.0 and b == 0.0:
        return a if math.copysign(1.0, a) > 0 else b
    return a if a >= b else b


def jdiv(a: float, b: float) -> float:
    """IEEE-754 double division as on the JVM (x/0 -> +-Infinity, 0/0 -> NaN)."""
    try:
        return a / b
    except ZeroDivisionError:
        if a != a or a == 0.0:
            return float("nan")
        return math.copysign(float("inf"), a) * math.copysign(1.0, b)


def double_to_long_bits(d: float) -> int:
    """java.lang.Double.doubleToLongBits (canonical NaN)."""
    if d != d:
        return 0x7FF8000000000000
    return struct.unpack("<q", struct.pack("<d", d))[0]


# --------------------------------------------------------------------------------------
# XXH64 as used by Spark's XxHash64Function (seed 42)
# --------------------------------------------------------------------------------------

P1 = 0x9E3779B185EBCA87
P2 = 0xC2B2AE3D27D4EB4F
P3 = 0x165667B19E3779F9
P4 = 0x85EBCA77C2B2AE63
P5 = 0x27D4EB2F165667C5
HLL_SEED = 42


def _rotl(x: int, r: int) -> int:
    x &= MASK64
    return ((x << r) | (x >> (64 - r))) & MASK64


def _fmix(h: int) -> int:
    h ^= h >> 33
    h = (h * P2) & MASK64
    h ^= h >> 29
    h = (h * P3) & MASK64
    h ^= h >> 32
    return h


def xxh64_long(v: int, seed: int = HLL_SEED) -> int:
    """XXH64.hashLong -> signed Java long."""
    h = (seed + P5 + 8) & MASK64
    h ^= (_rotl((v & MASK64) * P2, 31) * P1) & MASK64
    h = (_rotl(h, 27) * P1 + P4) & MASK64
    return to_i64(_fmix(h))


def xxh64_int(v: int, seed: int = HLL_SEED) -> int:
    """XXH64.hashInt -> signed Java long."""
    h = (seed + P5 + 4) & MASK64
    h ^= ((v & 0xFFFFFFFF) * P1) & MASK64
    h = (_rotl(h, 23) * P2 + P3) & MASK64
    return to_i64(_fmix(h))


def xxh64_bytes(b: bytes, seed: int = HLL_SEED) -> int:
    """XXH64.hashUnsafeBytes (little-endian words) -> signed Java long."""
    n = len(b)
    off = 0
    if n >= 32:
        v1 = (seed + P1 + P2) & MASK64
        v2 = (seed + P2) & MASK64
        v3 = seed & MASK64
        v4 = (seed - P1) & MASK64
        while off <= n - 32:
            w = struct.unpack_from("<4Q", b, off)
            v1 = (_rotl(v1 + w[0] * P2, 31) * P1) & MASK64
            v2 = (_rotl(v2 + w[1] * P2, 31) * P1) & MASK64
            v3 = (_rotl(v3 + w[2] * P2, 31) * P1) & MASK64
            v4 = (_rotl(v4 + w[3] * P2, 31) * P1) & MASK64
            off += 32
        h = (_rotl(v1, 1) + _rotl(v2, 7) + _rotl(v3, 12) + _rotl(v4, 18)) & MASK64
        for v in (v1, v2, v3, v4):
            v = (_rotl(v * P2, 31) * P1) & MASK64
            h ^= v
            h = (h * P1 + P4) & MASK64
    else:
        h = (seed + P5) & MASK64
    h = (h + n) & MASK64
    while off <= n - 8:
        k1 = struct.unpack_from("<Q", b, off)[0]
        h ^= (_rotl(k1 * P2, 31) * P1) & MASK64
        h = (_rotl(h, 27) * P1 + P4) & MASK64
        off += 8
    if off + 4 <= n:
        k = struct.unpack_from("<I", b, off)[0]
        h ^= (k * P1) & MASK64
        h = (_rotl(h, 23) * P2 + P3) & MASK64
        off += 4
    while off < n:
        h ^= (b[off] * P5) & MASK64
        h = (_rotl(h, 11) * P1) & MASK64
        off += 1
    return to_i64(_fmix(h))


# vectorised numpy forms (uint64 arithmetic wraps modulo 2^64)
_U = np.uint64


def _np_rotl(x, r):
    return (x << _U(r)) | (x >> _U(64 - r))


def _np_fmix(h):
    h = h ^ (h >> _U(33))
    h = h * _U(P2)
    h = h ^ (h >> _U(29))
    h = h * _U(P3)
    h = h ^ (h >> _U(32))
    return h


def np_xxh64_long(v: np.ndarray, seed: int = HLL_SEED) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = np.asarray(v).astype(np.int64).view(np.uint64)
        h = np.full(x.shape, (seed + P5 + 8) & MASK64, dtype=np.uint64)
        h ^= _np_rotl(x * _U(P2), 31) * _U(P1)
        h = _np_rotl(h, 27) * _U(P1) + _U(P4)
        return _np_fmix(h)


def np_xxh64_int(v: np.ndarray, seed: int = HLL_SEED) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = np.asarray(v).astype(np.int32).view(np.uint32).astype(np.uint64)
        h = np.full(x.shape, (seed + P5 + 4) & MASK64, dtype=np.uint64)
        h ^= x * _U(P1)
        h = _np_rotl(h, 23) * _U(P2) + _U(P3)
        return _np_fmix(h)


def np_double_to_long_bits(d: np.ndarray) -> np.ndarray:
    d = np.asarray(d, dtype=np.float64)
    bits = d.view(np.int64).copy()
    bits[np.isnan(d)] = 0x7FF8000000000000
    return bits


# --------------------------------------------------------------------------------------
# HLL++ (StatefulHyperloglogPlus.scala / HLLConstants.scala)
# --------------------------------------------------------------------------------------

RELATIVE_SD = 0.05
HLL_P = int(math.ceil(2.0 * math.log(1.106 / RELATIVE_SD) / math.log(2.0)))  # :157 -> 9
HLL_M = 1 << HLL_P  # :161 -> 512
IDX_SHIFT = 64 - HLL_P  # :159
W_PADDING = 1 << (HLL_P - 1)  # :160
REGISTER_SIZE = 6  # HLLConstants.scala:29
REGISTER_WORD_MASK = (1 << REGISTER_SIZE) - 1  # :31
REGISTERS_PER_WORD = 64 // REGISTER_SIZE  # :33 -> 10
NUM_WORDS = 52  # StatefulHyperloglogPlus.scala:154
HLL_K = 6  # HLLConstants.scala:35
THRESHOLDS = [10, 20, 40, 80, 220, 400, 900, 1800, 3100, 6500, 15500, 20000, 50000, 120000, 350000]
ALPHA_M2 = (0.7213 / (1.0 + 1.079 / HLL_M)) * HLL_M * HLL_M  # :163-168 (P >= 7 branch)


def _load_bias_tables():
    import json
    import os

    path = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "hll_p9_tables.json")
    with open(path) as f:
        t = json.load(f)
    return t["raw_estimate_p9"], t["bias_p9"]


RAW_ESTIMATE_P9, BIAS_P9 = _load_bias_tables()


def hll_index_and_pw(x_signed: int) -> Tuple[int, int]:
    """idx = x >>> IDX_SHIFT; pw = nlz((x << P) | W_PADDING) + 1 (:96-99)."""
    x = x_signed & MASK64
    idx = x >> IDX_SHIFT
    w = ((x << HLL_P) | W_PADDING) & MASK64
    pw = 64 - w.bit_length() + 1
    return idx, pw


def np_hll_registers(hashes_u64: np.ndarray, regs: Optional[np.ndarray] = None) -> np.ndarray:
    """Fold 64-bit hashes into 512 byte-registers (max of pw per index)."""
    if regs is None:
        regs = np.zeros(HLL_M, dtype=np.uint8)
    h = np.asarray(hashes_u64, dtype=np.uint64)
    if h.size == 0:
        return regs
    idx = (h >> _U(IDX_SHIFT)).astype(np.int64)
    w = (h << _U(HLL_P)) | _U(W_PADDING)
    # nlz via float exponent is unsafe for 64-bit; do it with bit_length on 32-bit halves
    hi = (w >> _U(32)).astype(np.uint64)
    lo = (w & _U(0xFFFFFFFF)).astype(np.uint64)
    nlz_hi = 32 - _bitlen32(hi)
    nlz_lo = 32 - _bitlen32(lo)
    nlz = np.where(hi != 0, nlz_hi, 32 + nlz_lo)
    pw = (nlz + 1).astype(np.uint8)
    np.maximum.at(regs, idx, pw)
    return regs


def _bitlen32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    n = np.zeros(x.shape, dtype=np.int64)
    for s in (16, 8, 4, 2, 1):
        m = x >= _U(1 << s)
        n += np.where(m, s, 0)
        x = np.where(m, x >> _U(s), x)
    n += (x > 0).astype(np.int64)
    return n


def registers_to_words(regs: Sequence[int]) -> List[int]:
    """512 registers -> 52 signed longs (10 x 6-bit registers per word, :102-112)."""
    words = [0] * NUM_WORDS
    for i, r in enumerate(regs):
        wo = i // REGISTERS_PER_WORD
        shift = REGISTER_SIZE * (i - wo * REGISTERS_PER_WORD)
        words[wo] |= (int(r) & REGISTER_WORD_MASK) << shift
    return [to_i64(w) for w in words]


def words_to_registers(words: Sequence[int]) -> List[int]:
    regs = []
    for i in range(HLL_M):
        wo = i // REGISTERS_PER_WORD
        shift = REGISTER_SIZE * (i - wo * REGISTERS_PER_WORD)
        regs.append(((words[wo] & MASK64) >> shift) & REGISTER_WORD_MASK)
    return regs


def hll_update_words(words: List[int], x_signed: int) -> None:
    """Exact StatefulHyperloglogPlus.update (:89-115) on a 52-word buffer."""
    idx, pw = hll_index_and_pw(x_signed)
    wo = idx // REGISTERS_PER_WORD
    word = words[wo] & MASK64
    shift = REGISTER_SIZE * (idx - wo * REGISTERS_PER_WORD)
    mask = REGISTER_WORD_MASK << shift
    m = (word & mask) >> shift
    if pw > m:
        words[wo] = to_i64((word & ~mask & MASK64) | (pw << shift))


def hll_merge_words(w1: Sequence[int], w2: Sequence[int]) -> List[int]:
    """DeequHyperLogLogPlusPlusUtils.merge (:188-208): per-register max."""
    dest = []
    idx = 0
    for wo in range(NUM_WORDS):
        a, b = w1[wo] & MASK64, w2[wo] & MASK64
        word = 0
        mask = REGISTER_WORD_MASK
        i = 0
        while idx < HLL_M and i < REGISTERS_PER_WORD:
            word |= max(a & mask, b & mask)
            mask <<= REGISTER_SIZE
            i += 1
            idx += 1
        dest.append(to_i64(word))
    return dest


def _estimate_bias(e: float) -> float:
    """DeequHyperLogLogPlusPlusUtils.estimateBias (:259-297) incl. Arrays.binarySearch."""
    est = RAW_ESTIMATE_P9
    n = len(est)
    lo, hi = 0, n - 1
    found = None
    while lo <= hi:  # java.util.Arrays.binarySearch(double[], ...)
        mid = (lo + hi) >> 1
        v = est[mid]
        if v < e:
            lo = mid + 1
        elif v > e:
            hi = mid - 1
        else:
            found = mid
            break
    nearest = found if found is not None else lo

    def distance(i):
        d = e - est[i]
        return d * d

    low = max(nearest - HLL_K + 1, 0)
    high = min(low + HLL_K, n)
    while high < n and distance(high) < distance(low):
        low += 1
        high += 1
    s = 0.0
    for i in range(low, high):
        s += BIAS_P9[i]
    return s / (high - low)


def hll_count(words: Sequence[int]) -> float:
    """DeequHyperLogLogPlusPlusUtils.count (:210-257) incl. the JVM `1 << Midx` Int quirk."""
    z_inverse = 0.0
    V = 0.0
    idx = 0
    for wo in range(len(words)):
        word = words[wo] & MASK64
        i = 0
        shift = 0
        while idx < HLL_M and i < REGISTERS_PER_WORD:
            m = (word >> shift) & REGISTER_WORD_MASK
            denom = to_i32(1 << (m & 31))  # Int << Long: shift count masked to 5 bits
            z_inverse += 1.0 / denom
            if m == 0:
                V += 1.0
            shift += REGISTER_SIZE
            i += 1
            idx += 1

    def e_bias_corrected():
        e = ALPHA_M2 / z_inverse
        if HLL_P < 19 and e < 5.0 * HLL_M:
            return e - _estimate_bias(e)
        return e

    if V > 0:
        H = HLL_M * math.log(HLL_M / V)
        estimate = H if H <= THRESHOLDS[HLL_P - 4] else e_bias_corrected()
    else:
        estimate = e_bias_corrected()
    return float(java_math_round(estimate))


def words_to_bytes(words: Sequence[int]) -> bytes:
    """wordsToBytes (:170-178): ByteBuffer default = big-endian."""
    return struct.pack(">52q", *[to_i64(w) for w in words])


def words_from_bytes(b: bytes) -> List[int]:
    assert len(b) == NUM_WORDS * 8
    return list(struct.unpack(">52q", b))


# --------------------------------------------------------------------------------------
# States (A12) -- exact State.sum semantics
# --------------------------------------------------------------------------------------


@dataclass(frozen=True)
class NumMatches:  # Size.scala:23-33
    numMatches: int

    def sum(self, o):
        return NumMatches(to_i64(self.numMatches + o.numMatches))

    def metricValue(self):
        return float(self.numMatches)


@dataclass(frozen=True)
class NumMatchesAndCount:  # Analyzer.scala:220-234
    numMatches: int
    count: int

    def sum(self, o):
        return NumMatchesAndCount(to_i64(self.numMatches + o.numMatches), to_i64(self.count + o.count))

    def metricValue(self):
        return float("nan") if self.count == 0 else float(self.numMatches) / self.count


@dataclass(frozen=True)
class SumState:  # Sum.scala:25-34
    sum_: float

    def sum(self, o):
        return SumState(self.sum_ + o.sum_)

    def metricValue(self):
        return self.sum_


@dataclass(frozen=True)
class MeanState:  # Mean.scala:25-34
    sum_: float
    count: int

    def sum(self, o):
        return MeanState(self.sum_ + o.sum_, to_i64(self.count + o.count))

    def metricValue(self):
        return float("nan") if self.count == 0 else jdiv(self.sum_, float(self.count))


@dataclass(frozen=True)
class StandardDeviationState:  # StandardDeviation.scala:25-45
    n: float
    avg: float
    m2: float

    def __post_init__(self):
        if not self.n > 0.0:
            raise ValueError("Standard deviation is undefined for n = 0.")

    def sum(self, o):
        newN = self.n + o.n
        delta = o.avg - self.avg
        deltaN = 0.0 if newN == 0.0 else delta / newN
        return StandardDeviationState(newN, self.avg + deltaN * o.n,
                                      self.m2 + o.m2 + delta * deltaN * self.n * o.n)

    def metricValue(self):
        q = jdiv(self.m2, self.n)
        return math.sqrt(q) if q >= 0 else float("nan")


@dataclass(frozen=True)
class MinState:  # Minimum.scala:25-34
    minValue: float

    def sum(self, o):
        return MinState(java_min(self.minValue, o.minValue))

    def metricValue(self):
        return self.minValue


@dataclass(frozen=True)
class MaxState:  # Maximum.scala:25-34
    maxValue: float

    def sum(self, o):
        return MaxState(java_max(self.maxValue, o.maxValue))

    def metricValue(self):
        return self.maxValue


@dataclass(frozen=True)
class CorrelationState:  # Correlation.scala:26-57
    n: float
    xAvg: float
    yAvg: float
    ck: float
    xMk: float
    yMk: float

    def __post_init__(self):
        if not self.n > 0.0:
            raise ValueError("Correlation undefined for n = 0.")

    def sum(self, o):
        n1, n2 = self.n, o.n
        newN = n1 + n2
        dx = o.xAvg - self.xAvg
        dxN = 0.0 if newN == 0.0 else dx / newN
        dy = o.yAvg - self.yAvg
        dyN = 0.0 if newN == 0.0 else dy / newN
        return CorrelationState(newN, self.xAvg + dxN * n2, self.yAvg + dyN * n2,
                                self.ck + o.ck + dx * dyN * n1 * n2,
                                self.xMk + o.xMk + dx * dxN * n1 * n2,
                                self.yMk + o.yMk + dy * dyN * n1 * n2)

    def metricValue(self):
        prod = self.xMk * self.yMk
        return jdiv(self.ck, math.sqrt(prod)) if prod >= 0 else float("nan")


@dataclass(frozen=True)
class ApproxCountDistinctState:  # ApproxCountDistinct.scala:26-40
    words: Tuple[int, ...]

    def sum(self, o):
        return ApproxCountDistinctState(tuple(hll_merge_words(self.words, o.words)))

    def metricValue(self):
        return hll_count(self.words)


@dataclass(frozen=True)
class DataTypeHistogram:  # DataType.scala:40-52
    numNull: int
    numFractional: int
    numIntegral: int
    numBoolean: int
    numString: int

    def sum(self, o):
        return DataTypeHistogram(self.numNull + o.numNull, self.numFractional + o.numFractional,
                                 self.numIntegral + o.numIntegral, self.numBoolean + o.numBoolean,
                                 self.numString + o.numString)

    def metricValue(self):
        raise TypeError("DataType has a HistogramMetric")


def merge_states(*states):
    """Analyzers.merge (Analyzer.scala:343-362)."""
    acc = None
    for s in states:
        if acc is None:
            acc = s
        elif s is not None:
            acc = acc.sum(s)
    return acc


# --------------------------------------------------------------------------------------
# Columns and the three-valued predicate evaluator (SQL semantics, Check.scala grammar)
# --------------------------------------------------------------------------------------


INTEGRAL = ("i64", "i32", "i16", "i8")  # LongType, IntegerType, ShortType, ByteType
FLOATING = ("f64", "f32")                # DoubleType, FloatType


def int_to_f32(v: int) -> float:
    """(float) v as Java's int / long -> float conversion rounds it (nearest, ties to even), exactly."""
    a = abs(int(v))
    nb = a.bit_length()
    if nb <= 24:
        return float(v)
    shift = nb - 24
    q, r = divmod(a, 1 << shift)
    half = 1 << (shift - 1)
    if r > half or (r == half and q & 1):
        q += 1
    return math.copysign(float(q << shift), v)


def float_to_int_bits(f: float) -> int:
    """java.lang.Float.floatToIntBits (every NaN as 0x7fc00000), as a signed int."""
    if f != f:
        return 0x7FC00000
    return struct.unpack("<i", struct.pack("<f", f))[0]


# DecimalType(p, s) (dtype "decimal(p,s)"; values: the unscaled Python ints).  Spark 2.2 reads a decimal through
# java.math.BigDecimal: Decimal.toDouble = BigDecimal.doubleValue (correctly rounded), Decimal.toString =
# BigDecimal.toString, and XxHash64 hashes hashLong(unscaled) for p <= 18, else BigInteger.toByteArray's bytes
# (InterpretedHashFunction.hash).  Sum is the exact decimal sum (sum(col) has type DecimalType(min(38, p + 10), s))
# cast to double at the end (Sum.scala:40).
def decimal_ps(dtype: str) -> Optional[Tuple[int, int]]:
    """(precision, scale) of a "decimal(p,s)" dtype, else None."""
    if not dtype.startswith("decimal("):
        return None
    p, s = dtype[8:-1].split(",")
    return int(p), int(s)


def decimal_to_double(u: int, s: int) -> float:
    """BigDecimal.doubleValue of unscaled u at scale s: Fraction -> float rounds to nearest, ties to even."""
    return float(Fraction(int(u), 10 ** s))


def decimal_to_string(u: int, s: int) -> str:
    """java.math.BigDecimal.toString (scale >= 0): plain unless the adjusted exponent is below -6."""
    u = int(u)
    sign = "-" if u < 0 else ""
    coeff = str(abs(u))
    adjusted = len(coeff) - 1 - s
    if s == 0:
        return sign + coeff
    if adjusted >= -6:
        if len(coeff) > s:
            return f"{sign}{coeff[:-s]}.{coeff[-s:]}"
        return f"{sign}0.{'0' * (s - len(coeff))}{coeff}"
    mant = coeff[0] + ("." + coeff[1:] if len(coeff) > 1 else "")
    return f"{sign}{mant}E{adjusted}"


def decimal_hash_input(u: int, p: int):
    """What XxHash64 hashes for a decimal: ("long", unscaled) for p <= 18, else ("bytes", toByteArray)."""
    u = int(u)
    if p <= 18:
        return "long", u
    bl = (u if u >= 0 else ~u).bit_length()  # BigInteger.bitLength
    return "bytes", u.to_bytes(bl // 8 + 1, "big", signed=True)


def decimal_hash(u: int, p: int) -> int:
    kind, v = decimal_hash_input(u, p)
    return xxh64_long(v) if kind == "long" else xxh64_bytes(v)


@dataclass
class OColumn:
    """A column for the oracle: dtype in {f64, f32, i64, i32, i16, i8, bool, date32, timestamp, utf8,
    decimal(p,s)}; values + boolean validity (bool: a bool array; date32: int32 days; timestamp: int64
    microseconds, UTC; decimal: the unscaled values as Python ints)."""

    dtype: str
    values: object  # np.ndarray for numerics, list[bytes|None] for utf8
    valid: np.ndarray  # bool

    def __len__(self):
        return len(self.valid)


class _Tok:
    def __init__(self, s: str):
        self.toks = []
        i = 0
        while i < len(s):
            c = s[i]
            if c.isspace():
                i += 1
            elif c == "`":
                j = s.index("`", i + 1)
                self.toks.append(("id", s[i + 1:j]))
                i = j + 1
            elif c == "'":
                j = s.index("'", i + 1)
                self.toks.append(("str", s[i + 1:j]))
                i = j + 1
            elif c.isdigit() or (c == "." and i + 1 < len(s) and s[i + 1].isdigit()):
                j = i
                while j < len(s) and (s[j].isdigit() or s[j] in ".eE" or
                                      (s[j] in "+-" and s[j - 1] in "eE")):
                    j += 1
                self.toks.append(("num", s[i:j]))
                i = j
            elif c.isalpha() or c == "_":
                j = i
                while j < len(s) and (s[j].isalnum() or s[j] == "_"):
                    j += 1
                w = s[i:j]
                if w.upper() in ("AND", "OR", "NOT", "IS", "NULL", "COALESCE", "IN", "TRUE", "FALSE"):
                    self.toks.append(("kw", w.upper()))
                else:
                    self.toks.append(("id", w))
                i = j
            elif s.startswith(("<=", ">=", "!=", "<>", "=="), i):
                self.toks.append(("op", s[i:i + 2]))
                i += 2
            elif c in "<>=(),-":
                self.toks.append(("op", c))
                i += 1
            else:
                raise ValueError(f"unexpected character {c!r} in {s!r}")
        self.pos = 0

    def peek(self):
        return self.toks[self.pos] if self.pos < len(self.toks) else (None, None)

    def take(self):
        t = self.peek()
        self.pos += 1
        return t


class OracleExpr:
    """Evaluates a Spark-SQL predicate string with three-valued logic over OColumns.

    Value model: (values, type, notnull) with type in {'int','dec','dbl','str','bool'}.
    Literal typing follows Spark 2.2: `3` int, `3.0` decimal, `3e0` double.
    Comparisons: int/dec vs int/dec exact (python ints / fractions); anything vs double
    in double; strings compared as UTF-8 bytes.
    """

    def __init__(self, text: str):
        self.text = text
        self.t = _Tok(text)
        self.ast = self._or()
        if self.t.peek()[0] is not None:
            raise ValueError(f"trailing tokens in {text!r}")

    def _or(self):
        a = self._and()
        while self.t.peek() == ("kw", "OR"):
            self.t.take()
            a = ("or", a, self._and())
        return a

    def _and(self):
        a = self._not()
        while self.t.peek() == ("kw", "AND"):
            self.t.take()
            a = ("and", a, self._not())
        return a

    def _not(self):
        if self.t.peek() == ("kw", "NOT"):
            self.t.take()
            return ("not", self._not())
        return self._cmp()

    def _cmp(self):
        a = self._atom()
        k, v = self.t.peek()
        if k == "op" and v in ("<", "<=", ">", ">=", "=", "==", "!=", "<>"):
            self.t.take()
            b = self._atom()
            v = {"==": "=", "<>": "!="}.get(v, v)
            return ("cmp", v, a, b)
        if (k, v) == ("kw", "IS"):
            self.t.take()
            neg = False
            if self.t.peek() == ("kw", "NOT"):
                self.t.take()
                neg = True
            assert self.t.take() == ("kw", "NULL")
            return ("isnotnull" if neg else "isnull", a)
        if (k, v) == ("kw", "IN") or (k, v) == ("kw", "NOT"):
            neg = False
            if v == "NOT":
                self.t.take()
                neg = True
            assert self.t.take() == ("kw", "IN")
            assert self.t.take() == ("op", "(")
            items = [self._atom()]
            while self.t.peek() == ("op", ","):
                self.t.take()
                items.append(self._atom())
            assert self.t.take() == ("op", ")")
            e = ("in", a, items)
            return ("not", e) if neg else e
        return a

    def _atom(self):
        k, v = self.t.take()
        if k == "op" and v == "(":
            e = self._or()
            assert self.t.take() == ("op", ")")
            return e
        if k == "op" and v == "-":
            k2, v2 = self.t.take()
            assert k2 == "num"
            return self._num("-" + v2)
        if k == "num":
            return self._num(v)
        if k == "str":
            return ("lit", "str", v.encode("utf-8"))
        if k == "kw" and v == "NULL":
            return ("lit", "null", None)
        if k == "kw" and v in ("TRUE", "FALSE"):
            return ("lit", "bool", v == "TRUE")
        if k == "kw" and v == "COALESCE":
            assert self.t.take() == ("op", "(")
            args = [self._or()]
            while self.t.peek() == ("op", ","):
                self.t.take()
                args.append(self._or())
            assert self.t.take() == ("op", ")")
            return ("coalesce", args)
        if k == "id":
            return ("col", v)
        raise ValueError(f"unexpected token {(k, v)} in {self.text!r}")

    @staticmethod
    def _num(s: str):
        from fractions import Fraction

        if "e" in s or "E" in s:
            return ("lit", "dbl", float(s))
        if "." in s:
            return ("lit", "dec", Fraction(s))
        return ("lit", "int", int(s))

    # ---- evaluation: returns (vals: list, typ, notnull: np.bool_ array) ----
    def eval(self, cols: dict, n: int):
        return self._ev(self.ast, cols, n)

    def eval_bool(self, cols: dict, n: int):
        vals, typ, nn = self._ev(self.ast, cols, n)
        if typ == "null":  # a bare NULL literal is a NULL boolean
            return np.zeros(n, dtype=bool), np.zeros(n, dtype=bool)
        assert typ == "bool", f"predicate {self.text!r} is not boolean"
        return np.array([bool(x) for x in vals], dtype=bool) & nn, nn

    def _ev(self, e, cols, n):
        from fractions import Fraction

        kind = e[0]
        if kind == "lit":
            typ, v = e[1], e[2]
            if typ == "null":
                return [None] * n, "null", np.zeros(n, dtype=bool)
            return [v] * n, typ, np.ones(n, dtype=bool)
        if kind == "col":
            c = cols[e[1]]
            if c.dtype == "f64":
                return [float(x) for x in c.values], "dbl", c.valid.copy()
            if c.dtype == "f32":  # FloatType: compared in float against integers, in double otherwise
                return [float(x) for x in c.values], "flt", c.valid.copy()
            if c.dtype in INTEGRAL:
                return [int(x) for x in c.values], "int", c.valid.copy()
            if c.dtype == "bool":
                return [bool(x) for x in c.values], "bool", c.valid.copy()
            if c.dtype == "utf8":
                return list(c.values), "str", c.valid.copy()
            if c.dtype in ("date32", "timestamp"):  # only their NULLs are read (IS [NOT] NULL)
                return [int(x) for x in c.values], c.dtype, c.valid.copy()
            if decimal_ps(c.dtype):  # DecimalType: exact values (vs int / decimal: exact; vs double: the cast)
                sc = decimal_ps(c.dtype)[1]
                return [Fraction(int(x), 10 ** sc) for x in c.values], "dec", c.valid.copy()
            raise NotImplementedError(c.dtype)
        if kind == "coalesce":
            parts = [self._ev(a, cols, n) for a in e[1]]
            typ = _widen([p[1] for p in parts if p[1] != "null"])
            vals = [None] * n
            nn = np.zeros(n, dtype=bool)
            for pv, pt, pn in parts:
                for i in range(n):
                    if not nn[i] and pn[i]:
                        vals[i] = _coerce(pv[i], pt, typ)
                        nn[i] = True
            return vals, typ, nn
        if kind == "cmp":
            op = e[1]
            av, at, an = self._ev(e[2], cols, n)
            bv, bt, bn = self._ev(e[3], cols, n)
            if {at, bt} & {"date32", "timestamp"}:
                raise NotImplementedError("date / timestamp comparison")  # outside the restated grammar
            if at == "str" or bt == "str":
                if at != bt:
                    raise NotImplementedError("string/number comparison")
                typ = "str"
            else:
                typ = _widen([at, bt])
            nn = an & bn
            out = []
            for i in range(n):
                if not nn[i]:
                    out.append(False)
                    continue
                x, y = _coerce(av[i], at, typ), _coerce(bv[i], bt, typ)
                out.append(_cmp(op, x, y))
            return out, "bool", nn
        if kind == "in":
            av, at, an = self._ev(e[1], cols, n)
            items = [self._ev(it, cols, n) for it in e[2]]
            # x IN (a,b) == x = a OR x = b (three-valued)
            t = np.zeros(n, dtype=bool)
            anynull = ~an
            for iv, it, inn in items:
                for i in range(n):
                    if an[i] and inn[i] and iv[i] == av[i]:
                        t[i] = True
                anynull = anynull | ~inn
            nn = t | ~anynull
            return list(t), "bool", nn
        if kind in ("and", "or"):
            av, _, an = self._ev(e[1], cols, n)
            bv, _, bn = self._ev(e[2], cols, n)
            a_t = np.array(av, dtype=bool) & an
            b_t = np.array(bv, dtype=bool) & bn
            a_f = ~np.array(av, dtype=bool) & an
            b_f = ~np.array(bv, dtype=bool) & bn
            if kind == "and":
                t = a_t & b_t
                f = a_f | b_f
            else:
                t = a_t | b_t
                f = a_f & b_f
            return list(t), "bool", t | f
        if kind == "not":
            av, _, an = self._ev(e[1], cols, n)
            return [not x for x in av], "bool", an
        if kind == "isnull":
            _, _, an = self._ev(e[1], cols, n)
            return list(~an), "bool", np.ones(n, dtype=bool)
        if kind == "isnotnull":
            _, _, an = self._ev(e[1], cols, n)
            return list(an), "bool", np.ones(n, dtype=bool)
        raise ValueError(kind)


class NpPredicate:
    """OracleExpr's semantics vectorised with numpy, for the numeric predicates of the full-scale parity
    runs (Compliance over 1e9 rows; the per-row evaluator above is the reference at small n and
    tests/test_oracle.py checks the two agree).  cols: {name: (dtype, values ndarray, valid bool ndarray)}
    with numeric dtypes only.

    Value model: (kind, v, notnull), kind in {int, dec, dbl, bool, null}; int / dec hold int64 arrays (a
    column, or an integral decimal coalesced into one) or Python ints / Fractions (literals).  int vs dec
    compares exactly (Spark 2.2 widens LongType vs DECIMAL to a decimal); anything vs double compares in
    double with NaN as the largest value (nanSafe ordering), as _cmp does.
    """

    def __init__(self, text: str):
        self.expr = OracleExpr(text)

    def eval_bool(self, cols: dict, n: int):
        """(TRUE rows, non-NULL rows) as bool arrays."""
        kind, v, nn = self._ev(self.expr.ast, cols, n)
        if kind == "null":
            z = np.zeros(n, dtype=bool)
            return z, z
        assert kind == "bool", self.expr.text
        return np.broadcast_to(np.asarray(v, dtype=bool), (n,)) & nn, nn

    def _ev(self, e, cols, n):
        from fractions import Fraction

        kind = e[0]
        if kind == "lit":
            typ, v = e[1], e[2]
            if typ == "null":
                return "null", None, np.zeros(n, dtype=bool)
            if typ == "str":
                raise NotImplementedError("string literal")
            return typ, v, np.ones(n, dtype=bool)
        if kind == "col":
            dtype, vals, valid = cols[e[1]]
            if dtype == "f64":
                return "dbl", np.asarray(vals, dtype=np.float64), np.asarray(valid, dtype=bool)
            if dtype == "f32":
                return "flt", np.asarray(vals, dtype=np.float32).astype(np.float64), np.asarray(valid, dtype=bool)
            if dtype in INTEGRAL:
                return "int", np.asarray(vals, dtype=np.int64), np.asarray(valid, dtype=bool)
            if dtype == "bool":
                return "bool", np.asarray(vals, dtype=bool), np.asarray(valid, dtype=bool)
            if dtype in ("date32", "timestamp"):  # only their NULLs are read (IS [NOT] NULL)
                return dtype, np.asarray(vals, dtype=np.int64), np.asarray(valid, dtype=bool)
            raise NotImplementedError(dtype)
        if kind == "coalesce":
            parts = [self._ev(a, cols, n) for a in e[1]]
            typ = _widen([p[0] for p in parts if p[0] != "null"])
            if typ in ("int", "dec"):
                vals, np_t = np.zeros(n, dtype=np.int64), np.int64
            elif typ in ("dbl", "flt"):
                vals, np_t = np.zeros(n, dtype=np.float64), np.float64
            else:
                raise NotImplementedError(typ)
            nn = np.zeros(n, dtype=bool)
            for pk, pv, pn in parts:
                if pk == "null":
                    continue
                if typ != "dbl" and isinstance(pv, Fraction):
                    if pv.denominator != 1:
                        raise NotImplementedError("non-integral decimal in COALESCE over an integral column")
                    pv = int(pv)
                take = ~nn & pn
                if typ == "flt" and not isinstance(pv, np.ndarray):  # an integer literal cast to float
                    pv = int_to_f32(int(pv)) if pk == "int" else float(pv)
                src = np.broadcast_to(np.asarray(float(pv) if typ == "dbl" and not isinstance(pv, np.ndarray) else pv,
                                                 dtype=np_t), (n,))
                vals[take] = src[take].astype(np_t)
                nn |= pn
            return typ, vals, nn
        if kind == "cmp":
            op = e[1]
            ak, av, an = self._ev(e[2], cols, n)
            bk, bv, bn = self._ev(e[3], cols, n)
            nn = an & bn
            if ak == "null" or bk == "null":
                return "bool", np.zeros(n, dtype=bool), np.zeros(n, dtype=bool)
            if {ak, bk} & {"date32", "timestamp"}:
                raise NotImplementedError("date / timestamp comparison")
            if "dbl" in (ak, bk):
                return "bool", _np_cmp_dbl(op, _as_f64(av), _as_f64(bv)) & nn, nn
            if "flt" in (ak, bk):  # FloatType: integers rounded to float, decimals to double (_widen)
                av, bv = _flt_operand(ak, av, bk), _flt_operand(bk, bv, ak)
                return "bool", _np_cmp_dbl(op, _as_f64(av), _as_f64(bv)) & nn, nn
            if ak == "bool" or bk == "bool":  # boolean vs boolean: false < true
                av = np.asarray(av).astype(np.int64) if isinstance(av, np.ndarray) else int(av)
                bv = np.asarray(bv).astype(np.int64) if isinstance(bv, np.ndarray) else int(bv)
            return "bool", _np_cmp_exact(op, av, bv, n) & nn, nn
        if kind == "in":
            ak, av, an = self._ev(e[1], cols, n)
            t = np.zeros(n, dtype=bool)
            anynull = ~an
            for it in e[2]:
                ik, iv, inn = self._ev(it, cols, n)
                if ik == "null":
                    anynull = anynull | ~inn
                    continue
                eq = _np_cmp_dbl("=", _as_f64(av), _as_f64(iv)) if "dbl" in (ak, ik) else _np_cmp_exact("=", av, iv, n)
                t |= eq & an & inn
                anynull = anynull | ~inn
            return "bool", t, t | ~anynull
        if kind in ("and", "or"):
            _, av, an = self._ev(e[1], cols, n)
            _, bv, bn = self._ev(e[2], cols, n)
            a_t, b_t = np.asarray(av, dtype=bool) & an, np.asarray(bv, dtype=bool) & bn
            a_f, b_f = ~np.asarray(av, dtype=bool) & an, ~np.asarray(bv, dtype=bool) & bn
            t, f = (a_t & b_t, a_f | b_f) if kind == "and" else (a_t | b_t, a_f & b_f)
            return "bool", t, t | f
        if kind == "not":
            _, av, an = self._ev(e[1], cols, n)
            return "bool", ~np.asarray(av, dtype=bool) & an, an
        if kind in ("isnull", "isnotnull"):
            _, _, an = self._ev(e[1], cols, n)
            return "bool", (~an if kind == "isnull" else an.copy()), np.ones(n, dtype=bool)
        raise NotImplementedError(kind)


def _as_f64(v):
    return v.astype(np.float64) if isinstance(v, np.ndarray) else np.float64(float(v))


def _flt_operand(kind, v, other):
    """An operand of a comparison with a FloatType side, as the double Spark compares: integers (ShortType /
    ByteType columns: exact; literals: rounded) cast to float, unless the other side is a decimal (double)."""
    if kind == "int" and other != "dec":
        if isinstance(v, np.ndarray):
            return v.astype(np.float32).astype(np.float64)  # (|v| < 2^24 for i16 / i8: exact)
        return int_to_f32(int(v))
    if isinstance(v, np.ndarray):
        return v
    return float(v)


def _np_cmp_dbl(op, x, y):
    xn, yn = np.isnan(x), np.isnan(y)
    with np.errstate(invalid="ignore"):
        c = np.where(xn | yn, np.where(xn & yn, 0, np.where(xn, 1, -1)), (x > y).astype(np.int8) - (x < y))
    return {"<": c < 0, "<=": c <= 0, ">": c > 0, ">=": c >= 0, "=": c == 0, "!=": c != 0}[op]


def _np_cmp_exact(op, x, y, n):
    """integers (int64 arrays) / exact literals (int, Fraction) compared exactly"""
    import math as _m
    from fractions import Fraction

    if not isinstance(x, np.ndarray) and not isinstance(y, np.ndarray):
        c = (x > y) - (x < y)
        r = {"<": c < 0, "<=": c <= 0, ">": c > 0, ">=": c >= 0, "=": c == 0, "!=": c != 0}[op]
        return np.full(n, r, dtype=bool)
    if not isinstance(x, np.ndarray):  # literal op array  ->  array op' literal
        op = {"<": ">", "<=": ">=", ">": "<", ">=": "<=", "=": "=", "!=": "!="}[op]
        x, y = y, x
    if isinstance(y, np.ndarray):
        return {"<": x < y, "<=": x <= y, ">": x > y, ">=": x >= y, "=": x == y, "!=": x != y}[op]
    q = Fraction(y)
    lo, hi = -(1 << 63), (1 << 63) - 1
    fl, ce = _m.floor(q), _m.ceil(q)

    def bound(b):  # clamp an integer bound into int64 (comparisons with out-of-range bounds saturate)
        return np.int64(min(max(b, lo), hi))

    if op == "<":
        return x < bound(ce) if ce <= hi else np.ones(n, dtype=bool)
    if op == ">=":
        return x >= bound(ce) if ce <= hi else np.zeros(n, dtype=bool)
    if op == "<=":
        return x <= bound(fl) if fl >= lo else np.zeros(n, dtype=bool)
    if op == ">":
        return x > bound(fl) if fl >= lo else np.ones(n, dtype=bool)
    eq = (x == bound(fl)) if (q.denominator == 1 and lo <= fl <= hi) else np.zeros(n, dtype=bool)
    return eq if op == "=" else ~eq


def _widen(types):
    """Spark 2.2's common type of a comparison / COALESCE: findTightestCommonType over the numeric precedence
    (int < float < double; an integer literal against a FloatType column is cast to float), DecimalPrecision
    (a decimal with a float / double: double; with an integer: decimal)."""
    types = [t for t in types if t != "null"]
    if not types:
        return "null"
    if "dbl" in types or ("flt" in types and "dec" in types):
        return "dbl"
    if "dec" in types:
        return "dec"
    if "flt" in types:
        return "flt"
    if "bool" in types:
        return "bool"
    if "str" in types:
        return "str"
    return "int"


def _coerce(v, frm, to):
    from fractions import Fraction

    if v is None:
        return None
    if to == "flt":
        return float(v) if frm == "flt" else int_to_f32(int(v))
    if to == "dbl":
        return float(v)
    if to == "dec":
        return Fraction(v)
    return v


def _cmp(op, x, y):
    if isinstance(x, float) or isinstance(y, float):
        # Spark compares doubles with NaN as the largest value (nanSafe ordering for =, <, >)
        xn, yn = x != x, y != y
        if xn or yn:
            c = 0 if (xn and yn) else (1 if xn else -1)
        else:
            c = (x > y) - (x < y)
    else:
        c = (x > y) - (x < y)
    return {"<": c < 0, "<=": c <= 0, ">": c > 0, ">=": c >= 0, "=": c == 0, "!=": c != 0}[op]


# --------------------------------------------------------------------------------------
# Spark aggregation semantics (partial per partition + ordered final merge)
# --------------------------------------------------------------------------------------


def _partitions(n: int, n_partitions: int):
    n_partitions = max(1, n_partitions)
    bounds = [(n * p) // n_partitions for p in range(n_partitions + 1)]
    return [(bounds[p], bounds[p + 1]) for p in range(n_partitions)]


def _as_double_list(c: OColumn):
    """Cast(child, DoubleType) of every value (exact for float and every integral type)."""
    if c.dtype in FLOATING:
        return [float(x) for x in c.values]
    ps = decimal_ps(c.dtype)
    if ps:  # Decimal.toDouble: correctly rounded
        return [decimal_to_double(int(x), ps[1]) for x in c.values]
    return [float(int(x)) for x in c.values]


def spark_stddev_buffer(x: List[float], sel: np.ndarray, n_partitions: int = 1):
    """CentralMomentAgg (momentOrder 2) partial updates + final merges; returns (n, avg, m2)."""
    partials = []
    for lo, hi in _partitions(len(sel), n_partitions):
        n = avg = m2 = 0.0
        for i in range(lo, hi):
            if sel[i]:
                newN = n + 1.0
                delta = x[i] - avg
                deltaN = delta / newN
                avg = avg + deltaN
                m2 = m2 + delta * (delta - deltaN)
                n = newN
        partials.append((n, avg, m2))
    n = avg = m2 = 0.0  # final aggregate starts from the initial (zero) buffer
    for n2, avg2, m22 in partials:
        newN = n + n2
        delta = avg2 - avg
        deltaN = 0.0 if newN == 0.0 else delta / newN
        avg = avg + deltaN * n2
        m2 = m2 + m22 + delta * deltaN * n * n2
        n = newN
    return n, avg, m2


def spark_corr_buffer(x: List[float], y: List[float], sel: np.ndarray, n_partitions: int = 1):
    """Corr partial updates + final merges; returns (n, xAvg, yAvg, ck, xMk, yMk)."""
    partials = []
    for lo, hi in _partitions(len(sel), n_partitions):
        n = xAvg = yAvg = ck = xMk = yMk = 0.0
        for i in range(lo, hi):
            if sel[i]:
                newN = n + 1.0
                dx = x[i] - xAvg
                dxN = dx / newN
                dy = y[i] - yAvg
                dyN = dy / newN
                newXAvg = xAvg + dxN
                newYAvg = yAvg + dyN
                ck = ck + dx * (y[i] - newYAvg)
                xMk = xMk + dx * (x[i] - newXAvg)
                yMk = yMk + dy * (y[i] - newYAvg)
                xAvg, yAvg, n = newXAvg, newYAvg, newN
        partials.append((n, xAvg, yAvg, ck, xMk, yMk))
    n = xAvg = yAvg = ck = xMk = yMk = 0.0
    for n2, xA2, yA2, ck2, xM2, yM2 in partials:
        n1 = n
        newN = n1 + n2
        dx = xA2 - xAvg
        dxN = 0.0 if newN == 0.0 else dx / newN
        dy = yA2 - yAvg
        dyN = 0.0 if newN == 0.0 else dy / newN
        xAvg = xAvg + dxN * n2
        yAvg = yAvg + dyN * n2
        ck = ck + ck2 + dx * dyN * n1 * n2
        xMk = xMk + xM2 + dx * dxN * n1 * n2
        yMk = yMk + yM2 + dy * dyN * n1 * n2
        n = newN
    return n, xAvg, yAvg, ck, xMk, yMk


def spark_sum(c: OColumn, sel: np.ndarray, n_partitions: int = 1):
    """sum(col): integral -> wrapping long sum; double -> sequential double sum; decimal(p, s) -> the exact sum in
    DecimalType(min(38, p + 10), s), NULL past that precision (Spark 2.2 overflow; an intermediate overflow depends
    on Spark's row order and is not restated), cast to double; None if empty."""
    if not sel.any():
        return None
    ps = decimal_ps(c.dtype)
    if ps:
        tot = sum(int(c.values[i]) for i in np.nonzero(sel)[0])
        if abs(tot) >= 10 ** min(38, ps[0] + 10):
            return None
        return decimal_to_double(tot, ps[1])
    parts = []
    for lo, hi in _partitions(len(sel), n_partitions):
        if not sel[lo:hi].any():
            continue
        if c.dtype in INTEGRAL:  # Sum of an integral child: LongType (wrapping)
            s = 0
            for i in range(lo, hi):
                if sel[i]:
                    s = to_i64(s + int(c.values[i]))
        else:
            s = 0.0
            for i in range(lo, hi):
                if sel[i]:
                    s += float(c.values[i])
        parts.append(s)
    tot = parts[0]
    for p in parts[1:]:
        tot = to_i64(tot + p) if c.dtype in INTEGRAL else tot + p
    return float(tot)


def _nan_safe_lt(a, b):
    an, bn = a != a, b != b
    if an or bn:
        return (not an) and bn
    return a < b


def spark_min(c: OColumn, sel: np.ndarray, is_max: bool = False):
    """min/max(col) with Spark's NaN-as-largest ordering; integral compared as integers."""
    if not sel.any():
        return None
    ps = decimal_ps(c.dtype)
    if ps:  # min / max of the exact decimals, cast to double
        vals = [int(c.values[i]) for i in np.nonzero(sel)[0]]
        return decimal_to_double(max(vals) if is_max else min(vals), ps[1])
    best = None
    for i in np.nonzero(sel)[0]:
        v = int(c.values[i]) if c.dtype in INTEGRAL else float(c.values[i])
        if best is None:
            best = v
        elif is_max:
            if _nan_safe_lt(best, v):
                best = v
        else:
            if _nan_safe_lt(v, best):
                best = v
    return float(best)


def hll_words_for(c: OColumn, sel: np.ndarray) -> Tuple[int, ...]:
    """stateful_approx_count_distinct registers for a column (XxHash64 seed 42)."""
    idx = np.nonzero(sel)[0]
    # Spark 2.2 XxHash64Function per type: hashLong for LongType / TimestampType / DoubleType (doubleToLongBits),
    # hashInt for IntegerType / ShortType / ByteType / DateType (widened to int), FloatType (floatToIntBits) and
    # BooleanType (1 / 0)
    if c.dtype in ("i64", "timestamp"):
        h = np_xxh64_long(np.asarray(c.values)[idx])
    elif c.dtype == "f64":
        h = np_xxh64_long(np_double_to_long_bits(np.asarray(c.values)[idx]))
    elif c.dtype in ("i32", "i16", "i8", "date32", "bool"):
        h = np_xxh64_int(np.asarray(c.values)[idx].astype(np.int64))
    elif c.dtype == "f32":
        h = np_xxh64_int(np.array([float_to_int_bits(float(x)) for x in np.asarray(c.values, dtype=np.float32)[idx]],
                                  dtype=np.int64))
    elif c.dtype == "utf8":
        h = np.array([xxh64_bytes(c.values[i]) & MASK64 for i in idx], dtype=np.uint64)
    elif decimal_ps(c.dtype):  # hashLong(unscaled) for p <= 18, else hashUnsafeBytes(BigInteger.toByteArray)
        p = decimal_ps(c.dtype)[0]
        h = np.array([decimal_hash(int(c.values[i]), p) & MASK64 for i in idx], dtype=np.uint64)
    else:
        raise ValueError(c.dtype)
    regs = np_hll_registers(h)
    return tuple(registers_to_words(regs.tolist()))


# --------------------------------------------------------------------------------------
# Analyzers -> Option[State]   (the oracle's runScanningAnalyzers)
# --------------------------------------------------------------------------------------


# StatefulDataType.scala:36-38.  Java's \\d is [0-9] (no UNICODE_CHARACTER_CLASS), and the Scala
# extractor calls Matcher.matches(), i.e. re.fullmatch: a trailing line terminator does not match.
_DT_FRACTIONAL = re.compile(rb"(-|\+)? ?[0-9]*\.[0-9]*")
_DT_INTEGRAL = re.compile(rb"(-|\+)? ?[0-9]*")
_DT_BOOLEAN = re.compile(rb"(true|false)")


def java_double_to_string(d: float) -> str:
    """java.lang.Double.toString: plain decimal for 1e-3 <= |d| < 1e7 (and zero), else computerized
    scientific notation ("1.0E7", "1.234E-5"), "NaN", "Infinity".  The digits are Python's shortest
    repr (Java's can differ in the last digit, which does not change the DataType class)."""
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    a = abs(d)
    if 1e-3 <= a < 1e7:
        r = repr(d)  # Python uses positional notation throughout [1e-4, 1e16)
        return r if "." in r else r + ".0"
    mant, exp = ("%.16e" % d).split("e")
    mant = mant.rstrip("0")
    return f"{mant}0E{int(exp)}" if mant.endswith(".") else f"{mant}E{int(exp)}"


def datatype_class(value: bytes) -> int:
    """StatefulDataType.update (:58-69): 1 FRACTIONAL, 2 INTEGRAL, 3 BOOLEAN, 4 STRING, first match
    wins.  `value` is the UTF-8 of the Java string; every pattern is ASCII-only, so a value with any
    byte >= 0x80 (decoded to a non-ASCII char, or U+FFFD if invalid) is a STRING either way."""
    if _DT_FRACTIONAL.fullmatch(value):
        return 1
    if _DT_INTEGRAL.fullmatch(value):
        return 2
    if _DT_BOOLEAN.fullmatch(value):
        return 3
    return 4


def java_float_to_string(f: float) -> str:
    """java.lang.Float.toString: the same forms as Double.toString (plain decimal for 1e-3 <= |f| < 1e7 and
    zero, else computerized scientific notation, "NaN", "Infinity") with float's shortest digits."""
    if math.isnan(f) or math.isinf(f) or f == 0.0 or not (1e-3 <= abs(f) < 1e7):
        if math.isnan(f) or math.isinf(f) or f == 0.0:
            return java_double_to_string(f)
        m, e = np.format_float_scientific(np.float32(f), unique=True, exp_digits=1).split("e")
        return f"{m if '.' in m and not m.endswith('.') else m.rstrip('.') + '.0'}E{int(e)}"
    r = np.format_float_positional(np.float32(f), unique=True)
    return r + "0" if r.endswith(".") else r


def _value_string(c: "OColumn", i: int) -> bytes:
    """CAST(value AS STRING) of a column value, as UTF-8 (timestamps in UTC)."""
    import datetime

    if c.dtype in ("utf8", "large_utf8"):
        return c.values[i]
    if c.dtype == "f64":
        return java_double_to_string(float(c.values[i])).encode()
    if c.dtype == "f32":
        return java_float_to_string(float(c.values[i])).encode()
    if c.dtype == "bool":
        return b"true" if c.values[i] else b"false"
    if c.dtype == "date32":
        return (datetime.date(1970, 1, 1) + datetime.timedelta(days=int(c.values[i]))).isoformat().encode()
    if decimal_ps(c.dtype):  # Decimal.toString = BigDecimal.toString
        return decimal_to_string(int(c.values[i]), decimal_ps(c.dtype)[1]).encode()
    if c.dtype == "timestamp":  # DateTimeUtils.timestampToString: yyyy-MM-dd HH:mm:ss[.fraction, zeros trimmed]
        t = datetime.datetime(1970, 1, 1) + datetime.timedelta(microseconds=int(c.values[i]))
        frac = f"{t.microsecond:06d}".rstrip("0")
        return (t.strftime("%Y-%m-%d %H:%M:%S") + ("." + frac if frac else "")).encode()
    return str(int(c.values[i])).encode()


def datatype_histogram(c: "OColumn", sel: np.ndarray) -> DataTypeHistogram:
    counts = [0, 0, 0, 0, 0]  # NULL_POS, FRACTIONAL_POS, INTEGRAL_POS, BOOLEAN_POS, STRING_POS
    for i in range(len(sel)):
        counts[datatype_class(_value_string(c, i)) if sel[i] else 0] += 1
    return DataTypeHistogram(*counts)


# PatternMatch (analyzers/PatternMatch.scala:46-55): sum(CASE WHEN where THEN
# (regexp_extract(col, pattern, 0) != "" ? 1 : 0) END) / conditionalCount(where).  Spark's RegExpExtract
# runs java.util.regex Matcher.find() on the value (UTF8String -> java String) and returns group 0, or ""
# without a match.  Python's `re` is the same leftmost-first backtracking engine for the constructs
# PatternMatch patterns use; the Java defaults that differ are restated here: ASCII \d \s \w (re.ASCII),
# `.` excludes \n \r \u0085 \u2028 \u2029, a trailing `$` also matches before a final line
# terminator (but not between \r and \n), named groups are (?<name>...), \e is ESC, \x{h..} a code point.
_JAVA_DOT = "[^\n\r\x85\u2028\u2029]"
_JAVA_END = "(?:\\Z|(?=\r\n\\Z)|(?<!\r)(?=\n\\Z)|(?=[\r\x85\u2028\u2029]\\Z))"


def java_regex_to_python(p: str) -> str:
    out, i, in_class = [], 0, False
    while i < len(p):
        c = p[i]
        if c == "\\" and i + 1 < len(p):
            d = p[i + 1]
            if d == "x" and i + 2 < len(p) and p[i + 2] == "{":
                j = p.index("}", i + 3)
                out.append("\\U%08x" % int(p[i + 3:j], 16))
                i = j + 1
                continue
            if d == "e":
                out.append("\\x1b")
            elif d == "0":  # \0n, \0nn, \0mnn
                j = i + 2
                while j < len(p) and j < i + 5 and p[j] in "01234567" and int(p[i + 2:j + 1], 8) <= 0o377:
                    j += 1
                out.append("\\x%02x" % int(p[i + 2:j], 8))
                i = j
                continue
            else:
                out.append(p[i:i + 2])
            i += 2
            continue
        if in_class:
            if c == "]":
                in_class = False
            out.append(c)
        elif c == "[":
            in_class = True
            out.append(c)
            if i + 1 < len(p) and p[i + 1] == "^":
                out.append("^")
                i += 1
        elif c == ".":
            out.append(_JAVA_DOT)
        elif c == "$" and i == len(p) - 1:
            out.append(_JAVA_END)
        elif p.startswith("(?<", i) and not p.startswith(("(?<=", "(?<!"), i):
            out.append("(?P<")
            i += 3
            continue
        else:
            out.append(c)
        i += 1
    return "".join(out)


_REGEX_CACHE: dict = {}


def regexp_extract_nonempty(value: bytes, pattern: str) -> bool:
    """regexp_extract(value, pattern, 0) != "" (Spark RegExpExtract: Matcher.find(), group 0)."""
    rx = _REGEX_CACHE.get(pattern)
    if rx is None:
        rx = _REGEX_CACHE[pattern] = re.compile(java_regex_to_python(pattern), re.ASCII)
    m = rx.search(value.decode("utf-8", "replace"))  # invalid UTF-8 -> U+FFFD, as UTF8String.toString
    return m is not None and m.group(0) != ""


# Grouping analyzers: FrequencyBasedAnalyzer.computeFrequencies (GroupingAnalyzers.scala:44-82) --
# count(*) per distinct tuple of the grouping columns over rows where all of them are non-null; numRows
# = data.count().  Grouping keys follow Spark 2.2's UnsafeRow: NaN canonical (setDouble), -0.0 and 0.0
# distinct (binary comparison), strings by bytes.
def _group_key(c: "OColumn", i: int):
    if c.dtype == "f64":
        v = float(c.values[i])
        return ("f", b"nan" if math.isnan(v) else struct.pack("<d", v))
    if c.dtype == "f32":  # FloatType in an UnsafeRow: NaN canonical, -0.0 and 0.0 distinct
        v = float(c.values[i])
        return ("f", b"nan" if math.isnan(v) else struct.pack("<f", v))
    if c.dtype in ("utf8", "large_utf8"):
        return ("s", c.values[i])
    return ("i", int(c.values[i]))


def frequencies(cols: dict, columns, n: int) -> dict:
    freq: dict = {}
    for i in range(n):
        if all(cols[c].valid[i] for c in columns):
            k = tuple(_group_key(cols[c], i) for c in columns)
            freq[k] = freq.get(k, 0) + 1
    return freq


@dataclass
class GroupingMetricState:
    """FrequenciesAndNumRows + the analyzer that reads it (its aggregationFunctions)."""
    op: str
    freq: dict
    numRows: int

    def metricValue(self):
        counts = list(self.freq.values())
        unique = sum(1 for c in counts if c == 1)
        if self.op == "Uniqueness":  # Uniqueness.scala:27-29
            return unique / self.numRows
        if self.op == "Distinctness":  # Distinctness.scala:29-31
            return len(counts) / self.numRows
        if self.op == "CountDistinct":  # CountDistinct.scala:25-31
            return float(len(counts))
        if self.op == "UniqueValueRatio":  # UniqueValueRatio.scala:25-36 (NULL sum unboxes to 0.0)
            return unique / len(counts) if counts else float("nan")
        if self.op == "MutualInformation":  # MutualInformation.scala:37-66: marginals from the joint counts
            px, py = {}, {}
            for (x, y), c in self.freq.items():
                px[x] = px.get(x, 0) + c
                py[y] = py.get(y, 0) + c
            n = self.numRows
            return sum((c / n) * math.log((c / n) / ((px[x] / n) * (py[y] / n))) for (x, y), c in self.freq.items())
        if self.op == "Entropy":  # Entropy.scala:29-41
            return sum(0.0 if c == 0 else -(c / self.numRows) * math.log(c / self.numRows) for c in counts)
        raise ValueError(self.op)


def histogram(cols: dict, column: str, n: int):
    """Histogram.computeStateFrom (Histogram.scala:51-66): CAST(col AS STRING), NULL -> "NullValue",
    count per string -> {value: count}; numberOfBins = number of groups."""
    freq: dict = {}
    c = cols[column]
    for i in range(n):
        k = _value_string(c, i).decode("utf-8", "replace") if c.valid[i] else "NullValue"
        freq[k] = freq.get(k, 0) + 1
    return freq


def _where(cols, n, where: Optional[str]):
    """(where_true, where_notnull) masks; no where -> all true."""
    if where is None:
        return np.ones(n, dtype=bool), np.ones(n, dtype=bool)
    return OracleExpr(where).eval_bool(cols, n)


def _conditional_count(cols, n, where):
    """conditionalCount (Analyzer.scala:404-408): count(*) or sum(cast(where as long))."""
    if where is None:
        return n
    t, nn = _where(cols, n, where)
    if not nn.any():
        return None
    return int(t.sum())


def compute_state(spec: tuple, cols: dict, n: int, n_partitions: int = 1):
    """spec = (op, args...) mirroring the Scala case classes; returns Option[State]."""
    op = spec[0]
    if op == "Size":
        c = _conditional_count(cols, n, spec[1])
        return None if c is None else NumMatches(c)
    if op == "Completeness":
        col, where = spec[1], spec[2]
        wt, _ = _where(cols, n, where)
        count = _conditional_count(cols, n, where)
        matches = int((cols[col].valid & wt).sum())
        if count is None or (n == 0):
            return None
        return NumMatchesAndCount(matches, count)
    if op == "Compliance":
        _, pred, where = spec[1], spec[2], spec[3]
        wt, _ = _where(cols, n, where)
        pt, pn = OracleExpr(pred).eval_bool(cols, n)
        # sum(cast(CASE WHEN where THEN pred END AS INT)): NULL if no non-null term
        nonnull_terms = pn & wt
        count = _conditional_count(cols, n, where)
        if not nonnull_terms.any() or count is None:
            return None
        return NumMatchesAndCount(int((pt & wt).sum()), count)
    if op in ("Sum", "Mean", "StandardDeviation", "Minimum", "Maximum", "ApproxCountDistinct"):
        col, where = spec[1], spec[2]
        c = cols[col]
        wt, _ = _where(cols, n, where)
        sel = c.valid & wt
        if op == "Sum":
            s = spark_sum(c, sel, n_partitions)
            return None if s is None else SumState(s)
        if op == "Mean":
            s = spark_sum(c, sel, n_partitions)
            return None if s is None else MeanState(s, int(sel.sum()))
        if op == "StandardDeviation":
            nn, avg, m2 = spark_stddev_buffer(_as_double_list(c), sel, n_partitions)
            return None if nn == 0.0 else StandardDeviationState(nn, avg, m2)
        if op in ("Minimum", "Maximum"):
            v = spark_min(c, sel, is_max=(op == "Maximum"))
            if v is None:
                return None
            return MinState(v) if op == "Minimum" else MaxState(v)
        return ApproxCountDistinctState(hll_words_for(c, sel))
    if op in ("Uniqueness", "Distinctness", "CountDistinct", "UniqueValueRatio", "Entropy", "MutualInformation"):
        columns = [spec[1]] if isinstance(spec[1], str) else list(spec[1])
        st = GroupingMetricState(op, frequencies(cols, columns, n), n)
        # the SQL sum over an empty frequencies table is NULL -> EmptyStateException (metricFromEmpty)
        if not st.freq and op in ("Uniqueness", "Distinctness", "Entropy", "MutualInformation"):
            return None
        return st
    if op == "PatternMatch":
        col, pattern, where = spec[1], spec[2], spec[3]
        c = cols[col]
        wt, _ = _where(cols, n, where)
        matches = sum(1 for i in range(n)
                      if wt[i] and c.valid[i] and regexp_extract_nonempty(_value_string(c, i), pattern))
        count = _conditional_count(cols, n, where)
        # the CASE term is never NULL when `where` holds: the sum is NULL iff no row passes `where`
        if not wt.any() or count is None:
            return None
        return NumMatchesAndCount(matches, count)
    if op == "DataType":  # stateful_datatype(conditionalSelection(column, where)); never NULL
        col, where = spec[1], spec[2]
        wt, _ = _where(cols, n, where)
        return datatype_histogram(cols[col], cols[col].valid & wt)
    if op == "Correlation":
        a, b, where = spec[1], spec[2], spec[3]
        wt, _ = _where(cols, n, where)
        sel = cols[a].valid & cols[b].valid & wt
        r = spark_corr_buffer(_as_double_list(cols[a]), _as_double_list(cols[b]), sel, n_partitions)
        return None if not r[0] > 0.0 else CorrelationState(*r)
    raise ValueError(op)


def metric_value(state) -> Optional[float]:
    return None if state is None else state.metricValue()


# --------------------------------------------------------------------------------------
# HdfsStateProvider formats (StateProvider.scala:81-83, 176-294) and identifiers
# --------------------------------------------------------------------------------------


def _mix_last(h: int, k: int) -> int:
    k = (k * 0xCC9E2D51) & 0xFFFFFFFF
    k = ((k << 15) | (k >> 17)) & 0xFFFFFFFF
    k = (k * 0x1B873593) & 0xFFFFFFFF
    return h ^ k


def _mix(h: int, k: int) -> int:
    h = _mix_last(h, k)
    h = ((h << 13) | (h >> 19)) & 0xFFFFFFFF
    return (h * 5 + 0xE6546B64) & 0xFFFFFFFF


def murmur3_string_hash(s: str, seed: int = 42) -> int:
    """scala.util.hashing.MurmurHash3.stringHash (UTF-16 code units, pairs per mix)."""
    units = []
    for ch in s:
        cp = ord(ch)
        if cp >= 0x10000:
            cp -= 0x10000
            units += [0xD800 + (cp >> 10), 0xDC00 + (cp & 0x3FF)]
        else:
            units.append(cp)
    h = seed & 0xFFFFFFFF
    i = 0
    while i + 1 < len(units):
        h = _mix(h, ((units[i] << 16) + units[i + 1]) & 0xFFFFFFFF)
        i += 2
    if i < len(units):
        h = _mix_last(h, units[i])
    h ^= len(units)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return to_i32(h)


def state_to_bytes(state) -> bytes:
    """Java DataOutputStream (big-endian) images written by HdfsStateProvider.persist."""
    if isinstance(state, NumMatches):
        return struct.pack(">q", state.numMatches)
    if isinstance(state, NumMatchesAndCount):
        return struct.pack(">qq", state.numMatches, state.count)
    if isinstance(state, SumState):
        return struct.pack(">d", state.sum_)
    if isinstance(state, MeanState):
        return struct.pack(">dq", state.sum_, state.count)
    if isinstance(state, MinState):
        return struct.pack(">d", state.minValue)
    if isinstance(state, MaxState):
        return struct.pack(">d", state.maxValue)
    if isinstance(state, StandardDeviationState):
        return struct.pack(">ddd", state.n, state.avg, state.m2)
    if isinstance(state, CorrelationState):
        return struct.pack(">dddddd", state.n, state.xAvg, state.yAvg, state.ck, state.xMk, state.yMk)
    if isinstance(state, ApproxCountDistinctState):
        b = words_to_bytes(state.words)
        return struct.pack(">i", len(b)) + b
    if isinstance(state, DataTypeHistogram):  # persistBytes(DataTypeHistogram.toBytes(...))
        b = struct.pack(">qqqqq", state.numNull, state.numFractional, state.numIntegral, state.numBoolean,
                        state.numString)
        return struct.pack(">i", len(b)) + b
    raise TypeError(type(state))


# --------------------------------------------------------------------------------------
# ApproxQuantile(s): the GPU path's contract (analyzers/ApproxQuantile.scala:49-103,
# ApproxQuantiles.scala:30-105).  Spark 2.2.2's QuantileSummaries.query answers min for
# q <= relativeError, max for q >= 1 - relativeError, otherwise a value whose rank is within
# ceil(relativeError * n) of ceil(q * n); the path returns the exact order statistic of that target
# rank (NaN last as java.lang.Double.compare, -0.0 < 0.0).  Pinned by the reference's band tests
# (AnalyzerTests.scala:533-565); GK's own order-dependent pick is not restated (parity vs GK
# unpinned -- any value inside its bound is a correct ApproxQuantile).
# --------------------------------------------------------------------------------------
def gk_digest_exact(values: np.ndarray, valid: np.ndarray, relative_error: float) -> Tuple[int, List[Tuple[float, int, int]]]:
    """(count, sampled) of the quantile state the GPU path builds (deequ_amd/quantiles.py module doc): the
    exact order statistics at ranks 1, 1 + s, ..., n with s = max(1, floor(2 e n)), e = 1 / (1 / relErr)
    (StatefulApproxQuantile's accuracy round trip, DeequFunctions.scala:63-71), g = rank gaps, delta = 0."""
    v = np.asarray(values)[np.asarray(valid, bool)]
    n = len(v)
    if n == 0:
        return 0, []
    e = 0.0 if relative_error == 0.0 else 1.0 / (1.0 / relative_error)
    s = max(1, int(math.floor(2 * e * n)))
    ranks = list(range(1, n + 1, s))
    if ranks[-1] != n:
        ranks.append(n)
    vals = approx_quantiles_exact(values, valid, [(r - 0.5) / n for r in ranks], 0.0)
    out, prev = [], 0
    for r, x in zip(ranks, vals):
        out.append((x, r - prev, 0))
        prev = r
    return n, out


def approx_quantiles_exact(values: np.ndarray, valid: np.ndarray, quantiles: Sequence[float],
                           relative_error: float = 0.01) -> Optional[List[float]]:
    v = np.asarray(values)[np.asarray(valid, bool)]
    if v.dtype == np.float32:  # FloatType: the exactly widened doubles
        v = v.astype(np.float64)
    n = len(v)
    if n == 0:
        return None
    if v.dtype == np.float64:
        bits = v.view(np.uint64).copy()
        bits[np.isnan(v)] = np.uint64(0x7FF8000000000000)
        sign = (bits >> np.uint64(63)) == 1
        keys = np.where(sign, ~bits, bits | np.uint64(1 << 63))
        order = np.sort(keys)
        back = np.where((order >> np.uint64(63)) == 1, order & np.uint64(MASK64 >> 1), ~order)
        srt = back.view(np.float64)
    else:
        srt = np.sort(v.astype(np.int64)).astype(np.float64)
    out = []
    for q in quantiles:
        if q <= relative_error:
            r = 1
        elif q >= 1.0 - relative_error:
            r = n
        else:
            r = int(math.ceil(q * n))
        r = min(n, max(1, r))
        out.append(float(srt[r - 1]))
    return out
