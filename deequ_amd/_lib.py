"""ctypes binding of libdqscan.so (include/dqscan.h).

The HIP library is the product: there is no fallback.  If the shared library is missing this
module raises at import time, and every scan goes through dq_plan_create / dq_scan / dq_finish.
"""
from __future__ import annotations

import ctypes
import os

ABI_VERSION = 6  # include/dqscan.h DQ_ABI_VERSION

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DQ_LIB_PATH") or os.path.join(_HERE, "libdqscan.so")  # override: diagnostic A/B builds

DQ_OK = 0
DQ_E_INVALID = -1
DQ_E_TYPE = -2
DQ_E_UNSUPPORTED = -3
DQ_E_HIP = -4
DQ_E_OOM = -5
DQ_E_STATE = -6

TYPE_F64, TYPE_I64, TYPE_I32, TYPE_UTF8, TYPE_LARGE_UTF8 = 1, 2, 3, 4, 5
# round 6: FloatType, ShortType, ByteType, BooleanType (bit-packed), DateType (int32 days), TimestampType (int64 us)
TYPE_F32, TYPE_I16, TYPE_I8, TYPE_BOOL, TYPE_DATE32, TYPE_TIMESTAMP = 6, 7, 8, 9, 10, 11
# DecimalType(p, s): 16-byte two's-complement unscaled values; its type code carries p and s (DQ_DECIMAL128)
TYPE_DECIMAL128 = 12


def decimal_type(precision: int, scale: int) -> int:
    """DQ_DECIMAL128(p, s): the type code of a DecimalType(p, s) column (1 <= p <= 38, 0 <= s <= p)."""
    if not (1 <= precision <= 38 and 0 <= scale <= precision):
        raise ValueError(f"DecimalType({precision},{scale}) is not a GPU column type (precision 1..38, scale 0..p)")
    return TYPE_DECIMAL128 | precision << 8 | scale << 16

# column-pass kernel variants (deequ_amd/csrc/dq_device.h ColVariant)
VARIANT_NAMES = {0: "validity", 1: "f64_stats", 2: "f64_stats_hll", 3: "f64_hll", 4: "i64_stats",
                 5: "i64_stats_hll", 6: "i64_hll", 7: "i32_stats", 8: "i32_stats_hll", 9: "i32_hll",
                 10: "utf8_hll", 11: "large_utf8_hll", 12: "utf8_dtype", 13: "utf8_hll_dtype",
                 14: "large_utf8_dtype", 15: "large_utf8_hll_dtype", 16: "f64_dtype",
                 17: "f32_stats", 18: "f32_stats_hll", 19: "f32_hll", 20: "i16_stats", 21: "i16_stats_hll",
                 22: "i16_hll", 23: "i8_stats", 24: "i8_stats_hll", 25: "i8_hll", 26: "f32_dtype", 27: "bool",
                 28: "d128_stats", 29: "d128_stats_hll", 30: "d128_hll", 31: "d128_dtype"}

OP_SIZE = 1
OP_COMPLETENESS = 2
OP_COMPLIANCE = 3
OP_SUM = 4
OP_MEAN = 5
OP_STDDEV = 6
OP_MIN = 7
OP_MAX = 8
OP_CORRELATION = 9
OP_APPROX_COUNT_DISTINCT = 10
OP_DATATYPE = 11
OP_PATTERN_MATCH = 12

PRED_COLUMN = 1
PRED_LIT_INT = 2
PRED_LIT_DECIMAL = 3
PRED_LIT_DOUBLE = 4
PRED_LIT_NULL = 5
PRED_LIT_BOOL = 6
PRED_CMP = 7
PRED_AND = 8
PRED_OR = 9
PRED_NOT = 10
PRED_IS_NULL = 11
PRED_IS_NOT_NULL = 12
PRED_COALESCE = 13
PRED_REGEX = 14

REGEX_RLIKE = 0             # col RLIKE p: NULL on NULL, find()
REGEX_EXTRACT_NONEMPTY = 1  # regexp_extract(col, p, 0) != '' as PatternMatch builds it: FALSE on NULL
REGEX_FULL = 2              # whole value in L(p): string = / IN lists; NULL on NULL

CMP_LT, CMP_LE, CMP_GT, CMP_GE, CMP_EQ, CMP_NE = 1, 2, 3, 4, 5, 6


class ColumnDesc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("nullable", ctypes.c_int32)]


class AnalyzerSpec(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("col_a", ctypes.c_int32), ("col_b", ctypes.c_int32),
                ("pred_root", ctypes.c_int32), ("where_root", ctypes.c_int32)]


class PredNode(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("a", ctypes.c_int32), ("b", ctypes.c_int32),
                ("cmp", ctypes.c_int32), ("i64", ctypes.c_int64), ("f64", ctypes.c_double)]


# dq_plan_options.pred_pass (enum dq_pred_pass)
PRED_PASS = {"auto": 0, "interpreter": 1, "compiled": 2}


class PlanOptions(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_int32), ("pred_pass", ctypes.c_int32), ("reserved", ctypes.c_int32 * 6)]


class ColumnView(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("validity", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("reserved", ctypes.c_int64)]


class _Size(ctypes.Structure):
    _fields_ = [("num_matches", ctypes.c_int64)]


class _Ratio(ctypes.Structure):
    _fields_ = [("num_matches", ctypes.c_int64), ("count", ctypes.c_int64)]


class _Sum(ctypes.Structure):
    _fields_ = [("sum", ctypes.c_double), ("partial", ctypes.c_int64), ("partial_hi", ctypes.c_int64),
                ("guard", ctypes.c_double), ("dec_scale", ctypes.c_int32), ("dec_digits", ctypes.c_int32)]


class _Mean(ctypes.Structure):
    _fields_ = [("sum", ctypes.c_double), ("count", ctypes.c_int64), ("partial", ctypes.c_int64),
                ("partial_hi", ctypes.c_int64), ("guard", ctypes.c_double), ("dec_scale", ctypes.c_int32),
                ("dec_digits", ctypes.c_int32)]


class _StdDev(ctypes.Structure):
    _fields_ = [("n", ctypes.c_double), ("avg", ctypes.c_double), ("m2", ctypes.c_double)]


class _MinMax(ctypes.Structure):
    _fields_ = [("value", ctypes.c_double)]


class _Corr(ctypes.Structure):
    _fields_ = [("n", ctypes.c_double), ("x_avg", ctypes.c_double), ("y_avg", ctypes.c_double),
                ("ck", ctypes.c_double), ("x_mk", ctypes.c_double), ("y_mk", ctypes.c_double)]


class _Hll(ctypes.Structure):
    _fields_ = [("words", ctypes.c_int64 * 52)]


class _DType(ctypes.Structure):
    _fields_ = [("num_null", ctypes.c_int64), ("num_fractional", ctypes.c_int64), ("num_integral", ctypes.c_int64),
                ("num_boolean", ctypes.c_int64), ("num_string", ctypes.c_int64)]


class _StateUnion(ctypes.Union):
    _fields_ = [("size", _Size), ("ratio", _Ratio), ("sum", _Sum), ("mean", _Mean), ("stddev", _StdDev),
                ("minmax", _MinMax), ("corr", _Corr), ("hll", _Hll), ("dtype", _DType)]


class FreqSummary(ctypes.Structure):
    _fields_ = [("num_groups", ctypes.c_int64), ("num_unique", ctypes.c_int64), ("num_values", ctypes.c_int64),
                ("entropy", ctypes.c_double)]


class State(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("has_value", ctypes.c_uint8 * 2), ("integral", ctypes.c_uint8),
                ("reserved", ctypes.c_uint8), ("u", _StateUnion)]


STATE_SIZE = ctypes.sizeof(State)


class DQError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"dqscan error {status}: {message}")
        self.status = status
        self.message = message


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C deequ_amd` or __graft_entry__.build(); "
            "the MI355X scan has no CPU fallback")
    # torch first: its HIP runtime is then the one libdqscan.so binds to, so device pointers, streams and
    # the device list are shared (loaded the other way round, a second runtime instance can see no device)
    import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    c = ctypes
    P = c.POINTER
    L.dq_abi_version.restype = c.c_int32
    L.dq_last_error.restype = c.c_char_p
    L.dq_plan_create.restype = c.c_int32
    L.dq_plan_create.argtypes = [P(AnalyzerSpec), c.c_int32, P(ColumnDesc), c.c_int32, P(PredNode), c.c_int32,
                                 c.c_int32, P(c.c_void_p)]
    L.dq_plan_create_ex.restype = c.c_int32
    L.dq_plan_create_ex.argtypes = [P(AnalyzerSpec), c.c_int32, P(ColumnDesc), c.c_int32, P(PredNode), c.c_int32,
                                    P(c.c_char_p), c.c_int32, c.c_int32, P(c.c_void_p)]
    L.dq_plan_create_opts.restype = c.c_int32
    L.dq_plan_create_opts.argtypes = [P(AnalyzerSpec), c.c_int32, P(ColumnDesc), c.c_int32, P(PredNode), c.c_int32,
                                      P(c.c_char_p), c.c_int32, P(PlanOptions), c.c_int32, P(c.c_void_p)]
    L.dq_plan_explain.restype = c.c_int64
    L.dq_plan_explain.argtypes = [P(AnalyzerSpec), c.c_int32, P(ColumnDesc), c.c_int32, P(PredNode), c.c_int32,
                                  P(c.c_char_p), c.c_int32, P(PlanOptions), c.c_char_p, c.c_int64]
    L.dq_plan_create_time.restype = c.c_int32
    L.dq_plan_create_time.argtypes = [c.c_void_p, P(c.c_double), P(c.c_double)]
    L.dq_regex_info.restype = c.c_int32
    L.dq_regex_info.argtypes = [c.c_char_p, c.c_int32, P(c.c_int32), P(c.c_int32)]
    L.dq_pred_pool_create.restype = c.c_int32
    L.dq_pred_pool_create.argtypes = [P(c.c_char_p), P(c.c_int32), c.c_int32, P(c.c_void_p)]
    L.dq_pred_pool_add.restype = c.c_int32
    L.dq_pred_pool_add.argtypes = [c.c_void_p, c.c_char_p, P(c.c_int32)]
    L.dq_pred_pool_add_regex.restype = c.c_int32
    L.dq_pred_pool_add_regex.argtypes = [c.c_void_p, c.c_int32, c.c_char_p, c.c_int32, P(c.c_int32)]
    L.dq_pred_pool_size.restype = c.c_int32
    L.dq_pred_pool_size.argtypes = [c.c_void_p]
    L.dq_pred_pool_nodes.restype = P(PredNode)
    L.dq_pred_pool_nodes.argtypes = [c.c_void_p]
    L.dq_pred_pool_num_patterns.restype = c.c_int32
    L.dq_pred_pool_num_patterns.argtypes = [c.c_void_p]
    L.dq_pred_pool_patterns.restype = P(c.c_char_p)
    L.dq_pred_pool_patterns.argtypes = [c.c_void_p]
    L.dq_pred_pool_destroy.restype = None
    L.dq_pred_pool_destroy.argtypes = [c.c_void_p]
    L.dq_regex_match_host.restype = c.c_int32
    L.dq_regex_match_host.argtypes = [c.c_char_p, c.c_int32, c.c_void_p, c.c_void_p, c.c_int64, c.c_void_p]
    L.dq_freq_build.restype = c.c_int32
    L.dq_freq_build.argtypes = [P(c.c_int32), c.c_int32, P(ColumnView), P(c.c_int64), c.c_int32, c.c_int32,
                                c.c_void_p, P(c.c_void_p)]
    L.dq_freq_merge.restype = c.c_int32
    L.dq_freq_merge.argtypes = [c.c_void_p, c.c_void_p, P(c.c_void_p)]
    L.dq_freq_summarize.restype = c.c_int32
    L.dq_freq_summarize.argtypes = [c.c_void_p, c.c_int64, P(FreqSummary)]
    L.dq_freq_num_groups.restype = c.c_int64
    L.dq_freq_num_groups.argtypes = [c.c_void_p]
    L.dq_freq_export.restype = c.c_int32
    L.dq_freq_export.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_int64]
    L.dq_mutual_information.restype = c.c_int32
    L.dq_mutual_information.argtypes = [P(c.c_int32), P(ColumnView), P(c.c_int64), c.c_int32, c.c_int64, c.c_int32,
                                        c.c_void_p, P(c.c_double), P(c.c_int32)]
    L.dq_approx_quantiles.restype = c.c_int32
    L.dq_approx_quantiles.argtypes = [c.c_int32, P(ColumnView), P(c.c_int64), c.c_int32, P(c.c_double), c.c_int32,
                                      c.c_double, c.c_int32, c.c_void_p, P(c.c_double), P(c.c_int64)]
    L.dq_quantile_digest.restype = c.c_int32
    L.dq_quantile_digest.argtypes = [c.c_int32, P(ColumnView), P(c.c_int64), c.c_int32, c.c_double, c.c_int32,
                                     c.c_void_p, P(c.c_double), P(c.c_int64), c.c_int64, P(c.c_int64), P(c.c_int64)]
    L.dq_freq_top.restype = c.c_int32
    L.dq_freq_top.argtypes = [c.c_void_p, c.c_int32, P(c.c_uint64), P(c.c_int64), P(c.c_uint64), P(c.c_int32)]
    L.dq_freq_destroy.restype = None
    L.dq_freq_destroy.argtypes = [c.c_void_p]
    L.dq_plan_set_stream.restype = c.c_int32
    L.dq_plan_set_stream.argtypes = [c.c_void_p, c.c_void_p]
    L.dq_scan.restype = c.c_int32
    L.dq_scan.argtypes = [c.c_void_p, P(ColumnView), c.c_int64, c.c_int64]
    L.dq_finish.restype = c.c_int32
    L.dq_finish.argtypes = [c.c_void_p, P(State)]
    L.dq_plan_reset.restype = c.c_int32
    L.dq_plan_reset.argtypes = [c.c_void_p]
    L.dq_plan_destroy.restype = None
    L.dq_plan_destroy.argtypes = [c.c_void_p]
    L.dq_plan_bytes_per_row_x1000.restype = c.c_int64
    L.dq_plan_bytes_per_row_x1000.argtypes = [c.c_void_p]
    L.dq_plan_num_launches.restype = c.c_int32
    L.dq_plan_num_launches.argtypes = [c.c_void_p]
    L.dq_plan_enable_timing.restype = c.c_int32
    L.dq_plan_enable_timing.argtypes = [c.c_void_p, c.c_int32]
    L.dq_plan_kernel_time.restype = c.c_int32
    L.dq_plan_kernel_time.argtypes = [c.c_void_p, c.c_int32, P(c.c_double), P(c.c_int64)]
    L.dq_plan_variant_bytes_per_row_x1000.restype = c.c_int64
    L.dq_plan_variant_bytes_per_row_x1000.argtypes = [c.c_void_p, c.c_int32]
    L.dq_plan_kernel_bytes_per_row_x1000.restype = c.c_int64
    L.dq_plan_kernel_bytes_per_row_x1000.argtypes = [c.c_void_p, c.c_int32]
    L.dq_plan_pred_compiled.restype = c.c_int32
    L.dq_plan_pred_compiled.argtypes = [c.c_void_p, c.c_char_p, c.c_int32]
    L.dq_plan_pred_wait.restype = c.c_int32
    L.dq_plan_pred_wait.argtypes = [c.c_void_p, c.c_int32]
    L.dq_state_merge.restype = c.c_int32
    L.dq_state_merge.argtypes = [P(State), P(State), P(State)]
    L.dq_state_combine.restype = c.c_int32
    L.dq_state_combine.argtypes = [P(State), P(State), P(State)]
    for fn in ("dq_state_merge_n", "dq_state_combine_n"):
        getattr(L, fn).restype = c.c_int32
        getattr(L, fn).argtypes = [P(State), P(State), c.c_int32, P(State)]
    L.dq_state_is_defined.restype = c.c_int32
    L.dq_state_is_defined.argtypes = [P(State)]
    L.dq_state_metric.restype = c.c_int32
    L.dq_state_metric.argtypes = [P(State), P(c.c_double)]
    L.dq_hll_estimate.restype = c.c_int32
    L.dq_hll_estimate.argtypes = [P(c.c_int64), P(c.c_double)]
    L.dq_state_to_bytes.restype = c.c_int64
    L.dq_state_to_bytes.argtypes = [P(State), c.c_void_p, c.c_int64]
    L.dq_state_from_bytes.restype = c.c_int32
    L.dq_state_from_bytes.argtypes = [c.c_int32, c.c_char_p, c.c_int64, P(State)]
    L.dq_state_identifier.restype = c.c_int32
    L.dq_state_identifier.argtypes = [c.c_char_p]
    if L.dq_abi_version() != ABI_VERSION:
        raise ImportError(f"libdqscan ABI {L.dq_abi_version()} != {ABI_VERSION}")
    return L


lib = _load()

# every symbol include/dqscan.h declares (checked by tests/test_boundary.py)
EXPORTED = [
    "dq_abi_version", "dq_last_error", "dq_plan_create", "dq_plan_create_ex", "dq_plan_create_opts",
    "dq_plan_create_time", "dq_plan_explain", "dq_regex_info", "dq_regex_match_host",
    "dq_pred_pool_create", "dq_pred_pool_add", "dq_pred_pool_add_regex", "dq_pred_pool_size", "dq_pred_pool_nodes",
    "dq_pred_pool_num_patterns", "dq_pred_pool_patterns", "dq_pred_pool_destroy",
    "dq_arrow_import", "dq_uploader_create", "dq_upload", "dq_upload_fence", "dq_upload_release", "dq_upload_sync",
    "dq_uploader_destroy",
    "dq_plan_set_stream", "dq_freq_build", "dq_freq_merge", "dq_freq_summarize", "dq_freq_num_groups",
    "dq_freq_export", "dq_freq_destroy", "dq_mutual_information", "dq_approx_quantiles", "dq_quantile_digest", "dq_freq_top", "dq_scan", "dq_finish",
    "dq_plan_reset", "dq_plan_destroy", "dq_plan_bytes_per_row_x1000", "dq_plan_num_launches",
    "dq_plan_enable_timing", "dq_plan_kernel_time", "dq_plan_variant_bytes_per_row_x1000",
    "dq_plan_kernel_bytes_per_row_x1000", "dq_plan_pred_compiled", "dq_plan_pred_wait",
    "dq_state_merge", "dq_state_combine", "dq_state_merge_n", "dq_state_combine_n", "dq_state_is_defined", "dq_state_metric", "dq_hll_estimate",
    "dq_state_to_bytes", "dq_state_from_bytes", "dq_state_identifier",
]


def check(status: int) -> None:
    if status != DQ_OK:
        raise DQError(status, lib.dq_last_error().decode("utf-8", "replace"))
