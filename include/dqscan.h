/*
 * dqscan.h -- C ABI of libdqscan.so, the MI355X (gfx950) replacement for Deequ's fused
 * single-pass metric scan.
 *
 * Reference interface this replaces (paths relative to src/main/scala/com/amazon/deequ/):
 *   AnalysisRunner.runScanningAnalyzers            analyzers/runners/AnalysisRunner.scala:279-326
 *     -> data.agg(aggregations...).collect().head   analyzers/runners/AnalysisRunner.scala:303
 *   ScanShareableAnalyzer.aggregationFunctions /
 *     fromAggregationResult(row, offset)           analyzers/Analyzer.scala:159-187
 *   State.sum / Analyzers.merge                    analyzers/Analyzer.scala:34-48, 343-362
 *   DeequHyperLogLogPlusPlusUtils.count            analyzers/catalyst/StatefulHyperloglogPlus.scala:210-257
 *   HdfsStateProvider persist / load byte images   analyzers/StateProvider.scala:176-294
 *
 * Call pattern of a drop-in shim (Scala/JNI, C++, or the Python host in deequ_amd/):
 *   dq_plan_create(specs, schema, predicate IR)    <- the GPU-eligible ScanShareableAnalyzers
 *   dq_scan(plan, columns, n_rows, chunk) ...      <- one or more row chunks, HBM-resident buffers
 *   dq_finish(plan, states)                        <- one aggregation "Row" slot set per spec
 *   dq_state_* / dq_hll_estimate                   <- state algebra for StateLoader/Persister merges
 *
 * All functions return DQ_OK (0) or a negative dq_status; dq_last_error() (thread-local) holds the
 * message.  A shim maps ANY failure of plan/scan/finish to a failure metric on every GPU-routed
 * analyzer, as runScanningAnalyzers does for an aggregation exception (AnalysisRunner.scala:310-313).
 * Plans are not thread-safe: one plan per calling thread.  State functions are pure and reentrant.
 */
#ifndef DQSCAN_H
#define DQSCAN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DQ_ABI_VERSION 6  /* 2: dq_state.reserved[0] = integral flag + Sum / Mean int64 partials; ingestion, pool and state-array entry points;
                             3: dq_plan_create_opts (predicate-pass mode), dq_plan_create_time, dq_plan_explain, dq_quantile_digest;
                             4: any number of analyzers / columns per plan (split into fused plans over the
                                per-plan capacities), AUTO compiles the predicate kernel in the background,
                                dq_plan_pred_wait;
                             5: column types F32 / I16 / I8 / BOOL / DATE32 / TIMESTAMP (scan, predicates, Arrow import);
                             6: DECIMAL128 (type codes carry precision / scale, dq_state Sum / Mean decimal partials) */

typedef int32_t dq_status;
#define DQ_OK 0
#define DQ_E_INVALID (-1)     /* bad argument / malformed spec */
#define DQ_E_TYPE (-2)        /* column type not valid for the analyzer (preconditions) */
#define DQ_E_UNSUPPORTED (-3) /* predicate outside the GPU grammar: route to the fallback */
#define DQ_E_HIP (-4)         /* HIP runtime / kernel failure */
#define DQ_E_OOM (-5)         /* device allocation failed */
#define DQ_E_STATE (-6)       /* state algebra misuse (op mismatch, bad byte image) */

/* Column physical types (Arrow layouts) and the Spark SQL types they carry.  The numeric types are the ones
 * Preconditions.isNumeric accepts (analyzers/Analyzer.scala:322-334): F64 / F32 / I64 / I32 / I16 / I8 /
 * DECIMAL128.  Values are converted to double as Spark casts them (exactly, or for a decimal correctly rounded:
 * Decimal.toDouble; Sum of an integral type is Spark's wrapping LongType sum, of a decimal the exact decimal sum
 * cast at the end); ApproxCountDistinct hashes each type as Spark 2.2's XxHash64Function does: hashLong for
 * LongType / TimestampType / DoubleType (doubleToLongBits) / DecimalType of precision <= 18 (the unscaled long),
 * hashInt for IntegerType / ShortType / ByteType / DateType (the value widened to int), FloatType
 * (floatToIntBits) and BooleanType (1 / 0), hashUnsafeBytes of BigInteger.toByteArray for a wider DecimalType.
 * BOOL / DATE32 / TIMESTAMP are not numeric: Completeness, Size, ApproxCountDistinct, DataType and IS [NOT] NULL
 * atoms (BOOL also = / != against TRUE / FALSE).  A DECIMAL128 type code carries its precision (1..38) and scale
 * (0..precision): DQ_DECIMAL128(p, s); every other code is its enum value alone. */
enum dq_type {
  DQ_TYPE_F64 = 1,        /* DoubleType: 8-byte values */
  DQ_TYPE_I64 = 2,        /* LongType: 8-byte values */
  DQ_TYPE_I32 = 3,        /* IntegerType: 4-byte values */
  DQ_TYPE_UTF8 = 4,       /* StringType: int32 offsets[n+1] + data bytes */
  DQ_TYPE_LARGE_UTF8 = 5, /* StringType with int64 offsets[n+1] (chunks > 2 GiB) */
  DQ_TYPE_F32 = 6,        /* FloatType: 4-byte values */
  DQ_TYPE_I16 = 7,        /* ShortType: 2-byte values */
  DQ_TYPE_I8 = 8,         /* ByteType: 1-byte values */
  DQ_TYPE_BOOL = 9,       /* BooleanType: LSB-first bit-packed values (Arrow `b`), bit 0 = row 0 of the chunk */
  DQ_TYPE_DATE32 = 10,    /* DateType: int32 days since 1970-01-01 (Arrow `tdD`) */
  DQ_TYPE_TIMESTAMP = 11, /* TimestampType: int64 microseconds since the epoch (Arrow `tsu:<timezone>`) */
  DQ_TYPE_DECIMAL128 = 12 /* DecimalType(p, s): 16-byte little-endian two's-complement unscaled values (Arrow
                             `d:p,s` / `d:p,s,128`); use the code DQ_DECIMAL128(p, s) */
};
#define DQ_TYPE_MAX 12
#define DQ_DECIMAL128(p, s) (DQ_TYPE_DECIMAL128 | ((p) << 8) | ((s) << 16))
#define DQ_TYPE_BASE(t) ((t) & 0xFF)
#define DQ_DECIMAL_PRECISION(t) (((t) >> 8) & 0xFF)
#define DQ_DECIMAL_SCALE(t) (((t) >> 16) & 0xFF)

/* Analyzer ops: the GPU-eligible ScanShareableAnalyzers. */
enum dq_op {
  DQ_OP_SIZE = 1,                 /* analyzers/Size.scala:36-48 */
  DQ_OP_COMPLETENESS = 2,         /* analyzers/Completeness.scala:26-46 */
  DQ_OP_COMPLIANCE = 3,           /* analyzers/Compliance.scala:37-53 */
  DQ_OP_SUM = 4,                  /* analyzers/Sum.scala:36-52 */
  DQ_OP_MEAN = 5,                 /* analyzers/Mean.scala:36-54 */
  DQ_OP_STDDEV = 6,               /* analyzers/StandardDeviation.scala:47-73 */
  DQ_OP_MIN = 7,                  /* analyzers/Minimum.scala:36-53 */
  DQ_OP_MAX = 8,                  /* analyzers/Maximum.scala:36-53 */
  DQ_OP_CORRELATION = 9,          /* analyzers/Correlation.scala:65-105 */
  DQ_OP_APPROX_COUNT_DISTINCT = 10,/* analyzers/ApproxCountDistinct.scala:47-64 */
  DQ_OP_DATATYPE = 11,            /* analyzers/DataType.scala:152-183, catalyst/StatefulDataType.scala:26-83 */
  DQ_OP_PATTERN_MATCH = 12        /* analyzers/PatternMatch.scala:37-56: pred_root = a DQ_PRED_REGEX node
                                     (mode DQ_REGEX_EXTRACT_NONEMPTY); state NumMatchesAndCount */
};

typedef struct dq_column_desc {
  int32_t type;     /* enum dq_type */
  int32_t nullable; /* 0: validity bitmaps are ignored (may be NULL) */
} dq_column_desc;

/* One analyzer instance (a Scala case class).  Unused fields = -1. */
typedef struct dq_analyzer_spec {
  int32_t op;         /* enum dq_op */
  int32_t col_a;      /* column index (COMPLETENESS..MAX, ACD, DATATYPE, CORRELATION first column) */
  int32_t col_b;      /* CORRELATION second column */
  int32_t pred_root;  /* COMPLIANCE predicate: root index into the predicate node pool */
  int32_t where_root; /* optional `where` filter root, -1 = none */
} dq_analyzer_spec;

/* Predicate IR: a pool of nodes, referenced by index.  This is the lowered form of the Spark SQL
 * expressions deequ builds with expr(...) (Check.scala:538-548, 670-871): comparisons with SQL
 * three-valued logic, AND / OR / NOT, IS [NOT] NULL, COALESCE(column, literal).  Literal typing
 * follows Spark 2.2: `3` -> LIT_INT, `3.0` -> LIT_DECIMAL (exact), `3e0` -> LIT_DOUBLE. */
enum dq_pred_kind {
  DQ_PRED_COLUMN = 1,      /* a = column index */
  DQ_PRED_LIT_INT = 2,     /* i64 */
  DQ_PRED_LIT_DECIMAL = 3, /* i64 = unscaled value, cmp = scale (value = i64 / 10^scale) */
  DQ_PRED_LIT_DOUBLE = 4,  /* f64 */
  DQ_PRED_LIT_NULL = 5,
  DQ_PRED_LIT_BOOL = 6,    /* i64 = 0 / 1 */
  DQ_PRED_CMP = 7,         /* a CMP b, cmp = enum dq_cmp */
  DQ_PRED_AND = 8,         /* a AND b */
  DQ_PRED_OR = 9,          /* a OR b */
  DQ_PRED_NOT = 10,        /* NOT a */
  DQ_PRED_IS_NULL = 11,    /* a IS NULL */
  DQ_PRED_IS_NOT_NULL = 12,/* a IS NOT NULL */
  DQ_PRED_COALESCE = 13,   /* COALESCE(a, b): a = COLUMN node, b = literal node */
  DQ_PRED_REGEX = 14       /* regex over a UTF8 column: a = COLUMN node, i64 = index into the plan's
                              patterns (dq_plan_create_ex), cmp = enum dq_regex_mode;
                              string equality / IN lists lower to mode DQ_REGEX_FULL */
};
/* DQ_PRED_REGEX semantics (java.util.regex Matcher.find on the value's code points):
 *   DQ_REGEX_RLIKE            `col RLIKE p`: NULL on a NULL value, else TRUE iff find() succeeds;
 *   DQ_REGEX_EXTRACT_NONEMPTY `CASE WHEN regexp_extract(col, p, 0) != '' THEN 1 ELSE 0` as PatternMatch
 *                             builds it (PatternMatch.scala:48-49): FALSE on NULL, never NULL; patterns
 *                             that can match the empty string are DQ_E_UNSUPPORTED (fallback). */
enum dq_regex_mode { DQ_REGEX_RLIKE = 0, DQ_REGEX_EXTRACT_NONEMPTY = 1, DQ_REGEX_FULL = 2 };
/*   DQ_REGEX_FULL             the whole value is in L(p) (no search, no `^` / `$` handling): string
 *                             equality `col = 'v'` / `col IN ('a', 'b')` lowered to p = (?:a|b) with
 *                             escaped literals; NULL on a NULL value. */
enum dq_cmp { DQ_CMP_LT = 1, DQ_CMP_LE = 2, DQ_CMP_GT = 3, DQ_CMP_GE = 4, DQ_CMP_EQ = 5, DQ_CMP_NE = 6 };

typedef struct dq_pred_node {
  int32_t kind;
  int32_t a;
  int32_t b;
  int32_t cmp;
  int64_t i64;
  double f64;
} dq_pred_node;

/* One column of one row chunk.  All pointers are DEVICE pointers (HBM-resident, e.g. uploaded
 * Spark/Arrow batches).  values: 16-byte aligned; validity: Arrow LSB-first bitmap, 4-byte
 * aligned, bit 0 = row 0 of the chunk, NULL when the column has no nulls.  UTF8 columns pass the
 * data bytes in `values` and the offsets (n_rows + 1 entries) in `offsets`. */
typedef struct dq_column_view {
  const void* values;
  const uint8_t* validity;
  const void* offsets;
  int64_t reserved; /* must be 0 */
} dq_column_view;

/* ---- Host ingestion: Arrow C Data Interface batches -> device chunks (no JVM in the data path) ----
 * The Arrow C Data Interface ABI (arrow.apache.org/docs/format/CDataInterface.html), as exported by
 * Spark's Arrow conversion, pyarrow (Array._export_to_c), arrow-rs / arrow-cpp. */
#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
#define ARROW_FLAG_DICTIONARY_ORDERED 1
#define ARROW_FLAG_NULLABLE 2
#define ARROW_FLAG_MAP_KEYS_SORTED 4
struct ArrowSchema {
  const char* format;
  const char* name;
  const char* metadata;
  int64_t flags;
  int64_t n_children;
  struct ArrowSchema** children;
  struct ArrowSchema* dictionary;
  void (*release)(struct ArrowSchema*);
  void* private_data;
};
struct ArrowArray {
  int64_t length;
  int64_t null_count;
  int64_t offset;
  int64_t n_buffers;
  int64_t n_children;
  const void** buffers;
  struct ArrowArray** children;
  struct ArrowArray* dictionary;
  void (*release)(struct ArrowArray*);
  void* private_data;
};
#endif /* ARROW_C_DATA_INTERFACE */

/* One column's HOST buffers (what dq_arrow_import finds in an ArrowArray; the caller keeps the Arrow
 * array alive until dq_upload returns).  Byte counts are the bytes dq_upload writes to the device. */
typedef struct dq_host_column {
  int32_t type;            /* enum dq_type */
  int32_t nullable;        /* 1 iff validity != NULL */
  int64_t n_rows;
  const void* values;      /* fixed-width values / UTF8 data bytes (from the first string's first byte) */
  const uint8_t* validity; /* LSB-first bitmap: row 0 is bit validity_bit of byte 0; NULL = no nulls */
  const void* offsets;     /* UTF8: n_rows + 1 offsets; offsets[0] == offset_base */
  int64_t value_bytes, validity_bytes, offset_bytes;
  int64_t offset_base;     /* subtracted from every offset by dq_upload (an Arrow slice's first offset) */
  int32_t validity_bit;    /* 0..7: dq_upload shifts the bitmap so that row 0 lands on bit 0 */
  int32_t reserved;
} dq_host_column;
/* Map an exported Arrow array (formats g = float64, f = float32, l = int64, i = int32, s = int16, c = int8,
 * b = boolean, tdD = date32, tsu:<tz> = timestamp[us], d:p,s[,128] = decimal128 (precision <= 38, scale 0..p),
 * u = utf8, U = large_utf8) to host column buffers; slices
 * at any row offset are rebased by dq_upload (a boolean slice's value bits are shifted like its validity:
 * validity_bit holds the slice's bit offset of both bitmaps).  DQ_E_UNSUPPORTED: other
 * types, nested / dictionary arrays.  DQ_E_INVALID: a required buffer is NULL (an empty array may
 * export NULL buffers: it maps to an empty column). */
dq_status dq_arrow_import(const struct ArrowSchema* schema, const struct ArrowArray* array, dq_host_column* out);
/* Pinned, n-buffered host -> device upload.  dq_upload copies one chunk's columns (CPU threads: host ->
 * pinned slot; DMA on the uploader's own stream: pinned -> device slot) and returns device views of the
 * slot, valid until the slot is reused n_slots uploads later.  Before scanning, make the scan stream wait
 * for the copy (dq_upload_fence); after enqueueing the scan, record the slot's release on that stream
 * (dq_upload_release) -- the DMA of a later chunk into the same slot waits for it.  So with n_slots = 2 the
 * upload of chunk k + 1 overlaps the scan of chunk k.  host_threads <= 0: up to 16 CPU threads. */
typedef struct dq_uploader dq_uploader;
dq_status dq_uploader_create(int32_t device, int32_t n_slots, int64_t slot_bytes, int32_t host_threads,
                             dq_uploader** out);
dq_status dq_upload(dq_uploader* u, const dq_host_column* cols, int32_t n_cols, dq_column_view* dev_views);
dq_status dq_upload_fence(dq_uploader* u, void* hip_stream);
dq_status dq_upload_release(dq_uploader* u, void* hip_stream);
dq_status dq_upload_sync(dq_uploader* u);
void dq_uploader_destroy(dq_uploader* u);

/* The aggregation-result slots of one analyzer (the reference's Row slice at its offset,
 * SURVEY §8b).  has_value[i] = SQL non-null flag of slot i; single-slot analyzers mirror slot 0
 * into has_value[1].  fromAggregationResult yields Some(state) iff both flags are 1 (and, for
 * StandardDeviation / Correlation, n > 0). */
typedef struct dq_state {
  int32_t op;           /* enum dq_op */
  uint8_t has_value[2];
  uint8_t integral;     /* SUM / MEAN of an integral column (1): `partial` holds Spark's int64 partial-aggregate
                           sum (wraps like Spark's LongType sum); dq_state_combine adds the partials and
                           casts, so row shards combine exactly as Spark's partial -> final merge.  Of a
                           DECIMAL128 column (2): `partial` / `partial_hi` hold the exact decimal sum (128-bit,
                           unscaled at scale `dec_scale`), `guard` the fp64 sum of the values (it tells a sum
                           past 2^127 from its wrapped image); an unscaled sum of 10^dec_digits or more (Spark
                           2.2's sum type DecimalType(min(38, p + 10), s) overflows: a NULL sum) makes the state
                           undefined */
  uint8_t reserved;
  union {
    struct { int64_t num_matches; } size;                     /* NumMatches */
    struct { int64_t num_matches; int64_t count; } ratio;     /* NumMatchesAndCount (Completeness, Compliance, PatternMatch) */
    struct { double sum; int64_t partial; int64_t partial_hi; double guard; int32_t dec_scale, dec_digits; } sum;
    /* SumState (+ integral / decimal partial) */
    struct { double sum; int64_t count; int64_t partial; int64_t partial_hi; double guard; int32_t dec_scale, dec_digits; } mean;
    /* MeanState (+ partial) */
    struct { double n, avg, m2; } stddev;                     /* StandardDeviationState */
    struct { double value; } minmax;                          /* MinState / MaxState */
    struct { double n, x_avg, y_avg, ck, x_mk, y_mk; } corr;  /* CorrelationState */
    struct { int64_t words[52]; } hll;                        /* ApproxCountDistinctState */
    struct { int64_t num_null, num_fractional, num_integral, num_boolean, num_string; } dtype;  /* DataTypeHistogram */
  } u;
} dq_state;

typedef struct dq_plan dq_plan;

/* Library identity. */
int32_t dq_abi_version(void);
const char* dq_last_error(void);

/* Plan: validate + dedup the analyzers, lower predicates, allocate device partial states. */
dq_status dq_plan_create(const dq_analyzer_spec* specs, int32_t n_specs, const dq_column_desc* schema,
                         int32_t n_cols, const dq_pred_node* pred_pool, int32_t n_pred, int32_t device,
                         dq_plan** out);
/* As dq_plan_create, plus the UTF-8 regex patterns DQ_PRED_REGEX nodes refer to (i64 = index).
 * Each pattern is compiled on the host into a byte-level search DFA (java.util.regex subset:
 * literals, `.`, classes, \d \s \w, groups, alternation, greedy / lazy quantifiers, leading `^`,
 * trailing `$`); backreferences, look-around, \b and inline flags are DQ_E_UNSUPPORTED. */
dq_status dq_plan_create_ex(const dq_analyzer_spec* specs, int32_t n_specs, const dq_column_desc* schema,
                            int32_t n_cols, const dq_pred_node* pred_pool, int32_t n_pred,
                            const char* const* patterns, int32_t n_patterns, int32_t device, dq_plan** out);
/* How the predicate pass of a plan runs (dq_plan_options.pred_pass).  AUTO: the kernel generated and
 * compiled for the plan's program when the generator takes it (numeric comparisons; Spark's whole-stage
 * code generation of the same expressions), else -- or when the compile fails -- the interpreter, with
 * the reason in dq_plan_pred_compiled's note.  A kernel not yet in the process's cache is obtained (from the
 * disk code-object cache, else compiled by hipRTC) on a background thread: plan creation does not wait for
 * it, the scan runs the interpreter until the kernel is ready and the compiled kernel from the next chunk on
 * (bit-identical results either way; dq_plan_pred_wait blocks for it).  INTERPRETER: always the interpreter (the reference
 * implementation the compiled kernel is tested against).  COMPILED: the compiled kernel (plan creation
 * waits for the compile) or DQ_E_UNSUPPORTED from dq_plan_create_opts (reason in dq_last_error) -- no
 * silent fallback. */
enum dq_pred_pass { DQ_PRED_PASS_AUTO = 0, DQ_PRED_PASS_INTERPRETER = 1, DQ_PRED_PASS_COMPILED = 2 };
typedef struct dq_plan_options {
  int32_t struct_size;  /* sizeof(dq_plan_options) as the caller was compiled (fields past it: defaults) */
  int32_t pred_pass;    /* enum dq_pred_pass */
  int32_t reserved[6];  /* 0 */
} dq_plan_options;
/* As dq_plan_create_ex with options (NULL = all defaults).  Replaces AnalysisRunner.runScanningAnalyzers'
 * plan step (AnalysisRunner.scala:279-326): one plan per run, created before the first chunk.
 * Like the reference's single data.agg (AnalysisRunner.scala:293-303) a plan takes any number of analyzers.
 * One fused pass holds at most 64 columns, 32 distinct predicates (Compliance predicates, `where` filters,
 * Completeness-with-`where` NOT NULL tests), 32 predicate counters, 8 distinct `where` filters of value
 * analyzers (Sum ... ApproxCountDistinct, Correlation), 256 column tasks and a 96-instruction predicate
 * program; a larger set is split -- analyzers grouped by their columns -- into several fused passes over
 * the same chunks, each reading only its own columns (dq_plan_explain shows the split).  Only a spec that
 * exceeds a limit by itself (e.g. a predicate over more than 64 columns or nested deeper than the
 * 16-entry operand stack) fails, with DQ_E_UNSUPPORTED: route it to the fallback set. */
dq_status dq_plan_create_opts(const dq_analyzer_spec* specs, int32_t n_specs, const dq_column_desc* schema,
                              int32_t n_cols, const dq_pred_node* pred_pool, int32_t n_pred,
                              const char* const* patterns, int32_t n_patterns, const dq_plan_options* opts,
                              int32_t device, dq_plan** out);
/* Compile a pattern without a GPU: DFA size (or the DQ_E_UNSUPPORTED reason in dq_last_error), and
 * the host walk of the same DFA over n values (UTF-8 bytes data[offsets[r] .. offsets[r + 1]))
 * for tests of the compiler; out[r] = 1 iff the value matches under `mode` (NULLs are the caller's). */
dq_status dq_regex_info(const char* pattern, int32_t mode, int32_t* n_states, int32_t* n_classes);
dq_status dq_regex_match_host(const char* pattern, int32_t mode, const uint8_t* data, const int64_t* offsets,
                              int64_t n, uint8_t* out);
/* Predicate compiler: Spark SQL predicate text -> the IR above, on the host (replaces Spark's expr(...)
 * parse of the strings deequ builds: Analyzer.scala:385-408 `where`, Check.scala:538-548, 670-871).
 * A pool holds the table's columns (name, enum dq_type; node column indices are positions in that list)
 * and accumulates the nodes and regex patterns of every root of one plan, ready for dq_plan_create_ex.
 * Grammar: OR / AND / NOT, comparisons < <= > >= = == != <>, IS [NOT] NULL, COALESCE(a, b), parentheses,
 * numeric literals typed as Spark 2.2 (`3` int, `3.0` exact decimal, `3e0` double), NULL / TRUE / FALSE,
 * string (in)equality and [NOT] IN ('a', ...) on a string column (lowered to a DQ_REGEX_FULL node).
 * dq_pred_pool_add: DQ_E_UNSUPPORTED (reason in dq_last_error) for text outside that grammar -- string
 * ordering, a numeric comparison of a string column, LIKE / RLIKE / BETWEEN, function calls, typed literal
 * suffixes, escapes -- i.e. route the analyzer to the Spark fallback; DQ_E_INVALID "no such column: x" for
 * an unknown column.  A failed add leaves the pool unchanged.  dq_pred_pool_add_regex appends a
 * DQ_PRED_REGEX root over `column` (PatternMatch; DQ_E_UNSUPPORTED outside the DFA subset).  Node and
 * pattern arrays stay valid until the next add or destroy. */
typedef struct dq_pred_pool dq_pred_pool;
dq_status dq_pred_pool_create(const char* const* names, const int32_t* types, int32_t n_cols, dq_pred_pool** out);
dq_status dq_pred_pool_add(dq_pred_pool* pool, const char* sql, int32_t* root);
dq_status dq_pred_pool_add_regex(dq_pred_pool* pool, int32_t column, const char* pattern, int32_t mode, int32_t* root);
int32_t dq_pred_pool_size(const dq_pred_pool* pool);
const dq_pred_node* dq_pred_pool_nodes(const dq_pred_pool* pool);
int32_t dq_pred_pool_num_patterns(const dq_pred_pool* pool);
const char* const* dq_pred_pool_patterns(const dq_pred_pool* pool);
void dq_pred_pool_destroy(dq_pred_pool* pool);
/* Launch on this hipStream_t from now on (NULL = the device null stream).  A new plan launches on its
   own non-blocking stream, which does not order against other streams: set the producer's stream. */
dq_status dq_plan_set_stream(dq_plan* plan, void* hip_stream);
/* Scan one chunk of rows (asynchronous on the plan's stream).  chunk_index must increase by one
 * per call starting at 0: chunk results are merged in that order, so results are deterministic. */
dq_status dq_scan(dq_plan* plan, const dq_column_view* cols, int64_t n_rows, int64_t chunk_index);
/* Synchronise and write one dq_state per spec (caller-allocated, n_specs entries).  The plan's device
 * accumulators come back through a small pinned host buffer the plan allocates on its first finish
 * (hipHostMalloc; freed by dq_plan_destroy). */
dq_status dq_finish(dq_plan* plan, dq_state* out_states);
/* Forget all scanned chunks (keeps allocations). */
dq_status dq_plan_reset(dq_plan* plan);
void dq_plan_destroy(dq_plan* plan);
/* Algorithmic HBM bytes one scan of n_rows reads (each needed buffer counted once; UTF8 data
 * bytes are data-dependent and reported by the caller). */
int64_t dq_plan_bytes_per_row_x1000(const dq_plan* plan);
/* Number of kernel launches one dq_scan issues. */
int32_t dq_plan_num_launches(const dq_plan* plan);
/* Optional per-kernel timing (hipEvents recorded on the launch stream around every launch).
 * kernel: 0 = predicate pass, 1 = all column-pass launches, 2 = pair (correlation) pass,
 * 3 = finalize, 16 + v = column-pass launches of variant v (see deequ_amd/csrc/dq_device.h).
 * dq_plan_kernel_time synchronises, then returns the summed duration and launch count since
 * timing was (re-)enabled. */
dq_status dq_plan_enable_timing(dq_plan* plan, int32_t on);
dq_status dq_plan_kernel_time(dq_plan* plan, int32_t kernel, double* total_ms, int64_t* launches);
/* Algorithmic bytes per row (x1000) the column-pass launch of variant v reads (excl. UTF8 data). */
int64_t dq_plan_variant_bytes_per_row_x1000(const dq_plan* plan, int32_t variant);
/* The same per timing kernel id (0 = predicate pass: its atoms' columns, 2 = pair pass: its columns,
 * 16 + v = variant v); UTF8 data bytes excluded. */
int64_t dq_plan_kernel_bytes_per_row_x1000(const dq_plan* plan, int32_t kernel);
/* 1 when the plan's predicate pass runs as a kernel compiled for its program (the Compliance / where
 * programs of numeric comparisons: whole-stage code generation as Spark does for the same expressions,
 * hipRTC for the device's gfx950 target), 0 when the interpreter runs it (or the plan has no predicates);
 * note (optional, cap bytes incl. the terminator) receives the reason the interpreter runs, or -- when
 * compiled -- where the code object came from ("hiprtc", "disk cache", "process cache"). */
int32_t dq_plan_pred_compiled(const dq_plan* plan, char* note, int32_t cap);
/* Wait up to timeout_ms (< 0: until done) for a background compile of the plan's predicate kernel (AUTO);
 * then 1 when the next dq_scan runs the compiled kernel, 0 when the interpreter runs it (compile failed, not
 * eligible, no predicates), or a negative dq_status. */
int32_t dq_plan_pred_wait(dq_plan* plan, int32_t timeout_ms);
/* EXPLAIN of the plan dq_plan_create_opts would build, on the host only (no device, no allocation, no
 * compile): the launches per scan, the column-pass variants, the pair pass, the predicate program and -- when
 * the predicate pass would be compiled -- the generated kernel source.  Writes at most cap bytes (incl. the
 * terminator) to out and returns the full text's size incl. the terminator (call with cap 0 to size the
 * buffer), or a negative dq_status (planning errors as dq_plan_create reports them). */
int64_t dq_plan_explain(const dq_analyzer_spec* specs, int32_t n_specs, const dq_column_desc* schema, int32_t n_cols,
                        const dq_pred_node* pred_pool, int32_t n_pred, const char* const* patterns, int32_t n_patterns,
                        const dq_plan_options* opts, char* out, int64_t cap);
/* Host wall time dq_plan_create* spent on the plan (ms), and the part of it spent obtaining the compiled
 * predicate kernel (hipRTC compile, or a code-object cache lookup); 0 for the latter without one. */
dq_status dq_plan_create_time(const dq_plan* plan, double* total_ms, double* pred_jit_ms);

/* Grouping analyzers (analyzers/GroupingAnalyzers.scala:44-82, 118-138): the frequencies
 * SELECT cols, COUNT(*) FROM data WHERE cols IS NOT NULL GROUP BY cols on the GPU (sort-based), and
 * the summary Uniqueness / Distinctness / CountDistinct / Entropy / UniqueValueRatio compute from.
 * cols: n_chunks x n_cols views, chunk-major (device pointers).  A single numeric column groups by
 * its exact value (NaN canonical, -0.0 != 0.0 as Spark 2.2); strings / several columns group by a
 * 64-bit tuple hash whose equal-hash neighbours are compared exactly (a collision between distinct
 * tuples is DQ_E_UNSUPPORTED, never a silent merge).  dq_freq_merge is FrequenciesAndNumRows.sum
 * (outer join adding counts).  Hashed tables carry a second, independently seeded hash per group, so a
 * merge of two tables whose distinct tuples share a first hash is DQ_E_UNSUPPORTED, not a silent
 * merge; more than 2^31 - 1 groups in the two tables together is DQ_E_UNSUPPORTED. */
typedef struct dq_freq_table dq_freq_table;
typedef struct dq_freq_summary {
  int64_t num_groups;  /* rows of the frequencies table (CountDistinct) */
  int64_t num_unique;  /* groups with count == 1 */
  int64_t num_values;  /* rows with every grouping column non-null */
  double entropy;      /* sum over groups of -(c / num_rows) * ln(c / num_rows) (Entropy.scala:31-37) */
} dq_freq_summary;
dq_status dq_freq_build(const int32_t* types, int32_t n_cols, const dq_column_view* cols, const int64_t* chunk_rows,
                        int32_t n_chunks, int32_t device, void* hip_stream, dq_freq_table** out);
dq_status dq_freq_merge(const dq_freq_table* a, const dq_freq_table* b, dq_freq_table** out);
dq_status dq_freq_summarize(const dq_freq_table* t, int64_t num_rows, dq_freq_summary* out);
int64_t dq_freq_num_groups(const dq_freq_table* t);
dq_status dq_freq_export(const dq_freq_table* t, uint64_t* keys, int64_t* counts, int64_t cap);
void dq_freq_destroy(dq_freq_table* t);
/* ApproxQuantile / ApproxQuantiles (analyzers/ApproxQuantile.scala:49-103, ApproxQuantiles.scala:30-105;
 * replaces their DeequFunctions.stateful_approx_quantile aggregation + PercentileDigest.getPercentiles).
 * One numeric column (DQ_TYPE_F64 / I64 / I32) over n_chunks chunk views; per quantile the exact order
 * statistic of rank ceil(q * n) over the non-null values (rank 1 if q <= relative_error, n if
 * q >= 1 - relative_error, as Spark 2.2's QuantileSummaries.query), which is inside the GK error bound
 * the reference guarantees.  NaN sorts last (java.lang.Double.compare), -0.0 before 0.0.  *count = the
 * number of non-null values (0: no digest, out untouched).  Parameters outside [0, 1] are DQ_E_INVALID
 * with the reference's MetricCalculationException message in dq_last_error(). */
#define DQ_MAX_QUANTILES 8
dq_status dq_approx_quantiles(int32_t type, const dq_column_view* cols, const int64_t* chunk_rows, int32_t n_chunks,
                              const double* quantiles, int32_t n_q, double relative_error, int32_t device,
                              void* hip_stream, double* out, int64_t* count);
/* ApproxQuantileState's digest (ApproxQuantile.scala:28-35, 69-80), every sample rank in two passes over the
 * column: the order keys (Double.compare order: NaN largest, -0.0 < 0.0) counted per bucket against splitters
 * from an evenly spaced sample, then only the buckets holding a sample rank compacted and radix-sorted; the
 * values at the 1-based ranks 1, 1 + s, 1 + 2 s, ..., n with s = max(1, floor(2 relative_error n)) -- the samples of a
 * QuantileSummaries with exact ranks (g = rank gaps, delta = 0; deequ_amd/quantiles.py).  *count = n
 * (0: every value NULL, no samples); *n_samples = the number of samples; DQ_E_INVALID when it exceeds cap
 * (call again with a larger buffer; relative_error 0 samples every value). */
dq_status dq_quantile_digest(int32_t type, const dq_column_view* cols, const int64_t* chunk_rows, int32_t n_chunks,
                             double relative_error, int32_t device, void* hip_stream, double* values, int64_t* ranks,
                             int64_t cap, int64_t* n_samples, int64_t* count);
/* Histogram (analyzers/Histogram.scala:33-99): the n largest groups by count (ties in key order):
 * key, count and -- for a table built from data with hashed keys (strings) -- one representative row
 * id (chunk << 40 | row) whose value the caller renders; ~0 when not available (merged tables). */
dq_status dq_freq_top(const dq_freq_table* t, int32_t n, uint64_t* keys, int64_t* counts, uint64_t* rep_rows,
                      int32_t* n_out);
/* MutualInformation(a, b) (analyzers/MutualInformation.scala:32-72): joint frequencies of the two
 * columns, their marginals summed from the joint counts, and
 * sum (pxy / N) * ln((pxy / N) / ((px / N) * (py / N))) with N = num_rows.  cols: n_chunks x 2 views.
 * *defined = 0 when no row has both values (the SQL sum is NULL -> EmptyStateException). */
dq_status dq_mutual_information(const int32_t* types, const dq_column_view* cols, const int64_t* chunk_rows,
                                int32_t n_chunks, int64_t num_rows, int32_t device, void* hip_stream, double* value,
                                int32_t* defined);

/* State algebra.
 * dq_state_merge:   Analyzers.merge / State.sum on Option[State] (Analyzer.scala:343-362):
 *                   None + x = x; Min/Max merge with java.lang.Math.min/max.
 * dq_state_combine: Spark partial-aggregate merge of two aggregation-result slot sets (row
 *                   shards of one scan: GPUs, chunks): SQL null-skipping per slot, NaN-as-largest
 *                   min/max ordering.  Used for the multi-GPU allgather merge. */
dq_status dq_state_merge(const dq_state* a, const dq_state* b, dq_state* out);
dq_status dq_state_combine(const dq_state* a, const dq_state* b, dq_state* out);
/* Element-wise over n slot sets (a whole run's analyzers in one call: the fixed rank-order merge of the
 * multi-GPU all-gather, the incremental StateLoader append).  out may alias a or b. */
dq_status dq_state_merge_n(const dq_state* a, const dq_state* b, int32_t n, dq_state* out);
dq_status dq_state_combine_n(const dq_state* a, const dq_state* b, int32_t n, dq_state* out);
/* 1 if fromAggregationResult would produce Some(state). */
int32_t dq_state_is_defined(const dq_state* s);
/* metricValue() of a defined state (DoubleMetric analyzers; DATATYPE has a histogram, not a double:
   DQ_E_STATE). */
dq_status dq_state_metric(const dq_state* s, double* out);
/* HLL++ estimate of 52 packed words, bit-exact with DeequHyperLogLogPlusPlusUtils.count. */
dq_status dq_hll_estimate(const int64_t* words52, double* out);

/* HdfsStateProvider byte images (Java DataOutputStream, big-endian).  Returns the image length,
 * or a negative dq_status; writes nothing when buf is NULL / cap too small (returns length). */
int64_t dq_state_to_bytes(const dq_state* s, uint8_t* buf, int64_t cap);
dq_status dq_state_from_bytes(int32_t op, const uint8_t* buf, int64_t len, dq_state* out);
/* HdfsStateProvider.toIdentifier: MurmurHash3.stringHash(analyzer.toString, 42) of UTF-8 text. */
int32_t dq_state_identifier(const char* analyzer_to_string_utf8);

#ifdef __cplusplus
}
#endif

#endif /* DQSCAN_H */
