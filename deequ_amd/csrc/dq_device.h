// dq_device.h -- POD structures shared by the planner (host) and the gfx950 kernels.
//
// HBM layout of one plan (all device-resident, allocated once at dq_plan_create):
//   ColTask[ncol_tasks], PairTask[npair_tasks], PredProgram        (static task tables)
//   ColPartial[ncol_tasks][kMaxWG]     per-workgroup partial states of the current scan
//   CorrPartial[npair][kMaxWG], PredPartial[kMaxWG]
//   ColPartial / CorrPartial / PredPartial accumulators (merged over chunks, in order)
//   uint32 hll[nhll][kHllCopies][512]  HLL registers, merged in by atomicMax (order-free); a
//                                      workgroup merges into copy blockIdx % kHllCopies
//   where bitmaps: uint64[n_rows/64] TRUE bits per `where` root used by column / pair tasks
#pragma once

#include <cstdint>

namespace dq {

constexpr int kBlock = 256;                 // threads per workgroup (4 waves of 64)
constexpr int kWaves = kBlock / 64;
constexpr int kRowsPerLane = 8;
constexpr int kRowsPerIter = kBlock * kRowsPerLane;  // 2048 rows per workgroup iteration
constexpr int kMaxWG = 4096;                // max row ranges (workgroups) per task per scan
constexpr int kTargetWGs = 8192;            // column/pair launch: aim for ~32 workgroups per CU
constexpr int kMaxCols = 64;                // columns one plan reads (ScanCols); more: dq_plan_create splits
constexpr int kMaxColTasks = 256;           // column tasks of one plan
constexpr int kMaxSchemaCols = 1 << 16;     // columns of one dq_plan_create call (split over plans of kMaxCols)
constexpr int kMaxWhere = 8;
constexpr int kHllCopies = 8;             // accumulator copies per HLL column (spreads the merge atomics)
constexpr int kPredAccCopies = 16;        // predicate-counter accumulator copies (compiled pass: one per blockIdx % 16)
constexpr int kMaxRoots = 32;
constexpr int kMaxCounters = 32;
constexpr int kMaxInstr = 96;
constexpr int kPredStack = 16;              // predicate pass: operand stack depth
constexpr int kMaxRegexWords = 32768;       // compiled regex DFAs of one plan (64 KB of LDS)

// column kinds seen by the kernels (physical layouts: DATE32 columns are CK_I32, TIMESTAMP columns CK_I64 --
// the planner's preconditions keep their non-numeric analyzers away)
enum ColKind : int32_t {
  CK_F64 = 1, CK_I64 = 2, CK_I32 = 3, CK_UTF8 = 4, CK_LUTF8 = 5,
  CK_F32 = 6, CK_I16 = 7, CK_I8 = 8, CK_BOOL = 9,  // (BOOL: LSB-first value bitmap)
  CK_D128 = 10,  // DecimalType: 16-byte two's-complement unscaled values (the column pass)
  // a decimal column's 64-bit halves as predicate atom operands (stride 16; the planner splits a 128-bit
  // comparison into atoms on them): the low word as a signed long (precision <= 18: the whole value), the high
  // word, and the low word with its sign bit flipped (unsigned order as signed order)
  CK_D128_LO = 11, CK_D128_HI = 12, CK_D128_LOU = 13,
};
constexpr bool ck_float(int k) { return k == CK_F64 || k == CK_F32; }
constexpr int ck_bytes(int k) {
  return k >= CK_D128 ? 16 : k == CK_F64 || k == CK_I64 ? 8 : k == CK_I32 || k == CK_F32 ? 4 : k == CK_I16 ? 2 : 1;
}

// column-pass variants (kind x what is accumulated); VALIDITY = count of selected rows only
enum ColVariant : int32_t {
  CV_VALIDITY = 0,
  CV_F64_S = 1, CV_F64_SH = 2, CV_F64_H = 3,
  CV_I64_S = 4, CV_I64_SH = 5, CV_I64_H = 6,
  CV_I32_S = 7, CV_I32_SH = 8, CV_I32_H = 9,
  CV_UTF8_H = 10, CV_LUTF8_H = 11,
  // DataType (StatefulDataType.scala:36-69): string columns classify every selected value (alone or
  // fused with the HLL pass); double columns count the values whose Double.toString is fractional
  CV_UTF8_D = 12, CV_UTF8_HD = 13, CV_LUTF8_D = 14, CV_LUTF8_HD = 15, CV_F64_D = 16,
  // round 6: FloatType / ShortType / ByteType values (converted to double exactly, hashed as Spark 2.2 does), the
  // DataType count of a float column, and a boolean column's selected / TRUE counts (+ its two HLL hashes)
  CV_F32_S = 17, CV_F32_SH = 18, CV_F32_H = 19,
  CV_I16_S = 20, CV_I16_SH = 21, CV_I16_H = 22,
  CV_I8_S = 23, CV_I8_SH = 24, CV_I8_H = 25,
  CV_F32_D = 26, CV_BOOL = 27,
  // DecimalType (ColTask::arg = precision | scale << 8): values cast to double as Decimal.toDouble (correctly
  // rounded), the exact 128-bit sum, Spark 2.2's decimal hash, and the DataType count of BigDecimal.toString
  CV_D128_S = 28, CV_D128_SH = 29, CV_D128_H = 30, CV_D128_D = 31,
};
constexpr int kNumVariants = 32;

// per-variant row-range counts of one scan (dq_finalize merges nr[i] partials for tasks [first, end))
// column-task ranges whose range count differs from the scan's default (string passes, the validity pass, a
// predicate pass's fused HLL tasks): at most one entry per launch group of a scan
constexpr int kMaxFinRanges = 2 * kNumVariants + 1;
struct FinRanges {
  int32_t n;
  int32_t first[kMaxFinRanges], end[kMaxFinRanges], nr[kMaxFinRanges];
};

struct ColTask {
  int32_t variant;   // ColVariant
  int32_t col;       // column index
  int32_t where;     // where-bitmap index or -1
  int32_t hll_slot;  // index into HLL partial / accumulator arrays, -1 if none
  int32_t arg;       // CV_D128_*: precision | scale << 8
  int32_t pad[3];
};

struct PairTask {
  int32_t col_x, col_y;
  int32_t kind_x, kind_y;
  int32_t where;
  int32_t pad[3];
};

// Correlation pairs sharing <= 8 distinct columns and one `where` (host-side planning unit; staged together).
constexpr int kTileCols = 8;
constexpr int kTilePairs = 32;
struct PairGroup {
  int32_t ncols;
  int32_t npairs;
  int32_t first_pair;               // pairs [first_pair, first_pair + npairs) of the pair-task table
  int32_t where;                    // where-bitmap index or -1
  int32_t cols[kTileCols];          // plan column indices
  int32_t kinds[kTileCols];         // numeric kinds (CK_F64 / CK_F32 / CK_I64 / CK_I32 / CK_I16 / CK_I8)
  int8_t pi[kTilePairs], pj[kTilePairs];  // local column index of x / y per pair
};

// Correlation pass (dq_pair.hip).  A workgroup task is one pair group (<= 8 columns, one `where`) and two
// wave tasks.  Wave w's position p holds the group's local column (p + w) % 8; both waves run the same
// fixed pattern of kPairSlots slots over their 8 positions, and the two rotations of that pattern are
// every pair of 8 columns exactly once (28 = 2 x 14).  The column-moment tasks (Mean / StandardDeviation /
// Sum / Min / Max of the same rows and `where`) sit at the even positions (local column c: wave c % 2,
// position c - c % 2), fused so each column is read from HBM once for its correlations AND its moments.
constexpr int kPairWaves = 2;
constexpr int kPairPos = 8;
constexpr int kPairSlots = 14;
constexpr int kPairMoments = 4;              // at positions 0, 2, 4, 6
constexpr int kPairSlotA[kPairSlots] = {0, 2, 4, 6, 0, 2, 4, 6, 0, 2, 4, 6, 0, 2};
constexpr int kPairSlotB[kPairSlots] = {1, 3, 5, 7, 2, 4, 6, 0, 3, 5, 7, 1, 4, 6};
struct PairWaveTask {
  int32_t where;                   // where-bitmap index or -1
  uint32_t pair_mask;              // bit q: slot q (positions kPairSlotA[q], kPairSlotB[q]) is a pair task
  uint32_t mom_mask;               // bit m: position 2 m has a column-moments task
  uint32_t swap_mask;              // bit q: the pair task's first column is position kPairSlotB[q]
  int32_t cols[kPairPos];          // plan column indices (an unused position repeats a used column)
  int32_t kinds[kPairPos];         // numeric kinds (CK_F64 / CK_F32 / CK_I64 / CK_I32 / CK_I16 / CK_I8)
  int32_t pair_out[kPairSlots];    // pair-task index of each active slot
  int32_t mom_out[kPairMoments];   // column-task index of each moments position
};
struct PairWG {
  PairWaveTask wave[kPairWaves];
};

// Per-workgroup partial of one column task.  Moments are Chan-mergeable (n, mean, m2).
struct alignas(16) ColPartial {
  double n, mean, m2;   // over selected rows, values converted to double
  double sum;           // fp64 sum of selected values (F64 columns)
  int64_t isum;         // wrapping int64 sum (I64 / I32 columns)
  int64_t count;        // selected rows (non-null AND where-true)
  int64_t nan_count;    // selected NaN values (F64)
  double fmin, fmax;    // min / max over selected non-NaN values (F64)
  int64_t pinf_count;   // selected +inf values (F64; kept out of the moments, added back in dq_finish)
  int64_t ninf_count;   // selected -inf values (F64)
  int64_t isum_hi;      // D128: high word of the exact 128-bit sum (isum its low word; `sum` the fp64 guard)
};
static_assert(sizeof(ColPartial) == 96, "ColPartial layout");

struct alignas(16) CorrPartial {
  double n, xa, ya, ck, xm, ym, pad0, pad1;
};
static_assert(sizeof(CorrPartial) == 64, "CorrPartial layout");

struct alignas(16) PredPartial {
  int64_t t[kMaxCounters];   // sum over rows of (pred TRUE  AND where TRUE)
  int64_t nn[kMaxCounters];  // sum over rows of (pred NOT NULL AND where TRUE)
};

// Predicate program: postfix over three-valued atoms.
enum PredOp : int32_t {
  PO_ATOM_CMP = 1,     // col_a CMP (col_b | literal)
  PO_ATOM_ISNULL = 2,  // col_a IS NULL
  PO_ATOM_NOTNULL = 3, // col_a IS NOT NULL
  PO_CONST = 4,        // push constant (null_res: 0 FALSE, 1 TRUE, 2 NULL)
  PO_AND = 5,
  PO_OR = 6,
  PO_NOT = 7,
  PO_STORE = 8,        // pop into root slot `slot`
  PO_ATOM_REGEX = 9,   // search DFA (lit_i = word offset in PredProgram::regex) over UTF8 column col_a;
                       // NULL value -> null_res (RLIKE: NULL, PatternMatch: FALSE)
};
enum CmpOp : int32_t { C_LT = 1, C_LE = 2, C_GT = 3, C_GE = 4, C_EQ = 5, C_NE = 6, C_FALSE = 7, C_TRUE = 8 };
enum CmpType : int32_t { CT_INT = 1, CT_DBL = 2 };
enum NullRes : int32_t { NR_FALSE = 0, NR_TRUE = 1, NR_NULL = 2 };

struct PredInstr {
  int32_t op;
  int32_t cmp;
  int32_t ctype;
  int32_t null_res;   // ATOM_CMP: result when col_a is NULL (COALESCE fallback), else NR_NULL
  int32_t col_a;
  int32_t col_b;      // -1: compare against the literal
  int32_t kind_a;
  int32_t kind_b;
  int64_t lit_i;
  double lit_d;
  int32_t slot;
  int32_t pad;
};

struct PredCounter {
  int32_t pred;   // root slot
  int32_t where;  // root slot or -1
};

struct PredProgram {
  const uint16_t* regex;           // device: concatenated DFAs (n_states, n_classes, start, flags,
                                   // cls[256], acc_end[n_states], trans[n_states][n_classes])
  int32_t regex_words;             // its length (uint16 words); staged into LDS by dq_pred_scan
  int32_t n_instr;
  int32_t n_counters;
  int32_t n_bitmaps;
  int32_t n_loads;                 // atoms (the instructions that read a column)
  int32_t n_roots;                 // root slots stored by the program
  int32_t stack_depth;             // max operand stack depth (<= kPredStack)
  int16_t load_instr[kMaxInstr];   // their instruction indices, in program order
  int32_t bitmap_root[kMaxWhere];  // root slot whose TRUE bits fill where-bitmap i
  PredCounter counters[kMaxCounters];
  PredInstr instr[kMaxInstr];
};

// Per-scan column pointers, passed by value as a kernel argument (copied at launch).
struct ScanCols {
  const void* values[kMaxCols];
  const uint32_t* validity[kMaxCols];
  const void* offsets[kMaxCols];
};

struct ScanBitmaps {
  uint64_t* where_bits[kMaxWhere];
  int64_t* rare_rows;  // per column task: the rows the string pass's fast path skipped since the reset
};

}  // namespace dq
