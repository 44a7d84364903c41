// dq_pred_jit.cpp -- the predicate pass compiled per plan (host C++; hipRTC for gfx950).
//
// The reference evaluates Compliance / `where` predicates with Spark's whole-stage code generation: each
// `expr(...)` becomes straight-line Java bytecode inside the one aggregation pass (AnalysisRunner.scala:303,
// Compliance.scala:37-53).  This is the same idea on the GPU.  dq_pred_scan interprets the postfix program
// per 512-row block (SQ counters: ~108 VALU + ~130 SALU per 64-row group for C3's four predicates, most of
// it decoding instructions and walking an LDS operand stack); for a program whose atoms are comparisons /
// IS [NOT] NULL on numeric columns the plan instead emits a kernel with the program unrolled into it:
//   * per wave, 512-row blocks (lane l: rows base + 64 j + l), each column's values loaded once per block;
//   * per 64-row group j: every atom is one ballot of a per-lane comparison (literals folded in), its
//     three-valued TRUE / NULL masks are 64-bit scalars, AND / OR / NOT are scalar mask ops, the counters
//     are scalar popcounts and a `where` root's TRUE mask is stored as its bitmap word;
//   * an HLL-only ApproxCountDistinct (no `where`) on a program column is hashed from the same registers
//     (XXH64 seed 42, the column pass's formulation, dq_hash.h), so that column is read from HBM once.
// The source is generated from the PredProgram the interpreter would run, compiled once per distinct source
// and device target (hipRTC for the device's gcnArchName; a process cache that also remembers failures, and a
// persistent code-object cache keyed by generator revision, target, hipRTC version and source), and launched in
// place of dq_pred_scan.  A program the generator does not take (regex atoms, strings, > 8 columns) or a failed
// compile keeps the interpreter and the column pass's HLL tasks -- unless the plan asked for DQ_PRED_PASS_COMPILED
// (dq_plan_create_opts), which then fails instead.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cinttypes>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <utility>
#include <vector>

#include "dq_device.h"
#include "dq_pred_jit.h"

namespace dq {

namespace {

// XXH64 pieces of dq_hash.h (its text, embedded at build time: build/dq_hash_src.inc)
const char* kHashSrc =
#include "dq_hash_src.inc"
    ;

const char* kPreamble = R"DQJIT(
#define DQ_JIT 1
typedef unsigned int uint32_t;
typedef int int32_t;
typedef unsigned long long uint64_t;
typedef long long int64_t;
typedef unsigned short uint16_t;
typedef short int16_t;
typedef unsigned char uint8_t;
typedef signed char int8_t;
typedef unsigned long long uintptr_t;
typedef const __attribute__((address_space(4))) uint32_t* dq_const_u32s;
)DQJIT";

const char* kHelpers = R"DQJIT(
namespace dqj {
using namespace dq;
struct Args {
  const char* values[8];
  const uint32_t* validity[8];
  uint64_t* where_bits[8];
  int64_t n_rows, rows_per_range;
  unsigned long long* acc_t;
  unsigned long long* acc_nn;
  char* col_part;
  uint32_t* hll_acc;
  int32_t hll_task[8];
  int32_t hll_slot[8];
};
// (hipRTC does not declare __builtin_amdgcn_inverse_ballot_w64: the lane's bit as a VALU test, and the hot
// exec-masked register max in asm)
__device__ __forceinline__ bool lane_bit(uint64_t m) { return (m >> __lane_id()) & 1ull; }
// ds_max_i32 under exec = m: LDS register max of the selected rows (regs_lds = the array's LDS address);
// the kernel waits for these (lgkmcnt) before its closing barrier
__device__ __forceinline__ void ds_max_masked(uint64_t m, uint32_t addr, int32_t q) {
  uint64_t save;
  asm volatile("s_and_saveexec_b64 %0, %1\n\tds_max_i32 %2, %3\n\ts_mov_b64 exec, %0"
               : "=&s"(save) : "s"(m), "v"(addr), "v"(q) : "memory", "scc");
}
// rows [r, r + 64) of the range below its end, from left = rows of the range from r on (32-bit: the scalar unit
// has no 64-bit ordered compare, so 64-bit row comparisons became VALU compares of SGPR pairs)
__device__ __forceinline__ uint64_t rows_mask(int32_t left) {
  return left >= 64 ? ~0ull : (left <= 0 ? 0ull : (1ull << left) - 1ull);
}
// validity words of a block (lanes 0..15: rows base + 32 l .. + 31).  A column without a bitmap gets the plan's
// all-ones bitmap (dq_plan.cpp), so the load is unconditional: no branch around it for the waitcnt pass to
// merge.  The 64-bit mask of row group j is then two readlanes: scalar loads of every group's words, hoisted
// by the compiler, overflowed the scalar file.
__device__ __forceinline__ uint32_t valid_words(const uint32_t* bm, int64_t base, int64_t n_rows, int lane) {
  // a global load with the word index clamped to the bitmap's last word (words past it belong to rows past
  // n_rows, which `inr` masks): a pointer instead of a four-register descriptor per column
  typedef const __attribute__((address_space(1))) uint32_t* gu32;
  const uint32_t last = (uint32_t)(((n_rows + 31) >> 5) - 1);
  const uint32_t w = (uint32_t)(base >> 5) + (uint32_t)(lane & 15);
  return ((gu32)bm)[w < last ? w : last];
}
__device__ __forceinline__ uint64_t group_mask(uint32_t w, int j) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)w, 2 * j + 1) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)w, 2 * j);
}
// Spark's ordering of doubles (nanSafeCompare): NaN = NaN, NaN above everything
__device__ __forceinline__ int spark_cmp(double a, double b) {
  const bool an = a != a, bn = b != b;
  if (an || bn) return (an && bn) ? 0 : (an ? 1 : -1);
  return (a > b) - (a < b);
}
__device__ __forceinline__ int32_t ffbh_raw(uint32_t x) {
  int32_t r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
// HLL key from the XXH64 state before its last multiply (dq_kernels.hip hll_key_from_fmix): register byte
// offset and q = pw - 1, or -1 when the rank needs the hash's low word (redone exactly)
__device__ __forceinline__ void hll_key(uint64_t b, uint32_t& addr, int32_t& q) {
  const uint32_t bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
  const uint32_t hi = __umulhi(bl, (uint32_t)XP3) + bl * (uint32_t)(XP3 >> 32) + bh * (uint32_t)XP3;
  addr = (hi >> 21) & 0x7FCu;
  q = ffbh_raw(hi << 9);
}
__device__ __forceinline__ void hll_exact(int32_t* regs, uint64_t x) {
  atomicMax(&regs[(uint32_t)(x >> 55)], (int32_t)__clzll((long long)((x << 9) | 256ull)));
}
}  // namespace dqj
)DQJIT";

std::string u64lit(uint64_t v) {
  char b[40];
  std::snprintf(b, sizeof b, "0x%016" PRIx64 "ull", v);
  return b;
}

// value expression of slot s row group j as int64 / double
// (the loads leave a 4- / 2- / 1-byte value zero-extended in the slot's uint64_t)
std::string as_int(int s, int kind) {
  const std::string v = "v" + std::to_string(s) + "[j]";
  switch (kind) {
    case CK_I32: return "(int64_t)(int32_t)(uint32_t)" + v;
    case CK_I16: return "(int64_t)(int16_t)(uint16_t)" + v;
    case CK_I8: return "(int64_t)(int8_t)(uint8_t)" + v;
    default: return "(int64_t)" + v;
  }
}
std::string as_dbl(int s, int kind) {
  const std::string v = "v" + std::to_string(s) + "[j]";
  if (kind == CK_F64) return "__longlong_as_double((long long)" + v + ")";
  if (kind == CK_F32) return "(double)__builtin_bit_cast(float, (uint32_t)" + v + ")";  // exact, as Spark's cast
  return "(double)" + as_int(s, kind);
}
const char* cmp_op(int c) {
  switch (c) {
    case C_LT: return "<";
    case C_LE: return "<=";
    case C_GT: return ">";
    case C_GE: return ">=";
    case C_EQ: return "==";
    default: return "!=";
  }
}

}  // namespace

// Size limits of a program the generator takes: every counter pair is pinned in SGPRs per row group (two per
// counter) next to the atoms' 64-bit masks; past ~24 counters LLVM's register allocation fails (after up to a
// minute of hipRTC time: 26 counters 9 s, 29 counters 70 s, measured in this container), so larger programs --
// a VerificationSuite with many Compliance checks -- stay on the interpreter, whose cost grows per atom anyway.
constexpr int kJitMaxCounters = 16, kJitMaxBitmaps = 8, kJitMaxInstr = 96;

bool pred_jit_eligible(const PredProgram& prog, const int32_t* col_kind, int32_t ncols, bool constant_ok) {
  if (prog.regex_words > 0 || (prog.n_loads == 0 && !constant_ok)) return false;
  if (prog.n_counters > kJitMaxCounters || prog.n_bitmaps > kJitMaxBitmaps || prog.n_instr > kJitMaxInstr) return false;
  std::vector<int32_t> cols;
  for (int i = 0; i < prog.n_instr; ++i) {
    const PredInstr& ins = prog.instr[i];
    if (ins.op == PO_ATOM_REGEX) return false;
    if (ins.op != PO_ATOM_CMP && ins.op != PO_ATOM_ISNULL && ins.op != PO_ATOM_NOTNULL) continue;
    for (int32_t c : {ins.col_a, ins.col_b}) {
      if (c < 0) continue;
      if (c >= ncols) return false;
      const int k = col_kind[c];
      if (k != CK_F64 && k != CK_I64 && k != CK_I32 && k != CK_F32 && k != CK_I16 && k != CK_I8) return false;
      bool seen = false;
      for (int32_t x : cols) seen = seen || x == c;
      if (!seen) cols.push_back(c);
    }
  }
  return (constant_ok || !cols.empty()) && cols.size() <= 8;
}

// The kernel source of `prog`; slot_col receives the program's distinct columns in slot order (the order of
// PredJitArgs::values / validity); fused HLL task h hashes slot hll[h].slot (its task and accumulator come
// in PredJitArgs::hll_task / hll_slot, so the source does not depend on task numbering).
// 64-row groups per wave block (<= 8: valid_words loads 16 validity dwords per lane group).  8 groups: 117
// VGPRs, 4 waves per SIMD, 0.870 ms per 125 M rows of C3; 4 groups (72 VGPRs, 7 waves) 0.871-0.904 ms, 2 groups
// 0.899-0.923 ms (profiles/r3_pred_ab.txt, r3u)
#ifndef DQ_JIT_GROUPS
#define DQ_JIT_GROUPS 8
#endif
constexpr int kJitGroups = DQ_JIT_GROUPS;  // (A/B builds: -DDQ_JIT_GROUPS=4)
// what may cross the barrier between a row group's predicate work and its hashing (sched_barrier mask; A/B
// builds: 0 = nothing crosses; 2 = VALU may cross: 0.838-0.847 vs 0.856-0.869 ms per 125 M rows of C3, r4i)
#ifndef DQ_JIT_SCHED_MASK
#define DQ_JIT_SCHED_MASK 2
#endif

std::string pred_jit_source(const PredProgram& prog, const int32_t* col_kind, std::vector<int32_t>& slot_col,
                            const std::vector<PredJitHll>& hll) {
  // each wave takes blocks of kJitGroups 64-row groups (the workgroup's four waves 4x that many rows)
  const std::string G = std::to_string(kJitGroups), WR = std::to_string(64 * kJitGroups),
                    BR = std::to_string(256 * kJitGroups);
  slot_col.clear();
  auto slot_of = [&](int32_t c) {
    for (size_t i = 0; i < slot_col.size(); ++i)
      if (slot_col[i] == c) return (int)i;
    slot_col.push_back(c);
    return (int)slot_col.size() - 1;
  };
  for (int i = 0; i < prog.n_instr; ++i) {
    const PredInstr& ins = prog.instr[i];
    if (ins.op != PO_ATOM_CMP && ins.op != PO_ATOM_ISNULL && ins.op != PO_ATOM_NOTNULL) continue;
    slot_of(ins.col_a);
    if (ins.col_b >= 0) slot_of(ins.col_b);
  }
  const int ns = (int)slot_col.size();
  std::vector<bool> need_vals(ns, false);
  for (int i = 0; i < prog.n_instr; ++i) {
    const PredInstr& ins = prog.instr[i];
    if (ins.op != PO_ATOM_CMP) continue;
    if (ins.cmp >= C_LT && ins.cmp <= C_NE) {
      need_vals[slot_of(ins.col_a)] = true;
      if (ins.col_b >= 0) need_vals[slot_of(ins.col_b)] = true;
    }
  }
  for (const PredJitHll& h : hll) need_vals[h.slot] = true;
  const int nh = (int)hll.size();

  std::string s;
  s.reserve(16384);
  s += kPreamble;
  s += kHashSrc;
  s += kHelpers;
  s += "extern \"C\" __global__ __launch_bounds__(256) void dq_pred_jit(dqj::Args A) {\n";
  s += "  using namespace dq; using namespace dqj;\n";
  s += "  __shared__ int32_t regs[" + std::to_string(nh > 0 ? nh * 512 : 1) + "];\n";
  s += "  __shared__ unsigned long long hcnt[" + std::to_string(nh > 0 ? nh : 1) + "];\n";
  s += "  __shared__ unsigned long long cacc[" + std::to_string(prog.n_counters > 0 ? 2 * prog.n_counters : 1) + "];\n";
  if (prog.n_counters > 0)
    s += "  if (threadIdx.x < " + std::to_string(2 * prog.n_counters) + ") cacc[threadIdx.x] = 0;\n";
  if (nh > 0) {
    s += "  for (int i = threadIdx.x; i < " + std::to_string(nh * 512) + "; i += 256) regs[i] = -1;\n";
    s += "  if (threadIdx.x < " + std::to_string(nh) + ") hcnt[threadIdx.x] = 0;\n";
  }
  s += "  __syncthreads();\n";
  s += "  const int lane = threadIdx.x & 63;\n";
  s += "  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n";
  s += "  const int64_t row0 = (int64_t)blockIdx.x * A.rows_per_range;\n";
  s += "  const int64_t row1 = row0 + A.rows_per_range < A.n_rows ? row0 + A.rows_per_range : A.n_rows;\n";
  for (int i = 0; i < ns; ++i) {
    const int k = col_kind[slot_col[i]];
    const int sz = ck_bytes(k);
    s += "  const uint32_t* vb" + std::to_string(i) + " = A.validity[" + std::to_string(i) + "];\n";
    if (need_vals[i])
      s += "  const __amdgpu_buffer_rsrc_t vr" + std::to_string(i) +
           " = __builtin_amdgcn_make_buffer_rsrc((void*)(A.values[" + std::to_string(i) + "] + row0 * " +
           std::to_string(sz) + "), (short)0, (int)((row1 - row0) * " + std::to_string(sz) + "), 0x00020000);\n";
  }
  // per-wave counters in 32 bits: a wave counts at most a quarter of its range's rows, and the planner's
  // ranges (>= 64 per chunk, dq_plan.cpp size_ranges) keep that far below 2^32 for any chunk HBM can hold
  for (int c = 0; c < prog.n_counters; ++c) s += "  uint32_t ct" + std::to_string(c) + " = 0, cn" + std::to_string(c) + " = 0;\n";
  for (int h = 0; h < nh; ++h) s += "  uint32_t hc" + std::to_string(h) + " = 0;\n";
  // values and validity words one block ahead, per row group: v[i][j] of the next block is loaded as soon as
  // row group j of this block is done with it (same registers), so the next block's loads are in flight
  // while this block is evaluated and hashed
  // the whole row offset goes in voffset (lane + block row + 64 j; the compiler moves the 64 j part into the
  // instruction's immediate offset): the descriptor's range check covers voffset + immediate, not soffset, so
  // a prefetch past the range's last row -- the next block of the range's last block -- reads 0 instead of
  // the bytes after the column
  auto load_vals = [&](int i, const std::string& soff, const std::string& j, const std::string& dst) {
    const int k = col_kind[slot_col[i]];
    const std::string si = std::to_string(i);
    if (k == CK_I32 || k == CK_F32)
      return dst + " = (uint64_t)__builtin_amdgcn_raw_buffer_load_b32(vr" + si + ", (lane + " + soff + " + 64 * " + j +
             ") * 4, 0, 2);\n";
    if (k == CK_I16)
      return dst + " = (uint64_t)__builtin_amdgcn_raw_buffer_load_b16(vr" + si + ", (lane + " + soff + " + 64 * " + j +
             ") * 2, 0, 2);\n";
    if (k == CK_I8)
      return dst + " = (uint64_t)__builtin_amdgcn_raw_buffer_load_b8(vr" + si + ", (lane + " + soff + " + 64 * " + j +
             "), 0, 2);\n";
    return "{ const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(vr" + si + ", (lane + " + soff + " + 64 * " + j +
           ") * 8, 0, 2); " + dst + " = ((uint64_t)w2[1] << 32) | w2[0]; }\n";
  };
  // the first block's loads in the loop's own issue order (row group by row group, each column's values, the
  // validity words after row group 0): the waitcnt pass merges the states the loop header is entered with, and
  // with a different prologue order it had settled on vmcnt(0) at every block's start (the whole next block
  // waited for before its first row group instead of each row group's own loads)
  for (int i = 0; i < ns; ++i) {
    const std::string si = std::to_string(i);
    if (need_vals[i]) s += "  uint64_t v" + si + "[" + G + "];\n";
    s += "  uint32_t vw" + si + ", vwn" + si + ";\n";
  }
  s += "#pragma unroll\n  for (int j = 0; j < " + G + "; ++j) {\n";
  for (int i = 0; i < ns; ++i)
    if (need_vals[i]) s += "    " + load_vals(i, "wave * " + WR, "j", "v" + std::to_string(i) + "[j]");
  s += "    if (j == 0) {\n";
  for (int i = 0; i < ns; ++i)
    s += "      vw" + std::to_string(i) + " = valid_words(vb" + std::to_string(i) + ", row0 + (int64_t)wave * " + WR +
         ", A.n_rows, lane);\n";
  // (the machine scheduler would otherwise issue them column by column)
  s += "    }\n    __builtin_amdgcn_sched_barrier(0);\n  }\n";
  // range-relative rows in 32 bits (scalar loop control and compares)
  s += "  const int32_t nrr = (int32_t)(row1 - row0);\n";
  s += "  for (int32_t rbk = 0; rbk < nrr; rbk += " + BR + ") {\n";
  s += "    const int soff = rbk + wave * " + WR + ";\n";
  s += "    if (soff >= nrr) break;\n";
  s += "    const int64_t base = row0 + soff;\n";
  s += "    const int32_t rem = nrr - soff;\n";
  for (int h = 0; h < nh; ++h) s += "    int32_t qmin" + std::to_string(h) + " = 0;\n";
  // a row group's predicate work (pt below): generated here, then placed in the row-group loop
  const size_t pt0 = s.size();
  s += "    const int64_t r = base + 64 * j;\n";
  s += "    const uint64_t inr = rows_mask(rem - 64 * j);\n";
  for (int i = 0; i < ns; ++i) s += "    const uint64_t va" + std::to_string(i) + " = group_mask(vw" + std::to_string(i) + ", j) & inr;\n";
  // the program: atoms and logic as scalar masks (SSA names, the operand stack resolved here)
  std::vector<std::pair<std::string, std::string>> stack;
  std::vector<std::pair<std::string, std::string>> roots(prog.n_roots > 0 ? prog.n_roots : 1);
  int tmp = 0;
  auto fresh = [&]() { return std::to_string(tmp++); };
  for (int i = 0; i < prog.n_instr; ++i) {
    const PredInstr& ins = prog.instr[i];
    const std::string id = fresh();
    const std::string T = "t" + id, N = "n" + id;
    switch (ins.op) {
      case PO_ATOM_CMP: {
        const int a = slot_of(ins.col_a), b = ins.col_b >= 0 ? slot_of(ins.col_b) : -1;
        const int ka = col_kind[ins.col_a], kb = b >= 0 ? col_kind[ins.col_b] : 0;
        std::string wc;
        if (ins.cmp == C_TRUE) wc = "~0ull";
        else if (ins.cmp < C_LT || ins.cmp > C_NE) wc = "0ull";
        else if (ins.ctype == CT_INT) {
          const std::string y = b >= 0 ? as_int(b, kb) : "(int64_t)" + u64lit((uint64_t)ins.lit_i);
          wc = "__builtin_amdgcn_ballot_w64(" + as_int(a, ka) + " " + cmp_op(ins.cmp) + " " + y + ")";
        } else {
          uint64_t lb;
          std::memcpy(&lb, &ins.lit_d, 8);
          const std::string y = b >= 0 ? as_dbl(b, kb) : "__longlong_as_double((long long)" + u64lit(lb) + ")";
          wc = "__builtin_amdgcn_ballot_w64(spark_cmp(" + as_dbl(a, ka) + ", " + y + ") " + cmp_op(ins.cmp) + " 0)";
        }
        const std::string va = "va" + std::to_string(a), vb = b >= 0 ? "va" + std::to_string(b) : "~0ull";
        const std::string nrt = ins.null_res == NR_TRUE ? "~0ull" : "0ull";
        const std::string nrn = ins.null_res == NR_NULL ? "~0ull" : "0ull";
        s += "    const uint64_t w" + id + " = " + wc + ";\n";
        s += "    const uint64_t " + T + " = (" + va + " & " + vb + " & w" + id + ") | (~" + va + " & " + vb + " & " + nrt + ");\n";
        s += "    const uint64_t " + N + " = ~" + vb + " | (~" + va + " & " + nrn + ");\n";
        stack.push_back({T, N});
        break;
      }
      case PO_ATOM_ISNULL:
      case PO_ATOM_NOTNULL: {
        const std::string va = "va" + std::to_string(slot_of(ins.col_a));
        s += "    const uint64_t " + T + " = " + (ins.op == PO_ATOM_ISNULL ? "~" : "") + va + ";\n";
        s += "    const uint64_t " + N + " = 0ull;\n";
        stack.push_back({T, N});
        break;
      }
      case PO_CONST:
        s += "    const uint64_t " + T + " = " + (ins.null_res == NR_TRUE ? "~0ull" : "0ull") + ";\n";
        s += "    const uint64_t " + N + " = " + (ins.null_res == NR_NULL ? "~0ull" : "0ull") + ";\n";
        stack.push_back({T, N});
        break;
      case PO_AND:
      case PO_OR: {
        if (stack.size() < 2) return std::string();
        const auto bb = stack.back();
        stack.pop_back();
        const auto aa = stack.back();
        stack.pop_back();
        const char* op = ins.op == PO_AND ? " & " : " | ";
        const char* fop = ins.op == PO_AND ? " | " : " & ";
        s += "    const uint64_t " + T + " = " + aa.first + op + bb.first + ";\n";
        s += "    const uint64_t f" + id + " = (~" + aa.first + " & ~" + aa.second + ")" + fop + "(~" + bb.first + " & ~" +
             bb.second + ");\n";
        s += "    const uint64_t " + N + " = ~" + T + " & ~f" + id + ";\n";
        stack.push_back({T, N});
        break;
      }
      case PO_NOT: {
        if (stack.empty()) return std::string();
        const auto aa = stack.back();
        stack.pop_back();
        s += "    const uint64_t " + T + " = ~" + aa.first + " & ~" + aa.second + ";\n";
        s += "    const uint64_t " + N + " = " + aa.second + ";\n";
        stack.push_back({T, N});
        break;
      }
      case PO_STORE:
        if (stack.empty() || ins.slot < 0 || ins.slot >= (int)roots.size()) return std::string();
        roots[ins.slot] = stack.back();
        stack.pop_back();
        break;
      default:
        return std::string();
    }
  }
  for (int c = 0; c < prog.n_counters; ++c) {
    const PredCounter pc = prog.counters[c];
    if (pc.pred < 0 || pc.pred >= (int)roots.size() || pc.where >= (int)roots.size()) return std::string();
    const std::string tw = pc.where < 0 ? "inr" : "(" + roots[pc.where].first + " & inr)";
    s += "    ct" + std::to_string(c) + " += (uint32_t)__builtin_popcountll(" + roots[pc.pred].first + " & " + tw + ");\n";
    s += "    cn" + std::to_string(c) + " += (uint32_t)__builtin_popcountll(~" + roots[pc.pred].second + " & " + tw + ");\n";
  }
  for (int b = 0; b < prog.n_bitmaps; ++b) {
    const int rt = prog.bitmap_root[b];
    if (rt < 0 || rt >= (int)roots.size()) return std::string();
    s += "    if (rem - 64 * j > 0 && lane == 0) A.where_bits[" + std::to_string(b) + "][r >> 6] = " + roots[rt].first + " & inr;\n";
  }
  // the group's counters are pinned here (left alone, LLVM sinks the popcount chains to the block's end
  // and every ballot of the block stays live until then: SGPR spills), and the group's predicate work
  // (scalar masks) completes before its hashing starts
  if (prog.n_counters > 0) {
    s += "    asm volatile(\"\" :";
    for (int c = 0; c < prog.n_counters; ++c)
      s += std::string(c ? "," : "") + " \"+s\"(ct" + std::to_string(c) + "), \"+s\"(cn" + std::to_string(c) + ")";
    s += ");\n";
  }
  const std::string pt = s.substr(pt0);
  s.resize(pt0);
  // (round 4: row group j + 1's predicate work emitted beside row group j's hashing, software-pipelined,
  // measured no different: 0.827-0.868 vs 0.829-0.852 ms per 125 M rows of C3, r4m)
  {
    s += "#pragma unroll\n  for (int j = 0; j < " + G + "; ++j) {\n" + pt;
    s += "    __builtin_amdgcn_sched_barrier(" + std::to_string(DQ_JIT_SCHED_MASK) + ");\n";
  }
  // fused HLL tasks: XXH64 of the slot's raw value (doubleToLongBits for fp64: NaN canonical), exec-masked
  // register max; the rare low-word rank redone exactly after the block.  All the group's hashes first (one
  // basic block: the scheduler interleaves the independent chains, each a dependent sequence of 64-bit
  // multiplies), then the register updates (each exec-masked ds_max ends a basic block).
  for (int h = 0; h < nh; ++h) {
    const PredJitHll& e = hll[h];
    const int k = col_kind[slot_col[e.slot]];
    const std::string hs = std::to_string(h), vs = "v" + std::to_string(e.slot) + "[j]";
    if (k == CK_I32) {
      s += "    const uint64_t hb" + hs + " = xxh64_int_head((uint32_t)" + vs + ");\n";
    } else if (k == CK_F64) {
      s += "    uint64_t raw" + hs + " = " + vs + ";\n";
      s += "    if (__longlong_as_double((long long)raw" + hs + ") != __longlong_as_double((long long)raw" + hs +
           ")) raw" + hs + " = 0x7FF8000000000000ull;\n";
      s += "    const uint64_t hb" + hs + " = xxh64_long_head(raw" + hs + ");\n";
    } else {
      s += "    const uint64_t hb" + hs + " = xxh64_long_head(" + vs + ");\n";
    }
    s += "    uint32_t addr" + hs + "; int32_t q" + hs + "; hll_key(hb" + hs + ", addr" + hs + ", q" + hs + ");\n";
  }
  for (int h = 0; h < nh; ++h) {
    const PredJitHll& e = hll[h];
    const std::string hs = std::to_string(h);
    s += "    {\n";
    s += "      const uint64_t sl = va" + std::to_string(e.slot) + " & inr;\n";
    s += "      hc" + hs + " += (uint32_t)__builtin_popcountll(sl);\n";
    s += "      asm volatile(\"\" : \"+s\"(hc" + hs + "));\n";
    s += "      qmin" + hs + " = q" + hs + " < qmin" + hs + " ? q" + hs + " : qmin" + hs + ";\n";
    s += "      ds_max_masked(sl, (uint32_t)(uintptr_t)(regs + " + std::to_string(h * 512) + ") + addr" + hs + ", q" + hs +
         ");\n";
    s += "    }\n";
  }
  for (int i = 0; i < ns; ++i)
    if (need_vals[i]) s += "    " + load_vals(i, "soff + " + BR, "j", "v" + std::to_string(i) + "[j]");
  // the next block's validity words right after row group 0 (loaded last, a whole block's loads would be
  // in flight ahead of them when the next block needs them)
  s += "    if (j == 0) {\n";
  for (int i = 0; i < ns; ++i)
    s += "      vwn" + std::to_string(i) + " = valid_words(vb" + std::to_string(i) + ", base + " + BR + ", A.n_rows, lane);\n";
  s += "    }\n";
  s += "  }\n";  // j
  for (int h = 0; h < nh; ++h) {
    const PredJitHll& e = hll[h];
    const int k = col_kind[slot_col[e.slot]];
    const std::string hs = std::to_string(h), vs = "v" + std::to_string(e.slot) + "[j]";
    s += "    if (__builtin_amdgcn_ballot_w64(qmin" + hs + " < 0) != 0) {\n";
    s += "#pragma unroll\n      for (int j = 0; j < " + G + "; ++j) {\n";
    s += "        if (!lane_bit(group_mask(vw" + std::to_string(e.slot) + ", j) & rows_mask(rem - 64 * j))) continue;\n";
    s += "        uint64_t cur;\n        " + load_vals(e.slot, "soff", "j", "cur");  // v[][j] holds the next block now
    if (k == CK_I32) {
      s += "        hll_exact(regs + " + std::to_string(h * 512) + ", xxh64_int((uint32_t)cur));\n";
    } else {
      s += "        uint64_t raw = cur;\n";
      if (k == CK_F64)
        s += "        if (__longlong_as_double((long long)raw) != __longlong_as_double((long long)raw)) raw = 0x7FF8000000000000ull;\n";
      s += "        hll_exact(regs + " + std::to_string(h * 512) + ", xxh64_long(raw));\n";
    }
    s += "      }\n    }\n";
  }
  for (int i = 0; i < ns; ++i) s += "    vw" + std::to_string(i) + " = vwn" + std::to_string(i) + ";\n";
  s += "  }\n";  // blk
  s += "  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // the last prefetches land before exit\n";
  // the workgroup's counters summed in LDS, then one global atomic per counter into one of kPredAccCopies
  // accumulator copies (blockIdx % copies; the host adds the copies): per-wave atomics on the same eight
  // addresses had serialized at the end of the launch (2048 -> 8192 workgroups: 0.84 -> 1.67 ms, r4o)
  s += "  if (lane == 0) {\n";
  for (int c = 0; c < prog.n_counters; ++c) {
    const std::string cs = std::to_string(c);
    s += "    atomicAdd(&cacc[" + std::to_string(2 * c) + "], (unsigned long long)ct" + cs + ");\n";
    s += "    atomicAdd(&cacc[" + std::to_string(2 * c + 1) + "], (unsigned long long)cn" + cs + ");\n";
  }
  for (int h = 0; h < nh; ++h) s += "    atomicAdd(&hcnt[" + std::to_string(h) + "], (unsigned long long)hc" + std::to_string(h) + ");\n";
  s += "  }\n";
  s += "  asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");\n";
  s += "  __syncthreads();\n";
  if (prog.n_counters > 0) {
    s += "  if (threadIdx.x < " + std::to_string(2 * prog.n_counters) + ") {\n";
    s += "    const int c = threadIdx.x >> 1;\n";
    s += "    unsigned long long* dst = ((threadIdx.x & 1) ? A.acc_nn : A.acc_t) + (size_t)(blockIdx.x % " +
         std::to_string(kPredAccCopies) + ") * " + std::to_string(sizeof(PredPartial) / 8) + " + c;\n";
    s += "    atomicAdd(dst, cacc[threadIdx.x]);\n";
    s += "  }\n";
  }
  if (nh > 0) {
    for (int h = 0; h < nh; ++h) {
        // ColPartial (dq_device.h, 96 bytes): n mean m2 sum isum count nan_count fmin fmax pinf ninf pad
      s += "  if (threadIdx.x == 0) {\n";
      s += "    char* p = A.col_part + ((size_t)A.hll_task[" + std::to_string(h) + "] * " + std::to_string(kMaxWG) +
           " + blockIdx.x) * 96;\n";
      s += "    uint64_t* w = reinterpret_cast<uint64_t*>(p);\n";
      s += "    w[0] = 0; w[1] = 0; w[2] = 0; w[3] = 0; w[4] = 0; w[5] = hcnt[" + std::to_string(h) + "]; w[6] = 0;\n";
      s += "    w[7] = 0x7FF0000000000000ull; w[8] = 0xFFF0000000000000ull; w[9] = 0; w[10] = 0; w[11] = 0;\n";
      s += "  }\n";
      s += "  {\n    uint32_t* dst = A.hll_acc + ((size_t)A.hll_slot[" + std::to_string(h) + "] * " + std::to_string(kHllCopies) +
           " + (blockIdx.x % " + std::to_string(kHllCopies) + ")) * 512;\n";
      s += "    for (int i = threadIdx.x; i < 512; i += 256) {\n";
      s += "      const uint32_t val = (uint32_t)(regs[" + std::to_string(h * 512) + " + i] + 1);\n";
      s += "      if (val > __builtin_nontemporal_load(dst + i)) atomicMax(dst + i, val);\n";
      s += "    }\n  }\n";
    }
  }
  s += "}\n";
  return s;
}

// hipRTC: the code object of `src` for `arch` (host only; no device needed)
bool pred_jit_compile_code(const std::string& src, const std::string& arch, std::vector<char>& code, std::string& err) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "dq_pred_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    err = "hiprtcCreateProgram failed";
    return false;
  }
  const std::string arch_opt = "--offload-arch=" + arch;
  const char* opts[] = {arch_opt.c_str(), "-O3", "-std=c++17"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    err = "hiprtc: " + log.substr(0, 2000);
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code.assign(n, 0);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  if (n == 0) {
    err = "hiprtc returned no code";
    return false;
  }
  return true;
}

namespace {

// generated-source revision: part of the disk-cache key, so code objects of an older generator are not reused
constexpr const char* kJitRevision = "dq_pred_jit r4f";
// disk-cache file header: magic, then the full key's length (u64, little-endian) and bytes, then the code object
constexpr char kCacheMagic[8] = {'D', 'Q', 'J', 'I', 'T', 'C', 'O', '1'};

uint64_t fnv1a64(const std::string& s, uint64_t h) {
  for (unsigned char c : s) h = (h ^ c) * 0x100000001B3ull;
  return h;
}

// a directory this user owns that no one else can write (the cache holds code this process loads and runs)
bool private_dir(const std::string& dir) {
  struct stat st;
  if (lstat(dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) return false;
  return st.st_uid == geteuid() && (st.st_mode & (S_IWGRP | S_IWOTH)) == 0;
}

// the persistent code-object cache directory: $DQ_JIT_CACHE_DIR ("off" disables it), else
// $XDG_CACHE_HOME/deequ_amd/jit, else $HOME/.cache/deequ_amd/jit; "" when none is usable -- including a
// directory not owned by this user or writable by its group / others (a planted code object would run)
std::string cache_dir() {
  const char* d = std::getenv("DQ_JIT_CACHE_DIR");
  std::string dir;
  if (d && *d) {
    if (std::strcmp(d, "off") == 0) return std::string();
    dir = d;
  } else if (const char* x = std::getenv("XDG_CACHE_HOME"); x && *x) {
    dir = std::string(x) + "/deequ_amd/jit";
  } else if (const char* h = std::getenv("HOME"); h && *h) {
    dir = std::string(h) + "/.cache/deequ_amd/jit";
  } else {
    return std::string();
  }
  // mkdir -p (0700: the cache holds code this user loads)
  for (size_t i = 1; i <= dir.size(); ++i)
    if (i == dir.size() || dir[i] == '/') {
      const std::string part = dir.substr(0, i);
      if (mkdir(part.c_str(), 0700) != 0 && errno != EEXIST) return std::string();
    }
  return private_dir(dir) ? dir : std::string();
}

// a cached code object built from exactly `key` (header compared byte for byte; owner checked)
bool read_cached(const std::string& path, const std::string& key, std::vector<char>& code) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  struct stat st;
  bool ok = fstat(fileno(f), &st) == 0 && S_ISREG(st.st_mode) && st.st_uid == geteuid();
  char magic[8];
  uint64_t klen = 0;
  ok = ok && std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kCacheMagic, 8) == 0 &&
       std::fread(&klen, 1, 8, f) == 8 && klen == key.size();
  if (ok) {
    std::string k(key.size(), '\0');
    ok = std::fread(&k[0], 1, k.size(), f) == k.size() && k == key;
  }
  if (ok) {
    const long at = std::ftell(f);
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f) - at;
    std::fseek(f, at, SEEK_SET);
    ok = n > 4;
    if (ok) {
      code.resize((size_t)n);
      ok = std::fread(code.data(), 1, (size_t)n, f) == (size_t)n;
    }
  }
  std::fclose(f);
  // an AMDGPU code object is an ELF file
  return ok && code[0] == 0x7F && code[1] == 'E' && code[2] == 'L' && code[3] == 'F';
}

void write_cached(const std::string& path, const std::string& key, const std::vector<char>& code) {
  const std::string tmp = path + ".tmp." + std::to_string((long)getpid());
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;
  const uint64_t klen = key.size();
  bool ok = std::fwrite(kCacheMagic, 1, 8, f) == 8 && std::fwrite(&klen, 1, 8, f) == 8 &&
            std::fwrite(key.data(), 1, key.size(), f) == key.size() &&
            std::fwrite(code.data(), 1, code.size(), f) == code.size();
  if (std::fclose(f) == 0 && ok) {
    if (std::rename(tmp.c_str(), path.c_str()) == 0) return;
  }
  std::remove(tmp.c_str());
}

// background compiles: joined at process exit (after the last plan, before hipRTC unloads)
struct Workers {
  std::mutex mu;
  std::vector<std::thread> threads;
  ~Workers() {
    std::lock_guard<std::mutex> lock(mu);
    for (std::thread& t : threads)
      if (t.joinable()) t.join();
  }
};

}  // namespace

// One (device, source) kernel: PENDING while hipRTC compiles it (on a background thread for AUTO plans), CODE
// once the code object exists (compiled or read from the disk cache), LOADED once a plan thread has loaded the
// module, FAILED with the reason (failures stay cached: a failing compile is not retried).  Its own mutex
// guards it, so a compile never holds the process-wide map's lock.
struct PredJitEntry {
  enum State { PENDING, CODE, LOADED, FAILED };
  std::mutex mu;
  std::condition_variable cv;
  State state = PENDING;
  std::vector<char> code;
  hipFunction_t fn = nullptr;
  std::string origin;  // "hiprtc" / "disk cache"
  std::string err;
};

namespace {

std::mutex g_map_mu;
std::map<std::pair<int, std::string>, PredJitRef> g_map;
Workers g_workers;  // declared after the map: destroyed (joined) first

// The code object of `src` for `device`: the disk cache, else hipRTC (then written to the disk cache).  Runs on a
// background thread for AUTO plans: everything that can take long -- hipRTC's first call loads the compiler
// (~0.15 s), a compile ~0.3 s -- stays off the plan-creating thread.
void obtain_code(PredJitRef e, std::string src, int device) {
  std::vector<char> code;
  std::string err, origin;
  bool ok = false;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    err = "hipGetDeviceProperties failed";
  } else {
    const std::string arch = prop.gcnArchName;
    int rv_major = 0, rv_minor = 0;
    hiprtcVersion(&rv_major, &rv_minor);
    const std::string key = std::string(kJitRevision) + "\n" + arch + "\nhiprtc " + std::to_string(rv_major) + "." +
                            std::to_string(rv_minor) + "\n" + src;
    char name[80];
    std::snprintf(name, sizeof name, "%016" PRIx64 "%016" PRIx64 ".co", fnv1a64(key, 0xCBF29CE484222325ull),
                  fnv1a64(key, 0x84222325CBF29CE4ull));
    const std::string dir = cache_dir();
    const std::string path = dir.empty() ? std::string() : dir + "/" + name;
    if (!path.empty() && read_cached(path, key, code)) {
      ok = true;
      origin = "disk cache";
    } else if (pred_jit_compile_code(src, arch, code, err)) {
      ok = true;
      origin = "hiprtc";
      if (!path.empty()) write_cached(path, key, code);
    }
  }
  std::lock_guard<std::mutex> lock(e->mu);
  if (ok) {
    e->code.swap(code);
    e->origin = origin;
    e->state = PredJitEntry::CODE;
  } else {
    e->err = err;
    e->state = PredJitEntry::FAILED;
  }
  e->cv.notify_all();
}

}  // namespace

PredJitRef pred_jit_request(const std::string& src, int device, bool background, double& ms) {
  const auto t0 = std::chrono::steady_clock::now();
  PredJitRef e;
  bool created = false;
  {
    std::lock_guard<std::mutex> lock(g_map_mu);  // held for the lookup only, never across hipRTC
    PredJitRef& slot = g_map[{device, src}];
    if (!slot) {
      slot = std::make_shared<PredJitEntry>();
      created = true;
    }
    e = slot;
  }
  if (created) {
    if (background) {
      std::lock_guard<std::mutex> lock(g_workers.mu);
      g_workers.threads.emplace_back(obtain_code, e, src, device);
    } else {
      obtain_code(e, src, device);
    }
  }
  ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return e;
}

hipFunction_t pred_jit_poll(const PredJitRef& e, int32_t wait_ms, std::string& note) {
  if (!e) {
    note = "no kernel requested";
    return nullptr;
  }
  std::unique_lock<std::mutex> lock(e->mu);
  auto done = [&] { return e->state != PredJitEntry::PENDING; };
  if (wait_ms < 0) e->cv.wait(lock, done);
  else if (wait_ms > 0) e->cv.wait_for(lock, std::chrono::milliseconds(wait_ms), done);
  switch (e->state) {
    case PredJitEntry::PENDING:
      note = "compiling in the background (hipRTC): the interpreter runs until it is ready";
      return nullptr;
    case PredJitEntry::FAILED:
      note = e->err;
      return nullptr;
    case PredJitEntry::LOADED:
      note = "process cache";
      return e->fn;
    case PredJitEntry::CODE: {  // load the module on this (plan) thread; it stays loaded for the process
      hipModule_t mod = nullptr;
      hipFunction_t fn = nullptr;
      if (hipModuleLoadData(&mod, e->code.data()) != hipSuccess) {
        e->err = note = "hipModuleLoadData failed";
        e->state = PredJitEntry::FAILED;
        return nullptr;
      }
      if (hipModuleGetFunction(&fn, mod, "dq_pred_jit") != hipSuccess) {
        e->err = note = "hipModuleGetFunction failed";
        e->state = PredJitEntry::FAILED;
        return nullptr;
      }
      e->fn = fn;
      e->state = PredJitEntry::LOADED;
      std::vector<char>().swap(e->code);
      note = e->origin;
      return fn;
    }
  }
  return nullptr;
}

hipError_t pred_jit_launch(hipFunction_t fn, const PredJitArgs& a, int32_t nranges, hipStream_t st) {
  PredJitArgs args = a;
  void* params[] = {&args};
  return hipModuleLaunchKernel(fn, (unsigned)nranges, 1, 1, kBlock, 1, 1, 0, st, params, nullptr);
}

}  // namespace dq

namespace dq {
bool pred_jit_pending(const PredJitRef& e) {
  if (!e) return false;
  std::lock_guard<std::mutex> lock(e->mu);
  return e->state == PredJitEntry::PENDING;
}
}  // namespace dq
