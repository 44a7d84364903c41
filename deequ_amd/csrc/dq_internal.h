// dq_internal.h -- host-side internals shared by the C ABI translation units.
#pragma once

#include <cstdarg>
#include <cstdint>

#include <hip/hip_runtime.h>  // (dq_decimal.h's host + device functions: every TU here is compiled as HIP)

#include "../../include/dqscan.h"
#include "dq_decimal.h"

namespace dq {

// Column type codes: a DECIMAL128 code carries (precision, scale) above its enum value (DQ_DECIMAL128); every other
// code is its enum value alone.
inline bool is_decimal(int32_t t) { return DQ_TYPE_BASE(t) == DQ_TYPE_DECIMAL128; }
inline bool type_valid(int32_t t) {
  if (t >= DQ_TYPE_F64 && t <= DQ_TYPE_TIMESTAMP) return true;
  if ((t & ~0xFFFFFF) != 0 || !is_decimal(t)) return false;
  const int p = DQ_DECIMAL_PRECISION(t), s = DQ_DECIMAL_SCALE(t);
  return p >= 1 && p <= kDecMaxPrecision && s <= p;
}
// dq_decimal.h's constants for host code (dq_state.cpp)
const DecTab& dec_host_tab();
// Sum of a DECIMAL128 column as Spark 2.2 finishes it: the exact sum (128-bit, wrapped) at scale s cast to double;
// false when the sum is Spark's NULL (unscaled magnitude >= 10^digits, or the fp64 guard says the wrapped image is
// not the sum)
bool dec_sum_value(int64_t lo, int64_t hi, double guard, int s, int digits, double& out);

// HLL++ geometry (StatefulHyperloglogPlus.scala:154-161, HLLConstants.scala:27-35)
constexpr int kHllP = 9;
constexpr int kHllM = 1 << kHllP;       // 512 registers
constexpr int kHllRegisterBits = 6;
constexpr int kHllRegsPerWord = 10;     // 64 / 6
constexpr int kHllWords = 52;
constexpr int kHllK = 6;

// Thread-local last error; returns `code` for `return set_error(...)` chaining.
dq_status set_error(dq_status code, const char* fmt, ...);

double java_min(double a, double b);
double java_max(double a, double b);
int64_t java_math_round(double a);
void hll_registers_to_words(const uint8_t* regs512, int64_t* words52);
double hll_count(const int64_t* words52);
int32_t state_is_defined(const dq_state& s);
dq_status state_merge(const dq_state& a, const dq_state& b, dq_state& o);
dq_status state_combine(const dq_state& a, const dq_state& b, dq_state& o);
dq_status state_metric(const dq_state& s, double& out);
int64_t state_to_bytes(const dq_state& s, uint8_t* buf, int64_t cap);
dq_status state_from_bytes(int32_t op, const uint8_t* buf, int64_t len, dq_state& o);
int32_t murmur3_string_hash_utf8(const char* s, uint32_t seed);

}  // namespace dq
