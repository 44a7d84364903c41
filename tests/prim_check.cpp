// prim_check.cpp -- test harness over the device primitives of deequ_amd/csrc/dq_prim.hip (tests/test_prim_gpu.py).
// Built by deequ_amd/Makefile into deequ_amd/build/libdqprimcheck.so with dq_prim's object; not part of the product
// ABI.  Every entry point takes device pointers (torch tensors), allocates its scratch, runs on the null stream and
// returns the hipError_t of the call (0 = success).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../deequ_amd/csrc/dq_prim.h"

namespace {
struct Scratch {
  void* p = nullptr;
  hipError_t alloc(size_t b) { return hipMalloc(&p, b < 256 ? 256 : b); }
  ~Scratch() {
    if (p) (void)hipFree(p);
  }
};
}  // namespace

extern "C" {

int prim_sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const void* vals_in, void* vals_out, int val_bytes,
                    int64_t n, int begin_bit, int end_bit, int descending) {
  Scratch s;
  const size_t tb = dq::prim::sort_temp_bytes(n, val_bytes);
  if (hipError_t e = s.alloc(tb)) return (int)e;
  if (hipError_t e = dq::prim::sort_pairs(keys_in, keys_out, vals_in, vals_out, val_bytes, n, begin_bit, end_bit,
                                          descending != 0, s.p, tb, nullptr))
    return (int)e;
  return (int)hipDeviceSynchronize();
}

int prim_exclusive_sum_i64(const int64_t* in, int64_t* out, int64_t n) {
  Scratch s;
  if (hipError_t e = s.alloc(dq::prim::scan_temp_bytes(n))) return (int)e;
  if (hipError_t e = dq::prim::exclusive_sum_i64(in, out, n, s.p, nullptr)) return (int)e;
  return (int)hipDeviceSynchronize();
}

int prim_inclusive_sum_u32(const uint32_t* in, uint32_t* out, int64_t n) {
  Scratch s;
  if (hipError_t e = s.alloc(dq::prim::scan_temp_bytes(n))) return (int)e;
  if (hipError_t e = dq::prim::inclusive_sum_u32(in, out, n, s.p, nullptr)) return (int)e;
  return (int)hipDeviceSynchronize();
}

// runs + per-run sums / firsts of vals (either may be null); *num_runs_host gets the run count
int prim_runs(const uint64_t* keys, int64_t n, uint64_t* unique, int64_t* starts, int64_t* lengths,
              const int64_t* sum_vals, int64_t* sums, const uint64_t* first_vals, uint64_t* firsts,
              int64_t* num_runs_host, int32_t* run_of) {
  Scratch s, r, nr;
  if (hipError_t e = s.alloc(dq::prim::runs_temp_bytes(n))) return (int)e;
  if (hipError_t e = r.alloc(dq::prim::run_sums_temp_bytes(n))) return (int)e;
  if (hipError_t e = nr.alloc(8)) return (int)e;
  int64_t* d_num = static_cast<int64_t*>(nr.p);
  if (hipError_t e = dq::prim::runs(keys, n, unique, starts, lengths, d_num, s.p, nullptr, run_of)) return (int)e;
  if (sum_vals && sums && starts)
    if (hipError_t e = dq::prim::run_sums_i64(sum_vals, n, starts, d_num, sums, r.p, nullptr)) return (int)e;
  if (first_vals && firsts && starts)
    if (hipError_t e = dq::prim::run_firsts_u64(first_vals, n, starts, d_num, firsts, nullptr)) return (int)e;
  if (hipError_t e = hipMemcpy(num_runs_host, d_num, 8, hipMemcpyDeviceToHost)) return (int)e;
  return (int)hipDeviceSynchronize();
}

}  // extern "C"
