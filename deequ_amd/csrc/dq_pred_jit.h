// dq_pred_jit.h -- the predicate pass compiled per plan (dq_pred_jit.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "dq_device.h"

namespace dq {

// kernel argument block (layout shared with the generated source's dqj::Args)
struct PredJitArgs {
  const char* values[8];
  const uint32_t* validity[8];
  uint64_t* where_bits[8];
  int64_t n_rows, rows_per_range;
  unsigned long long* acc_t;
  unsigned long long* acc_nn;
  char* col_part;
  uint32_t* hll_acc;
  int32_t hll_task[8];  // fused HLL task h: column task (ColPartial row) and HLL accumulator slot
  int32_t hll_slot[8];
};

// an HLL-only column task hashed by the predicate kernel: its program slot
struct PredJitHll {
  int32_t slot;
};

// col_kind[c]: CK_* of plan column c
// constant_ok: a program with no atoms passes (the split's capacity probe: a constant root can join any part)
bool pred_jit_eligible(const PredProgram& prog, const int32_t* col_kind, int32_t ncols, bool constant_ok = false);
std::string pred_jit_source(const PredProgram& prog, const int32_t* col_kind, std::vector<int32_t>& slot_col,
                            const std::vector<PredJitHll>& hll);
// hipRTC compile of `src` for `arch` (host only)
bool pred_jit_compile_code(const std::string& src, const std::string& arch, std::vector<char>& code, std::string& err);
// The kernel of `src` on `device`, from the process cache, the disk cache, or hipRTC -- on a background thread
// when `background` (the caller polls), else before returning; ms: host time spent in the request.
struct PredJitEntry;
using PredJitRef = std::shared_ptr<PredJitEntry>;
PredJitRef pred_jit_request(const std::string& src, int device, bool background, double& ms);
// The loaded function once the code object exists (the module is loaded on the calling thread), else null;
// wait_ms: how long to wait for a pending compile (0: not at all, < 0: until it has finished).  note: the code
// object's origin, or why there is no function.
hipFunction_t pred_jit_poll(const PredJitRef& e, int32_t wait_ms, std::string& note);
// true while the compile is still running
bool pred_jit_pending(const PredJitRef& e);
hipError_t pred_jit_launch(hipFunction_t fn, const PredJitArgs& a, int32_t nranges, hipStream_t st);

}  // namespace dq
