// dq_prim.h -- device-wide primitives of the grouping and quantile paths, hand-written for gfx950 (dq_prim.hip):
// a stable LSD radix sort of 64-bit keys carrying 0-, 4- or 8-byte values, prefix sums, and runs of equal keys.
// Every call is asynchronous on `stream`; `temp` is caller-owned scratch of at least the *_temp_bytes() size, and
// nothing else is allocated.  Item counts are < 2^31 (the grouping path's limit: dq_freq_build refuses more).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace dq {
namespace prim {

// Radix sort: by key bits [begin_bit, end_bit) (the bits at and above end_bit are taken to be equal in every key:
// callers pass the highest bit in which their keys differ); ascending, or descending over that bit range; equal keys
// keep their input order either way.  keys_in / vals_in are read only; keys_out / vals_out get the sorted sequence
// (they must not overlap the inputs).  val_bytes: 0 (keys only; vals_* ignored), 4 or 8.  Below 2^30 keys the call
// ends with a synchronisation of `stream` (it reads back the look-back's give-up flag: hipErrorLaunchTimeOut if a
// tile's wait for its predecessors ever exceeded its bound, so a wrong order is never returned).
size_t sort_temp_bytes(int64_t n, int val_bytes);
hipError_t sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const void* vals_in, void* vals_out, int val_bytes,
                      int64_t n, int begin_bit, int end_bit, bool descending, void* temp, size_t temp_bytes,
                      hipStream_t stream);

// Prefix sums (wrapping integer arithmetic): out[i] = in[0] + ... + in[i - 1] (exclusive) or + in[i] (inclusive).
// out may alias in.
size_t scan_temp_bytes(int64_t n);
hipError_t exclusive_sum_i64(const int64_t* in, int64_t* out, int64_t n, void* temp, hipStream_t stream);
hipError_t inclusive_sum_u32(const uint32_t* in, uint32_t* out, int64_t n, void* temp, hipStream_t stream);

// Runs of equal keys of keys[0 .. n) (sorted, or any order: a run is a maximal stretch of equal neighbours):
// unique[r] = run r's key, starts[r] = its first index, lengths[r] = its length, run_of[i] = the run holding position
// i (any of the four may be null), *num_runs (device memory) = the number of runs.  Each output array holds up to n
// entries (n < 2^31).
size_t runs_temp_bytes(int64_t n);
hipError_t runs(const uint64_t* keys, int64_t n, uint64_t* unique, int64_t* starts, int64_t* lengths,
                int64_t* num_runs, void* temp, hipStream_t stream, int32_t* run_of = nullptr);

// Per-run reductions over the runs() of the same n keys (starts / num_runs from runs(), on the device):
// sums[r] = the wrapping sum of vals over run r; firsts[r] = vals[starts[r]].
size_t run_sums_temp_bytes(int64_t n);
hipError_t run_sums_i64(const int64_t* vals, int64_t n, const int64_t* starts, const int64_t* num_runs, int64_t* sums,
                        void* temp, hipStream_t stream);
hipError_t run_firsts_u64(const uint64_t* vals, int64_t n, const int64_t* starts, const int64_t* num_runs,
                          uint64_t* firsts, hipStream_t stream);

}  // namespace prim
}  // namespace dq
