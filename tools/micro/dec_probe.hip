// dec_probe.hip -- diagnostic: dq_decimal.h's conversion on the device for the values on stdin ("lo hi s" per line);
// prints the result bits and the intermediate terms, to compare with the host formulation (tests/decimal_check.cpp).
#include <hip/hip_runtime.h>
#include <cinttypes>
#include <cstdio>
#include <vector>
#include "../../deequ_amd/csrc/dq_decimal.h"
#define DQ_DEC_TABLE static __constant__ const
#include "../../deequ_amd/csrc/dq_dec_tables.inc"
#undef DQ_DEC_TABLE
using namespace dq;
__global__ void probe(const uint64_t* in, int n, double* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DecTab t{kDecP10Lo, kDecP10Hi, kDecRcpHi, kDecRcpLo};
  const uint64_t lo = in[3 * i], hi = in[3 * i + 1];
  const int s = (int)in[3 * i + 2];
  const u128 a = dec_mag(lo, hi);
  const double ah = (double)a;
  const double al = (double)(i128)(a - (u128)ah);
  out[8 * i + 0] = dec_to_double(lo, hi, s, t);
  out[8 * i + 1] = ah;
  out[8 * i + 2] = al;
  out[8 * i + 3] = t.rh[s];
  out[8 * i + 4] = t.rl[s];
  out[8 * i + 5] = (double)(uint64_t)a;
  out[8 * i + 6] = (double)(int64_t)(a - (u128)ah);
  out[8 * i + 7] = 0;
}
int main() {
  std::vector<uint64_t> in;
  unsigned long long lo, hi;
  int s;
  while (std::scanf("%llu %llu %d", &lo, &hi, &s) == 3) { in.push_back(lo); in.push_back(hi); in.push_back((uint64_t)s); }
  const int n = (int)(in.size() / 3);
  uint64_t* din; double* dout;
  hipMalloc(&din, in.size() * 8); hipMalloc(&dout, (size_t)n * 64);
  hipMemcpy(din, in.data(), in.size() * 8, hipMemcpyHostToDevice);
  probe<<<(n + 63) / 64, 64>>>(din, n, dout);
  std::vector<double> out((size_t)n * 8);
  hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 7; ++k) std::printf("%a ", out[8 * i + k]);
    std::printf("\n");
  }
  return 0;
}
