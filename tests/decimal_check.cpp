// decimal_check.cpp -- host harness for tests/test_decimal_host.py: runs dq_decimal.h (the formulation the
// kernels run) on the host.  stdin: lines "lo hi scale precision" (lo / hi the unscaled value's 64-bit halves as
// unsigned decimals); stdout per line: "<double bits hex> <xxh64 hex> <DataType class>".
#include <cinttypes>
#include <cstdio>

#include "dq_decimal.h"

#define DQ_DEC_TABLE static const
#include "dq_dec_tables.inc"

int main() {
  const dq::DecTab t{kDecP10Lo, kDecP10Hi, kDecRcpHi, kDecRcpLo};
  unsigned long long lo, hi;
  int s, p;
  while (std::scanf("%llu %llu %d %d", &lo, &hi, &s, &p) == 4) {
    const double d = dq::dec_to_double(lo, hi, s, t, p <= 18);  // (the kernels pass narrow for precision <= 18)
    std::printf("%016" PRIx64 " %016" PRIx64 " %d\n", dq::dec_bits(d), dq::dec_hash(lo, hi, p),
                dq::dec_dt_class(lo, hi, s, t));
  }
  return 0;
}
