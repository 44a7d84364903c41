// Host build of the kernels' XXH64 formulations (deequ_amd/csrc/dq_hash.h), driven by
// tests/test_hash_formulation.py against the golden vectors.  Reads "len hex" lines on stdin and
// prints the signed hash of fmix_tail(xxh64_short_head()) and of the split (deferred-round) form
// xxh64_short_head_split() for every byte alignment 0..3 of the string (lengths <= 28), fed as the UTF8 kernel
// feeds it: two aligned 16-byte loads realigned with alignbit, and garbage (0xA5) in the bytes past the
// string; with "W len hex" lines, fmix_tail(xxh64_upto63_head()) over a 64-byte window (lengths <= 63).
#include <cstdio>
#include <cstring>
#include <vector>

#include "../deequ_amd/csrc/dq_hash.h"

int main() {
  int len;
  char tag[8], hex[256];
  while (std::scanf("%7s %d %255s", tag, &len, hex) == 3) {
    unsigned char bytes[64] = {0};
    for (int i = 0; i < len; ++i) std::sscanf(hex + 2 * i, "%2hhx", &bytes[i]);
    if (tag[0] == 'W') {
      for (int align = 0; align < 4; ++align) {
        unsigned char buf[96];
        std::memset(buf, 0xA5, sizeof(buf));
        std::memcpy(buf + align, bytes, len);
        uint32_t d[17];
        std::memcpy(d, buf, 68);
        uint32_t w[16];
        for (int k = 0; k < 16; ++k) w[k] = dq::alignbit32(d[k + 1], d[k], align * 8u);
        const uint64_t h = dq::fmix_tail(dq::xxh64_upto63_head(w, (uint32_t)len, dq::MulP5{}));
        std::printf("%lld%c", (long long)h, align == 3 ? '\n' : ' ');
      }
      continue;
    }
    for (int align = 0; align < 4; ++align) {
      unsigned char buf[96];
      std::memset(buf, 0xA5, sizeof(buf));
      std::memcpy(buf + align, bytes, len);
      uint32_t d[8];
      std::memcpy(d, buf, 32);
      const uint32_t sh = align * 8u;
      uint32_t w[8];
      for (int k = 0; k < 7; ++k) w[k] = dq::alignbit32(d[k + 1], d[k], sh);
      w[7] = d[7];
      const uint64_t h = dq::fmix_tail(dq::xxh64_short_head(w, (uint32_t)len, dq::MulP5{}));
      const uint64_t hs = dq::fmix_tail(dq::xxh64_short_head_split(w, (uint32_t)len, dq::MulP5{}));
      std::printf("%lld %lld%c", (long long)h, (long long)hs, align == 3 ? '\n' : ' ');
    }
  }
  std::printf("LONG %lld INT %lld\n", (long long)dq::xxh64_long(42u), (long long)dq::xxh64_int(7u));
  return 0;
}
