// dq_regex.h -- PatternMatch / RLIKE pattern -> byte-level search DFA (host compiler, dq_regex.cpp).
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/dqscan.h"

namespace dq {

// DFA states: 0 = dead, 1 = sticky accept (a match was found; patterns without a trailing `$`),
// 2.. = the rest.  A walk stops early in states 0 / 1; the row matches iff acc_end[final state].
struct RegexDfa {
  int n_states = 0, n_classes = 0, start = 0;
  bool end_anchored = false;
  uint8_t cls[256] = {0};              // byte -> equivalence class
  std::vector<uint8_t> acc_end;        // [n_states]
  std::vector<uint16_t> trans;         // [n_states][n_classes]
};

dq_status regex_compile(const char* pattern, int32_t mode, RegexDfa& out);
// device blob (uint16 words): n_states, n_classes, start, flags, cls[256], acc_end[ns], trans[ns*nc]
void regex_serialize(const RegexDfa& d, std::vector<uint16_t>& blob);
bool regex_run(const RegexDfa& d, const uint8_t* s, int64_t len);
constexpr int kRegexHeader = 4 + 256;

}  // namespace dq
