// jit_check.cpp -- host harness for tests/test_pred_jit_source.py: generates the compiled predicate pass's
// source (deequ_amd/csrc/dq_pred_jit.cpp) for a few programs and compiles each with hipRTC for gfx950, as
// dq_plan_create does -- without loading it (no GPU needed).  Usage: jit_check OUTDIR; prints one line per
// program: "<name> <eligible> <compile rc (0 ok)> <code bytes>" and writes OUTDIR/<name>.co.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "dq_pred_jit.h"

using namespace dq;

namespace {

PredInstr cmp(int col, int op, long long lit, int kind, int colb = -1, int nr = NR_NULL, int ctype = CT_INT) {
  PredInstr i{};
  i.op = PO_ATOM_CMP;
  i.cmp = op;
  i.ctype = ctype;
  i.null_res = nr;
  i.col_a = col;
  i.col_b = colb;
  i.kind_a = kind;
  i.kind_b = colb >= 0 ? kind : 0;
  i.lit_i = lit;
  i.lit_d = (double)lit;
  return i;
}
PredInstr op(int o, int slot = 0) {
  PredInstr i{};
  i.op = o;
  i.slot = slot;
  i.col_a = i.col_b = -1;
  return i;
}
PredInstr isnull(int col) {
  PredInstr i{};
  i.op = PO_ATOM_ISNULL;
  i.col_a = col;
  i.col_b = -1;
  return i;
}

PredProgram make(const std::vector<PredInstr>& code, int n_roots, int n_counters, int n_bitmaps) {
  PredProgram p;
  std::memset(&p, 0, sizeof p);
  p.n_instr = (int32_t)code.size();
  for (size_t i = 0; i < code.size(); ++i) p.instr[i] = code[i];
  for (int i = 0; i < p.n_instr; ++i)
    if (p.instr[i].op == PO_ATOM_CMP || p.instr[i].op == PO_ATOM_ISNULL || p.instr[i].op == PO_ATOM_NOTNULL)
      p.load_instr[p.n_loads++] = (int16_t)i;
  p.n_roots = n_roots;
  p.n_counters = n_counters;
  for (int c = 0; c < n_counters; ++c) p.counters[c] = PredCounter{c, -1};
  p.n_bitmaps = n_bitmaps;
  for (int b = 0; b < n_bitmaps; ++b) p.bitmap_root[b] = b;
  p.stack_depth = 4;
  return p;
}

int run(const char* outdir, const char* name, const PredProgram& prog, const int32_t* kinds, int ncols,
        const std::vector<PredJitHll>& hll) {
  const bool eligible = pred_jit_eligible(prog, kinds, ncols);
  std::vector<int32_t> slots;
  const std::string src = eligible ? pred_jit_source(prog, kinds, slots, hll) : std::string();
  int rc = -1;
  size_t bytes = 0;
  if (!src.empty()) {
    std::vector<char> code;
    std::string err;
    rc = pred_jit_compile_code(src, "gfx950", code, err) ? 0 : 1;
    if (rc != 0) {
      std::fprintf(stderr, "%s: %s\n", name, err.c_str());
    } else {
      bytes = code.size();
      const std::string path = std::string(outdir) + "/" + name + ".co";
      if (FILE* f = std::fopen(path.c_str(), "wb")) {
        std::fwrite(code.data(), 1, bytes, f);
        std::fclose(f);
      }
    }
  }
  std::printf("%s %d %d %zu\n", name, eligible ? 1 : 0, rc, bytes);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const char* outdir = argc > 1 ? argv[1] : ".";
  // C3's four Compliance predicates over i0..i3, with the four HLL-only tasks of those columns
  {
    std::vector<PredInstr> code = {cmp(0, C_GE, 0, CK_I64), op(PO_STORE, 0), isnull(1),
                                   cmp(1, C_GE, 10, CK_I64), cmp(1, C_LE, 1000, CK_I64), op(PO_AND), op(PO_OR),
                                   op(PO_STORE, 1), cmp(2, C_LT, 0, CK_I64, 3), op(PO_STORE, 2)};
    code.push_back(cmp(3, C_GE, 0, CK_I64, -1, NR_TRUE, CT_DBL));
    code.push_back(op(PO_STORE, 3));
    const int32_t kinds[4] = {CK_I64, CK_I64, CK_I64, CK_I64};
    run(outdir, "c3", make(code, 4, 4, 0), kinds, 4, {{0}, {1}, {2}, {3}});
  }
  // fp64 / int32 atoms, NOT, a `where` bitmap, no fused HLL
  {
    std::vector<PredInstr> code = {cmp(0, C_GT, 3, CK_F64, -1, NR_NULL, CT_DBL), op(PO_NOT), op(PO_STORE, 0),
                                   cmp(1, C_NE, 7, CK_I32), cmp(0, C_LT, 1, CK_F64, -1, NR_FALSE, CT_DBL),
                                   op(PO_OR), op(PO_STORE, 1)};
    const int32_t kinds[2] = {CK_F64, CK_I32};
    run(outdir, "mixed", make(code, 2, 2, 1), kinds, 2, {});
  }
  // FloatType / ShortType / ByteType atoms (round 6): 4- / 2- / 1-byte loads, float widened to double
  {
    std::vector<PredInstr> code = {cmp(0, C_GE, 16777216, CK_F32, -1, NR_NULL, CT_DBL), op(PO_STORE, 0),
                                   cmp(1, C_LT, -100, CK_I16), cmp(2, C_NE, 0, CK_I8, -1, NR_TRUE), op(PO_AND),
                                   op(PO_STORE, 1)};
    PredInstr mix = cmp(2, C_LT, 0, CK_I8, 1, NR_NULL, CT_INT);  // i8 vs i16 column
    mix.kind_b = CK_I16;
    code.push_back(mix);
    code.push_back(op(PO_STORE, 2));
    const int32_t kinds[3] = {CK_F32, CK_I16, CK_I8};
    run(outdir, "narrow", make(code, 3, 3, 0), kinds, 3, {});
  }
  // a string column in the program: not eligible (the interpreter runs it)
  {
    std::vector<PredInstr> code = {isnull(0), op(PO_STORE, 0)};
    const int32_t kinds[1] = {CK_UTF8};
    run(outdir, "string", make(code, 1, 1, 0), kinds, 1, {});
  }
  return 0;
}
