"""The compiled predicate pass's generator (deequ_amd/csrc/dq_pred_jit.cpp) on the host: the kernel source it
writes for C3's four Compliance predicates (with the four fused HLL tasks) and for an fp64 / int32 program
with NOT and a `where` bitmap compiles with hipRTC for gfx950, as dq_plan_create does, into a code object
with no scratch and at most 128 VGPRs (4 waves per SIMD); a program over a string column is left to the
interpreter.  No GPU: the code objects are only inspected (GPU parity of the same kernels: test_gpu_parity)."""
import os
import re
import shutil
import subprocess

import pytest

from tests.conftest import ROOT

CSRC = os.path.join(ROOT, "deequ_amd", "csrc")
INC = os.path.join(ROOT, "deequ_amd", "build", "dq_hash_src.inc")
HIPCC = "/opt/rocm/bin/hipcc"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(READELF) and os.path.exists(INC)),
                    reason="needs hipcc, llvm-readelf and the built deequ_amd/build (run __graft_entry__.build())")
def test_generated_kernels_compile(tmp_path):
    exe = tmp_path / "jit_check"
    subprocess.run([HIPCC, "-std=c++17", "-O1", "-I", CSRC, "-I", os.path.dirname(INC), "-o", str(exe),
                    os.path.join(ROOT, "tests", "jit_check.cpp"), os.path.join(CSRC, "dq_pred_jit.cpp"), "-lhiprtc"],
                   check=True, capture_output=True)
    out = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, check=True, timeout=300)
    res = {line.split()[0]: [int(x) for x in line.split()[1:]] for line in out.stdout.splitlines()}
    assert res["string"][0] == 0, "a string column must stay on the interpreter"
    for name in ("c3", "mixed", "narrow"):
        eligible, rc, nbytes = res[name]
        assert eligible == 1 and rc == 0 and nbytes > 0, (name, res[name], out.stderr[-2000:])
        notes = subprocess.run([READELF, "--notes", str(tmp_path / f"{name}.co")], capture_output=True, text=True,
                               check=True).stdout
        assert ".name:           dq_pred_jit" in notes or re.search(r"\.name:\s+dq_pred_jit\b", notes)
        scratch = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", notes).group(1))
        vgprs = int(re.search(r"\.vgpr_count:\s+(\d+)", notes).group(1))
        assert scratch == 0, f"{name}: the generated kernel uses scratch ({scratch} bytes)"
        assert vgprs <= 128, f"{name}: {vgprs} VGPRs (< 4 waves per SIMD)"
    # the next block's loads stay in flight through the block: C3's kernel waits for a row group's own loads
    # with a good part of the next block still in flight (vmcnt >= 10 of its 36 loads per block), or drains everything
    # (vmcnt(0): the rare exact-rank redo, the exit) -- the shallow waits (vmcnt(6), (7), (8)) are what a
    # prologue issued out of the loop's order left at every block's start (the waitcnt pass merges the loop
    # header's entry states; round 4)
    objdump = os.path.join(os.path.dirname(READELF), "llvm-objdump")
    dis = subprocess.run([objdump, "-d", "--mcpu=gfx950", str(tmp_path / "c3.co")], capture_output=True, text=True,
                         check=True).stdout
    waits = [int(x) for x in re.findall(r"s_waitcnt vmcnt\((\d+)\)", dis)]
    assert waits and not [w for w in waits if 0 < w < 10], sorted(set(waits))
    shutil.rmtree(tmp_path, ignore_errors=True)
