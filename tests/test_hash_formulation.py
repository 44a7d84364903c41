"""The kernels' branch-free short-string XXH64 (deequ_amd/csrc/dq_hash.h), built for the host,
equals the golden vectors (independent `xxhash` package) for every length <= 28 and byte alignment,
both in one piece and split as the kernel runs a deferred 24..28-byte string; and the rare path's
64-byte-window form (xxh64_upto63_head) for every length <= 63."""
import os
import subprocess

from tests.conftest import ROOT


def test_short_string_formulation(tmp_path, hash_vectors):
    exe = tmp_path / "hash_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(ROOT, "tests", "hash_check.cpp")],
                   check=True)
    cases = [(len(bytes.fromhex(h)) if h else 0, h, v) for h, v in hash_vectors["bytes"]]
    cases = [c for c in cases if c[0] <= 28]
    inp = "".join(f"S {n} {h or '00'}\n" for n, h, _ in cases)
    out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    for (n, h, v), line in zip(cases, out):
        assert [int(x) for x in line.split()] == [v] * 8, (n, h)
    longs = dict((a, b) for a, b in hash_vectors["long"])
    ints = dict((a, b) for a, b in hash_vectors["int"])
    last = out[-1].split()
    assert int(last[1]) == longs[42] and int(last[3]) == ints[7]


def test_window63_formulation(tmp_path):
    """xxh64_upto63_head over a 64-byte window: every length 0..63 (one 32-byte stripe + merge from 32 on, then
    the short remainder), each byte alignment, garbage past the string -- against the `xxhash` package."""
    import numpy as np
    import xxhash

    exe = tmp_path / "hash_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(ROOT, "tests", "hash_check.cpp")],
                   check=True)
    rng = np.random.default_rng(63)
    vals = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in range(64) for _ in range(3)]
    inp = "".join(f"W {len(v)} {v.hex() or '00'}\n" for v in vals)
    out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    for v, line in zip(vals, out):
        want = xxhash.xxh64_intdigest(v, seed=42)
        want = want - (1 << 64) if want >= 1 << 63 else want
        assert [int(x) for x in line.split()] == [want] * 4, len(v)
