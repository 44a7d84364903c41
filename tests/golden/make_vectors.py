"""Write hash_vectors.json: XXH64 (seed 42) golden vectors from the independent `xxhash`
package (3.8.1), in the three forms Spark's XxHash64Function uses (StatefulHyperloglogPlus.scala:93):
hashLong (8 LE bytes of the long / doubleToLongBits of a double), hashInt (4 LE bytes) and
hashUnsafeBytes (UTF-8 bytes).  Also JVM quirk cases for the HLL estimate (:222)."""
import json
import os
import struct

import xxhash


def s64(x):
    return x - (1 << 64) if x >> 63 else x


def main():
    longs = [0, 1, -1, 42, 123456789, -987654321, (1 << 63) - 1, -(1 << 63), 10000, 999999999999]
    ints = [0, 1, -1, 7, 2147483647, -2147483648, 100000]
    doubles = [0.0, -0.0, 1.0, -1.0, 1.5, 3.141592653589793, 1e300, -1e-300,
               float("inf"), float("-inf"), float("nan"), 1000.123456]
    out = {"seed": 42, "long": [], "int": [], "double": [], "bytes": []}
    for v in longs:
        out["long"].append([v, s64(xxhash.xxh64_intdigest(struct.pack("<q", v), seed=42))])
    for v in ints:
        out["int"].append([v, s64(xxhash.xxh64_intdigest(struct.pack("<i", v), seed=42))])
    for v in doubles:
        bits = 0x7FF8000000000000 if v != v else struct.unpack("<q", struct.pack("<d", v))[0]
        out["double"].append([repr(v), bits, s64(xxhash.xxh64_intdigest(struct.pack("<q", bits), seed=42))])
    base = "héllo wörld, the quick brown fox jumps over the lazy dog 0123456789"
    for n in list(range(0, 41)) + [63, 64, 65, 100]:
        b = (base * 3).encode("utf-8")[:n]
        out["bytes"].append([b.hex(), s64(xxhash.xxh64_intdigest(b, seed=42))])
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hash_vectors.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=0)
    print(dst)


if __name__ == "__main__":
    main()
