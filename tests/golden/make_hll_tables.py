"""Extract the HLL++ precision-9 interpolation data (RAW_ESTIMATE_DATA[5], BIAS_DATA[5]).

These are the published empirical HLL++ bias-correction points (Heule et al. 2013,
appendix), which the reference carries as data in
src/main/scala/com/amazon/deequ/analyzers/catalyst/HLLConstants.scala:51 and :84
(p = 9 because RELATIVE_SD = 0.05, StatefulHyperloglogPlus.scala:155-157).
This script reads that file as text (numbers only) and writes hll_p9_tables.json,
which is committed so the GPU box does not need /root/reference.
"""
import json
import os
import re
import sys

SRC = "/root/reference/src/main/scala/com/amazon/deequ/analyzers/catalyst/HLLConstants.scala"


def arrays_after(text, name):
    start = text.index(f"val {name}")
    block = text[start:]
    rows = re.findall(r"Array\(([^()]*)\)", block)
    return [[float(x) for x in r.split(",")] for r in rows[:15]]


def main():
    text = open(SRC).read()
    raw = arrays_after(text, "RAW_ESTIMATE_DATA")
    bias = arrays_after(text, "BIAS_DATA")
    out = {"source": "HLLConstants.scala:51 (RAW_ESTIMATE_DATA(5)), :84 (BIAS_DATA(5))",
           "raw_estimate_p9": raw[5], "bias_p9": bias[5]}
    assert len(out["raw_estimate_p9"]) == len(out["bias_p9"])
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hll_p9_tables.json")
    with open(dst, "w") as f:
        json.dump(out, f)
    print(dst, len(raw[5]))


if __name__ == "__main__":
    sys.exit(main())
