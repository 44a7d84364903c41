"""Static VALU / VMEM / LDS / SALU instruction counts of the loops of each kernel in a hipcc
--save-temps .s file (diagnostic).  Usage: python tools/isa_loops.py file.s [name-filter]"""
import collections
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\w+):.*$", text, re.M):
        name = m.group(1)
        end = text.find(".Lfunc_end", m.end())
        if end > 0 and "s_endpgm" in text[m.end():end]:
            yield name, text[m.end():end]


def loops(body):
    lines = [l.split(";")[0].strip() for l in body.split("\n")]
    lines = [l for l in lines if l and not l.startswith(".") or (l.startswith(".LBB") and l.endswith(":"))]
    labels = {l[:-1]: i for i, l in enumerate(lines) if l.endswith(":")}
    for i, l in enumerate(lines):
        m = re.match(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                seg = [x for x in lines[labels[tgt]:i + 1] if not x.endswith(":")]
                yield tgt, seg


def classify(seg):
    c = collections.Counter()
    ops = collections.Counter()
    for l in seg:
        op = l.split()[0]
        ops[op] += 1
        if op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith(("buffer_", "global_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c, ops


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, body in kernels(text):
        if filt not in name:
            continue
        print(name)
        for tgt, seg in loops(body):
            c, ops = classify(seg)
            if c["valu"] < 20:
                continue
            print(f"  loop {tgt}: {dict(c)}")
            print("    " + ", ".join(f"{k}:{v}" for k, v in ops.most_common(24)))
