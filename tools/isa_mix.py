"""Instruction mix of one kernel in a hipcc ``--save-temps`` gfx950 assembly file, per basic block.

Usage: python tools/isa_mix.py <file.s> <kernel-substring> [--blocks]
Prints the whole-kernel opcode histogram (top 40) and, with --blocks, each basic block's size
and its MFMA / VALU / LDS / VMEM / SALU counts (hot loops are the blocks with the MFMAs)."""
import collections
import re
import sys


def kernel_lines(path, key):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start + 1:end]


def klass(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    path, key = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, key)
    ops = collections.Counter()
    blocks = []
    cur = ["entry", collections.Counter()]
    for l in body:
        t = l.strip()
        if re.match(r"^\.LBB\S*:", t):
            blocks.append(cur)
            cur = [t.split(":")[0], collections.Counter()]
            continue
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        ops[op] += 1
        cur[1][klass(op)] += 1
        cur[1]["_" + op] += 1
    blocks.append(cur)
    print("total", sum(ops.values()))
    for op, c in ops.most_common(40):
        print(f"{c:5d} {op}")
    if "--blocks" in sys.argv:
        for name, c in blocks:
            n = sum(v for k, v in c.items() if not k.startswith("_"))
            print(f"{name:12s} n={n:4d} mfma={c['mfma']:3d} valu={c['valu']:4d} lds={c['lds']:3d} "
                  f"vmem={c['vmem']:3d} salu={c['salu']:3d}")
            if c["mfma"]:
                top = sorted(((v, k[1:]) for k, v in c.items() if k.startswith("_v_")), reverse=True)[:14]
                print("      " + ", ".join(f"{k}:{v}" for v, k in top))


if __name__ == "__main__":
    main()
