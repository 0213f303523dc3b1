"""Where a kernel spills: scratch loads/stores per basic block of a hipcc --cuda-device-only -S dump,
with each block's instruction count.  Usage: python tools/asm_spills.py kernels.s <mangled-kernel-name>"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    name = sys.argv[2]
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j].splitlines()
    blk, order, counts, sizes = "entry", ["entry"], {}, {}
    for line in body:
        m = re.match(r"^(\.LBB\w+):", line)
        if m:
            blk = m.group(1)
            order.append(blk)
            continue
        if line.startswith("\t") and not line.strip().startswith((";", ".")):
            sizes[blk] = sizes.get(blk, 0) + 1
        if "scratch_" in line:
            c = counts.setdefault(blk, [0, 0])
            c[0 if "load" in line else 1] += 1
    tot = [sum(v[0] for v in counts.values()), sum(v[1] for v in counts.values())]
    print(f"{name}: {len(body)} lines, scratch loads {tot[0]} stores {tot[1]}")
    for b in order:
        if b in counts:
            print(f"  {b:16s} insts {sizes.get(b, 0):6d}  scratch load {counts[b][0]:4d} store {counts[b][1]:4d}")


if __name__ == "__main__":
    main()
