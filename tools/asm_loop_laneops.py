"""SGPR-spill lane traffic (v_readlane / v_writelane) per loop of one kernel in a hipcc
--cuda-device-only -S dump: for each natural loop (back edge target .. source, in layout order) the
instructions and lane ops it holds.  Usage: python tools/asm_loop_laneops.py kernels.s <mangled-name>"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    name = sys.argv[2]
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    order, size, lane, edges, blk = ["entry"], {}, {}, [], "entry"
    for line in s[i:j].splitlines():
        m = re.match(r"^(\.LBB\w+):", line)
        if m:
            blk = m.group(1)
            order.append(blk)
            continue
        t = line.strip()
        if not t or t.startswith((";", ".")):
            continue
        size[blk] = size.get(blk, 0) + 1
        if "readlane" in t or "writelane" in t:
            lane[blk] = lane.get(blk, 0) + 1
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", t)
        if m and m.group(1) in order:
            edges.append((order.index(m.group(1)), order.index(blk)))
    outer = sorted({(a, b) for a, b in edges if not any(a2 <= a and b <= b2 and (a2, b2) != (a, b) for a2, b2 in edges)})
    print(f"kernel total: {sum(size.values())} instructions, {sum(lane.values())} lane ops")
    for a, b in outer:
        blks = order[a:b + 1]
        print(f"loop {order[a]}..{order[b]}: {sum(size.get(x, 0) for x in blks)} instructions, "
              f"{sum(lane.get(x, 0) for x in blks)} lane ops")


if __name__ == "__main__":
    main()
