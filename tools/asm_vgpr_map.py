"""Per basic block of one kernel in a hipcc -S dump: instruction count, highest VGPR index used and
scratch ops — shows which code region sets the kernel's register allocation.
Usage: python tools/asm_vgpr_map.py kernels.s <mangled-kernel-name> [min_vgpr]"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    name = sys.argv[2]
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    blk, rows = "entry", {"entry": [0, -1, 0, []]}
    order = ["entry"]
    for line in s[i:j].splitlines():
        m = re.match(r"^(\.LBB\w+):", line)
        if m:
            blk = m.group(1)
            order.append(blk)
            rows[blk] = [0, -1, 0, []]
            continue
        t = line.strip()
        if not t or t.startswith((";", ".")):
            continue
        r = rows[blk]
        r[0] += 1
        idx = [int(x) for x in re.findall(r"\bv\[\d+:(\d+)\]", t)] + [int(x) for x in re.findall(r"\bv(\d+)\b", t)]
        if idx:
            r[1] = max(r[1], max(idx))
        if "scratch_" in t:
            r[2] += 1
        op = t.split()[0]
        if len(r[3]) < 4 and op in ("s_sleep", "s_memrealtime", "v_permlane32_swap_b32", "s_setprio", "v_exp_f32",
                                     "v_cos_f32", "v_mad_u64_u32", "ds_read_b64", "global_store_dwordx2"):
            r[3].append(op)
    for b in order:
        n, mx, sc, tags = rows[b]
        if mx >= lo:
            print(f"{b:14s} insts {n:5d} maxV {mx:4d} scratch {sc:3d} {' '.join(sorted(set(tags)))}")


if __name__ == "__main__":
    main()
