"""Scratch (private segment) use per kernel from a `hipcc --offload-device-only -S` dump: the frame
size the kernel descriptor reserves and the number of instructions in the kernel body that actually
read or write scratch (scratch_* / buffer_* through the private segment).

Usage: hipcc ... --offload-device-only -S kernels.hip -o k.s
       python tools/asm_scratch.py k.s [substring ...]
"""
import re
import subprocess
import sys


def main():
    s = open(sys.argv[1]).read()
    keys = sys.argv[2:]
    print(f"{'kernel':58s} {'scr/B':>6s} {'scratch instr':>14s}")
    for m in re.finditer(r"^\s*\.amdhsa_kernel (\S+)$", s, re.M):
        name = m.group(1)
        seg = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", s[m.end():m.end() + 400])
        start = s.find("\n" + name + ":")
        end = s.find(".Lfunc_end", start)
        body = s[start:end].splitlines()
        n = sum(1 for l in body if re.match(r"\s*(scratch_|buffer_(load|store))", l))
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        if keys and not any(k in dm for k in keys):
            continue
        print(f"{dm[:58]:58s} {int(seg.group(1)) if seg else -1:6d} {n:14d}")


if __name__ == "__main__":
    main()
