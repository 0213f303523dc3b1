"""Per-kernel VGPR / spill / scratch / occupancy table from a hipcc -Rpass-analysis=kernel-resource-usage log.

Usage: hipcc ... -Rpass-analysis=kernel-resource-usage -c kernels.hip 2> ru.log
       python tools/resource_usage.py ru.log [substring ...]
"""
import re
import subprocess
import sys


def parse(path):
    rows, cur = {}, None
    for line in open(path):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+([\w \[\]/]+): (\S+) \[", line)
        if m and cur:
            rows[cur][m.group(1).strip()] = m.group(2)
    return rows


def main():
    rows = parse(sys.argv[1])
    keys = sys.argv[2:]
    print(f"{'kernel':58s} {'VGPR':>5s} {'spill':>6s} {'scr/B':>6s} {'SGPRsp':>7s} {'occ':>4s}")
    for k, v in rows.items():
        dm = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
        dm = dm.split("(")[0]
        if keys and not any(s in dm for s in keys):
            continue
        print(f"{dm:58s} {v.get('VGPRs', '?'):>5s} {v.get('VGPRs Spill', '?'):>6s} "
              f"{v.get('ScratchSize [bytes/lane]', '?'):>6s} {v.get('SGPRs Spill', '?'):>7s} "
              f"{v.get('Occupancy [waves/SIMD]', '?'):>4s}")


if __name__ == "__main__":
    main()
