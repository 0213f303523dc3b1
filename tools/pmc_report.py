"""Per wave-sweep averages of the counters tools/gpu_pmc_stalls.sh collected (its reduced pass files
gpurun_out/pmc_<W>/p*.txt), optionally beside an earlier report of the same format.

    python3 tools/pmc_report.py c2 250 [profiles/r03_c2_pmc_stalls.txt]

250 = sweeps over the two dispatches (50 warm-up + 200).  SQ cycle counters are in quad-cycles.
"""
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = sys.argv[1] if len(sys.argv) > 1 else "c2"
sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 250
base_path = sys.argv[3] if len(sys.argv) > 3 else None

tot, head = {}, []
for path in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{W}", "p*.txt"))):
    for line in open(path):
        if line.startswith("#"):
            head.append(line[1:].strip())
            continue
        k, v = line.split()
        tot[k] = float(v)
base = {}
if base_path:
    for line in open(base_path):
        f = line.split()
        if len(f) >= 6 and f[1] == "total" and f[3] == "per":
            base[f[0]] = float(f[5])

n_disp = int(head[0].split(":")[1].split()[0]) if head else 2
waves = tot.get("SQ_WAVES", 1.0) / n_disp  # waves per dispatch
den = waves * sweeps
print(f"# tools/gpu_pmc_stalls.sh {W} (4 separate --pmc passes, kernel-trace only; tools/pmc_run.py: {n_disp}"
      f" dispatches, {sweeps} sweeps, {waves:,.0f} waves each); per wave and sweep; SQ cycle counters in"
      " quad-cycles" + (f"; last column: {os.path.basename(base_path)}" if base_path else ""))
for k in sorted(tot):
    pw = tot[k] / den if k != "SQ_WAVES" else 0.0
    line = f"{k:26s} total {tot[k]:12.5g}   per wave-sweep {pw:10.1f}"
    if k in base and k != "SQ_WAVES":
        d = pw - base[k]
        line += f"   was {base[k]:10.1f} ({d:+.1f}, {100 * d / base[k]:+.1f}%)" if base[k] else f"   was {base[k]:10.1f}"
    print(line)


def r(a, b):
    return tot.get(a, 0.0) / tot[b] if tot.get(b) else float("nan")


print(f"wait_any / wave_cycles {r('SQ_WAIT_ANY', 'SQ_WAVE_CYCLES'):.3f}; active_valu / wave_cycles "
      f"{r('SQ_ACTIVE_INST_VALU', 'SQ_WAVE_CYCLES'):.3f}; lds_bank_conflict / active_lds "
      f"{r('SQ_LDS_BANK_CONFLICT', 'SQ_ACTIVE_INST_LDS'):.3f}")
