"""Per-wave averages of the counters collected by tools/gpu_pmc_stalls.sh for the sweep kernel."""
import csv
import glob
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = sys.argv[1] if len(sys.argv) > 1 else "c2"
vals = {}
for path in glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{W}", "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        if "sweep_kernel" not in r["Kernel_Name"]:
            continue
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
m = {k: statistics.mean(v) for k, v in vals.items()}
waves = m.get("SQ_WAVES", 1)
print(f"{W}: sweep_kernel dispatches averaged; waves/dispatch = {waves:.0f}")
for k in sorted(m):
    print(f"  {k:28s} {m[k]:14.1f}   per wave {m[k] / waves:10.1f}")
