"""Reduce one rocprofv3 --pmc pass (tools/gpu_pmc_stalls.sh) to per-counter totals over the
dispatches of one kernel, so the raw per-dispatch CSVs need not travel back from the GPU box.

    python3 tools/pmc_reduce.py <pass dir> <kernel substring>   ->  <pass dir>.txt
"""
import csv
import glob
import os
import sys

d, kern = sys.argv[1], sys.argv[2]
tot, disp = {}, set()
for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        if kern not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        disp.add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
with open(d.rstrip("/") + ".txt", "w") as f:
    f.write(f"# {kern}: {len(disp)} dispatches\n")
    for k in sorted(tot):
        f.write(f"{k} {tot[k]:.6g}\n")
print(open(d.rstrip("/") + ".txt").read())
