#!/bin/bash
# c2 HBM traffic of the persistent kernel with and without the MH-variate producer/consumer split
# (CLV_PC_CHUNKS 0 / 1): FETCH_SIZE and WRITE_SIZE passes over one 20,000-sweep dispatch each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp; mkdir -p gpurun_out
B="python3 $R/bench.py --workload c2 --no-cpu-baseline --scaling-configs= --no-c1-leg --warmup 0 --steps 20000 --no-kernel-timing"
for PC in 0 1; do
  for P in FETCH_SIZE WRITE_SIZE; do
    D=$R/gpurun_out/pct_${PC}_$P
    CLV_PC_CHUNKS=$PC timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d $D -o run --output-format csv -- $B > $D.log 2>&1; rc=$?
    echo pc=$PC $P rc=$rc
    [ $rc -eq 0 ] || exit $rc
  done
done
python3 - <<'PY'
import csv, glob
for pc in (0, 1):
    kb = {}
    for P in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"gpurun_out/pct_{pc}_{P}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == P and "persist_kernel" in r["Kernel_Name"]:
                    kb[P] = kb.get(P, 0.0) + float(r["Counter_Value"])
    f, w = kb.get("FETCH_SIZE", 0.0), kb.get("WRITE_SIZE", 0.0)
    print(f"pc={pc}: FETCH_SIZE {f:.0f} KB, WRITE_SIZE {w:.0f} KB; corrected (x2 read, x1 write) "
          f"{(2 * f + w) * 1024 / 20000 / 1e6:.3f} MB per sweep")
PY
