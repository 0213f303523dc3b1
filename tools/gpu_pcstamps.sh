#!/bin/bash
# Stamp timelines of c2's persistent kernel by placement (shared CU vs alone) at CLV_PC_CHUNKS 0/1/2.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for N in 0 1 2; do
  CLV_PC_CHUNKS=$N timeout -k 10 240 python tools/persist_breakdown.py c2 1500 > gpurun_out/pcstamps_$N.log 2>&1; rc=$?
  echo pc=$N rc=$rc; grep -v "^/opt" gpurun_out/pcstamps_$N.log | head -40
  [ $rc -eq 0 ] || exit $rc
done
