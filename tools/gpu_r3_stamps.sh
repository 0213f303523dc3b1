#!/bin/bash
# c2 persistent-kernel timeline at the final kernels (stamps build), and the shipped library's wall time.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 240 python tools/persist_breakdown.py c2 1500 > gpurun_out/r3_stamps_c2.log 2>&1; rc=$?
echo rc=$rc; grep -v "^/opt" gpurun_out/r3_stamps_c2.log | head -60
