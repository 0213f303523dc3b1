#!/bin/bash
# (Measured in round 4 before the producer / consumer hand-off was removed: its CLV_PC_CHUNKS arms and build/nopc refer to that code.)
# A/B: exponent-field scaling in exp_fast (build/scaletab) vs the in-tree library, two passes, at
# c2 / c4 / c5; then c2's producer / consumer chunks 0 vs 1 (CLV_PC_CHUNKS).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
STEPS=3000 bash tools/gpu_libab.sh "default build/scaletab/libclvmcmc.so default build/scaletab/libclvmcmc.so" c2 c4 c5 || exit $?
STEPS=5000 bash tools/gpu_ab.sh CLV_PC_CHUNKS "0 1 0 1" c2 || exit $?
