#!/bin/bash
# Round 3: c2 — same-chain producer / consumer dealing (build/early: fresh kernargs, producers
# first), 0-3 chunks per consumer, twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export CLV_LIB_PATH=$R/build/early/libclvmcmc.so
for rep in 1 2; do
  STEPS=5000 bash tools/gpu_envab.sh "CLV_PC_CHUNKS=0 CLV_PC_CHUNKS=1 CLV_PC_CHUNKS=2 CLV_PC_CHUNKS=3 CLV_PC_CHUNKS=2,CLV_PC_LOAD=250" c2 || exit $?
done
