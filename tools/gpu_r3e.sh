#!/bin/bash
# Round 3: c2 — producers drawing the consumers' chunks before their own next-sweep work
# (build/early) vs after (build/fresh), twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  CLV_LIB_PATH=$R/build/fresh/libclvmcmc.so STEPS=5000 bash tools/gpu_envab.sh "CLV_PC_CHUNKS=0 CLV_PC_CHUNKS=1" c2 || exit $?
  CLV_LIB_PATH=$R/build/early/libclvmcmc.so STEPS=5000 bash tools/gpu_envab.sh "CLV_PC_CHUNKS=1 CLV_PC_CHUNKS=2 CLV_PC_CHUNKS=3" c2 || exit $?
done
