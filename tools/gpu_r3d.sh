#!/bin/bash
# Round 3: c2 producer / consumer load sweep on the fresh-kernarg variant (build/fresh), twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export CLV_LIB_PATH=$R/build/fresh/libclvmcmc.so
for rep in 1 2; do
  STEPS=5000 bash tools/gpu_envab.sh "CLV_PC_CHUNKS=0 CLV_PC_CHUNKS=1 CLV_PC_CHUNKS=2,CLV_PC_LOAD=200 CLV_PC_CHUNKS=2,CLV_PC_LOAD=230 CLV_PC_CHUNKS=3,CLV_PC_LOAD=200" c2 || exit $?
done
