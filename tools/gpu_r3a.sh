#!/bin/bash
# Round 3: the GPU suite + smoke, then A/B runs: the MH-variate producer / consumer split
# (CLV_PC_CHUNKS) and cost-measurement library variants (tools/build_variant.sh, built before the
# split) on c2, and the variants on c4.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
STEPS=3000 bash tools/gpu_envab.sh "CLV_PC_CHUNKS=0 CLV_PC_CHUNKS=2 CLV_PC_CHUNKS=3 CLV_PC_CHUNKS=1" c2 || exit $?
STEPS=3000 bash tools/gpu_libab.sh "build/r6/libclvmcmc.so build/t3c/libclvmcmc.so build/pack/libclvmcmc.so" c2 || exit $?
STEPS=1000 bash tools/gpu_libab.sh "default build/r6/libclvmcmc.so build/t3c/libclvmcmc.so build/pack/libclvmcmc.so" c4
