#!/bin/bash
# Round 3: the GPU suite + smoke, then A/B runs: c2 with the MH-variate producer / consumer split
# (CLV_PC_CHUNKS) and the packed-variate / Philox-round library variants; c4 and c5 with the
# stride kernel on / off (CLV_STRIDE); c3 with the placement map + split.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
STEPS=3000 bash tools/gpu_envab.sh "CLV_PC_CHUNKS=0 CLV_PC_CHUNKS=2 CLV_PC_CHUNKS=3 CLV_PC_CHUNKS=1" c2 || exit $?
STEPS=1000 bash tools/gpu_envab.sh "CLV_STRIDE=0 CLV_STRIDE=1" c4 || exit $?
STEPS=1000 bash tools/gpu_envab.sh "CLV_STRIDE=0 CLV_STRIDE=1" c5 || exit $?
STEPS=3000 bash tools/gpu_libab.sh "build/pack/libclvmcmc.so build/r6/libclvmcmc.so" c2 || exit $?
STEPS=3000 bash tools/gpu_envab.sh "CLV_WG_MAP=0 CLV_WG_MAP=1" c3
