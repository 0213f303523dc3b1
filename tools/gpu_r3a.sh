#!/bin/bash
# Round 3, first GPU call: the GPU suite + smoke, then an A/B of cost-measurement library variants
# (tools/build_variant.sh) on c2 and c4.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
STEPS=3000 bash tools/gpu_libab.sh "default build/r6/libclvmcmc.so build/t3c/libclvmcmc.so build/pack/libclvmcmc.so" c2 c4
