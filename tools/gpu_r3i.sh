#!/bin/bash
# Round 3: A/B of the packed t3 transform / exec-masked MH accept (in-tree = both) on c2, c4, c5,
# then the stamp timelines of the producer/consumer split.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
STEPS=5000 bash tools/gpu_libab.sh "build/base/libclvmcmc.so default build/masked/libclvmcmc.so build/packed/libclvmcmc.so build/base/libclvmcmc.so default" c2 || exit $?
STEPS=1000 bash tools/gpu_libab.sh "build/base/libclvmcmc.so default" c4 c5 || exit $?
bash tools/gpu_pcstamps.sh
