#!/bin/bash
# Round 3: GPU suite + smoke at the new defaults, then c3 / c1 A/B of the fresh-kernarg persistent
# kernel (in-tree) vs build/nofresh.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
STEPS=5000 bash tools/gpu_libab.sh "default build/nofresh/libclvmcmc.so default build/nofresh/libclvmcmc.so" c3 c2
