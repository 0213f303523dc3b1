#!/bin/bash
# Round 3 (session 3): GPU suite + smoke at HEAD, then the round profile of c2 / c4 / c5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
bash tools/gpu_profile_round.sh c2 c4 c5 || exit $?
STEPS=5000 bash tools/gpu_libab.sh "default build/pack/libclvmcmc.so" c2 c4 c5
