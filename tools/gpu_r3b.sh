#!/bin/bash
# Round 3 (resumed): GPU suite + smoke, then A/B of the round-3 knobs: c2 producer/consumer
# split (CLV_PC_CHUNKS), c4/c5 stride kernel on/off (CLV_STRIDE).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
STEPS=3000 bash tools/gpu_envab.sh "CLV_PC_CHUNKS=0 CLV_PC_CHUNKS=3" c2 || exit $?
STEPS=1000 bash tools/gpu_envab.sh "CLV_STRIDE=0 CLV_STRIDE=1" c4 || exit $?
STEPS=1000 bash tools/gpu_envab.sh "CLV_STRIDE=0 CLV_STRIDE=1" c5
