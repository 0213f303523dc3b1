#!/bin/bash
# Round 3: the statistics unit size at c4 / c5 on the shipped kernels, two passes each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
STEPS=1000 bash tools/gpu_bpu.sh "8 16 8 16" c4 || exit $?
STEPS=1000 bash tools/gpu_bpu.sh "16 32 16 32" c5
