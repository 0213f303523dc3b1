#!/bin/bash
# Round 3: c2 A/B — in-tree library vs the fresh-kernarg variant (build/fresh), and the opt-in
# producer / consumer split at 1 and 2 chunks; each twice, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  STEPS=5000 bash tools/gpu_libab.sh "default build/fresh/libclvmcmc.so" c2 || exit $?
  STEPS=5000 bash tools/gpu_envab.sh "CLV_PC_CHUNKS=1 CLV_PC_CHUNKS=2" c2 || exit $?
done
