#!/bin/bash
# GPU tests, then A/B of the in-tree library against build/base on c2/c3 (persistent kernel).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit $rc
STEPS=5000 bash tools/gpu_libab.sh "build/base/libclvmcmc.so default build/base/libclvmcmc.so default" c2 c3
