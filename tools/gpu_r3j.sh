#!/bin/bash
# Round 3: the deferred level-2 draw (launch per sweep) — its bitwise GPU tests, then A/B against
# the draw in the sweep's own tail (CLV_DEFER=0) on c4 / c5, and the unit size at c4 / c5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "deferred or persistent_kernel_bitwise or stride_kernel_bitwise" > gpurun_out/pytest_defer.log 2>&1; rc=$?
echo pytest_rc=$rc; tail -3 gpurun_out/pytest_defer.log
[ $rc -eq 0 ] || exit $rc
STEPS=${STEPS:-1000} bash tools/gpu_envab.sh "CLV_DEFER=0 CLV_DEFER=1 CLV_DEFER=0 CLV_DEFER=1" c4 c5 || exit $?
STEPS=1000 bash tools/gpu_bpu.sh "8 16" c4 || exit $?
STEPS=1000 bash tools/gpu_bpu.sh "16 32" c5
