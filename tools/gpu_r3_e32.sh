#!/bin/bash
# A/B of the 32-entry exp table (CLV_EXP32=1, build/e32): its accuracy test, then c2 / c4 / c5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CLV_LIB_PATH=$R/build/e32/libclvmcmc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "fast_exp_accuracy or mh_step_matches" > gpurun_out/e32_tests.log 2>&1; echo e32_tests_rc=$?; tail -3 gpurun_out/e32_tests.log
STEPS=5000 bash tools/gpu_libab.sh "default build/e32/libclvmcmc.so default build/e32/libclvmcmc.so" c2 || exit $?
STEPS=1000 bash tools/gpu_libab.sh "default build/e32/libclvmcmc.so" c4 c5
