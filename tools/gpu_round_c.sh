#!/bin/bash
# Persistent-kernel parity test, default bench line, round profiles, c2 sweep timeline.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider -k "persistent" > gpurun_out/pytest_persist.log 2>&1; rc=$?
echo pytest_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_persist.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo bench_rc=$rc; tail -1 gpurun_out/bench_default.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile_round.sh c2 c3 c4 c5 || exit $?
CLV_LIB_PATH=$R/mcmc_clv_model_amd/libclvmcmc_stamps.so timeout -k 10 120 python tools/persist_breakdown.py c2 > gpurun_out/persist_c2.log 2>&1; echo stamps_rc=$?; tail -12 gpurun_out/persist_c2.log
exit 0
