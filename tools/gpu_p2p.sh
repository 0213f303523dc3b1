#!/bin/bash
# Peer-exchange (world size > 1 persistent kernel) tests, then the persistent/sharded parity tests,
# then the whole GPU suite; stops at the first crash or time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_p2p.py \
  -p no:cacheprovider > gpurun_out/pytest_p2p.log 2>&1; rc=$?
echo p2p_rc=$rc; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pytest_p2p.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider -rA \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest_rc=$rc; grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -20
exit $rc
