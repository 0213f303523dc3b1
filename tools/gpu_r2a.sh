#!/bin/bash
# Round-2 check on the box: GPU tests + smoke, the driver's exact bench command, and a kernel +
# HIP-API trace of that command (where the fixed per-clv_run cost goes).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider -rA --timeout 300 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo pytest_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -15
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench20.log 2>&1; rc=$?
echo bench20_rc=$rc; tail -c 1500 gpurun_out/bench20.log; echo
[ $rc -eq 0 ] || exit $rc
if [ "${TRACE:-1}" = "1" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/r2_trace20 -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --scaling-configs "" > gpurun_out/r2_trace20.log 2>&1; rc=$?
echo trace_rc=$rc
fi
exit $rc
