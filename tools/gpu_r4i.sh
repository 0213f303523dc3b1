#!/bin/bash
# Round 4: GPU suite at the deferred-draw sources, then the driver command and its breakdown, then
# the crossover / P/C / timing-record batch.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider -rf \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -8
[ $rc -eq 0 ] || exit $rc
REPS=3 bash tools/gpu_driver_cmd.sh || exit $?
timeout -k 10 180 python tools/driver_breakdown.py > gpurun_out/r4i_breakdown.jsonl 2> gpurun_out/r4i_breakdown.err || exit $?
grep median gpurun_out/r4i_breakdown.jsonl
CLV_DEFER=0 LABEL=nodefer timeout -k 10 180 python tools/driver_breakdown.py > gpurun_out/r4i_breakdown_nodefer.jsonl 2>&1 || exit $?
grep median gpurun_out/r4i_breakdown_nodefer.jsonl
bash tools/gpu_r4h.sh
