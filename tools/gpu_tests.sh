#!/bin/bash
# GPU parity tests + smoke on the box; test failures (rc 1) do not stop later steps, crashes do.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest_rc=$rc; grep -E "passed|failed|FAILED|bit-identical" gpurun_out/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo smoke_rc=$rc; tail -2 gpurun_out/smoke.log
[ $rc -le 1 ] || exit $rc
exit 0
