#!/bin/bash
# Round 3 final measurements: GPU suite + smoke, the default bench line, the driver's command (3x),
# and the launch intercept at c2.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo bench_rc=$rc
[ $rc -eq 0 ] || exit $rc
tail -1 gpurun_out/bench_default.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['ms_per_step'], l['roofline']['sweep_kernel_us'], {k: round(v['ms_per_step']*1e3,2) for k,v in (l['configs'] or {}).items()})"
REPS=3 bash tools/gpu_driver_cmd.sh || exit $?
bash tools/gpu_launch_intercept.sh
