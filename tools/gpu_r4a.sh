#!/bin/bash
# Round-4 baseline at HEAD: the driver's command 3x and the step breakdown (host / sync / kernel,
# cold vs clocks ramped).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
REPS=3 bash tools/gpu_driver_cmd.sh || exit $?
timeout -k 10 180 python tools/driver_breakdown.py > gpurun_out/r4a_breakdown.jsonl 2> gpurun_out/r4a_breakdown.err || exit $?
cat gpurun_out/r4a_breakdown.jsonl
