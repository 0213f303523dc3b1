#!/bin/bash
# Round-4 baseline at HEAD: the driver's command 3x, the step breakdown (host / sync / kernel,
# cold vs clocks ramped), the default bench without the CPU leg (c4 / c5 burn-in + stored phases).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
REPS=3 bash tools/gpu_driver_cmd.sh || exit $?
timeout -k 10 180 python tools/driver_breakdown.py > gpurun_out/r4a_breakdown.jsonl 2> gpurun_out/r4a_breakdown.err || exit $?
cat gpurun_out/r4a_breakdown.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4a_bench_default.log 2>&1 || exit $?
tail -c 3000 gpurun_out/r4a_bench_default.log
