#!/bin/bash
# Fixed cost of one persistent launch at c2: the timed launch's duration (HIP events) at several
# sweep counts; the intercept of duration vs sweeps is the launch's prologue/epilogue cost, the
# slope the steady-state sweep.  Lines into gpurun_out/intercept.jsonl.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; : > gpurun_out/intercept.jsonl
for N in 1 2 5 20 100 1000; do
  timeout -k 10 120 python bench.py --gpus 1 --steps $N --warmup 5 --no-cpu-baseline --scaling-configs= \
    >> gpurun_out/intercept.jsonl 2> gpurun_out/intercept_$N.err; rc=$?
  echo steps_${N}_rc=$rc
  [ $rc -eq 0 ] || exit $rc
done
exit 0
