#!/bin/bash
# The driver's command, twice (full line: c1 leg, CPU baseline, c4/c5 configs).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/default.jsonl; : > $O
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/default_run.log 2> gpurun_out/default_run.err; rc=$?
  echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/default_run.log >> $O
done
