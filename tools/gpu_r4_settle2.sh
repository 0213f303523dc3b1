#!/bin/bash
# Clock-settle length sweep on the driver's command (--steps 20 --warmup 5).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/settle2.jsonl; : > $O
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-c1-leg --scaling-configs="
for ms in 100 300 1000 0 100 300 1000; do
  timeout -k 10 180 $B --clock-settle-ms $ms > gpurun_out/settle_run.log 2> gpurun_out/settle_run.err; rc=$?
  echo "rc=$rc settle=$ms"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/settle_run.log >> $O
done
