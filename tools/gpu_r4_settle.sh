#!/bin/bash
# The driver's command (--steps 20 --warmup 5) with and without the clock-settle phase, 3 runs each,
# then the full default command once.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/settle.jsonl; : > $O
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-c1-leg --scaling-configs="
for i in 1 2 3; do
  for ms in 25 0; do
    timeout -k 10 180 $B --clock-settle-ms $ms > gpurun_out/settle_run.log 2> gpurun_out/settle_run.err; rc=$?
    echo "rc=$rc settle=$ms"; [ $rc -eq 0 ] || exit $rc
    tail -1 gpurun_out/settle_run.log >> $O
  done
done
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/settle_default.log 2> gpurun_out/settle_default.err; rc=$?
echo "default rc=$rc"; exit $rc
