#!/bin/bash
# c4 / c5 launch-per-sweep timeline (stamps build): customer phase, tail split.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for w in c4 c5; do
  timeout -k 10 240 python tools/stamp_breakdown.py $w 300 > gpurun_out/tail_$w.log 2>&1; rc=$?
  echo "$w rc=$rc"; grep -v "^/opt" gpurun_out/tail_$w.log | head -40; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 240 python tools/persist_breakdown.py c2 1500 > gpurun_out/r4_c2_persist_timeline.txt 2>&1; rc=$?
echo "c2 persist rc=$rc"; grep -v "^/opt" gpurun_out/r4_c2_persist_timeline.txt | head -30; exit $rc
