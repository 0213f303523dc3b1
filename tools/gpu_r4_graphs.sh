#!/bin/bash
# Verdict r3 #4: the RCCL fallback path (ShardedSampler, world size 1 via --force-sharded) at the
# driver's 20-sweep step, graph-replayed (--graph-chunk 32: 16 + 4 sweep graphs) against eager
# (--graph-chunk 0), and at 2,000 sweeps.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/graphs.jsonl; : > $O
B="python3 bench.py --force-sharded --no-cpu-baseline --no-c1-leg --scaling-configs="
for args in "--steps 20 --warmup 5 --graph-chunk 32" "--steps 20 --warmup 5 --graph-chunk 0" \
            "--steps 2000 --warmup 100 --graph-chunk 32" "--steps 2000 --warmup 100 --graph-chunk 0"; do
  timeout -k 10 240 $B $args > gpurun_out/graphs_step.log 2> gpurun_out/graphs_step.err; rc=$?
  echo "rc=$rc $args"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/graphs_step.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['args']='$args'; print(json.dumps(d))" >> $O
done
exit 0
