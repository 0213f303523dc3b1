#!/bin/bash
# Bench lines for every workload on one GPU (+ the sharded/RCCL path forced at world size 1).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for W in c1 c3 c4 c5; do
  timeout -k 10 600 python bench.py --workload $W "$@" > gpurun_out/bench_$W.log 2>&1; rc=$?; echo bench_${W}_rc=$rc; tail -1 gpurun_out/bench_$W.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --workload c2 --force-sharded --no-cpu-baseline --steps 3000 --warmup 300 > gpurun_out/bench_c2_sharded.log 2>&1; rc=$?; echo bench_c2_sharded_rc=$rc; tail -3 gpurun_out/bench_c2_sharded.log
exit $rc
