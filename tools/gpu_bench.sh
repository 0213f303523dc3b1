#!/bin/bash
# bench.py default line (event-timed launches) + the hipGraph-replay variant for comparison.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1; rc=$?; echo bench_rc=$rc; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline --no-kernel-timing "$@" > gpurun_out/bench_graph.log 2>&1; rc=$?; echo bench_graph_rc=$rc; tail -1 gpurun_out/bench_graph.log
exit $rc
