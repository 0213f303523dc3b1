#!/bin/bash
# Round-end evidence on one box: the default bench line (c2, 19,000 timed sweeps, CPU legs, c4/c5
# configurations), the driver's own command (--steps 20 --warmup 5), and the end-to-end drop-in
# fits next to the reference's published runtimes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo bench_default_rc=$rc
[ $rc -eq 0 ] || { tail -5 gpurun_out/bench_default.log; exit $rc; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1; rc=$?; echo bench_driver_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/e2e_fits.py > gpurun_out/e2e.jsonl 2> gpurun_out/e2e.err; rc=$?; echo e2e_rc=$rc
exit $rc
