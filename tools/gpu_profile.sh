#!/bin/bash
# rocprofv3: kernel-trace stats of a bench run, then separate PMC passes (FETCH_SIZE, WRITE_SIZE,
# VALU/wave counters) — never combined with sys/runtime traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
W=${WORKLOAD:-c2}
B="python3 $R/bench.py --workload $W --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/trace -o run --output-format csv -- $B --steps 4000 --warmup 400 > gpurun_out/prof_trace.log 2>&1; rc=$?; echo trace_rc=$rc; tail -1 gpurun_out/prof_trace.log
[ $rc -eq 0 ] || exit $rc
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  tag=$(echo $P | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/prof/$tag -o run --output-format csv -- $B --steps 300 --warmup 50 > gpurun_out/prof_$tag.log 2>&1; rc=$?; echo ${tag}_rc=$rc
  [ $rc -eq 0 ] || exit $rc
done
exit 0
