#!/bin/bash
# Round profile of the default bench workload: rocprofv3 kernel-trace stats, PMC passes
# (FETCH_SIZE, WRITE_SIZE, VALU counters — separate passes), and the FETCH/WRITE calibration
# kernels (tools/calib_fetch.hip) for the 4/8-B-per-lane access widths.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
W=${WORKLOAD:-c2}
B="python3 $R/bench.py --workload $W --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/trace -o run --output-format csv -- $B --steps 19000 --warmup 1000 > gpurun_out/prof_trace.log 2>&1; rc=$?; echo trace_rc=$rc; tail -1 gpurun_out/prof_trace.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  tag=$(echo $P | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/prof/$tag -o run --output-format csv -- $B --steps 300 --warmup 50 > gpurun_out/prof_$tag.log 2>&1; rc=$?; echo ${tag}_rc=$rc
  [ $rc -eq 0 ] || exit $rc
done
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/prof/calib_$P -o run --output-format csv -- $R/tools/calib_fetch > gpurun_out/prof_calib_$P.log 2>&1; rc=$?; echo calib_${P}_rc=$rc
  [ $rc -eq 0 ] || exit $rc
done
exit 0
