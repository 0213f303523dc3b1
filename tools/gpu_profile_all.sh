#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes for several workloads (shorter runs for the big ones).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
for W in "$@"; do
  mkdir -p gpurun_out/prof_$W
  B="python3 $R/bench.py --workload $W --no-cpu-baseline --timing-steps 300"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$W/trace -o run --output-format csv -- $B --steps 1000 --warmup 200 > gpurun_out/prof_${W}_trace.log 2>&1; rc=$?; echo ${W}_trace_rc=$rc
  [ $rc -eq 0 ] || exit $rc
  for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    tag=$(echo $P | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -k 10 600 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/prof_$W/$tag -o run --output-format csv -- $B --steps 100 --warmup 20 > gpurun_out/prof_${W}_$tag.log 2>&1; rc=$?; echo ${W}_${tag}_rc=$rc
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
