#!/bin/bash
# Round profile of the bench workloads given as arguments (default c2): per workload
#  1. rocprofv3 --kernel-trace --stats of the bench command (c2: exactly the default command);
#  2. separate PMC passes (FETCH_SIZE / WRITE_SIZE / VALU+wave counters), each its own run, of the
#     sampler alone (tools/pmc_run.py): one persistent dispatch of the whole 20,000-sweep workload,
#     or 100 sweep launches;
# then the FETCH/WRITE calibration kernels (tools/calib_fetch) once.  Summaries are formed on the
# CPU side afterwards (tools/summarize_profile.py --prof gpurun_out/prof_<W> ...).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
[ $# -gt 0 ] || set -- c2
for W in "$@"; do
  D=$R/gpurun_out/prof_$W; mkdir -p $D
  # "<w>stored": workload <w> with every sweep a stored sweep (bench.py --phase stored)
  WL=${W%stored}; PH=burnin; [ "$WL" != "$W" ] && PH=stored
  case $WL in
    c2|c3|c1) TR="--steps 19000 --warmup 5"; PS=20000 ;;  # PMC: the whole 20,000-sweep workload, one dispatch
    c4_shard8) TR="--steps 9000 --warmup 5"; PS=10000 ;;  # (persistent since round 6: its 10,000-sweep run)
    *)        TR="--steps 2000 --warmup 200 --timing-steps 500"; PS=100 ;;
  esac
  B="python3 $R/bench.py --workload $WL --phase $PH --no-cpu-baseline --scaling-configs= --no-c1-leg --no-stored-phase --no-whole-run"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $B $TR > $D/prof_trace.log 2>&1; rc=$?
  echo ${W}_trace_rc=$rc; tail -1 $D/prof_trace.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
  for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    tag=$(echo $P | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    # the sampler alone (tools/pmc_run.py): one persistent dispatch of PS sweeps, or PS sweep launches
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d $D/$tag -o run --output-format csv -- python3 $R/tools/pmc_run.py $W 0 $PS > $D/prof_$tag.log 2>&1; rc=$?
    echo ${W}_${tag}_rc=$rc
    [ $rc -eq 0 ] || exit $rc
  done
done
if [ ! -x tools/calib_fetch ]; then echo "tools/calib_fetch missing (build it on the CPU side)"; exit 0; fi
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/prof_calib/calib_$P -o run --output-format csv -- $R/tools/calib_fetch > gpurun_out/prof_calib_$P.log 2>&1; rc=$?; echo calib_${P}_rc=$rc
  [ $rc -eq 0 ] || exit $rc
done
exit 0
