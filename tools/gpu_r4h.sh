#!/bin/bash
# (Measured in round 4 before the producer / consumer hand-off was removed: its CLV_PC_CHUNKS arms and build/nopc refer to that code.)
# Round 4, third batch: persistent / launch crossover (second case set); c2 with the producer /
# consumer hand-off (chunks 1), without it (chunks 0) and compiled out (build/nopc), two passes;
# the driver step with the timed launch bracketed by hipEventRecord vs the dispatch's timestamps.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CROSSOVER_SET=2 timeout -k 10 400 python tools/persist_crossover.py > gpurun_out/r4h_crossover.jsonl 2> gpurun_out/r4h_crossover.err || exit $?
cat gpurun_out/r4h_crossover.jsonl
for pass in 1 2; do
  for V in "default:1" "default:0" "build/nopc/libclvmcmc.so:0"; do
    L=${V%%:*}; C=${V##*:}
    if [ "$L" = "default" ]; then unset CLV_LIB_PATH; else export CLV_LIB_PATH=$R/$L; fi
    CLV_PC_CHUNKS=$C timeout -k 10 120 python bench.py --no-cpu-baseline --scaling-configs "" --no-c1-leg --steps 5000 \
      --warmup 300 --timing-steps 1000 > gpurun_out/r4h_pc.log 2>&1 || exit $?
    python - gpurun_out/r4h_pc.log "$L chunks=$C" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(l['ms_per_step']*1e3,3), l['roofline']['sweep_kernel_us'])
PY
  done
done
unset CLV_LIB_PATH
for T in 1 0; do
  CLV_TIMING_RECORD=$T LABEL="record$T" timeout -k 10 120 python tools/driver_breakdown.py > gpurun_out/r4h_rec$T.jsonl 2>&1 || exit $?
  grep median gpurun_out/r4h_rec$T.jsonl
done
