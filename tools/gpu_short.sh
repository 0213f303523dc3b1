#!/bin/bash
# Short-run behaviour of the default bench (the driver's --steps 20 --warmup 5): per-sweep kernel time
# vs warm-up length and timed length.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for cfg in "20 5" "20 2000" "200 5" "2000 5" "20 5"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --scaling-configs "" ${BENCH_ARGS} > gpurun_out/short_$1_$2.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo rc=$rc; tail -5 gpurun_out/short_$1_$2.log; exit $rc; }
  python - gpurun_out/short_$1_$2.log $1 $2 <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l["roofline"]
print(f"steps {sys.argv[2]:>5s} warmup {sys.argv[3]:>5s}: {l['ms_per_step']*1e3:7.2f} us/step, kernel {r['sweep_kernel_us']:.2f} us/sweep, launch {r['launch_us']:.1f} us")
PY
done
