#!/bin/bash
# Driver-length bench (--steps 20 --warmup 5) under each CLV_SYNC wait mode, with and without the
# event-timed launch.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for m in 0 1 2 0 1 2; do
  for kt in "" "--no-kernel-timing"; do
    CLV_SYNC=$m timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --scaling-configs "" $kt > gpurun_out/sync_$m.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo rc=$rc; tail -5 gpurun_out/sync_$m.log; exit $rc; }
    python - gpurun_out/sync_$m.log "$m $kt" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l["roofline"] or {}
print(f"sync {sys.argv[2]:24s}: {l['ms_per_step']*1e3:7.2f} us/step, kernel {r.get('sweep_kernel_us')} us/sweep, launch {r.get('launch_us')} us")
PY
  done
done
