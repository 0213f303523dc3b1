#!/bin/bash
# Driver-length bench with the timed launch's events from the dispatch (default) or recorded around it.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for i in 1 2 3; do
  for m in 0 1; do
    CLV_TIMING_RECORD=$m timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --scaling-configs "" > gpurun_out/tab_$m.log 2>&1 || exit 1
    python - gpurun_out/tab_$m.log $m <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l["roofline"] or {}
print(f"record={sys.argv[2]}: {l['ms_per_step']*1e3:7.2f} us/step, kernel {r.get('sweep_kernel_us')} us/sweep, launch {r.get('launch_us')} us")
PY
  done
done
