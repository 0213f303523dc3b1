#!/bin/bash
# The driver's bench command (--steps 20 --warmup 5) several times: per-step and kernel time.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for i in $(seq ${REPS:-3}); do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --scaling-configs= ${BENCH_ARGS} > gpurun_out/d$i.log 2>&1 || exit 1
  python - gpurun_out/d$i.log <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{l['ms_per_step']*1e3:.2f} us/step, kernel {l['roofline']['sweep_kernel_us']} us/sweep")
PY
done
