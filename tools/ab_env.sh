#!/bin/bash
# A/B of environment settings on short bench lines (primary workload only):
#   WL="c2 c3" STEPS=5000 REPS=2 tools/ab_env.sh "" "CLV_X=1" "CLV_X=1 CLV_Y=2"
# prints workload, settings, kernel us per sweep (events), wall us per step.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for E in "$@"; do
    for W in ${WL:-c2}; do
      env $E timeout -k 10 120 python bench.py --workload $W --steps ${STEPS:-5000} --warmup 200 --no-cpu-baseline \
        --scaling-configs= --no-c1-leg --no-stored-phase --no-whole-run > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
      python - "$W" "$E" <<'PY'
import json, sys
l = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
print(sys.argv[1], repr(sys.argv[2]), round(l["roofline"]["sweep_kernel_us"], 3), round(l["ms_per_step"] * 1e3, 3), flush=True)
PY
    done
  done
done
