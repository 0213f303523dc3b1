#!/bin/bash
# A/B of environment settings on short bench runs:  tools/gpu_envab.sh "CLV_WG_MAP=0 CLV_WG_MAP=1" c3
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
ENVS=$1; shift
for W in "$@"; do
  for E in $ENVS; do
    env ${E//,/ } timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --scaling-configs= --no-c1-leg --steps ${STEPS:-5000} \
      --warmup 300 --timing-steps 500 > gpurun_out/eab_${W}_${E}.log 2>&1; rc=$?
    echo ${W} ${E} rc=$rc; python - "gpurun_out/eab_${W}_${E}.log" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=l["roofline"] or {}
print(f"  us/step={l['ms_per_step']*1e3:.2f} kernel_us={r.get('sweep_kernel_us')}")
PY
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
