#!/bin/bash
# A/B of the statistics unit size (blocks per unit) on the launch-per-sweep workloads:
#   tools/gpu_bpu.sh "8 16 32 64" c4
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
BPUS=$1; shift
for W in "$@"; do
  for B in $BPUS; do
    timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --scaling-configs= --no-c1-leg --steps ${STEPS:-1000} \
      --warmup 200 --timing-steps 500 --blocks-per-unit $B > gpurun_out/bpu_${W}_${B}.log 2>&1; rc=$?
    echo ${W} bpu=${B} rc=$rc; python - "gpurun_out/bpu_${W}_${B}.log" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=l["roofline"] or {}
print(f"  us/step={l['ms_per_step']*1e3:.2f} kernel_us={r.get('sweep_kernel_us')}")
PY
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
