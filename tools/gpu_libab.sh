#!/bin/bash
# A/B of library variants (tools/build_variant.sh) on short bench runs:
#   tools/gpu_libab.sh "default build/mb4/libclvmcmc.so ..." c4 c5
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
LIBS=$1; shift
for W in "$@"; do
  for L in $LIBS; do
    tag=$(echo $L | tr '/' '_')
    if [ "$L" = "default" ]; then unset CLV_LIB_PATH; else export CLV_LIB_PATH=$R/$L; fi
    timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --scaling-configs "" --no-c1-leg --steps ${STEPS:-2000} --warmup 200 \
      --timing-steps 500 > gpurun_out/lab_${W}_${tag}.log 2>&1; rc=$?
    echo ${W} ${L} rc=$rc; python - "gpurun_out/lab_${W}_${tag}.log" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=l["roofline"] or {}
print(f"  value={l['value']:.4e} us/step={l['ms_per_step']*1e3:.2f} kernel_us={r.get('sweep_kernel_us')} frac={r.get('frac')}")
PY
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
