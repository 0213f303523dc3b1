#!/bin/bash
# A/B arms "LIB@ENV=V,ENV=V ..." (LIB: default or a build/ variant; ENV part optional) on workload W
# (default c2), STEPS sweeps each (default 5000).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
W=${W:-c2}
for A in $1; do
  L=${A%%@*}; E=""; [ "$A" != "$L" ] && E=${A#*@}
  tag=$(echo "$A" | tr '/@,=' '____')
  if [ "$L" = "default" ]; then unset CLV_LIB_PATH; else export CLV_LIB_PATH=$R/$L; fi
  env $(echo $E | tr ',' ' ') timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --scaling-configs "" --no-c1-leg \
    --steps ${STEPS:-5000} --warmup 200 --timing-steps 500 > gpurun_out/eab_${W}_${tag}.log 2>&1; rc=$?
  echo "$W $A rc=$rc"; python - "gpurun_out/eab_${W}_${tag}.log" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=l["roofline"] or {}
print(f"  value={l['value']:.4e} us/step={l['ms_per_step']*1e3:.3f} kernel_us={r.get('sweep_kernel_us')}")
PY
  [ $rc -eq 0 ] || exit $rc
done
exit 0
