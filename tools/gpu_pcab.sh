#!/bin/bash
# A/B of the producer/consumer split at c2: "LIB:CHUNKS ..." (LIB = default or a build/ variant),
# CLV_PC_CHUNKS per arm, STEPS sweeps (default 5000) per bench run.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
W=${W:-c2}
for A in $1; do
  L=${A%%:*}; N=${A##*:}; tag=$(echo $L | tr '/' '_')_pc$N
  if [ "$L" = "default" ]; then unset CLV_LIB_PATH; else export CLV_LIB_PATH=$R/$L; fi
  CLV_PC_CHUNKS=$N timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --scaling-configs "" --no-c1-leg \
    --steps ${STEPS:-5000} --warmup 200 > gpurun_out/pcab_${W}_${tag}.log 2>&1; rc=$?
  echo $W $L pc=$N rc=$rc; python - "gpurun_out/pcab_${W}_${tag}.log" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=l["roofline"] or {}
print(f"  value={l['value']:.4e} us/step={l['ms_per_step']*1e3:.3f} kernel_us={r.get('sweep_kernel_us')}")
PY
  [ $rc -eq 0 ] || exit $rc
done
exit 0
