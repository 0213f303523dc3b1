#!/bin/bash
# A/B: the chain's last unit stores its sums / draws after the level-2 draw (in-tree, bivariate)
# vs before it (build/earlystore), c4 in the stored phase (every sweep stores) and burn-in, 2 passes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for pass in 1 2; do for PH in stored burnin; do for L in default build/earlystore/libclvmcmc.so; do
  if [ "$L" = "default" ]; then unset CLV_LIB_PATH; else export CLV_LIB_PATH=$R/$L; fi
  timeout -k 10 120 python bench.py --workload c4 --phase $PH --no-cpu-baseline --scaling-configs "" --no-c1-leg \
    --steps 2000 --warmup 200 --timing-steps 500 > gpurun_out/r4j.log 2>&1 || exit $?
  python - gpurun_out/r4j.log "c4 $PH $L" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(l['ms_per_step']*1e3,3), l['roofline']['sweep_kernel_us'])
PY
done; done; done
unset CLV_LIB_PATH
# occupancy: c4's sweep_kernel_occ4<2,5> at 5 waves per SIMD (96 VGPRs, spills) vs 4
for pass in 1 2; do for L in default build/occ5/libclvmcmc.so; do
  if [ "$L" = "default" ]; then unset CLV_LIB_PATH; else export CLV_LIB_PATH=$R/$L; fi
  timeout -k 10 120 python bench.py --workload c4 --no-cpu-baseline --scaling-configs "" --no-c1-leg \
    --steps 2000 --warmup 200 --timing-steps 500 > gpurun_out/r4j.log 2>&1 || exit $?
  python - gpurun_out/r4j.log "c4 occ $L" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(l['ms_per_step']*1e3,3), l['roofline']['sweep_kernel_us'])
PY
done; done
unset CLV_LIB_PATH
