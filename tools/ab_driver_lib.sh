#!/bin/bash
# The driver's bench command (--gpus 1 --steps 20 --warmup 5) A/B: the shipped library against a
# variant build (tools/build_variant.sh), alternating, REPS times each:
#   REPS=3 tools/ab_driver_lib.sh build/NAME/libclvmcmc.so
# prints label, wall us per step, kernel us per sweep.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for i in $(seq ${REPS:-3}); do
  for V in shipped "$1"; do
    if [ "$V" = shipped ]; then unset CLV_LIB_PATH; else export CLV_LIB_PATH=$V; fi
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_ab.log 2>&1 || { tail -5 gpurun_out/drv_ab.log; exit 1; }
    python - "$V" <<'PY'
import json, sys
l = json.loads(open("gpurun_out/drv_ab.log").read().strip().splitlines()[-1])
print(sys.argv[1], round(l["ms_per_step"] * 1e3, 3), l["roofline"]["sweep_kernel_us"], flush=True)
PY
  done
done
