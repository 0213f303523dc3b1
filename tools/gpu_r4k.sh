#!/bin/bash
# Round 4 at the final kernels: GPU suite, the driver's command 3x, the default bench without the
# CPU legs (c4 / c5 burn-in + stored phases), then the round's profiles.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider -rf \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -8
[ $rc -eq 0 ] || exit $rc
REPS=3 bash tools/gpu_driver_cmd.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4k_bench_default.log 2>&1 || exit $?
python - gpurun_out/r4k_bench_default.log <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c2", round(l["ms_per_step"]*1e3,3), l["roofline"]["sweep_kernel_us"])
for k,v in (l.get("configs") or {}).items():
    print(k, round(v["ms_per_step"]*1e3,2), "stored" in v and round(v["stored"]["ms_per_step"]*1e3,2))
PY
bash tools/gpu_r4_profile.sh
