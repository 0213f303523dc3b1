#!/bin/bash
# A/B of an environment knob on short bench runs: tools/gpu_ab.sh VAR "v1 v2" c2 c3 ...
# (TESTS=1 first runs the persistent/p2p parity tests.)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
VAR=$1; VALS=$2; shift 2
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_p2p.py \
    tests/test_gpu_parity.py -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_ab.log 2>&1; rc=$?
  echo pytest_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_ab.log | tail -15
  [ $rc -eq 0 ] || exit $rc
fi
for W in "$@"; do
  for V in $VALS; do
    env $VAR=$V timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --scaling-configs "" --steps ${STEPS:-5000} --warmup 300 \
      --timing-steps 1000 > gpurun_out/ab_${W}_${V}.log 2>&1; rc=$?
    echo ${W}_${VAR}=${V}_rc=$rc; python - "gpurun_out/ab_${W}_${V}.log" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=l["roofline"] or {}
print(f"  value={l['value']:.4e} us/step={l['ms_per_step']*1e3:.2f} kernel_us={r.get('sweep_kernel_us')} frac={r.get('frac')}")
PY
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
