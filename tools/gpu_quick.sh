#!/bin/bash
# Quick perf check: GPU tests (optional, TESTS=1) then short bench lines for the given workloads.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider -rA ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo pytest_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -15
  [ $rc -le 1 ] || exit $rc
fi
for W in "$@"; do
  timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --scaling-configs "" --no-c1-leg --steps ${STEPS:-3000} --warmup 300 --timing-steps 1000 > gpurun_out/q_$W.log 2>&1; rc=$?
  echo ${W}_rc=$rc; python - "$W" <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/q_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r=l["roofline"] or {}
print(sys.argv[1], f"value={l['value']:.4e} ms/step={l['ms_per_step']*1e3:.2f}us kernel={r.get('sweep_kernel_us')}us frac={r.get('frac')}")
PY
  [ $rc -eq 0 ] || exit $rc
done
exit 0
