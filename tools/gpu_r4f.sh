#!/bin/bash
# Round 4, second batch: parity suite at the restructured sweep-kernel stores; c4 / c5 burn-in and
# stored phases (default bench, no CPU leg); persistent vs launch-per-sweep crossover.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4f_bench_default.log 2>&1 || exit $?
python - gpurun_out/r4f_bench_default.log <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k,v in (l.get("configs") or {}).items():
    print(k, round(v["ms_per_step"]*1e3,2), "stored" in v and round(v["stored"]["ms_per_step"]*1e3,2))
PY
timeout -k 10 300 python tools/persist_crossover.py > gpurun_out/r4f_crossover.jsonl 2> gpurun_out/r4f_crossover.err || exit $?
cat gpurun_out/r4f_crossover.jsonl
