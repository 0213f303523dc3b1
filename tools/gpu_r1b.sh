#!/bin/bash
# Sharded path check (eager vs torch.cuda graph incl. RCCL all-gather) + the new sharded tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -k "sharded" -rA > gpurun_out/pytest_sharded.log 2>&1; rc=$?
echo pytest_sharded_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_sharded.log | tail -12
[ $rc -le 1 ] || exit $rc
for GC in 32 0; do
  timeout -k 10 300 python bench.py --workload c2 --force-sharded --no-cpu-baseline --steps 3200 --warmup 320 --graph-chunk $GC > gpurun_out/b_sh_$GC.log 2>&1; rc=$?
  echo sharded_gc${GC}_rc=$rc; tail -1 gpurun_out/b_sh_$GC.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
exit 0
