#!/bin/bash
# One GPU session (gpurun) of named steps, each under a time limit of its own; the session stops at
# the first step that crashes or times out (pytest's rc 1 = test failures does not stop it).
#   tests      pytest -m gpu (-x, per-test timeout) and __graft_entry__.smoke()
#   driver     the driver's bench command (--gpus 1 --steps 20 --warmup 5)   -> gpurun_out/bench_driver.log
#   default    the default bench line (19,000 timed sweeps, CPU legs, configs) -> gpurun_out/bench_default.log
#   e2e        the drop-in fits end to end (tools/e2e_fits.py)                 -> gpurun_out/e2e.jsonl
#   rehearse   bench.py at world size 2 with both ranks on this GPU (gloo group; BENCH_ARGS appended)
#                                                                           -> gpurun_out/rehearse_n2.log
#   profile:W  rocprofv3 trace + PMC passes of workload W (tools/gpu_profile_round.sh W)
#   stalls:W   the stall / issue counters of workload W (tools/gpu_pmc_stalls.sh W)
#   stamps:W   one sweep's in-kernel timeline of workload W (diagnostic library libclvmcmc_stamps.so)
# Usage: tools/gpu_session.sh tests driver e2e
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider -rA --timeout 300 \
        --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
      echo tests_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -15
      [ $rc -le 1 ] || exit $rc
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      echo smoke_rc=$rc; tail -2 gpurun_out/smoke.log
      [ $rc -le 1 ] || exit $rc ;;
    driver)
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_driver.log 2>&1; rc=$?
      echo driver_rc=$rc; tail -c 600 gpurun_out/bench_driver.log
      [ $rc -eq 0 ] || exit $rc ;;
    default)
      timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_default.log 2>&1; rc=$?
      echo default_rc=$rc; tail -c 600 gpurun_out/bench_default.log
      [ $rc -eq 0 ] || exit $rc ;;
    e2e)
      timeout -k 10 600 python tools/e2e_fits.py > gpurun_out/e2e.jsonl 2> gpurun_out/e2e.err; rc=$?
      echo e2e_rc=$rc; cat gpurun_out/e2e.jsonl | cut -c1-300
      [ $rc -eq 0 ] || exit $rc ;;
    rehearse)
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 2 --steps ${STEPS:-20} --warmup 5 --one-gpu-rehearsal ${BENCH_ARGS} \
        > gpurun_out/rehearse_n2.log 2>&1; rc=$?
      echo rehearse_rc=$rc; grep -v Warning gpurun_out/rehearse_n2.log | tail -c 2500
      [ $rc -eq 0 ] || exit $rc ;;
    stamps:*)
      # the diagnostic library (make -C mcmc_clv_model_amd/csrc STAMPS=1): one sweep's timeline
      W=${step#stamps:}
      case $W in c4|c5) T=tools/stamp_breakdown.py ;; *) T=tools/persist_breakdown.py ;; esac
      timeout -k 10 300 python $T $W > gpurun_out/stamps_$W.txt 2>&1; rc=$?
      echo stamps_${W}_rc=$rc; tail -45 gpurun_out/stamps_$W.txt
      [ $rc -eq 0 ] || exit $rc ;;
    profile:*)
      bash tools/gpu_profile_round.sh ${step#profile:} || exit $? ;;
    stalls:*)
      bash tools/gpu_pmc_stalls.sh ${step#stalls:} || exit $? ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
