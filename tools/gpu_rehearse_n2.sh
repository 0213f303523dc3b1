#!/bin/bash
# bench.py at world size 2 on the one-GPU box (both ranks on device 0, gloo group): the driver's
# N > 1 command path incl. the c4 / c5 configurations (peer exchange, fused exchange).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps ${STEPS:-20} --warmup 5 --one-gpu-rehearsal ${BENCH_ARGS} \
  > gpurun_out/rehearse_n2.log 2>&1; rc=$?
echo rc=$rc; grep -v Warning gpurun_out/rehearse_n2.log | tail -c 3000
exit $rc
