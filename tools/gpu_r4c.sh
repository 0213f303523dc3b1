#!/bin/bash
# Host-path variants of the driver's 20-sweep step (median of 5 each): end-of-launch wait by
# hipStreamSynchronize / hipEventQuery spin / hipEventSynchronize, with and without the timing events.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; : > gpurun_out/r4c_host.jsonl
for T in 1 0; do for S in 0 1 2; do
  CLV_SYNC=$S TIMING=$T LABEL="sync$S-timing$T" timeout -k 10 120 python tools/driver_breakdown.py \
    >> gpurun_out/r4c_host.jsonl 2> gpurun_out/r4c_host.err || exit $?
done; done
grep median gpurun_out/r4c_host.jsonl
