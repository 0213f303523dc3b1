#!/bin/bash
# Short-launch timeline (stamps build; built here before the GPU steps).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 180 python tools/launch_timeline.py > gpurun_out/r4d_timeline.jsonl 2> gpurun_out/r4d_timeline.err || exit $?
cat gpurun_out/r4d_timeline.jsonl
