#!/bin/bash
# Is the driver step's excess over steady state the GPU clock ramp or the sampler's cold caches?
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
timeout -k 10 300 env CASES=cold,after_long,after_busy,long_then_idle REPS=5 python3 tools/driver_breakdown.py > gpurun_out/ramp.jsonl 2> gpurun_out/ramp.err; rc=$?
echo rc=$rc; grep median gpurun_out/ramp.jsonl; exit $rc
