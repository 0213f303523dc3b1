# Scratch GPU session script (overwritten per experiment).
# Round 6: rocprofv3 --kernel-trace --stats of the driver's exact bench command (N = 1).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
D=$GRAFT_REPO_ROOT/gpurun_out/prof_driver; mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $D/prof_trace.log 2>&1; rc=$?
echo driver_trace_rc=$rc; tail -c 300 $D/prof_trace.log
