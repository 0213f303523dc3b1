R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest_rc=$rc; grep -E "passed|failed|FAILED|bit-identical" gpurun_out/pytest_gpu.log | tail -15
[ $rc -le 1 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/trace -o run --output-format csv -- python3 $R/bench.py --steps 4000 --warmup 400 --no-cpu-baseline > gpurun_out/prof_trace.log 2>&1; rc=$?; echo trace_rc=$rc; tail -2 gpurun_out/prof_trace.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/prof/fetch -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1; rc=$?; echo fetch_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/prof/write -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/prof_write.log 2>&1; rc=$?; echo write_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/prof/valu -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/prof_valu.log 2>&1; rc=$?; echo valu_rc=$rc
find gpurun_out/prof -name "*.csv" | head -20
