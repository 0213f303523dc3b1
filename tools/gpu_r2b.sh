timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit $rc
bash tools/gpu_libab.sh "default build/mb4/libclvmcmc.so build/mb4np/libclvmcmc.so" c4 c5
