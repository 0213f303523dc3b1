# Scratch GPU session script (overwritten per experiment; the round-6 diagnostics ran from it).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/mcmc_clv_model_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_parity.py -x -q -k "p2p or persistent or resume or sharded or clock" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { tail -30 gpurun_out/c_tests.log; exit 1; }
tail -2 gpurun_out/c_tests.log
for rep in 1 2; do for lib in $PWD/build/head/libclvmcmc.so $L/libclvmcmc.so; do
  CLV_LIB_PATH=$lib timeout -k 10 300 python tools/fx_ab.py 3 9 300000 2 300 2>&1 | grep "^{" || exit 1
  CLV_LIB_PATH=$lib timeout -k 10 300 python tools/fx_ab.py 2 5 250000 2 300 2>&1 | grep "^{" || exit 1
  CLV_PERSISTENT=1 CLV_LIB_PATH=$lib timeout -k 10 300 python tools/persist_breakdown.py c4_shard8 3000 > gpurun_out/c_wall.txt 2>&1 || exit 1
  echo c4_shard8 $lib $(tail -1 gpurun_out/c_wall.txt)
done; done
