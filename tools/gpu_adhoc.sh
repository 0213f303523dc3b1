# Scratch GPU session script (overwritten per experiment).
# Round 6: the persistent level-2 workgroup polls one element per block partial until it arrives (in-tree)
# vs the whole record every poll (build/noflag = -DCLV_L2_FLAG_POLL=0): bitwise tests, then wall us
# per sweep of c4's 8-rank shard, c2 and c1 (persistent), alternating, two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/mcmc_clv_model_amd/libclvmcmc.so; B=$PWD/build/noflag/libclvmcmc.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_p2p.py -x -q -k "persistent or sharded or p2p or resume or full_size or deferred or determinism" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { tail -30 gpurun_out/c_tests.log; exit 1; }
tail -1 gpurun_out/c_tests.log
for rep in 1 2; do for lib in $B $L; do
  for W in c4_shard8 c2 c1 c3; do
    CLV_LIB_PATH=$lib timeout -k 10 300 python tools/persist_breakdown.py $W 3000 > gpurun_out/c_wall.txt 2>&1 || { tail -5 gpurun_out/c_wall.txt; exit 1; }
    echo $W $(basename $(dirname $lib)) $(grep "wall:" gpurun_out/c_wall.txt | cut -d'(' -f1)
  done
done; done
