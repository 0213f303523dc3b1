# Scratch GPU session script (overwritten per experiment).
# Round 6: the new full-size c4-shard persistent-vs-launch bitwise test.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "c4_eight_rank_shard" -p no:cacheprovider --timeout 200 --timeout-method thread 2>&1 | tail -5
