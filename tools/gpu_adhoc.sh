# Scratch GPU session script (overwritten per experiment).
# Round 6: sweep time of the c2 persistent kernel under the scratch sampler's settings (tools/settle_speed.py).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/settle_speed.py 2>&1 | grep -v amdgpu.ids
