#!/bin/bash
# Round-4 profiles at the final sources: rocprofv3 kernel trace + calibrated PMC passes of c2, c4,
# c5 (burn-in) and c4 / c5 in the stored phase (bench.py --phase stored).  Summaries on the CPU
# side: tools/summarize_profile.py r04_<w>_... --prof gpurun_out/prof_<w> --calib gpurun_out/prof_calib
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_profile_round.sh ${PROFILE_SET:-c2 c4 c5 c4stored c5stored}
