"""Diagnostic: the G3 envelope statistics (tests/test_gpu_statistics.py) for several ensemble seeds:
fraction of customers within 4 sigma per statistic, and the worst |z|."""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.test_gpu_statistics import SD_FLOOR, _run_envelope  # noqa: E402

for name in sys.argv[1].split(","):
    for seed in [int(s) for s in sys.argv[2].split(",")]:
        f, g, d = _run_envelope(name, seed=seed)
        M_ref = int(f["M"])
        row = []
        for k, v in g.items():
            M = v.shape[0]
            m_g, s_g = v.mean(0), v.std(0, ddof=1)
            m_r, s_r = f[k + "_mean"], f[k + "_sd"]
            se = np.sqrt(np.maximum(s_r, SD_FLOOR[k]) ** 2 / M_ref + np.maximum(s_g, SD_FLOOR[k]) ** 2 / M)
            z = (m_g - m_r) / se
            pop_r, pop_g = f[k + "_chains"], v.mean(1)
            zp = (pop_g.mean() - pop_r.mean()) / np.sqrt(pop_r.var(ddof=1) / M_ref + pop_g.var(ddof=1) / M)
            row.append(f"{k}: {np.mean(np.abs(z) <= 4.0):.4f} centred {np.mean(np.abs(z - z.mean()) <= 4.0):.4f} "
                       f"(mean z {z.mean():+.2f}, pop z {zp:+.2f})")
        print(name, seed, " | ".join(row), flush=True)
