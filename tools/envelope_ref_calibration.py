"""Calibration of the G3 envelope test (tests/test_gpu_statistics.py) — TEST INFRASTRUCTURE.

Runs further independent 16-chain ensembles of the bitwise-pinned reference restatement
(oracle/ref_cpu.py) and scores them against the committed fixture with the test's own statistics:
the fraction of customers within 4 sigma and the mean per-customer z.  What the reference scores
against itself is the bar the GPU sampler's ensembles can be held to.

Usage: python tools/envelope_ref_calibration.py c1_bi_k1 2000,3000 [M]
       python tools/envelope_ref_calibration.py full_bi_k2 5000 [M]   (c2 at 1000 + 1000 sweeps)
"""
import os
import sys
from multiprocessing import Pool

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.helpers import cdnow, golden  # noqa: E402
from tests.test_gpu_statistics import SD_FLOOR  # noqa: E402


def _chain(args):
    name, seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import ref_cpu as orc
    f = golden(f"envelope_{name}.npz")
    covs = [str(c) for c in f["covariates"]]
    fn = orc.mcmc_draw_parameters if str(f["kind"]) == "bi" else orc.mcmc_draw_parameters_rfm_m
    data = str(f["data"]) if "data" in f.files else "abe"
    d = fn(cdnow(data), covs, mcmc=int(f["mcmc"]), burnin=int(f["burnin"]), thin=1, chains=1, seed=seed, trace=0)
    l1 = d["level_1"][0]
    st = dict(log_lambda=np.log(l1[:, :, 0]).mean(0), log_mu=np.log(l1[:, :, 1]).mean(0),
              p_alive=l1[:, :, 3].mean(0), lam=l1[:, :, 0].mean(0))
    if l1.shape[2] == 5:
        st["log_eta"] = np.log(l1[:, :, 4]).mean(0)
    return st


def main():
    name = sys.argv[1]
    bases = [int(s) for s in sys.argv[2].split(",")]
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    f = golden(f"envelope_{name}.npz")
    M_ref = int(f["M"])
    with Pool(8) as pool:
        res = pool.map(_chain, [(name, b + m) for b in bases for m in range(M)])
    for i, b in enumerate(bases):
        rs = res[i * M:(i + 1) * M]
        row = []
        for k in rs[0]:
            v = np.stack([r[k] for r in rs])
            m_g, s_g = v.mean(0), v.std(0, ddof=1)
            se = np.sqrt(np.maximum(f[k + "_sd"], SD_FLOOR[k]) ** 2 / M_ref + np.maximum(s_g, SD_FLOOR[k]) ** 2 / M)
            z = (m_g - f[k + "_mean"]) / se
            pop_r, pop_g = f[k + "_chains"], v.mean(1)
            zp = (pop_g.mean() - pop_r.mean()) / np.sqrt(pop_r.var(ddof=1) / M_ref + pop_g.var(ddof=1) / M)
            row.append(f"{k}: {np.mean(np.abs(z) <= 4.0):.4f} centred {np.mean(np.abs(z - z.mean()) <= 4.0):.4f} "
                       f"(mean z {z.mean():+.2f}, pop z {zp:+.2f})")
        print(name, "reference seeds", b, "..", b + M - 1, " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
