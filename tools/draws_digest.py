"""SHA-256 digests of short Philox-mode runs (tools only): run twice, once per library
(CLV_LIB_PATH=...), to check that an A/B build leaves every returned bit unchanged.
Cases: c2-shaped (bi, 1 covariate, persistent kernel) and c3-shaped (tri) on full CDNOW, and a
launch-per-sweep bivariate K = 5 run on synthetic data (150,000 customers x 2 chains: too many
workgroups for the persistent grid).
Usage: python tools/draws_digest.py"""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mcmc_clv_model_amd import mcmc_draw_parameters, mcmc_draw_parameters_rfm_m  # noqa: E402
from mcmc_clv_model_amd.data import synthetic_cbs  # noqa: E402
from tests.helpers import cdnow  # noqa: E402


def digest(d):
    h = hashlib.sha256()
    for k in ("level_1", "level_2"):
        for a in d[k]:
            h.update(np.ascontiguousarray(a).tobytes())
    h.update(np.asarray(d["log_likelihood"], dtype=np.float64).tobytes())
    return h.hexdigest()[:16]


def main():
    full = cdnow("full")
    kw = dict(mcmc=100, burnin=100, thin=1, chains=2, seed=7, trace=0)
    print("c2-shaped", digest(mcmc_draw_parameters(full, ["first_sales_scaled"], **kw)), flush=True)
    print("c3-shaped", digest(mcmc_draw_parameters_rfm_m(full, ["gender_F", "age_scaled"], **kw)), flush=True)
    syn = synthetic_cbs(150000, 5, seed=3)
    print("bi K=5 launch", digest(mcmc_draw_parameters(syn, [f"c{k}" for k in range(1, 5)], **kw)),
          flush=True)


if __name__ == "__main__":
    main()
