"""Drop-in for ``src/models/bivariate/mcmc.py`` (Abe 2009 HB Pareto/NBD, lambda & mu).

``mcmc_draw_parameters`` keeps the reference's signature, defaults, validation errors, trace
line and return layout (bivariate/mcmc.py:437-504); the sweeps run on the GPU
(csrc/kernels.hip).  Keyword-only extras:

* ``draw_sink``: "full" (level_1 draws, reference layout), "summary" (per-customer posterior
  means kept on device; ``level_1`` is None), "summary+pct" (as "summary", plus Table 4's
  per-customer 2.5/97.5 percentiles of lambda and mu from a float32 store of the draws:
  ``out["summary"]["level1"]``, which ``analysis.compute_table4(out)`` uses), "none".
* ``rng``: "philox" (counter-based, default) or "replay" (test mode: consume variates recorded
  from the reference's numpy Generator, ``replay_tape``).
* ``device``: HIP device ordinal (-1 = current).
* ``devices``: several device ordinals — the run is spread over them from this process
  (``shard="chains"``: chain groups, one host thread each; ``"customers"``: every chain's customers
  split into shards exchanging the level-2 statistics each sweep by peer stores or device copies,
  ``exchange`` = "auto" | "p2p" | "copy"; ``"auto"``: chains when they divide evenly), with the
  single-device run's output bit for bit (sampler.fit_multi, csrc/group.hip).
"""
from __future__ import annotations

from typing import Optional, Sequence

from .analysis import draw_future_transactions  # bi:506-546 (posterior predictive, csrc/analysis.hip)
from .sampler import build_problem, fit

__all__ = ["mcmc_draw_parameters", "draw_future_transactions"]


def mcmc_draw_parameters(cal_cbs, covariates: Optional[Sequence[str]] = None, mcmc: int = 2500,
                         burnin: int = 500, thin: int = 50, chains: int = 2, seed: Optional[int] = None,
                         trace: int = 100, n_mh_steps: int = 20, *, draw_sink: str = "full",
                         rng: str = "philox", device: int = -1, replay_tape=None,
                         replay_sweeps: Optional[int] = None, devices: Optional[Sequence[int]] = None,
                         shard: str = "auto", exchange: str = "auto"):
    """Run the Abe (2009) Gibbs/MH sampler on calibration CBS (bivariate/mcmc.py:437).

    Returns dict(level_1=[(n_draws, N, 4) per chain: lambda, mu, tau, z],
                 level_2=[(n_draws, 2K+3) per chain: beta.T.ravel(), Sigma00, Sigma01, Sigma11],
                 log_likelihood=np.float64)
    """
    if covariates is None:
        covariates = []
    for col in ("x", "t_x", "T_cal"):  # bi:461-465
        if col not in cal_cbs:
            raise ValueError(f"cal_cbs missing required column '{col}'")
    if not all(col in cal_cbs for col in covariates):
        raise ValueError("some covariate columns not in cal_cbs")
    p = build_problem(cal_cbs, covariates, D=2)
    return fit(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=seed, trace=trace,
               n_mh_steps=n_mh_steps, draw_sink=draw_sink, rng=rng, device=device,
               replay_tape=replay_tape, replay_sweeps=replay_sweeps, devices=devices, shard=shard,
               exchange=exchange)
