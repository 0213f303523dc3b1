"""Drop-in for ``src/models/trivariate/mcmc.py`` (Abe 2015 "RFM-M": lambda, mu, eta).

``mcmc_draw_parameters_rfm_m`` keeps the reference's signature, defaults and return layout
(trivariate/mcmc.py:580-657; like the reference it does not validate columns and needs a
``log_s`` column).  Keyword-only extras as in :mod:`mcmc_clv_model_amd.bivariate`.
"""
from __future__ import annotations

from typing import Optional, Sequence

from .analysis import draw_future_transactions_rfm_m as draw_future_transactions  # tri:660-749
from .sampler import build_problem, fit

__all__ = ["mcmc_draw_parameters_rfm_m", "draw_future_transactions"]


def mcmc_draw_parameters_rfm_m(cal_cbs, covariates: Optional[Sequence[str]] = None, mcmc: int = 2500,
                               burnin: int = 500, thin: int = 50, chains: int = 2,
                               seed: Optional[int] = None, trace: int = 100, n_mh_steps: int = 20, *,
                               draw_sink: str = "full", rng: str = "philox", device: int = -1,
                               replay_tape=None, replay_sweeps: Optional[int] = None,
                               devices: Optional[Sequence[int]] = None, shard: str = "auto", exchange: str = "auto"):
    """3-dimensional HB Pareto/NBD + spend sampler (trivariate/mcmc.py:580).

    Returns {"level_1": [(n_draws, N, 5) per chain: lambda, mu, tau, z, eta],
             "level_2": [(n_draws, 3K+6) per chain], "log_likelihood": float}
    """
    if covariates is None:
        covariates = []
    p = build_problem(cal_cbs, covariates, D=3)
    out = fit(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=seed, trace=trace,
              n_mh_steps=n_mh_steps, draw_sink=draw_sink, rng=rng, device=device,
              replay_tape=replay_tape, replay_sweeps=replay_sweeps, devices=devices, shard=shard,
               exchange=exchange)
    out["log_likelihood"] = float(out["log_likelihood"])  # tri:652 returns a Python float
    return out
