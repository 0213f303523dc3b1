"""CPU oracle of the reference's posterior-analysis helpers — TEST INFRASTRUCTURE ONLY.

Clean-room numpy restatement (nothing in ``mcmc_clv_model_amd`` imports it) of:

* ``draw_future_transactions`` — bivariate ``src/models/bivariate/mcmc.py:506-546`` and
  trivariate ``src/models/trivariate/mcmc.py:660-749`` (same numpy Generator calls in the same
  order, so outputs are bitwise equal to the reference's for the same seed);
* ``post_mean_lambdas`` / ``post_mean_mus`` / ``chain_total_loglik`` / ``compute_table4`` —
  ``src/models/utils/analysis_bi_helpers.py:15-27, 52-72, 75-166``;
* the posterior-predictive weekly tracking loop of ``src/models/bivariate/analysis_abe.py:444-464``.

Pinned by ``tests/golden/make_goldens.py`` (``analysis`` step), which runs the reference's own
functions on the same draws and refuses to write fixtures unless this restatement agrees bit for
bit (the weekly loop is inline script code in the reference: restated from the listed lines).
"""
from __future__ import annotations

import numpy as np
from scipy.special import gammaln


def draw_future_transactions_bi(cbs, draws, T_star=39.0, seed=None):
    rng = np.random.default_rng(seed)
    T_cal = cbs["T_cal"].to_numpy()
    out = []
    for chain in draws["level_1"]:
        for draw in chain:
            lam, tau, z = draw[:, 0], draw[:, 2], draw[:, 3] > 0.5
            ts = np.full_like(T_cal, T_star, dtype=float)
            ts[~z] = np.clip(tau[~z] - T_cal[~z], 0.0, T_star)
            out.append(rng.poisson(lam=lam * ts))
    return np.array(out)


def draw_future_transactions_tri(cbs, draws, T_star=39.0, *, simulate_spend=True, sigma_s=0.50, seed=None):
    rng = np.random.default_rng(seed)
    T_cal = cbs["T_cal"].to_numpy(float)
    xs, sp = [], []
    for chain in draws["level_1"]:
        for draw in chain:
            lam, mu, tau, zf, eta = draw.T
            alive = zf > 0.5
            ts = np.full_like(T_cal, T_star, dtype=float)
            ts[~alive] = np.clip(tau[~alive] - T_cal[~alive], a_min=0.0, a_max=T_star)
            x = rng.poisson(lam=lam * ts)
            xs.append(x)
            if simulate_spend:
                if x.sum() > 0:
                    idx = np.repeat(np.arange(len(x)), x)
                    per = rng.lognormal(mean=eta[idx], sigma=sigma_s, size=len(idx))
                    tot = np.bincount(idx, weights=per, minlength=len(x))
                else:
                    tot = np.zeros_like(x, dtype=float)
                sp.append(tot)
    xf = np.vstack(xs)
    return (xf, np.vstack(sp)) if simulate_spend else xf


def post_mean_lambdas(draws):
    return np.concatenate(draws["level_1"], axis=0)[:, :, 0].mean(axis=0)


def post_mean_mus(draws):
    return np.concatenate(draws["level_1"], axis=0)[:, :, 1].mean(axis=0)


def chain_total_loglik(level1_chains, cbs):
    x = cbs["x"].to_numpy()
    T_cal = cbs["T_cal"].to_numpy()
    totals = []
    for chain in level1_chains:
        for draw in chain:
            lam, mu, tau, z = draw[:, 0], draw[:, 1], draw[:, 2], draw[:, 3] > 0.5
            ll = x * np.log(lam) + (1 - z) * np.log(mu) - (lam + mu) * (z * T_cal + (1 - z) * tau) - gammaln(x + 1)
            totals.append(ll.sum())
    return np.mean(totals)


def table4_stats(draws, mu_cap=0.05):
    """The per-customer columns compute_table4 builds before ranking (analysis_bi_helpers.py:79-107)."""
    a = np.concatenate(draws["level_1"], axis=0)
    mu_raw = a[:, :, 1]
    return dict(mean_lambda=a[:, :, 0].mean(axis=0),
                lambda_p025=np.percentile(a[:, :, 0], 2.5, axis=0),
                lambda_p975=np.percentile(a[:, :, 0], 97.5, axis=0),
                mean_mu_capped=np.clip(mu_raw, None, mu_cap).mean(axis=0),
                mu_p025=np.percentile(mu_raw, 2.5, axis=0),
                mu_p975=np.percentile(mu_raw, 97.5, axis=0),
                mean_z=a[:, :, 3].mean(axis=0))


def weekly_tracking(draws, birth_week, times):
    """analysis_abe.py:444-464 restated: per draw d a Generator seeded d, per week one Poisson per
    customer of rate lambda * 1[b < t <= b + tau]; mean over draws of the weekly sums."""
    inc = np.zeros_like(times, dtype=float)
    per_chain = len(draws["level_1"][0])
    n_draws = per_chain * len(draws["level_1"])
    for d in range(n_draws):
        lv = draws["level_1"][d // per_chain][d % per_chain]
        lam, tau = lv[:, 0], lv[:, 2]
        rng = np.random.default_rng(d)
        for j, t in enumerate(times):
            active = (t > birth_week) & (t <= birth_week + tau)
            inc[j] += rng.poisson(lam=lam * 1.0 * active).sum()
    return inc / n_draws


def weekly_tracking_expectation(draws, birth_week, times):
    """E[inc_hb_weekly]: the mean over draws of sum_i lambda_i 1[b_i < t <= b_i + tau_i]."""
    a = np.concatenate(draws["level_1"], axis=0)
    lam, tau = a[:, :, 0], a[:, :, 2]
    out = np.zeros(len(times))
    for j, t in enumerate(times):
        out[j] = np.mean(np.sum(lam * ((t > birth_week) & (t <= birth_week + tau)), axis=1))
    return out
