"""Posterior analysis on the GPU, drop-in for the reference's helpers.

Reference functions mirrored (same names, arguments, defaults and return layout):

* ``draw_future_transactions`` — ``src/models/bivariate/mcmc.py:506-546`` (counts) and, as
  ``draw_future_transactions_rfm_m`` / ``trivariate.draw_future_transactions``,
  ``src/models/trivariate/mcmc.py:660-749`` (counts and lognormal spend totals).
* ``post_mean_lambdas``, ``post_mean_mus``, ``chain_total_loglik``, ``compute_table4`` —
  ``src/models/utils/analysis_bi_helpers.py:15-27, 52-72, 75-166``.
* ``posterior_weekly_tracking`` — the posterior-predictive weekly repeat-transaction curve of
  ``src/models/bivariate/analysis_abe.py:444-464`` (inline script code in the reference).

The per-customer / per-draw work runs in ``csrc/analysis.hip`` through the C ABI (``clv_predict``,
``clv_track``, ``clv_level1_summary``, ``clv_chain_total_loglik``); the host only reshapes and
formats (pandas).  Random draws come from Philox streams keyed by ``seed`` (the reference uses
one numpy Generator), so simulated outputs match the reference in distribution; the statistics
(means, percentiles) are exact.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Any, Dict, Optional

import numpy as np
import pandas as pd

from . import _lib
from ._lib import check, dptr
from .sampler import resolve_seed

__all__ = ["draw_future_transactions", "draw_future_transactions_rfm_m", "post_mean_lambdas", "post_mean_mus",
           "chain_total_loglik", "compute_table4", "level1_summary", "posterior_weekly_tracking"]


def _stacked_level1(level1_chains) -> np.ndarray:
    if level1_chains is None:
        raise ValueError("level-1 draws are needed (run the sampler with draw_sink='full')")
    a = np.ascontiguousarray(np.concatenate(list(level1_chains), axis=0), dtype=np.float64)
    if a.ndim != 3 or a.shape[2] not in (4, 5):
        raise ValueError("level_1 draws must be (n_draws, n_customers, 4 or 5) per chain")
    return a


def _L():
    L = _lib.lib()
    if _lib.device_count() < 1:
        raise _lib.ClvError("no HIP device visible; the analysis kernels have no CPU fallback")
    return L


def _i64p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


def _predict(cbs, draws, T_star, seed, simulate_spend, sigma_s, device):
    L = _L()
    a = _stacked_level1(draws["level_1"])
    nd, n, w = a.shape
    T_cal = np.ascontiguousarray(cbs["T_cal"].to_numpy(float))
    if T_cal.shape[0] != n:
        raise ValueError("cbs and draws disagree on the number of customers")
    x = np.empty((nd, n), np.int64)
    spend = np.empty((nd, n), np.float64) if simulate_spend else None
    check(L.clv_predict(int(device), dptr(a), nd, n, w, dptr(T_cal), float(T_star), resolve_seed(seed),
                        1 if simulate_spend else 0, float(sigma_s), _i64p(x), dptr(spend) if spend is not None else None))
    return x, spend


def draw_future_transactions(cbs: pd.DataFrame, draws: Dict[str, Any], T_star: float = 39.0,
                             seed: Optional[int] = None, *, device: int = -1) -> np.ndarray:
    """Posterior-predictive transactions in (T_cal, T_cal + T_star] (bivariate/mcmc.py:506-546):
    x* ~ Poisson(lambda * tau*), tau* = T_star if alive else clip(tau - T_cal, 0, T_star).
    Returns int64 (n_draws_total, n_customers), chains stacked in order."""
    return _predict(cbs, draws, T_star, seed, False, 0.5, device)[0]


def draw_future_transactions_rfm_m(cbs: pd.DataFrame, draws: Dict[str, Any], T_star: float = 39.0, *,
                                   simulate_spend: bool = True, sigma_s: float = 0.50, seed: Optional[int] = None,
                                   device: int = -1):
    """RFM-M posterior predictive (trivariate/mcmc.py:660-749): counts as above and, with
    ``simulate_spend``, per-customer totals of x* lognormal(mean=eta, sigma=sigma_s) spends (eta is
    the level-1 column 4, passed as the log-mean like the reference). Returns ``x_future`` or
    ``(x_future, spend_future)``."""
    x, spend = _predict(cbs, draws, T_star, seed, simulate_spend, sigma_s, device)
    return (x, spend) if simulate_spend else x


def level1_summary(draws: Dict[str, Any], mu_cap: float = 0.05, *, device: int = -1) -> pd.DataFrame:
    """Per-customer posterior statistics computed on the GPU: means of lambda, mu, min(mu, mu_cap),
    z, tau (and eta), and numpy-'linear' 2.5 / 97.5 percentiles of lambda and mu.  A result of
    ``draw_sink="summary+pct"`` (no level-1 draws) carries them already, formed on the device at
    the end of the run (``draws["summary"]["level1"]``; mu_cap 0.05 only)."""
    if draws.get("level_1") is None and isinstance(draws.get("summary"), dict) and "level1" in draws["summary"]:
        if mu_cap != _lib.SUMMARY_MU_CAP:
            raise ValueError("a summary run's capped mean of mu uses mu_cap = 0.05")
        return draws["summary"]["level1"]
    L = _L()
    a = _stacked_level1(draws["level_1"])
    nd, n, w = a.shape
    out = np.empty((n, len(_lib.L1_STATS)), np.float64)
    check(L.clv_level1_summary(int(device), dptr(a), nd, n, w, float(mu_cap), dptr(out)))
    cols = list(_lib.L1_STATS if w == 5 else _lib.L1_STATS[:-1])
    return pd.DataFrame(out[:, :len(cols)], columns=cols)


def post_mean_lambdas(draws) -> np.ndarray:
    """analysis_bi_helpers.py:15-20 — per-customer posterior mean of lambda over all chains' draws."""
    return level1_summary(draws)["mean_lambda"].to_numpy()


def post_mean_mus(draws) -> np.ndarray:
    """analysis_bi_helpers.py:22-27 — per-customer posterior mean of mu over all chains' draws."""
    return level1_summary(draws)["mean_mu"].to_numpy()


def chain_total_loglik(level1_chains, cbs, *, device: int = -1) -> float:
    """analysis_bi_helpers.py:52-72 — mean over draws of the total log-likelihood
    sum_i [x log(lam) + (1-z) log(mu) - (lam+mu)(z T + (1-z) tau) - gammaln(x+1)]."""
    L = _L()
    a = _stacked_level1(level1_chains)
    nd, n, w = a.shape
    x = np.ascontiguousarray(cbs["x"].to_numpy(), dtype=np.int32)
    T_cal = np.ascontiguousarray(cbs["T_cal"].to_numpy(float))
    out = ctypes.c_double()
    check(L.clv_chain_total_loglik(int(device), dptr(a), nd, n, w, x.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                   dptr(T_cal), ctypes.byref(out)))
    return float(out.value)


def compute_table4(draws, xstar_draws=None) -> pd.DataFrame:
    """analysis_bi_helpers.py:75-166 — Table 4 of Abe (2009): customer-level statistics (per-customer
    reductions on the GPU), ranked by expected validation-period transactions, top/bottom 10 plus
    Ave/Min/Max rows, rounded like the paper.  ``xstar_draws`` is accepted and unused, as in the
    reference."""
    s = level1_summary(draws, mu_cap=0.05)
    mean_lambda = s["mean_lambda"].to_numpy()
    mean_mu = s["mean_mu_capped"].to_numpy()
    mean_z = s["mean_z"].to_numpy()
    t_star = 39
    mean_xstar = mean_z * (mean_lambda / mean_mu) * (1.0 - np.exp(-mean_mu * t_star))
    with np.errstate(divide="ignore"):
        mean_lifetime = np.where(mean_mu > 0, (1.0 / mean_mu) / 52.0, np.inf)
    surv_1yr = np.exp(-mean_mu * 52)
    df = pd.DataFrame({
        "Mean(λ)": mean_lambda,
        "2.5% tile λ": s["lambda_p025"].to_numpy(),
        "97.5% tile λ": s["lambda_p975"].to_numpy(),
        "Mean(μ)": mean_mu,
        "2.5% tile μ": s["mu_p025"].to_numpy(),
        "97.5% tile μ": s["mu_p975"].to_numpy(),
        "Mean exp lifetime (yrs)": mean_lifetime,
        "Survival rate (1yr)": surv_1yr,
        "P(alive at T_cal)": mean_z,
        "Exp # of trans in val period": mean_xstar,
    })
    df.index.name = "Customer ID"
    df_sorted = df.sort_values("Exp # of trans in val period", ascending=False).reset_index(drop=True)
    df_sorted.insert(0, "ID", df_sorted.index + 1)
    top10, bottom10 = df_sorted.iloc[:10], df_sorted.iloc[-10:]
    ave_row = df.mean().to_frame().T.assign(ID="Ave")
    min_row = df.min().to_frame().T.assign(ID="Min")
    max_row = df.max().to_frame().T.assign(ID="Max")
    out = pd.concat([top10, pd.DataFrame({"ID": ["…"]}), bottom10, ave_row, min_row, max_row],
                    ignore_index=True).set_index("ID")
    lam_cols = ["Mean(λ)", "2.5% tile λ", "97.5% tile λ"]
    mu_cols = ["Mean(μ)", "2.5% tile μ", "97.5% tile μ"]
    out[lam_cols] = out[lam_cols].round(3)
    out[mu_cols] = out[mu_cols].round(4)
    out["Mean exp lifetime (yrs)"] = out["Mean exp lifetime (yrs)"].round(2)
    out["Survival rate (1yr)"] = out["Survival rate (1yr)"].round(3)
    out["P(alive at T_cal)"] = out["P(alive at T_cal)"].round(3)
    out["Exp # of trans in val period"] = out["Exp # of trans in val period"].round(2)
    return out


def posterior_weekly_tracking(draws, birth_week, times, seed: Optional[int] = 0, *, device: int = -1) -> np.ndarray:
    """Posterior-predictive weekly repeat transactions (bivariate/analysis_abe.py:444-464): for every
    week t in ``times`` (ascending), the mean over all draws of the simulated transactions of the
    customers with birth_week < t <= birth_week + tau (rate lambda per unit time).  The reference
    draws one Poisson per customer and week; their sum is drawn here as one exact Poisson of the
    summed rate (same distribution).  Returns inc_hb_weekly (float64, len(times)); np.cumsum gives
    the tracking curve."""
    L = _L()
    a = _stacked_level1(draws["level_1"])
    nd, n, w = a.shape
    b = np.ascontiguousarray(np.asarray(birth_week, dtype=np.float64))
    t = np.ascontiguousarray(np.asarray(times, dtype=np.float64))
    if b.shape[0] != n:
        raise ValueError("birth_week must have one entry per customer")
    out = np.empty(t.shape[0], np.float64)
    check(L.clv_track(int(device), dptr(a), nd, n, w, dptr(b), dptr(t), t.shape[0], resolve_seed(seed), dptr(out)))
    return out
