"""CPU oracle for the Abe (2009/2015) HB Pareto/NBD Gibbs/MH sweep.

TEST INFRASTRUCTURE ONLY.  Nothing in ``mcmc_clv_model_amd`` imports this
module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker / the timed CPU baseline.

This is a clean-room numpy restatement of the reference sampler
(lucagem29/mcmc_clv_model):

* bivariate  ``src/models/bivariate/mcmc.py``  (abbrev. ``bi``)
* trivariate ``src/models/trivariate/mcmc.py`` (abbrev. ``tri``)

It consumes a ``numpy.random.Generator`` in exactly the reference's order, so
for the same seed its output is BITWISE equal to the reference's
(pinned by ``tests/golden/make_goldens.py``, which imports the reference in the
build container and checks equality before writing any fixture).  Every random
variate passes through :class:`Stream`, which can record it; the recorded
"tape" is what the HIP sampler's replay mode consumes, so the GPU trajectory
can be compared with the reference trajectory draw for draw.

Third-party arithmetic the reference relies on (restated here, pinned by the
same bitwise check): numpy 2.2 ``Generator`` (PCG64; ``random``,
``exponential`` = scale * standard_exponential, ``standard_t``, ``normal`` =
loc + scale * standard_normal, ``chisquare``, ``multivariate_normal`` via SVD)
and scipy 1.15 ``invwishart.rvs`` (Bartlett decomposition, BLAS trsm/trmm).
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import scipy.linalg
from scipy.linalg import get_blas_funcs


# ---------------------------------------------------------------------------
# Variate stream (records what it hands out)
# ---------------------------------------------------------------------------
class Stream:
    """Wraps a numpy Generator; optionally records every variate it hands out.

    ``tape`` is a list with one dict per sweep; :meth:`begin_sweep` opens it.
    """

    def __init__(self, rng: np.random.Generator, record: bool = False):
        self.rng = rng
        self.record = record
        self.tape: List[Dict[str, Any]] = []

    def begin_sweep(self) -> None:
        if self.record:
            self.tape.append({})

    def _rec(self, key: str, val, append: bool = False):
        if self.record:
            cur = self.tape[-1]
            if append:
                cur.setdefault(key, []).append(np.array(val, copy=True))
            else:
                cur[key] = np.array(val, copy=True)
        return val

    # bi:200 / tri:277  rng.random(N)
    def random(self, n: int, key: str) -> np.ndarray:
        return self._rec(key, self.rng.random(n))

    # bi:217 / tri:294  rng.exponential(scale) == scale * standard_exponential
    def standard_exponential(self, n: int, key: str) -> np.ndarray:
        return self._rec(key, self.rng.standard_exponential(n))

    # bi:316-317 / tri:435-436
    def standard_t3(self, n: int, key: str) -> np.ndarray:
        return self._rec(key, self.rng.standard_t(df=3, size=n), append=True)

    def random_step(self, n: int, key: str) -> np.ndarray:
        return self._rec(key, self.rng.random(n), append=True)

    # tri:333 rng.normal(loc, scale) == loc + scale * standard_normal
    def standard_normal(self, n: int, key: str) -> np.ndarray:
        return self._rec(key, self.rng.standard_normal(n))

    # scipy invwishart._inv_standard_rvs: normal(size=(1, n_tril)), chisquare(dfs, size=(1, dim))
    def bartlett(self, dim: int, df: float):
        n_tril = dim * (dim - 1) // 2
        normals = self.rng.normal(size=(1, n_tril))[0]
        chi_dfs = (df - dim + 1) + np.arange(dim)
        chi2 = self.rng.chisquare(df=chi_dfs, size=(1, dim))[0]
        self._rec("iw_normal", normals)
        self._rec("iw_chi2", chi2)
        return normals, chi2

    # numpy Generator.multivariate_normal(mean, cov) with method='svd'
    def mvn_noise(self, cov: np.ndarray) -> np.ndarray:
        """Returns the zero-mean part ``z @ factor.T`` of numpy's MVN draw."""
        z = self.rng.standard_normal((1, cov.shape[0]))
        (u, s, vh) = np.linalg.svd(cov)
        factor = u * np.sqrt(s)
        noise = (z @ factor.T)[0]
        self._rec("mvn_z", z[0])
        self._rec("mvn_noise", noise)
        return noise


# ---------------------------------------------------------------------------
# Latent draws
# ---------------------------------------------------------------------------
def p_alive(tx, Tcal, lambdas, mus):
    """bi:195-199 (tri:274-276): P(alive) in the overflow-safe rewrite."""
    mu_lam = mus + lambdas
    z = mu_lam * (Tcal - tx)
    exp_neg_z = np.exp(-z)
    return (mu_lam * exp_neg_z) / (mu_lam * exp_neg_z + mus * (1.0 - exp_neg_z))


def draw_z(tx, Tcal, lambdas, mus, stream: Stream) -> np.ndarray:
    """bi:193-200, tri:272-277."""
    p = p_alive(tx, Tcal, lambdas, mus)
    return stream.random(p.shape[0], "u_z") < p


def tau_churned(tx, Tcal, ml, u):
    """bi:222-226: inverse CDF of Exp(ml) truncated to [t_x, T_cal], clamped at 700."""
    ml_tx = np.minimum(700.0, ml * tx)
    ml_T = np.minimum(700.0, ml * Tcal)
    return -np.log((1 - u) * np.exp(-ml_tx) + u * np.exp(-ml_T)) / ml


def draw_tau(tx, Tcal, lambdas, mus, z, stream: Stream) -> np.ndarray:
    """bi:203-227, tri:280-304.  RNG order: all alive exponentials, then churned uniforms."""
    mu_lam = mus + lambdas
    tau = np.empty_like(tx)
    alive_idx = np.where(z)[0]
    v = np.zeros_like(tx)          # per-customer variate actually consumed (for replay)
    if alive_idx.size:
        e = stream.standard_exponential(alive_idx.size, "e_alive")
        v[alive_idx] = e
        tau[alive_idx] = Tcal[alive_idx] + (1.0 / mus[alive_idx]) * e
    churn_idx = np.where(~z)[0]
    if churn_idx.size:
        ml = mu_lam[churn_idx]
        u = stream.random(churn_idx.size, "u_churn")
        v[churn_idx] = u
        tau[churn_idx] = tau_churned(tx[churn_idx], Tcal[churn_idx], ml, u)
    stream._rec("v_tau", v)
    return tau


# ---------------------------------------------------------------------------
# Level 2: conjugate multivariate regression (replaces bayesm::rmultireg)
# ---------------------------------------------------------------------------
def level2_posterior(X, Y, hyper):
    """bi:243-256, tri:355-370: (V_beta, B_hat, S_n, nu_n)."""
    A0, B0, nu0, S0 = hyper["A_0"], hyper["beta_0"], hyper["nu_00"], hyper["gamma_00"]
    XtX = X.T @ X
    V_beta = np.linalg.inv(XtX + A0)
    B_hat = V_beta @ (X.T @ Y + A0 @ B0)
    E = Y - X @ B_hat
    C = B_hat - B0
    S_n = S0 + E.T @ E + C.T @ A0 @ C
    nu_n = nu0 + X.shape[0]
    return V_beta, B_hat, S_n, nu_n


def invwishart_from_variates(S_n, normals, chi2):
    """scipy 1.15 invwishart.rvs (``_multivariate.py`` invwishart_gen.rvs/_rvs):
    C = chol(S_n) lower; A lower with N(0,1) below and sqrt(chi2) on the diagonal;
    Sigma = (C A^-1)(C A^-1)^T via BLAS trsm/trmm."""
    dim = S_n.shape[0]
    C = scipy.linalg.cholesky(S_n, lower=True)
    A = np.zeros((dim, dim))
    r, c = np.tril_indices(dim, k=-1)
    A[r, c] = normals
    A[np.arange(dim), np.arange(dim)] = chi2 ** 0.5
    trsm = get_blas_funcs(("trsm"), (A,))
    trmm = get_blas_funcs(("trmm"), (A,))
    CA = trsm(1.0, A, C, side=1, lower=True)
    return trmm(1.0, CA, CA, side=1, lower=True, trans_a=True)


def draw_level_2(X, Y, hyper, stream: Stream):
    """bi:233-262, tri:340-380.  Returns (beta K×D, Sigma D×D)."""
    V_beta, B_hat, S_n, nu_n = level2_posterior(X, Y, hyper)
    normals, chi2 = stream.bartlett(S_n.shape[0], nu_n)
    Sigma = invwishart_from_variates(S_n, normals, chi2)
    # Quirk Q1 (bi:261): row-major B_hat.ravel() paired with kron(Sigma, V) (column-major order).
    noise = stream.mvn_noise(np.kron(Sigma, V_beta))
    beta = (B_hat.ravel() + noise).reshape(B_hat.shape)
    stream._rec("B_hat", B_hat)
    stream._rec("S_n", S_n)
    stream._rec("beta", beta)
    stream._rec("Sigma", Sigma)
    return beta, Sigma


# ---------------------------------------------------------------------------
# Level 1: random-walk MH on (log lambda, log mu)
# ---------------------------------------------------------------------------
def log_posterior(ll, lm, x, z, T_cal, tau, mv_mean, inv_Sigma):
    """bi:291-310 (tri:410-429). Quirks: lm > 5 => -inf (Q3)."""
    diff_l = ll - mv_mean[:, 0]
    diff_m = lm - mv_mean[:, 1]
    lik = x * ll + (1 - z) * lm - (np.exp(ll) + np.exp(lm)) * (z * T_cal + (1 - z) * tau)
    prior = -0.5 * (diff_l ** 2 * inv_Sigma[0, 0]
                    + 2 * diff_l * diff_m * inv_Sigma[0, 1]
                    + diff_m ** 2 * inv_Sigma[1, 1])
    res = lik + prior
    return np.where(lm > 5.0, -np.inf, res)


def draw_level_1(x, T_cal, X, lambdas, mus, z, tau, beta, Sigma, stream: Stream, n_mh_steps=20):
    """bi:268-339, tri:387-458.  Proposal scale is Sigma[d,d] (variance, quirk Q2);
    for D=3 the 3x3 inverse is used through its [0:2,0:2] block (quirk Q4)."""
    inv_Sigma = np.linalg.inv(Sigma)
    mv_mean = X @ beta
    log_lambda = np.log(lambdas)
    log_mu = np.log(mus)
    N = log_lambda.size
    with np.errstate(invalid="ignore", over="ignore"):
        cur_lp = log_posterior(log_lambda, log_mu, x, z, T_cal, tau, mv_mean, inv_Sigma)
        for _ in range(n_mh_steps):
            eps_lambda = Sigma[0, 0] * stream.standard_t3(N, "t_l")
            eps_mu = Sigma[1, 1] * stream.standard_t3(N, "t_m")
            prop_ll = np.clip(log_lambda + eps_lambda, -70.0, 70.0)
            prop_lm = np.clip(log_mu + eps_mu, -70.0, 70.0)
            prop_lp = log_posterior(prop_ll, prop_lm, x, z, T_cal, tau, mv_mean, inv_Sigma)
            mhr = np.exp(prop_lp - cur_lp)
            accept = mhr > stream.random_step(N, "u_acc")
            log_lambda[accept] = prop_ll[accept]
            log_mu[accept] = prop_lm[accept]
            cur_lp[accept] = prop_lp[accept]
    return np.exp(log_lambda), np.exp(log_mu)


def draw_eta(log_s, X, beta, Sigma, omega2, stream: Stream):
    """tri:306-333: conjugate normal for log spend; returns the log-scale draw."""
    prior_mean = (X @ beta)[:, 2]
    prior_var = Sigma[2, 2]
    post_var = 1.0 / (1.0 / omega2 + 1.0 / prior_var)
    post_mean = post_var * (log_s / omega2 + prior_mean / prior_var)
    zeta = stream.standard_normal(log_s.shape[0], "eta_z")
    return post_mean + np.sqrt(post_var) * zeta


def lik_terms(x, T_cal, lambdas, mus, z, tau):
    """bi:415-427: per-customer likelihood term used for the stored log-likelihood."""
    log_lambda = np.log(lambdas)
    log_mu = np.log(mus)
    return x * log_lambda + (1 - z) * log_mu - (lambdas + mus) * (z * T_cal + (1 - z) * tau)


# ---------------------------------------------------------------------------
# Setup shared by both samplers
# ---------------------------------------------------------------------------
def init_state(x, t_x, T_cal):
    """bi:368-370 / tri:489-491 (x is an int64 column; pandas mean == float64 sum / n)."""
    lam_init = x.astype(np.float64).sum() / x.size / np.mean(np.where(t_x == 0, T_cal, t_x))
    lambdas = np.full(x.size, lam_init)
    mus = 1.0 / (t_x + 0.5 / lam_init)
    return lam_init, lambdas, mus


def design_matrix(cbs, covariates: Sequence[str]):
    """bi:467-470, tri:615-618."""
    df = cbs.copy().reset_index(drop=True)
    df["intercept"] = 1.0
    cols = ["intercept"] + list(covariates)
    return df, df[cols].to_numpy(float)


def default_hyper(K: int, D: int):
    """bi:474-479 (D=2: nu0 = 3+K), tri:622-626 (D=3: nu0 = 4+K)."""
    nu_00 = (3 if D == 2 else 4) + K
    return dict(beta_0=np.zeros((K, D)), A_0=np.eye(K) * 0.01, nu_00=nu_00,
                gamma_00=nu_00 * np.eye(D))


def n_draws_of(mcmc: int, thin: int) -> int:
    return (mcmc - 1) // thin + 1


def is_stored(step: int, burnin: int, thin: int) -> bool:
    return step > burnin and (step - 1 - burnin) % thin == 0


# ---------------------------------------------------------------------------
# Chains
# ---------------------------------------------------------------------------
def run_chain_bi(chain_id, x, t_x, T_cal, X, hyper, mcmc, burnin, thin, stream: Stream,
                 trace, n_mh_steps, n_sweeps: Optional[int] = None, on_sweep=None):
    """bi:346-431.  ``n_sweeps`` truncates the run (trajectory fixtures); ``on_sweep(step)`` is
    called after every sweep (bench.py's CPU-baseline timer)."""
    N, K = X.shape
    n_draws = n_draws_of(mcmc, thin)
    lvl1 = np.empty((n_draws, N, 4))
    lvl2 = np.empty((n_draws, 2 * K + 3))
    ll_chain = []
    lam_init, lambdas, mus = init_state(x, t_x, T_cal)
    hyper["beta_0"][0, 0] = math.log(lambdas.mean())
    hyper["beta_0"][0, 1] = math.log(mus.mean())
    z = np.ones(N, dtype=bool)
    tau = T_cal + 1.0
    store_idx = -1
    tot = burnin + mcmc if n_sweeps is None else n_sweeps
    for step in range(1, tot + 1):
        if trace and step % trace == 0:
            print(f"chain {chain_id} | step {step}/{burnin + mcmc}")
        stream.begin_sweep()
        z = draw_z(t_x, T_cal, lambdas, mus, stream)
        tau = draw_tau(t_x, T_cal, lambdas, mus, z, stream)
        beta, Sigma = draw_level_2(X, np.column_stack([np.log(lambdas), np.log(mus)]), hyper, stream)
        lambdas, mus = draw_level_1(x, T_cal, X, lambdas, mus, z, tau, beta, Sigma, stream, n_mh_steps)
        if is_stored(step, burnin, thin):
            store_idx += 1
            lambdas = np.exp(np.log(lambdas))       # bi:405-406 (quirk Q5)
            mus = np.exp(np.log(mus))
            lvl1[store_idx, :, 0] = lambdas
            lvl1[store_idx, :, 1] = mus
            lvl1[store_idx, :, 2] = tau
            lvl1[store_idx, :, 3] = z.astype(float)
            lvl2[store_idx, : 2 * K] = beta.T.ravel()
            lvl2[store_idx, -3:] = [Sigma[0, 0], Sigma[0, 1], Sigma[1, 1]]
            ll_chain.append(np.mean(lik_terms(x, T_cal, lambdas, mus, z, tau)))
        if stream.record:
            st = stream.tape[-1]
            st.update(z=z.copy(), tau=tau.copy(), lam=lambdas.copy(), mu=mus.copy())
        if on_sweep is not None:
            on_sweep(step)
    return dict(level_1=lvl1, level_2=lvl2, log_likelihood=np.array(ll_chain))


def run_chain_tri(chain_id, x, t_x, T_cal, log_s, X, hyper, mcmc, burnin, thin, stream: Stream,
                  trace, n_mh_steps, n_sweeps: Optional[int] = None, omega2: Optional[float] = None,
                  log_s_mean: Optional[float] = None, on_sweep=None):
    """tri:465-574.  ``omega2`` / ``log_s_mean`` are pandas ``var()`` / ``mean()`` of log_s
    (tri:494, tri:499) — computed by the caller from the Series."""
    N, K = X.shape
    n_draws = n_draws_of(mcmc, thin)
    lvl1 = np.empty((n_draws, N, 5))
    lvl2 = np.empty((n_draws, 3 * K + 6))
    ll_chain = []
    lam_init, lambdas, mus = init_state(x, t_x, T_cal)
    eta = np.ones(N)
    hyper["beta_0"][0, 0] = math.log(lambdas.mean())
    hyper["beta_0"][0, 1] = math.log(mus.mean())
    hyper["beta_0"][0, 2] = log_s_mean
    z = np.ones(N, dtype=bool)
    tau = T_cal + 1.0
    beta, Sigma = hyper["beta_0"], hyper["gamma_00"].copy()
    store_idx = -1
    tot = burnin + mcmc if n_sweeps is None else n_sweeps
    for step in range(1, tot + 1):
        if trace and step % trace == 0:
            print(f"chain {chain_id} | step {step}/{burnin + mcmc}")
        stream.begin_sweep()
        if stream.record:
            stream.tape[-1].update(beta_in=np.array(beta, copy=True), Sigma_in=Sigma.copy())
        z = draw_z(t_x, T_cal, lambdas, mus, stream)
        tau = draw_tau(t_x, T_cal, lambdas, mus, z, stream)
        lambdas, mus = draw_level_1(x, T_cal, X, lambdas, mus, z, tau, beta, Sigma, stream, n_mh_steps)
        eta = np.clip(eta, 1e-6, None)
        eta = np.exp(draw_eta(log_s, X, beta, Sigma, omega2, stream))
        beta, Sigma = draw_level_2(
            X, np.column_stack([np.log(lambdas), np.log(mus), np.log(eta)]), hyper, stream)
        if is_stored(step, burnin, thin):
            store_idx += 1
            lambdas = np.exp(np.log(lambdas))
            mus = np.exp(np.log(mus))
            lvl1[store_idx, :, 0] = lambdas
            lvl1[store_idx, :, 1] = mus
            lvl1[store_idx, :, 2] = tau
            lvl1[store_idx, :, 4] = eta
            lvl1[store_idx, :, 3] = z.astype(float)
            lvl2[store_idx, : 3 * K] = beta.T.ravel()
            lvl2[store_idx, -6:] = [Sigma[0, 0], Sigma[0, 1], Sigma[0, 2],
                                    Sigma[1, 1], Sigma[1, 2], Sigma[2, 2]]
            ll_chain.append(np.mean(lik_terms(x, T_cal, lambdas, mus, z, tau)))
        if stream.record:
            st = stream.tape[-1]
            st.update(z=z.copy(), tau=tau.copy(), lam=lambdas.copy(), mu=mus.copy(), eta=eta.copy())
        if on_sweep is not None:
            on_sweep(step)
    return dict(level_1=lvl1, level_2=lvl2, log_likelihood=np.array(ll_chain))


# ---------------------------------------------------------------------------
# Public oracle entry points (same signatures as the reference)
# ---------------------------------------------------------------------------
def mcmc_draw_parameters(cal_cbs, covariates=None, mcmc=2500, burnin=500, thin=50, chains=2,
                         seed=None, trace=100, n_mh_steps=20, *, record=False, n_sweeps=None):
    """bi:437-504."""
    if covariates is None:
        covariates = []
    for col in ("x", "t_x", "T_cal"):
        if col not in cal_cbs:
            raise ValueError(f"cal_cbs missing required column '{col}'")
    if not all(col in cal_cbs for col in covariates):
        raise ValueError("some covariate columns not in cal_cbs")
    cbs, X = design_matrix(cal_cbs, covariates)
    K = X.shape[1]
    hyper = default_hyper(K, 2)
    x = cbs["x"].to_numpy()
    t_x = cbs["t_x"].to_numpy()
    T_cal = cbs["T_cal"].to_numpy()
    l1, l2, lls, tapes = [], [], [], []
    for ch in range(chains):
        stream = Stream(np.random.default_rng(None if seed is None else seed + ch), record)
        d = run_chain_bi(ch + 1, x, t_x, T_cal, X,
                         {k: v.copy() if isinstance(v, np.ndarray) else v for k, v in hyper.items()},
                         mcmc, burnin, thin, stream, trace, n_mh_steps, n_sweeps)
        l1.append(d["level_1"]); l2.append(d["level_2"]); lls.append(d["log_likelihood"])
        tapes.append(stream.tape)
    out = dict(level_1=l1, level_2=l2,
               log_likelihood=np.mean(np.concatenate(lls)) if sum(map(len, lls)) else np.nan)
    if record:
        out["tape"] = tapes
    return out


def mcmc_draw_parameters_rfm_m(cal_cbs, covariates=None, mcmc=2500, burnin=500, thin=50, chains=2,
                               seed=None, trace=100, n_mh_steps=20, *, record=False, n_sweeps=None):
    """tri:580-657 (no column validation in the reference; needs ``log_s``)."""
    if covariates is None:
        covariates = []
    cbs, X = design_matrix(cal_cbs, covariates)
    K = X.shape[1]
    hyper = default_hyper(K, 3)
    x = cbs["x"].to_numpy()
    t_x = cbs["t_x"].to_numpy()
    T_cal = cbs["T_cal"].to_numpy()
    log_s = cbs["log_s"].to_numpy()
    omega2 = cbs["log_s"].var()
    log_s_mean = cbs["log_s"].mean()
    l1, l2, lls, tapes = [], [], [], []
    for ch in range(chains):
        stream = Stream(np.random.default_rng(None if seed is None else seed + ch), record)
        d = run_chain_tri(ch + 1, x, t_x, T_cal, log_s, X,
                          {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in hyper.items()},
                          mcmc, burnin, thin, stream, trace, n_mh_steps, n_sweeps,
                          omega2=omega2, log_s_mean=log_s_mean)
        l1.append(d["level_1"]); l2.append(d["level_2"]); lls.append(d["log_likelihood"])
        tapes.append(stream.tape)
    out = {"level_1": l1, "level_2": l2,
           "log_likelihood": float(np.mean(np.concatenate(lls, axis=0))) if sum(map(len, lls)) else float("nan")}
    if record:
        out["tape"] = tapes
    return out
