"""GPU statistical parity of the Philox-mode sampler with the reference.

The reference's PCG64 stream cannot be reproduced by a parallel counter-based RNG, so parity in
production mode is distributional: the fixtures hold per-customer posterior
summaries of M = 8 independent chains of the reference (oracle, bitwise equal to it), and the
GPU's M chains must agree within Monte-Carlo tolerance.  The published Table 3 (config 1) is a
second, looser pin.
"""
import json
import os

import numpy as np
import pytest
from scipy.special import gammaln

from tests.helpers import GOLDEN, cdnow, golden

pytestmark = pytest.mark.gpu

SD_FLOOR = dict(log_lambda=1e-3, log_mu=1e-3, p_alive=2e-3, lam=1e-5, log_eta=1e-3)


def _run_envelope(name, M=16, seed=777):
    from mcmc_clv_model_amd import mcmc_draw_parameters, mcmc_draw_parameters_rfm_m
    f = golden(f"envelope_{name}.npz")
    covs = [str(c) for c in f["covariates"]]
    fn = mcmc_draw_parameters if str(f["kind"]) == "bi" else mcmc_draw_parameters_rfm_m
    data = str(f["data"]) if "data" in f.files else "abe"
    kw = dict(mcmc=int(f["mcmc"]), burnin=int(f["burnin"]), thin=1, chains=M, seed=seed, trace=0)
    if data in ("full", "synthetic"):  # 20k+ customers: the on-device running means (summary sink)
        if data == "synthetic":
            from mcmc_clv_model_amd.data import synthetic_cbs
            df = synthetic_cbs(int(f["data_n"]), int(f["data_K"]), int(f["data_D"]), seed=int(f["data_seed"]))
            assert frame_sha256(df) == str(f["data_sha256"]), "synthetic envelope data differ from the fixture's"
        else:
            df = cdnow("full")
        d = fn(df, covs, draw_sink="summary", **kw)
        sm = d["summary"]
        assert sm["n_draws"] == int(f["mcmc"])
        st = dict(log_lambda=sm["log_lambda"], log_mu=sm["log_mu"], p_alive=sm["z"], lam=sm["lambda"])
        if "log_eta" in sm:
            st["log_eta"] = sm["log_eta"]
        return f, st, d
    d = fn(cdnow("abe"), covs, **kw)
    stats = dict(log_lambda=[], log_mu=[], p_alive=[], lam=[], log_eta=[])
    for l1 in d["level_1"]:
        stats["log_lambda"].append(np.log(l1[:, :, 0]).mean(0))
        stats["log_mu"].append(np.log(l1[:, :, 1]).mean(0))
        stats["p_alive"].append(l1[:, :, 3].mean(0))
        stats["lam"].append(l1[:, :, 0].mean(0))
        if l1.shape[2] == 5:
            stats["log_eta"].append(np.log(l1[:, :, 4]).mean(0))
    return f, {k: np.stack(v) for k, v in stats.items() if v}, d


def frame_sha256(df):
    import hashlib
    h = hashlib.sha256()
    for c in df.columns:
        h.update(c.encode())
        h.update(np.ascontiguousarray(df[c].to_numpy()).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("name", ["c1_bi_k1", "abe_bi_k2", "abe_tri_k3", "full_bi_k2", "full_tri_k3",
                                  "synth_bi_k5", "synth_tri_k9"])
def test_posterior_envelope_vs_reference_ensemble(name):
    """Population means within 4 standard errors of the chain-to-chain spread (the common shift of
    every customer that the slowly mixing hyper-parameters cause); per customer, after that common
    shift is removed, |z| <= 4 with z = (mean_gpu - mean_ref) / sqrt(sd_ref^2/M + sd_gpu^2/M) for
    >= 99% of customers; per level-2 parameter, the mean of the chains' posterior medians differs by
    <= 4.5 two-sample standard errors (M = 16 vs 16 chains).
    Calibration (tools/envelope_ref_calibration.py, tools/envelope_seeds.py): three further 16-chain
    ensembles of the reference itself score, on c1 (M1, 2000 + 2000 sweeps), mean per-customer z
    -0.7 / -2.0 / -1.4 against the fixture's ensemble and population z down to -3.5 — so the
    UNcentred per-customer fraction fails for the reference itself (0.958, 0.988) while the centred
    one stays >= 0.991; five GPU ensembles score centred >= 0.997, population |z| <= 2.7.  Two
    independent 8-chain reference ensembles also differ by up to |z| = 2.8 on Sigma01/Sigma11.
    full_bi_k2 / full_tri_k3 are c2 and c3 (full CDNOW, 23,570 customers, their covariates) at
    reduced length (1000 + 1000 sweeps; oracle re-pinned bitwise to the reference on these exact
    inputs, oracle_pin_full.json); the GPU side keeps its per-customer means on device (summary
    sink) — the production path of the 1M/10M configurations.  synth_bi_k5 / synth_tri_k9 are the
    c4 / c5 models (U(-1,1) covariates, K = 5 bivariate, K = 9 trivariate) on 20,000
    synthetic customers at the same reduced length — the covariate counts that select the c4 / c5
    kernel instances (oracle re-pinned bitwise on these inputs, oracle_pin_synth.json)."""
    f, g, d = _run_envelope(name)
    M_ref = int(f["M"])
    for k, v in g.items():
        M = v.shape[0]
        m_g, s_g = v.mean(0), v.std(0, ddof=1)
        m_r, s_r = f[k + "_mean"], f[k + "_sd"]
        se = np.sqrt(np.maximum(s_r, SD_FLOOR[k]) ** 2 / M_ref + np.maximum(s_g, SD_FLOOR[k]) ** 2 / M)
        z = (m_g - m_r) / se
        frac = np.mean(np.abs(z - z.mean()) <= 4.0)  # the common shift is the population test below
        assert frac >= 0.99, f"{name}/{k}: only {frac:.4f} of customers within 4 sigma (mean z {z.mean():+.2f})"
        pop_r = f[k + "_chains"]
        pop_g = v.mean(1)
        se_pop = np.sqrt(pop_r.var(ddof=1) / M_ref + pop_g.var(ddof=1) / M)
        assert abs(pop_g.mean() - pop_r.mean()) <= 4 * se_pop + 1e-12, (k, pop_g.mean(), pop_r.mean(), se_pop)
    med_g = np.median(np.stack(d["level_2"]), axis=1)      # (M, n_params) chain medians
    med_r = f["level2_median"]
    se = np.sqrt(med_g.var(0, ddof=1) / len(med_g) + med_r.var(0, ddof=1) / len(med_r))
    z = (med_g.mean(0) - med_r.mean(0)) / np.maximum(se, 1e-12)
    assert np.all(np.abs(z) <= 4.5), (np.abs(z).round(2), med_g.mean(0), med_r.mean(0))


def _table3():
    t = json.load(open(os.path.join(GOLDEN, "published_table3.json")))["Table 3"]
    rows = {r.get("A"): r for r in t}
    q = lambda label: [rows[label][c] for c in ("B", "C", "D")]  # noqa: E731  (HB M1 column)
    return dict(beta_l0=q("Purchase rate log(λ) - Intercept"), beta_m0=q("Dropout rate log(μ) - Intercept"),
                s00=q("sigma^2_λ = var[log λ]"),
                s01=q("sigma^2_μ = var[log μ]"),      # mislabelled in the sheet: column holds Sigma01
                s11=q("sigma_λ_μ = cov[log λ, log μ]"),  # ... and this one Sigma11
                corr=q("Correlation computed from Γ₀"), loglik=rows["Marginal log-likelihood"]["C"])


def test_published_table3_config1():
    """Config 1 exactly as run_mcmc_abe.py:61-71 (M1, 4 chains, burnin 10000, 4000 draws, seed 42).
    Chain-0 level-2 quantiles (analysis_abe.py:146) vs abe_replication.xlsx Table 3 "HB M1": each
    of our medians lies inside the published 95% interval and each published median inside ours;
    the marginal log-likelihood (chain_total_loglik, analysis_bi_helpers.py:52-72) within 1%."""
    from mcmc_clv_model_amd import mcmc_draw_parameters
    cbs = cdnow("abe")
    d = mcmc_draw_parameters(cbs, [], mcmc=4000, burnin=10000, thin=1, chains=4, seed=42, trace=0)
    l2 = d["level_2"][0]
    corr = l2[:, -2] / np.sqrt(l2[:, -3] * l2[:, -1])
    ours = dict(beta_l0=l2[:, 0], beta_m0=l2[:, 1], s00=l2[:, 2], s01=l2[:, 3], s11=l2[:, 4], corr=corr)
    pub = _table3()
    for k, v in ours.items():
        q = np.percentile(v, [2.5, 50, 97.5])
        p = pub[k]
        assert p[0] <= q[1] <= p[2], (k, q, p)
        assert q[0] <= p[1] <= q[2], (k, q, p)
    x = cbs["x"].to_numpy()
    total_loglik = float(d["log_likelihood"]) * len(cbs) - gammaln(x + 1).sum()
    assert abs(total_loglik - pub["loglik"]) <= 0.01 * abs(pub["loglik"]), (total_loglik, pub["loglik"])


# ---------------------------------------------------------------------------------------------
# Invariance of the SHIPPED MH step (verdict r3: the production step, not the replay instance)
def _target_lp(ll, lm, x, z, w, m, P):
    """bi:291-310 for one customer (K = 1 mean row m, precision P), up to a constant; Q3 cap."""
    dl, dm = ll - m[0], lm - m[1]
    with np.errstate(over="ignore", invalid="ignore"):
        lp = x * ll + (1 - z) * lm - w * (np.exp(ll) + np.exp(lm)) - 0.5 * (P[0, 0] * dl * dl + 2 * P[0, 1] * dl * dm
                                                                              + P[1, 1] * dm * dm)
    return np.where(lm > 5.0, -np.inf, lp)


def _exact_sample(n, x, z, w, m, P, rng):
    """n exact draws of the customer's (log lambda, log mu) target by rejection from a wide
    Student-t(4) envelope around the grid mode (the bound M taken on a fine grid x 1.5)."""
    g = np.linspace(-16, 8, 1201)
    LL, LM = np.meshgrid(g, g, indexing="ij")
    lp = _target_lp(LL, LM, x, z, w, m, P)
    i = np.unravel_index(np.argmax(lp), lp.shape)
    mode = np.array([LL[i], LM[i]])
    prob = np.exp(lp - lp.max())
    mu = np.array([(prob * LL).sum(), (prob * LM).sum()]) / prob.sum()
    cov = np.cov(np.stack([LL.ravel(), LM.ravel()]), aweights=prob.ravel())
    Sc = 4.0 * cov
    Si = np.linalg.inv(Sc)
    ldet = np.log(np.linalg.det(Sc))

    def lq(a, b):  # bivariate t(4) log density (up to its constant, consistently)
        d = np.stack([a - mu[0], b - mu[1]], -1)
        qf = np.einsum("...i,ij,...j->...", d, Si, d)
        return -0.5 * ldet - 3.0 * np.log1p(qf / 4.0)
    logM = np.max(lp - lp.max() - lq(LL, LM)) + np.log(1.5)
    out = []
    got = 0
    Lc = np.linalg.cholesky(Sc)
    while got < n:
        k = 4 * (n - got) + 1000
        y = rng.standard_normal((k, 2)) @ Lc.T / np.sqrt(rng.chisquare(4, (k, 1)) / 4.0) + mu
        la = _target_lp(y[:, 0], y[:, 1], x, z, w, m, P) - lp.max() - lq(y[:, 0], y[:, 1]) - logM
        assert np.nanmax(la[np.isfinite(la)]) <= 0.0, "envelope bound violated"
        acc = np.log(rng.random(k)) < la
        out.append(y[acc])
        got += int(acc.sum())
    return np.concatenate(out)[:n], (LL, LM, prob), mode


@pytest.mark.parametrize("case", ["alive", "churned"])
def test_shipped_mh_step_preserves_the_target(case):
    """The production MH step (kernels.hip mh_step: fp32 Student-t(3) proposal by the shipped
    t3_f32 transform, the kernels' own fp32 log2 U (v_log_f32), table exp, accept iff pm <= 5 and plp > cur + ln2 log2 U)
    leaves the reference's level-1 target (bi:291-310) invariant: 400,000 exact draws of one
    customer's (log lambda, log mu) posterior (rejection sampling, numpy) go through 20 steps of the
    device step with the device's own Philox variates (clv_debug_variates: the sweep kernels' t_l,
    t_m and log2 of the accept uniforms, all formed on the device as the sweeps form them); the moments after the steps must equal the target's (grid
    quadrature) within 5 standard errors.  The same test with the accept threshold shifted by
    ln 2 * 0.15 (the acceptance ratio scaled by 2^0.15, +11%) must fail it — the test's power (a CPU
    simulation of this test flags a 2^0.05 bias at 5-7 standard errors, 2^0.02 at 3.5-5)."""
    import ctypes

    from mcmc_clv_model_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(31 if case == "alive" else 32)
    S = np.array([[1.37, 0.33], [0.33, 3.80]])  # Table 3's HB M1 medians (Sigma)
    P = np.linalg.inv(S)
    m = np.array([-3.5, -3.7])
    x, z, T, tau = (3, 1, 39.0, 39.0) if case == "alive" else (5, 0, 39.0, 12.5)
    w = T if z else tau
    n, steps = 400_000, 20
    pts, (LL, LM, prob), _ = _exact_sample(n, x, z, w, m, P, rng)
    pr = prob / prob.sum()
    exact = dict(ll=(pr * LL).sum(), lm=(pr * LM).sum(), ll2=(pr * LL * LL).sum(), lm2=(pr * LM * LM).sum(),
                 llm=(pr * LL * LM).sum())

    tl = np.empty((steps, n), np.float32)
    tm = np.empty((steps, n), np.float32)
    ua = np.empty((steps, n), np.float32)
    log2u = np.empty((steps, n), np.float32)  # the kernels' own log2 U (v_log_f32), verdict r4 #4
    dummy = [np.empty(n) for _ in range(4)]
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
    dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    assert L.clv_debug_variates(4242, 0, 7, n, steps, fp(tl), fp(tm), fp(ua), *[dp(d) for d in dummy],
                                fp(log2u)) == 0

    xs = np.full(n, x, np.int32)
    zs = np.full(n, z, np.uint8)
    Ts, taus = np.full(n, T), np.full(n, tau)
    mean = np.ascontiguousarray(np.tile(m, (n, 1)))
    prec = np.array([P[0, 0], P[0, 1], P[1, 1]])
    scale = np.array([S[0, 0], S[1, 1]])

    def run(shift):
        cur = np.ascontiguousarray(pts.copy())
        out = np.zeros((n, 7))
        for j in range(steps):
            t3 = np.ascontiguousarray(np.stack([tl[j], tm[j]], -1))
            lu = np.ascontiguousarray((log2u[j] + shift).astype(np.float32))
            assert L.clv_debug_mh_step(n, xs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       zs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), dp(Ts), dp(taus), dp(mean),
                                       dp(prec), dp(cur), fp(t3), dp(scale), fp(lu), dp(out)) == 0
            cur = np.ascontiguousarray(out[:, 4:6])
        return cur, float(np.mean(out[:, 4] != pts[:, 0]))

    def zscores(a):
        ll, lm = a[:, 0], a[:, 1]
        zs_ = {}
        for k, v in dict(ll=ll, lm=lm, ll2=ll * ll, lm2=lm * lm, llm=ll * lm).items():
            zs_[k] = (v.mean() - exact[k]) / (v.std() / np.sqrt(n))
        return zs_

    z_in = zscores(pts)
    assert max(abs(v) for v in z_in.values()) < 5, z_in  # the exact sample is exact
    after, moved = run(0.0)
    assert moved > 0.3, moved  # the chain moves
    z_out = zscores(after)
    assert max(abs(v) for v in z_out.values()) < 5, z_out
    biased, _ = run(-0.15)  # accept ratio x 2^0.15: must be detected
    z_b = zscores(biased)
    assert max(abs(v) for v in z_b.values()) > 5, z_b
