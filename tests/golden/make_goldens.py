"""Generate the committed golden fixtures under tests/golden/ (run in the build container only).

It imports the reference (lucagem29/mcmc_clv_model at /root/reference, read-only, with
PYTHONDONTWRITEBYTECODE so nothing is written there), first checks that the CPU oracle
(oracle/ref_cpu.py) is BITWISE equal to the reference on several configurations, and only then
writes fixtures.  The reference never travels to the GPU box; these fixtures (data, not code)
do.

Fixtures written:
  cdnow_{abe,full}_cbs.npz   CBS columns of data/processed/cdnow_{abe,full}CBS.csv (data inputs)
  philox_kat.json            Random123 Philox4x32-10 known-answer vectors (+ extra vectors)
  formulas.npz               G1: p_alive / tau / log_posterior / level-2 algebra from the reference
  replay_*.npz               G2: recorded variates + the reference's outputs for replay parity
  envelope_*.npz             G3: per-customer posterior summaries over M independent reference chains
                             (abe subset: c1/bi K=2/tri K=3; full CDNOW: c2 and c3 at reduced length)
  oracle_pin_full.json       the bitwise oracle-vs-reference checks on the full CDNOW c2/c3 inputs
  published_table3.json      abe_replication.xlsx "Table 3" (published loose pins)
  oracle_pin.json            the bitwise oracle-vs-reference checks that passed
  analysis_abe400.npz        row f: the reference's analysis helpers (draw_future_transactions bi/tri,
                             post_mean_*, chain_total_loglik, compute_table4) on fixed draws
  analysis_pin.json          the oracle/analysis_cpu.py-vs-reference checks that passed
  elog_abe.npz               row f4: cdnow_abeElog.csv and the reference elog2cbs outputs (W with
                             hold-out, D without, W without a sales column)
  generator_bi.npz           row f4: a 20,000-customer sample of the reference's generate_pareto_abe

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py [--skip-envelope]
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import re
import sys
import zipfile
from multiprocessing import Pool
from xml.etree import ElementTree as ET

os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
sys.dont_write_bytecode = True

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

from oracle import philox as oph  # noqa: E402
from oracle import ref_cpu as orc  # noqa: E402

DATA_COLS = ["x", "t_x", "T_cal", "sales", "first_sales_scaled", "age_scaled", "gender_binary"]


def ref_modules():
    sys.path.insert(0, REF)
    from src.models.bivariate import mcmc as rbi  # noqa: E402
    from src.models.trivariate import mcmc as rtri  # noqa: E402
    return rbi, rtri


def load_cbs(name):
    df = pd.read_csv(os.path.join(REF, "data", "processed", f"cdnow_{name}CBS.csv"))
    return df


def prepare(df):
    """Driver-side columns: log_s (tri run_mcmc_full.py:60-67), gender_F (tri run_mcmc_abe.py:100-105)."""
    df = df.copy()
    with np.errstate(divide="ignore"):
        df["log_s"] = np.log(df["sales"] / (df["x"] + 1)).replace(-np.inf, 0.0).fillna(0.0)
    df["gender_F"] = 1 - df["gender_binary"]
    return df


def bitwise_equal(a, b):
    if isinstance(a, dict):
        return all(bitwise_equal(a[k], b[k]) for k in ("level_1", "level_2", "log_likelihood"))
    if isinstance(a, list):
        return len(a) == len(b) and all(bitwise_equal(x, y) for x, y in zip(a, b))
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype == np.float64:
        return bool(np.array_equal(a.view(np.uint64), b.view(np.uint64)))
    return bool(np.array_equal(a, b))


# ---------------------------------------------------------------------------------------------
def pin_oracle(rbi, rtri):
    df = prepare(load_cbs("abe"))
    checks = []
    cases = [
        ("bi", [], 256, 7, dict(mcmc=6, burnin=4, thin=2, chains=2)),
        ("bi", ["first_sales_scaled"], 300, 11, dict(mcmc=5, burnin=3, thin=1, chains=2)),
        ("bi", ["first_sales_scaled", "age_scaled", "gender_F"], 200, 3, dict(mcmc=4, burnin=2, thin=3, chains=1)),
        ("tri", [], 256, 5, dict(mcmc=6, burnin=2, thin=2, chains=2)),
        ("tri", ["gender_F", "age_scaled"], 300, 9, dict(mcmc=5, burnin=2, thin=1, chains=2)),
        ("bi", [], 2357, 42, dict(mcmc=3, burnin=3, thin=1, chains=1)),
    ]
    for kind, covs, n, seed, kw in cases:
        sub = df.iloc[:n].copy()
        if kind == "bi":
            a = rbi.mcmc_draw_parameters(sub, covs, seed=seed, trace=0, **kw)
            b = orc.mcmc_draw_parameters(sub, covs, seed=seed, trace=0, **kw)
        else:
            a = rtri.mcmc_draw_parameters_rfm_m(sub, covs, seed=seed, trace=0, **kw)
            b = orc.mcmc_draw_parameters_rfm_m(sub, covs, seed=seed, trace=0, **kw)
        ok = bitwise_equal(a, b)
        checks.append(dict(kind=kind, covariates=covs, n=n, seed=seed, **kw, bitwise_equal=ok))
        print("pin", kind, covs, n, ok)
        if not ok:
            raise SystemExit("oracle is NOT bitwise equal to the reference; refusing to write fixtures")
    # the reference's own smoke test (bi:553-559) on its synthetic generator
    beta = np.array([[0.18, -2.5]])
    gamma = np.array([[0.05, 0.1], [0.1, 0.2]])
    cbs, _ = rbi.generate_pareto_abe(50, 32, 32, beta, gamma, seed=42)
    a = rbi.mcmc_draw_parameters(cbs, mcmc=100, burnin=50, thin=10, chains=1, trace=0, seed=123)
    b = orc.mcmc_draw_parameters(cbs, mcmc=100, burnin=50, thin=10, chains=1, trace=0, seed=123)
    ok = bitwise_equal(a, b)
    checks.append(dict(kind="bi_smoke_bi553", n=50, seed=123, bitwise_equal=ok,
                       level2_shape=list(a["level_2"][0].shape)))
    print("pin smoke", ok, a["level_2"][0].shape)
    if not ok:
        raise SystemExit("oracle differs from the reference on the reference's smoke test")
    np.savez_compressed(os.path.join(HERE, "smoke_bi553.npz"),
                        x=cbs["x"].to_numpy(np.int64), t_x=cbs["t_x"].to_numpy(), T_cal=cbs["T_cal"].to_numpy(),
                        level_2=a["level_2"][0], level_1=a["level_1"][0], log_likelihood=a["log_likelihood"])
    with open(os.path.join(HERE, "oracle_pin.json"), "w") as f:
        json.dump(dict(numpy=np.__version__, pandas=pd.__version__, checks=checks), f, indent=1)


# ---------------------------------------------------------------------------------------------
def write_data():
    for name in ("abe", "full"):
        df = load_cbs(name)
        np.savez_compressed(os.path.join(HERE, f"cdnow_{name}_cbs.npz"),
                            **{c: (df[c].to_numpy(np.int64) if c in ("x", "gender_binary") else df[c].to_numpy(np.float64))
                               for c in DATA_COLS})
        print("data", name, len(df))


def write_philox_kat():
    kat = [
        dict(ctr=[0, 0, 0, 0], key=[0, 0], out=["6627e8d5", "e169c58d", "bc57ac4c", "9b00dbd8"]),
        dict(ctr=[0xffffffff] * 4, key=[0xffffffff] * 2, out=["408f276d", "41c83b0e", "a20bc7c6", "6d5451fd"]),
        dict(ctr=[0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], key=[0xa4093822, 0x299f31d0],
             out=["d16cfe09", "94fdcceb", "5001e420", "24126ea1"]),
    ]
    for k in kat:
        got = oph.philox4x32_10(np.array(k["ctr"], np.uint32), k["key"][0], k["key"][1])
        assert [f"{v:08x}" for v in got] == k["out"], "oracle Philox fails Random123 KAT"
    rng = np.random.default_rng(2025)
    extra_ctr = rng.integers(0, 2 ** 32, size=(64, 4), dtype=np.uint64).astype(np.uint32)
    extra_key = rng.integers(0, 2 ** 32, size=2, dtype=np.uint64).astype(np.uint32)
    extra_out = oph.philox4x32_10(extra_ctr, extra_key[0], extra_key[1])
    with open(os.path.join(HERE, "philox_kat.json"), "w") as f:
        json.dump(dict(random123=kat, extra=dict(key=[int(v) for v in extra_key], ctr=extra_ctr.tolist(),
                                                 out=extra_out.tolist())), f)
    print("philox kat ok")


# ---------------------------------------------------------------------------------------------
def write_formulas(rbi, rtri):
    """G1: exact outputs of the reference's own functions on random inputs (incl. edge cases)."""
    rng = np.random.default_rng(7)
    out = {}
    n = 1024
    tx = rng.uniform(0, 38, n) * (rng.random(n) < 0.7)
    T = np.maximum(tx + rng.uniform(0, 10, n), 27.0)
    lam = np.exp(rng.uniform(-8, 3, n))
    mu = np.exp(rng.uniform(-10, 2, n))
    cbs = pd.DataFrame(dict(t_x=tx, T_cal=T))
    g = np.random.default_rng(11)
    gc = copy.deepcopy(g)
    z = rbi.draw_z(cbs, lam, mu, g)
    u = gc.random(n)
    out.update(z_tx=tx, z_T=T, z_lam=lam, z_mu=mu, z_u=u, z_out=z, z_p=orc.p_alive(tx, T, lam, mu))
    assert np.array_equal(orc.p_alive(tx, T, lam, mu) > u, z)
    # tau
    g = np.random.default_rng(12)
    gc = copy.deepcopy(g)
    tau = rbi.draw_tau(cbs, lam, mu, z, g)
    st = orc.Stream(gc, record=True)
    st.begin_sweep()
    tau2 = orc.draw_tau(tx, T, lam, mu, z, st)
    assert np.array_equal(tau.view(np.uint64), tau2.view(np.uint64))
    out.update(tau_out=tau, tau_v=st.tape[0]["v_tau"])
    # log posterior edge cases (bi:291-310): lm > 5 -> -inf, -inf - -inf -> NaN in the ratio
    ll = rng.uniform(-75, 75, n)
    lm = rng.uniform(-75, 8, n)
    xx = rng.integers(0, 40, n)
    zz = rng.random(n) < 0.5
    mv = rng.normal(-3.5, 1, (n, 2))
    S = np.array([[1.4, 0.2], [0.2, 2.5]])
    with np.errstate(over="ignore", invalid="ignore"):
        lp = orc.log_posterior(ll, lm, xx, zz, T, tau, mv, np.linalg.inv(S))
    out.update(lp_ll=ll, lp_lm=lm, lp_x=xx, lp_z=zz, lp_T=T, lp_tau=tau, lp_mv=mv, lp_S=S, lp_out=lp)
    # level-2 algebra for K in {1,2,5,9}, D in {2,3}, through the reference's own _draw_level_2
    for D in (2, 3):
        for K in (1, 2, 5, 9):
            N = 500
            X = np.column_stack([np.ones(N), rng.uniform(-1, 1, (N, K - 1))])
            Y = rng.normal([-3.5, -3.7, 3.2][:D], 1.0, (N, D))
            hyper = orc.default_hyper(K, D)
            hyper["beta_0"][0, :] = [-3.4, -3.6, 3.1][:D]
            g = np.random.default_rng(100 + 10 * D + K)
            gc = copy.deepcopy(g)
            if D == 2:
                beta_r, Sigma_r = rbi._draw_level_2(X, Y[:, 0], Y[:, 1], hyper, g)
            else:
                beta_r, Sigma_r = rtri._draw_level_2(X, Y[:, 0], Y[:, 1], Y[:, 2], hyper, g)
            st = orc.Stream(gc, record=True)
            st.begin_sweep()
            beta_o, Sigma_o = orc.draw_level_2(X, Y, hyper, st)
            assert np.array_equal(beta_o, beta_r) and np.array_equal(Sigma_o, Sigma_r)
            V, Bh, Sn, nun = orc.level2_posterior(X, Y, hyper)
            t = st.tape[0]
            p = f"l2_D{D}_K{K}_"
            out.update({p + "X": X, p + "Y": Y, p + "B0": hyper["beta_0"], p + "nu0": hyper["nu_00"],
                        p + "V": V, p + "Bhat": Bh, p + "Sn": Sn, p + "nun": nun,
                        p + "iw_normal": t["iw_normal"], p + "iw_chi2": t["iw_chi2"], p + "mvn_z": t["mvn_z"],
                        p + "Sigma": Sigma_r, p + "beta": beta_r})
    # draw_eta (tri:306-333)
    N = 300
    X = np.column_stack([np.ones(N), rng.uniform(-1, 1, (N, 2))])
    log_s = rng.normal(3.2, 0.7, N)
    beta = rng.normal(0, 1, (3, 3))
    Sig = np.array([[1.4, 0.2, 0.1], [0.2, 2.5, 0.0], [0.1, 0.0, 0.5]])
    g = np.random.default_rng(5)
    gc = copy.deepcopy(g)
    cbs = pd.DataFrame(dict(intercept=1.0, c1=X[:, 1], c2=X[:, 2], log_s=log_s))
    eta_r = rtri.draw_eta(cbs, None, beta, Sig, 0.47, g, ["intercept", "c1", "c2"])
    st = orc.Stream(gc, record=True)
    st.begin_sweep()
    eta_o = orc.draw_eta(log_s, X, beta, Sig, 0.47, st)
    assert np.array_equal(eta_r, eta_o)
    out.update(eta_X=X, eta_log_s=log_s, eta_beta=beta, eta_Sigma=Sig, eta_omega2=0.47,
               eta_z=st.tape[0]["eta_z"], eta_out=eta_r)
    np.savez_compressed(os.path.join(HERE, "formulas.npz"), **out)
    print("formulas ok")


# ---------------------------------------------------------------------------------------------
def pack_tape(tape, n, S, D):
    """Pack the oracle's per-sweep recorded variates into the device replay layout
    (include/clvmcmc.h clv_set_replay_tape)."""
    stride = n * (2 + 3 * S + (1 if D == 3 else 0)) + 40
    out = np.zeros((len(tape), stride))
    for s, sw in enumerate(tape):
        o = out[s]
        o[0:n] = sw["u_z"]
        o[n:2 * n] = sw["v_tau"]
        for j in range(S):
            o[(2 + 3 * j) * n:(3 + 3 * j) * n] = sw["t_l"][j]
            o[(3 + 3 * j) * n:(4 + 3 * j) * n] = sw["t_m"][j]
            o[(4 + 3 * j) * n:(5 + 3 * j) * n] = sw["u_acc"][j]
        if D == 3:
            o[(2 + 3 * S) * n:(3 + 3 * S) * n] = sw["eta_z"]
        h = stride - 40
        nt = len(sw["iw_normal"])
        o[h:h + nt] = sw["iw_normal"]
        o[h + 3:h + 3 + len(sw["iw_chi2"])] = sw["iw_chi2"]
        o[h + 6:h + 6 + len(sw["mvn_noise"])] = sw["mvn_noise"]
    return out


SYNTH_COV_SEED = 4242  # the U(-1,1) covariate columns c1..c8 added to the abe rows of the K=5 / K=9 cases


def with_synthetic_covariates(df, n_cov, seed=SYNTH_COV_SEED):
    """c1..c{n_cov}: U(-1,1) covariates (the c4/c5 covariate model) on CDNOW rows."""
    df = df.copy()
    rng = np.random.default_rng(seed)
    cov = rng.uniform(-1.0, 1.0, size=(len(df), n_cov))
    for k in range(n_cov):
        df[f"c{k + 1}"] = cov[:, k]
    return df


def write_replay(rbi, rtri, only_names=None):
    df = prepare(load_cbs("abe"))
    cases = [
        # name, kind, covariates, N, S, chains, seed, mcmc (all stored: burnin 0, thin 1)
        ("bi_k1", "bi", [], 300, 5, 2, 42, 3),
        ("bi_k2", "bi", ["first_sales_scaled"], 256, 20, 1, 7, 3),
        ("tri_k3", "tri", ["gender_F", "age_scaled"], 200, 20, 1, 11, 3),
        ("bi_k1_s0", "bi", [], 64, 0, 1, 3, 2),
        # the c4 / c5 kernel instances (verdict r2 #1): bivariate K=5 (sweep_kernel_occ4<2,5>, covariates
        # in registers) and trivariate K=9 (sweep_kernel<3,9>, covariate rows in LDS); 384 customers =
        # one full and one half-filled 256-customer block
        ("bi_k5", "bi", [f"c{k}" for k in range(1, 5)], 384, 20, 1, 13, 3),
        ("tri_k9", "tri", [f"c{k}" for k in range(1, 9)], 384, 20, 1, 17, 3),
    ]
    for name, kind, covs, n, S, chains, seed, mcmc in cases:
        if only_names and name not in only_names:
            continue
        base = with_synthetic_covariates(df, 8) if covs and covs[0] == "c1" else df
        sub = base.iloc[:n].copy().reset_index(drop=True)
        kw = dict(mcmc=mcmc, burnin=0, thin=1, chains=chains, seed=seed, trace=0, n_mh_steps=S)
        fn_r = rbi.mcmc_draw_parameters if kind == "bi" else rtri.mcmc_draw_parameters_rfm_m
        fn_o = orc.mcmc_draw_parameters if kind == "bi" else orc.mcmc_draw_parameters_rfm_m
        ref = fn_r(sub, covs, **kw)
        ora = fn_o(sub, covs, **kw)
        assert bitwise_equal(ref, ora), name
        D = 2 if kind == "bi" else 3
        n_rec = mcmc + (1 if D == 2 else 0)  # bivariate: the draw after the last sweep belongs to sweep mcmc+1
        rec = fn_o(sub, covs, **dict(kw, mcmc=n_rec), record=True)
        tapes = np.stack([pack_tape(rec["tape"][c], n, S, D) for c in range(chains)])
        per_sweep_beta = np.stack([[sw["beta"] for sw in rec["tape"][c]] for c in range(chains)])
        per_sweep_sigma = np.stack([[sw["Sigma"] for sw in rec["tape"][c]] for c in range(chains)])
        cols = dict(x=sub["x"].to_numpy(np.int64), t_x=sub["t_x"].to_numpy(), T_cal=sub["T_cal"].to_numpy(),
                    log_s=sub["log_s"].to_numpy())
        for c in covs:
            cols["cov_" + c] = sub[c].to_numpy(np.float64)
        np.savez_compressed(
            os.path.join(HERE, f"replay_{name}.npz"), kind=kind, covariates=np.array(covs, dtype="U32"),
            D=D, S=S, chains=chains, seed=seed, mcmc=mcmc, n_tape_sweeps=n_rec, tape=tapes,
            level_1=np.stack(ref["level_1"]), level_2=np.stack(ref["level_2"]),
            log_likelihood=float(ref["log_likelihood"]), beta=per_sweep_beta, Sigma=per_sweep_sigma, **cols)
        print("replay", name, tapes.shape)


# ---------------------------------------------------------------------------------------------
SYNTH_ENVELOPE = {  # name -> (kind, K, D, data seed): 20,000 synthetic customers (c4 / c5 model)
    "synth_bi_k5": ("bi", 5, 2, 20251017),
    "synth_tri_k9": ("tri", 9, 3, 20251018),
}
SYNTH_ENVELOPE_N = 20_000


def synthetic_data(name):
    """The envelope's synthetic CBS: the product's vectorised generator (mcmc_clv_model_amd/data.py,
    plain numpy), regenerated bit for bit by the GPU test from the stored seed (sha256 checked)."""
    from mcmc_clv_model_amd.data import synthetic_cbs
    kind, K, D, seed = SYNTH_ENVELOPE[name]
    return synthetic_cbs(SYNTH_ENVELOPE_N, K, D, seed=seed)


def frame_sha256(df):
    import hashlib
    h = hashlib.sha256()
    for c in df.columns:
        h.update(c.encode())
        h.update(np.ascontiguousarray(df[c].to_numpy()).tobytes())
    return h.hexdigest()


def _envelope_chain(args):
    kind, covs, seed, burnin, mcmc = args[:5]
    data = args[5] if len(args) > 5 else "abe"
    os.environ["OMP_NUM_THREADS"] = "1"
    df = synthetic_data(data) if data in SYNTH_ENVELOPE else prepare(load_cbs(data))
    fn = orc.mcmc_draw_parameters if kind == "bi" else orc.mcmc_draw_parameters_rfm_m
    d = fn(df, covs, mcmc=mcmc, burnin=burnin, thin=1, chains=1, seed=seed, trace=0)
    l1 = d["level_1"][0]
    st = dict(log_lambda=np.log(l1[:, :, 0]).mean(0), log_mu=np.log(l1[:, :, 1]).mean(0),
              p_alive=l1[:, :, 3].mean(0), lam=l1[:, :, 0].mean(0))
    if kind == "tri":
        st["log_eta"] = np.log(l1[:, :, 4]).mean(0)
    return st, np.median(d["level_2"][0], axis=0), float(d["log_likelihood"])


def write_envelope(M=16, burnin=2000, mcmc=2000):
    cases = [("c1_bi_k1", "bi", []), ("abe_bi_k2", "bi", ["first_sales_scaled"]),
             ("abe_tri_k3", "tri", ["gender_F", "age_scaled"])]
    jobs = [(kind, covs, 1000 + m, burnin, mcmc) for _, kind, covs in cases for m in range(M)]
    with Pool(min(8, len(jobs))) as pool:  # 1 thread per process
        res = pool.map(_envelope_chain, jobs)
    for ci, (name, kind, covs) in enumerate(cases):
        rs = res[ci * M:(ci + 1) * M]
        keys = rs[0][0].keys()
        out = dict(kind=kind, covariates=np.array(covs, dtype="U32"), M=M, burnin=burnin, mcmc=mcmc)
        for k in keys:
            v = np.stack([r[0][k] for r in rs])
            out[k + "_mean"] = v.mean(0)
            out[k + "_sd"] = v.std(0, ddof=1)
            out[k + "_chains"] = v.mean(1)  # population mean per chain
        out["level2_median"] = np.stack([r[1] for r in rs])
        out["loglik"] = np.array([r[2] for r in rs])
        np.savez_compressed(os.path.join(HERE, f"envelope_{name}.npz"), **out)
        print("envelope", name)


def write_envelope_full(rbi, rtri, M=16, burnin=1000, mcmc=1000):
    """G3 at full size ("c2 and c3 at reduced length"): the full CDNOW CBS (23,570
    customers) with c2's covariate (bivariate K=2) and c3's (trivariate K=3).  First re-pins the
    oracle bitwise against the reference on these exact inputs (4 sweeps, 2 chains, every sweep
    stored), then runs M independent oracle chains of burnin + mcmc sweeps."""
    df = prepare(load_cbs("full"))
    cases = [("full_bi_k2", "bi", ["first_sales_scaled"]), ("full_tri_k3", "tri", ["gender_F", "age_scaled"])]
    pins = []
    for name, kind, covs in cases:
        kw = dict(mcmc=2, burnin=2, thin=1, chains=2, seed=7, trace=0)
        fn_r = rbi.mcmc_draw_parameters if kind == "bi" else rtri.mcmc_draw_parameters_rfm_m
        fn_o = orc.mcmc_draw_parameters if kind == "bi" else orc.mcmc_draw_parameters_rfm_m
        assert bitwise_equal(fn_r(df, covs, **kw), fn_o(df, covs, **kw)), name
        pins.append(dict(case=name, n=len(df), covariates=covs, **kw, bitwise=True))
        print("pinned", name)
    jobs = [(kind, covs, 3000 + m, burnin, mcmc, "full") for _, kind, covs in cases for m in range(M)]
    with Pool(min(8, len(jobs))) as pool:  # 1 thread per process
        res = pool.map(_envelope_chain, jobs, chunksize=1)
    for ci, (name, kind, covs) in enumerate(cases):
        rs = res[ci * M:(ci + 1) * M]
        out = dict(kind=kind, covariates=np.array(covs, dtype="U32"), M=M, burnin=burnin, mcmc=mcmc,
                   data=np.array("full"), seeds=np.array([3000 + m for m in range(M)]))
        for k in rs[0][0].keys():
            v = np.stack([r[0][k] for r in rs])
            out[k + "_mean"] = v.mean(0)
            out[k + "_sd"] = v.std(0, ddof=1)
            out[k + "_chains"] = v.mean(1)
        out["level2_median"] = np.stack([r[1] for r in rs])
        out["loglik"] = np.array([r[2] for r in rs])
        np.savez_compressed(os.path.join(HERE, f"envelope_{name}.npz"), **out)
        print("envelope", name)
    with open(os.path.join(HERE, "oracle_pin_full.json"), "w") as f:
        json.dump(dict(reference=REF, checks=pins), f, indent=1)


def write_envelope_synth(rbi, rtri, M=16, burnin=1000, mcmc=1000):
    """G3 for the c4 / c5 kernel instances (verdict r2 #1): 20,000 synthetic customers of the c4
    model (bivariate, K = 5) and the c5 model (trivariate, K = 9) — the covariate counts that select
    sweep_kernel_occ4<2,5> and the LDS-covariate sweep_kernel<3,9> — at reduced length.  The oracle
    is first re-pinned bitwise against the reference on these exact inputs (4 sweeps, 2 chains)."""
    pins = []
    names = list(SYNTH_ENVELOPE)
    for name in names:
        kind, K, D, dseed = SYNTH_ENVELOPE[name]
        df = synthetic_data(name)
        covs = [f"c{k}" for k in range(1, K)]
        kw = dict(mcmc=2, burnin=2, thin=1, chains=2, seed=7, trace=0)
        fn_r = rbi.mcmc_draw_parameters if kind == "bi" else rtri.mcmc_draw_parameters_rfm_m
        fn_o = orc.mcmc_draw_parameters if kind == "bi" else orc.mcmc_draw_parameters_rfm_m
        assert bitwise_equal(fn_r(df, covs, **kw), fn_o(df, covs, **kw)), name
        pins.append(dict(case=name, n=len(df), covariates=covs, data_seed=dseed, sha256=frame_sha256(df), **kw,
                         bitwise=True))
        print("pinned", name)
    jobs = [(SYNTH_ENVELOPE[name][0], [f"c{k}" for k in range(1, SYNTH_ENVELOPE[name][1])], 5000 + m, burnin, mcmc,
             name) for name in names for m in range(M)]
    with Pool(min(8, len(jobs))) as pool:  # 1 thread per process
        res = pool.map(_envelope_chain, jobs, chunksize=1)
    for ci, name in enumerate(names):
        kind, K, D, dseed = SYNTH_ENVELOPE[name]
        rs = res[ci * M:(ci + 1) * M]
        out = dict(kind=kind, covariates=np.array([f"c{k}" for k in range(1, K)], dtype="U32"), M=M, burnin=burnin,
                   mcmc=mcmc, data=np.array("synthetic"), data_seed=dseed, data_n=SYNTH_ENVELOPE_N, data_K=K,
                   data_D=D, data_sha256=np.array(frame_sha256(synthetic_data(name))),
                   seeds=np.array([5000 + m for m in range(M)]))
        for k in rs[0][0].keys():
            v = np.stack([r[0][k] for r in rs])
            out[k + "_mean"] = v.mean(0)
            out[k + "_sd"] = v.std(0, ddof=1)
            out[k + "_chains"] = v.mean(1)
        out["level2_median"] = np.stack([r[1] for r in rs])
        out["loglik"] = np.array([r[2] for r in rs])
        np.savez_compressed(os.path.join(HERE, f"envelope_{name}.npz"), **out)
        print("envelope", name)
    with open(os.path.join(HERE, "oracle_pin_synth.json"), "w") as f:
        json.dump(dict(reference=REF, checks=pins), f, indent=1)


# ---------------------------------------------------------------------------------------------
def read_xlsx_sheets(path):
    ns = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main"}
    rel_ns = "{http://schemas.openxmlformats.org/officeDocument/2006/relationships}id"
    z = zipfile.ZipFile(path)
    shared = []
    if "xl/sharedStrings.xml" in z.namelist():
        for si in ET.fromstring(z.read("xl/sharedStrings.xml")).findall("m:si", ns):
            shared.append("".join(t.text or "" for t in si.iter("{%s}t" % ns["m"])))
    wb = ET.fromstring(z.read("xl/workbook.xml"))
    rels = ET.fromstring(z.read("xl/_rels/workbook.xml.rels"))
    rmap = {r.get("Id"): r.get("Target") for r in rels}
    sheets = {}
    for sh in wb.find("m:sheets", ns):
        target = rmap[sh.get(rel_ns)]
        target = target.lstrip("/")
        target = target if target.startswith("xl/") else "xl/" + target
        rows = []
        for row in ET.fromstring(z.read(target)).iter("{%s}row" % ns["m"]):
            cells = {}
            for c in row.findall("m:c", ns):
                ref = c.get("r")
                col = re.match(r"[A-Z]+", ref).group(0)
                v = c.find("m:v", ns)
                val = None
                if c.get("t") == "s" and v is not None:
                    val = shared[int(v.text)]
                elif c.get("t") == "inlineStr":
                    val = "".join(t.text or "" for t in c.iter("{%s}t" % ns["m"]))
                elif v is not None:
                    try:
                        val = float(v.text)
                    except ValueError:
                        val = v.text
                cells[col] = val
            rows.append(cells)
        sheets[sh.get("name")] = rows
    return sheets


def write_published():
    sheets = read_xlsx_sheets(os.path.join(REF, "outputs", "excel", "abe_replication.xlsx"))
    with open(os.path.join(HERE, "published_table3.json"), "w") as f:
        json.dump({k: v for k, v in sheets.items() if "3" in k or "4" in k}, f, indent=0)
    print("published sheets", list(sheets))


# ---------------------------------------------------------------------------------------------
def write_analysis(rbi, rtri):
    """Row f fixtures: the reference's analysis helpers on fixed draws (bitwise-pinned oracle)."""
    sys.path.insert(0, REF)
    from src.models.utils import analysis_bi_helpers as rh  # noqa: E402
    from oracle import analysis_cpu as oan  # noqa: E402
    df = prepare(load_cbs("abe")).iloc[:400].copy()
    bi = rbi.mcmc_draw_parameters(df, [], mcmc=60, burnin=40, thin=2, chains=2, seed=5, trace=0)
    tri = rtri.mcmc_draw_parameters_rfm_m(df, [], mcmc=40, burnin=20, thin=2, chains=2, seed=6, trace=0)
    xs_bi = rbi.draw_future_transactions(df, bi, T_star=39.0, seed=42)
    xs_tri, sp_tri = rtri.draw_future_transactions(df, tri, T_star=39.0, seed=43)
    checks = dict(
        xstar_bi=bitwise_equal(xs_bi, oan.draw_future_transactions_bi(df, bi, 39.0, seed=42)),
        xstar_tri=all(bitwise_equal(a, b) for a, b in zip((xs_tri, sp_tri),
                                                         oan.draw_future_transactions_tri(df, tri, 39.0, seed=43))),
        post_mean_lambdas=bitwise_equal(rh.post_mean_lambdas(bi), oan.post_mean_lambdas(bi)),
        post_mean_mus=bitwise_equal(rh.post_mean_mus(bi), oan.post_mean_mus(bi)),
        chain_total_loglik=bitwise_equal(rh.chain_total_loglik(bi["level_1"], df),
                                         oan.chain_total_loglik(bi["level_1"], df)),
    )
    t4 = rh.compute_table4(bi, xs_bi)
    st = oan.table4_stats(bi)
    # the reference's Table 4 summary rows (Ave/Min/Max) from the oracle's per-customer columns
    checks["table4_ave_row"] = bool(np.isclose(float(t4.loc["Ave", "Mean(λ)"]), round(st["mean_lambda"].mean(), 3)))
    print("analysis pin", checks)
    if not all(checks.values()):
        raise SystemExit("analysis oracle differs from the reference; refusing to write fixtures")
    elog = pd.read_csv(os.path.join(REF, "data", "raw", "cdnow_abeElog.csv"), parse_dates=["date"])
    first = elog["date"].min()
    elog["week"] = ((elog["date"] - first) // pd.Timedelta("7D")).astype(int) + 1
    cust = pd.read_csv(os.path.join(REF, "data", "processed", "cdnow_abeCBS.csv"))["cust"].iloc[:400]
    birth = elog.groupby("cust")["week"].min().reindex(cust).to_numpy(np.float64)
    times = np.arange(1, int(elog["week"].max()) + 1, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "analysis_abe400.npz"),
                        x=df["x"].to_numpy(np.int64), t_x=df["t_x"].to_numpy(), T_cal=df["T_cal"].to_numpy(),
                        bi_level1=np.stack(bi["level_1"]), tri_level1=np.stack(tri["level_1"]),
                        xstar_bi=xs_bi, xstar_tri=xs_tri, spend_tri=sp_tri,
                        post_mean_lambdas=rh.post_mean_lambdas(bi), post_mean_mus=rh.post_mean_mus(bi),
                        chain_total_loglik=rh.chain_total_loglik(bi["level_1"], df),
                        table4=t4.to_numpy(dtype=object).astype(str), table4_index=np.array(t4.index.astype(str).tolist(), dtype=str),
                        table4_columns=np.array(t4.columns, dtype=str),
                        birth_week=birth, times=times,
                        tracking_ref=oan.weekly_tracking(bi, birth, times), **{f"t4_{k}": v for k, v in st.items()})
    with open(os.path.join(HERE, "analysis_pin.json"), "w") as f:
        json.dump(dict(checks=checks, note="reference helpers vs oracle/analysis_cpu.py on the same draws"), f, indent=1)


# ---------------------------------------------------------------------------------------------
def write_dataprep(rbi):
    """Row f4 fixtures: the reference's elog2cbs (utils/elog2cbs2param.py) on the CDNOW 1/10 event
    log, and a sample of its synthetic generator (bi:95-187)."""
    sys.path.insert(0, REF)
    from src.models.utils.elog2cbs2param import elog2cbs as ref_elog2cbs  # noqa: E402
    elog = pd.read_csv(os.path.join(REF, "data", "raw", "cdnow_abeElog.csv"))
    elog["date"] = pd.to_datetime(elog["date"])
    out = {}
    cases = {"hold": dict(units="W", T_cal="1997-09-30", T_tot="1998-06-30"),
             "nohold": dict(units="D", T_cal=None, T_tot=None)}
    for tag, kw in cases.items():
        cbs = ref_elog2cbs(elog, **kw)
        for c in cbs.columns:
            v = cbs[c]
            out[f"{tag}_{c}"] = v.to_numpy(dtype="datetime64[ns]").view(np.int64) if c == "first" else v.to_numpy()
    nos = ref_elog2cbs(elog[["cust", "date"]], units="W", T_cal="1997-09-30", T_tot="1998-06-30")
    for c in ("x", "sales", "sales_x", "x_star", "sales_star"):
        out[f"nosales_{c}"] = nos[c].to_numpy()
    np.savez_compressed(os.path.join(HERE, "elog_abe.npz"), cust=elog["cust"].to_numpy(np.int64),
                        date_ns=elog["date"].to_numpy(dtype="datetime64[ns]").view(np.int64),
                        sales=elog["sales"].to_numpy(np.float64), **out)
    beta = np.array([[0.18, -2.5], [0.3, -0.2]])
    gamma = np.array([[0.05, 0.1], [0.1, 0.2]])
    cbs, el = rbi.generate_pareto_abe(20000, 32.0, [20.0, 32.0], beta, gamma, seed=2025)
    np.savez_compressed(os.path.join(HERE, "generator_bi.npz"), beta=beta, gamma=gamma, T_cal_in=32.0,
                        T_star=np.array([20.0, 32.0]), n_elog=len(el),
                        **{c: cbs[c].to_numpy(np.float64) for c in cbs.columns})
    print("dataprep", {k: v.shape for k, v in out.items() if k.endswith("_x")}, len(cbs), len(el))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-envelope", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("--replay-names", default="", help="comma-separated subset of the replay cases")
    a = ap.parse_args()
    rbi, rtri = ref_modules()
    only = set(a.only.split(",")) if a.only else None
    steps = [("pin", lambda: pin_oracle(rbi, rtri)), ("data", write_data), ("philox", write_philox_kat),
             ("formulas", lambda: write_formulas(rbi, rtri)), ("replay", lambda: write_replay(rbi, rtri, set(a.replay_names.split(",")) if a.replay_names else None)),
             ("published", write_published), ("analysis", lambda: write_analysis(rbi, rtri)),
             ("dataprep", lambda: write_dataprep(rbi))]
    if not a.skip_envelope:
        steps.append(("envelope", write_envelope))
        steps.append(("envelope_full", lambda: write_envelope_full(rbi, rtri)))
        steps.append(("envelope_synth", lambda: write_envelope_synth(rbi, rtri)))
    for name, fn in steps:
        if only is None or name in only:
            fn()


if __name__ == "__main__":
    main()
