"""CPU: the oracle against the reference's own outputs (golden fixtures made by importing the
reference; see tests/golden/make_goldens.py).  Bitwise wherever the reference is deterministic."""
import json
import os

import numpy as np
import pytest

from oracle import philox as oph
from oracle import ref_cpu as orc
from tests.helpers import GOLDEN, bits, cdnow, golden, replay_case


def test_oracle_pin_record_all_bitwise():
    pin = json.load(open(os.path.join(GOLDEN, "oracle_pin.json")))
    assert pin["checks"] and all(c["bitwise_equal"] for c in pin["checks"])
    for name in ("oracle_pin_full.json", "oracle_pin_synth.json"):  # c2/c3 inputs; c4/c5-model inputs
        pin = json.load(open(os.path.join(GOLDEN, name)))
        assert pin["checks"] and all(c["bitwise"] for c in pin["checks"])


@pytest.mark.parametrize("name", ["synth_bi_k5", "synth_tri_k9"])
def test_synthetic_envelope_inputs_regenerate(name):
    """The c4/c5-model envelope fixtures store the generator seed, not the data: the product's
    generator (mcmc_clv_model_amd/data.py, numpy) must regenerate the exact inputs the oracle ran on."""
    import hashlib
    from mcmc_clv_model_amd.data import synthetic_cbs
    f = golden(f"envelope_{name}.npz")
    df = synthetic_cbs(int(f["data_n"]), int(f["data_K"]), int(f["data_D"]), seed=int(f["data_seed"]))
    h = hashlib.sha256()
    for c in df.columns:
        h.update(c.encode())
        h.update(np.ascontiguousarray(df[c].to_numpy()).tobytes())
    assert h.hexdigest() == str(f["data_sha256"])
    assert f["log_lambda_mean"].shape == (int(f["data_n"]),) and int(f["M"]) == 16


def test_reference_smoke_bi553_reproduced_bitwise():
    """The reference's only built-in test (bi:553-559): 50 synthetic customers, seed 123."""
    f = golden("smoke_bi553.npz")
    import pandas as pd
    cbs = pd.DataFrame(dict(x=f["x"], t_x=f["t_x"], T_cal=f["T_cal"]))
    d = orc.mcmc_draw_parameters(cbs, mcmc=100, burnin=50, thin=10, chains=1, trace=0, seed=123)
    assert d["level_2"][0].shape == (10, 5)
    assert np.array_equal(bits(d["level_2"][0]), bits(f["level_2"]))
    assert np.array_equal(bits(d["level_1"][0]), bits(f["level_1"]))
    assert bits(d["log_likelihood"]) == bits(f["log_likelihood"])


def test_formulas_p_alive_tau():
    f = golden("formulas.npz")
    p = orc.p_alive(f["z_tx"], f["z_T"], f["z_lam"], f["z_mu"])
    assert np.array_equal(bits(p), bits(f["z_p"]))
    assert np.array_equal(p > f["z_u"], f["z_out"])
    z = f["z_out"]
    ml = f["z_mu"] + f["z_lam"]
    tau = np.empty_like(f["z_tx"])
    v = f["tau_v"]
    tau[z] = f["z_T"][z] + (1.0 / f["z_mu"][z]) * v[z]
    tau[~z] = orc.tau_churned(f["z_tx"][~z], f["z_T"][~z], ml[~z], v[~z])
    assert np.array_equal(bits(tau), bits(f["tau_out"]))


def test_formulas_log_posterior_edge_cases():
    f = golden("formulas.npz")
    with np.errstate(over="ignore", invalid="ignore"):
        lp = orc.log_posterior(f["lp_ll"], f["lp_lm"], f["lp_x"], f["lp_z"], f["lp_T"], f["lp_tau"], f["lp_mv"],
                               np.linalg.inv(f["lp_S"]))
    assert np.array_equal(bits(lp), bits(f["lp_out"]))
    assert np.all(np.isneginf(lp[f["lp_lm"] > 5.0]))        # quirk Q3
    with np.errstate(invalid="ignore"):
        assert np.isnan(np.exp(lp[f["lp_lm"] > 5.0] - lp[f["lp_lm"] > 5.0])).all()  # -inf - -inf


@pytest.mark.parametrize("D", [2, 3])
@pytest.mark.parametrize("K", [1, 2, 5, 9])
def test_formulas_level2(D, K):
    f = golden("formulas.npz")
    p = f"l2_D{D}_K{K}_"
    hyper = orc.default_hyper(K, D)
    hyper["beta_0"] = f[p + "B0"].copy()
    V, Bh, Sn, nun = orc.level2_posterior(f[p + "X"], f[p + "Y"], hyper)
    assert np.array_equal(bits(V), bits(f[p + "V"]))
    assert np.array_equal(bits(Bh), bits(f[p + "Bhat"]))
    assert np.array_equal(bits(Sn), bits(f[p + "Sn"]))
    Sig = orc.invwishart_from_variates(Sn, f[p + "iw_normal"], f[p + "iw_chi2"])
    assert np.array_equal(bits(Sig), bits(f[p + "Sigma"]))
    # beta = B_hat.ravel() + MVN noise of kron(Sigma, V) (quirk Q1: row-major ravel)
    (u, s, vh) = np.linalg.svd(np.kron(Sig, V))
    noise = (f[p + "mvn_z"][None, :] @ (u * np.sqrt(s)).T)[0]
    beta = (Bh.ravel() + noise).reshape(Bh.shape)
    assert np.array_equal(bits(beta), bits(f[p + "beta"]))


def test_level2_sufficient_statistic_identity():
    """S_n = S0 + Y'Y + B0'A0B0 - R'B_hat (what the device computes from block partials)
    equals the reference's S0 + E'E + C'A0C (bi:253-255) to rounding."""
    f = golden("formulas.npz")
    for D in (2, 3):
        for K in (1, 2, 5, 9):
            p = f"l2_D{D}_K{K}_"
            X, Y = f[p + "X"], f[p + "Y"]
            hyper = orc.default_hyper(K, D)
            hyper["beta_0"] = f[p + "B0"].copy()
            A0, B0, S0 = hyper["A_0"], hyper["beta_0"], hyper["gamma_00"]
            R = X.T @ Y + A0 @ B0
            Bh = f[p + "V"] @ R
            Sn = S0 + Y.T @ Y + B0.T @ A0 @ B0 - R.T @ Bh
            np.testing.assert_allclose(Sn, f[p + "Sn"], rtol=1e-11, atol=1e-9)


def test_formulas_draw_eta():
    f = golden("formulas.npz")
    beta, Sig, om = f["eta_beta"], f["eta_Sigma"], float(f["eta_omega2"])
    prior_mean = (f["eta_X"] @ beta)[:, 2]
    post_var = 1.0 / (1.0 / om + 1.0 / Sig[2, 2])
    post_mean = post_var * (f["eta_log_s"] / om + prior_mean / Sig[2, 2])
    assert np.array_equal(bits(post_mean + np.sqrt(post_var) * f["eta_z"]), bits(f["eta_out"]))


@pytest.mark.parametrize("name", ["bi_k1", "bi_k2", "tri_k3", "bi_k1_s0", "bi_k5", "tri_k9"])
def test_oracle_replay_fixtures_bitwise(name):
    """The oracle regenerates the reference's recorded outputs exactly (fixture = reference run)."""
    df, covs, f = replay_case(name)
    fn = orc.mcmc_draw_parameters if str(f["kind"]) == "bi" else orc.mcmc_draw_parameters_rfm_m
    d = fn(df, covs, mcmc=int(f["mcmc"]), burnin=0, thin=1, chains=int(f["chains"]), seed=int(f["seed"]),
           trace=0, n_mh_steps=int(f["S"]))
    assert np.array_equal(bits(np.stack(d["level_1"])), bits(f["level_1"]))
    assert np.array_equal(bits(np.stack(d["level_2"])), bits(f["level_2"]))
    assert bits(d["log_likelihood"]) == bits(f["log_likelihood"])


def test_replay_tape_layout_matches_recorded_variates():
    """The packed device tape holds exactly the variates the reference consumed."""
    df, covs, f = replay_case("bi_k1")
    d = orc.mcmc_draw_parameters(df, covs, mcmc=int(f["n_tape_sweeps"]), burnin=0, thin=1, chains=int(f["chains"]),
                                 seed=int(f["seed"]), trace=0, n_mh_steps=int(f["S"]), record=True)
    n, S = len(df), int(f["S"])
    tape = f["tape"]
    for c in range(int(f["chains"])):
        for s, sw in enumerate(d["tape"][c]):
            assert np.array_equal(tape[c, s, :n], sw["u_z"])
            assert np.array_equal(tape[c, s, n:2 * n], sw["v_tau"])
            for j in range(S):
                assert np.array_equal(tape[c, s, (2 + 3 * j) * n:(3 + 3 * j) * n], sw["t_l"][j])
            h = tape.shape[2] - 40
            assert np.array_equal(tape[c, s, h + 6:h + 6 + 2], sw["mvn_noise"])


def test_philox_known_answers():
    kat = json.load(open(os.path.join(GOLDEN, "philox_kat.json")))
    for k in kat["random123"]:
        got = oph.philox4x32_10(np.array(k["ctr"], np.uint32), k["key"][0], k["key"][1])
        assert [f"{v:08x}" for v in got] == k["out"]
    e = kat["extra"]
    got = oph.philox4x32_10(np.array(e["ctr"], np.uint32), e["key"][0], e["key"][1])
    assert np.array_equal(got, np.array(e["out"], np.uint32))


def test_philox_variate_distributions():
    from scipy import stats
    v = oph.sweep_variates(20250718, 3, 17, 40000, 3)
    for j in range(3):
        assert stats.kstest(v["t_l"][j].astype(float), "t", args=(3,)).pvalue > 1e-4
        assert stats.kstest(v["t_m"][j].astype(float), "t", args=(3,)).pvalue > 1e-4
        assert stats.kstest(v["u_acc"][j].astype(float), "uniform").pvalue > 1e-4
        assert abs(np.corrcoef(v["t_l"][j], v["t_m"][j])[0, 1]) < 0.03
    assert stats.kstest(v["u_z"], "uniform").pvalue > 1e-4
    assert stats.kstest(v["e_alive"], "expon").pvalue > 1e-4
    assert stats.kstest(v["eta_z"], "norm").pvalue > 1e-4
    c = [oph.chi2_draw(5, 0, s, 0, 40.0) for s in range(1500)]
    assert stats.kstest(c, "chi2", args=(40,)).pvalue > 1e-4


def test_cdnow_fixture_data():
    abe, full = cdnow("abe"), cdnow("full")
    assert len(abe) == 2357 and len(full) == 23570
    assert (abe["x"] >= 0).all() and (abe["t_x"] <= abe["T_cal"]).all()
    assert int((full["sales"] == 0).sum()) >= 1    # zero-spend rows -> log_s = 0
