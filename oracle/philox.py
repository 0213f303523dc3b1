"""numpy restatement of the sampler's Philox-mode random stream — TEST INFRASTRUCTURE ONLY.

Mirrors ``mcmc_clv_model_amd/csrc/philox.h`` (counter layout, slots, uniform conversions and the
Student-t(3) / normal / exponential / chi-square transforms) so tests can check the device's
variates value by value.  Philox4x32-10 itself is pinned by the Random123 known-answer vectors
in ``tests/golden/philox_kat.json``.

Note: the reference itself uses numpy's PCG64 (bivariate/mcmc.py:486); this stream is the
build's replacement, so it is pinned by KATs and distribution tests, not by the reference.
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

STREAM_CUSTOMER, STREAM_HYPER = 0, 1
SLOT_ZTAU, SLOT_ETA, SLOT_MH0 = 0, 1, 2
HSLOT_NORMAL0, HSLOT_BETA_NORMAL0, HSLOT_GAMMA0, HSLOT_GAMMA_STRIDE = 0, 4, 64, 256
GAMMA_MAX_ATTEMPTS = 100


def philox4x32_10(ctr, k0, k1):
    """ctr: (..., 4) uint32 array; k0, k1: uint32 scalars or arrays broadcastable to ctr[..., 0]."""
    c = np.asarray(ctr, dtype=np.uint32)
    x0, x1, x2, x3 = (c[..., i].astype(np.uint64) for i in range(4))
    k0 = np.asarray(k0, dtype=np.uint32).astype(np.uint64)
    k1 = np.asarray(k1, dtype=np.uint32).astype(np.uint64)
    for _ in range(10):
        p0 = M0 * x0
        p1 = M1 * x2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        x0, x1, x2, x3 = (hi1 ^ x1 ^ k0) & MASK32, lo1, (hi0 ^ x3 ^ k1) & MASK32, lo0
        k0 = (k0 + np.uint64(W0)) & MASK32
        k1 = (k1 + np.uint64(W1)) & MASK32
    return np.stack([x0, x1, x2, x3], axis=-1).astype(np.uint32)


def chain_key(seed: int, chain: int):
    s = (int(seed) + int(chain)) & ((1 << 64) - 1)
    return np.uint32(s & 0xFFFFFFFF), np.uint32(s >> 32)


def u53(lo, hi):
    v = ((hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)) >> np.uint64(11)
    return v.astype(np.float64) * 2.0 ** -53


def u53_open0(lo, hi):
    v = ((hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)) >> np.uint64(11)
    return (v + np.uint64(1)).astype(np.float64) * 2.0 ** -53


def uf32(w):
    return (w.astype(np.float32) * np.float32(2.0 ** -32) + np.float32(2.0 ** -33)).astype(np.float32)


def customer_blocks(seed, chain, customers, sweep, slot):
    k0, k1 = chain_key(seed, chain)
    customers = np.asarray(customers, dtype=np.uint32)
    ctr = np.zeros(customers.shape + (4,), dtype=np.uint32)
    ctr[..., 0] = customers
    ctr[..., 1] = sweep
    ctr[..., 2] = slot
    ctr[..., 3] = STREAM_CUSTOMER
    return philox4x32_10(ctr, k0, k1)


def hyper_block(seed, chain, slot, sweep):
    k0, k1 = chain_key(seed, chain)
    return philox4x32_10(np.array([slot, sweep, 0, STREAM_HYPER], dtype=np.uint32), k0, k1)


def t3_f32(u, v):
    """Student-t(3) by Bailey's trigonometric polar form: sqrt(3 (U^(-2/3) - 1)) cos(2 pi V)
    (csrc/philox.h:t3_f32; fp32 like the device's v_log/v_exp/v_sqrt/v_cos); v in revolutions."""
    p = np.exp2(np.float32(-2.0 / 3.0) * np.log2(u)).astype(np.float32)
    # fmaf(3, p, -3): 3 p - 3 is exact in fp64 (p >= 1 has 24 bits), then one rounding to fp32
    r = np.sqrt((3.0 * p.astype(np.float64) - 3.0).astype(np.float32)).astype(np.float32)
    return (r * np.cos(v.astype(np.float64) * (2.0 * np.pi))).astype(np.float32)


def angle_hi(w):
    return ((w & np.uint32(0xFFFF0000)).astype(np.float32) * np.float32(2.0 ** -32)).astype(np.float32)


def angle_lo(w):
    return ((w << np.uint32(16)).astype(np.uint32).astype(np.float32) * np.float32(2.0 ** -32)).astype(np.float32)


MH_PACK = False  # csrc/philox.h CLV_MH_PACK: four MH steps from three Philox blocks


def uf24(w):
    """(w[23:0] + 1) 2^-24 in (0, 1] (csrc/philox.h uf24; exact in fp32)."""
    return ((w & np.uint32(0xFFFFFF)).astype(np.float32) * np.float32(2.0 ** -24) + np.float32(2.0 ** -24)).astype(np.float32)


def angle12(hi8_word, lo4):
    """(hi8_word[31:24] . lo4) 2^-12 revolutions (csrc/philox.h angle12; exact in fp32)."""
    return ((hi8_word >> np.uint32(24)).astype(np.float32) * np.float32(2.0 ** -8)
            + lo4.astype(np.float32) * np.float32(2.0 ** -12)).astype(np.float32)


def mh_step_words(seed, chain, cust, sweep, j):
    """Uniforms of MH step j: (radius u of t_l, radius u of t_m, angle of t_l, angle of t_m, accept u)."""
    if MH_PACK:  # chunk q = j // 4: blocks SLOT_MH0 + 3q + {0, 1, 2}; step i = j % 4 takes words 3i..3i+2
        q, i = divmod(j, 4)
        W = np.concatenate([customer_blocks(seed, chain, cust, sweep, SLOT_MH0 + 3 * q + k) for k in range(3)], axis=1)
        a, b, c = W[:, 3 * i], W[:, 3 * i + 1], W[:, 3 * i + 2]
        return (uf24(a), uf24(b), angle12(a, (c >> np.uint32(24)) & np.uint32(0xF)), angle12(b, c >> np.uint32(28)),
                uf24(c))
    w = customer_blocks(seed, chain, cust, sweep, SLOT_MH0 + j)
    return uf32(w[:, 0]), uf32(w[:, 1]), angle_hi(w[:, 2]), angle_lo(w[:, 2]), uf32(w[:, 3])


def sweep_variates(seed, chain, sweep, n, n_steps):
    """The Philox-mode variates of one sweep for customers 0..n-1 (see csrc/philox.h): MH step j
    takes its radius uniforms of t_l / t_m, two angles and the accept uniform from the customer's
    Philox blocks SLOT_MH0 + ... (MH_PACK: four steps per three blocks, 24-bit uniforms, 12-bit
    angles; else one block per step, 32-bit words, 16-bit angles)."""
    cust = np.arange(n)
    r = customer_blocks(seed, chain, cust, sweep, SLOT_ZTAU)
    out = dict(u_z=u53(r[:, 0], r[:, 1]), u_tau=u53(r[:, 2], r[:, 3]),
               e_alive=-np.log(u53_open0(r[:, 2], r[:, 3])))
    re = customer_blocks(seed, chain, cust, sweep, SLOT_ETA)
    out["eta_z"] = np.sqrt(-2.0 * np.log(u53_open0(re[:, 0], re[:, 1]))) * np.cos(2.0 * np.pi * u53(re[:, 2], re[:, 3]))
    tl = np.empty((n_steps, n), np.float32)
    tm = np.empty((n_steps, n), np.float32)
    ua = np.empty((n_steps, n), np.float32)
    for j in range(n_steps):
        ul, um, al, am, uacc = mh_step_words(seed, chain, cust, sweep, j)
        tl[j] = t3_f32(ul, al)
        tm[j] = t3_f32(um, am)
        ua[j] = uacc
    out.update(t_l=tl, t_m=tm, u_acc=ua)
    return out


def hyper_normal(seed, chain, slot, sweep):
    r = hyper_block(seed, chain, slot, sweep)
    return float(np.sqrt(-2.0 * np.log(u53_open0(r[0:1], r[1:2])[0])) * np.cos(2.0 * np.pi * u53(r[2:3], r[3:4])[0]))


def chi2_draw(seed, chain, sweep, idx, df):
    """Marsaglia–Tsang Gamma(df/2) * 2 exactly as csrc/kernels.hip:chi2_draw."""
    alpha = 0.5 * df
    dd = alpha - 1.0 / 3.0
    cc = 1.0 / np.sqrt(9.0 * dd)
    for at in range(GAMMA_MAX_ATTEMPTS):
        slot = HSLOT_GAMMA0 + idx * HSLOT_GAMMA_STRIDE + 2 * at
        x = hyper_normal(seed, chain, slot, sweep)
        t = cc * x
        if t <= -1.0:
            continue
        v1 = t * (3.0 + t * (3.0 + t))
        r2 = hyper_block(seed, chain, slot + 1, sweep)
        lu = np.log(u53_open0(r2[0:1], r2[1:2])[0])
        if lu < 0.5 * x * x + dd * (3.0 * np.log1p(t) - v1):
            return 2.0 * dd * (1.0 + v1)
    return df
