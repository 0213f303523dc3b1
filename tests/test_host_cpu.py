"""CPU: the C-ABI library loads and exports every declared symbol; host-side setup is
bit-identical to the reference's; the product fails loudly without a GPU; the sharded exchange
(world_size 2, gloo) reproduces the single-process fixed-order reduction bit for bit."""
import ctypes
import os
import socket

import numpy as np
import pytest

from oracle import ref_cpu as orc
from tests.helpers import bits, cdnow


def test_library_loads_and_exports_header_symbols():
    from mcmc_clv_model_amd import _lib
    L = _lib.lib()
    names = _lib.exported_symbols()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), f"{n} declared in include/clvmcmc.h but not exported"
    assert L.clv_abi_version() == _lib.ABI_VERSION
    for i, st in enumerate((_lib.ClvConfig, _lib.ClvData, _lib.ClvPrior)):
        assert L.clv_sizeof(i) == ctypes.sizeof(st)


def test_default_blocks_per_unit_matches_python_plan():
    from mcmc_clv_model_amd import _lib
    from mcmc_clv_model_amd.distributed import default_blocks_per_unit
    L = _lib.lib()
    for n in (1, 255, 256, 2357, 23570, 131072, 131073, 1_000_000, 10_000_000, 4_000_000_000):
        assert L.clv_default_blocks_per_unit(n) == default_blocks_per_unit(n)


@pytest.mark.parametrize("D,covs", [(2, []), (2, ["first_sales_scaled"]), (3, ["gender_F", "age_scaled"])])
def test_host_setup_is_reference_identical(D, covs):
    """Constants handed to the device = what the reference computes (bi:367-379, 467-479, 248-249)."""
    from mcmc_clv_model_amd.sampler import build_problem, make_prior
    df = cdnow("abe")
    p = build_problem(df, covs, D)
    cbs, X = orc.design_matrix(df, covs)
    lam_init, lambdas, mus = orc.init_state(cbs["x"].to_numpy(), cbs["t_x"].to_numpy(), cbs["T_cal"].to_numpy())
    assert bits(p.lam_init) == bits(lam_init)
    hyper = orc.default_hyper(X.shape[1], D)
    V, *_ = orc.level2_posterior(X, np.zeros((len(df), D)), hyper)
    assert np.array_equal(bits(p.V), bits(V))
    assert p.beta_0[0, 0] == np.log(lambdas.mean()) and p.beta_0[0, 1] == np.log(mus.mean())
    if D == 3:
        assert p.omega2 == cbs["log_s"].var() and p.beta_0[0, 2] == cbs["log_s"].mean()
    pr = make_prior(p)
    assert pr.nu_n == hyper["nu_00"] + len(df)
    assert np.array_equal(p.cov, X[:, 1:].T)


def test_validation_errors_before_device():
    from mcmc_clv_model_amd import mcmc_draw_parameters
    df = cdnow("abe", 10)
    with pytest.raises(ValueError, match="cal_cbs missing required column 'x'"):
        mcmc_draw_parameters(df.drop(columns=["x"]))
    with pytest.raises(ValueError, match="some covariate columns not in cal_cbs"):
        mcmc_draw_parameters(df, ["nope"])


def test_seed_resolution():
    """seed + chain keys the chain (bi:486); numpy accepts any non-negative int, so seeds beyond the
    64-bit Philox key are folded deterministically (SeedSequence hash), never rejected."""
    from mcmc_clv_model_amd.sampler import resolve_seed
    assert resolve_seed(42) == 42 and resolve_seed(0) == 0 and resolve_seed((1 << 63) - 1) == (1 << 63) - 1
    big = [resolve_seed(v) for v in (1 << 63, 1 << 64, 3 ** 200, 3 ** 200 + 1)]
    assert big == [resolve_seed(v) for v in (1 << 63, 1 << 64, 3 ** 200, 3 ** 200 + 1)]  # deterministic
    assert len(set(big)) == 4 and all(0 <= v < (1 << 63) for v in big)
    with pytest.raises(ValueError):
        resolve_seed(-1)
    assert 0 <= resolve_seed(None) < (1 << 63)


def test_persistent_residency_margin():
    """Verdict r2 #6: the persistent kernels need every workgroup resident, so the grid must fit the
    admitted blocks per CU — min(occupancy API, 8, floor(800 / (ceil(sgpr/16)*16 + 16))), the
    MI355X guide's rule, at the maximum SGPR count — less a margin of one slot per 32 CUs.  At
    2 blocks per CU on 256 CUs (512 slots, 504 allowed): c2 / c3 (4 chains x (93 + 1) = 376) and
    c4 at 8 ranks (a shard of the 1M-customer plan: 496 blocks + 1 level-2 workgroup = 497) fit."""
    from mcmc_clv_model_amd import _lib
    from mcmc_clv_model_amd.distributed import plan
    L = _lib.lib()
    fits = lambda wgs, bpc=2: bool(L.clv_debug_persist_fits(wgs, bpc, 256))  # noqa: E731
    assert fits(4 * (93 + 1))
    p8 = plan(1_000_000, 8)
    nb_rank = -(-(p8.shard(0)[1] - p8.shard(0)[0]) // 256)
    assert nb_rank == 496 and fits(nb_rank + 1)
    assert fits(504) and not fits(505) and not fits(512) and not fits(0)
    assert not L.clv_debug_persist_fits(10, 0, 256)
    assert fits(6 * 256 - 8, 7) and not fits(6 * 256 - 7, 7)  # the SGPR term caps 7 / 8 blocks per CU at 6


def test_persistent_choice_by_grid_density():
    """Verdict r3 #8 / r5 #4: which grids run the persistent kernel (world size 1, and the peer
    exchange at world size > 1).  Round 4's density cap came from the level-2 workgroup's
    lane-per-block slot resets (~7k partial-line write-throughs ahead of its draw at ~500 blocks);
    with coalesced resets the persistent kernel wins at every measured density
    (profiles/r06_persist_crossover*.jsonl: c4's 8-rank shard, 1 chain x 497 workgroups, 14.1 vs
    20.3 us per sweep), so it runs wherever the grid fits — c4 at 8 ranks included."""
    from mcmc_clv_model_amd import _lib
    from mcmc_clv_model_amd.distributed import plan
    L = _lib.lib()
    pick = lambda D, K, C, wgs, bpc=2: bool(L.clv_debug_persist_choice(D, K, C, wgs, bpc, 256))  # noqa: E731
    assert pick(2, 2, 4, 4 * (93 + 1)) and pick(3, 3, 4, 4 * (93 + 1))        # c2, c3
    assert pick(2, 1, 4, 4 * (10 + 1))                                      # c1 (2,357 customers)
    p8 = plan(1_000_000, 8)
    nb_rank = -(-(p8.shard(0)[1] - p8.shard(0)[0]) // 256)
    assert nb_rank == 496 and pick(2, 5, 1, nb_rank + 1)                    # c4 at 8 ranks: 14.1 vs 20.3 us
    assert pick(2, 2, 4, 476) and pick(2, 2, 2, 472) and pick(3, 3, 1, 431)  # 10.3 / 19.0, 10.6 / 19.0, 15.6 / 20.6
    assert pick(3, 9, 1, 236)                                               # spilling instance: 20.1 vs 20.8 us
    assert not pick(2, 2, 4, 505) and not pick(2, 5, 1, 505)                # does not fit at all


def test_no_cpu_fallback_without_gpu():
    """The product path raises instead of silently running on the CPU."""
    from mcmc_clv_model_amd import _lib, mcmc_draw_parameters
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_lib.ClvError, match="no HIP device"):
        mcmc_draw_parameters(cdnow("abe", 100), mcmc=2, burnin=0, thin=1, chains=1, seed=1, trace=0)


def test_c_abi_rejects_bad_configs():
    """Argument checks in clv_create run before any device call."""
    from mcmc_clv_model_amd import _lib
    from mcmc_clv_model_amd.sampler import build_problem, make_prior
    L = _lib.lib()
    p = build_problem(cdnow("abe", 300), [], 2)
    base = dict(abi_version=_lib.ABI_VERSION, D=2, K=1, n_mh_steps=20, burnin=0, mcmc=2, thin=1, n_chains=1, chain_first=0,
                rng_mode=0, draw_sink=0, device=-1, seed=1, n_global=300, shard_begin=0, world_size=1, rank=0,
                blocks_per_rank=0, blocks_per_unit=0, stream=0)
    data = _lib.ClvData(n=300, x=p.x.ctypes.data, t_x=p.t_x.ctypes.data, T_cal=p.T_cal.ctypes.data)
    pr = make_prior(p)
    for bad in (dict(D=4), dict(K=10), dict(thin=0), dict(n_chains=0), dict(abi_version=_lib.ABI_VERSION + 1),
                dict(draw_sink=4), dict(blocks_per_unit=3),
                dict(world_size=2, rank=0, blocks_per_rank=0), dict(rng_mode=1, world_size=2, blocks_per_rank=2),
                dict(n_global=299), dict(shard_begin=256)):
        cfg = _lib.ClvConfig(**dict(base, **bad))
        h = ctypes.c_void_p()
        rc = L.clv_create(ctypes.byref(cfg), ctypes.byref(data), ctypes.byref(pr), ctypes.byref(h))
        assert rc == -1, (bad, rc)
        assert L.clv_last_error()


# ---------------------------------------------------------------------------------------------
# Sharded exchange on CPU (gloo): plan + all_gather layout + the hyper kernel's fixed-order sum.
def wave_reduce(acc: np.ndarray) -> np.ndarray:
    """numpy restatement of block_reduce's per-wave part (kernels.hip): (64, NS) lane values ->
    (NS,) totals, with the device's addition order: v_permlane32_swap halving, v_permlane16_swap
    halving, then a DPP row_ror 8/4/2/1 allreduce within 16-lane rows."""
    NS = acc.shape[1]
    H1, H2 = (NS + 1) // 2, ((NS + 1) // 2 + 1) // 2
    w1 = np.zeros((64, H1))
    for j in range(H1):
        a = acc[:, j].copy()
        b = acc[:, j + H1].copy() if j + H1 < NS else np.zeros(64)
        a2, b2 = a.copy(), b.copy()
        a2[32:], b2[:32] = b[:32], a[32:]
        w1[:, j] = a2 + b2
    w2 = np.zeros((64, H2))
    for j in range(H2):
        a = w1[:, j].copy()
        b = w1[:, j + H2].copy() if j + H2 < H1 else np.zeros(64)
        a2, b2 = a.copy(), b.copy()
        for r in (1, 3):
            a2[16 * r:16 * r + 16], b2[16 * (r - 1):16 * r] = b[16 * (r - 1):16 * r], a[16 * r:16 * r + 16]
        w2[:, j] = a2 + b2
    lanes = np.arange(64)
    rot = lambda R: (lanes & ~15) | ((lanes + R) & 15)  # noqa: E731  (row_ror:R source lane)
    for R in (8, 4, 2, 1):
        w2 = w2 + w2[rot(R)]
    out = np.zeros(NS)
    for row in range(4):
        for j in range(H2):
            i1 = j + (H2 if row & 1 else 0)
            idx = i1 + (H1 if row >> 1 else 0)
            if i1 < H1 and idx < NS:
                out[idx] = w2[16 * row, j]
    return out


def fixed_order_sum(units: np.ndarray, n_units_global: int, upr: int, world: int, chain: int, n_chains: int):
    """numpy restatement of hyper_body's reduction order (kernels.hip): thread t of 256 sums
    units t, t+256, ... sequentially; each 64-lane wave reduces as wave_reduce(); the 4 waves'
    totals are added in wave order.  units: gathered [world][chain][stride][units_per_rank]."""
    stride = units.shape[2]
    acc = np.zeros((256, stride))
    for t in range(256):
        for u in range(t, n_units_global, 256):
            r, lu = divmod(u, upr)
            acc[t] += units[r, chain, :, lu]
    waves = [wave_reduce(acc[64 * w:64 * (w + 1)]) for w in range(4)]
    return ((waves[0] + waves[1]) + waves[2]) + waves[3]


def _unit_partials(stats_per_customer: np.ndarray, begin: int, end: int, plan, n_chains: int):
    """Block partials (sum of 256 customers, butterfly order irrelevant here: shard-local and
    identical on every rank layout) grouped into units, as the device lays them out."""
    stride = stats_per_customer.shape[-1]
    bpr, G = plan.blocks_per_rank, plan.blocks_per_unit
    blocks = np.zeros((n_chains, bpr, stride))
    for b in range(bpr):
        lo, hi = begin + b * 256, min(end, begin + (b + 1) * 256)
        if lo < hi:
            blocks[:, b] = stats_per_customer[:, lo:hi].sum(1)
    units = np.zeros((n_chains, stride, bpr // G))  # statistic-major, as clv_partials() exposes it
    for u in range(bpr // G):
        for bb in range(G):
            units[:, :, u] += blocks[:, u * G + bb]
    return units


def _worker(rank, world, port, n_global, q):
    import torch
    import torch.distributed as dist
    from mcmc_clv_model_amd import distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(0)
    C, stride = 2, 5
    stats = rng.normal(size=(C, n_global, stride))
    plan = D.plan(n_global, world)
    b, e = plan.shard(rank)
    units = _unit_partials(stats, b, e, plan, C)
    local = torch.from_numpy(units.reshape(-1).copy())
    gathered = torch.zeros(local.numel() * world, dtype=torch.float64)
    D.exchange(local, gathered)
    g = gathered.numpy().reshape(world, C, stride, plan.units_per_rank)
    sums = [fixed_order_sum(g, plan.n_units_global, plan.units_per_rank, world, c, C) for c in range(C)]
    q.put((rank, np.stack(sums), (b, e)))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n_global", [23570, 140_000, 1_000_000])  # c2, a mid size, c4 (1M, strong scaling)
def test_sharded_exchange_world2_gloo_matches_single_process(n_global):
    import multiprocessing as mp
    from mcmc_clv_model_amd import distributed as D
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_global, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: world 1
    rng = np.random.default_rng(0)
    stats = rng.normal(size=(2, n_global, 5))
    plan1 = D.plan(n_global, 1)
    u1 = _unit_partials(stats, 0, n_global, plan1, 2)[None]
    ref = np.stack([fixed_order_sum(u1, plan1.n_units_global, plan1.units_per_rank, 1, c, 2) for c in range(2)])
    (_, s0, (b0, e0)), (_, s1, (b1, e1)) = res
    assert b0 == 0 and e0 == b1 and e1 == n_global           # contiguous cover
    assert b1 % (256 * D.plan(n_global, 2).blocks_per_unit) == 0
    assert np.array_equal(bits(s0), bits(s1))                 # every rank draws identically
    assert np.array_equal(bits(s0), bits(ref))                # ... and equal to 1 GPU, bit for bit


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_plan_covers_and_aligns(world):
    from mcmc_clv_model_amd import distributed as D
    for n in (1, 300, 23570, 1_000_000, 10_000_000):
        p = D.plan(n, world)
        spans = [p.shard(r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
        assert p.blocks_per_rank % p.blocks_per_unit == 0
        assert p.blocks_per_unit == D.default_blocks_per_unit(n)  # world-independent unit size
        assert p.units_per_rank * world >= p.n_units_global


def test_philox_header_host_build_kat_and_hoisting(tmp_path):
    """csrc/philox.h compiled for the host with g++: Random123 KATs and SlotPhilox (hoisted
    slot-independent products, used by the sweep kernel) bit-identical to plain Philox4x32-10."""
    import subprocess
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "philox_host_check.cpp")
    exe = str(tmp_path / "philox_check")
    subprocess.run(["g++", "-O2", "-std=c++17", src, "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout


@pytest.mark.parametrize("C,nb,n_cu", [(4, 93, 256), (3, 93, 256), (4, 94, 256), (2, 200, 256), (8, 40, 256),
                                       (1, 300, 256), (4, 40, 256), (4, 200, 256), (1, 496, 256)])
def test_persistent_placement_map(C, nb, n_cu):
    """clv_debug_wg_map (host code, capi.hip persist_wg_map): the placement of the persistent grid is
    a permutation of every (chain, block) incl. each chain's level-2 workgroup; when the grid has
    more workgroups than CUs (but at most two per CU), the workgroups dispatched onto the same CU
    (linear i and i + n_cu) belong to the same chain, and each level-2 workgroup shares its CU with
    one of its own chain's customer workgroups (chains of >= 256 blocks: alone on a CU, round 6);
    otherwise the identity."""
    from mcmc_clv_model_amd import _lib
    L = _lib.lib()
    T = C * (nb + 1)
    out = (ctypes.c_int32 * T)()
    assert L.clv_debug_wg_map(C, nb, n_cu, out) == 0
    m = np.array(out[:], dtype=np.int64)
    chain, block = m >> 16, m & 0xFFFF
    assert sorted(zip(chain.tolist(), block.tolist())) == [(c, b) for c in range(C) for b in range(nb + 1)]
    P = T - n_cu
    if P <= 0 or T > 2 * n_cu:
        assert np.array_equal(m, [(c << 16) | b for c in range(C) for b in range(nb + 1)])
        return
    for i in range(P):
        assert chain[i] == chain[i + n_cu], (i, chain[i], chain[i + n_cu])
    l2 = np.flatnonzero(block == nb)
    if nb >= 256:  # (CLV_L2_ALONE_MIN_NB) its lanes poll two blocks each: the level-2 workgroup alone on a CU
        assert all(P <= i < n_cu for i in l2)
    else:  # every level-2 workgroup sits on a shared CU, beside one of its chain's customer workgroups
        assert all(i < P or i >= n_cu for i in l2)
    pairs = np.bincount(chain[:P], minlength=C)
    assert pairs.max() - pairs.min() <= 1  # shared CUs spread evenly over the chains


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_bench_scaling_workloads(world, monkeypatch):
    """bench.py's BASELINE multi-GPU configurations: c4 keeps the same problem at
    every N (strong scaling), c5 grows by its per-GPU size (weak scaling), with the covariate
    counts K = 5 / 9; the shard plan covers every customer.  Sizes scaled down 1000x here."""
    import bench
    from mcmc_clv_model_amd import distributed as D
    monkeypatch.setitem(bench.WORKLOADS, "c4", bench.WORKLOADS["c4"][:1] + ("synthetic:1000:5:20250718",)
                        + bench.WORKLOADS["c4"][2:])
    monkeypatch.setitem(bench.WORKLOADS, "c5", bench.WORKLOADS["c5"][:1] + ("synthetic:1250:9:20250719",)
                        + bench.WORKLOADS["c5"][2:])
    df4, D4, covs4 = bench.load_workload("c4", world)[:3]
    df5, D5, covs5 = bench.load_workload("c5", world)[:3]
    assert (len(df4), D4, len(covs4) + 1) == (1000, 2, 5)
    assert (len(df5), D5, len(covs5) + 1) == (1250 * world, 3, 9)
    assert set(covs5) <= set(df5.columns) and "log_s" in df5.columns
    for n in (len(df4), len(df5)):
        pl = D.plan(n, world)
        spans = [pl.shard(r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == n


def test_multi_device_plan():
    """devices= (sampler.multi_plan): chain groups cover every chain once, in order, one group per
    device used; 'auto' shards customers when chains do not divide evenly or the sink pools chains."""
    from mcmc_clv_model_amd.sampler import multi_plan
    for chains in range(1, 10):
        for n_dev in range(1, 9):
            mode, groups = multi_plan(chains, n_dev, "full", "chains")
            assert mode == "chains" and len(groups) == min(chains, n_dev)
            assert [c for f, k in groups for c in range(f, f + k)] == list(range(chains))
            assert max(k for _, k in groups) - min(k for _, k in groups) <= 1
            auto = multi_plan(chains, n_dev, "full")[0]
            assert auto == ("chains" if chains % n_dev == 0 else "customers")
    assert multi_plan(4, 2, "summary+pct")[0] == "customers"
    with pytest.raises(ValueError, match="summary\\+pct"):
        multi_plan(4, 2, "summary+pct", "chains")
    with pytest.raises(ValueError, match="shard must be"):
        multi_plan(4, 2, "full", "rows")


def test_fast_log_table_and_method():
    """log_fast's table (tools/gen_log_table.py -> csrc/fastmath.h LOG_TAB) as compiled, and the
    method with exact fma (fractions) against 60-digit logs: <= 1 ulp on a sample across the range."""
    import math
    import re
    import struct
    import sys
    from decimal import Decimal, getcontext
    from fractions import Fraction
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_log_table as g
    src = open(os.path.join(ROOT, "mcmc_clv_model_amd", "csrc", "fastmath.h")).read()
    body = src[src.index("LOG_TAB[2 * LOG_TAB_N] = {"):]
    body = body[body.index("{") + 1:body.index("};")]
    vals = [float.fromhex(v) for v in re.findall(r"-?0x[0-9a-fp.+-]+", body)]
    tab = g.table()
    assert vals == [v for pair in tab for v in pair]
    hi, lo = g.ln2_split()
    assert f"LOG_LN2_HI = {hi.hex()};" in src and f"LOG_LN2_LO = {lo.hex()};" in src
    getcontext().prec = 60

    def fma(a, b, c):
        return float(Fraction(a) * Fraction(b) + Fraction(c))

    def log_fast(x):
        ix = struct.unpack("<Q", struct.pack("<d", x))[0]
        h = ix >> 32
        t = (h - g.OFF_HI) & 0xFFFFFFFF
        k = (t - (1 << 32) if t >> 31 else t) >> 20
        invc, logc = tab[(t >> 12) & 255]
        z = struct.unpack("<d", struct.pack("<Q", (((h - (t & 0xFFF00000)) & 0xFFFFFFFF) << 32) | (ix & 0xFFFFFFFF)))[0]
        r = fma(z, invc, -1.0)
        assert abs(r) <= 2.0 ** -9
        p = fma(r, -1.0 / 6.0, 1.0 / 5.0)
        p = fma(p, r, -1.0 / 4.0)
        p = fma(p, r, 1.0 / 3.0)
        p = fma(p, r, -0.5)
        return fma(float(k), hi, logc) + fma(float(k), lo, fma(r * r, p, r))

    rng = np.random.default_rng(5)
    xs = list(np.exp(rng.uniform(-700, 700, 400))) + list(rng.uniform(0.5, 2.0, 400)) + \
        list(1.0 + rng.uniform(-2e-3, 2e-3, 200)) + [1.0, 2.0, 0.5, 1 - 2.0 ** -53, 1 + 2.0 ** -52, 2.0 ** -1022]
    for x in xs:
        x = float(x)
        y, ref = log_fast(x), float(Decimal(x).ln())
        assert (y == 0.0) if ref == 0.0 else abs(y - ref) <= math.ulp(ref), x


def test_fast_cos_table_and_method():
    """cos2pi_u53's table (tools/gen_log_table.py -> csrc/fastmath.h COS_TAB) as compiled, and the
    method with exact fma (fractions) on random 53-bit uniforms of all four quadrants: within
    1.5e-15 of math.cos(2 pi u) (whose own argument rounding is up to ~5e-16)."""
    import math
    import re
    import sys
    from fractions import Fraction
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_log_table as g
    src = open(os.path.join(ROOT, "mcmc_clv_model_amd", "csrc", "fastmath.h")).read()
    body = src[src.index("COS_TAB[2 * COS_TAB_N] = {"):]
    body = body[body.index("{") + 1:body.index("};")]
    tab = g.cos_table()
    assert [float.fromhex(v) for v in re.findall(r"-?0x[0-9a-fp.+-]+", body)] == [v for p in tab for v in p]

    def fma(a, b, c):
        return float(Fraction(a) * Fraction(b) + Fraction(c))

    two_pi = 2.0 * math.pi

    def cos2pi(lo, hi):
        q, (c, s) = hi >> 30, tab[(hi >> 22) & 255]
        d = fma(float(hi & 0x3FFFFF), two_pi * 2.0 ** -32, float(lo >> 11) * (two_pi * 2.0 ** -53))
        x, y = (s, c) if q & 1 else (c, s)
        x, y = (-x if q in (1, 2) else x), (-y if q >= 2 else y)
        d2 = d * d
        cm1 = fma(fma(d2, -1.0 / 720.0, 1.0 / 24.0), d2, -0.5) * d2
        sn = fma(d2 * d, fma(d2, 1.0 / 120.0, -1.0 / 6.0), d)
        return fma(-y, sn, fma(x, cm1, x))

    rng = np.random.default_rng(6)
    for lo, hi in rng.integers(0, 2 ** 32, (3000, 2), dtype=np.uint64):
        lo, hi = int(lo), int(hi)
        u = ((hi << 32 | lo) >> 11) * 2.0 ** -53
        assert abs(cos2pi(lo, hi) - math.cos(two_pi * u)) <= 1.5e-15


def test_sharded_graph_sizes_cover_any_step():
    """Verdict r3 #4: the RCCL path's torch.cuda graphs.  A step of n sweeps replays chunk-sized
    graphs and then the binary decomposition of the rest, so the driver's 20-sweep step (chunk 32)
    replays the 16- and 4-sweep graphs instead of ~5 eager host calls per sweep; every size used is
    one captured at the first step."""
    from mcmc_clv_model_amd.distributed import graph_sizes, graph_sizes_all
    assert graph_sizes(20, 32) == [16, 4]
    assert graph_sizes(5, 32) == [4, 1]
    assert graph_sizes(70, 32) == [32, 32, 4, 2]
    assert graph_sizes(0, 32) == [] and graph_sizes(7, 0) == []
    assert graph_sizes_all(32) == [32, 16, 8, 4, 2, 1] and graph_sizes_all(24) == [24, 16, 8, 4, 2, 1]
    for chunk in (1, 3, 24, 32, 64):
        for n in range(0, 200):
            g = graph_sizes(n, chunk)
            assert sum(g) == n and set(g) <= set(graph_sizes_all(chunk))


def test_sharded_step_replays_graphs_for_20_sweeps():
    """ShardedSampler.step on the RCCL path with graph_chunk 32 (bench.py's default) and the
    driver's 20 steps: graphs are captured once (at the first graph-using step, e.g. the warm-up)
    and the 20-sweep step replays graphs only — no eager sweeps."""
    from mcmc_clv_model_amd import distributed as Dm

    class FakeGraph:
        def __init__(self, k):
            self.k, self.n = k, 0

        def replay(self):
            self.n += 1

    class FakeS:
        done = 0

        def note_sweeps(self, k):
            self.done += k

    class Stub:
        torch = __import__("torch")
        exchange, graph_chunk, timing, graph = "rccl", 32, False, None
        stream = None
        s = FakeS()
        eager = []

        def _capture(self, k):
            return FakeGraph(k)

        def _eager(self, n):
            self.eager.append(n)

    import contextlib
    st = Stub()
    orig = Stub.torch.cuda.stream
    Stub.torch.cuda.stream = lambda s: contextlib.nullcontext()
    try:
        Dm.ShardedSampler.step(st, 5)      # warm-up: captures every size
        assert sorted(st.graph) == [1, 2, 4, 8, 16, 32]
        caps = dict(st.graph)
        Dm.ShardedSampler.step(st, 20)     # the timed step
    finally:
        Stub.torch.cuda.stream = orig
    assert st.graph == caps and st.eager == [0, 0]
    assert st.graph[16].n == 1 and st.graph[4].n == 2 and st.graph[1].n == 1 and st.s.done == 25


@pytest.mark.parametrize("val,want", [(None, 10000.0), ("300", 300.0), ("0.5", 1.0), ("  250 ", 250.0),
                                      ("1e3", 1000.0), ("-5", 1.0), ("1e9", 3.6e6), ("abc", None), ("", None),
                                      ("250ms", None), ("inf", None), ("nan", None), ("-inf", None), ("0x10", None)])
def test_run_wait_ms_parses_like_clv_create(monkeypatch, val, want):
    """CLV_WAIT_TIMEOUT_MS is a finite decimal number of ms clamped to [1 ms, 1 h]
    (capi.hip parse_wait_ms); inf / nan / hex / trailing text are rejected — by clv_create (EINVAL)
    and here (ValueError) alike, so no value reaches the kernel's (uint64_t)(ms * 1e5)."""
    from mcmc_clv_model_amd.distributed import run_wait_ms
    if val is None:
        monkeypatch.delenv("CLV_WAIT_TIMEOUT_MS", raising=False)
    else:
        monkeypatch.setenv("CLV_WAIT_TIMEOUT_MS", val)
    if want is None:
        with pytest.raises(ValueError):
            run_wait_ms()
    else:
        assert run_wait_ms() == want


def test_bench_config_times_the_stored_phase(monkeypatch):
    """Verdict r3 #3 / r4 #1, #5: a configuration leg times a burn-in window AND a window of stored
    sweeps (the running-sum read-modify-write of bi:402-428, summary sink), continuing the same
    chains past the burn-in, each with a roofline from an event-timed pass over further sweeps
    (bound and its evidence printed), both byte accountings (summary sink +0; the
    kernel's own incl. the sums' read-modify-write), and the whole BASELINE run's rate.  Stub
    sampler, no GPU."""
    import torch

    import bench
    from mcmc_clv_model_amd import sampler as S

    log = []
    timing = []

    class Fake:
        n = 500

        def __init__(self, p, **kw):
            self.kw, self.done = kw, 0
            self.t = False

        def run(self, n):
            log.append((self.done + 1, self.done + n, self.t))
            self.done += n

        def synchronize(self):
            pass

        def launch_info(self):
            return dict(persistent=False)

        def set_timing(self, on):
            self.t = on
            timing.append(on)

        def kernel_time(self):
            n = sum(b - a + 1 for a, b, t in log if t)
            return dict(sweep_ms=0.085 * n, sweep_launches=n, hyper_ms=0.0, hyper_launches=0)

        def clock_ghz(self):
            return 0.0  # the launch-per-sweep kernel keeps no record ...

        def clock_probe(self, us):
            return 2.25  # ... so the line takes the probe kernel's reading

        def close(self):
            pass

    monkeypatch.setattr(S, "HipSampler", Fake)
    monkeypatch.setattr(S, "build_problem", lambda df, covs, D: None)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setitem(bench.WORKLOADS, "c4", bench.WORKLOADS["c4"][:1] + ("synthetic:500:5:20250718",)
                        + bench.WORKLOADS["c4"][2:])
    r = bench.run_leg("c4", 1, 0, 0, None, 1000, 200)
    burnin = bench.WORKLOADS["c4"][4]
    assert [(a, b) for a, b, _ in log] == [(1, 200), (201, 1200), (1201, 2200), (2201, burnin + 100),
                                           (burnin + 101, burnin + 1100), (burnin + 1101, burnin + 2100)]
    assert [t for _, _, t in log] == [False, False, True, False, False, True]  # events only on the roofline passes
    assert r["phase"].startswith("burn-in") and r["stored"]["sweeps"] == f"{burnin + 101}..{burnin + 1100}"
    D, K = 2, 5
    assert r["bytes_per_unit"] == round(bench.survey_bytes(D, K, 0.0, "summary"), 2) == 84.0
    assert r["stored"]["bytes_per_unit"] == 84.0  # the summary sink adds 0
    assert r["stored"]["bytes_per_unit_kernel"] == 84.0 + 144.0
    roof = r["roofline"]
    assert roof["bound"] in ("hbm", "valu", "latency", "unmeasured") and "rule" in roof["bound_evidence"]
    assert abs(roof["launch_us"] - 85.0) < 1e-6 and roof["sweeps_per_launch"] == 1
    assert abs(roof["achieved"] - 84.0 * 500 / 85e-6 / 1e9) < 1e-3
    assert r["stored"]["roofline"]["bound"] is not None
    # verdict r5 weak 3: each phase's traffic and counters come from that phase's committed profile
    src, src_st = roof["traffic_source"], r["stored"]["roofline"]["traffic_source"]
    assert "_c4_" in src and "stored" not in src, src
    assert "_c4stored_" in src_st, src_st
    assert "c4stored" in r["stored"]["roofline"]["bound_evidence"]["source"]
    assert r["stored"]["roofline"]["traffic"] != roof["traffic"] and "running sums" in r["stored"]["roofline"]["traffic_note"]
    assert bench.profile_name("c5", "stored") == "c5stored" and bench.profile_name("c5", "burnin") == "c5"
    assert r["gpu_clock_ghz"] == 2.25 and r["stored"]["gpu_clock_ghz"] == 2.25  # verdict r5 #6: a clock on every leg
    assert r["gpu_clock_source"].startswith("clv_clock_probe") and r["gpu_clock_probe_ghz"] == 2.25
    tb, ts = r["ms_per_step"], r["stored"]["ms_per_step"]
    n = 500
    want = n * 10000 / (5000 * tb + 5000 * ts) * 1e3
    assert abs(r["whole_run"]["value"] / want - 1) < 1e-9
    log.clear()
    r1 = bench.run_leg("c4", 1, 0, 0, None, 1000, 200, stored_phase=False)
    assert [(a, b) for a, b, _ in log] == [(1, 200), (201, 1200), (1201, 2200)] and "stored" not in r1


def test_bench_clock_settle_runs_a_scratch_sampler(monkeypatch):
    """The clock settle before each timed window sweeps a scratch sampler of its own (seed 7, no draws
    kept) over the same customers: the timed sampler runs exactly the warm-up and the timed steps,
    the scratch is closed with the leg, and the line names the settle work.  Stub samplers, no GPU."""
    import torch

    import bench
    from mcmc_clv_model_amd import sampler as S

    made = []

    class Fake:
        n = 500

        def __init__(self, p, **kw):
            self.kw, self.log, self.closed = kw, [], False
            made.append(self)

        def run(self, n):
            self.log.append(n)

        def synchronize(self):
            pass

        def launch_info(self):
            return dict(persistent=True)

        def set_timing(self, on):
            pass

        def kernel_time(self):
            return dict(sweep_ms=0.2, sweep_launches=20, hyper_ms=0.0, hyper_launches=0)

        def clock_ghz(self):
            return 2.38

        def clock_probe(self, us):
            return 2.4

        def host_times(self):
            return {}

        def close(self):
            self.closed = True

    monkeypatch.setattr(S, "HipSampler", Fake)
    monkeypatch.setattr(S, "build_problem", lambda df, covs, D: None)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    r = bench.run_leg("c2", 1, 0, 0, None, 20, 5, settle_ms=5.0, stored_phase=False)
    timed, scratch = made
    assert timed.kw["seed"] == 42 and timed.log == [5, 20]  # warm-up, then exactly the timed steps
    assert scratch.kw["seed"] == 7 and scratch.kw["draw_sink"] == "none" and scratch.kw["chains"] == timed.kw["chains"]
    assert len(scratch.log) >= 1 and scratch.closed and timed.closed
    assert r["clock_settle_ms"] >= 5.0 and r["clock_settle_work"].startswith("sweeps of a scratch sampler")
    monkeypatch.setattr(bench, "SETTLE_WORK", "matmul")
    monkeypatch.setattr(bench, "settle_clocks", lambda ms, dev, scratch=None: 0.005)
    made.clear()
    r = bench.run_leg("c2", 1, 0, 0, None, 20, 5, settle_ms=5.0, stored_phase=False)
    assert len(made) == 1 and r["clock_settle_work"] == "fp64 matmuls"


def test_bench_primary_is_a_baseline_configuration():
    """Verdict r4 #7: the line's `value` is a BASELINE configuration at every N — c2 (configs[1]) on
    one GPU, the 8-GPU weak-scaling c5 (configs[4]) at N > 1 — and the other configurations run as
    `configs` legs (N = 1: c3, c4, c5; N > 1: c4 strong scaling and c2 tiled per rank, labelled
    non-BASELINE in the line)."""
    import bench
    assert bench.primary_workload(1) == "c2" and bench.BASELINE_INDEX["c2"] == 1
    for n in (2, 4, 8):
        assert bench.primary_workload(n) == "c5" and bench.BASELINE_INDEX["c5"] == 4
        assert bench.config_legs(n, "c5") == ["c4", "c2"]
    assert bench.config_legs(1, "c2") == ["c3", "c4", "c5", "c4_shard8"]
    assert bench.WORKLOADS["c4_shard8"][1].endswith(":shard0of8") and "c4_shard8" not in bench.BASELINE_INDEX
    assert bench.survey_bytes(2, 2, 0.1, "full") == pytest.approx(63.2) and \
        bench.survey_bytes(3, 3, 0.1, "full") == pytest.approx(96.0)
    assert bench.survey_bytes(2, 5, 1.0, "summary") == 84.0 and bench.survey_bytes(3, 9, 1.0, "summary") == 140.0
    assert bench.survey_bytes(2, 1, 1.0, "full") == 84.0
