"""Host side of the HIP sampler: reference-identical setup + the libclvmcmc handle.

The reference computes its setup on the host (design matrix, priors, initial values); this
module does the same with the same numpy/pandas operations so the constants handed to the
device are bit-identical to the reference's:

* design matrix / priors ........ bivariate/mcmc.py:467-479, trivariate/mcmc.py:615-626
* initial lambda, mu, beta_0 .... bivariate/mcmc.py:367-374, trivariate/mcmc.py:488-499
* V = inv(X'X + A0) ............. bivariate/mcmc.py:248-249 (constant across sweeps)

Everything per sweep runs on the GPU (kernels.hip).
"""
from __future__ import annotations

import ctypes
import weakref
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check, dptr

BLOCK_SIZE = _lib.BLOCK


@dataclass
class Problem:
    """One CBS table prepared for the sampler (all arrays host-side, float64 unless noted)."""
    D: int
    K: int
    x: np.ndarray            # int32 repeat transactions
    t_x: np.ndarray
    T_cal: np.ndarray
    cov: np.ndarray          # (K-1, N) C-contiguous, non-intercept columns of X
    log_s: Optional[np.ndarray]
    lam_init: float
    beta_0: np.ndarray       # K x D (intercept row set from the data)
    A_0: np.ndarray
    nu_00: float
    gamma_00: np.ndarray
    V: np.ndarray            # inv(X'X + A0)
    omega2: float = 1.0
    covariates: List[str] = field(default_factory=list)

    @property
    def N(self) -> int:
        return int(self.x.shape[0])


def build_problem(cal_cbs, covariates: Optional[Sequence[str]], D: int) -> Problem:
    """Mirror of the reference's setup (see module docstring) for a pandas CBS DataFrame."""
    covariates = list(covariates or [])
    cbs = cal_cbs.copy().reset_index(drop=True)
    cbs["intercept"] = 1.0
    cols = ["intercept"] + covariates
    X = cbs[cols].to_numpy(float)
    N, K = X.shape
    if K > _lib.MAX_K:
        raise ValueError(f"at most {_lib.MAX_K - 1} covariates are supported (got {K - 1})")
    x = cbs["x"].to_numpy()
    t_x = np.ascontiguousarray(cbs["t_x"].to_numpy(), dtype=np.float64)
    T_cal = np.ascontiguousarray(cbs["T_cal"].to_numpy(), dtype=np.float64)
    if N and (np.any(x < 0) or np.any(x > np.iinfo(np.int32).max) or np.any(x != np.round(x))):
        raise ValueError("x must hold non-negative integer counts")

    # bi:368-374 / tri:489-499
    lam_init = cbs["x"].mean() / np.mean(np.where(cbs["t_x"] == 0, cbs["T_cal"], cbs["t_x"]))
    lambdas = np.full(N, lam_init)
    mus = 1.0 / (t_x + 0.5 / lam_init)
    beta_0 = np.zeros((K, D))
    beta_0[0, 0] = math.log(lambdas.mean())
    beta_0[0, 1] = math.log(mus.mean())
    log_s = None
    omega2 = 1.0
    if D == 3:
        log_s = np.ascontiguousarray(cbs["log_s"].to_numpy(), dtype=np.float64)
        omega2 = float(cbs["log_s"].var())
        beta_0[0, 2] = cbs["log_s"].mean()
    A_0 = np.eye(K) * 0.01
    nu_00 = (3 if D == 2 else 4) + K
    gamma_00 = nu_00 * np.eye(D)
    V = np.linalg.inv(X.T @ X + A_0)
    return Problem(D=D, K=K, x=np.ascontiguousarray(x, dtype=np.int32), t_x=t_x, T_cal=T_cal,
                   cov=np.ascontiguousarray(X[:, 1:].T), log_s=log_s, lam_init=float(lam_init),
                   beta_0=beta_0, A_0=A_0, nu_00=float(nu_00), gamma_00=gamma_00, V=V,
                   omega2=omega2, covariates=covariates)


def make_prior(p: Problem, n_global: Optional[int] = None) -> _lib.ClvPrior:
    pr = _lib.ClvPrior()
    K, D = p.K, p.D
    pr.lam_init = p.lam_init
    cholV = np.linalg.cholesky(p.V)
    A0B0 = p.A_0 @ p.beta_0
    S0B = p.gamma_00 + p.beta_0.T @ p.A_0 @ p.beta_0
    for i, v in enumerate(p.V.ravel()):
        pr.V[i] = v
    for i, v in enumerate(cholV.ravel()):
        pr.chol_V[i] = v
    for i, v in enumerate(A0B0.ravel()):
        pr.A0B0[i] = v
    for i, v in enumerate(S0B.ravel()):
        pr.S0_B0A0B0[i] = v
    pr.nu_n = p.nu_00 + (p.N if n_global is None else n_global)
    for i, v in enumerate(p.beta_0.ravel()):
        pr.beta_init[i] = v
    for i, v in enumerate(p.gamma_00.ravel()):
        pr.sigma_init[i] = v
    pr.omega2 = p.omega2
    return pr


def resolve_seed(seed: Optional[int]) -> int:
    if seed is None:  # reference: default_rng(None) -> OS entropy (bi:486)
        return int(np.random.SeedSequence().entropy) & ((1 << 63) - 1)
    seed = int(seed)
    if seed < 0:  # numpy: default_rng(seed + ch) with a negative seed raises (bi:486)
        raise ValueError("expected non-negative integer")
    if seed >= 1 << 63:
        # numpy accepts any non-negative int (default_rng(seed + ch), bi:486); the Philox key holds
        # 64 bits, so a larger seed is folded to 63 bits deterministically through numpy's own
        # SeedSequence hash (chain c then keys on the folded seed + c)
        w = np.random.SeedSequence(seed).generate_state(2, np.uint32)
        return (int(w[0]) | (int(w[1]) << 32)) & ((1 << 63) - 1)
    return seed


# "summary+pct": the summary sums plus a float32 (lambda, mu) store for Table 4's percentiles
_SINKS = {"full": _lib.SINK_FULL, "summary": _lib.SINK_SUMMARY, "summary+pct": _lib.SINK_SUMMARY_PCT,
          "none": _lib.SINK_NONE}
_RNGS = {"philox": _lib.RNG_PHILOX, "replay": _lib.RNG_REPLAY}


class HipSampler:
    """One libclvmcmc handle: ``chains`` chains of one problem (or one shard of it) on one GPU."""

    def __init__(self, p: Problem, *, mcmc: int, burnin: int, thin: int, chains: int, seed: int,
                 n_mh_steps: int = 20, draw_sink: str = "full", rng: str = "philox", device: int = -1,
                 chain_first: int = 0, n_global: Optional[int] = None, shard_begin: int = 0,
                 world_size: int = 1, rank: int = 0, blocks_per_rank: int = 0, blocks_per_unit: int = 0,
                 stream: int = 0, prior: Optional[_lib.ClvPrior] = None):
        L = _lib.lib()
        if draw_sink not in _SINKS:
            raise ValueError(f"draw_sink must be one of {sorted(_SINKS)}")
        if rng not in _RNGS:
            raise ValueError(f"rng must be one of {sorted(_RNGS)}")
        if _lib.device_count() < 1:
            raise _lib.ClvError("no HIP device visible; the sampler has no CPU fallback")
        self.p = p
        self.D, self.K, self.n = p.D, p.K, p.N
        self.chains = int(chains)
        self.mcmc, self.burnin, self.thin = int(mcmc), int(burnin), int(thin)
        self.n_draws = (self.mcmc - 1) // self.thin + 1 if self.mcmc >= 1 else 0
        self.draw_sink = draw_sink
        cfg = _lib.ClvConfig()
        cfg.abi_version = _lib.ABI_VERSION
        cfg.D, cfg.K, cfg.n_mh_steps = p.D, p.K, int(n_mh_steps)
        cfg.burnin, cfg.mcmc, cfg.thin = self.burnin, self.mcmc, self.thin
        cfg.n_chains, cfg.chain_first = self.chains, int(chain_first)
        cfg.rng_mode, cfg.draw_sink, cfg.device = _RNGS[rng], _SINKS[draw_sink], int(device)
        cfg.seed = int(seed)
        cfg.n_global = int(p.N if n_global is None else n_global)
        cfg.shard_begin = int(shard_begin)
        cfg.world_size, cfg.rank = int(world_size), int(rank)
        cfg.blocks_per_rank, cfg.blocks_per_unit = int(blocks_per_rank), int(blocks_per_unit)
        cfg.stream = int(stream)
        self.cfg = cfg
        data = _lib.ClvData()
        data.n = p.N
        self._keep = [p.x, p.t_x, p.T_cal, p.cov, p.log_s]
        data.x = p.x.ctypes.data if p.N else None
        data.t_x = p.t_x.ctypes.data if p.N else None
        data.T_cal = p.T_cal.ctypes.data if p.N else None
        data.covariates = p.cov.ctypes.data if (p.K > 1 and p.N) else None
        data.log_s = p.log_s.ctypes.data if (p.D == 3 and p.N) else None
        self.prior = prior if prior is not None else make_prior(p, cfg.n_global)
        h = ctypes.c_void_p()
        check(L.clv_create(ctypes.byref(cfg), ctypes.byref(data), ctypes.byref(self.prior), ctypes.byref(h)))
        self.h = h
        self._L = L

    # ---- lifecycle
    def close(self) -> None:
        """Destroy the handle.  A live HipGroup over this shard is closed first: clv_group_destroy
        disconnects and synchronises its shards, so it must never run after a shard is gone."""
        for grp in list(getattr(self, "_groups", ())):
            grp.close()
        if getattr(self, "h", None):
            self._L.clv_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- running
    def run(self, n_sweeps: int) -> None:
        check(self._L.clv_run(self.h, int(n_sweeps)))

    def rollback(self) -> None:
        """Undo the last completed persistent clv_run (clv_rollback)."""
        check(self._L.clv_rollback(self.h))

    def sweep(self) -> None:
        check(self._L.clv_sweep(self.h))

    def hyper(self, gathered_ptr: Optional[int] = None) -> None:
        check(self._L.clv_hyper(self.h, gathered_ptr))

    def partials(self):
        ptr = ctypes.c_void_p()
        nd = ctypes.c_int64()
        st = ctypes.c_int32()
        check(self._L.clv_partials(self.h, ctypes.byref(ptr), ctypes.byref(nd), ctypes.byref(st)))
        return ptr.value, nd.value, st.value

    def set_stream(self, stream: int) -> None:
        check(self._L.clv_set_stream(self.h, int(stream)))

    def note_sweeps(self, n: int) -> None:
        check(self._L.clv_note_sweeps(self.h, int(n)))

    def copy_partials(self, dst_ptr: int) -> None:
        check(self._L.clv_copy_partials(self.h, ctypes.c_void_p(dst_ptr)))

    def synchronize(self) -> None:
        check(self._L.clv_synchronize(self.h))

    def host_times(self) -> dict:
        """clv_debug_host_times of the last persistent clv_run, as microsecond splits: hipSetDevice,
        the start event's record, the launch call, the end event's record, the wait for the end,
        the return path."""
        hn = (ctypes.c_int64 * 8)()
        check(self._L.clv_debug_host_times(self.h, hn))
        h = [x / 1e3 for x in hn]
        if not h[0] or not h[6]:
            return {}
        names = ("set_device", "start_event", "launch_call", "end_event", "wait", "return")
        return {k: round(h[i + 1] - h[i], 3) for i, k in enumerate(names)}

    def clock_ghz(self) -> float:
        """clv_clock_ghz: the average shader clock (GHz) over the last run(), recorded by the
        persistent kernel; 0.0 when nothing was recorded (a run of fewer than 2 sweeps, or one
        without the persistent kernel: the launch-per-sweep kernel keeps no record — see
        clock_probe)."""
        v = ctypes.c_double(0.0)
        check(self._L.clv_clock_ghz(self.h, ctypes.byref(v)))
        return float(v.value)

    def clock_probe(self, us: float = 50.0) -> float:
        """clv_clock_probe: the shader clock (GHz) read by a `us`-microsecond probe kernel enqueued
        on this sampler's stream behind the launches already there (csrc/probe.hip)."""
        v = ctypes.c_double(0.0)
        check(self._L.clv_clock_probe(self.h, float(us), ctypes.byref(v)))
        return float(v.value)

    def launch_info(self) -> dict:
        """How clv_run launches (clv_launch_info): persistent kernel or one launch per sweep."""
        out = (ctypes.c_int64 * 6)()
        check(self._L.clv_launch_info(self.h, out))
        return dict(persistent=bool(out[0]), persist_blocks_per_cu=int(out[1]), n_cu=int(out[2]),
                    workgroups=int(out[3]))

    # ---- peer exchange (world size > 1 through the persistent kernel, include/clvmcmc.h)
    IPC_HANDLE_BYTES = 64

    def p2p_info(self) -> dict:
        """clv_p2p_info: peer exchange possible / connected, the mail buffer, and whether clv_run
        runs it in one persistent launch (else one fused sweep launch per sweep)."""
        out = (ctypes.c_int64 * 6)()
        check(self._L.clv_p2p_info(self.h, out))
        return dict(capable=bool(out[0]), connected=bool(out[1]), mail_bytes=int(out[2]), mail_ptr=int(out[3]),
                    persistent=bool(out[4]), mail_memory={0: "uncached", 1: "fine-grained", 2: "device"}.get(int(out[5])))

    def p2p_export(self) -> bytes:
        """This rank's mail buffer as a hipIpcMemHandle (bytes) for the other ranks."""
        buf = ctypes.create_string_buffer(self.IPC_HANDLE_BYTES)
        check(self._L.clv_p2p_export(self.h, buf))
        return buf.raw

    def p2p_connect(self, handles: Optional[Sequence[bytes]] = None, ptrs: Optional[Sequence[int]] = None) -> None:
        """Every rank's mail: IPC handles (one process per GPU) or device pointers (one process)."""
        if handles is not None:
            blob = ctypes.create_string_buffer(b"".join(handles), self.IPC_HANDLE_BYTES * len(handles))
            check(self._L.clv_p2p_connect(self.h, blob, None))
        else:
            arr = (ctypes.c_uint64 * len(ptrs))(*[int(p) for p in ptrs])
            check(self._L.clv_p2p_connect(self.h, None, arr))

    def p2p_set_persistent(self, on: bool) -> None:
        """clv_p2p_set_persistent: the persistent peer exchange (where its grid fits) or the fused one."""
        check(self._L.clv_p2p_set_persistent(self.h, 1 if on else 0))

    def p2p_disconnect(self) -> None:
        """clv_p2p_disconnect: forget the peers' mail (a sharded run() needs p2p_connect again)."""
        check(self._L.clv_p2p_disconnect(self.h))

    def set_wait_timeout(self, ms: float) -> None:
        """clv_set_wait_timeout: the bound of every in-kernel wait (ms)."""
        check(self._L.clv_set_wait_timeout(self.h, float(ms)))

    @property
    def sweeps_done(self) -> int:
        return int(self._L.clv_sweeps_done(self.h))

    def set_replay_tape(self, tape: np.ndarray, n_sweeps: int) -> None:
        tape = np.ascontiguousarray(tape, dtype=np.float64)
        stride = self.replay_sweep_stride
        if tape.size != self.chains * n_sweeps * stride:
            raise ValueError(f"tape has {tape.size} doubles, expected {self.chains * n_sweeps * stride}")
        check(self._L.clv_set_replay_tape(self.h, dptr(tape), int(n_sweeps)))

    @property
    def replay_sweep_stride(self) -> int:
        return int(self._L.clv_replay_sweep_stride(self.h))

    # ---- outputs
    def level1_buffer(self) -> np.ndarray:
        """An uninitialised host array in the level-1 layout [chain][draw][n][D+2] (reference:
        bi:360-364), for stream_draws / read_draws(out=...)."""
        return np.empty((self.chains, self.n_draws, self.n, self.D + 2))

    def stream_draws(self, level1: Optional[np.ndarray]) -> None:
        """clv_stream_draws: copy the level-1 draws into ``level1`` while the sampler runs (host copy
        pool, overlapped with later sweeps); read_draws(out=level1) then only finishes the copy.
        ``None`` stops streaming."""
        if level1 is not None:
            C, nd, n, D = self.chains, self.n_draws, self.n, self.D
            if (level1.shape != (C, nd, n, D + 2) or level1.dtype != np.float64 or not level1.flags.c_contiguous
                    or not level1.flags.writeable):
                raise ValueError("level1 must be a writeable C-contiguous float64 array of shape (chains, n_draws, n, D+2)")
        self._stream_buf = level1  # kept alive while the library writes into it
        check(self._L.clv_stream_draws(self.h, dptr(level1)))

    def read_draws(self, level1: bool = True, out: Optional[np.ndarray] = None):
        C, nd, n, D, K = self.chains, self.n_draws, self.n, self.D, self.K
        l1 = None
        if level1 and self.draw_sink == "full":
            l1 = out if out is not None else self.level1_buffer()
        l2 = np.empty((C, nd, D * K + D * (D + 1) // 2))
        ll = np.empty((C, nd))
        check(self._L.clv_read_draws(self.h, dptr(l1), dptr(l2), dptr(ll)))
        return l1, l2, ll

    def flush(self) -> None:
        """Draw a pending deferred level-2 draw now (clv_get_state with only the hyper output)."""
        hyp = np.empty((self.chains, self.K * self.D + self.D * self.D))
        check(self._L.clv_get_state(self.h, None, None, dptr(hyp)))

    def read_summary(self):
        sums = np.empty((self.chains, _lib.N_SUM_STATS, self.n))  # also for "summary+pct"
        k = ctypes.c_int64()
        check(self._L.clv_read_summary(self.h, dptr(sums), ctypes.byref(k)))
        return sums, int(k.value)

    def get_state(self):
        C, n, D, K = self.chains, self.n, self.D, self.K
        lam, mu = np.empty((C, n)), np.empty((C, n))
        hyp = np.empty((C, K * D + D * D))
        check(self._L.clv_get_state(self.h, dptr(lam), dptr(mu), dptr(hyp)))
        beta = hyp[:, : K * D].reshape(C, K, D)
        sigma = hyp[:, K * D:].reshape(C, D, D)
        return lam, mu, beta, sigma

    def set_state(self, lam, mu, beta, sigma, sweeps_done: int) -> None:
        C, n, D, K = self.chains, self.n, self.D, self.K
        lam = np.ascontiguousarray(np.broadcast_to(lam, (C, n)), dtype=np.float64)
        mu = np.ascontiguousarray(np.broadcast_to(mu, (C, n)), dtype=np.float64)
        hyp = np.concatenate([np.broadcast_to(beta, (C, K, D)).reshape(C, K * D),
                              np.broadcast_to(sigma, (C, D, D)).reshape(C, D * D)], axis=1)
        hyp = np.ascontiguousarray(hyp, dtype=np.float64)
        check(self._L.clv_set_state(self.h, dptr(lam), dptr(mu), dptr(hyp), int(sweeps_done)))

    # ---- posterior analysis on the draws this sampler holds in HBM (draw_sink="full", run done)
    def predict(self, T_star: float = 39.0, seed: Optional[int] = None, simulate_spend: bool = False,
                sigma_s: float = 0.5):
        """clv_predict_sampler: analysis.draw_future_transactions without the host round trip."""
        nd = self.chains * self.n_draws
        x = np.empty((nd, self.n), np.int64)
        spend = np.empty((nd, self.n), np.float64) if simulate_spend else None
        check(self._L.clv_predict_sampler(self.h, float(T_star), resolve_seed(seed), 1 if simulate_spend else 0,
                                          float(sigma_s), x.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                          dptr(spend)))
        return (x, spend) if simulate_spend else x

    def level1_summary(self, mu_cap: float = 0.05) -> np.ndarray:
        """clv_level1_summary_sampler: [n][len(_lib.L1_STATS)] per-customer statistics (full sink:
        from the level-1 draws in HBM; "summary+pct": means from the running sums, percentiles from
        the float32 (lambda, mu) store)."""
        out = np.empty((self.n, len(_lib.L1_STATS)), np.float64)
        check(self._L.clv_level1_summary_sampler(self.h, float(mu_cap), dptr(out)))
        return out

    def chain_total_loglik(self) -> float:
        out = ctypes.c_double()
        check(self._L.clv_chain_total_loglik_sampler(self.h, ctypes.byref(out)))
        return float(out.value)

    def track(self, birth_week, times, seed: Optional[int] = 0) -> np.ndarray:
        b = np.ascontiguousarray(np.asarray(birth_week, dtype=np.float64))
        t = np.ascontiguousarray(np.asarray(times, dtype=np.float64))
        out = np.empty(t.shape[0], np.float64)
        check(self._L.clv_track_sampler(self.h, dptr(b), dptr(t), t.shape[0], resolve_seed(seed), dptr(out)))
        return out

    def set_timing(self, enable: bool) -> None:
        check(self._L.clv_set_timing(self.h, 1 if enable else 0))

    def kernel_time(self):
        a, b = ctypes.c_double(), ctypes.c_double()
        na, nb = ctypes.c_int64(), ctypes.c_int64()
        check(self._L.clv_kernel_time(self.h, ctypes.byref(a), ctypes.byref(na), ctypes.byref(b), ctypes.byref(nb)))
        return dict(sweep_ms=a.value, sweep_launches=na.value, hyper_ms=b.value, hyper_launches=nb.value)


_EXCHANGES = {"auto": _lib.EXCHANGE_AUTO, "p2p": _lib.EXCHANGE_P2P, "copy": _lib.EXCHANGE_COPY}


class HipGroup:
    """clv_group (include/clvmcmc.h): the shards of one problem — HipSampler handles of ranks
    0..n-1 of a world of n, on their own devices or sharing one — run from this one thread, with
    the unit partials exchanged per sweep by peer stores (persistent kernels, "p2p") or
    stream-ordered device-to-device copies ("copy").  Does not own the shards."""

    def __init__(self, shards: Sequence[HipSampler], exchange: str = "auto"):
        if exchange not in _EXCHANGES:
            raise ValueError(f"exchange must be one of {sorted(_EXCHANGES)}")
        L = _lib.lib()
        arr = (ctypes.c_void_p * len(shards))(*[sh.h.value for sh in shards])
        h = ctypes.c_void_p()
        check(L.clv_group_create(arr, len(shards), _EXCHANGES[exchange], ctypes.byref(h)))
        self.h, self._L, self.shards = h, L, list(shards)
        for sh in self.shards:  # back-references: a shard's close() closes this group first
            if not hasattr(sh, "_groups"):
                sh._groups = weakref.WeakSet()
            sh._groups.add(self)

    def run(self, n_sweeps: int) -> None:
        check(self._L.clv_group_run(self.h, int(n_sweeps)))

    @property
    def exchange(self) -> str:
        return {_lib.EXCHANGE_P2P: "p2p", _lib.EXCHANGE_COPY: "copy"}[int(self._L.clv_group_exchange(self.h))]

    def close(self) -> None:
        if getattr(self, "h", None):
            self._L.clv_group_destroy(self.h)
            self.h = None
        for sh in getattr(self, "shards", ()):
            g = getattr(sh, "_groups", None)
            if g is not None:
                g.discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def trace_marks(total: int, trace: int) -> List[int]:
    """Steps at which the reference prints its trace line (bi:383-384: ``step % trace == 0``)."""
    return [m for m in range(trace, total + 1, trace)] if trace else []


def run_with_trace(s: HipSampler, total: int, trace: int, n_chains_label: int = 1, chain_offset: int = 0) -> None:
    """Run ``total`` sweeps, printing the reference's trace line (bi:383-384) for every chain at
    every step that is a multiple of ``trace``, in the reference's order: its chains run one after
    another (bi:484), so all lines of chain 1 come before any line of chain 2.  Here the chains
    advance together: chain 1's lines are printed live (as the reference does, before the step
    runs), the other chains' lines — identical text — once all sweeps are done."""
    marks = trace_marks(total, trace)
    done = 0
    for m in marks:
        if m - 1 > done:  # the reference prints at the start of step m
            s.run(m - 1 - done)
            done = m - 1
        print(f"chain {chain_offset + 1} | step {m}/{total}")
    if total > done:
        s.run(total - done)
    for ch in range(1, n_chains_label):
        for m in marks:
            print(f"chain {chain_offset + ch + 1} | step {m}/{total}")


def _assemble(D: int, chains: int, l1, l2, ll, sums, k: int, n_draws: int, draw_sink: str, level1_stats) -> dict:
    """The reference's output layout (bi:499-504) from [chain]-leading arrays: level_1 / level_2
    lists with one array per chain, the marginal log-likelihood = mean over all chains' per-draw
    means, and (summary sinks) the per-customer running means."""
    out = dict(level_1=[l1[c] for c in range(chains)] if l1 is not None else None,
               level_2=[l2[c] for c in range(chains)],
               log_likelihood=np.mean(ll.reshape(-1)) if ll.size else np.float64("nan"))
    if draw_sink in ("summary", "summary+pct"):
        names = [nm for nm in _lib.SUM_STATS if D == 3 or nm not in ("eta", "log_eta")]
        out["summary"] = dict(n_draws=k, **{nm: sums[:, _lib.SUM_STATS.index(nm), :] / max(k, 1) for nm in names})
        if draw_sink == "summary+pct" and k == n_draws and k > 0:
            # per-customer posterior statistics pooled over chains (Table 4's columns)
            import pandas as pd
            cols = list(_lib.L1_STATS if D == 3 else _lib.L1_STATS[:-1])
            out["summary"]["level1"] = pd.DataFrame(level1_stats()[:, :len(cols)], columns=cols)
    return out


def fit(p: Problem, *, mcmc: int, burnin: int, thin: int, chains: int, seed, trace: int, n_mh_steps: int,
        draw_sink: str = "full", rng: str = "philox", device: int = -1, replay_tape=None,
        replay_sweeps: Optional[int] = None, devices: Optional[Sequence[int]] = None, shard: str = "auto",
        exchange: str = "auto") -> dict:
    """Run all chains of one problem in one batched launch sequence and return the reference's
    output layout (bi:499-504).  ``devices`` (two or more): the run is spread over those devices
    in this process (:func:`fit_multi`)."""
    if chains < 1:
        raise ValueError("chains must be >= 1")
    if thin < 1:
        raise ValueError("thin must be >= 1")
    if devices is not None:
        devices = [int(d) for d in devices]
        if not devices:
            raise ValueError("devices must name at least one device")
        if len(devices) > 1:
            if rng != "philox":
                raise ValueError("devices= runs need rng='philox' (the replay tape is a single-device test mode)")
            return fit_multi(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=seed, trace=trace,
                             n_mh_steps=n_mh_steps, draw_sink=draw_sink, devices=devices, shard=shard,
                             exchange=exchange)
        device = devices[0]
    s = HipSampler(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=resolve_seed(seed),
                   n_mh_steps=n_mh_steps, draw_sink=draw_sink, rng=rng, device=device)
    try:
        if rng == "replay":
            if replay_tape is None:
                raise ValueError("rng='replay' needs replay_tape")
            s.set_replay_tape(replay_tape, replay_sweeps)
        l1 = None
        if draw_sink == "full" and s.n_draws > 0 and p.N > 0:
            # the draws reach the returned arrays while later sweeps run (clv_stream_draws)
            l1 = s.level1_buffer()
            s.stream_draws(l1)
        run_with_trace(s, burnin + mcmc, trace, n_chains_label=chains)
        l1, l2, ll = s.read_draws(level1=draw_sink == "full", out=l1)
        sums, k = s.read_summary() if draw_sink in ("summary", "summary+pct") else (None, 0)
        return _assemble(p.D, chains, l1, l2, ll, sums, k, s.n_draws, draw_sink,
                         lambda: s.level1_summary(_lib.SUMMARY_MU_CAP))
    finally:
        s.close()


def multi_plan(chains: int, n_dev: int, draw_sink: str, shard: str = "auto"):
    """How :func:`fit_multi` spreads a run over ``n_dev`` devices: ("chains", [(first chain,
    chains), ...] one group per device used) or ("customers", None).  "auto" takes chain groups
    when the chains divide evenly over the devices and the sink does not pool chains."""
    if shard not in ("auto", "chains", "customers"):
        raise ValueError("shard must be 'auto', 'chains' or 'customers'")
    if chains < 1 or n_dev < 1:
        raise ValueError("chains and devices must be >= 1")
    if shard == "auto":
        shard = "chains" if (chains % n_dev == 0 and draw_sink != "summary+pct") else "customers"
    if shard == "chains" and draw_sink == "summary+pct":
        raise ValueError("draw_sink='summary+pct' pools every chain's draws: use shard='customers'")
    if shard == "customers":
        return shard, None
    n_grp = min(n_dev, chains)
    sizes = [chains // n_grp + (1 if g < chains % n_grp else 0) for g in range(n_grp)]
    return shard, [(sum(sizes[:g]), sizes[g]) for g in range(n_grp)]


def fit_multi(p: Problem, *, mcmc: int, burnin: int, thin: int, chains: int, seed, trace: int, n_mh_steps: int,
              draw_sink: str, devices: Sequence[int], shard: str = "auto", exchange: str = "auto") -> dict:
    """One run over several devices of this process (SURVEY §8b ``devices=``), same output as the
    single-device run, bit for bit:

    * ``shard="chains"``: the chains in contiguous groups, one group per device, each group run from
      its own host thread (the reference runs its chains one after another, bi:481-488 — they are
      independent; Philox draws depend on (seed, chain, customer, sweep) only);
    * ``shard="customers"``: every chain's customers split into contiguous shards (the shard plan
      of :mod:`distributed`), one per device, exchanging the level-2 statistics every sweep
      (:class:`HipGroup`: peer stores from persistent kernels where every grid fits at once, else
      device-to-device copies; ``exchange`` forces one);
    * ``"auto"``: chains when they divide evenly over the devices (and the sink is not
      "summary+pct", whose percentiles pool all chains), else customers."""
    import threading
    n_dev = len(devices)
    shard, groups = multi_plan(chains, n_dev, draw_sink, shard)
    seed = resolve_seed(seed)
    total = burnin + mcmc
    kw = dict(mcmc=mcmc, burnin=burnin, thin=thin, seed=seed, n_mh_steps=n_mh_steps, draw_sink=draw_sink)
    if shard == "chains":
        n_grp = len(groups)
        firsts = [g[0] for g in groups]
        sizes = [g[1] for g in groups]
        samplers = []
        try:
            for g in range(n_grp):
                samplers.append(HipSampler(p, chains=sizes[g], chain_first=firsts[g], device=devices[g], **kw))
            errs = []

            def go(g):
                try:
                    if g == 0:  # chain 1's trace lines live, as the reference prints them
                        run_with_trace(samplers[0], total, trace, n_chains_label=1)
                    else:
                        samplers[g].run(total)
                except Exception as e:  # noqa: BLE001 - re-raised below
                    errs.append(e)
            th = [threading.Thread(target=go, args=(g,)) for g in range(n_grp)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            if errs:
                raise errs[0]
            for ch in range(1, chains):
                for m in trace_marks(total, trace):
                    print(f"chain {ch + 1} | step {m}/{total}")
            reads = [sm.read_draws(level1=draw_sink == "full") for sm in samplers]
            l1 = np.concatenate([r[0] for r in reads], axis=0) if draw_sink == "full" else None
            l2 = np.concatenate([r[1] for r in reads], axis=0)
            ll = np.concatenate([r[2] for r in reads], axis=0)
            sums, k = (None, 0)
            if draw_sink == "summary":
                rs = [sm.read_summary() for sm in samplers]
                sums, k = np.concatenate([r[0] for r in rs], axis=0), rs[0][1]
            return _assemble(p.D, chains, l1, l2, ll, sums, k, samplers[0].n_draws, draw_sink, None)
        finally:
            for sm in samplers:
                sm.close()
    # customers
    from . import distributed as Dm
    plan = Dm.plan(p.N, n_dev)
    prior = make_prior(p, p.N)
    shards = []
    group = None
    try:
        for r in range(n_dev):
            b, e = plan.shard(r)
            shards.append(HipSampler(Dm.slice_problem(p, b, e), chains=chains, device=devices[r], n_global=p.N,
                                     shard_begin=r * plan.blocks_per_rank * BLOCK_SIZE, world_size=n_dev, rank=r,
                                     blocks_per_rank=plan.blocks_per_rank, blocks_per_unit=plan.blocks_per_unit,
                                     prior=prior, **kw))
        group = HipGroup(shards, exchange)
        done = 0
        for m in trace_marks(total, trace):  # as run_with_trace: chain 1 live, the others after
            if m - 1 > done:
                group.run(m - 1 - done)
                done = m - 1
            print(f"chain 1 | step {m}/{total}")
        if total > done:
            group.run(total - done)
        for ch in range(1, chains):
            for m in trace_marks(total, trace):
                print(f"chain {ch + 1} | step {m}/{total}")
        reads = [sh.read_draws(level1=draw_sink == "full") for sh in shards]
        l1 = np.concatenate([r[0] for r in reads], axis=2) if draw_sink == "full" else None
        l2, ll = reads[0][1], reads[0][2]  # every shard drew the same level 2 (same bits)
        sums, k = (None, 0)
        if draw_sink in ("summary", "summary+pct"):
            rs = [sh.read_summary() for sh in shards]
            sums, k = np.concatenate([r[0] for r in rs], axis=2), rs[0][1]
        out = _assemble(p.D, chains, l1, l2, ll, sums, k, shards[0].n_draws, draw_sink,
                        lambda: np.concatenate([sh.level1_summary(_lib.SUMMARY_MU_CAP) for sh in shards], axis=0))
        out["exchange"] = group.exchange
        return out
    finally:
        if group is not None:
            group.close()
        for sh in shards:
            sh.close()
