"""Customer sharding across GPUs: one process per GPU, one exchange per sweep.

Customers are conditionally independent given (beta, Sigma) (bivariate/mcmc.py:193-339), so
each rank sweeps its own contiguous customer range; the only coupling is the level-2 draw
(bivariate/mcmc.py:233-262), which needs the sufficient statistics X'Y, Y'Y of ALL customers.
Per sweep each rank publishes its unit partials, one ``all_gather_into_tensor`` over
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X; "gloo" in the CPU tests)
assembles [world][chain][stride][units_per_rank], and every rank performs the identical
fixed-order sum and the identical level-2 draw (same Philox counter), so no broadcast is needed
and results are bitwise independent of the GPU count.

``exchange="p2p"`` (or "auto": p2p where possible and verified, else RCCL) replaces the host
collective per sweep: the ranks swap hipIpcMemHandles of their mail buffers once, and the
persistent sweep kernel's level-2 workgroup of each chain stores its rank's unit partials
straight into every rank's mail over xGMI, waits for all ranks' units in its own mail and sums
them in the same global order — one kernel launch per step per rank, same bits as RCCL.

Shard plan (a function of n_global and world only):
  blocks_per_unit G  = clv_default_blocks_per_unit(n_global)     (units <= 512)
  blocks_per_rank    = ceil(ceil(n_blocks / world) / G) * G
  shard r            = customers [r * blocks_per_rank * 256, min(n, (r+1) * blocks_per_rank * 256))
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib

BLOCK = _lib.BLOCK
VERIFY_WAIT_MS = 500.0  # in-kernel wait bound while the peer exchange is checked against RCCL


def run_wait_ms() -> float:
    """The wait bound afterwards: clv_create's default with peers (10 s) or CLV_WAIT_TIMEOUT_MS,
    under clv_create's rule (capi.hip parse_wait_ms): a finite decimal number of ms, blanks around
    it allowed, clamped to [1 ms, 1 h]; anything else (hex, inf, nan, trailing text) is rejected —
    clv_create fails on it, so this raises ValueError."""
    import os
    import re
    v = os.environ.get("CLV_WAIT_TIMEOUT_MS")
    if v is None:
        return 10000.0
    t = v.strip(" \t\n")
    if not re.fullmatch(r"[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?", t):
        raise ValueError(f"CLV_WAIT_TIMEOUT_MS must be a finite decimal number of ms (got {v!r})")
    ms = float(t)
    if ms != ms or abs(ms) > 1e300:
        raise ValueError(f"CLV_WAIT_TIMEOUT_MS must be a finite decimal number of ms (got {v!r})")
    return min(3.6e6, max(1.0, ms))


def graph_sizes_all(chunk: int) -> list:
    """The graph sizes a step may replay: ``chunk`` and every power of two below it."""
    out, k = [int(chunk)], 1
    while k < chunk:
        out.append(k)
        k *= 2
    return sorted(set(out), reverse=True)


def graph_sizes(n: int, chunk: int) -> list:
    """Graph replays covering ``n`` sweeps: as many ``chunk``-sweep graphs as fit, then the binary
    decomposition of the rest (a 20-sweep step with chunk 32 replays the 16- and 4-sweep graphs),
    so no step of any length falls back to eager launches."""
    out = []
    if chunk <= 0:
        return out
    while n >= chunk:
        out.append(int(chunk))
        n -= chunk
    k = 1
    while k * 2 <= n:
        k *= 2
    while n > 0:
        if n >= k:
            out.append(k)
            n -= k
        k //= 2
    return out


def default_blocks_per_unit(n_global: int) -> int:
    """Same rule as clv_default_blocks_per_unit (C) — kept in Python for CPU-side planning."""
    nb = -(-n_global // BLOCK)
    g = 1
    while -(-nb // g) > 512:
        g *= 2
    return g


@dataclass(frozen=True)
class ShardPlan:
    n_global: int
    world: int
    blocks_per_unit: int
    blocks_per_rank: int

    @property
    def units_per_rank(self) -> int:
        return self.blocks_per_rank // self.blocks_per_unit

    @property
    def n_units_global(self) -> int:
        nb = -(-self.n_global // BLOCK)
        return -(-nb // self.blocks_per_unit)

    def shard(self, rank: int):
        """[begin, end) customer range of ``rank``."""
        b = rank * self.blocks_per_rank * BLOCK
        e = min(self.n_global, (rank + 1) * self.blocks_per_rank * BLOCK)
        return min(b, self.n_global), max(min(b, self.n_global), e)


def plan(n_global: int, world: int, blocks_per_unit: Optional[int] = None) -> ShardPlan:
    if n_global < 1 or world < 1:
        raise ValueError("n_global and world must be >= 1")
    G = blocks_per_unit or default_blocks_per_unit(n_global)
    nb = -(-n_global // BLOCK)
    per = -(-nb // world)
    bpr = -(-per // G) * G
    return ShardPlan(n_global=n_global, world=world, blocks_per_unit=G, blocks_per_rank=bpr)


def slice_problem(p, begin: int, end: int):
    """The rank-local view of a Problem (setup constants stay global, like the reference's)."""
    from dataclasses import replace
    return replace(p, x=np.ascontiguousarray(p.x[begin:end]), t_x=np.ascontiguousarray(p.t_x[begin:end]),
                   T_cal=np.ascontiguousarray(p.T_cal[begin:end]),
                   cov=np.ascontiguousarray(p.cov[:, begin:end]),
                   log_s=None if p.log_s is None else np.ascontiguousarray(p.log_s[begin:end]))


def exchange(local, gathered, group=None) -> None:
    """All-gather this rank's unit partials (1-D tensor) into ``gathered`` (world * len).
    A "gloo" group (tests: several ranks sharing one GPU, which RCCL refuses) goes through host
    copies."""
    import torch.distributed as dist
    if local.is_cuda and dist.get_backend(group) == "gloo":
        h = gathered.new_empty(gathered.shape, device="cpu")
        dist.all_gather_into_tensor(h, local.cpu(), group=group)
        gathered.copy_(h)
        return
    dist.all_gather_into_tensor(gathered, local, group=group)


class _DeviceArray:
    """A float64 device buffer owned by the HIP library, exposed to torch without a copy."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = dict(shape=(int(n),), typestr="<f8", data=(int(ptr), False), version=3,
                                             strides=None)


class ShardedSampler:
    """This rank's shard of a problem on its GPU; sweeps with one all-gather per sweep.

    ``graph_chunk`` > 0: at the first step, that many sweeps (kernels, RCCL all-gather, level-2
    kernel) and every power of two below it are captured into torch.cuda graphs; a step of n
    sweeps replays ``graph_sizes(n, graph_chunk)`` of them (the sweep index lives in device memory,
    so a graph serves any step) — one replay per chunk instead of ~5 host calls per sweep, for
    steps of any length.
    """

    def __init__(self, p_global, *, rank: int, world: int, chains: int, mcmc: int, burnin: int, thin: int,
                 seed: int, n_mh_steps: int = 20, draw_sink: str = "summary", device: int = 0, group=None,
                 graph_chunk: int = 0, exchange: str = "rccl", verify_sweeps: int = 8):
        import torch
        from .sampler import HipSampler, make_prior
        self.torch = torch
        self.plan = plan(p_global.N, world)
        b, e = self.plan.shard(rank)
        self.begin, self.end = b, e
        self.rank, self.world, self.group = rank, world, group
        self.graph_chunk, self.graph, self.timing = int(graph_chunk), None, False
        torch.cuda.set_device(device)
        # One explicit stream carries the sampler's launches AND the exchange (copy, all-gather):
        # a sampler-owned non-blocking stream would not be ordered against torch's default stream.
        self.stream = torch.cuda.Stream(device=device)
        self.base_stream = self.stream.cuda_stream
        prior = make_prior(p_global, p_global.N)
        self.s = HipSampler(slice_problem(p_global, b, e), mcmc=mcmc, burnin=burnin, thin=thin, chains=chains,
                            seed=seed, n_mh_steps=n_mh_steps, draw_sink=draw_sink, device=device,
                            n_global=p_global.N, shard_begin=rank * self.plan.blocks_per_rank * BLOCK,
                            world_size=world, rank=rank, blocks_per_rank=self.plan.blocks_per_rank,
                            blocks_per_unit=self.plan.blocks_per_unit, stream=self.base_stream, prior=prior)
        self.n = self.s.n
        ptr, nd, _ = self.s.partials()
        # zero-copy view of the sampler's own unit-partial buffer: the sweep (or group) kernel
        # writes it, the all-gather reads it — no device-to-device copy node per sweep
        self.local = torch.as_tensor(_DeviceArray(ptr, nd), device=f"cuda:{device}")
        self.gathered = torch.zeros(nd * world, dtype=torch.float64, device=f"cuda:{device}")
        self.cur = self.stream  # the stream launches go to (a capture stream while capturing)
        self.D = p_global.D
        if self.D == 2:  # bivariate: the draw for sweep 1 comes from the initial state (bi:393)
            self._exchange_and_hyper()
        if exchange not in ("rccl", "p2p", "auto"):
            raise ValueError("exchange must be 'rccl', 'p2p' or 'auto'")
        self.exchange = "rccl"
        self.p2p_note = None
        if exchange != "rccl" and world > 1:
            self._setup_p2p(required=exchange == "p2p", verify_sweeps=int(verify_sweeps))

    # ---- peer exchange: the persistent kernel writes unit partials into every rank's mail over xGMI
    def _all_ok(self, ok: bool) -> bool:
        """True iff ``ok`` on every rank (MIN all-reduce over the process group)."""
        import torch.distributed as dist
        dev = "cpu" if dist.get_backend(self.group) == "gloo" else self.gathered.device
        t = self.torch.tensor([1 if ok else 0], dtype=self.torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(t.item())

    def _setup_p2p(self, required: bool, verify_sweeps: int) -> None:
        """Connect the ranks' mail buffers (hipIpcMemHandle exchange over the process group) so
        that clv_run runs all sweeps of a step in ONE persistent launch per rank, with no host
        collective per sweep.  ``verify_sweeps`` > 0 (burn-in sweeps only) first runs that many
        sweeps through the RCCL path and, from the same state, through the peer path, and keeps
        the peer path only if every rank's state is bitwise identical (else RCCL, or an error
        when ``required``)."""
        import torch.distributed as dist
        if verify_sweeps > 0 and self.s.sweeps_done + verify_sweeps > self.s.burnin:
            # the check replays sweeps from a saved state: only burn-in sweeps (nothing stored twice)
            if required:
                raise ValueError("verify_sweeps must fit in the burn-in (nothing may be stored twice); "
                                 "pass verify_sweeps=0 to skip the check")
            self.p2p_note = "not verified (burn-in shorter than verify_sweeps): all-gather path kept"
            return
        capable = self._all_ok(self.s.p2p_info()["capable"])
        if not capable:
            if required:
                raise _lib.ClvError("p2p exchange: not available on every rank")
            self.p2p_note = "not capable on every rank"
            return
        handles = [None] * self.world
        dist.all_gather_object(handles, self.s.p2p_export(), group=self.group)
        # the persistent peer exchange first where every rank's grid fits, then the fused one (one
        # sweep launch per sweep, same mail and bits), then RCCL: each path is kept only once it has
        # reproduced the RCCL path's state bitwise on every rank
        paths = ([True] if self._all_ok(self.s.p2p_info()["persistent"]) else []) + [False]
        notes = []
        for persistent in paths:
            err = None
            try:
                self.s.p2p_set_persistent(persistent)
                self.s.p2p_connect(handles=handles)
            except Exception as e:  # noqa: BLE001 - reported below, on every rank
                err = e
            kind = "persistent" if persistent else "fused"
            if not self._all_ok(err is None):
                notes.append(f"{kind}: connect failed ({err})")
                continue
            dist.barrier(group=self.group)
            ok, err = self._verify_p2p(verify_sweeps) if verify_sweeps > 0 else (True, None)
            if ok:
                self.exchange = "p2p"
                self.p2p_note = "; ".join(notes + [f"{kind} exchange" + (
                    f" verified bitwise against RCCL over {verify_sweeps} sweeps" if verify_sweeps > 0 else "")])
                return
            notes.append(f"{kind}: verification against RCCL failed ({err or 'state differs'})")
        try:
            self.s.p2p_disconnect()
        except Exception:  # noqa: BLE001
            pass
        if required:
            raise _lib.ClvError("p2p exchange: " + "; ".join(notes))
        self.p2p_note = "; ".join(notes)

    def _verify_p2p(self, verify_sweeps: int):
        """Run ``verify_sweeps`` sweeps through the RCCL path and, from the same state, through the
        connected peer path; (True, None) iff every rank's state is bitwise identical.  The state is
        restored either way, and the ranks leave in step."""
        import torch.distributed as dist
        n0 = self.s.sweeps_done
        snap = self.s.get_state()
        self._eager(verify_sweeps)
        self.synchronize()
        ref = self.s.get_state()
        self.s.set_state(*snap, n0)
        dist.barrier(group=self.group)
        err = None
        # the ranks leave the barrier together, so the check's launches start within
        # milliseconds of each other: a short wait bound makes a failed check cost well under
        # a second instead of the run's 10 s bound (which absorbs host-side skew later on)
        self.s.set_wait_timeout(VERIFY_WAIT_MS)
        try:
            self.s.run(verify_sweeps)
            got = self.s.get_state()
            same = all(np.array_equal(a.view(np.uint64), b.view(np.uint64)) for a, b in zip(ref, got))
        except Exception as e:  # noqa: BLE001
            same, err = False, e
        finally:
            try:  # never mask the verification's outcome with an exception from the restore
                self.s.set_wait_timeout(run_wait_ms())
            except Exception as e:  # noqa: BLE001
                err = err or e
        ok = self._all_ok(same)
        self.s.set_state(*snap, n0)  # (the chosen path, or the next, carries on from the same state)
        dist.barrier(group=self.group)
        return ok, err

    def _exchange_and_hyper(self) -> None:
        with self.torch.cuda.stream(self.cur):
            exchange(self.local, self.gathered, self.group)
        self.s.hyper(self.gathered.data_ptr())

    def _eager(self, n: int) -> None:
        for _ in range(n):
            self.s.sweep()
            self._exchange_and_hyper()

    def step(self, n: int = 1) -> None:
        torch = self.torch
        if self.exchange == "p2p":  # one persistent launch per rank; every rank calls with the same n
            err = None
            try:
                self.s.run(n)
            except _lib.ClvError as e:  # a wait timed out: this rank's state is unchanged
                err = e
            if self._all_ok(err is None):
                return
            # some rank's launch failed: every rank returns to the state before this step (ranks
            # whose launch completed undo it) and the step is redone through the all-gather path
            if err is None:
                self.s.rollback()
            self.exchange = "rccl"
            self.p2p_note = (f"peer exchange failed at sweep {self.s.sweeps_done + 1} "
                             f"({err or 'on another rank'}); continued on the all-gather path")
            self.graph = None
        left = n
        if self.graph_chunk and not self.timing:
            if self.graph is None:  # every chunk size at the first such step (a warm-up step):
                self.graph = {k: self._capture(k) for k in graph_sizes_all(self.graph_chunk)}
            for k in graph_sizes(left, self.graph_chunk):
                with torch.cuda.stream(self.stream):
                    self.graph[k].replay()
                self.s.note_sweeps(k)
                left -= k
        self._eager(left)

    def _capture(self, k: int):
        """k sweeps (sweep + group kernels, the all-gather, the level-2 kernel) captured into one
        torch.cuda graph; the sweep index lives in device memory, so a graph serves any step."""
        torch = self.torch
        self.synchronize()
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(device=self.stream.device)
        with torch.cuda.graph(g, stream=cap):
            self.s.set_stream(cap.cuda_stream)
            self.cur = cap
            try:
                self._eager(k)
            finally:
                self.cur = self.stream
        self.s.set_stream(self.base_stream)
        self.s.note_sweeps(-k)  # capture recorded the launches, it ran nothing
        torch.cuda.synchronize()
        return g

    def launch_info(self) -> dict:
        """clv_launch_info, with ``persistent`` = this rank runs whole steps in one launch (p2p with
        a resident grid; else p2p runs one fused sweep launch per sweep)."""
        info = self.s.launch_info()
        info["persistent"] = self.exchange == "p2p" and self.s.p2p_info()["persistent"]
        return info

    def clock_ghz(self) -> float:
        """This rank's average shader clock over its last clv_run as the persistent kernel records it
        (p2p exchange with a resident grid); 0.0 where nothing was recorded: the fused exchange's
        launch-per-sweep kernel and the RCCL path (clv_sweep / clv_hyper) keep no record — see
        clock_probe."""
        return self.s.clock_ghz() if self.exchange == "p2p" else 0.0

    def clock_probe(self, us: float = 50.0) -> float:
        """This rank's shader clock read by a probe kernel behind its launches (clv_clock_probe)."""
        return self.s.clock_probe(us)

    def set_timing(self, enable: bool) -> None:
        self.timing = bool(enable)
        self.s.set_timing(enable)

    def kernel_time(self):
        return self.s.kernel_time()

    def synchronize(self) -> None:
        self.s.synchronize()
        self.torch.cuda.synchronize()

    def close(self) -> None:
        self.graph = None
        self.s.close()
