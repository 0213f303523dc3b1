#!/usr/bin/env python
"""bench.py — MCMC customer-sweeps/s of the HIP sampler on MI355X (BASELINE.json metric).

One step = one sweep (z, tau, level-2 draw, 20 MH steps, storage) of every chain over every
customer.  N=1 workload = BASELINE.json configs[1] ("c2"): bivariate M2 on the full CDNOW CBS
(23,570 customers, covariate first_sales_scaled), 4 chains, burnin 10000 / mcmc 10000 / thin 10,
seed 42, 20 MH steps.  --gpus N > 1 (launched by torch.distributed.run, one rank per GPU) is
weak scaling: every rank holds one 23,570-customer CDNOW copy of a N x 23,570-customer problem
and the ranks exchange the level-2 sufficient statistics once per sweep: by default (--exchange
auto) the persistent kernel of each rank stores its unit partials into every rank's IPC-mapped
mail over xGMI (after a bitwise check against the RCCL path), else one RCCL all_gather per sweep.

Prints ONE JSON line (rank 0).  value = chains * customers * steps / wall time of the timed
region (world size 1: one persistent-kernel launch when the grid fits at once, else hipGraph
replay of the fused sweep launches; max over ranks).  roofline: the dominant kernel's algorithmic
bytes per launch / its launch duration, measured with HIP start/stop events — for the persistent
kernel on the timed region's own launch; for launch-per-sweep paths on the launches of a second
pass over further sweeps of the same run (per-launch events force host-issued launches, so that
pass gives kernel durations, not `value`); traffic from the committed rocprofv3 PMC summary.  cpu_baseline: the bitwise-pinned numpy restatement of
the reference (oracle/ref_cpu.py) on 1 core.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

WORKLOADS = {
    # name: (D, data, covariates, chains, burnin, mcmc, thin, draw_sink)   (SURVEY.md §8 notation)
    "c1": (2, "abe", [], 4, 10000, 4000, 1, "full"),                      # run_mcmc_abe.py:61-71
    "c2": (2, "full", ["first_sales_scaled"], 4, 10000, 10000, 10, "full"),  # BASELINE configs[1]
    "c3": (3, "full", ["gender_F", "age_scaled"], 4, 10000, 10000, 10, "full"),
    # synthetic: 1M customers K=5 bivariate; 1.25M customers per GPU K=9 trivariate
    "c4": (2, "synthetic:1000000:5:20250718", ["c1", "c2", "c3", "c4"], 1, 5000, 5000, 1, "summary"),
    "c5": (3, "synthetic:1250000:9:20250719", [f"c{k}" for k in range(1, 9)], 1, 5000, 5000, 1, "summary"),
}


def algorithmic_bytes(D: int, K: int, stored_frac: float, draw_sink: str) -> float:
    """HBM bytes one (chain, customer) moves per sweep in the sweep kernel:
    read x (4) + t_x, T (16) + K-1 covariates (8 each) + log_s (D=3: 8) + lambda, mu (16);
    write lambda, mu (16); per stored sweep (share `stored_frac`): the level-1 draw 8(D+2)
    (full sink) or the read-modify-write of 9 (D=2) / 11 (D=3) running sums (summary sinks; plus
    the float32 (lambda, mu) pair, 8, for "summary+pct")."""
    rd = 4 + 16 + 8 * (K - 1) + (8 if D == 3 else 0) + 16
    wr = 16
    if draw_sink == "full":
        per_store = 8.0 * (D + 2)
    elif draw_sink in ("summary", "summary+pct"):
        per_store = 16.0 * (9 if D == 2 else 11) + (8.0 if draw_sink == "summary+pct" else 0.0)
    else:
        per_store = 0.0
    return rd + wr + per_store * stored_frac


def _kernel_matches(name: str, kname: str, D: int, K: int) -> bool:
    """A profiled kernel is the workload's instance: its name and template arguments <D, K, ...>."""
    return kname in name and f"<{D}, {K}," in name


def committed_traffic(workload: str, sharded: bool, kname: str = "sweep_kernel", D: int = 0, K: int = 0):
    """HBM bytes per sweep-kernel launch from the committed rocprofv3 PMC summary of this workload
    (profiles/*_summary.json written by tools/summarize_profile.py): FETCH_SIZE and WRITE_SIZE
    corrected by the calibration kernels of tools/calib_fetch.hip; None if absent."""
    import glob
    if sharded:
        return None
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{workload}_*summary.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        for name, k in d.get("kernels", {}).items():
            if _kernel_matches(name, kname, D, K) and "traffic_bytes" in k:
                best = dict(bytes_per_sweep=k["traffic_bytes"] / k.get("sweeps_per_dispatch", 1),
                            source=os.path.basename(path),
                            counters="FETCH_SIZE x %.2f + WRITE_SIZE x %.2f (calibrated, tools/calib_fetch.hip)"
                                     % (k["traffic_correction"]["read"], k["traffic_correction"]["write"]))
    return best


N_SIMDS = 1024  # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
N_XCDS = 8      # GRBM_GUI_ACTIVE is summed over the 8 XCDs


def committed_counters(workload: str, sharded: bool, kname: str = "sweep_kernel", D: int = 0, K: int = 0):
    """Counter evidence for the roofline's `bound` from the committed rocprofv3 summary of this
    workload (tools/summarize_profile.py): VALU busy = SQ_ACTIVE_INST_VALU (quad-cycles, x4) summed
    over the kernel's waves / (1,024 SIMDs x the dispatch's cycles, GRBM_GUI_ACTIVE / 8 XCDs) — the
    share of SIMD cycles issuing VALU work — and the VALU-active share of the waves' lifetime."""
    import glob
    if sharded:
        return None
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{workload}_*summary.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        for name, k in d.get("kernels", {}).items():
            if _kernel_matches(name, kname, D, K) and "valu_active_quadcycles_per_wave" in k and k.get("grbm_gui_active"):
                cycles = k["grbm_gui_active"] / N_XCDS
                busy = 4.0 * k["valu_active_quadcycles_per_wave"] * k["waves"] / (N_SIMDS * cycles)
                best = dict(valu_busy_frac=round(busy, 4),
                            valu_active_frac_of_wave_lifetime=round(k["valu_active_frac_of_wave_lifetime"], 4),
                            valu_insts_per_wave=round(k["valu_insts_per_wave"], 1), waves=k["waves"],
                            source=os.path.basename(path))
    return best


def load_workload(name: str, world: int = 1):
    """CBS of a workload.  CDNOW: the committed CBS columns (weak scaling: one copy per rank).
    Synthetic: mcmc_clv_model_amd.data.synthetic_cbs with n per GPU (c5 weak scaling: n x world)."""
    import numpy as np
    import pandas as pd
    from mcmc_clv_model_amd.data import add_driver_columns, synthetic_cbs
    D, data, covs, chains, burnin, mcmc, thin, sink = WORKLOADS[name]
    if data.startswith("synthetic:"):
        _, n, K, seed = data.split(":")
        n = int(n) * (world if name == "c5" else 1)
        df = synthetic_cbs(n, int(K), D, seed=int(seed))
    else:
        d = np.load(os.path.join(ROOT, "tests", "golden", f"cdnow_{data}_cbs.npz"), allow_pickle=False)
        df = add_driver_columns(pd.DataFrame({k: d[k] for k in d.files}))
        if world > 1:
            df = pd.concat([df] * world, ignore_index=True)
    return df, D, covs, chains, burnin, mcmc, thin, sink


def stored_fraction(burnin: int, thin: int, first: int, last: int) -> float:
    """Share of sweeps first..last (1-based, inclusive) that store a draw (bi:402)."""
    n = sum(1 for s in range(first, last + 1) if s > burnin and (s - 1 - burnin) % thin == 0)
    return n / max(1, last - first + 1)


def cpu_baseline_child(workload: str, warm: int, timed: int) -> None:
    """Runs in a fresh process with OMP/OPENBLAS threads = 1: the oracle (numpy port of the
    reference, bitwise equal to it) sweeping 1 chain of the workload."""
    import numpy as np
    from oracle import ref_cpu as orc
    df, D, covs, chains, burnin, mcmc, thin, sink = load_workload(workload)
    cbs, X = orc.design_matrix(df, covs)
    K = X.shape[1]
    hyper = orc.default_hyper(K, D)
    stamps = {}

    def on_sweep(step):
        if step in (warm, warm + timed):
            stamps[step] = time.perf_counter()

    stream = orc.Stream(np.random.default_rng(42))
    x, t_x, T = cbs["x"].to_numpy(), cbs["t_x"].to_numpy(), cbs["T_cal"].to_numpy()
    if D == 2:
        orc.run_chain_bi(1, x, t_x, T, X, hyper, mcmc, burnin, thin, stream, 0, 20, n_sweeps=warm + timed,
                         on_sweep=on_sweep)
    else:
        orc.run_chain_tri(1, x, t_x, T, cbs["log_s"].to_numpy(), X, hyper, mcmc, burnin, thin, stream, 0, 20,
                          n_sweeps=warm + timed, omega2=cbs["log_s"].var(), log_s_mean=cbs["log_s"].mean(),
                          on_sweep=on_sweep)
    dt = stamps[warm + timed] - stamps[warm]
    print(json.dumps(dict(s_per_sweep=dt / timed, value=len(df) * timed / dt)))


def cpu_baseline(workload: str, warm: int = 20, timed: int = 200, parallel: bool = True):
    if WORKLOADS[workload][1].startswith("synthetic:"):  # ~3 s/sweep on one core
        warm, timed = 2, 5
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1",
               HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--workload", workload,
                          "--cpu-warm", str(warm), "--cpu-timed", str(timed)],
                         capture_output=True, text=True, env=env, check=True, timeout=900)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    n = len(load_workload(workload)[0])
    res = dict(value=r["value"], unit="customer-sweeps/s", cores=1, kind="port",
               s_per_sweep=r["s_per_sweep"],
               sample=f"oracle/ref_cpu.py (numpy restatement, bitwise equal to the reference) on {workload}: "
                      f"1 chain x {n} customers, {timed} timed sweeps after {warm} warm-up sweeps, 1 thread")
    if not parallel:
        return res
    # also an all-cores throughput — P independent single-threaded chains in P
    # processes at once (the reference runs its chains sequentially; this is its best case)
    procs = min(16, os.cpu_count() or 1)  # the GPU box's CPU share is 16 (gpurun)
    t_warm, t_timed = max(2, warm // 4), max(5, timed // 4)
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--workload", workload,
                            "--cpu-warm", str(t_warm), "--cpu-timed", str(t_timed)],
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, env=env) for _ in range(procs)]
    vals = []
    for p in ps:
        o, _ = p.communicate(timeout=900)
        if p.returncode == 0:
            vals.append(json.loads(o.strip().splitlines()[-1])["value"])
    if len(vals) == procs:
        res["all_cores"] = dict(value=sum(vals), cores=procs,
                                sample=f"{procs} processes x 1 chain, {t_timed} timed sweeps each after {t_warm}, "
                                       "1 thread each, run concurrently")
    return res


def settle_clocks(ms: float, device: int) -> float:
    """Hold the GPU busy for `ms` of wall time with fp64 matmuls (work unrelated to the sampler,
    outside every timed region), so that a short timed window runs at the clocks a whole run sees:
    the driver's 20-sweep window after 5 one-sweep warm-up calls otherwise starts from the idle
    power state and pays ~0.85 us per sweep of clock ramp (tools/driver_breakdown.py, cases cold /
    after_busy / after_long / long_then_idle: profiles/r04_clock_ramp.jsonl).  Returns the seconds
    spent."""
    import torch
    if ms <= 0:
        return 0.0
    a = torch.randn(2048, 2048, dtype=torch.float64, device=f"cuda:{device}")
    b = a
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < ms / 1e3:
        b = torch.tanh(a @ b * 1e-3)
        torch.cuda.synchronize()
    del a, b
    return time.perf_counter() - t0


def measure_config(name: str, world: int, rank: int, local_rank: int, dist, steps: int, warmup: int,
                   graph_chunk: int, exchange: str, stored_phase: bool = True, settle_ms: float = 0.0) -> dict:
    """One BASELINE multi-GPU configuration at this world size: c4 = 1M bivariate
    customers K=5 sharded over the ranks (strong scaling: the same problem at every N), c5 = 1.25M
    trivariate customers K=9 per rank (weak scaling).  Wall time of `steps` sweeps (max over ranks)
    after `warmup` sweeps; HBM fraction of the algorithmic bytes against N x 8 TB/s.  With
    `stored_phase` (and a burn-in longer than the window) the same chains then continue past the
    burn-in and `steps` stored sweeps are timed too (`stored`: each also read-modify-writes the
    customer's running sums), and `whole_run` combines both phases' per-sweep times over the
    BASELINE run's burn-in + mcmc sweeps."""
    import torch
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    df, D, covs, chains, burnin, mcmc, thin, sink = load_workload(name, world)
    n_total = len(df)
    p = build_problem(df, covs, D)
    del df
    mcmc0 = mcmc
    mcmc = max(mcmc, warmup + steps - burnin, 100 + steps)
    if world == 1:
        kern = HipSampler(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=42, draw_sink=sink,
                          device=local_rank)
        run, sync = kern.run, kern.synchronize
    else:
        from mcmc_clv_model_amd.distributed import ShardedSampler
        kern = ShardedSampler(p, rank=rank, world=world, chains=chains, mcmc=mcmc, burnin=burnin, thin=thin, seed=42,
                              draw_sink=sink, device=local_rank, graph_chunk=graph_chunk, exchange=exchange,
                              verify_sweeps=8)
        run, sync = kern.step, kern.synchronize
    del p

    def timed(n: int) -> float:
        """Wall time of n sweeps bracketed by barrier + synchronize, max over ranks."""
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(n)
        sync()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        dt = time.perf_counter() - t0
        if dist:
            t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local_rank}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    settle_clocks(settle_ms, local_rank)  # (the problem build above left the GPU idle for seconds)
    run(warmup)
    sync()
    dt = timed(steps)  # burn-in sweeps warmup+1 .. warmup+steps
    # the stored phase (verdict r3: half of the BASELINE run; every sweep after burn-in
    # read-modify-writes the customer's running sums, bi:402-428): continue the same chains into
    # it, 100 sweeps past the boundary (warm), then time `steps` stored sweeps
    phases = None
    K = len(covs) + 1
    kname = "sweep_kernel"  # (c4 / c5: launch-per-sweep; the committed profiles are of that kernel)

    def traffic(tag):  # calibrated PMC bytes per (chain, customer) sweep from the committed profile
        tr = committed_traffic(tag, False, kname, D, K) if world == 1 else None
        return None if not tr else dict(bytes_per_unit=round(tr["bytes_per_sweep"] / (chains * n_total), 2),
                                        source=tr["source"])
    if stored_phase and burnin > warmup + steps:
        done = warmup + steps
        run(burnin + 100 - done)
        sync()
        dt_st = timed(steps)
        first = burnin + 101
        bpu_st = algorithmic_bytes(D, len(covs) + 1, stored_fraction(burnin, thin, first, first + steps - 1), sink)
        v_st = chains * n_total * steps / dt_st
        t_b, t_s = dt / steps, dt_st / steps  # s per sweep in each phase
        whole = chains * n_total * (burnin + mcmc0) / (burnin * t_b + mcmc0 * t_s)
        phases = dict(
            stored=dict(value=v_st, ms_per_step=t_s * 1e3, sweeps=f"{first}..{first + steps - 1}",
                        bytes_per_unit=round(bpu_st, 2),
                        hbm_frac=round(bpu_st * v_st / 1e9 / (world * HBM_PEAK_GBS), 5),
                        measured_traffic=traffic(f"{name}stored")),
            whole_run=dict(value=whole, sweeps=f"{burnin} burn-in + {mcmc0} stored",
                           note="customer-sweeps/s of the BASELINE run from the two phases' per-sweep times"))
    linfo = kern.launch_info()
    persistent = linfo["persistent"]
    exch = getattr(kern, "exchange", None)
    note = getattr(kern, "p2p_note", None)
    kern.close()
    value = chains * n_total * steps / dt
    bpu = algorithmic_bytes(D, K, stored_fraction(burnin, thin, warmup + 1, warmup + steps), sink)
    data = WORKLOADS[name][1]
    return dict(workload=f"{name}: {'bivariate' if D == 2 else 'trivariate'}, K={K}, " +
                         ("synthetic (mcmc_clv_model_amd.data.synthetic_cbs)" if data.startswith("synthetic:") else
                          f"CDNOW {data} CBS"),
                scaling="strong" if name == "c4" else "weak", value=value, unit="customer-sweeps/s",
                n_customers=n_total, customers_per_gpu=n_total // world, chains=chains, steps=steps, warmup=warmup,
                ms_per_step=dt / steps * 1e3, draw_sink=sink,
                hbm_frac=round(bpu * value / 1e9 / (world * HBM_PEAK_GBS), 5), bytes_per_unit=round(bpu, 2),
                path=("persistent kernel" if persistent else "launch-per-sweep sweep kernel") +
                     ("" if world == 1 else
                      (", unit partials stored into every rank's mail over xGMI by the kernel (no host collective)"
                       if exch == "p2p" else ", RCCL all-gather + level-2 kernel per sweep") +
                      (f" ({note})" if note else "")),
                phase=f"burn-in (sweeps {warmup + 1}..{warmup + steps})", measured_traffic=traffic(name),
                **(phases or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=19000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true", help="skip the event-timed roofline pass")
    ap.add_argument("--timing-steps", type=int, default=3000, help="sweeps in the event-timed roofline pass")
    ap.add_argument("--graph-chunk", type=int, default=32,
                    help="sharded path: sweeps (incl. the RCCL all-gather) per captured torch.cuda graph; 0 = eager")
    ap.add_argument("--force-sharded", action="store_true",
                    help="use the sharded path (torch.distributed exchange) even at world size 1")
    ap.add_argument("--exchange", default="auto", choices=["auto", "p2p", "rccl"],
                    help="world size > 1: unit-partial exchange per sweep — p2p = persistent kernel storing into "
                         "every rank's IPC-mapped mail over xGMI (auto: where it fits and verifies bitwise "
                         "against RCCL), rccl = all_gather per sweep")
    ap.add_argument("--scaling-configs", default="c4,c5",
                    help="BASELINE multi-GPU configurations also measured at this N (c4 strong, c5 weak "
                         "scaling), reported under `configs`; '' to skip")
    ap.add_argument("--scaling-steps", type=int, default=1000)
    ap.add_argument("--blocks-per-unit", type=int, default=0,
                    help="(world size 1, A/B) blocks per statistics unit instead of the plan's (0)")
    ap.add_argument("--phase", default="burnin", choices=["burnin", "stored"],
                    help="(profiling) stored: the sampler's burn-in is 0, so every timed sweep is a stored sweep "
                         "(the running sums' read-modify-write / the draws' stores of bi:402-428)")
    ap.add_argument("--no-c1-leg", dest="c1_leg", action="store_false",
                    help="skip BASELINE configs[0] (c1 on the GPU and its 1-core CPU leg)")
    ap.add_argument("--one-gpu-rehearsal", action="store_true",
                    help="world size > 1 on a one-GPU box: every rank on device 0, gloo process group (the "
                         "exchange paths are exercised; the numbers are not a scaling measurement)")
    ap.add_argument("--clock-settle-ms", type=float, default=100.0,
                    help="GPU busy time (fp64 matmuls, unrelated work) just before the warm-up, so the timed "
                         "window starts at the clocks of a running job, not the idle power state; 0 = off")
    ap.add_argument("--cpu-baseline-child", action="store_true")
    ap.add_argument("--cpu-warm", type=int, default=20)
    ap.add_argument("--cpu-timed", type=int, default=200)
    a = ap.parse_args()
    if a.cpu_baseline_child:
        cpu_baseline_child(a.workload, a.cpu_warm, a.cpu_timed)
        return

    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.one_gpu_rehearsal:
        local_rank = 0
        a.graph_chunk = 0  # (a gloo exchange cannot be captured in a graph)
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    dist = None
    sharded = world > 1 or a.force_sharded
    if sharded:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if a.one_gpu_rehearsal:  # RCCL refuses two ranks on one GPU
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))

    from mcmc_clv_model_amd import _lib
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem

    df, D, covs, chains, burnin, mcmc, thin, sink = load_workload(a.workload, world)
    if a.phase == "stored":
        mcmc, burnin = mcmc + burnin, 0
    total = a.warmup + a.steps + (0 if a.no_kernel_timing else min(a.steps, a.timing_steps))
    mcmc_workload = mcmc
    mcmc = max(mcmc, total - burnin)  # draw buffers also cover the sweeps of the roofline pass
    n_total = len(df)
    if not sharded:
        p = build_problem(df, covs, D)
        s = HipSampler(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=42, draw_sink=sink,
                       device=local_rank, blocks_per_unit=a.blocks_per_unit)
        run = s.run
        sync = s.synchronize
        kern = s
    else:
        from mcmc_clv_model_amd.distributed import ShardedSampler
        p = build_problem(df, covs, D)
        ss = ShardedSampler(p, rank=rank, world=world, chains=chains, mcmc=mcmc, burnin=burnin, thin=thin, seed=42,
                            draw_sink=sink, device=local_rank, graph_chunk=a.graph_chunk,
                            exchange=a.exchange if world > 1 else "rccl", verify_sweeps=8)
        run = ss.step
        sync = ss.synchronize
        kern = ss

    K = len(covs) + 1
    timing = not a.no_kernel_timing
    info = kern.launch_info()
    persistent = info["persistent"]
    one_launch = persistent   # all sweeps of a clv_run in one launch
    p2p = sharded and persistent
    # persistent kernel: the timed launch itself is bracketed by HIP start/stop events recorded on
    # the sampler's stream (the launch's stream), inside the timed region; the warm-up sweeps run
    # through that same path (events included, their times discarded), so the timed call is not
    # the first of its kind in the process
    live = timing and one_launch
    settle_s = settle_clocks(a.clock_settle_ms, local_rank)
    if live:
        kern.set_timing(True)
    if one_launch:  # the warm-up steps one call each: the host path of a call is warm when timed
        for _ in range(a.warmup):
            run(1)
            sync()
            torch.cuda.synchronize()
    else:
        run(a.warmup)
    sync()
    if live:
        kern.kernel_time()
        kern.set_timing(True)  # (counters reset: only the timed launch is harvested below)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.steps)                      # timed region: persistent launch / hipGraph replay / sharded steps
    if sharded:
        sync()                        # (HipSampler.run returns when its launches are done)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    host_us = kern.host_times() if (persistent and not sharded) else None  # where the step's host time went
    kt_live = None
    if live:
        kt_live = kern.kernel_time()
        kern.set_timing(False)
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    units = chains * n_total * a.steps
    value = units / dt

    # Launch-per-sweep paths: a roofline pass continues the same sweeps with HIP start/stop events
    # on every sweep launch (hipExtLaunchKernelGGL: the dispatch's own timestamps).  Launches are
    # then host-issued, which leaves gaps between kernels, so that pass yields kernel durations,
    # not `value`.  The persistent kernel's durations come from the timed launch itself.
    roofline = None
    n_local = kern.n
    if live:
        n_t = a.steps
        frac = stored_fraction(burnin, thin, a.warmup + 1, a.warmup + a.steps)
    else:
        n_t = min(a.steps, a.timing_steps)
        frac = stored_fraction(burnin, thin, a.warmup + a.steps + 1, a.warmup + a.steps + n_t)
    bpu = algorithmic_bytes(D, K, frac, sink)
    if timing:
        if live:
            kt = kt_live
        else:
            kern.set_timing(True)
            run(n_t)
            sync()
            kt = kern.kernel_time()
            kern.set_timing(False)
        if kt["sweep_launches"]:
            # kt["sweep_launches"] counts sweeps; the persistent kernel runs all n_t in ONE launch
            t_sweep = kt["sweep_ms"] / kt["sweep_launches"] * 1e-3
            spl = n_t if one_launch else 1               # sweeps per launch
            t_launch = t_sweep * spl
            units = chains * n_local * spl               # (chain, customer) sweeps per launch
            achieved = bpu * units / t_launch / 1e9
            kname = "persist_kernel" if persistent else "sweep_kernel"
            roofline = dict(bound=None, achieved=round(achieved, 3), peak=HBM_PEAK_GBS, unit="GB/s",
                            frac=round(achieved / HBM_PEAK_GBS, 6), traffic=None,
                            kernel=("persist_kernel (one launch for all sweeps of a clv_run; level-2 workgroup "
                                    "per chain" + ("; unit partials exchanged over xGMI" if p2p else "") + ")")
                            if persistent else
                            ("sweep_kernel (incl. fused level-2 tail)" if not sharded else "sweep_kernel"),
                            bytes_per_unit=round(bpu, 3), units_per_launch=units, sweeps_per_launch=spl,
                            launch_us=round(t_launch * 1e6, 3), sweep_kernel_us=round(t_sweep * 1e6, 3),
                            timed_launches=kt["sweep_launches"] // spl,
                            events=("the timed region's launch" if live else
                                    f"a roofline pass of {n_t} further sweeps, one event pair per launch"))
            tr = committed_traffic(a.workload, sharded and not p2p, kname, D, K)
            if tr:  # HBM bytes per launch (calibrated PMC), per sweep x sweeps per launch
                roofline["traffic"] = round(tr["bytes_per_sweep"] * spl)
                roofline["traffic_source"] = f"{tr['source']}: {tr['counters']}"
            if kt["hyper_launches"]:
                roofline["hyper_kernel_us"] = round(kt["hyper_ms"] / kt["hyper_launches"] * 1e3, 3)
            # bound: from the counters (HBM traffic rate vs peak, VALU busy share), not assumed
            ev = committed_counters(a.workload, sharded and not p2p, kname, D, K) or {}
            if roofline["traffic"] is not None:
                ev["hbm_traffic_frac"] = round(roofline["traffic"] / t_launch / 1e9 / HBM_PEAK_GBS, 4)
            if ev.get("hbm_traffic_frac", 0.0) >= 0.6:
                roofline["bound"] = "hbm"
            elif ev.get("valu_busy_frac", 0.0) >= 0.7:
                roofline["bound"] = "valu"
            elif "valu_busy_frac" in ev:
                roofline["bound"] = "latency"
            else:
                roofline["bound"] = "unmeasured"
            ev["rule"] = "hbm if measured HBM traffic >= 0.6 of peak; else valu if VALU busy >= 0.7; else latency"
            roofline["bound_evidence"] = ev

    kern.close()
    extra = {}
    for name in [c for c in a.scaling_configs.split(",") if c]:
        # warm-up of 200 sweeps (the launch-per-sweep path captures its 64-sweep hipGraph on first use;
        # clocks ramp), then 1,000 timed sweeps: c4 ~0.09 s, c5 ~0.13 s per GPU
        extra[name] = measure_config(name, world, rank, local_rank, dist, a.scaling_steps, 200, a.graph_chunk,
                                     a.exchange if world > 1 else "rccl", settle_ms=a.clock_settle_ms)

    if world == 1 and not a.force_sharded and a.c1_leg:
        # BASELINE configs[0] ("Bivariate M1, Abe 1/10 CDNOW subset, 4000 iters on CPU numpy reference
        # path"): the same 4-chain c1 sampler on the GPU (2,000 sweeps after 80), next to its 1-core
        # CPU leg in cpu_baseline["c1"]
        extra["c1"] = measure_config("c1", 1, rank, local_rank, None, 2000, 80, 0, "rccl", stored_phase=False,
                                     settle_ms=a.clock_settle_ms)

    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline and not a.force_sharded:
            cpu = cpu_baseline(a.workload)
            if a.c1_leg and a.workload != "c1":
                c1 = cpu_baseline("c1", parallel=False)
                cpu["c1"] = dict(value=c1["value"], unit=c1["unit"], cores=1, kind=c1["kind"],
                                 s_per_sweep=c1["s_per_sweep"], sample=c1["sample"],
                                 gpu_value=extra["c1"]["value"] if "c1" in extra else None,
                                 gpu_speedup=(extra["c1"]["value"] / c1["value"]) if "c1" in extra else None)
        wl = WORKLOADS[a.workload]
        line = dict(
            metric="MCMC sweeps/sec x N_customers (customer-sweeps/s)", value=value, unit="customer-sweeps/s",
            n_gpus=world, steps=a.steps, warmup=a.warmup, ms_per_step=dt / a.steps * 1e3, higher_is_better=True,
            scaling="weak", vs_baseline=None, dtype="f64",
            proposal_dtype="f32",  # t3 proposal noise and accept log-uniforms; state, posterior f64
            data=(f"synthetic CBS ({n_total} customers, mcmc_clv_model_amd.data.synthetic_cbs)"
                  if WORKLOADS[a.workload][1].startswith("synthetic:") else
                  (f"CDNOW {WORKLOADS[a.workload][1]} CBS ({n_total // world:,} real customers, "
                   f"tests/golden/cdnow_{WORKLOADS[a.workload][1]}_cbs.npz)")
                  + ("" if world == 1 else f", tiled x{world} (one copy per rank)")),
            config=dict(workload=f"{a.workload}: {'bivariate' if D == 2 else 'trivariate'} M2, covariates {covs}",
                        n_customers=n_total, chains=chains, n_mh_steps=20, burnin=burnin, mcmc=mcmc_workload,
                        thin=thin, seed=42, draw_sink=sink, parallelism=f"customer-shard x{world}",
                        **({"phase": "stored (profiling: burn-in 0, every sweep stores)"} if a.phase == "stored" else {}),
                        timed_region=(f"one persistent-kernel launch of {a.steps} sweeps" if persistent else
                                      "hipGraph replay of fused sweep launches") if not sharded else
                        (f"one persistent-kernel launch of {a.steps} sweeps per rank, unit partials stored into "
                         "every rank's IPC-mapped mail over xGMI (no host collective per sweep)") if p2p else
                        f"torch.cuda graph replay ({a.graph_chunk} sweeps: sweep + group kernels, RCCL all_gather, "
                        "level-2 kernel)" if a.graph_chunk else "eager: sweep + group kernels, RCCL all_gather, level-2"),
            clock_settle_ms=round(settle_s * 1e3, 1),  # GPU busy with unrelated work before the warm-up
            roofline=roofline, cpu_baseline=cpu,
            host_us=(dict(host_us, clv_run_total=round(sum(host_us.values()), 3), timed_region=round(dt * 1e6, 3))
                     if host_us else None),
            exchange=(None if world == 1 and not sharded else
                      dict(kind=kern.exchange, note=kern.p2p_note, requested=a.exchange if world > 1 else "rccl")),
            speedup_vs_cpu_1core=(value / cpu["value"]) if cpu else None,
            configs=extra or None,
        )
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
