#!/usr/bin/env python
"""bench.py — MCMC customer-sweeps/s of the HIP sampler on MI355X (BASELINE.json metric).

One step = one sweep (z, tau, level-2 draw, 20 MH steps, storage) of every chain over every
customer.  The primary workload is a BASELINE configuration at every N:
  N = 1   configs[1] "c2": bivariate M2 on the full CDNOW CBS (23,570 customers, covariate
          first_sales_scaled), 4 chains, burnin 10000 / mcmc 10000 / thin 10, seed 42, 20 MH steps;
  N > 1   configs[4] "c5": trivariate M2, synthetic, 1.25M customers per GPU with 8 covariates
          (weak scaling: 10M customers at N = 8), one process per GPU (torch.distributed.run),
          sharded over the ranks with one exchange of the level-2 statistics per sweep (the fused
          peer exchange over xGMI, verified bitwise against the RCCL all-gather path, else RCCL).
The other BASELINE configurations run as `configs` legs (N = 1: c3, c4, c5 and c1; N > 1: c4
strong scaling, and c2 tiled once per rank, labelled non-BASELINE), each with its own roofline
(and bound evidence), c2 / c3 / c4 / c5 with a stored-sweep sub-line, c2 / c3 with the drop-in's
whole BASELINE run timed end to end through mcmc_draw_parameters (run_mcmc_abe.py:60-77).

Prints ONE JSON line (rank 0).  value = chains * customers * steps / wall time of the timed region
(max over ranks).  roofline: the dominant kernel's algorithmic bytes (SURVEY §8d per (chain,
customer) sweep) per launch / its launch duration measured with HIP events on the sampler's stream
— for the persistent kernel on the timed region's own launch; for launch-per-sweep paths on a pass
over further sweeps (per-launch events), with measured traffic and the counters of the committed
rocprofv3 summaries (profiles/).  cpu_baseline: the bitwise-pinned numpy restatement of the
reference (oracle/ref_cpu.py) on 1 core (c2, and c1 / c3 under configs).
"""
from __future__ import annotations

import argparse
import contextlib
import io
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
    "c3": (3, "full", ["gender_F", "age_scaled"], 4, 10000, 10000, 10, "full"),  # configs[2]
    # synthetic: 1M customers K=5 bivariate; 1.25M customers per GPU K=9 trivariate
    "c4": (2, "synthetic:1000000:5:20250718", ["c1", "c2", "c3", "c4"], 1, 5000, 5000, 1, "summary"),
    "c5": (3, "synthetic:1250000:9:20250719", [f"c{k}" for k in range(1, 9)], 1, 5000, 5000, 1, "summary"),
    # NOT a BASELINE configuration: the instance one GPU runs in c4's 8-rank run — rank 0's shard of
    # distributed.plan(1M, 8), 496 blocks = 126,976 customers of the c4 set (verdict r5 #4), at world size 1
    "c4_shard8": (2, "synthetic:1000000:5:20250718:shard0of8", ["c1", "c2", "c3", "c4"], 1, 5000, 5000, 1, "summary"),
}
BASELINE_INDEX = {"c1": 0, "c2": 1, "c3": 2, "c4": 3, "c5": 4}


def primary_workload(world: int) -> str:
    """The BASELINE configuration the line's `value` is quoted on: c2 on one GPU (configs[1]); the
    8-GPU weak-scaling run c5 (configs[4], 1.25M customers per GPU) at N > 1 (verdict r4 #7)."""
    return "c2" if world == 1 else "c5"


def config_legs(world: int, primary: str):
    """The `configs` legs: every other BASELINE configuration at this N (c1 and c3 are one-GPU
    configurations; at N > 1 c2 runs tiled once per rank, a non-BASELINE rehearsal of the
    CDNOW-size exchange)."""
    if world == 1:  # (+ c4_shard8: the per-GPU instance of c4's 8-rank run, a single-GPU proxy)
        return [c for c in ("c3", "c4", "c5", "c4_shard8") if c != primary]
    return [c for c in ("c4", "c2") if c != primary]


def survey_bytes(D: int, K: int, stored_frac: float, draw_sink: str) -> float:
    """SURVEY §8d's algorithmic HBM bytes per (chain, customer) sweep: read x 4, t_x 8, T 8,
    8 (K-1) covariates, (D = 3) log_s 8, 8 D of state; write 8 D of state; per stored sweep the
    8 (D+2) B level-1 draw (full sink) or +0 (summary sinks), amortised by `stored_frac`.
    c1 84 (thin 1), c2 60 + 3.2, c3 92 + 4.0, c4 84, c5 140."""
    rd = 4 + 8 + 8 + 8 * (K - 1) + (8 if D == 3 else 0) + 8 * D
    wr = 8 * D
    per_store = 8.0 * (D + 2) if draw_sink == "full" else 0.0
    return rd + wr + per_store * stored_frac


def algorithmic_bytes(D: int, K: int, stored_frac: float, draw_sink: str) -> float:
    """The sweep kernel's own streaming bytes per (chain, customer) sweep: as
    survey_bytes but with the carried state only (lambda, mu: 16 B each way — eta is redrawn from
    its conjugate posterior every sweep, tri:306-333, never read back), and on stored sweeps of the
    summary sinks the read-modify-write of 9 (D=2) / 11 (D=3) running sums (+ the float32
    (lambda, mu) pair for "summary+pct")."""
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


def _summaries(workload: str):
    import glob
    out = []
    workload = workload.replace("_", "")  # profile names carry no "_" inside the workload (profile_name)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{workload}_*summary.json"))):
        try:
            out.append((path, json.load(open(path))))
        except Exception:
            continue
    return out


def committed_traffic(workload: str, kname: str, D: int, K: int):
    """HBM bytes per sweep of the workload's kernel from the latest committed rocprofv3 PMC summary
    (profiles/r*_<workload>_*summary.json, tools/summarize_profile.py): FETCH_SIZE and WRITE_SIZE
    corrected by the calibration of tools/calib_fetch.hip; None if absent."""
    best = None
    for path, d in _summaries(workload):
        for name, k in d.get("kernels", {}).items():
            if _kernel_matches(name, kname, D, K) and "traffic_bytes" in k:
                best = dict(bytes_per_sweep=k["traffic_bytes"] / k.get("sweeps_per_dispatch", 1),
                            source=os.path.basename(path),
                            counters="FETCH_SIZE x %.2f + WRITE_SIZE x %.2f (calibrated, tools/calib_fetch.hip)"
                                     % (k["traffic_correction"]["read"], k["traffic_correction"]["write"]))
    return best


N_SIMDS = 1024  # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
N_XCDS = 8      # GRBM_GUI_ACTIVE is summed over the 8 XCDs


def committed_counters(workload: str, kname: str, D: int, K: int):
    """Counter evidence for the roofline's `bound` from the latest committed rocprofv3 summary of the
    workload: VALU busy = SQ_ACTIVE_INST_VALU (quad-cycles, x4) summed over the kernel's waves /
    (1,024 SIMDs x the dispatch's cycles, GRBM_GUI_ACTIVE / 8 XCDs) — the share of SIMD cycles
    issuing VALU work — and the VALU-active share of the waves' lifetime."""
    best = None
    for path, d in _summaries(workload):
        for name, k in d.get("kernels", {}).items():
            if _kernel_matches(name, kname, D, K) and "valu_active_quadcycles_per_wave" in k and k.get("grbm_gui_active"):
                cycles = k["grbm_gui_active"] / N_XCDS
                busy = 4.0 * k["valu_active_quadcycles_per_wave"] * k["waves"] / (N_SIMDS * cycles)
                best = dict(valu_busy_frac=round(busy, 4),
                            valu_active_frac_of_wave_lifetime=round(k["valu_active_frac_of_wave_lifetime"], 4),
                            valu_insts_per_wave=round(k["valu_insts_per_wave"], 1), waves=k["waves"],
                            source=os.path.basename(path))
                if k["waves"] <= 2 * N_SIMDS:  # a grid resident at once (the persistent kernel): the
                    # SIMDs holding ceil(waves / SIMDs) waves set the period
                    per_simd = -(-int(k["waves"]) // N_SIMDS)
                    best["waves_per_simd_max"] = per_simd
                    best["valu_busy_frac_max_simd"] = round(busy * per_simd * N_SIMDS / k["waves"], 4)
    return best


BOUND_RULE = ("hbm if measured HBM traffic >= 0.6 of peak; else valu if VALU busy >= 0.7 (for a grid resident at "
              "once: on the SIMDs holding the most waves); else latency")


def load_workload(name: str, world: int = 1):
    """CBS of a workload.  CDNOW: the committed CBS columns (N > 1: one copy per rank).
    Synthetic: mcmc_clv_model_amd.data.synthetic_cbs with n per GPU (c5 weak scaling: n x world)."""
    import numpy as np
    import pandas as pd
    from mcmc_clv_model_amd.data import add_driver_columns, synthetic_cbs
    D, data, covs, chains, burnin, mcmc, thin, sink = WORKLOADS[name]
    if data.startswith("synthetic:"):
        _, n, K, seed, *shard = data.split(":")
        n = int(n) * (world if name == "c5" else 1)
        df = synthetic_cbs(n, int(K), D, seed=int(seed))
        if shard:  # "shard<r>of<w>": rank r's customers of distributed.plan(n, w)
            from mcmc_clv_model_amd.distributed import plan
            r, w = (int(v) for v in shard[0][len("shard"):].split("of"))
            b, e = plan(n, w).shard(r)
            df = df.iloc[b:e].reset_index(drop=True)
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
    hyper = orc.default_hyper(X.shape[1], D)
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
    """the oracle on 1 core (c1 / c2 / c3: >= 200 timed sweeps after 20; c4 / c5: 5
    after 2), and with `parallel` an all-cores throughput (P single-threaded chains at once)."""
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


def settle_clocks(ms: float, device: int, scratch=None) -> float:
    """Hold the GPU busy for `ms` of wall time outside every timed region, so that a short timed
    window runs at the clocks a whole run sees: the driver's 20-sweep window after 5 one-sweep
    warm-up calls otherwise starts from the idle power state and pays ~0.85 us per sweep of clock
    ramp (tools/driver_breakdown.py, cases cold / after_busy / after_long / long_then_idle:
    profiles/r04_clock_ramp.jsonl).  `scratch`: a sampler of its own over the same customers
    (scratch_sampler) whose sweeps are the busy work — the clock the governor settles at depends on
    the load, and fp64 matmuls (the fallback without one) left the c2 window at 2.25 GHz against
    the 2.38 of a whole run of sweeps.  The timed sampler's chains are untouched.
    Returns the seconds spent."""
    import torch
    if ms <= 0:
        return 0.0
    t0 = time.perf_counter()
    if scratch is not None:
        n = 16
        while True:
            t1 = time.perf_counter()
            scratch.run(n)
            scratch.synchronize()
            torch.cuda.synchronize()
            now = time.perf_counter()
            if now - t0 >= ms / 1e3:
                break
            n = max(1, min(4 * n, 4096, int(n * 2e-3 / max(now - t1, 1e-6))))  # ~2 ms per call
        return time.perf_counter() - t0
    a = torch.randn(2048, 2048, dtype=torch.float64, device=f"cuda:{device}")
    b = a
    while time.perf_counter() - t0 < ms / 1e3:
        b = torch.tanh(a @ b * 1e-3)
        torch.cuda.synchronize()
    del a, b
    return time.perf_counter() - t0


SETTLE_WORK = "sampler"  # --settle-work (A/B: "matmul" = the fp64 matmuls of rounds 4-5)


def scratch_sampler(p, chains: int, device: int):
    """The clock-settle work of a leg (settle_clocks): a world-size-1 sampler over the same customers
    (at N > 1 the rank's own shard), seed 7, no draws kept — the same kernel family as the timed
    sampler, its own handle, state and stream.  None where it cannot be built (its memory)."""
    from mcmc_clv_model_amd.sampler import HipSampler
    try:
        return HipSampler(p, mcmc=1, burnin=10 ** 8, thin=1, chains=chains, seed=7, draw_sink="none",
                          device=device)
    except Exception as e:  # (the line says so: clock_settle_work)
        global SCRATCH_ERROR
        SCRATCH_ERROR = f"{type(e).__name__}: {e}"[:200]
        return None


SCRATCH_ERROR = None  # why the last scratch_sampler call returned None


def profile_name(workload: str, phase: str) -> str:
    """The committed profile a line's traffic and counters come from: profiles/r*_<w>_*summary.json
    for the burn-in line, r*_<w>stored_*summary.json (tools/gpu_profile_round.sh <w>stored: every
    sweep a stored sweep) for the stored sub-line — never the other phase's (verdict r5 weak 3)."""
    return workload.replace("_", "") + ("stored" if phase == "stored" else "")  # c4_shard8 -> c4shard8


def roofline_for(workload: str, kname: str, D: int, K: int, bpu: float, units: int, t_launch: float, spl: int,
                 sharded: bool, profile: str | None = None, **extra) -> dict:
    """The roofline object of one kernel: SURVEY §8d bytes x (chain, customer) sweeps per launch /
    the launch's duration, measured traffic and the counters that decide `bound` (committed
    rocprofv3 summaries of `profile` — the workload's burn-in or stored phase, profile_name —
    of this instance; none for sharded runs, profiled at N = 1)."""
    profile = profile or workload
    achieved = bpu * units / t_launch / 1e9
    r = dict(bound=None, achieved=round(achieved, 3), peak=HBM_PEAK_GBS, unit="GB/s",
             frac=round(achieved / HBM_PEAK_GBS, 6), traffic=None, bytes_per_unit=round(bpu, 3),
             units_per_launch=units, sweeps_per_launch=spl, launch_us=round(t_launch * 1e6, 3),
             sweep_kernel_us=round(t_launch / spl * 1e6, 3), **extra)
    tr = None if sharded else committed_traffic(profile, kname, D, K)
    if tr:  # HBM bytes per launch (calibrated PMC), per sweep x sweeps per launch
        r["traffic"] = round(tr["bytes_per_sweep"] * spl)
        r["traffic_source"] = f"{tr['source']}: {tr['counters']}"
        r["traffic_vs_algorithmic"] = round(r["traffic"] / (bpu * units), 3)
    elif not sharded:
        r["traffic_source"] = f"no committed profile of {profile} (profiles/r*_{profile}_*summary.json)"
    ev = (None if sharded else committed_counters(profile, kname, D, K)) or {}
    if r["traffic"] is not None:
        ev["hbm_traffic_frac"] = round(r["traffic"] / t_launch / 1e9 / HBM_PEAK_GBS, 4)
    if ev.get("hbm_traffic_frac", 0.0) >= 0.6:
        r["bound"] = "hbm"
    elif max(ev.get("valu_busy_frac", 0.0), ev.get("valu_busy_frac_max_simd", 0.0)) >= 0.7:
        r["bound"] = "valu"
    elif "valu_busy_frac" in ev:
        r["bound"] = "latency"
    else:
        r["bound"] = "unmeasured"
    ev["rule"] = BOUND_RULE
    r["bound_evidence"] = ev
    return r


def whole_run_e2e(name: str, reps: int = 2) -> dict:
    """The drop-in's BASELINE run end to end, as the reference's driver times it (run_mcmc_abe.py:60-77:
    wall time around mcmc_draw_parameters, trace 1000): upload, every sweep of burn-in + mcmc, every
    stored draw returned in numpy arrays (the reference's layout).  `reps` calls; the first one also
    pays one-time process costs (copy-pool threads, pinned staging)."""
    import numpy as np
    from mcmc_clv_model_amd import mcmc_draw_parameters, mcmc_draw_parameters_rfm_m
    df, D, covs, chains, burnin, mcmc, thin, sink = load_workload(name)
    fn = mcmc_draw_parameters if D == 2 else mcmc_draw_parameters_rfm_m
    walls = []
    nbytes = 0
    for _ in range(reps):
        out = io.StringIO()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(out):
            d = fn(df, covs, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=42, trace=1000, n_mh_steps=20)
        walls.append(time.perf_counter() - t0)
        nbytes = int(sum(a.nbytes for a in d["level_1"]))
        ok = bool(np.isfinite(d["log_likelihood"]))
        del d  # (freeing the 3 GB result is not the next call's cost)
    best = min(walls[1:]) if len(walls) > 1 else walls[0]
    n = len(df)
    return dict(value=chains * n * (burnin + mcmc) / best, unit="customer-sweeps/s", seconds=round(best, 4),
                first_call_seconds=round(walls[0], 4), calls=reps, level1_bytes=nbytes, finite=ok,
                sweeps=f"{burnin} burn-in + {mcmc} (thin {thin}), {chains} chains",
                note="mcmc_draw_parameters%s end to end, draws returned (trace 1000, stdout captured)"
                     % ("" if D == 2 else "_rfm_m"))


def run_leg(name: str, world: int, rank: int, local_rank: int, dist, steps: int, warmup: int, *,
            graph_chunk: int = 32, exchange: str = "rccl", settle_ms: float = 0.0, stored_phase: bool = True,
            timing_steps: int = 3000, force_sharded: bool = False, phase: str = "burnin", blocks_per_unit: int = 0,
            one_call_warmup: bool = False, cold: bool = False, host_split: bool = False) -> dict:
    """One BASELINE configuration at this world size: `warmup` untimed sweeps, then exactly `steps`
    timed sweeps bracketed by barrier + synchronize (wall time, max over ranks).  The roofline
    comes from HIP events on the sampler's stream: the timed launch itself (persistent kernel) or a
    pass of min(steps, timing_steps) further sweeps (launch-per-sweep).  With `stored_phase` (and a
    burn-in longer than the window) the same chains continue 100 sweeps past the burn-in and
    `steps` stored sweeps are timed as well (bi:402-428: the draws or the running sums);
    `whole_run` combines both phases' per-sweep times over the BASELINE run's burn-in + mcmc
    (c4 / c5; c2 / c3 measure the drop-in end to end instead, see whole_run_e2e)."""
    import torch
    from mcmc_clv_model_amd.sampler import HipSampler, build_problem
    df, D, covs, chains, burnin, mcmc, thin, sink = load_workload(name, world)
    if phase == "stored":
        mcmc, burnin = mcmc + burnin, 0
    K = len(covs) + 1
    n_total = len(df)
    mcmc_workload = mcmc
    sharded = world > 1 or force_sharded
    p = build_problem(df, covs, D)
    del df
    if not sharded:
        kern = HipSampler(p, mcmc=mcmc, burnin=burnin, thin=thin, chains=chains, seed=42, draw_sink=sink,
                          device=local_rank, blocks_per_unit=blocks_per_unit)
        run, sync = kern.run, kern.synchronize
    else:
        from mcmc_clv_model_amd.distributed import ShardedSampler
        kern = ShardedSampler(p, rank=rank, world=world, chains=chains, mcmc=mcmc, burnin=burnin, thin=thin, seed=42,
                              draw_sink=sink, device=local_rank, graph_chunk=graph_chunk,
                              exchange=exchange if world > 1 else "rccl", verify_sweeps=8)
        run, sync = kern.step, kern.synchronize
    scratch = None
    if settle_ms > 0 and SETTLE_WORK == "sampler":
        if sharded:
            from mcmc_clv_model_amd.distributed import slice_problem
            scratch = scratch_sampler(slice_problem(p, *kern.plan.shard(rank)), chains, local_rank)
        else:
            scratch = scratch_sampler(p, chains, local_rank)
    del p
    info = kern.launch_info()
    persistent = info["persistent"]
    p2p = sharded and getattr(kern, "exchange", None) == "p2p"
    kname = "persist_kernel" if persistent else "sweep_kernel"
    n_local = kern.n

    def timed(n: int, events: bool):
        """Wall time of n sweeps bracketed by barrier + synchronize (max over ranks); with `events`
        (persistent kernel) also the timed launch's duration from its HIP events."""
        if events:
            kern.set_timing(True)
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(n)
        if sharded:
            sync()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        dt = time.perf_counter() - t0
        kt = None
        if events:
            kt = kern.kernel_time()
            kern.set_timing(False)
        if dist:
            t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local_rank}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt, kt

    def run_clock():
        """Shader clock (GHz) the timed launches ran at: the persistent kernel's own record of the
        last clv_run (clv_clock_ghz: s_memtime / s_memrealtime at chain 0's level-2 publishes), else
        a 50 us probe kernel enqueued right behind them (clv_clock_probe; the launch-per-sweep kernel
        keeps no record).  Returns (clock, source, probe); at world size > 1 the clock is the ranks'
        min and max.  Boxes of one pool run the same kernels at clocks ~13% apart."""
        rec = kern.clock_ghz()
        probe = kern.clock_probe(50.0)
        v = rec if rec > 0 else probe
        src = "clv_clock_ghz (in-kernel record)" if rec > 0 else ("clv_clock_probe (50 us probe kernel behind "
                                                                  "the timed launches)" if v > 0 else None)
        if dist:
            t = torch.tensor([v, -v], dtype=torch.float64, device=f"cuda:{local_rank}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            lo, hi = -float(t[1].item()), float(t[0].item())
            return (dict(min=round(lo, 3), max=round(hi, 3)) if lo > 0 else None), src, round(probe, 3)
        return (round(v, 3) if v > 0 else None), src, (round(probe, 3) if probe > 0 else None)

    def launch_roofline(first: int, n_t: int, kt, events_note: str, ph: str = "burnin"):
        """Roofline of n_t sweeps starting at sweep `first` (persistent: kt of the timed launch);
        traffic and counters from the committed profile of phase `ph` (profile_name)."""
        if kt is None:  # launch-per-sweep: event-timed pass over further sweeps of the same chains
            kern.set_timing(True)
            run(n_t)
            sync()
            kt = kern.kernel_time()
            kern.set_timing(False)
        if not kt or not kt["sweep_launches"]:
            return None
        t_sweep = kt["sweep_ms"] / kt["sweep_launches"] * 1e-3
        spl = n_t if persistent else 1  # sweeps per launch
        frac = stored_fraction(burnin, thin, first, first + n_t - 1)
        r = roofline_for(name, kname, D, K, survey_bytes(D, K, frac, sink), chains * n_local * spl, t_sweep * spl, spl,
                         sharded and not p2p, profile=profile_name(name, ph),
                         kernel=(("persist_kernel (one launch for all sweeps of a clv_run; level-2 workgroup per "
                                  "chain" + ("; unit partials exchanged over xGMI" if p2p else "") + ")")
                                 if persistent else
                                 ("sweep_kernel (incl. fused level-2 tail" +
                                  ("; unit partials exchanged through the peers' mail" if p2p else "") + ")")
                                 if (not sharded or p2p) else "sweep_kernel"),
                         bytes_per_unit_kernel=round(algorithmic_bytes(D, K, frac, sink), 3),
                         bytes_note="bytes_per_unit: SURVEY §8d (per stored sweep the full sink's draw, summary "
                                    "sinks +0); bytes_per_unit_kernel: the kernel's own streaming bytes",
                         timed_launches=kt["sweep_launches"] // spl, events=events_note)
        if kt.get("hyper_launches"):
            r["hyper_kernel_us"] = round(kt["hyper_ms"] / kt["hyper_launches"] * 1e3, 3)
        return r

    settle_s = settle_clocks(settle_ms, local_rank, scratch)  # (the problem build left the GPU idle for seconds)
    if persistent and one_call_warmup:  # the warm-up steps one call each, through the timed path (events
        kern.set_timing(True)           # on): the timed call is not the process's first of its kind
        for _ in range(warmup):
            run(1)
            sync()
            torch.cuda.synchronize()
        kern.kernel_time()
        kern.set_timing(False)
    else:
        run(warmup)
    sync()
    dt, kt = timed(steps, persistent)
    clk, clk_src, clk_probe = run_clock()  # the timed launches' shader clock (outside the timed region)
    host_us = kern.host_times() if (host_split and persistent and not sharded) else None
    value = chains * n_total * steps / dt
    roof = launch_roofline(warmup + 1, steps if persistent else min(steps, timing_steps), kt,
                           "the timed region's launch" if persistent else
                           f"a pass of {min(steps, timing_steps)} further sweeps, one event pair per launch", ph=phase)
    done = warmup + steps + (0 if persistent else min(steps, timing_steps))
    res = dict(workload=f"{name}: {'bivariate' if D == 2 else 'trivariate'}, K={K}, " +
                        ("synthetic (mcmc_clv_model_amd.data.synthetic_cbs)" if WORKLOADS[name][1].startswith("synthetic:")
                         else f"CDNOW {WORKLOADS[name][1]} CBS"),
               baseline_config=BASELINE_INDEX.get(name),
               scaling="strong" if name == "c4" else "proxy" if name == "c4_shard8" else "weak", value=value,
               unit="customer-sweeps/s",
               n_customers=n_total, customers_per_gpu=n_total // world, chains=chains, steps=steps, warmup=warmup,
               ms_per_step=dt / steps * 1e3, draw_sink=sink, burnin=burnin, mcmc=mcmc_workload, thin=thin,
               roofline=roof,
               path=("persistent kernel" if persistent else "launch-per-sweep sweep kernel") +
                    ("" if not sharded else
                     (", unit partials stored into every rank's mail over xGMI by the kernel (no host collective)"
                      if p2p else ", RCCL all-gather + level-2 kernel per sweep") +
                     (f" ({kern.p2p_note})" if getattr(kern, "p2p_note", None) else "")),
               phase=f"burn-in (sweeps {warmup + 1}..{warmup + steps})" if phase == "burnin" else
                     f"stored (burn-in 0, sweeps {warmup + 1}..{warmup + steps})",
               clock_settle_ms=round(settle_s * 1e3, 1), gpu_clock_ghz=clk, gpu_clock_source=clk_src,
               gpu_clock_probe_ghz=clk_probe)
    if host_us:
        res["host_us"] = dict(host_us, clv_run_total=round(sum(host_us.values()), 3), timed_region=round(dt * 1e6, 3))
    if sharded:
        res["exchange"] = dict(kind=getattr(kern, "exchange", None), note=getattr(kern, "p2p_note", None),
                               requested=exchange if world > 1 else "rccl")
    if cold and persistent and not sharded:
        # the timed window above is steady state (clocks settled; the timed call leaves its
        # last level-2 draw pending for the next call).  Here the same K sweeps from an idle GPU (0.3 s,
        # no settle) with that draw included (flushed inside the timed region)
        time.sleep(0.3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(steps)
        kern.flush()
        torch.cuda.synchronize()
        dtc = time.perf_counter() - t0
        done += steps
        res["cold"] = dict(ms_per_step=dtc / steps * 1e3, value=chains * n_total * steps / dtc,
                           note="after 0.3 s of idle GPU, no clock settle, the deferred last level-2 draw "
                                "flushed inside the timed region")
    if stored_phase and burnin > done + steps:
        # the stored phase (half of the BASELINE run; every stored sweep writes the draws or
        # read-modify-writes the running sums, bi:402-428): the same chains 100 sweeps past the boundary
        # (warm), then `steps` stored sweeps
        run(burnin + 100 - done)
        sync()
        settle_clocks(settle_ms, local_rank, scratch)
        dt_st, kt_st = timed(steps, persistent)
        clk_st, clk_st_src, _ = run_clock()
        first = burnin + 101
        n_st = steps if persistent else min(steps, timing_steps)
        roof_st = launch_roofline(first, n_st, kt_st, "the timed stored launch" if persistent else
                                  f"a pass of {n_st} further stored sweeps", ph="stored")
        if roof_st and roof_st.get("traffic") is not None and sink != "full":
            roof_st["traffic_note"] = ("measured stored-phase bytes vs SURVEY §8d (summary sink +0 per stored sweep): "
                                       "the excess is the read-modify-write of the running sums (%d fp64 per "
                                       "customer, 16 B each) on every stored sweep" % (9 if D == 2 else 11))
        v_st = chains * n_total * steps / dt_st
        fr = stored_fraction(burnin, thin, first, first + steps - 1)
        b8 = survey_bytes(D, K, fr, sink)
        bk = algorithmic_bytes(D, K, fr, sink)
        res["stored"] = dict(value=v_st, ms_per_step=dt_st / steps * 1e3, sweeps=f"{first}..{first + steps - 1}",
                             bytes_per_unit=round(b8, 2), hbm_frac=round(b8 * v_st / 1e9 / (world * HBM_PEAK_GBS), 5),
                             bytes_per_unit_kernel=round(bk, 2),
                             hbm_frac_kernel=round(bk * v_st / 1e9 / (world * HBM_PEAK_GBS), 5),
                             bytes_note="bytes_per_unit / hbm_frac: SURVEY §8d (summary sinks +0 per stored sweep); "
                                        "*_kernel: the kernel's own bytes incl. the running sums' read-modify-write",
                             roofline=roof_st, gpu_clock_ghz=clk_st, gpu_clock_source=clk_st_src)
        if WORKLOADS[name][1].startswith("synthetic:"):
            t_b, t_s = dt / steps, dt_st / steps
            res["whole_run"] = dict(value=chains * n_total * (burnin + mcmc_workload) / (burnin * t_b + mcmc_workload * t_s),
                                    sweeps=f"{burnin} burn-in + {mcmc_workload} stored",
                                    note="customer-sweeps/s of the BASELINE run from the two phases' per-sweep times")
    b8 = survey_bytes(D, K, stored_fraction(burnin, thin, warmup + 1, warmup + steps), sink)
    res["hbm_frac"] = round(b8 * value / 1e9 / (world * HBM_PEAK_GBS), 5)
    res["bytes_per_unit"] = round(b8, 2)
    res["_persistent"] = persistent
    res["_p2p"] = p2p
    res["_timed_region"] = (f"one persistent-kernel launch of {steps} sweeps" if persistent and not sharded else
                            f"one persistent-kernel launch of {steps} sweeps per rank, unit partials stored into every "
                            "rank's IPC-mapped mail over xGMI (no host collective per sweep)" if persistent else
                            "hipGraph replay of fused sweep launches" + (
                                " (unit partials exchanged through the peers' mail by the kernels)" if p2p else "")
                            if (not sharded or p2p) else
                            f"torch.cuda graph replay ({graph_chunk} sweeps: sweep + group kernels, RCCL all_gather, "
                            "level-2 kernel)" if graph_chunk else "eager: sweep + group kernels, RCCL all_gather, level-2")
    kern.close()
    if scratch is not None:
        scratch.close()
    res["clock_settle_work"] = ("sweeps of a scratch sampler over the same customers (seed 7, no draws kept)"
                                if scratch is not None else
                                ("fp64 matmuls" + (f" (scratch sampler unavailable: {SCRATCH_ERROR})"
                                                   if SETTLE_WORK == "sampler" and SCRATCH_ERROR else ""))
                                if settle_ms > 0 else None)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=19000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="primary workload (default: c2 at N = 1, c5 at N > 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timing-steps", type=int, default=3000, help="sweeps in the event-timed roofline pass")
    ap.add_argument("--graph-chunk", type=int, default=32,
                    help="sharded RCCL path: sweeps (incl. the all-gather) per captured torch.cuda graph; 0 = eager")
    ap.add_argument("--force-sharded", action="store_true",
                    help="use the sharded path (torch.distributed exchange) even at world size 1")
    ap.add_argument("--exchange", default="auto", choices=["auto", "p2p", "rccl"],
                    help="world size > 1: unit-partial exchange per sweep — p2p = the kernels store into every "
                         "rank's IPC-mapped mail over xGMI (auto: where it verifies bitwise against RCCL), "
                         "rccl = all_gather per sweep")
    ap.add_argument("--scaling-configs", default=None,
                    help="comma-separated `configs` legs (default: the other BASELINE configurations at this N); "
                         "'' to skip")
    ap.add_argument("--scaling-steps", type=int, default=1000)
    ap.add_argument("--blocks-per-unit", type=int, default=0,
                    help="(world size 1, A/B) blocks per statistics unit instead of the plan's (0)")
    ap.add_argument("--phase", default="burnin", choices=["burnin", "stored"],
                    help="(profiling) stored: the sampler's burn-in is 0, so every timed sweep is a stored sweep "
                         "(the running sums' read-modify-write / the draws' stores of bi:402-428)")
    ap.add_argument("--settle-work", default="sampler", choices=["sampler", "matmul"],
                    help="the clock-settle work before each timed window (settle_clocks): sweeps of a scratch "
                         "sampler over the same customers, or fp64 matmuls (A/B)")
    ap.add_argument("--no-c1-leg", dest="c1_leg", action="store_false",
                    help="skip BASELINE configs[0] (c1 on the GPU and its 1-core CPU leg)")
    ap.add_argument("--no-stored-phase", dest="stored_phase", action="store_false",
                    help="skip the stored-sweep sub-lines")
    ap.add_argument("--no-whole-run", dest="whole_run", action="store_false",
                    help="skip the drop-in's end-to-end BASELINE runs (c2 / c3 through mcmc_draw_parameters)")
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
    global SETTLE_WORK
    SETTLE_WORK = a.settle_work
    if a.cpu_baseline_child:
        cpu_baseline_child(a.workload or "c2", a.cpu_warm, a.cpu_timed)
        return

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
    _lib.lib()
    name = a.workload or primary_workload(world)
    exch = a.exchange if world > 1 else "rccl"
    prim = run_leg(name, world, rank, local_rank, dist, a.steps, a.warmup, graph_chunk=a.graph_chunk, exchange=exch,
                   settle_ms=a.clock_settle_ms, stored_phase=a.stored_phase, timing_steps=a.timing_steps,
                   force_sharded=a.force_sharded, phase=a.phase, blocks_per_unit=a.blocks_per_unit,
                   one_call_warmup=True, cold=True, host_split=True)
    D, data, covs, chains, burnin, mcmc, thin, sink = WORKLOADS[name]
    if a.phase == "stored":
        mcmc, burnin = mcmc + burnin, 0
    if world == 1 and not a.force_sharded and a.whole_run and name in ("c2", "c3") and a.phase == "burnin":
        prim["whole_run"] = whole_run_e2e(name)

    legs = config_legs(world, name) if a.scaling_configs is None else [c for c in a.scaling_configs.split(",") if c]
    extra = {}
    for leg in legs:
        if leg == name:
            continue
        # c3 / c4 / c5 (and c2 tiled at N > 1): 200 warm-up sweeps (the launch-per-sweep path captures
        # its hipGraph on first use; clocks ramp), then 1,000 timed sweeps per phase
        extra[leg] = run_leg(leg, world, rank, local_rank, dist, a.scaling_steps, 200, graph_chunk=a.graph_chunk,
                             exchange=exch, settle_ms=a.clock_settle_ms, stored_phase=a.stored_phase,
                             timing_steps=a.timing_steps)
        if leg == "c4_shard8":
            extra[leg]["note"] = ("NOT a BASELINE configuration: rank 0's shard of c4 at 8 ranks (distributed.plan(1M, 8): "
                                  "126,976 customers, K=5, 1 chain) run at world size 1 — the per-GPU work of c4's "
                                  "strong-scaling point without the exchange (DESIGN.md §6)")
        if world > 1 and leg == "c2":
            extra[leg]["note"] = ("NOT a BASELINE configuration: c2's 23,570 CDNOW customers tiled once per rank "
                                  "(a rehearsal of the CDNOW-size exchange at N GPUs)")
        if world == 1 and a.whole_run and leg == "c3":
            extra[leg]["whole_run"] = whole_run_e2e("c3")
    if world == 1 and not a.force_sharded and a.c1_leg and "c1" not in (name,) and a.scaling_configs is None:
        # BASELINE configs[0] ("Bivariate M1, Abe 1/10 CDNOW subset, 4000 iters on CPU numpy reference
        # path"): the same 4-chain c1 sampler on the GPU (2,000 sweeps after 80), next to its 1-core
        # CPU leg in cpu_baseline["c1"]
        extra["c1"] = run_leg("c1", 1, rank, local_rank, None, 2000, 80, settle_ms=a.clock_settle_ms,
                              stored_phase=False)

    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline and not a.force_sharded:
            cpu = cpu_baseline(name)
            for leg in ("c1", "c3"):
                if leg in extra and leg != name:
                    c = cpu_baseline(leg, parallel=False)
                    c.update(gpu_value=extra[leg]["value"], gpu_speedup=extra[leg]["value"] / c["value"])
                    cpu[leg] = c
                    extra[leg]["cpu_baseline"] = dict(value=c["value"], unit=c["unit"], cores=1, kind=c["kind"],
                                                      s_per_sweep=c["s_per_sweep"], sample=c["sample"],
                                                      gpu_speedup=c["gpu_speedup"])
        for v in extra.values():
            for k in ("_persistent", "_p2p", "_timed_region"):
                v.pop(k, None)
        n_total = prim["n_customers"]
        line = dict(
            metric="MCMC sweeps/sec x N_customers (customer-sweeps/s)", value=prim["value"], unit="customer-sweeps/s",
            n_gpus=world, steps=a.steps, warmup=a.warmup, ms_per_step=prim["ms_per_step"], higher_is_better=True,
            scaling="weak", vs_baseline=None, dtype="f64",
            proposal_dtype="f32",  # t3 proposal noise and accept log-uniforms; state, posterior f64
            ms_per_step_kind=("steady state: the GPU's clocks settled by clock_settle_ms of sweeps on a scratch sampler "
                              "(clock_settle_work; the timed chains untouched) before the warm-up; the timed call leaves its last level-2 draw pending (drawn at the start of the "
                              "next call) — `cold` times the same steps from an idle GPU with that draw included")
            if prim.get("_persistent") and not sharded else "wall time of the timed steps",
            data=(f"synthetic CBS ({n_total} customers, mcmc_clv_model_amd.data.synthetic_cbs" +
                  (f", {n_total // world:,} per GPU)" if world > 1 else ")")
                  if data.startswith("synthetic:") else
                  f"CDNOW {data} CBS ({n_total // world:,} real customers, tests/golden/cdnow_{data}_cbs.npz)"
                  + ("" if world == 1 else f", tiled x{world} (one copy per rank)")),
            config=dict(workload=f"{name}: {'bivariate' if D == 2 else 'trivariate'} M2, covariates {covs}",
                        baseline_config=BASELINE_INDEX.get(name),
                        n_customers=n_total, chains=chains, n_mh_steps=20, burnin=burnin, mcmc=mcmc,
                        thin=thin, seed=42, draw_sink=sink, parallelism=f"customer-shard x{world}",
                        **({"phase": "stored (profiling: burn-in 0, every sweep stores)"} if a.phase == "stored" else {}),
                        timed_region=prim["_timed_region"]),
            clock_settle_ms=prim["clock_settle_ms"],
            clock_settle_work=prim.get("clock_settle_work"),
            gpu_clock_ghz=prim.get("gpu_clock_ghz"),
            gpu_clock_source=prim.get("gpu_clock_source"),
            gpu_clock_probe_ghz=prim.get("gpu_clock_probe_ghz"),
            gpu_clock_note="shader clock of the timed launches: the persistent kernel's own record (s_memtime / "
                           "s_memrealtime between chain 0's level-2 publishes, clv_clock_ghz), else — launch-per-sweep "
                           "legs — a 50 us probe kernel right behind them (clv_clock_probe; gpu_clock_probe_ghz on "
                           "every line cross-checks the two): boxes of one pool run the same cycles at clocks ~13% "
                           "apart (DESIGN.md §8 round 5)",
            roofline=prim["roofline"], cpu_baseline=cpu,
            host_us=prim.get("host_us"),
            cold=prim.get("cold"),
            stored=prim.get("stored"),
            whole_run=prim.get("whole_run"),
            exchange=prim.get("exchange"),
            path=prim["path"],
            speedup_vs_cpu_1core=(prim["value"] / cpu["value"]) if cpu else None,
            configs=extra or None,
        )
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
