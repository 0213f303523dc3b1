"""ctypes binding of libclvmcmc.so (C ABI declared in include/clvmcmc.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU is visible,
every sampler call raises.  torch (when importable) is imported before the library so that
``libamdhip64.so.7`` resolves to the HIP runtime torch already loaded — one runtime per
process, so device pointers and streams can be shared with torch.distributed (RCCL).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_uint8, POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_uint32, c_uint64, c_void_p

try:  # share torch's HIP runtime when torch is present (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the single-GPU path
    torch = None

LIB_NAME = "libclvmcmc.so"
LIB_PATH = os.environ.get("CLV_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

ABI_VERSION = 2
BLOCK = 256
MAX_K = 9
MAX_D = 3
RNG_PHILOX, RNG_REPLAY = 0, 1
SINK_FULL, SINK_SUMMARY, SINK_NONE, SINK_SUMMARY_PCT = 0, 1, 2, 3
EXCHANGE_AUTO, EXCHANGE_P2P, EXCHANGE_COPY = 0, 1, 2
SUM_STATS = ("lambda", "mu", "z", "log_lambda", "log_mu", "lambda2", "mu2", "eta", "log_eta", "mu_capped", "tau")
SUMMARY_MU_CAP = 0.05  # CLV_SUMMARY_MU_CAP: the "mu_capped" sum is of min(mu, 0.05) (analysis_bi_helpers.py:89)
N_SUM_STATS = len(SUM_STATS)
TAPE_HYPER = 40


class ClvConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", c_int32), ("D", c_int32), ("K", c_int32), ("n_mh_steps", c_int32),
        ("burnin", c_int32), ("mcmc", c_int32), ("thin", c_int32), ("n_chains", c_int32),
        ("chain_first", c_int32), ("rng_mode", c_int32), ("draw_sink", c_int32), ("device", c_int32),
        ("seed", c_uint64), ("n_global", c_int64), ("shard_begin", c_int64),
        ("world_size", c_int32), ("rank", c_int32), ("blocks_per_rank", c_int32),
        ("blocks_per_unit", c_int32), ("stream", c_uint64),
    ]


class ClvData(ctypes.Structure):
    _fields_ = [
        ("n", c_int64), ("x", c_void_p), ("t_x", c_void_p), ("T_cal", c_void_p),
        ("covariates", c_void_p), ("log_s", c_void_p),
    ]


class ClvPrior(ctypes.Structure):
    _fields_ = [
        ("lam_init", c_double), ("V", c_double * 81), ("chol_V", c_double * 81), ("A0B0", c_double * 27),
        ("S0_B0A0B0", c_double * 9), ("nu_n", c_double), ("beta_init", c_double * 27),
        ("sigma_init", c_double * 9), ("omega2", c_double),
    ]


_lib = None


class ClvError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load libclvmcmc.so (once) and declare every entry point of include/clvmcmc.h."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ClvError(
            f"{LIB_NAME} is not built ({LIB_PATH}); run `make -C mcmc_clv_model_amd/csrc` "
            "or `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    sp = c_void_p
    dp = POINTER(c_double)
    sigs = {
        "clv_abi_version": (c_int32, []),
        "clv_default_blocks_per_unit": (c_int32, [c_int64]),
        "clv_sizeof": (c_int64, [c_int32]),
        "clv_last_error": (c_char_p, []),
        "clv_device_count": (c_int32, [POINTER(c_int32)]),
        "clv_create": (c_int32, [POINTER(ClvConfig), POINTER(ClvData), POINTER(ClvPrior), POINTER(sp)]),
        "clv_destroy": (None, [sp]),
        "clv_set_replay_tape": (c_int32, [sp, dp, c_int64]),
        "clv_replay_sweep_stride": (c_int64, [sp]),
        "clv_run": (c_int32, [sp, c_int64]),
        "clv_rollback": (c_int32, [sp]),
        "clv_sweep": (c_int32, [sp]),
        "clv_hyper": (c_int32, [sp, c_void_p]),
        "clv_partials": (c_int32, [sp, POINTER(c_void_p), POINTER(c_int64), POINTER(c_int32)]),
        "clv_copy_partials": (c_int32, [sp, c_void_p]),
        "clv_synchronize": (c_int32, [sp]),
        "clv_sweeps_done": (c_int64, [sp]),
        "clv_clock_ghz": (c_int32, [sp, POINTER(c_double)]),
        "clv_clock_probe": (c_int32, [sp, c_double, POINTER(c_double)]),
        "clv_launch_info": (c_int32, [sp, POINTER(c_int64)]),
        "clv_p2p_info": (c_int32, [sp, POINTER(c_int64)]),
        "clv_p2p_export": (c_int32, [sp, c_void_p]),
        "clv_p2p_connect": (c_int32, [sp, c_void_p, POINTER(c_uint64)]),
        "clv_p2p_disconnect": (c_int32, [sp]),
        "clv_p2p_set_persistent": (c_int32, [sp, c_int32]),
        "clv_set_wait_timeout": (c_int32, [sp, c_double]),
        "clv_set_stream": (c_int32, [sp, c_uint64]),
        "clv_note_sweeps": (c_int32, [sp, c_int64]),
        "clv_read_draws": (c_int32, [sp, dp, dp, dp]),
        "clv_stream_draws": (c_int32, [sp, dp]),
        "clv_read_summary": (c_int32, [sp, dp, POINTER(c_int64)]),
        "clv_get_state": (c_int32, [sp, dp, dp, dp]),
        "clv_set_state": (c_int32, [sp, dp, dp, dp, c_int64]),
        "clv_set_timing": (c_int32, [sp, c_int32]),
        "clv_kernel_time": (c_int32, [sp, dp, POINTER(c_int64), dp, POINTER(c_int64)]),
        "clv_debug_philox": (c_int32, [c_uint32, c_uint32, POINTER(c_uint32), c_int64, POINTER(c_uint32)]),
        "clv_debug_variates": (c_int32, [c_uint64, c_int32, c_uint32, c_int64, c_int32, POINTER(c_float),
                                         POINTER(c_float), POINTER(c_float), dp, dp, dp, dp, POINTER(c_float)]),
        "clv_debug_log2u_scan": (c_int32, [c_uint64, c_uint64, dp]),
        "clv_debug_host_times": (c_int32, [sp, POINTER(c_int64)]),
        "clv_debug_t3": (c_int32, [POINTER(c_uint32), c_int64, c_int32, POINTER(c_float), POINTER(c_float)]),
        "clv_debug_level2": (c_int32, [c_int32, c_int32, POINTER(ClvPrior), dp, dp, dp, dp, dp, dp, dp]),
        "clv_debug_hyper_variates": (c_int32, [c_uint64, c_int32, c_uint32, c_double, c_int64, dp, dp]),
        "clv_debug_stamps": (c_int32, [sp, POINTER(c_uint64)]),
        "clv_debug_wg_stamps": (c_int32, [sp, POINTER(c_uint64)]),
        "clv_debug_exp": (c_int32, [dp, c_int64, dp]),
        "clv_debug_log": (c_int32, [dp, c_int64, dp]),
        "clv_debug_mh_step": (c_int32, [c_int64, POINTER(c_int32), POINTER(c_uint8), dp, dp, dp, dp, dp,
                                        POINTER(c_float), dp, POINTER(c_float), dp]),
        "clv_debug_wg_map": (c_int32, [c_int32, c_int32, c_int32, POINTER(c_int32)]),
        "clv_debug_persist_choice": (c_int32, [c_int32, c_int32, c_int32, c_int64, c_int32, c_int32]),
        "clv_debug_persist_fits": (c_int32, [c_int64, c_int32, c_int32]),
        "clv_group_create": (c_int32, [POINTER(sp), c_int32, c_int32, POINTER(sp)]),
        "clv_group_run": (c_int32, [sp, c_int64]),
        "clv_group_exchange": (c_int32, [sp]),
        "clv_group_destroy": (None, [sp]),
        "clv_predict": (c_int32, [c_int32, dp, c_int64, c_int64, c_int32, dp, c_double, c_uint64, c_int32, c_double,
                                  POINTER(c_int64), dp]),
        "clv_predict_sampler": (c_int32, [sp, c_double, c_uint64, c_int32, c_double, POINTER(c_int64), dp]),
        "clv_track": (c_int32, [c_int32, dp, c_int64, c_int64, c_int32, dp, dp, c_int32, c_uint64, dp]),
        "clv_track_sampler": (c_int32, [sp, dp, dp, c_int32, c_uint64, dp]),
        "clv_level1_summary": (c_int32, [c_int32, dp, c_int64, c_int64, c_int32, c_double, dp]),
        "clv_level1_summary_sampler": (c_int32, [sp, c_double, dp]),
        "clv_chain_total_loglik": (c_int32, [c_int32, dp, c_int64, c_int64, c_int32, POINTER(c_int32), dp, dp]),
        "clv_chain_total_loglik_sampler": (c_int32, [sp, dp]),
        "clv_elog2cbs": (c_int32, [c_int32, c_int64, POINTER(c_int64), POINTER(c_int64), dp, c_int64, c_int64, c_int64,
                                   POINTER(c_int64), POINTER(c_int64), POINTER(c_int64), dp, dp, dp, dp,
                                   POINTER(c_int64), dp, dp, POINTER(c_int64), dp]),
        "clv_generate_pareto_abe": (c_int32, [c_int32, c_int64, c_int32, dp, dp, dp, dp, c_int32, dp, c_uint64,
                                              POINTER(c_int64), dp, dp, dp, dp, POINTER(c_uint8), POINTER(c_int64), dp,
                                              POINTER(c_int64), POINTER(c_int64), c_int64, POINTER(c_int64), dp]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.clv_abi_version() != ABI_VERSION:
        raise ClvError("libclvmcmc.so ABI version mismatch; rebuild it")
    for i, st in enumerate((ClvConfig, ClvData, ClvPrior)):
        if L.clv_sizeof(i) != ctypes.sizeof(st):
            raise ClvError(f"ctypes mirror of {st.__name__} does not match the C struct; rebuild")
    _lib = L
    return L


# Columns of clv_level1_summary() (include/clvmcmc.h CLV_L1_*).
L1_STATS = ("mean_lambda", "lambda_p025", "lambda_p975", "mean_mu", "mean_mu_capped", "mu_p025", "mu_p975",
            "mean_z", "mean_tau", "mean_eta")


def exported_symbols():
    """Names of every entry point declared in include/clvmcmc.h (checked by the CPU tests)."""
    import re
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "clvmcmc.h")
    with open(hdr) as f:
        return sorted(set(re.findall(r"\b(clv_[a-z0-9_]+)\s*\(", f.read())))


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().clv_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(msg)
        raise ClvError(f"libclvmcmc error {rc}: {msg}")


def dptr(a):
    """ctypes double* of a C-contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(POINTER(c_double))


def device_count() -> int:
    n = c_int32(0)
    rc = lib().clv_device_count(ctypes.byref(n))
    if rc != 0:
        return 0
    return n.value
