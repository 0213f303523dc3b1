"""Host-code driver for the AddressSanitizer build (tests/test_host_asan.py runs it in a child
process with the clang ASan runtime preloaded): every host-only path of the C ABI — argument
validation, the failure/cleanup path of clv_create (no device here), the persistent grid's
placement map, the group's validation — on ctypes structs laid out as the Python binding does."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from mcmc_clv_model_amd import _lib  # noqa: E402  (struct mirrors only; the library is loaded below)

L = ctypes.CDLL(sys.argv[1])
sp = ctypes.c_void_p
L.clv_sizeof.restype = ctypes.c_int64
L.clv_last_error.restype = ctypes.c_char_p
L.clv_create.argtypes = [ctypes.POINTER(_lib.ClvConfig), ctypes.POINTER(_lib.ClvData), ctypes.POINTER(_lib.ClvPrior),
                         ctypes.POINTER(sp)]
L.clv_debug_wg_map.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
L.clv_group_create.argtypes = [ctypes.POINTER(sp), ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(sp)]
L.clv_default_blocks_per_unit.argtypes = [ctypes.c_int64]
L.clv_destroy.argtypes = [sp]
L.clv_group_destroy.argtypes = [sp]

for i, st in enumerate((_lib.ClvConfig, _lib.ClvData, _lib.ClvPrior)):
    assert L.clv_sizeof(i) == ctypes.sizeof(st), st
assert L.clv_abi_version() == _lib.ABI_VERSION

n = 700
x = np.arange(n, dtype=np.int32) % 5
tx = np.linspace(0.0, 30.0, n)
T = np.full(n, 39.0)
cov = np.linspace(-1.0, 1.0, 2 * n)
logs = np.zeros(n)
data = _lib.ClvData(n=n, x=x.ctypes.data, t_x=tx.ctypes.data, T_cal=T.ctypes.data, covariates=cov.ctypes.data,
                    log_s=logs.ctypes.data)
pr = _lib.ClvPrior(lam_init=0.3, nu_n=5.0 + n, omega2=1.0)
base = dict(abi_version=_lib.ABI_VERSION, D=2, K=3, n_mh_steps=20, burnin=2, mcmc=3, thin=1, n_chains=2,
            chain_first=0, rng_mode=0, draw_sink=0, device=-1, seed=1, n_global=n, shard_begin=0, world_size=1,
            rank=0, blocks_per_rank=0, blocks_per_unit=0, stream=0)
bad = [dict(D=4), dict(K=0), dict(K=10), dict(thin=0), dict(n_chains=0), dict(abi_version=0), dict(draw_sink=7),
       dict(blocks_per_unit=3), dict(n_global=n - 1), dict(shard_begin=256), dict(world_size=2, blocks_per_rank=0),
       dict(world_size=2, rank=2, blocks_per_rank=2), dict(rng_mode=1, world_size=2, blocks_per_rank=2),
       dict(n_mh_steps=-1), dict(burnin=-1), dict(n_global=1 << 33)]
for b in bad:
    h = sp()
    rc = L.clv_create(ctypes.byref(_lib.ClvConfig(**dict(base, **b))), ctypes.byref(data), ctypes.byref(pr),
                      ctypes.byref(h))
    assert rc == -1 and not h.value, (b, rc)
    assert L.clv_last_error()
# valid configurations: no device in this process, so each fails inside the allocation sequence and
# takes clv_create's cleanup path (clv_destroy of a partly built sampler)
for b in (dict(), dict(D=3), dict(draw_sink=1), dict(draw_sink=3), dict(world_size=2, blocks_per_rank=2, n_global=n + 600),
          dict(K=1)):
    h = sp()
    rc = L.clv_create(ctypes.byref(_lib.ClvConfig(**dict(base, **b))), ctypes.byref(data), ctypes.byref(pr),
                      ctypes.byref(h))
    assert rc != 0 and not h.value, (b, rc)
L.clv_destroy(None)
for nc, nb, ncu in [(1, 1, 256), (4, 93, 256), (4, 127, 256), (2, 300, 256), (8, 63, 256), (3, 5, 7), (1, 511, 256)]:
    out = np.full(nc * (nb + 1), -1, np.int32)
    assert L.clv_debug_wg_map(nc, nb, ncu, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))) == 0
    assert sorted(out.tolist()) == sorted((c << 16) | b for c in range(nc) for b in range(nb + 1))
for v in (1, 255, 256, 131072, 131073, 10 ** 7, 10 ** 9):
    assert L.clv_default_blocks_per_unit(v) >= 1
g = sp()
assert L.clv_group_create(None, 2, 0, ctypes.byref(g)) == -1
arr = (sp * 2)(None, None)
assert L.clv_group_create(arr, 2, 0, ctypes.byref(g)) == -1
assert L.clv_group_create(arr, 2, 9, ctypes.byref(g)) == -1
L.clv_group_destroy(None)
print("asan host driver ok")
