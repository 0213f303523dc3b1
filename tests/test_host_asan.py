"""SURVEY §5 (race detection / sanitizers): the C ABI's host code under AddressSanitizer.

`make -C mcmc_clv_model_amd/csrc` (build()) also links libclvmcmc_asan.so: capi / group host code
compiled with -fsanitize=address for the host side only (device code as shipped).  The driver
(tests/asan_host_driver.py) runs every host-only path — argument validation, clv_create's cleanup
path after a failed allocation sequence (no device in this container), the placement map, the
group's validation — in a child process with the clang ASan runtime preloaded; any invalid access
aborts it with an AddressSanitizer report.  (GPU-side sanitizers are not available on the pool.)"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mcmc_clv_model_amd", "libclvmcmc_asan.so")


def _asan_runtime():
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True,
                         text=True)
    path = out.stdout.strip()
    return path if out.returncode == 0 and os.path.isfile(path) else None


def test_host_code_under_asan():
    rt = _asan_runtime()
    if rt is None or not os.path.exists(LIB):
        pytest.skip("ASan runtime or libclvmcmc_asan.so (make -C mcmc_clv_model_amd/csrc asan) not available")
    syms = subprocess.run(["nm", "-D", "--undefined-only", LIB], capture_output=True, text=True).stdout
    assert "__asan_report_load8" in syms, "libclvmcmc_asan.so is not instrumented"
    env = dict(os.environ, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "asan_host_driver.py"), LIB], capture_output=True,
                       text=True, env=env, timeout=300, cwd=ROOT)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0 and "asan host driver ok" in r.stdout, (r.returncode, r.stderr[-4000:])
