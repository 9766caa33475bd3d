"""Host code under AddressSanitizer: libkrca's host-only translation units
(api.cpp, ppr_pack.cpp — Makefile target `asan`) and oracle/krca_oracle.c (oracle Makefile
`asan`) built with -fsanitize=address and driven by tests/host_asan_driver.py in a subprocess
with the clang ASan runtime preloaded.  GPU code is not sanitized (no GPU ASan on this pool)."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime():
    c = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    return c[0] if c else None


@pytest.mark.skipif(_runtime() is None, reason="clang ASan runtime not installed")
def test_host_code_under_asan():
    csrc = os.path.join(ROOT, "kubernetes-rca-system_amd", "csrc")
    for d in (csrc, os.path.join(ROOT, "oracle")):
        r = subprocess.run(["make", "-C", d, "asan"], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    env = dict(os.environ, LD_PRELOAD=_runtime(), ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               KRCA_ORACLE_LIB=os.path.join(ROOT, "oracle", "_build", "libkrca_oracle_asan.so"))
    lib = os.path.join(ROOT, "kubernetes-rca-system_amd", "lib", "asan", "libkrca_host_asan.so")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "host_asan_driver.py"), lib], env=env,
                       capture_output=True, text=True, timeout=600)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0 and "host-asan-ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
