"""The C ABI's host code under AddressSanitizer (SURVEY §5 "race detection /
sanitizers": an -fsanitize=address host build of the C-ABI for CPU-side unit
tests).  `make asan` builds build/libgym_amd_asan.so with the host half of
every ga_* entry point instrumented (the device code is built as usual); a
python run with the ASan runtime preloaded then drives test_abi.py -- symbol
exports, struct layout, the gap table, every invalid-argument case -- through
that library.  Any heap/stack error in the argument validation aborts the run.
No GPU is touched."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime():
    rts = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return rts[-1] if rts else None


def test_abi_checks_under_asan(tmp_path):
    rt = _runtime()
    if rt is None:
        pytest.skip("no ASan runtime in this ROCm install")
    r = subprocess.run(["make", "-C", ROOT, "asan"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lib = os.path.join(ROOT, "build", "libgym_amd_asan.so")
    env = {**os.environ, "LD_PRELOAD": rt, "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
           "GYM_AMD_LIB": lib, "PYTHONPATH": ROOT}
    probe = ("import ctypes; from gym_amd import _lib; L = _lib.lib(); "
             "assert _lib.LIB_PATH.endswith('libgym_amd_asan.so'); "
             "assert hasattr(ctypes.CDLL(None), '__asan_init'); print('asan-active')")
    r = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    assert r.returncode == 0 and "asan-active" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "pytest", os.path.join(ROOT, "tests", "test_abi.py"), "-q",
                        "-p", "no:cacheprovider"], env=env, capture_output=True, text=True, timeout=600,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "AddressSanitizer" not in r.stderr
