"""Host-code sanitizers (CPU only - GPU ASan / xnack runs are not available on this
pool). Two layers:

* ``tools/host_sanitize.cpp`` - the pure-host launch planning (weight-gradient XCD packing,
  ``csrc/include/wgrad_pack.h``) built with ``-fsanitize=address,undefined`` and run on random
  and malformed inputs; always runs (g++ only).
* the ASan build of the whole native library (``python csrc/build.py --asan``: bindings and
  launchers instrumented, device code not) loaded under the ASan runtime; its static
  initialisers, op registration and the host-only ops run clean. Skipped when that variant is
  not built (it takes minutes; ``tools/asan_run.sh`` builds and runs it).
"""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_planning_code_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_sanitize"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", f"-I{ROOT / 'csrc/include'}",
           str(ROOT / "tools/host_sanitize.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "asan" in (r.stderr or "").lower():
        pytest.skip("sanitizer runtime not available: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and "host_sanitize ok" in r.stdout, r.stdout + r.stderr


def _asan_runtime():
    try:
        out = subprocess.run(["hipcc", "-print-file-name=libclang_rt.asan-x86_64.so"],
                             capture_output=True, text=True, timeout=60).stdout.strip()
    except Exception:
        return None
    return out if out and os.path.isabs(out) and os.path.exists(out) else None


def test_native_library_asan_build_loads_clean():
    lib = ROOT / "vi_normflows_amd/_native/libvinf_hip_asan.so"
    rt = _asan_runtime()
    if not lib.exists() or rt is None:
        pytest.skip("ASan variant not built (python csrc/build.py --asan) or no ASan runtime")
    code = ("import torch; torch.ops.load_library(%r); v = torch.ops.vinf; "
            "p = v.gemm_persist(-1); q = v.gemm_wgrad_xcd_pack(-1); "
            "v.gemm_wgrad_xcd_pack(q); v.gemm_persist(p); print('asan load ok', p, q)" % str(lib))
    env = dict(os.environ, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               VINF_NATIVE_LIB=str(lib))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0 and "asan load ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr
