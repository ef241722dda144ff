#!/usr/bin/env python3
"""Build the vi_normflows_amd native library for gfx950 with hipcc directly.

No hipify, no torch.utils.cpp_extension: every ``csrc/kernels/*.hip`` file is a
CDNA4 kernel translation unit compiled with ``hipcc --offload-arch=gfx950``,
``csrc/bindings/*.cpp`` registers them as ``torch.ops.vinf.*`` and the objects
are linked into ``vi_normflows_amd/_native/libvinf_hip.so`` (in-tree, so the
built library travels with the repository snapshot to the GPU box).

Usage:  python csrc/build.py [--force] [--jobs N] [--debug] [--save-temps]
The build is incremental (object newer than its source and every header).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
OUT_DIR = ROOT / "vi_normflows_amd" / "_native"
OUT_LIB = OUT_DIR / "libvinf_hip.so"
OBJ_DIR = ROOT / "build" / "obj"
ARCH = os.environ.get("VINF_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (need ROCm at /opt/rocm)")


def _torch_paths():
    import torch  # noqa: F401  (import only to locate headers/libs)
    from torch.utils import cpp_extension as ce

    return ce.include_paths(), ce.library_paths(), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _headers() -> list[Path]:
    return sorted((CSRC / "include").glob("*.h"))


def _stale(obj: Path, src: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(p.stat().st_mtime > t for p in [src, *deps])


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout)
        raise RuntimeError(f"compile failed: {cmd[-1]}")
    if r.stdout.strip():
        sys.stderr.write(r.stdout)


def build(force: bool = False, jobs: int | None = None, debug: bool = False,
          save_temps: bool = False, verbose: bool = True) -> Path:
    hipcc = _hipcc()
    incs, libdirs, abi = _torch_paths()
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    headers = _headers()
    opt = ["-O0", "-g"] if debug else ["-O3"]
    common = ["-std=c++17", "-fPIC", f"-I{CSRC / 'include'}", "-Wno-unused-result",
              "-Wno-deprecated-declarations"]
    kernel_flags = common + opt + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
    if save_temps:
        kernel_flags += ["-save-temps=obj"]
    bind_flags = common + ["-O2", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
                           f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                           "-DTORCH_API_INCLUDE_EXTENSION_H"] + [f"-I{p}" for p in incs]
    jobs_list = []
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        obj = OBJ_DIR / (src.stem + ".o")
        jobs_list.append((src, obj, [hipcc, "-c", *kernel_flags, "-o", str(obj), str(src)]))
    for src in sorted((CSRC / "bindings").glob("*.cpp")):
        obj = OBJ_DIR / ("bind_" + src.stem + ".o")
        jobs_list.append((src, obj, [hipcc, "-c", *bind_flags, "-o", str(obj), str(src)]))
    todo = [j for j in jobs_list if force or _stale(j[1], j[0], headers)]
    n = jobs or min(8, os.cpu_count() or 4)
    if todo:
        if verbose:
            print(f"[vinf build] compiling {len(todo)} unit(s) for {ARCH} with {n} job(s)",
                  file=sys.stderr)
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            futs = [ex.submit(_run, cmd) for _, _, cmd in todo]
            for f in futs:
                f.result()
    objs = [str(o) for _, o, _ in jobs_list]
    need_link = force or not OUT_LIB.exists() or any(
        Path(o).stat().st_mtime > OUT_LIB.stat().st_mtime for o in objs)
    if need_link:
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(OUT_LIB), *objs]
        for d in libdirs:
            link += [f"-L{d}", f"-Wl,-rpath,{d}"]
        link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lamdhip64"]
        _run(link)
        if verbose:
            print(f"[vinf build] linked {OUT_LIB.relative_to(ROOT)}", file=sys.stderr)
    return OUT_LIB


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--save-temps", action="store_true")
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs, debug=a.debug, save_temps=a.save_temps)


if __name__ == "__main__":
    main()
