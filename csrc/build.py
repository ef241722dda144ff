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
ARCH = "gfx950"   # MI355X (CDNA4) only


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
          save_temps: bool = False, verbose: bool = True, variant: str = "",
          defines: list[str] | None = None, asan: bool = False) -> Path:
    """Build the library. ``variant`` builds ``libvinf_hip_<variant>.so`` from its own object
    directory (A/B experiments, loaded with ``VINF_NATIVE_LIB``); ``defines`` adds ``-D`` macros
    to the kernel units; ``asan`` instruments the HOST code only (``-Xarch_host
    -fsanitize=address``; device code is never sanitized on this pool) - run it with the
    ASan runtime preloaded (``tools/asan_run.sh``)."""
    hipcc = _hipcc()
    incs, libdirs, abi = _torch_paths()
    if asan and not variant:
        variant = "asan"
    obj_dir = OBJ_DIR / variant if variant else OBJ_DIR
    out_lib = OUT_DIR / f"libvinf_hip_{variant}.so" if variant else OUT_LIB
    obj_dir.mkdir(parents=True, exist_ok=True)
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    headers = _headers()
    opt = ["-O0", "-g"] if debug else ["-O3"]
    common = ["-std=c++17", "-fPIC", f"-I{CSRC / 'include'}", "-Wno-unused-result",
              "-Wno-deprecated-declarations"] + [f"-D{d}" for d in (defines or [])]
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-g"] \
        if asan else []
    kernel_flags = common + opt + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"] + san
    if save_temps:
        kernel_flags += ["-save-temps=obj"]
    bind_flags = common + ["-O1" if asan else "-O2", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
                           f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                           "-DTORCH_API_INCLUDE_EXTENSION_H"] + [f"-I{p}" for p in incs] + san
    jobs_list = []
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        obj = obj_dir / (src.stem + ".o")
        jobs_list.append((src, obj, [hipcc, "-c", *kernel_flags, "-o", str(obj), str(src)]))
    for src in sorted((CSRC / "bindings").glob("*.cpp")):
        obj = obj_dir / ("bind_" + src.stem + ".o")
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
    need_link = force or not out_lib.exists() or any(
        Path(o).stat().st_mtime > out_lib.stat().st_mtime for o in objs)
    if need_link:
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(out_lib), *objs]
        if asan:
            link += ["-fsanitize=address", "-shared-libasan"]
        for d in libdirs:
            link += [f"-L{d}", f"-Wl,-rpath,{d}"]
        link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lamdhip64"]
        _run(link)
        if verbose:
            print(f"[vinf build] linked {out_lib.relative_to(ROOT)}", file=sys.stderr)
    return out_lib


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--save-temps", action="store_true")
    ap.add_argument("--variant", default="", help="build libvinf_hip_<variant>.so")
    ap.add_argument("-D", dest="defines", action="append", default=[],
                    help="extra preprocessor define for the kernel units (repeatable)")
    ap.add_argument("--asan", action="store_true",
                    help="AddressSanitizer on the host code (bindings + launchers) only")
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs, debug=a.debug, save_temps=a.save_temps,
          variant=a.variant, defines=a.defines, asan=a.asan)


if __name__ == "__main__":
    main()
