"""In-tree build of the gfx950 HIP extension ``ncnet_amd/_C.so``.

Variants (the sanitizer tier):
* ``release`` (default): ``-O3`` -> ``_C.so``;
* ``debug``: ``-O1 -g -DNCNET_DEBUG=1`` -> ``_C_debug.so``: device-side bounds
  checks (``NCNET_CHECK`` in csrc/common.h) print the failing condition with
  file:line from the kernel instead of silently reading out of range;
* ``asan``: host code (pybind bindings and every launcher) built with
  AddressSanitizer by clang (``-Xarch_host -fsanitize=address``; device code
  unsanitized, GPU ASan is not available here) -> ``_C_asan.so``; run with
  ``LD_PRELOAD=<libclang_rt.asan-x86_64.so> ASAN_OPTIONS=detect_leaks=0``
  (``asan_runtime()`` returns the path).
``NCNET_EXT=debug|asan`` makes ``ops._ext`` import that variant.

Each ``csrc/*.hip`` file is compiled by hipcc for gfx950 only (no torch
headers, so kernels rebuild in seconds); ``bindings.cpp`` is the only
translation unit that includes torch.  Objects are relinked into one shared
library that lives next to the package, so it travels to the GPU box with the
repository snapshot.  Rebuilds are incremental (mtime based).

    python -m ncnet_amd.build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG / "_build"
TARGET = PKG / "_C.so"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("NCNET_OFFLOAD_ARCH", "gfx950")

HIP_FLAGS = [
    "-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-mcode-object-version=5",
    "-ffp-contract=fast", "-Wno-unused-result", "-Wno-unused-variable",
]
# release compiles also emit the compiler's per-kernel resource remarks, kept
# next to the objects (``<stem>.resources.txt``, keyed by resource_key) so
# ncnet_amd.kernel_resources / tests/test_kernel_resources.py read them instead
# of compiling every source a second time
RES_FLAG = "-Rpass-analysis=kernel-resource-usage"


def resource_key(src: Path) -> str:
    """Hash of what a source's device code depends on: its text, every csrc
    header and the compile flags."""
    import hashlib
    h = hashlib.sha256(" ".join(HIP_FLAGS).encode())
    for f in [src, *sorted(CSRC.glob("*.h"))]:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()


def resource_cache(src: Path) -> Path:
    return BUILD / (src.stem + ".resources.txt")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths()
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, libdir, abi


def _newer(src: Path, dst: Path, deps=()) -> bool:
    if not dst.exists():
        return True
    t = dst.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


VARIANTS = ("release", "debug", "asan")
CLANGXX = os.path.join(ROCM, "lib", "llvm", "bin", "clang++")


def asan_runtime() -> str:
    """The clang AddressSanitizer runtime matching hipcc (LD_PRELOAD it)."""
    import glob
    hits = sorted(glob.glob(os.path.join(ROCM, "lib", "llvm", "lib", "clang", "*", "lib", "linux",
                                         "libclang_rt.asan-x86_64.so")))
    if not hits:
        raise FileNotFoundError("libclang_rt.asan-x86_64.so not found under ROCm's LLVM")
    return hits[-1]


def target_for(variant: str) -> Path:
    return TARGET if variant == "release" else PKG / f"_C_{variant}.so"


def build(force: bool = False, jobs: int | None = None, verbose: bool = False, variant: str = "release") -> Path:
    if variant not in VARIANTS:
        raise ValueError(f"variant must be one of {VARIANTS}")
    bdir = BUILD if variant == "release" else PKG / f"_build_{variant}"
    target = target_for(variant)
    modname = target.stem
    bdir.mkdir(exist_ok=True)
    headers = sorted(CSRC.glob("*.h"))
    hip_srcs = sorted(CSRC.glob("*.hip"))
    inc, libdir, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    hip_flags = list(HIP_FLAGS)
    if variant == "debug":
        hip_flags = [f for f in hip_flags if f != "-O3"] + ["-O1", "-g", "-DNCNET_DEBUG=1"]
    elif variant == "asan":
        hip_flags = [f for f in hip_flags if f != "-O3"] + ["-O1", "-g", "-Xarch_host", "-fsanitize=address",
                                                             "-Xarch_host", "-fno-omit-frame-pointer"]

    steps = []
    objs = []
    remarks = {}                                       # step index -> (cache file, key)
    for src in hip_srcs:
        obj = bdir / (src.stem + ".o")
        objs.append(obj)
        if force or _newer(src, obj, headers) or (variant == "release" and not resource_cache(src).exists()):
            cmd = [HIPCC, *hip_flags, "-I", str(CSRC), "-c", str(src), "-o", str(obj)]
            if variant == "release":
                remarks[len(steps)] = (resource_cache(src), resource_key(src))
                cmd.append(RES_FLAG)
            steps.append(cmd)
    bsrc = CSRC / "bindings.cpp"
    bobj = bdir / "bindings.o"
    objs.append(bobj)
    if force or _newer(bsrc, bobj):
        cxx = ["g++", "-O2"] if variant != "asan" else [CLANGXX, "-O1", "-g", "-fsanitize=address",
                                                        "-fno-omit-frame-pointer"]
        cmd = cxx + ["-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                     f"-DTORCH_EXTENSION_NAME={modname}", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", py_inc,
                     "-I", os.path.join(ROCM, "include"), "-Wno-deprecated-declarations"]
        for p in inc:
            cmd += ["-I", p]
        cmd += ["-c", str(bsrc), "-o", str(bobj)]
        steps.append(cmd)

    if steps:
        jobs = jobs or min(len(steps), max(1, (os.cpu_count() or 4) // 2), 16)
        with cf.ThreadPoolExecutor(jobs) as ex:
            for i, out in enumerate(ex.map(_run, steps)):
                if i in remarks:
                    path, key = remarks[i]
                    lines = [ln for ln in out.splitlines() if RES_FLAG in ln]
                    path.write_text(f"# key {key}\n" + "\n".join(lines) + "\n")
                    out = "\n".join(ln for ln in out.splitlines() if RES_FLAG not in ln)
                if verbose and out.strip():
                    print(out)
    if force or steps or not target.exists() or any(o.stat().st_mtime > target.stat().st_mtime for o in objs):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(target) + ".tmp",
                "-L", libdir, "-Wl,-rpath," + libdir, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
                "-ltorch_hip", "-ltorch_python", "-L", os.path.join(ROCM, "lib"), "-lamdhip64", "-lhipblaslt",
                "-Wl,-rpath," + os.path.join(ROCM, "lib")]
        if variant == "asan":
            link += ["-shared-libasan", "-fsanitize=address"]
        _run(link)
        os.replace(str(target) + ".tmp", target)
    return target


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--variant", choices=VARIANTS, default="release")
    ap.add_argument("--debug", action="store_true", help="same as --variant debug")
    ap.add_argument("--asan", action="store_true", help="same as --variant asan")
    a = ap.parse_args(argv)
    variant = "debug" if a.debug else "asan" if a.asan else a.variant
    out = build(force=a.force, jobs=a.j, verbose=a.v, variant=variant)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
