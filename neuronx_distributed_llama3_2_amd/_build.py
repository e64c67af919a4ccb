"""In-tree build of the CDNA4 extension `_C` (hipcc --offload-arch=gfx950, no hipify, no JIT cache).

Every `csrc/*.hip` file is a self-contained kernel translation unit (HIP runtime headers only, so
each compiles in seconds); the `csrc/*.cpp` host TUs (pybind bindings, the hipBLASLt GEMM tuner)
are the only ones that include the torch headers.
Objects are cached under `build/` keyed on source + header mtimes and compiled in parallel, then
linked into `neuronx_distributed_llama3_2_amd/_C*.so` next to this file, so the built library
travels with the source tree (e.g. to a GPU box) and is what `import` loads.

Usage:  python -m neuronx_distributed_llama3_2_amd._build [--force] [--jobs N]
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR.parent / "build" / "nxd_csrc"
ARCH = os.environ.get("NXD_OFFLOAD_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
LIB_PATH = PKG_DIR / ("_C" + EXT_SUFFIX)


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    return os.path.join(rocm, "bin", "hipcc")


def _torch_flags():
    import torch

    tdir = Path(torch.__file__).resolve().parent
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    inc = [
        f"-I{os.path.join(rocm, 'include')}",
        f"-I{tdir / 'include'}",
        f"-I{tdir / 'include' / 'torch' / 'csrc' / 'api' / 'include'}",
        f"-I{sysconfig.get_paths()['include']}",
    ]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = [
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
    ]
    libdir = tdir / "lib"
    libs = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip",
            "-ltorch_hip", "-lamdhip64", "-lhipblaslt", "-ldl"]
    return inc, defs, libs


# per-TU extra flags.  flash_attn_bwd: without VGPR-form MFMAs the allocator gives the short S/dP
# chains AGPRs and spills two of the 16 resident dK/dV accumulator tiles to scratch every tile.
_EXTRA_FLAGS = {"flash_attn_bwd": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _needs_build(src: Path, obj: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(p.stat().st_mtime > t for p in [src, *deps])


def _compile(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    return r.returncode, r.stdout, cmd


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    if not os.path.exists(hipcc):
        raise RuntimeError(f"hipcc not found at {hipcc}")
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.h"))
    kernels = sorted(CSRC.glob("*.hip"))
    inc, defs, libs = _torch_flags()
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-fno-gpu-rdc", f"-I{CSRC}",
              "-Wno-unused-result", "-Wno-unused-variable"]
    jobs_list = []
    objs = []
    for src in kernels:
        obj = BUILD_DIR / (src.stem + ".o")
        objs.append(obj)
        if force or _needs_build(src, obj, headers):
            jobs_list.append([hipcc, *common, *_EXTRA_FLAGS.get(src.stem, []), "-c", str(src), "-o", str(obj)])
    # host-side C++ translation units that include the torch headers (bindings, hipBLASLt tuner)
    for src in sorted(CSRC.glob("*.cpp")):
        obj = BUILD_DIR / (src.stem + ".o")
        objs.append(obj)
        if force or _needs_build(src, obj, headers):
            jobs_list.append([hipcc, "-x", "hip", *common, *inc, *defs, "-c", str(src), "-o", str(obj)])
    jobs = jobs or min(8, os.cpu_count() or 4, 16)
    failures = []
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for rc, out, cmd in ex.map(_compile, jobs_list):
                if verbose or rc != 0:
                    sys.stderr.write(out)
                if rc != 0:
                    failures.append(" ".join(cmd))
    if failures:
        raise RuntimeError("HIP compilation failed:\n" + "\n".join(failures))
    if force or jobs_list or not LIB_PATH.exists() or any(o.stat().st_mtime > LIB_PATH.stat().st_mtime for o in objs):
        tmp = LIB_PATH.with_suffix(".tmp.so")
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-fno-gpu-rdc", *map(str, objs), "-o", str(tmp), *libs]
        rc, out, _ = _compile(cmd)
        if rc != 0:
            sys.stderr.write(out)
            raise RuntimeError("link failed: " + " ".join(cmd))
        os.replace(tmp, LIB_PATH)
    return LIB_PATH


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    p = build(force=a.force, jobs=a.jobs, verbose=a.verbose)
    print(p)


if __name__ == "__main__":
    main()
