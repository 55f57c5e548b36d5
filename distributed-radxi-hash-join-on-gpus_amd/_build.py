"""In-tree native build: hipcc for gfx950, no JIT cache, no hipify.

Produces (all git-ignored, but shipped to the GPU box by gpurun):
  _C<EXT_SUFFIX>          the pybind11 module (core + kernels + bindings)
  build/bin/hjoin_bench   standalone C++ CLI (no Python/torch), the analog of
                          the reference's `program` (/root/reference/main.cpp)

Objects are cached by a hash of (source, every header, flags), so rebuilding
after touching one kernel recompiles one file.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG / "build"
ARCH = os.environ.get("HPCJOIN_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
             "-Wno-unused-variable", "-Wno-unused-result"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-Wno-unused-result"]


def _torch_paths():
    import torch  # noqa: F401  (only for include/lib locations)
    from torch.utils import cpp_extension as ce
    tdir = Path(torch.__file__).resolve().parent
    incs = [str(tdir / "include"), str(tdir / "include" / "torch" / "csrc" / "api" / "include")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, str(tdir / "lib"), abi


def _sources():
    core, kernels, bindings = [], [], []
    for p in sorted(CSRC.rglob("*")):
        if p.suffix == ".hip":
            kernels.append(p)
        elif p.suffix == ".cpp":
            if p.parent.name == "bindings":
                bindings.append(p)
            elif p.parent.name == "apps":
                continue
            else:
                core.append(p)
    return core, kernels, bindings


def _header_digest() -> str:
    h = hashlib.sha1()
    for p in sorted(CSRC.rglob("*.h")):
        h.update(p.read_bytes())
    return h.hexdigest()


def _obj(src: Path, flags, hdr: str) -> Path:
    h = hashlib.sha1(src.read_bytes() + hdr.encode() + " ".join(flags).encode()).hexdigest()[:16]
    rel = str(src.relative_to(CSRC)).replace("/", "_")
    return BUILD / "obj" / f"{rel}.{h}.o"


def _run(cmd, verbose=False):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def ext_path() -> Path:
    return PKG / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def build(jobs: int | None = None, verbose: bool = False, with_cli: bool = True) -> Path:
    jobs = jobs or min(16, os.cpu_count() or 4)
    (BUILD / "obj").mkdir(parents=True, exist_ok=True)
    (BUILD / "bin").mkdir(parents=True, exist_ok=True)
    hdr = _header_digest()
    core, kernels, bindings = _sources()
    tinc, tlib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    common_defs = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    jobs_list = []
    extra = os.environ.get("HPCJOIN_EXTRA_HIPFLAGS", "").split()  # profiling builds (e.g. -DHPCJOIN_SCATTER_PROF)
    for s in kernels:
        f = HIP_FLAGS + common_defs + extra
        jobs_list.append((s, [HIPCC, *f, "-c", str(s)], f))
    for s in core:
        f = CXX_FLAGS + common_defs
        jobs_list.append((s, [HIPCC, *f, "-c", str(s)], f))
    bind_flags = CXX_FLAGS + common_defs + ["-D__HIP_PLATFORM_AMD__", "-DTORCH_EXTENSION_NAME=_C",
                                            "-DTORCH_API_INCLUDE_EXTENSION_H", f"-I{ROCM}/include",
                                            f"-I{py_inc}"] + [f"-I{i}" for i in tinc]
    for s in bindings:
        jobs_list.append((s, ["g++", *bind_flags, "-c", str(s)], bind_flags))

    def compile_one(item):
        src, cmd, flags = item
        obj = _obj(src, flags, hdr)
        if not obj.exists():
            tmp = obj.with_suffix(".tmp.o")
            _run(cmd + ["-o", str(tmp)], verbose)
            tmp.rename(obj)
        return src, obj

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = dict(ex.map(compile_one, jobs_list))

    # drop objects of older source/header versions (keeps the gpurun snapshot small)
    keep = {o.name for o in objs.values()}
    for stale in (BUILD / "obj").glob("*.o"):
        if stale.name not in keep and not stale.name.startswith("apps_"):
            stale.unlink()
    core_objs = [str(objs[s]) for s in core + kernels]
    bind_objs = [str(objs[s]) for s in bindings]
    out = ext_path()
    tmp_out = out.with_name(out.name + ".tmp")
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *core_objs, *bind_objs, "-o", str(tmp_out),
          f"-L{tlib}", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10", f"-Wl,-rpath,{tlib}",
          f"-L{ROCM}/lib", "-lrccl", "-lrocprofiler-sdk-roctx", "-lamdhip64"], verbose)
    os.replace(tmp_out, out)

    if with_cli:
        cli_src = CSRC / "apps" / "hjoin_bench.cpp"
        f = CXX_FLAGS + common_defs
        cli_obj = _obj(cli_src, f, hdr)
        if not cli_obj.exists():
            _run([HIPCC, *f, "-c", str(cli_src), "-o", str(cli_obj)], verbose)
        _run([HIPCC, f"--offload-arch={ARCH}", str(cli_obj), *core_objs, "-o", str(BUILD / "bin" / "hjoin_bench"),
              f"-L{ROCM}/lib", "-lrccl", "-lrocprofiler-sdk-roctx", "-lamdhip64", "-lpthread"], verbose)
    return out


SANITIZERS = {
    # host code only: GPU sanitizers are not available on the MI355X pool
    "address": ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined"],
    "thread": ["-Xarch_host", "-fsanitize=thread"],
}


def build_sanitized(kind: str = "address", jobs: int | None = None, verbose: bool = False) -> Path:
    """Host self-test (csrc/apps/host_selftest.cpp) with the runtime compiled
    under ASan+UBSan ("address") or TSan ("thread").  Kernels are linked
    unsanitized (they never run on this path)."""
    jobs = jobs or min(16, os.cpu_count() or 4)
    san = SANITIZERS[kind]
    odir = BUILD / f"san-{kind}"
    odir.mkdir(parents=True, exist_ok=True)
    hdr = _header_digest()
    core, kernels, _ = _sources()
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-std=c++17", "-fPIC", *san]
    srcs = core + [CSRC / "apps" / "host_selftest.cpp"]

    def compile_one(src):
        h = hashlib.sha1(src.read_bytes() + hdr.encode() + " ".join(flags).encode()).hexdigest()[:16]
        obj = odir / f"{str(src.relative_to(CSRC)).replace('/', '_')}.{h}.o"
        if not obj.exists():
            _run([HIPCC, *flags, "-c", str(src), "-o", str(obj) + ".tmp"], verbose)
            os.replace(str(obj) + ".tmp", obj)
        return obj

    kflags = HIP_FLAGS + ["-D_GLIBCXX_USE_CXX11_ABI=1"]

    def compile_kernel(src):
        # The kernels are not sanitized: the main build's object of the same
        # source, headers and flags is reused when it exists (a gfx950 compile
        # of partition.hip takes minutes).
        main = _obj(src, kflags, hdr)
        if main.exists():
            return main
        obj = odir / f"{str(src.relative_to(CSRC)).replace('/', '_')}.{hashlib.sha1(src.read_bytes() + hdr.encode()).hexdigest()[:16]}.k.o"
        if not obj.exists():
            _run([HIPCC, *kflags, "-c", str(src), "-o", str(obj) + ".tmp"], verbose)
            os.replace(str(obj) + ".tmp", obj)
        return obj

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs)) + list(ex.map(compile_kernel, kernels))
    link_san = ["-fsanitize=address,undefined"] if kind == "address" else ["-fsanitize=thread"]
    out = BUILD / "bin" / f"host_selftest_{kind}"
    (BUILD / "bin").mkdir(parents=True, exist_ok=True)
    _run([HIPCC, f"--offload-arch={ARCH}", "-fno-gpu-sanitize", *link_san, *map(str, objs), "-o", str(out),
          f"-L{ROCM}/lib", "-lrccl", "-lrocprofiler-sdk-roctx", "-lamdhip64", "-lpthread"], verbose)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "sanitize":
        print(build_sanitized(sys.argv[2], verbose="-v" in sys.argv))
        sys.exit(0)
    p = build(verbose="-v" in sys.argv)
    print(p)
