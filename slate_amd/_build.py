"""In-tree native build of slate_amd's extensions.

Two pybind11 extension modules are produced next to this file:

* ``_hip.so``  -- every CDNA4 kernel, compiled by ``hipcc --offload-arch=gfx950``
  (one translation unit per kernel family/dtype so builds run in parallel).
* ``_host.so`` -- the native host runtime (tile/MOSI table, slab memory pool,
  trace recorder, Philox matrix generator, host tile kernels for the
  ``Target.Host*`` CPU path), compiled by ``g++ -fopenmp``.

Objects are cached under ``build/`` and rebuilt when a source or any header
of the same directory is newer.  Used by ``__graft_entry__.build()``,
``setup.py`` and ``python slate_amd/_build.py``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
BUILD = os.path.join(ROOT, "build")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"


def _pybind_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _jobs():
    for k in ("MAX_JOBS", "CMAKE_BUILD_PARALLEL_LEVEL"):
        if os.environ.get(k, "").isdigit():
            return max(1, min(16, int(os.environ[k])))
    return max(1, min(16, os.cpu_count() or 4))


def _build_module(name, srcdir, exts, compiler, cflags, ldflags, verbose=False, extra_objs=(), extra_deps=()):
    srcs = sorted(sum((glob.glob(os.path.join(srcdir, "*" + e)) for e in exts), []))
    headers = (glob.glob(os.path.join(srcdir, "*.hpp")) + glob.glob(os.path.join(HERE, "csrc", "include", "*.hpp"))
               + list(extra_deps))
    objdir = os.path.join(BUILD, name)
    os.makedirs(objdir, exist_ok=True)
    ext_suffix = ".so"
    target = os.path.join(HERE, name + ext_suffix)
    # a change of compiler flags rebuilds every object of the module
    stamp = os.path.join(objdir, ".flags")
    flags = " ".join([compiler] + cflags)
    old_flags = open(stamp).read() if os.path.exists(stamp) else None
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if old_flags != flags or _newer(o, [s] + headers):
            todo.append((s, o))

    def compile_one(so):
        s, o = so
        cmd = [compiler] + cflags + ["-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        return o

    if todo:
        with cf.ThreadPoolExecutor(_jobs()) as ex:
            for f in [ex.submit(compile_one, so) for so in todo]:
                f.result()
    objs = objs + list(extra_objs)
    if todo or _newer(target, objs):
        _run([compiler] + ["-shared", "-o", target] + objs + ldflags)
    if old_flags != flags:
        with open(stamp, "w") as f:
            f.write(flags)
    return target


def _host_arch_flags():
    """Host ISA: portable by default (the module must load on any x86-64
    host); SLATE_AMD_HOST_MARCH=x86-64-v3 (or native) opts in to AVX2 code.
    Complex arithmetic keeps the full C99 semantics (no -fcx-limited-range:
    the naive forms overflow / underflow past |x| ~ 1e154, which the tester's
    _ofl/_ufl matrix scalings exercise)."""
    m = os.environ.get("SLATE_AMD_HOST_MARCH", "")
    return ["-march=" + m] if m else []


def build(verbose=False, hip=True, host=True):
    inc = ["-I" + p for p in _pybind_includes()] + ["-I" + os.path.join(HERE, "csrc", "include")]
    out = []
    if host:
        out.append(_build_module(
            "_host", os.path.join(HERE, "csrc", "host"), [".cpp"], "g++",
            ["-O3", "-std=c++17", "-fPIC", "-fopenmp", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]
            + _host_arch_flags() + inc,
            ["-fopenmp"], verbose))
    if host:
        # C ABI (include/slate_amd/c_api.h): embeds the Python runtime
        pyinc = sysconfig.get_paths()["include"]
        libdir = sysconfig.get_config_var("LIBDIR") or "/usr/lib"
        pylib = "python" + sysconfig.get_config_var("LDVERSION")
        out.append(_build_module(
            "libslate_amd_c", os.path.join(HERE, "csrc", "capi"), [".cpp"], "g++",
            ["-O2", "-std=c++17", "-fPIC", "-I" + pyinc],
            ["-L" + libdir, "-l" + pylib], verbose))
    if hip:
        hipcc = os.path.join(ROCM, "bin", "hipcc")
        out.append(_build_module(
            "_hip", os.path.join(HERE, "csrc", "hip"), [".hip"], hipcc,
            ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
             "-x", "hip"] + inc,
            ["--offload-arch=" + ARCH, "-L" + os.path.join(ROCM, "lib"), "-lamdhip64"], verbose))
        # Python-free native library (include/slate_amd/slate_native.hh): the
        # same kernel objects (minus the pybind11 units) + the C++ host
        # runtime / drivers of csrc/native, linked against HIP and RCCL only
        kobjs = [o for o in sorted(glob.glob(os.path.join(BUILD, "_hip", "*.hip.o")))
                 if os.path.basename(o) not in ("bindings.hip.o", "devpool.hip.o")]
        out.append(_build_module(
            "libslate_amd_native", os.path.join(HERE, "csrc", "native"), [".hip"], hipcc,
            ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-x", "hip",
             "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROCM, "include")],
            ["--offload-arch=" + ARCH, "-L" + os.path.join(ROCM, "lib"), "-lamdhip64", "-lrccl",
             "-Wl,-rpath," + os.path.join(ROCM, "lib")], verbose, extra_objs=kobjs,
            extra_deps=glob.glob(os.path.join(ROOT, "include", "slate_amd", "*.hh"))
            + glob.glob(os.path.join(HERE, "csrc", "hip", "*.hpp"))))
        out.append(_build_native_example(verbose))
        out.append(_build_native_example(verbose, "bench_native"))
        # the header-only C++ API (slate_amd.hh) over the NATIVE handle C API
        out.append(_build_native_example(verbose, "ex_cpp_api_native", "ex_cpp_api"))
        out.append(_build_native_c_example(verbose))
        out.append(_build_native_c_example(verbose, "ex_native_lapack"))
        out.append(_build_native_c_example(verbose, "ex_native_handles"))
    return out


def _build_native_example(verbose=False, name="ex_native", src_name=None):
    """examples/cpp/<name>.cc -> slate_amd/<name>: a plain g++ C++17
    program against include/slate_amd/slate_native.hh and
    libslate_amd_native.so (rpath $ORIGIN), no Python.  Built in-tree next
    to the library so it travels to the GPU box with the snapshot
    (ex_native: the example / tests; bench_native: bench.py --impl native)."""
    src = os.path.join(ROOT, "examples", "cpp", (src_name or name) + ".cc")
    lib = os.path.join(HERE, "libslate_amd_native.so")
    target = os.path.join(HERE, name)
    hdr = os.path.join(ROOT, "include", "slate_amd", "slate_native.hh")
    if _newer(target, [src, lib, hdr]):
        cmd = ["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"), src, "-o", target,
               "-L" + HERE, "-lslate_amd_native", "-Wl,-rpath,$ORIGIN"]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
    return target


def _build_native_c_example(verbose=False, name="ex_native_scalapack"):
    """examples/c/<name>.c -> slate_amd/<name>: a plain C program calling the
    ScaLAPACK / BLACS / LAPACK / handle symbols of libslate_amd_native.so (no
    Python, no MPI)."""
    src = os.path.join(ROOT, "examples", "c", name + ".c")
    lib = os.path.join(HERE, "libslate_amd_native.so")
    target = os.path.join(HERE, name)
    if _newer(target, [src, lib]):
        cmd = ["gcc", "-O2", "-std=gnu11", src, "-o", target, "-I" + os.path.join(ROOT, "include"),
               "-L" + HERE, "-lslate_amd_native", "-lm",
               "-Wl,-rpath,$ORIGIN"]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
    return target


if __name__ == "__main__":
    for t in build(verbose="-v" in sys.argv):
        print("built", t)
