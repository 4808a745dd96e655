#!/usr/bin/env python3
"""In-tree, incremental builder of the framework's native extensions (no hipify, no JIT cache).

    python build_native.py            # build what changed
    python build_native.py --clean    # rebuild everything

Produces, next to the Python sources (so they ship with the repo snapshot to the GPU box):

* ``tensorflow_distributed_learning_amd/_C*.so``      hand-written gfx950 HIP kernels + bindings.
  ``.hip`` files are compiled by ``hipcc --offload-arch=gfx950`` directly (CDNA4 only);
  binding ``.cpp`` files by the host C++ compiler against the torch headers.
* ``tensorflow_distributed_learning_amd/_native*.so`` C++ runtime (rendezvous/KV store,
  TCP ring all-reduce, host data helpers); pure host C++, builds without ROCm.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = "tensorflow_distributed_learning_amd"
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build", "native")
ARCH = os.environ.get("TDL_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_flags():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [
        os.path.join(tdir, "include"),
        os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
        sysconfig.get_paths()["include"],
    ]
    abi = int(getattr(torch._C, "_GLIBCXX_USE_CXX11_ABI", 1))
    return inc, os.path.join(tdir, "lib"), abi


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _newest_header():
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _stale(src, obj, hdr_mtime):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or hdr_mtime > t


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n  " + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _compile_all(jobs, nproc):
    if not jobs:
        return
    with cf.ThreadPoolExecutor(max_workers=nproc) as ex:
        futs = {ex.submit(_run, cmd): out for cmd, out in jobs}
        for f in cf.as_completed(futs):
            f.result()
            print(f"  built {os.path.relpath(futs[f], HERE)}", flush=True)


def build_hip_ext(nproc, verbose=False):
    inc, tlib, abi = _torch_flags()
    hdr = _newest_header()
    odir = os.path.join(BUILD, "_C")
    os.makedirs(odir, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{CSRC}", f"-I{ROCM}/include"]
    # diagnostics builds (A/B variants of a kernel): extra device-compile flags, e.g. "-DTDL_W3_SCHED"
    # (touch the source or --clean when switching: objects are rebuilt by modification time only)
    extra = os.environ.get("TDL_EXTRA_HIPFLAGS", "").split()
    jobs, objs = [], []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        objs.append(obj)
        if _stale(src, obj, hdr):
            jobs.append(([hipcc, "-c", "-x", "hip", f"--offload-arch={ARCH}", "-fno-gpu-rdc", *common, *extra, src, "-o", obj], obj))
    host_defs = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C"]
    for src in [os.path.join(CSRC, n) for n in ("bindings.cpp", "ops_bindings.cpp", "comm_bindings.cpp", "rccl_comm.cpp")]:
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        objs.append(obj)
        if _stale(src, obj, hdr):
            jobs.append((["c++", "-c", *common, *host_defs, *[f"-I{i}" for i in inc], src, "-o", obj], obj))
    _compile_all(jobs, nproc)
    out = os.path.join(HERE, PKG, "_C" + _ext_suffix())
    if jobs or not os.path.exists(out):
        _run(["c++", "-shared", "-o", out, *objs, f"-L{tlib}", f"-L{ROCM}/lib", f"-Wl,-rpath,{tlib}",
              "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip", "-lamdhip64"])
        print(f"  linked {os.path.relpath(out, HERE)}", flush=True)
    return out


def build_native_ext(nproc):
    inc, tlib, abi = _torch_flags()
    hdr = _newest_header()
    srcs = sorted(glob.glob(os.path.join(CSRC, "native", "*.cpp")))
    if not srcs:
        return None
    odir = os.path.join(BUILD, "_native")
    os.makedirs(odir, exist_ok=True)
    flags = ["-O3", "-std=c++17", "-fPIC", "-pthread", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{CSRC}",
             "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_native", *[f"-I{i}" for i in inc]]
    jobs, objs = [], []
    for src in srcs:
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        objs.append(obj)
        if _stale(src, obj, hdr):
            jobs.append((["c++", "-c", *flags, src, "-o", obj], obj))
    _compile_all(jobs, nproc)
    out = os.path.join(HERE, PKG, "_native" + _ext_suffix())
    if jobs or not os.path.exists(out):
        _run(["c++", "-shared", "-pthread", "-o", out, *objs, f"-L{tlib}", f"-Wl,-rpath,{tlib}",
              "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python"])
        print(f"  linked {os.path.relpath(out, HERE)}", flush=True)
    return out


def build_selftest(sanitize: str) -> str:
    """Standalone C++ self-test of the runtime (csrc/native/tests/native_selftest.cpp + store.cpp +
    ring.cpp) under a sanitizer: ``address`` = ASan + UBSan, ``thread`` = TSan (race detection).
    Host code only (GPU sanitizers are not used on this pool)."""
    odir = os.path.join(BUILD, "selftest")
    os.makedirs(odir, exist_ok=True)
    srcs = [os.path.join(CSRC, "native", "tests", "native_selftest.cpp"),
            os.path.join(CSRC, "native", "store.cpp"), os.path.join(CSRC, "native", "ring.cpp")]
    out = os.path.join(odir, f"native_selftest_{sanitize}")
    newest = max([os.path.getmtime(x) for x in srcs] + [_newest_header()])
    if os.path.exists(out) and os.path.getmtime(out) >= newest:
        return out
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"] if sanitize == "address" \
        else ["-fsanitize=thread"]
    # ROCm's clang: its TSan runtime intercepts pthread_cond_clockwait (what libstdc++'s
    # condition_variable::wait_for calls); GCC 11's does not and reports false double locks
    cxx = os.path.join(ROCM, "llvm", "bin", "clang++")
    if not os.path.exists(cxx):
        cxx = "c++"
    _run([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", *san, f"-I{CSRC}", *srcs,
          "-o", out])
    print(f"  built {os.path.relpath(out, HERE)}", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--sanitize", choices=["address", "thread"], default=None,
                    help="build only the sanitizer self-test binary of the C++ runtime")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--only", choices=["hip", "native"], default=None)
    args = ap.parse_args(argv)
    if args.clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    if args.sanitize:
        print(build_selftest(args.sanitize))
        return 0
    if args.only in (None, "native"):
        build_native_ext(args.j)
    if args.only in (None, "hip"):
        build_hip_ext(args.j)


if __name__ == "__main__":
    sys.exit(main())
