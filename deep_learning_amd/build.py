"""Builds the in-tree HIP C-ABI library ``deep_learning_amd/libdlamd.so`` for gfx950.

``python -m deep_learning_amd.build`` (also called by ``__graft_entry__.build()``).
Sources are compiled in parallel with hipcc and linked against RCCL; objects go
to ``deep_learning_amd/_build/`` and are rebuilt only when a source or header is
newer than its object.
"""
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
# DLAMD_VARIANT=name builds an experiment variant (extra -D flags from DLAMD_DEFINES)
# into libdlamd_<name>.so with its own object directory; the default build is untouched.
VARIANT = os.environ.get("DLAMD_VARIANT", "")
OUT = os.path.join(HERE, "libdlamd%s.so" % ("_" + VARIANT if VARIANT else ""))
OBJ = os.path.join(HERE, "_build" + ("_" + VARIANT if VARIANT else ""))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DLAMD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-munsafe-fp-atomics",
         "-Wno-unused-result", "-I" + os.path.join(ROOT, "include")] + \
    (["-D" + d for d in os.environ.get("DLAMD_DEFINES", "").split()] if VARIANT else [])


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(ROOT, "include", "dlamd.h"))
    return hs


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    newest = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if os.path.exists(obj) and os.path.getmtime(obj) >= newest:
        return obj
    cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include"), "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, r.stdout, r.stderr))
    return obj


HOST_SRCS = [os.path.join(HERE, "csrc_host", f) for f in ("dlio.cpp", "dlpk.cpp")]
HOST_OUT = os.path.join(HERE, "libdlio.so")


def build_host(verbose=True):
    """The native TFRecord reader and load-style batch decoder (include/dlio.h): plain host C++,
    g++, no GPU code."""
    deps = HOST_SRCS + [os.path.join(ROOT, "include", "dlio.h")]
    if os.path.exists(HOST_OUT) and os.path.getmtime(HOST_OUT) >= max(os.path.getmtime(d) for d in deps):
        return HOST_OUT
    cmd = [os.environ.get("CXX", "g++"), "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall",
           "-I" + os.path.join(ROOT, "include")] + HOST_SRCS + ["-o", HOST_OUT]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("g++ failed for %s:\n%s\n%s" % (HOST_SRCS, r.stdout, r.stderr))
    if verbose:
        print("built", HOST_OUT)
    return HOST_OUT


def build(verbose=True):
    if not VARIANT:
        build_host(verbose)
    os.makedirs(OBJ, exist_ok=True)
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(o) for o in objs):
        return OUT
    cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", OUT] + objs + [
        "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s\n%s" % (r.stdout, r.stderr))
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build()
    sys.exit(0)
