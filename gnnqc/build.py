"""Build the native libraries in-tree (no JIT cache, no hipify).

    python -m gnnqc.build            # host lib + gfx950 HIP lib
    python -m gnnqc.build --host     # host lib only

* ``csrc/host/*.cpp``    -> ``gnnqc/_lib/libgnnqc_host.so``  (g++, C ABI, ctypes)
* ``csrc/kernels/*.hip`` -> ``gnnqc/_lib/libgnnqc_hip.so``   (hipcc --offload-arch=gfx950,
  torch op registration through ``TORCH_LIBRARY``; linked against the libtorch of the
  running interpreter)

Objects are compiled in parallel and only rebuilt when a source or header changed.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
LIB_DIR = os.path.join(ROOT, "gnnqc", "_lib")
BUILD_DIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("GNNQC_ARCH", "gfx950")


def _hash_files(paths):
    h = hashlib.sha1()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build_host(verbose=False) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    out = os.path.join(LIB_DIR, "libgnnqc_host.so")
    stamp = out + ".sha1"
    digest = _hash_files(srcs + [__file__])
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == digest:
        return out
    cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-msse4.2", *srcs, "-o", out]
    if verbose:
        print(" ".join(cmd))
    _run(cmd)
    with open(stamp, "w") as f:
        f.write(digest)
    return out


def _torch_flags():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    libdir = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
                                          "-D__HIP_PLATFORM_AMD__=1"]
    ldflags = [f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
               f"-Wl,-rpath,{libdir}"]
    return cflags, ldflags


def build_hip(verbose=False, jobs=None) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    os.makedirs(BUILD_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    headers = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    if not srcs:
        raise RuntimeError("no HIP sources found")
    cflags, ldflags = _torch_flags()
    # GNNQC_CHAIN_PROF_BUILD=1: compile the chain kernels' per-step phase clocks in (diagnostics
    # only: scripts/chain_phase_prof.py; they slow the chain launches when compiled in)
    prof = ["-DGQ_CHAIN_PROF"] if os.environ.get("GNNQC_CHAIN_PROF_BUILD", "0") == "1" else []
    hdr_digest = _hash_files(headers + [__file__]) + ("prof" if prof else "")
    common = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
              "-munsafe-fp-atomics", f"-I{os.path.join(CSRC, 'kernels')}", *prof, *cflags]

    def compile_one(src):
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        stamp = obj + ".sha1"
        digest = _hash_files([src]) + hdr_digest
        if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == digest:
            return obj, False
        cmd = common + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
        with open(stamp, "w") as f:
            f.write(digest)
        return obj, True

    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", "8")), 8)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(compile_one, srcs))
    objs = [o for o, _ in results]
    out = os.path.join(LIB_DIR, "libgnnqc_hip.so")
    if any(rebuilt for _, rebuilt in results) or not os.path.exists(out):
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out, *ldflags]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    return out


def build_all(verbose=False, host_only=False):
    outs = [build_host(verbose)]
    if not host_only:
        outs.append(build_hip(verbose))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", action="store_true", help="build only the host library")
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args(argv)
    for p in build_all(args.verbose, args.host):
        print("built", p)


if __name__ == "__main__":
    sys.exit(main())
