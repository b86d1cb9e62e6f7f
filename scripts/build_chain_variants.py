#!/usr/bin/env python3
"""Compile-time variants of one kernel file for same-box A/B runs: lstm_chain.hip (default, or the
file named by --src=<stem>) rebuilt with extra -D definitions (ring depths / start leads, see the
#ifndef block at the top of the file), linked with the other objects of the normal build into
gnnqc/_lib/variants/<name>.so. Select one with GNNQC_HIP_LIB=<path> (gnnqc.utils.native). Run
`python -m gnnqc.build` first.

    python scripts/build_chain_variants.py lead1="-DCHAIN_LEAD1=1 -DCHAINB_LEAD=1" d4="-DCHAIN_D=4"
    python scripts/build_chain_variants.py --src=lstm_tm d6="-DTMW_D=6"
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv):
    from gnnqc.build import ARCH, BUILD_DIR, CSRC, LIB_DIR, _torch_flags
    cflags, ldflags = _torch_flags()
    stem = "lstm_chain"
    if argv and argv[0].startswith("--src="):
        stem, argv = argv[0].split("=", 1)[1], argv[1:]
    src = os.path.join(CSRC, "kernels", f"{stem}.hip")
    others = [o for o in sorted(glob.glob(os.path.join(BUILD_DIR, "*.hip.o"))) if not o.endswith(f"{stem}.hip.o")]
    out_dir = os.path.join(LIB_DIR, "variants")
    os.makedirs(out_dir, exist_ok=True)
    specs = [a.split("=", 1) for a in argv]

    def one(spec):
        name, defs = spec
        obj = os.path.join(BUILD_DIR, f"{stem}.{name}.o")
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
               "-munsafe-fp-atomics", f"-I{os.path.join(CSRC, 'kernels')}", *defs.split(), *cflags, "-c", src, "-o", obj]
        subprocess.run(cmd, check=True)
        lib = os.path.join(out_dir, f"{name}.so")
        subprocess.run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", *others, obj, "-o", lib, *ldflags],
                       check=True)
        return lib

    with cf.ThreadPoolExecutor(max_workers=len(specs)) as ex:
        for lib in ex.map(one, specs):
            print("built", lib)


if __name__ == "__main__":
    main(sys.argv[1:])
