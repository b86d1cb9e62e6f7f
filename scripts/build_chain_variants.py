#!/usr/bin/env python3
"""Compile-time variants of the chain kernels for same-box A/B runs: lstm_chain.hip rebuilt with
extra -D definitions (ring depths / start leads, see the #ifndef block at the top of the file),
linked with the other objects of the normal build into gnnqc/_lib/variants/<name>.so. Select one with
GNNQC_HIP_LIB=<path> (gnnqc.utils.native). Run `python -m gnnqc.build` first.

    python scripts/build_chain_variants.py lead1="-DCHAIN_LEAD1=1 -DCHAINB_LEAD=1" d4="-DCHAIN_D=4"
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
    src = os.path.join(CSRC, "kernels", "lstm_chain.hip")
    others = [o for o in sorted(glob.glob(os.path.join(BUILD_DIR, "*.hip.o"))) if not o.endswith("lstm_chain.hip.o")]
    out_dir = os.path.join(LIB_DIR, "variants")
    os.makedirs(out_dir, exist_ok=True)
    specs = [a.split("=", 1) for a in argv]

    def one(spec):
        name, defs = spec
        obj = os.path.join(BUILD_DIR, f"lstm_chain.{name}.o")
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
