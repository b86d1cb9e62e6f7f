#!/usr/bin/env python3
"""All-reduce cost of the flat gradient buffer (753 KB) from one GPU: the Trainer's in-graph
collective timed on its own (Trainer.measure_allreduce) for RCCL on a one-rank nccl group (forced
collective), the one-shot peer kernel on the same group, and the peer kernel between two processes
sharing the GPU (handles exchanged over gloo). One JSON line each (the DP worker of
tests/test_dp_gpu.py). Cross-GPU numbers need a multi-GPU node (the driver's scaling run)."""
import json
import os
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    from test_dp_gpu import _run
    base = Path(tempfile.mkdtemp(prefix="ar_us_"))
    cases = [
        ("rccl_1rank_in_graph", 1, "nccl", dict(chain=True, NB="16", GNNQC_DP_FORCE_COLLECTIVE="1")),
        ("peer_1rank_in_graph", 1, "nccl", dict(chain=True, NB="16", GNNQC_DP_FORCE_COLLECTIVE="1",
                                                 GNNQC_PEER_ALLREDUCE="1")),
        ("peer_2rank_same_gpu", 2, "gloo", dict(NB="16", GNNQC_PEER_ALLREDUCE="1")),
    ]
    for name, world, backend, kw in cases:
        res = _run(base / name, world, backend, **kw)
        print(json.dumps({"case": name, "world": world, "backend": backend,
                          "ar_us": [r["ar_us"] for r in res], "peer": [r["peer"] for r in res],
                          "dp_graph": res[0]["dp_graph"], "steps": res[0]["steps"]}), flush=True)


if __name__ == "__main__":
    main()
