#!/usr/bin/env python3
"""Integrated-gradients throughput (BASELINE config v): explained windows/s for the CML GCN.

    python scripts/bench_ig.py [--batches K] [--m-steps 100] [--batch 128]
    torchrun --nproc-per-node N scripts/bench_ig.py ...     (batches sharded over ranks)

Each explained window costs m_steps + 1 forward + backward passes (reference
``xai/libs/integrated_gradients.py:898-1012``: a Python loop over alphas; here the alphas
are stacked on the batch axis, ``gnnqc.xai.ig.IntegratedGradients``). Random-init weights,
synthetic data of the CML example shape. Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=4, help="timed batches per rank")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=324, help="windows explained per attribute() call "
                    "(324 = one full 32768-row path chunk)")
    ap.add_argument("--m-steps", type=int, default=100)
    ap.add_argument("--max-rows", type=int, default=32768, help="path rows (windows x path points) per pass")
    args = ap.parse_args(argv)

    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    from gnnqc.models import GCNClassifier
    from gnnqc.parallel import dist as D
    from gnnqc.xai.ig import IntegratedGradients, completeness_gap

    dev = D.init_distributed()
    world, rank = D.world_size(), D.rank()
    torch.manual_seed(0)
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    mc = C.default("model_cml")
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=23, n_minutes=28 * 1440, seed=7))
    store = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
    model = GCNClassifier(mc, pc).to(dev)
    D.broadcast_module(model)
    ig = IntegratedGradients(model, "cml", m_steps=args.m_steps, max_rows=args.max_rows)
    n = store.n_windows
    B = args.batch

    def batch(i):
        start = ((i * world + rank) * B) % max(1, n - B)
        return store.gather(torch.arange(start, start + B, device=dev))

    for i in range(args.warmup):
        ig.attribute(batch(i))
    D.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    gap = 0.0
    for i in range(args.batches):
        res = ig.attribute(batch(args.warmup + i))
        if i == args.batches - 1:
            gap = float(completeness_gap(res).abs().max().item())
    if dev.type == "cuda":
        torch.cuda.synchronize()
    D.barrier()
    dt = D.max_over_ranks(time.perf_counter() - t0)
    windows = args.batches * B * world
    if rank == 0:
        print(json.dumps({
            "metric": "integrated-gradients explained windows/s, CML GCN", "value": round(windows / dt, 2),
            "unit": "windows/s (whole job)", "n_gpus": world, "m_steps": args.m_steps,
            "passes_per_window": args.m_steps + 1, "batch": B, "ms_per_batch": round(1e3 * dt / args.batches, 3),
            "completeness_gap_max": gap, "dtype": "bf16", "data": "synthetic CML (23 links x 28 days), random init",
        }), flush=True)
    D.destroy()


if __name__ == "__main__":
    main()
