"""Per-layer timing of the persistent LSTM kernels on the CML GCN TimeLayer shapes.

    python scripts/lstm_microbench.py [--M 128 1024] [--reps 50]

Prints one JSON line per (layer, M): forward with training stores (h, c, gates),
forward inference (h only), backward recurrence, and the weight-gradient kernel,
in microseconds and ns per time step.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LAYERS = [(181, 18, 16), (181, 16, 16), (60, 16, 32), (60, 32, 32), (20, 32, 64), (20, 64, 64), (6, 64, 128)]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[128, 1024])
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default=None, help="T,Din,H of a single layer shape")
    args = ap.parse_args()
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    for M in args.M:
        layers = LAYERS if not args.only else [tuple(int(v) for v in args.only.split(","))]
        for T, Din, H in layers:
            g = torch.Generator().manual_seed(T * H)
            x = torch.randn(M, T, Din, generator=g).to(dev)
            W = (torch.randn(Din, 4 * H, generator=g) * 0.3).to(dev)
            U = (torch.randn(H, 4 * H, generator=g) * 0.3).to(dev)
            b = torch.zeros(4 * H, device=dev)
            h, c, gt = ops.lstm_fwd(x, W, U, b, True, True)
            dh = torch.randn_like(h)
            dz = ops.lstm_bwd(dh, gt, c, U, True)
            dW, dU, db = torch.zeros_like(W), torch.zeros_like(U), torch.zeros_like(b)
            r = {"M": M, "T": T, "Din": Din, "H": H,
                 "fwd_train_us": timeit(lambda: ops.lstm_fwd(x, W, U, b, True, True), args.reps),
                 "fwd_infer_us": timeit(lambda: ops.lstm_fwd(x, W, U, b, False, True), args.reps),
                 "bwd_us": timeit(lambda: ops.lstm_bwd(dh, gt, c, U, True), args.reps),
                 "grads_us": timeit(lambda: ops.lstm_grads(dz, x, h, W, dW, dU, db, True), args.reps)}
            if H in (16, 32):
                Mp = (M + 15) // 16 * 16
                xt = torch.zeros(T, Mp, Din, device=dev)
                xt[:, :M] = x.transpose(0, 1)
                ht, gt2, ct = ops.lstm_tm_fwd(xt, W, U, b, True)
                dht = torch.randn_like(ht)
                r["tm_fwd_train_us"] = timeit(lambda: ops.lstm_tm_fwd(xt, W, U, b, True), args.reps)
                r["tm_fwd_infer_us"] = timeit(lambda: ops.lstm_tm_fwd(xt, W, U, b, False), args.reps)
                r["tm_bwd_fused_us"] = timeit(lambda: ops.lstm_tm_bwd(dht, gt2, ct, xt, ht, W, U, b, dW, dU, db, True),
                                              args.reps)
                e = torch.zeros(0, device=dev)
                r["tm_bwd_nowgrad_us"] = timeit(lambda: ops.lstm_tm_bwd(dht, gt2, ct, xt, ht, W, U, b, e, e, e, True),
                                                args.reps)
                for k in ("tm_fwd_train_us", "tm_fwd_infer_us", "tm_bwd_fused_us", "tm_bwd_nowgrad_us"):
                    r[k.replace("_us", "_ns_per_step")] = round(r[k] * 1000.0 / T, 1)
            for k in ("fwd_train_us", "fwd_infer_us", "bwd_us"):
                r[k.replace("_us", "_ns_per_step")] = round(r[k] * 1000.0 / T, 1)
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
