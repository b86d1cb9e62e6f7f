#!/usr/bin/env python3
"""HIP-event timings of the CML GCN kernels at the benched shape (B = 128 windows, T = 181,
N = 23 links, Cin = 2, F = 16, time-major output [T, 128, 20]): gcn_prep (training),
gcn_pool_fwd, gcn_pool_bwd, gcn_bwd_finalize. One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=20, iters=10):
    """GPU time per call: ``reps`` calls captured into one HIP graph (host launch overhead of
    the small kernels would otherwise dominate), replayed ``iters`` times."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / (reps * iters), 2)


def main():
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, T, N, Cin, F, Ca = 128, 181, 23, 2, 16, 2
    x = torch.randn(B, T, N, Cin, device=dev)
    adj = (torch.rand(B, N, N, device=dev) < 0.3).float()
    mask = (torch.rand(B, N, device=dev) < 0.9).float()
    anom = torch.randn(B, T, Ca, device=dev)
    ap = torch.zeros(0, dtype=torch.long, device=dev)
    W, b = torch.randn(Cin, F, device=dev), torch.randn(F, device=dev)
    gamma, beta, alpha = torch.ones(F, device=dev), torch.zeros(F, device=dev), torch.full((F,), 0.3, device=dev)
    rm, rv = torch.zeros(F, device=dev), torch.ones(F, device=dev)
    Mp, Cp = 128, 20
    res = {}
    res["gcn_prep"] = timeit(lambda: ops.gcn_prep(x, adj, mask, ap, True, 0, W, b, gamma, beta, rm, rv, True, 0.99, 1e-3))
    w, S, st = ops.gcn_prep(x, adj, mask, ap, True, 0, W, b, gamma, beta, rm, rv, True, 0.99, 1e-3)
    res["gcn_pool_fwd"] = timeit(lambda: ops.gcn_pool_fwd(x, w, anom, W, b, st[2], st[3], alpha, Mp, Cp))
    dout = torch.randn(T, Mp, Cp, device=dev)
    res["gcn_pool_bwd"] = timeit(lambda: ops.gcn_pool_bwd(x, w, dout, W, b, st[2], st[3], alpha, Ca, True))
    acc = ops.gcn_pool_bwd(x, w, dout, W, b, st[2], st[3], alpha, Ca, True)
    sinks = [torch.zeros_like(t) for t in (W, b, gamma, beta, alpha)]
    res["gcn_bwd_finalize"] = timeit(lambda: ops.gcn_bwd_finalize(acc, S, W, b, st, True, *sinks))
    res["acc_rows"] = acc.shape[0]
    tiny = torch.zeros(16, device=dev)
    res["floor_tiny_add"] = timeit(lambda: tiny.add_(1.0))                  # a trivial one-workgroup kernel
    big = torch.zeros(1 << 20, device=dev)
    res["floor_4MB_add"] = timeit(lambda: big.add_(1.0))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
