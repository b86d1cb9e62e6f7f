"""Localise conv1d_bwd dx errors on the GPU (which rows / taps / channels)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnnqc.ops.conv import conv1d_act_eager  # noqa: E402
from gnnqc.utils.native import hip_ops  # noqa: E402

ops = hip_ops()
dev = torch.device("cuda:0")


def ref_dx(dy, y, W, alpha):
    dz = dy.double() * torch.where(y.double() > 0, 1.0, alpha)
    k, cin, cout = W.shape
    return conv1d_act_eager(dz.cpu(), W.double().cpu().flip(0).transpose(1, 2), torch.zeros(cin, dtype=torch.double), 1.0)


for (k, cin, cout, T, M) in [(5, 18, 16, 181, 37), (5, 16, 16, 181, 37), (3, 16, 16, 20, 5), (1, 16, 16, 20, 5),
                             (5, 16, 32, 20, 5), (5, 32, 16, 20, 5)]:
    g = torch.Generator().manual_seed(1)
    x = torch.randn(M, T, cin, generator=g)
    W = torch.randn(k, cin, cout, generator=g) * 0.2
    dy = torch.randn(M, T, cout, generator=g)
    for ymode in ("pos", "neg", "rand"):
        y = {"pos": torch.ones(M, T, cout), "neg": -torch.ones(M, T, cout), "rand": torch.randn(M, T, cout, generator=g)}[ymode]
        e = torch.zeros(0, device=dev)
        dx = ops.conv1d_bwd(dy.to(dev), y.to(dev), x.to(dev), W.to(dev), 0.3, False, e, e, True).double().cpu()
        r = ref_dx(dy, y, W, 0.3)
        err = (dx - r).abs()
        rel = (err.max() / r.abs().max()).item()
        where = err.amax(dim=(0, 2))
        bad_t = (where > 0.05 * r.abs().max()).nonzero().flatten().tolist()
        bad_c = (err.amax(dim=(0, 1)) > 0.05 * r.abs().max()).nonzero().flatten().tolist()
        print(f"k={k} cin={cin} cout={cout} T={T} y={ymode}: rel {rel:.4f} bad_t {bad_t[:12]} bad_c {bad_c}", flush=True)
    # forward vs eager
    b = torch.zeros(cout)
    yy, gg = ops.conv1d_fwd(x.to(dev), W.to(dev), b.to(dev), 0.3, False, True)
    rf = conv1d_act_eager(x.double(), W.double(), b.double(), 0.3)
    print("   fwd rel", ((yy.double().cpu() - rf).abs().max() / rf.abs().max()).item(), flush=True)
