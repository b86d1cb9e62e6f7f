#!/usr/bin/env python3
"""Dump the forward chain's outputs (h, gates, c, pooled, argmax per stage) for a fixed random input
to OUT (torch.save), to diff two builds' saved state on the host. CML shape (8 tiles, T = 181)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    units = [16, 16, 32, 32, 64, 64]
    pools = [0, 3, 0, 3, 0, 3]
    Ws, Us, bs = [], [], []
    for i, H in enumerate(units):
        dw = 18 if i == 0 else units[i - 1]
        Ws.append(torch.randn(dw, 4 * H, device=dev) * 0.3)
        Us.append(torch.randn(H, 4 * H, device=dev) * 0.3)
        bs.append(torch.randn(4 * H, device=dev) * 0.1)
    x = torch.randn(181, 128, 20, device=dev)
    x[..., 18:] = 0
    outs = ops.lstm_chain_fwd(x, Ws, Us, bs, pools, True)
    torch.cuda.synchronize()
    torch.save([o.float().cpu() if o.dtype != torch.uint8 else o.cpu() for o in outs], os.environ["OUT"])


if __name__ == "__main__":
    main()
