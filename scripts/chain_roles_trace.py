#!/usr/bin/env python3
"""Role-split chain forward (lstm_chain.hip chain_stage_roles) profile: per stage (tile 0) the
stage timeline (s_memrealtime, us) and, per role (compute / loader / storer), the loop cycles and the
cycles spent waiting at the step barriers (s_memtime, GNNQC_CHAIN_ROLES=2). The role that waits
least sets the step time. Also the kernel time with roles off / on / profiled. One JSON line each."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    M, Mp = 128, 128
    torch.manual_seed(0)
    units = [16, 16, 32, 32, 64, 64]
    pools = [0, 3, 0, 3, 0, 3]
    Ws, Us, bs = [], [], []
    for i, H in enumerate(units):
        dw = 18 if i == 0 else units[i - 1]
        Ws.append(torch.randn(dw, 4 * H, device=dev) * 0.3)
        Us.append(torch.randn(H, 4 * H, device=dev) * 0.3)
        bs.append(torch.randn(4 * H, device=dev) * 0.1)
    x = torch.randn(181, Mp, 20, device=dev)
    nt8 = 8
    mode = os.environ.get("GNNQC_CHAIN_ROLES", "1")

    def run():
        return ops.lstm_chain_fwd(x, Ws, Us, bs, pools, True)

    for _ in range(5):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        run()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / 50
    tr = ops.lstm_chain_trace(x).cpu()
    st = tr[:512].view(256, 2)
    t0 = int(st[:6 * nt8:nt8, 0].min())
    stages = [[round((int(st[s * nt8, 0]) - t0) / 100, 1), round((int(st[s * nt8, 1]) - t0) / 100, 1)]
              for s in range(6)]
    rt = tr[6912:6912 + 6 * 256].view(256, 6)
    roles = [[int(v) for v in rt[s * nt8]] for s in range(6)] if mode == "2" else None
    print(json.dumps({"roles_mode": mode, "us": round(us, 2), "stages": stages, "role_cycles": roles}), flush=True)


if __name__ == "__main__":
    main()
