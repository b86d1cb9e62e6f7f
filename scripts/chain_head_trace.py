#!/usr/bin/env python3
"""Timeline of the CML TimeLayer kernels: the six-stage chain (lstm_chain_fwd / _bwd, per-stage
start / end from the kernels' s_memrealtime trace, tile 0, us after the first workgroup started)
and the time4 + head kernels (time4_head_fwd / _bwd); launch times are HIP-event means of 50.
One JSON line per measurement."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def stages(ops, x, k, nt8, mid=False):
    tr = ops.lstm_chain_trace(x).cpu()
    m = tr[512:768]
    tr = tr[:512].view(256, 2)
    t0 = int(tr[:k * nt8:nt8, 0].min())
    out = []
    for s in range(k):
        row = [round((int(tr[s * nt8, 0]) - t0) / 100, 1)]
        if mid:
            row.append(round((int(m[s * nt8]) - t0) / 100, 1))
        row.append(round((int(tr[s * nt8, 1]) - t0) / 100, 1))
        out.append(row)
    return out


def t4marks(ops, x, ntiles=8):
    """time4 kernel marks per tile (us after the first tile started): start, prologue, steps..., end."""
    tr = ops.time4_trace(x).cpu()[:16 * ntiles].view(ntiles, 16)
    t0 = int(tr[:, 0].min())
    return [[round((int(v) - t0) / 100, 1) for v in row if int(v) >= t0] for row in tr]


def main():
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    M = int(os.environ.get("M", "128"))
    Mp = (M + 15) // 16 * 16
    torch.manual_seed(0)
    units = [16, 16, 32, 32, 64, 64, 128]
    pools = [0, 3, 0, 3, 0, 3, 0]
    din = 20
    Ws, Us, bs = [], [], []
    for i, H in enumerate(units):
        dw = 18 if i == 0 else units[i - 1]
        Ws.append(torch.randn(dw, 4 * H, device=dev) * 0.3)
        Us.append(torch.randn(H, 4 * H, device=dev) * 0.3)
        bs.append(torch.randn(4 * H, device=dev) * 0.1)
    head = [torch.randn(128, 64, device=dev) * 0.1, torch.zeros(64, device=dev),
            torch.randn(64, 64, device=dev) * 0.1, torch.zeros(64, device=dev),
            torch.randn(64, 1, device=dev) * 0.1, torch.zeros(1, device=dev)]
    y = (torch.rand(M, device=dev) < 0.2).float()
    mask = torch.ones(M, device=dev)
    x = torch.randn(181, Mp, din, device=dev)
    nt8 = (Mp // 16 + 7) // 8 * 8
    e = torch.zeros(0, device=dev)
    hc = (0.3, 0.3, 1.0, 5.0)
    us6 = timeit(lambda: ops.lstm_chain_fwd(x, Ws[:6], Us[:6], bs[:6], pools[:6], True))
    print(json.dumps({"fwd": "chain6", "us": round(us6, 2), "stages": stages(ops, x, 6, nt8)}), flush=True)
    # time4 + head + loss as the seventh stage of the forward launch (lstm_chain_head_fwd)
    uh = timeit(lambda: ops.lstm_chain_head_fwd(x, Ws[:6], Us[:6], bs[:6], pools[:6], True, Ws[6], Us[6], bs[6], head,
                                                y, mask, M, *hc, e.double(), e))
    print(json.dumps({"fwd": "chain6+time4head", "us": round(uh, 2), "stages": stages(ops, x, 7, nt8)}), flush=True)
    outs = ops.lstm_chain_fwd_pack(x, Ws[:6], Us[:6], bs[:6], pools[:6], True, Ws[6], Us[6])
    pk = outs.pop()
    up = timeit(lambda: ops.lstm_chain_fwd_pack(x, Ws[:6], Us[:6], bs[:6], pools[:6], True, Ws[6], Us[6]))
    print(json.dumps({"fwd": "chain6+pack", "us": round(up, 2)}), flush=True)
    xt = outs[5 * 5 + 3]
    ut = timeit(lambda: ops.time4_head_fwd(xt, Ws[6], Us[6], bs[6], pk, True, head, y, mask, M, *hc, e.double(), e))
    print(json.dumps({"fwd": "time4+head", "us": round(ut, 2), "marks": t4marks(ops, x)}), flush=True)
    ue = timeit(lambda: ops.time4_head_fwd(xt, Ws[6], Us[6], bs[6], pk, False, head, y, mask, M, *hc, e.double(), e))
    print(json.dumps({"fwd": "time4+head eval", "us": round(ue, 2), "marks": t4marks(ops, x)}), flush=True)
    h4, g4, c4, logits, loss = ops.time4_head_fwd(xt, Ws[6], Us[6], bs[6], pk, True, head, y, mask, M, *hc, e.double(), e)
    hg = [torch.zeros_like(p) for p in head]
    one = torch.ones(1, device=dev)
    ub = timeit(lambda: ops.time4_head_bwd(one, xt, h4, g4, c4, Ws[6], Us[6], pk, head, y, mask, M, *hc, hg))
    print(json.dumps({"bwd": "head+time4", "us": round(ub, 2), "marks": t4marks(ops, x)}), flush=True)
    dz4, dxt = ops.time4_head_bwd(one, xt, h4, g4, c4, Ws[6], Us[6], pk, head, y, mask, M, *hc, hg)
    e8 = torch.zeros(0, dtype=torch.uint8, device=dev)
    xw = [din] + units[:-1]
    Ts = [outs[5 * i].shape[0] for i in range(6)]
    order6 = list(reversed(range(6)))
    a6 = (dxt, [outs[5 * i + 1] for i in order6], [outs[5 * i + 2] for i in order6], [Ws[i] for i in order6],
          [Us[i] for i in order6], [outs[5 * i + 4] if pools[i] else e8 for i in order6],
          [pools[i] for i in order6], [xw[i] for i in order6], [Ts[i] for i in order6])
    ub6 = timeit(lambda: ops.lstm_chain_bwd(*a6))
    print(json.dumps({"bwd": "chain6", "us": round(ub6, 2), "stages": stages(ops, x, 6, nt8, True)}), flush=True)
    # time4 + head backward as the first stage of the backward launch (lstm_chain_head_bwd);
    # stage 6 of the timeline is time4 (its blocks follow the six chain stages)
    ubh = timeit(lambda: ops.lstm_chain_head_bwd(one, xt, h4, g4, c4, Ws[6], Us[6], pk, e, head, y, mask, M, *hc, hg, *a6[1:]))
    print(json.dumps({"bwd": "time4head+chain6", "us": round(ubh, 2), "stages": stages(ops, x, 7, nt8, True)}),
          flush=True)
    both = timeit(lambda: (ops.time4_head_fwd(xt, Ws[6], Us[6], bs[6], pk, True, head, y, mask, M, *hc, e.double(), e),
                           ops.time4_head_bwd(one, xt, h4, g4, c4, Ws[6], Us[6], pk, head, y, mask, M, *hc, hg)))
    print(json.dumps({"time4_head_fwd_bwd_us": round(both, 2)}), flush=True)
    st = ops.lstm_chain_status(x).cpu().tolist()
    print(json.dumps({"status": st}), flush=True)


if __name__ == "__main__":
    main()
