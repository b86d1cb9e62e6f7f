#!/usr/bin/env python3
"""Microbenchmark of the cross-CU chain forward (lstm_chain.hip): time of the first k stages
of the CML LSTM stack (k = 1..6) vs the per-layer kernels. Prints one JSON line per k."""
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


def main():
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    M = int(os.environ.get("M", "128"))
    Mp = (M + 15) // 16 * 16
    torch.manual_seed(0)
    units = [16, 16, 32, 32, 64, 64]
    pools = [0, 3, 0, 3, 0, 3]
    din = 20
    Ws, Us, bs = [], [], []
    for i, H in enumerate(units):
        dw = 18 if i == 0 else units[i - 1]
        Ws.append(torch.randn(dw, 4 * H, device=dev) * 0.3)
        Us.append(torch.randn(H, 4 * H, device=dev) * 0.3)
        bs.append(torch.randn(4 * H, device=dev) * 0.1)
    x = torch.randn(181, Mp, din, device=dev)
    nt8 = (Mp // 16 + 7) // 8 * 8
    for k in []:
        us = timeit(lambda: ops.lstm_chain_fwd(x, Ws[:k], Us[:k], bs[:k], pools[:k], True))
        tr = ops.lstm_chain_trace(x).cpu()[:512].view(256, 2)
        t0 = int(tr[:k * nt8:nt8, 0].min())
        # per stage (tile 0): start / end in us after the first workgroup started (100 MHz ticks)
        st = [[round((int(tr[s * nt8, 0]) - t0) / 100, 1), round((int(tr[s * nt8, 1]) - t0) / 100, 1)]
              for s in range(k)]
        print(json.dumps({"stages": k, "chain_us": round(us, 2), "stage_start_end_us": st}), flush=True)
    for cfg in []:
        k = len(cfg)
        us = timeit(lambda: ops.lstm_chain_fwd(x, Ws[:1] + [Ws[1]] * (k - 1), Us[:1] + [Us[1]] * (k - 1),
                                               bs[:1] + [bs[1]] * (k - 1), cfg, True))
        tr = ops.lstm_chain_trace(x).cpu()[:512].view(256, 2)
        t0 = int(tr[:k * nt8:nt8, 0].min())
        st = [[round((int(tr[s * nt8, 0]) - t0) / 100, 1), round((int(tr[s * nt8, 1]) - t0) / 100, 1)]
              for s in range(k)]
        print(json.dumps({"h16_stages": k, "chain_us": round(us, 2), "stage_start_end_us": st}), flush=True)
    # backward chain on the full stack (per-stage start / end, top layer = stage 0)
    outs = ops.lstm_chain_fwd(x, Ws, Us, bs, pools, True)
    order = list(reversed(range(6)))
    e8 = torch.zeros(0, dtype=torch.uint8, device=dev)
    xw = [din] + units[:-1]
    Ts = [outs[5 * i].shape[0] for i in range(6)]
    last = outs[5 * 5]
    dh = torch.randn(Ts[5] // 3, Mp, 64, device=dev)
    for k in []:
        sel = order[:k]
        args = (dh, [outs[5 * i + 1] for i in sel], [outs[5 * i + 2] for i in sel], [Ws[i] for i in sel],
                [Us[i] for i in sel], [outs[5 * i + 4] if pools[i] else e8 for i in sel], [pools[i] for i in sel],
                [xw[i] for i in sel], [Ts[i] for i in sel])
        us = timeit(lambda: ops.lstm_chain_bwd(*args))
        tr = ops.lstm_chain_trace(x).cpu()
        mid = tr[512:]
        tr = tr[:512].view(256, 2)
        t0 = int(tr[:k * nt8:nt8, 0].min())
        st = [[round((int(tr[s * nt8, 0]) - t0) / 100, 1), round((int(mid[s * nt8]) - t0) / 100, 1),
               round((int(tr[s * nt8, 1]) - t0) / 100, 1)] for s in range(k)]
        print(json.dumps({"bwd_stages": k, "chain_us": round(us, 2), "stage_start_end_us": st}), flush=True)
    order = [0, 1, 2, 3]
    for i in order:      # single-stage chain backward of each layer (body cost without hand-offs)
        sel = [i]
        dhi = torch.randn(Ts[i] // 3 if pools[i] else Ts[i], Mp, units[i], device=dev)
        args = (dhi, [outs[5 * i + 1]], [outs[5 * i + 2]], [Ws[i]], [Us[i]], [outs[5 * i + 4] if pools[i] else e8],
                [pools[i]], [xw[i]], [Ts[i]])
        us = timeit(lambda: ops.lstm_chain_bwd(*args))
        tr = ops.lstm_chain_trace(x).cpu()
        st = [round((int(tr[512]) - int(tr[0])) / 100, 1), round((int(tr[1]) - int(tr[0])) / 100, 1)]
        print(json.dumps({"layer": i, "chain1_bwd_us": round(us, 2), "setup_end_us": st}), flush=True)
    for i in order:
        g, c = outs[5 * i + 1], outs[5 * i + 2]
        T = outs[5 * i].shape[0]
        dhi = torch.randn(T, Mp, units[i], device=dev)
        us = timeit(lambda: ops.lstm_tm_bwd_dz(dhi, g, c, Ws[i], Us[i], T, None, 0))
        print(json.dumps({"layer": i, "bwd_dz_us": round(us, 2)}), flush=True)
    # per-layer kernels for reference
    h = x
    for i in range(6):
        hh = h
        us = timeit(lambda: ops.lstm_tm_fwd(hh, Ws[i], Us[i], bs[i], True, pools[i]))
        out = ops.lstm_tm_fwd(hh, Ws[i], Us[i], bs[i], True, pools[i])
        h = out[3] if pools[i] else out[0]
        print(json.dumps({"layer": i, "H": units[i], "T": hh.shape[0], "tm_fwd_us": round(us, 2)}), flush=True)
    st = ops.lstm_chain_status(x).cpu().tolist()
    print(json.dumps({"status": st}))


if __name__ == "__main__":
    main()
