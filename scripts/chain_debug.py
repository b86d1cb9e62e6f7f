#!/usr/bin/env python3
"""Chain-kernel triage on the GPU box: runs the forward chain (and the headed forward) once with a
small debug spin limit (chain control word 6: a consumer gives up quickly instead of spinning for
seconds), then prints the control words (launch epoch, finished workgroups, spin-timeout flag),
per-stage start / end times of tile 0 from the kernel trace, and each stage's h against the
per-layer time-major kernels (max |diff|). One JSON line per check."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gnnqc.ops.lstm import chain_ctl
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    M = Mp = 128
    T = int(os.environ.get("T", "181"))
    units = [16, 16, 32, 32, 64, 64, 128]
    pools = [0, 3, 0, 3, 0, 3]
    Ws, Us, bs = [], [], []
    for i, H in enumerate(units):
        dw = 18 if i == 0 else units[i - 1]
        Ws.append(torch.randn(dw, 4 * H, device=dev) * 0.3)
        Us.append(torch.randn(H, 4 * H, device=dev) * 0.3)
        bs.append(torch.randn(4 * H, device=dev) * 0.1)
    x = torch.randn(T, Mp, 20, device=dev)
    x[..., 18:] = 0
    ctl = chain_ctl(dev)
    ctl[6] = int(os.environ.get("SPIN", "4000"))
    torch.cuda.synchronize()
    st0 = ops.lstm_chain_status(x).cpu().tolist()
    ns = int(os.environ.get("NS", "6"))
    for _ in range(int(os.environ.get("REPS", "5"))):      # (the trace keeps the last launch)
        outs = ops.lstm_chain_fwd(x, Ws[:ns], Us[:ns], bs[:ns], pools[:ns], True)
    torch.cuda.synchronize()
    st1 = ops.lstm_chain_status(x).cpu().tolist()
    tr = ops.lstm_chain_trace(x).cpu()[:512].view(256, 2)
    print(json.dumps({"check": "chain_fwd status", "before": st0[:4], "after": st1[:4], "repolls": (st1[9] - st0[9]) if len(st1) > 9 else None}), flush=True)
    nt8 = 8
    t0 = int(tr[0, 0])
    rows = []
    for s in range(ns):
        b = s * nt8
        rows.append({"stage": s, "start_us": round((int(tr[b, 0]) - t0) / 100, 2), "end_us": round((int(tr[b, 1]) - t0) / 100, 2)})
    print(json.dumps({"check": "trace tile 0 (us)", "stages": rows}), flush=True)
    # the backward chain on those saved states (same debug spin limit)
    if os.environ.get("BWD", "1") == "1":
        order = list(reversed(range(ns)))
        e8 = torch.zeros(0, dtype=torch.uint8, device=dev)
        xw = [20] + units[:ns - 1]
        last = outs[5 * (ns - 1) + 3] if pools[ns - 1] else outs[5 * (ns - 1)]
        dh = torch.randn_like(last) * 0.1
        st2 = ops.lstm_chain_status(x).cpu().tolist()
        for _ in range(int(os.environ.get("REPS", "5"))):
            res = ops.lstm_chain_bwd(dh, [outs[5 * i + 1] for i in order], [outs[5 * i + 2] for i in order],
                                     [Ws[i] for i in order], [Us[i] for i in order],
                                     [outs[5 * i + 4] if pools[i] else e8 for i in order], [pools[i] for i in order],
                                     [xw[i] for i in order], [outs[5 * i].shape[0] for i in order])
        torch.cuda.synchronize()
        st3 = ops.lstm_chain_status(x).cpu().tolist()
        tr = ops.lstm_chain_trace(x).cpu()[:512].view(256, 2)
        t0 = int(tr[0, 0])
        rows = [{"stage": k, "end_us": round((int(tr[k * nt8, 1]) - t0) / 100, 2)} for k in range(ns)]
        print(json.dumps({"check": "chain_bwd status", "before": st2[:4], "after": st3[:4], "repolls": (st3[9] - st2[9]) if len(st3) > 9 else None, "trace": rows,
                          "dx_finite": bool(torch.isfinite(res[ns]).all())}), flush=True)
    # per-layer reference of stage 0 and 1 (time-major kernels, same bf16 operands)
    ctl[6] = 0
    h0 = outs[0]
    ref0 = ops.lstm_tm_fwd(x, Ws[0], Us[0], bs[0], False)[0]
    if ref0 is not None:
        print(json.dumps({"check": "stage0 h vs lstm_tm_fwd", "max_abs_diff": float((h0 - ref0[:T]).abs().max()),
                          "nan": bool(torch.isnan(h0).any())}), flush=True)
    for s in range(ns):
        h = outs[5 * s]
        print(json.dumps({"check": f"stage{s} h", "shape": list(h.shape), "finite": bool(torch.isfinite(h).all()),
                          "absmax": float(h.abs().max())}), flush=True)


if __name__ == "__main__":
    main()
