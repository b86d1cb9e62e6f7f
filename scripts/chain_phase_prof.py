#!/usr/bin/env python3
"""Per-step phase clocks of the chain kernels' stages (GNNQC_CHAIN_PROF=1; tile 0, wave 0,
s_memtime ticks): median over the first 64 steps of every phase of the step loop, per stage.
Forward marks (compute wave 0): 0 loop top, 1 pre-activations out of the MFMAs, 2 gates / cell /
outputs stored, 3 after the step barrier. Backward: 0 top, 1 cell phase done, 2 next dh staged,
3 after the barrier, 4 dh_rec (U dz) ready, 5 dx MFMAs done. One JSON line per launch kind."""
import json
import os
import sys

os.environ["GNNQC_CHAIN_PROF"] = "1"
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def phases(pr, nmarks):
    out = []
    for s in range(pr.shape[0]):
        v = pr[s]
        if int(v[:, 0].max()) == 0:
            continue
        steps = [r for r in v.tolist() if r[0] > 0 and all(r[k] > 0 for k in range(nmarks))]
        if len(steps) < 4:
            continue
        t = torch.tensor(steps, dtype=torch.float64)
        d = (t[:, 1:nmarks] - t[:, :nmarks - 1]).median(0).values.tolist()
        per = (t[1:, 0] - t[:-1, 0]).median().item()
        out.append({"stage": s, "steps": len(steps), "step_ticks": round(per, 1), "phase_ticks": [round(x, 1) for x in d]})
    return out


def marks_rel(pr, nmarks):
    """Median of (mark k - mark 0) per stage for k < nmarks (marks written by other waves included)."""
    out = []
    for s in range(pr.shape[0]):
        v = pr[s].to(torch.float64)
        ok = (v[:, 0] > 0)
        if int(ok.sum()) < 4:
            continue
        row = {"stage": s}
        for k in range(1, nmarks):
            m = ok & (v[:, k] > 0)
            if int(m.sum()) >= 4:
                row[f"m{k}"] = round(float((v[m, k] - v[m, 0]).median()), 1)
        out.append(row)
    return out


def main():
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    M, Mp = 128, 128
    torch.manual_seed(0)
    units = [16, 16, 32, 32, 64, 64, 128]
    pools = [0, 3, 0, 3, 0, 3]
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
    x = torch.randn(181, Mp, 20, device=dev)
    e = torch.zeros(0, device=dev)
    hc = (0.3, 0.3, 1.0, 5.0)
    for _ in range(3):
        outs = ops.lstm_chain_head_fwd(x, Ws[:6], Us[:6], bs[:6], pools, True, Ws[6], Us[6], bs[6], head, y, mask, M,
                                       *hc, e.double(), e)
    torch.cuda.synchronize()
    pf = ops.lstm_chain_prof(x).cpu()
    print(json.dumps({"launch": "fwd (chain6 + time4 stage)", "stages": phases(pf, 4)}), flush=True)
    # I/O waves (marks 4..6 of the step whose x they stage: start, tile staged, next load issued),
    # relative to compute wave 0's step start
    # (+ m7: the publisher wave reaches the step barrier)
    print(json.dumps({"launch": "fwd marks vs compute start", "stages": marks_rel(pf, 8)}), flush=True)
    h4, g4, c4, logits, loss = outs[-5:]
    hb = outs[-6]          # (the head backward the forward launch precomputed)
    pk = outs[-7]
    outs = outs[:-7]
    xt = outs[5 * 5 + 3]
    hg = [torch.zeros_like(p) for p in head]
    one = torch.ones(1, device=dev)
    e8 = torch.zeros(0, dtype=torch.uint8, device=dev)
    order = list(reversed(range(6)))
    xw = [20] + units[:5]
    chain_args = ([outs[5 * i + 1] for i in order], [outs[5 * i + 2] for i in order], [Ws[i] for i in order],
                  [Us[i] for i in order], [outs[5 * i + 4] if pools[i] else e8 for i in order],
                  [pools[i] for i in order], [xw[i] for i in order], [outs[5 * i].shape[0] for i in order])
    for _ in range(3):
        ops.lstm_chain_head_bwd(one, xt, h4, g4, c4, Ws[6], Us[6], pk, hb, head, y, mask, M, *hc, hg, *chain_args)
    torch.cuda.synchronize()
    pb = ops.lstm_chain_prof(x).cpu()
    # H = 16 stages (chain_bwd_stage_io) mark 0 top, 1 cell done, 2 after the barrier, 3 dh_rec ready,
    # 4 dx done; the split-K stages (H >= 32) 0..5 as in the docstring
    print(json.dumps({"launch": "bwd (time4 stage + chain6)", "stages": phases(pb, 5)}), flush=True)
    # H = 16 stages' I/O waves: marks 5..7 = staging start, tile staged, next loads issued
    # (non-I/O H = 16 stages: m6 the dx wave's tile is in LDS, m7 the publisher's stores are issued)
    print(json.dumps({"launch": "bwd marks vs compute start", "stages": marks_rel(pb, 8)}), flush=True)
    st = ops.lstm_chain_status(x).cpu().tolist()
    print(json.dumps({"status": st}), flush=True)


if __name__ == "__main__":
    main()
