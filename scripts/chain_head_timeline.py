#!/usr/bin/env python3
"""Timeline of the CML forward chain launch with time4 + head as its last stage (the headline step's
forward): per-stage start / end of tile 0 and the time4 / head workgroups' end times, from the
chain's s_memrealtime trace (100 MHz), read at the start of the backward (before the backward launch
overwrites it). Bench shape (23 links x 28 days, B = 128), eager steps. One JSON line per step."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    from gnnqc.models import GCNClassifier
    import gnnqc.ops.lstm as L
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    from gnnqc.train.loss import calculate_weights
    from gnnqc.utils.native import hip_ops
    dev = torch.device("cuda:0")
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    mc = C.default("model_cml")
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=23, n_minutes=28 * 1440, seed=7))
    st = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
    torch.manual_seed(0)
    model = GCNClassifier(mc, pc).to(dev)
    opt = make_optimizer("adam", model.parameters(), mc.learning_rate)
    tr = Trainer(model, st, opt, calculate_weights(mc), False, use_graph=False, batch_size=128)
    rows = []
    orig = L._HipLSTMChainHead.backward

    def bwd(ctx, *a):
        x = ctx.saved_tensors[0]
        ns = len(ctx.pools)
        t = hip_ops().lstm_chain_trace(x).cpu()
        nt8 = 8
        blocks = (ns + 1) * nt8
        tt = t[: 2 * blocks].view(blocks, 2).double()
        t0 = float(tt[:, 0][tt[:, 0] > 0].min())
        us = lambda v: round((float(v) - t0) / 100, 2)      # noqa: E731
        mid = t[512:768].double()
        rows.append({"stages": [{"stage": s, "start_us": us(tt[s * nt8, 0]), "end_us": us(tt[s * nt8, 1])}
                                for s in range(ns)],
                     # time4 workgroups: reverse... forward steps done / head forward done
                     "t4_steps_done_us": [us(mid[ns * nt8 + r]) for r in range(nt8)],
                     "t4_head_fwd_done_us": [us(mid[64 + ns * nt8 + r]) for r in range(nt8)],
                     "t4_head_end_us": [us(tt[ns * nt8 + r, 1]) for r in range(nt8)],
                     "t4_head_start_us": us(tt[ns * nt8, 0])})
        return orig(ctx, *a)

    L._HipLSTMChainHead.backward = staticmethod(bwd)
    ids = torch.arange(128, device=dev)
    brows = []
    for _ in range(6):
        tr.train_step(ids)
        torch.cuda.synchronize()
        # the backward launch's trace: blocks [0, nt8) = time4 + head backward, then stage k of the
        # reverse chain at (k + 1) nt8 (top layer first)
        xs = st.x if hasattr(st, "x") else ids
        t = hip_ops().lstm_chain_trace(ids.float()).cpu()
        nt8, nsb = 8, 7
        mid = t[512:768].double()
        tt = t[: 2 * nsb * nt8].view(nsb * nt8, 2).double()
        t0 = float(tt[:, 0][tt[:, 0] > 0].min())
        us = lambda v: round((float(v) - t0) / 100, 2)      # noqa: E731
        brows.append({"bwd_blocks_tile0": [{"block_row": k, "start_us": us(tt[k * nt8, 0]),
                                            "loop_start_us": us(mid[k * nt8]) if k < nsb - 1 else None,
                                            "end_us": us(tt[k * nt8, 1]),
                                            "tile_end_us": [us(tt[k * nt8 + r, 1]) for r in range(nt8)]}
                                           for k in range(nsb)],
                      "bwd_last_end_us": us(tt[:, 1].max()),
                      # time4 + head backward workgroups (block rows 6): head backward done / reverse steps done
                      "t4b_head_done_us": [us(mid[6 * nt8 + r]) for r in range(nt8)],
                      "t4b_steps_done_us": [us(mid[64 + 6 * nt8 + r]) for r in range(nt8)]})
    for r in rows[-2:]:
        print(json.dumps(r), flush=True)
    for r in brows[-2:]:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
