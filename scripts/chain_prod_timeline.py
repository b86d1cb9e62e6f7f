#!/usr/bin/env python3
"""Timeline of the CML forward chain launch with the GCN forward as producer workgroups
(gcn_fused.h gcn_prod_body): tile 0's stage start / end and the producers' start, first-pass-stored
and end times (quantiles over the 128 sample rows), from the chain's s_memrealtime trace (100 MHz),
read at the start of the backward. Bench shape (23 links x 28 days, B = 128), eager steps."""
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

    def q(v):
        v = sorted(v)
        return [round(v[0], 2), round(v[len(v) // 2], 2), round(v[-1], 2)] if v else None

    def bwd(ctx, *a):
        x = ctx.saved_tensors[0]
        ns = len(ctx.pools)
        t = hip_ops().lstm_chain_trace(x).cpu().double()
        nt8 = 8
        tt = t[:512].view(256, 2)
        t0 = float(tt[: (ns + 1) * nt8, 0][tt[: (ns + 1) * nt8, 0] > 0].min())
        us = lambda v: (float(v) - t0) / 100      # noqa: E731
        first = (ns + 1) * nt8
        prod = [k for k in range(first, 256) if tt[k, 0] > 0 and tt[k, 1] >= tt[k, 0] and us(tt[k, 0]) > -1e3
                and us(tt[k, 1]) < 1e4]
        rows.append({"stages": [{"stage": s, "start_us": round(us(tt[s * nt8, 0]), 2),
                                 "end_us": round(us(tt[s * nt8, 1]), 2)} for s in range(ns)],
                     "t4_end_us": round(us(tt[ns * nt8, 1]), 2),
                     "producer_blocks": len(prod),
                     "prod_start_us_min_med_max": q([us(tt[k, 0]) for k in prod]),
                     **{f"prod_{name}_us_min_med_max": q([us(v) for v in t[640 + k:768:4].tolist()
                                                          if v > 0 and -1e3 < us(v) < 1e4])
                        for k, name in enumerate(("loads_in", "bn_prepped", "rows_stored"))},
                     "prod_end_us_min_med_max": q([us(tt[k, 1]) for k in prod])})
        return orig(ctx, *a)

    L._HipLSTMChainHead.backward = staticmethod(bwd)
    ids = torch.arange(128, device=dev)
    for _ in range(6):
        tr.train_step(ids)
        torch.cuda.synchronize()
    for r in rows[-2:]:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
