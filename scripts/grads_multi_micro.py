#!/usr/bin/env python3
"""Time the CML step's batched weight-gradient launch (``lstm_grads_multi``) and its reduction by job
subset: the jobs of one real eager training step (bench shape) are captured at ``pipe_flush`` and
replayed alone (HIP events, 50 launches each). Answers which jobs set the launch's duration, i.e.
what moving the upper layers' passes into the chain backward would leave behind. One JSON line per
subset. (The replays add into the gradient buffers: timing only.)"""
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
    ops = hip_ops()
    dev = torch.device("cuda:0")
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    mc = C.default("model_cml")
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=23, n_minutes=28 * 1440, seed=7))
    st = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
    torch.manual_seed(0)
    model = GCNClassifier(mc, pc).to(dev)
    opt = make_optimizer("adam", model.parameters(), mc.learning_rate)
    tr = Trainer(model, st, opt, calculate_weights(mc), False, use_graph=False, batch_size=128)
    cap = {}
    orig = ops.lstm_grads_multi

    class Spy:
        def __getattr__(self, k):
            if k == "lstm_grads_multi":
                def f(*a):
                    cap["args"] = a
                    return orig(*a)
                return f
            return getattr(ops, k)

    L_hip = L.__dict__.get("hip_ops")
    import gnnqc.utils.native as N
    real = N.hip_ops
    N.hip_ops = lambda: Spy()
    try:
        ids = torch.arange(128, device=dev)
        for _ in range(3):
            tr.train_step(ids)
    finally:
        N.hip_ops = real
    torch.cuda.synchronize()
    a = cap["args"]
    gz, gx, gh, gW, per, hs, gws, rws, rW, rdW, rdU, rdb, gt, gi = a
    H = [w.shape[1] // 4 for w in gW]
    T = [z.shape[0] - 1 for z in gz]
    print(json.dumps({"jobs": [{"H": h, "T": t, "Din": w.shape[0], "ws_floats": g.numel()}
                               for h, t, w, g in zip(H, T, gW, gws)], "gcn_job": len(gt) > 0,
                      "n_reduce": len(rws)}), flush=True)
    e = []

    def timed(fn, n=50):
        for _ in range(5):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for x, y in ev:
            x.record()
            fn()
            y.record()
        torch.cuda.synchronize()
        return round(1e3 * sum(x.elapsed_time(y) for x, y in ev) / n, 2)

    def grads(sel, gcn=True):
        return lambda: orig([gz[k] for k in sel], [gx[k] for k in sel], [gh[k] for k in sel], [gW[k] for k in sel],
                            [per[k] for k in sel], [hs[k] for k in sel], [gws[k] for k in sel], e, e, e, e, e,
                            gt if gcn else e, gi if gcn else [])

    def reds(sel):
        return lambda: orig(e, e, e, e, [], [], e, [rws[k] for k in sel], [rW[k] for k in sel],
                            [rdW[k] for k in sel], [rdU[k] for k in sel], [rdb[k] for k in sel], e, [])
    e = []
    alln = list(range(len(gz)))
    bottom = [k for k in alln if H[k] == 16]
    upper = [k for k in alln if H[k] != 16]
    rows = {"grads_all+gcn": timed(grads(alln)), "grads_all_nogcn": timed(grads(alln, False)),
            "grads_bottom(H16)+gcn": timed(grads(bottom)), "grads_bottom_nogcn": timed(grads(bottom, False)),
            "grads_upper_nogcn": timed(grads(upper, False)),
            "reduce_all": timed(reds(list(range(len(rws))))),
            "reduce_bottom": timed(reds([k for k in range(len(rws)) if rW[k].shape[1] // 4 == 16]))}
    for k in alln:
        rows[f"grads_job{k}_H{H[k]}_T{T[k]}"] = timed(grads([k], False))
    print(json.dumps(rows), flush=True)


if __name__ == "__main__":
    main()
