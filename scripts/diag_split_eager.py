#!/usr/bin/env python3
"""Diagnostic: eager Trainer steps, one-graph vs split-optimizer layout, each run twice (run-to-run
noise vs layout difference), per-parameter relative differences after 6 steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    dev = torch.device("cuda:0")
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=14, n_minutes=6 * 1440, seed=11))
    mc = C.default("model_cml")
    st = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
    steps = int(os.environ.get("STEPS", "6"))

    def run(split, graph):
        os.environ["GNNQC_SPLIT_OPT_GRAPH"] = "1" if split else "0"
        torch.manual_seed(0)
        model = GCNClassifier(mc, pc).to(dev)
        opt = make_optimizer("adam", model.parameters(), 1e-3)
        tr = Trainer(model, st, opt, {0: 1.0, 1: 5.0}, use_graph=graph, batch_size=64)
        loader = DeviceLoader(st, list(range(st.n_windows)), 64, shuffle=True)
        losses = []
        for row in list(loader.batch_ids())[:steps]:
            tr.train_step(row)
            losses.append(float(tr.last_loss.item()))
        torch.cuda.synchronize()
        return {n: p.detach().clone() for n, p in model.named_parameters()}, losses

    res = {}
    for split in (False, True):
        for graph in (False, True):
            for rep in (0, 1):
                res[(split, graph, rep)] = run(split, graph)
                print(split, graph, rep, ["%.6f" % v for v in res[(split, graph, rep)][1]], flush=True)
    base = res[(False, True, 0)][0]
    for key, (p, _) in res.items():
        tot = sum(((p[n] - base[n]) ** 2).sum().item() for n in base) ** 0.5
        worst = sorted(((((p[n] - base[n]).norm() / (base[n].norm() + 1e-12)).item(), n) for n in base),
                       reverse=True)[:4]
        print(key, "total %.3e" % tot, ["%s %.2e" % (n, v) for v, n in worst], flush=True)


if __name__ == "__main__":
    main()
