#!/usr/bin/env python3
"""Diagnostic: which host operations synchronise inside IntegratedGradients.attribute (CML GCN)?
torch.cuda.set_sync_debug_mode('warn') reports every synchronising call with its stack; also
host vs device time per attribute() call."""
import os
import sys
import time
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    from gnnqc.models import GCNClassifier
    from gnnqc.xai.ig import IntegratedGradients
    dev = torch.device("cuda:0")
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=23, n_minutes=28 * 1440, seed=7))
    store = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
    model = GCNClassifier(C.default("model_cml"), pc).to(dev)
    ig = IntegratedGradients(model, "cml", m_steps=100, max_rows=16384)
    B = 128

    def batch(i):
        return store.gather(torch.arange(i * B, i * B + B, device=dev))

    ig.attribute(batch(0))
    torch.cuda.synchronize()
    seen = set()

    def show(message, category, filename, lineno, file=None, line=None):
        st = "".join(traceback.format_stack(limit=12)[:-1])
        key = st[-600:]
        if key in seen:
            return
        seen.add(key)
        print("SYNC:", message, "\n", st, flush=True)

    warnings.showwarning = show
    torch.cuda.set_sync_debug_mode("warn")
    t0 = time.perf_counter()
    res = ig.attribute(batch(1))
    t1 = time.perf_counter()
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("host %.2f ms, host+drain %.2f ms" % (1e3 * (t1 - t0), 1e3 * (t2 - t0)), flush=True)
    for n in (3, 6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            ig.attribute(batch(2 + i))
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("%d batches: host %.2f ms/batch, wall %.2f ms/batch" % (n, 1e3 * (t1 - t0) / n, 1e3 * (t2 - t0) / n))


if __name__ == "__main__":
    main()
