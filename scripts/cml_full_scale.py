#!/usr/bin/env python3
"""Full-size CML network through the whole pipeline on one MI355X (VERDICT r1 "next" item 5).

Shape of the reference's full dataset (``notebooks/prepare_raw_cml.ipynb`` cell 9): 3,904 links x
133,920 minutes, 20 flagged links. Synthetic data (no network access: the real set is not
available), random-init weights. Reports, as ONE JSON line:

* generation and preprocessing wall time (neighbourhoods, gap filling, targets, windows,
  rolling-median statistics) and the host peak RSS;
* the HBM footprint of the DeviceStore (every window's inputs stay resident) and the peak of one
  training fold;
* one CV fold (fold 0 of 5, the reference's splitter) trained with the config's epochs in bf16 and,
  with ``--fp32``, again in fp32: ROC-AUC / MCC of the held-out fold and training windows/s.

    python scripts/cml_full_scale.py [--epochs E] [--fp32] [--sensors S --minutes M --flagged F]
    python scripts/cml_full_scale.py --all-folds      (5-fold CV at full size, bf16)
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _rss_gb() -> float:
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024 ** 2


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sensors", type=int, default=3904)
    ap.add_argument("--minutes", type=int, default=133920)
    ap.add_argument("--flagged", type=int, default=20)
    ap.add_argument("--epochs", type=int, default=None, help="default: model config (10)")
    ap.add_argument("--fp32", action="store_true", help="also train the fold in fp32")
    ap.add_argument("--fold", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-train", action="store_true", help="stop after the DeviceStore")
    ap.add_argument("--all-folds", action="store_true",
                    help="bf16: all 5 folds of the reference's splitter (the headline 5-fold CV protocol at full size)")
    args = ap.parse_args(argv)

    import numpy as np
    import torch
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset, prepare_cml_groups
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw_network
    from gnnqc.train.cv import run_cv

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    rec = {"what": "CML full-network shape: generation, preprocessing, HBM footprint, one CV fold",
           "data": f"synthetic ({args.sensors} links x {args.minutes} min @1min, {args.flagged} flagged), "
                   "random-init weights", "device": str(dev)}
    t0 = time.time()
    raw = make_cml_raw_network(n_sensors=args.sensors, n_flagged=args.flagged, n_minutes=args.minutes, seed=3)
    rec["generate_s"] = round(time.time() - t0, 1)
    rec["raw_gb"] = round(sum(v.data.nbytes for v in raw.variables.values() if v.data.dtype != bool) / 1e9, 2)
    print(json.dumps({"stage": "generated", **rec}), flush=True)

    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
    t0 = time.time()
    groups = prepare_cml_groups(raw, pc)
    rec["groups_s"] = round(time.time() - t0, 1)
    rec["group_sizes"] = [int(len(g.sensor_ids)) for g in groups]
    t0 = time.time()
    ws = create_windows_dataset(pc, groups=groups)
    rec["windows_s"] = round(time.time() - t0, 1)
    rec["n_windows"] = int(ws.n_windows)
    del raw
    print(json.dumps({"stage": "preprocessed", **rec}), flush=True)

    if dev.type == "cuda":
        torch.cuda.reset_peak_memory_stats()
        m0 = torch.cuda.memory_allocated()
    t0 = time.time()
    store = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
    if dev.type == "cuda":
        torch.cuda.synchronize()
        rec["store_hbm_gb"] = round((torch.cuda.memory_allocated() - m0) / 1e9, 3)
    rec["store_s"] = round(time.time() - t0, 1)
    rec["host_peak_rss_gb"] = round(_rss_gb(), 2)
    print(json.dumps({"stage": "store", **rec}), flush=True)

    if args.all_folds and not args.no_train:
        mc = C.default("model_cml")
        mc.runtime.compute_dtype = "bf16"
        if args.epochs:
            mc["epochs"] = int(args.epochs)
        t0 = time.time()
        res = run_cv(pc, mc, ws, folds=5, device=dev, store=store, verbose=2)
        folds = [{"auc": round(f["auc"], 4), "mcc": round(f["mcc"], 4), "n_train": f["n_train"],
                  "n_test": f["n_test"], "epochs": len(f["loss_curve"])} for f in res["per_fold"]]
        aucs = [f["auc"] for f in folds]
        rec["cv5_bf16"] = {"mean_auc": round(float(np.mean(aucs)), 4), "std_auc": round(float(np.std(aucs)), 4),
                           "folds": folds, "seconds": round(time.time() - t0, 1)}
        print(json.dumps({"stage": "cv5_bf16", **rec["cv5_bf16"]}), flush=True)
    runs = [] if (args.no_train or args.all_folds) else ["bf16"] + (["fp32"] if args.fp32 else [])
    for dt in runs:
        mc = C.default("model_cml")
        mc.runtime.compute_dtype = dt
        if args.epochs:
            mc["epochs"] = int(args.epochs)
        if dev.type == "cuda":
            torch.cuda.reset_peak_memory_stats()
        t0 = time.time()
        res = run_cv(pc, mc, ws, folds=5, device=dev, store=store, fold_ids=[args.fold], verbose=2)
        f = res["per_fold"][0]
        secs = time.time() - t0
        out = {"auc": round(f["auc"], 4), "mcc": round(f["mcc"], 4), "n_train": f["n_train"], "n_test": f["n_test"],
               "test_pos_rate": round(f["test_pos_rate"], 4), "epochs": len(f["loss_curve"]),
               "loss_curve": f["loss_curve"], "fold_s": round(secs, 1),
               "train_windows_per_s_incl_eval": round(f["n_train"] * len(f["loss_curve"]) / secs, 1)}
        if dev.type == "cuda":
            out["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated() / 1e9, 3)
        rec[f"fold{args.fold}_{dt}"] = out
        print(json.dumps({"stage": f"fold_{dt}", **out}), flush=True)
    rec["host_peak_rss_gb"] = round(_rss_gb(), 2)
    line = json.dumps(rec)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
