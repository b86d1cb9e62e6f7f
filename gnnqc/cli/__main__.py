"""Command line entry points (the reference's notebook pipeline).

    python -m gnnqc.cli synth      --ds cml --out data/cml_raw.nc [--sensors 23 --days 28 --flagged 1]
    python -m gnnqc.cli preprocess --ds cml [--synthetic] [--tfrecords]
    python -m gnnqc.cli train      --ds cml [--baseline] [--synthetic] [--set model.epochs=5]
    python -m gnnqc.cli evaluate   --ds cml --model-dir models/model_cml
    python -m gnnqc.cli cv         --ds cml --folds 5 [--baseline|--both] [--synthetic]
    python -m gnnqc.cli explain    --ds cml --model-dir models/model_cml      (integrated gradients)
    python -m gnnqc.cli analyse    --xai-dir xplain/ig                         (attribution analysis)

Multi-GPU: launch with ``torchrun --nproc-per-node N -m gnnqc.cli ...`` (one rank per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np


def _windows(args, pc):
    from ..data.preprocessing import create_windows_dataset
    from .common import make_raw
    raw = make_raw(args, pc)
    return create_windows_dataset(pc, raw=raw)


def cmd_synth(args):
    from .common import load_configs, make_raw
    pc, _ = load_configs(args)
    args.synthetic = True
    ds = make_raw(args, pc)
    out = args.out or pc.raw_dataset_path
    ds.to_netcdf(out)
    print(json.dumps({"written": out, "dims": ds.dims}))


def cmd_preprocess(args):
    from ..data.preprocessing import create_sensors_ncfiles, create_tfrecords_dataset, create_windows_dataset
    from .common import load_configs, make_raw
    pc, _ = load_configs(args)
    raw = make_raw(args, pc)
    if pc.get("per_sensor", pc.ds_type == "cml") and pc.get("create_nc_files", True):
        paths = create_sensors_ncfiles(raw, pc)
        print(f"wrote {len(paths)} neighbourhood files to {pc.ncfiles_dir}")
    ws = create_windows_dataset(pc, raw=raw)
    out = create_tfrecords_dataset(pc, ws, write_records=args.tfrecords, max_records=args.max_records)
    print(json.dumps({"windows": ws.n_windows, "groups": len(ws.groups), "positive_rate":
                      float(np.mean(ws.labels_flat())), "out": out}))


def cmd_train(args):
    from ..ckpt import save_model
    from ..data.preprocessing import create_batched_dataset, load_dataset
    from ..data.store import DeviceStore
    from ..eval import calculate_metrics, calculate_threshold
    from ..models import create_model
    from ..parallel import dist as D
    from ..train import flatten_predictions, predict, train_model
    from .common import load_configs, resolve_device
    pc, mc = load_configs(args)
    dev = resolve_device(args.device)
    ws = _windows(args, pc)
    norm = pc.get("normalization") or ("rolling_median" if pc.ds_type == "cml" else "scale_range")
    store = DeviceStore(ws, norm, pc.graph, device=dev)
    tr, va, te = load_dataset(pc, ws)
    kinds = [False, True] if args.both else [args.baseline]
    for baseline in kinds:
        import torch
        torch.manual_seed(args.seed)
        model = create_model(mc, pc, baseline=baseline).to(dev)
        tl, pc, _ = create_batched_dataset(tr, pc, store, rank=D.rank(), world_size=D.world_size(), baseline=baseline)
        vl, _, _ = create_batched_dataset(va, pc, store, shuffle=False, baseline=baseline, rank=D.rank(),
                                          world_size=D.world_size())
        out_dir = (mc.baseline_model.model_path if baseline else mc.model_path)
        hist, model = train_model(model, mc, pc, tl, vl if len(va) else None, baseline=baseline, store=store,
                                  checkpoint_path=os.path.join(out_dir, "checkpoint"),
                                  log_path=os.path.join(out_dir, "train_log.jsonl"),
                                  resume_dir=os.path.join(out_dir, "resume") if args.resume_every else None,
                                  resume=args.resume)
        if D.is_main():
            save_model(model, out_dir, preproc_config=pc)
        if len(te):
            thr = 0.5
            if len(va):
                thr, _ = calculate_threshold(mc, pc, vl, model, baseline=baseline, store=store)
            tel, _, _ = create_batched_dataset(te, pc, store, shuffle=False, baseline=baseline, rank=D.rank(),
                                               world_size=D.world_size())
            r = flatten_predictions(predict(model, store, tel, baseline))
            if D.is_main():
                mcc, prec, rec, acc, auc, *_ = calculate_metrics(r["y"] > 0.5, r["p"] > thr, r["p"], mc, thr,
                                                                 baseline=baseline)
                print(json.dumps({"model": "baseline" if baseline else "gcn", "threshold": thr, "auc": auc,
                                  "mcc": mcc, "precision": prec, "recall": rec, "accuracy": acc}))
    D.destroy()


def cmd_evaluate(args):
    from ..ckpt import load_model
    from ..data.preprocessing import create_batched_dataset, load_dataset
    from ..data.store import DeviceStore
    from ..eval import calculate_metrics, calculate_threshold
    from ..train import flatten_predictions, predict
    from .common import load_configs, resolve_device
    pc, mc = load_configs(args)
    dev = resolve_device(args.device)
    model = load_model(args.model_dir, device=dev)
    baseline = type(model).__name__ == "BaselineClassifier"
    ws = _windows(args, pc)
    store = DeviceStore(ws, model.model_normalization if not baseline else model.normalization, pc.graph, device=dev)
    tr, va, te = load_dataset(pc, ws)
    vl, _, _ = create_batched_dataset(va, pc, store, shuffle=False, baseline=baseline)
    thr, idx = calculate_threshold(mc, pc, vl, model, baseline=baseline, store=store)
    tel, _, _ = create_batched_dataset(te, pc, store, shuffle=False, baseline=baseline)
    r = flatten_predictions(predict(model, store, tel, baseline))
    mcc, prec, rec, acc, auc, *_ = calculate_metrics(r["y"] > 0.5, r["p"] > thr, r["p"], mc, thr, baseline=baseline)
    print(json.dumps({"threshold": thr, "auc": auc, "mcc": mcc, "precision": prec, "recall": rec, "accuracy": acc}))


def cmd_cv(args):
    from ..data.store import DeviceStore
    from ..parallel import dist as D
    from ..train.cv import run_cv
    from .common import load_configs, resolve_device
    pc, mc = load_configs(args)
    dev = resolve_device(args.device)
    ws = _windows(args, pc)
    norm = pc.get("normalization") or ("rolling_median" if pc.ds_type == "cml" else "scale_range")
    store = DeviceStore(ws, norm, pc.graph, device=dev)
    if D.is_main():
        print(json.dumps({"windows": ws.n_windows, "positive_rate": float(np.mean(ws.labels_flat())),
                          "groups": len(ws.groups)}), flush=True)
    kinds = [False, True] if args.both else [args.baseline]
    out = {}
    for baseline in kinds:
        s = run_cv(pc, mc, ws, folds=args.folds, baseline=baseline, store=store, seed=args.seed,
                   gap_days=args.gap_days, log_path=args.log, max_folds=args.max_folds,
                   fold_ids=[int(v) for v in args.fold_ids.split(",")] if args.fold_ids else None,
                   fold_per_rank=args.fold_per_gpu)
        out[s["model"]] = s
        if D.is_main():
            print(json.dumps({"model": s["model"], "mean_auc": round(s["mean_auc"], 4), "std_auc": round(s["std_auc"], 4),
                              "mean_mcc": round(s["mean_mcc"], 4),
                              "fold_auc": [round(r["auc"], 4) for r in s["per_fold"]]}), flush=True)
    if args.out and D.is_main():
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    D.destroy()


def cmd_explain(args):
    from ..xai.ig import run_explainer
    run_explainer(args)


def cmd_analyse(args):
    from ..xai.analyse import run_analyser
    run_analyser(args)


def main(argv=None):
    from .common import add_common
    ap = argparse.ArgumentParser(prog="gnnqc")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = add_common(sub.add_parser("synth", help="write a synthetic raw dataset"))
    p.add_argument("--out", default=None)
    p.set_defaults(fn=cmd_synth)
    p = add_common(sub.add_parser("preprocess", help="neighbourhood files + window index (+ TFRecords)"))
    p.add_argument("--tfrecords", action="store_true", help="also write SequenceExample TFRecord files")
    p.add_argument("--max-records", type=int, default=None)
    p.set_defaults(fn=cmd_preprocess)
    p = add_common(sub.add_parser("train", help="train GCN (or baseline), save, evaluate on test"))
    p.add_argument("--baseline", action="store_true")
    p.add_argument("--both", action="store_true")
    p.add_argument("--resume", action="store_true",
                   help="continue from <model_path>/resume/resume.pt if present (e.g. under torchrun --max-restarts)")
    p.add_argument("--resume-every", type=int, default=1, help="full-state checkpoint every K epochs (0: off)")
    p.set_defaults(fn=cmd_train)
    p = add_common(sub.add_parser("evaluate", help="threshold on val + test metrics of a saved model"))
    p.add_argument("--model-dir", required=True)
    p.set_defaults(fn=cmd_evaluate)
    p = add_common(sub.add_parser("cv", help="k-fold cross validation (mean ROC-AUC)"))
    p.add_argument("--folds", type=int, default=5)
    p.add_argument("--baseline", action="store_true")
    p.add_argument("--both", action="store_true")
    p.add_argument("--gap-days", type=int, default=None)
    p.add_argument("--max-folds", type=int, default=None, help="only run the first K folds")
    p.add_argument("--fold-ids", default=None, help="comma list: only run these folds (e.g. 0,1)")
    p.add_argument("--fold-per-gpu", action="store_true",
                   help="with N processes: each GPU trains its own folds (no DP all-reduce); results merged")
    p.add_argument("--out", default=None)
    p.add_argument("--log", default=None)
    p.set_defaults(fn=cmd_cv)
    p = add_common(sub.add_parser("explain", help="integrated gradients for a saved model"))
    p.add_argument("--model-dir", required=True)
    p.add_argument("--xai-config", default=None)
    p.add_argument("--out-dir", default=None)
    p.add_argument("--max-batches", type=int, default=None)
    p.add_argument("--shard", default=None, help="i/n: process every n-th batch starting at i (like a SLURM array task)")
    p.set_defaults(fn=cmd_explain)
    p = add_common(sub.add_parser("analyse", help="aggregate / plot saved IG attributions"))
    p.add_argument("--xai-dir", required=True)
    p.add_argument("--xai-config", default=None)
    p.set_defaults(fn=cmd_analyse)
    args = ap.parse_args(argv)
    args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
