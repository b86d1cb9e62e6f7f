"""K-fold cross-validation driver.

The reference ships the splitter (``load_dataset_CV``, ``xai/libs/preprocessing_functions.py:804-836``)
and the CV-aware trainer (``train_model(CV=True)`` monitoring ``loss``,
``xai/libs/fit_model.py:94-99``) but not the fold loop behind the paper's
"mean ROC-AUC under 5-fold CV" headline (``README.md:10``). :func:`run_cv` is
that loop: for every fold, a fresh model is trained on the other folds and scored
on the held-out fold (exact ROC-AUC plus MCC / precision / recall / accuracy at
the fold's max-MCC threshold); the mean AUC is the headline metric.
"""
from __future__ import annotations

import json
import time
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from ..data.preprocessing import create_batched_dataset, load_dataset_CV
from ..data.store import DeviceStore
from ..eval import metrics as M
from ..models import BaselineClassifier, GCNClassifier
from ..parallel import dist as D
from .engine import flatten_predictions, predict
from .fit import train_model


def run_cv(preproc_config, model_config, windows, folds: Optional[int] = None, baseline: bool = False,
           device="cpu", seed: int = 0, store: Optional[DeviceStore] = None, gap_days: Optional[int] = None,
           verbose: int = 1, log_path: Optional[str] = None, max_folds: Optional[int] = None,
           fold_ids: Optional[List[int]] = None, fold_per_rank: bool = False,
           progress: Optional[Callable[[Dict], None]] = None) -> Dict:
    """``fold_ids`` runs only those folds (e.g. to spread a CV over several jobs; merge
    the per-fold JSONL lines with :func:`summarize_folds`). ``progress`` is called with each
    finished fold's result on the rank that ran it (e.g. a progress line on stderr).

    ``fold_per_rank`` (one process per GPU): instead of data-parallel training of every fold,
    rank r trains folds r, r + world, ... on its own GPU with no collective in its steps (the
    folds are independent - 5 folds on 8 GPUs finish in one fold's time, no all-reduce at all);
    the per-fold results are gathered on every rank at the end."""
    pc = preproc_config
    mc = model_config
    k = int(folds or pc.get("split_numb", 5))
    pc["split_numb"] = k
    pc.dataset["split_numb"] = k
    norm = pc.get("normalization") or ("rolling_median" if windows.ds_type == "cml" else "scale_range")
    store = store or DeviceStore(windows, norm, pc.graph, device=device)
    results: List[Dict] = []
    todo = list(range(min(k, int(max_folds)) if max_folds else k))
    if fold_ids is not None:
        todo = [int(f) for f in fold_ids if 0 <= int(f) < k]
    if fold_per_rank and D.global_world_size() > 1:
        mine = todo[D.global_rank()::D.global_world_size()]
        with D.local():
            part = run_cv(pc, mc, windows, k, baseline, device, seed, store, gap_days, verbose, None, None,
                          mine if mine else [], False, progress)["per_fold"] if mine else []
        merged = sorted((r for chunk in D.all_gather_object(part) for r in chunk), key=lambda r: r["fold"])
        if log_path and D.is_main():
            with open(log_path, "a") as f:
                for r in merged:
                    f.write(json.dumps(r) + "\n")
        return summarize_folds(merged, "baseline" if baseline else "gcn", windows.ds_type, k)
    rank, world = D.rank(), D.world_size()
    for fold in todo:
        t0 = time.time()
        tr, te, pcf = load_dataset_CV(pc, windows, fold, gap_days=gap_days)
        torch.manual_seed(seed + fold)
        model = (BaselineClassifier if baseline else GCNClassifier)(mc, pcf).to(store.device)
        train_loader, pcf, _ = create_batched_dataset(tr, pcf, store, shuffle=True, baseline=baseline, rank=rank,
                                                      world_size=world)
        test_loader, _, _ = create_batched_dataset(te, pcf, store, shuffle=False, baseline=baseline, rank=rank,
                                                   world_size=world)
        hist, model = train_model(model, mc, pcf, train_loader, None, baseline=baseline, CV=True, split_numb=fold,
                                  store=store, verbose=max(0, verbose - 1))
        r = flatten_predictions(predict(model, store, test_loader, baseline))
        y, p = r["y"] > 0.5, r["p"]
        if y.size:
            auc = M.roc_auc_score(y, p)
            thr = M.select_threshold(p, y, verbose=False)
            yp = p > thr
            scores = {"auc": auc, "mcc": M.matthews_corrcoef(y, yp), "precision": M.precision_score(y, yp),
                      "recall": M.recall_score(y, yp), "accuracy": M.accuracy_score(y, yp), "threshold": thr}
        else:       # no labelled window in the held-out fold (tiny data): no score, the mean skips it
            scores = {k2: float("nan") for k2 in ("auc", "mcc", "precision", "recall", "accuracy", "threshold")}
        res = {"fold": fold, **scores,
               "n_train": int(len(tr)), "n_test": int(len(te)), "test_pos_rate": float(y.mean()) if y.size else 0.0,
               "final_train_loss": float(hist.history["loss"][-1]), "seconds": time.time() - t0,
               "loss_curve": [round(float(v), 5) for v in hist.history["loss"]]}
        results.append(res)
        if progress is not None:
            progress(res)
        if verbose and D.is_main():
            print(json.dumps({k2: (round(v, 4) if isinstance(v, float) else v) for k2, v in res.items()
                              if k2 != "loss_curve"}), flush=True)
        if log_path and D.is_main():
            with open(log_path, "a") as f:
                f.write(json.dumps(res) + "\n")
    return summarize_folds(results, "baseline" if baseline else "gcn", windows.ds_type, k)


def summarize_folds(results: List[Dict], model: str, ds_type: str, folds: int) -> Dict:
    """Headline summary (mean / std ROC-AUC, mean MCC) of per-fold result dicts."""
    aucs = np.array([r["auc"] for r in results], dtype=np.float64)
    aucs = aucs[np.isfinite(aucs)]                 # (a fold without labelled windows has no score)
    mccs = np.array([r["mcc"] for r in results], dtype=np.float64)
    mccs = mccs[np.isfinite(mccs)]
    return {
        "model": model, "ds_type": ds_type, "folds": folds, "folds_run": sorted(int(r["fold"]) for r in results),
        "mean_auc": float(aucs.mean()) if aucs.size else float("nan"),
        "std_auc": float(aucs.std()) if aucs.size else float("nan"),
        "mean_mcc": float(mccs.mean()) if mccs.size else float("nan"),
        "per_fold": results,
    }


__all__ = ["run_cv", "summarize_folds"]
