"""``train_model`` and callbacks (``libs/fit_model.py``, ``xai/libs/fit_model.py``).

Keras ``fit`` semantics reproduced on the device engine:

* optimiser by name with ``learning_rate`` (adam / sgd / rmsprop);
* loss ``binary_crossentropy`` with ``class_weight`` from :func:`calculate_weights`;
* metrics recall, binary_accuracy, precision, auc, tp, fp, tn, fn (+ ``val_`` twins);
* ``EarlyStopping(monitor='val_loss' | 'loss' in CV mode, patience, restore_best_weights)``;
* ``ModelCheckpoint(save_best_only)`` -> :mod:`gnnqc.ckpt`;
* step LR schedule: unchanged before ``after_epochs``, then ``lr *= rate`` each epoch;
* ``PlotLossesKeras`` -> JSONL log (+ PNG loss curve at the end); wandb if importable
  and ``model_config.wandb.use``.

Returns ``(history, model)`` like the reference; ``history.history`` is the dict of
per-epoch metric lists.
"""
from __future__ import annotations

import copy
import json
import os
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops.optim import make_optimizer
from ..parallel import dist as D
from .engine import Trainer
from .loss import calculate_weights


class History:
    def __init__(self):
        self.history: Dict[str, List[float]] = {}
        self.epoch: List[int] = []

    def append(self, epoch: int, logs: Dict[str, float]):
        self.epoch.append(epoch)
        for k, v in logs.items():
            self.history.setdefault(k, []).append(float(v))


class Callback:
    def on_train_begin(self, state):
        pass

    def on_epoch_begin(self, epoch, state):
        pass

    def on_epoch_end(self, epoch, logs, state):
        pass

    def on_train_end(self, state):
        pass


class LearningRateScheduler(Callback):
    def __init__(self, after_epochs: int, rate: float):
        self.after_epochs, self.rate = int(after_epochs), float(rate)

    def on_epoch_begin(self, epoch, state):
        opt = state["optimizer"]
        if epoch >= self.after_epochs:
            opt.lr = opt.lr * self.rate


class EarlyStopping(Callback):
    def __init__(self, monitor: str = "val_loss", patience: int = 10, restore_best_weights: bool = True):
        self.monitor, self.patience, self.restore = monitor, int(patience), restore_best_weights
        self.best = np.inf
        self.wait = 0
        self.best_state = None

    def on_epoch_end(self, epoch, logs, state):
        cur = logs.get(self.monitor)
        if cur is None:
            return
        if cur < self.best:
            self.best = cur
            self.wait = 0
            if self.restore:
                self.best_state = copy.deepcopy({k: v.detach().clone() for k, v in state["model"].state_dict().items()})
        else:
            self.wait += 1
            if self.wait >= self.patience:
                state["stop"] = True
                if self.restore and self.best_state is not None:
                    state["model"].load_state_dict(self.best_state)

    def state_dict(self):
        return {"best": float(self.best), "wait": int(self.wait),
                "best_state": {k: v.cpu() for k, v in self.best_state.items()} if self.best_state else None}

    def load_state_dict(self, sd):
        self.best, self.wait = float(sd["best"]), int(sd["wait"])
        self.best_state = sd.get("best_state")


class ResumeCallback(Callback):
    """Per-epoch full-state checkpoint for ``train_model(resume=...)``."""

    def __init__(self, path: str, every: int = 1):
        self.path, self.every = path, max(1, int(every))

    def on_epoch_end(self, epoch, logs, state):
        if (epoch + 1) % self.every == 0:
            from .resilience import save_resume
            save_resume(self.path, state["model"], state["optimizer"], epoch, state.get("history"),
                        state.get("callbacks", ()))


class ModelCheckpoint(Callback):
    def __init__(self, path: str, monitor: str = "val_loss", save_best_only: bool = True, preproc_config=None):
        self.path, self.monitor, self.best_only = path, monitor, save_best_only
        self.best = np.inf
        self.preproc_config = preproc_config

    def on_epoch_end(self, epoch, logs, state):
        cur = logs.get(self.monitor, np.inf)
        if (not self.best_only) or cur < self.best:
            self.best = min(self.best, cur)
            if D.is_main():
                from ..ckpt import save_model
                save_model(state["model"], self.path, optimizer=state["optimizer"], epoch=epoch,
                           preproc_config=self.preproc_config)


class JSONLLogger(Callback):
    """Rank-0 metrics stream (stands in for livelossplot's PlotLossesKeras)."""

    def __init__(self, path: Optional[str], plot: bool = True):
        self.path, self.plot = path, plot
        self.rows = []

    def on_epoch_end(self, epoch, logs, state):
        row = {"epoch": epoch, "lr": state["optimizer"].lr, **logs}
        self.rows.append(row)
        if self.path and D.is_main():
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            with open(self.path, "a") as f:
                f.write(json.dumps(row) + "\n")

    def on_train_end(self, state):
        if not (self.plot and self.path and D.is_main() and self.rows):
            return
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except Exception:   # pragma: no cover
            return
        keys = [k for k in ("loss", "auc", "recall", "precision") if k in self.rows[0]]
        fig, axes = plt.subplots(1, len(keys), figsize=(4 * len(keys), 3))
        axes = np.atleast_1d(axes)
        ep = [r["epoch"] for r in self.rows]
        for ax, k in zip(axes, keys):
            ax.plot(ep, [r[k] for r in self.rows], label=k)
            if "val_" + k in self.rows[0]:
                ax.plot(ep, [r["val_" + k] for r in self.rows], label="val_" + k)
            ax.set_title(k)
            ax.legend()
        fig.tight_layout()
        fig.savefig(os.path.splitext(self.path)[0] + ".png", dpi=80)
        plt.close(fig)


class WandbCallback(Callback):
    """Optional wandb logging of the XAI trainer (``xai/libs/fit_model.py:72-111``)."""

    def __init__(self, project: str, config: dict, tags=None):
        import wandb  # noqa: F401  (raises if absent)
        self.wandb = wandb
        self.run = wandb.init(project=project, config=config, tags=tags)

    def on_epoch_end(self, epoch, logs, state):
        self.wandb.log({"epoch": epoch, **logs})

    def on_train_end(self, state):
        self.wandb.finish()


class MCCCustom(Callback):
    """Epoch-end MCC on train / validation predictions (``libs/fit_model.py:28-58``)."""

    def __init__(self, store, train_loader, val_loader=None, baseline=False):
        self.store, self.train, self.val, self.baseline = store, train_loader, val_loader, baseline

    def on_epoch_end(self, epoch, logs, state):
        from ..eval.metrics import mcc_metric
        from .engine import flatten_predictions, predict
        r = flatten_predictions(predict(state["model"], self.store, self.train, self.baseline))
        logs["MCC_score_train"] = round(mcc_metric(r["y"], r["p"]), 5)
        if self.val is not None:
            r = flatten_predictions(predict(state["model"], self.store, self.val, self.baseline))
            logs["MCC_score_val"] = round(mcc_metric(r["y"], r["p"]), 5)


def train_model(model, model_config, preproc_config, train_dataset_batched, val_dataset_batched=None,
                baseline: bool = False, classes_weights=None, labels=None, CV: bool = False,
                split_numb: Optional[int] = None, store=None, callbacks: Optional[List[Callback]] = None,
                checkpoint_path: Optional[str] = None, log_path: Optional[str] = None, use_graph: Optional[bool] = None,
                verbose: int = 1, resume_dir: Optional[str] = None, resume: bool = False):
    """Fit ``model`` on a :class:`~gnnqc.data.store.DeviceLoader` (reference signature + extras).

    ``resume_dir``: write a full-state ``resume.pt`` there after every epoch;
    ``resume=True``: continue from it if present (see :mod:`gnnqc.train.resilience`)."""
    store = store or train_dataset_batched.store
    if classes_weights is None:
        if labels is None and model_config.get("weight_classes", {}).get("calculate", False):
            labels = store.labels(train_dataset_batched.ids).cpu().numpy()
        classes_weights = calculate_weights(model_config, labels)
    runtime = model_config.get("runtime") or {}
    opt = make_optimizer(model_config.get("optimizer", "adam"), model.parameters(),
                         model_config.get("learning_rate", 1e-3), guard=bool(runtime.get("nonfinite_guard", True)))
    D.broadcast_module(model)
    if use_graph is None:
        use_graph = bool(runtime.get("hip_graphs", True))
    trainer = Trainer(model, store, opt, classes_weights, baseline, use_graph=use_graph,
                      batch_size=train_dataset_batched.batch_size)
    monitor = "loss" if (CV or val_dataset_batched is None) else "val_loss"
    cbs: List[Callback] = [EarlyStopping(monitor, model_config.get("es_patience", 10), True)]
    if checkpoint_path:
        cbs.append(ModelCheckpoint(checkpoint_path, monitor, True, preproc_config))
    sched = model_config.get("learning_learn_scheduler") or {}
    if sched.get("use", False):
        cbs.append(LearningRateScheduler(sched.get("after_epochs", 5), sched.get("rate", 0.95)))
    cbs.append(JSONLLogger(log_path, plot=True))
    wb = model_config.get("wandb") or {}
    if wb.get("use", False):
        try:
            cfg = {**dict(preproc_config), **dict(model_config), "classes_weights": classes_weights,
                   "split_numb": split_numb}
            cbs.append(WandbCallback(wb.get("project", "gnnqc"), json.loads(json.dumps(cfg, default=str)),
                                     wb.get("tags")))
        except Exception as e:   # wandb absent: keep training, say so
            if verbose:
                print(f"wandb disabled: {e}")
    cbs += list(callbacks or [])
    resume_dir = resume_dir or runtime.get("resume_dir")
    saver = ResumeCallback(resume_dir, runtime.get("resume_every", 1)) if resume_dir else None
    history = History()
    state = {"model": model, "optimizer": opt, "stop": False, "trainer": trainer, "history": history,
             "callbacks": cbs}
    start_epoch = 0
    if resume and resume_dir:
        from .resilience import load_resume, restore
        rs = load_resume(resume_dir)
        if rs is not None:
            start_epoch = restore(rs, model, opt, history, cbs)
            trainer.global_step = opt.iterations
            if verbose and D.is_main():
                print(f"resumed from {resume_dir} at epoch {start_epoch + 1}", flush=True)
    for cb in cbs:
        cb.on_train_begin(state)
    for epoch in range(start_epoch, int(model_config.get("epochs", 10))):
        for cb in cbs:
            cb.on_epoch_begin(epoch, state)
        t0 = time.time()
        logs = trainer.train_epoch(train_dataset_batched, epoch)
        if val_dataset_batched is not None:
            logs.update(trainer.evaluate(val_dataset_batched, "val_"))
        logs["lr"] = opt.lr
        logs["epoch_time_s"] = time.time() - t0
        for cb in cbs:
            cb.on_epoch_end(epoch, logs, state)
        history.append(epoch, logs)
        if saver is not None:     # after every callback and the history: a consistent snapshot
            saver.on_epoch_end(epoch, logs, state)
        if verbose and D.is_main():
            shown = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items() if k in
                               ("loss", "auc", "recall", "precision", "val_loss", "val_auc", "lr", "epoch_time_s"))
            print(f"Epoch {epoch + 1}/{model_config.get('epochs', 10)} - {shown}", flush=True)
        if state["stop"]:
            break
    for cb in cbs:
        cb.on_train_end(state)
    model.trainer = None
    return history, model


__all__ = ["train_model", "calculate_weights", "History", "Callback", "EarlyStopping", "ModelCheckpoint",
           "LearningRateScheduler", "JSONLLogger", "WandbCallback", "MCCCustom", "ResumeCallback"]
