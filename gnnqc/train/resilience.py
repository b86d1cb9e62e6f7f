"""Failure handling around training: resume checkpoints, fault injection.

The reference has no fault tolerance; Keras ``EarlyStopping(restore_best_weights)``
(``libs/fit_model.py:89``) is its only related mechanism. Here:

* :class:`ResumeCheckpoint` writes ``<dir>/resume.pt`` at the end of every epoch
  (rank 0, atomically via rename): model state (incl. BN statistics), optimiser
  state (Adam slots, lr, attempted/applied/skipped steps), callback state (early
  stopping), the history so far and every RNG stream (python, numpy, torch CPU and
  GPU). ``train_model(resume=...)`` restarts at the next epoch. The data cursor is
  implicit: :class:`~gnnqc.data.store.DeviceLoader` derives each epoch's order from
  ``(seed, epoch)`` only, so a resumed run sees exactly the batches it would have seen.
  With ``torchrun --max-restarts N`` and ``resume="auto"`` a crashed job restarts
  from its last completed epoch (elastic restart of the same world size).
* Non-finite gradients never reach the weights: the optimiser's device-side guard
  (:mod:`gnnqc.ops.optim`, ``grad_guard`` in ``csrc/kernels/adam.hip``) skips the step;
  the per-epoch count is logged as ``skipped_steps``.
* :class:`FaultInjector` (env driven, for tests and drills):
  ``GNNQC_FI_KILL_RANK_AT_STEP="<rank>:<step>"`` (or ``"<step>"`` for rank 0) ends that
  rank with exit code :data:`FI_EXIT_CODE` right after global step ``<step>``;
  ``GNNQC_FI_NAN_AT_STEP="<step>[,<step>...]"`` poisons the gradient of those steps with
  a NaN (exercises the guard, also inside a captured HIP graph).
"""
from __future__ import annotations

import os
import random
import sys
from typing import Optional

import numpy as np
import torch

from ..parallel import dist as D

FI_EXIT_CODE = 75
RESUME_FILE = "resume.pt"


# ------------------------------------------------------------------ RNG state
def rng_state() -> dict:
    st = {"python": _py_state(random.getstate()), "torch": torch.get_rng_state()}
    name, keys, pos, has_gauss, cached = np.random.get_state()
    st["numpy"] = {"keys": torch.from_numpy(np.asarray(keys, dtype=np.int64)), "pos": int(pos),
                   "has_gauss": int(has_gauss), "cached": float(cached)}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = [s for s in torch.cuda.get_rng_state_all()]
    return st


def set_rng_state(st: dict):
    random.setstate(_py_unstate(st["python"]))
    torch.set_rng_state(st["torch"])
    n = st["numpy"]
    np.random.set_state(("MT19937", n["keys"].numpy().astype(np.uint32), n["pos"], n["has_gauss"], n["cached"]))
    if "cuda" in st and torch.cuda.is_available():
        states = st["cuda"][:torch.cuda.device_count()]
        for i, s in enumerate(states):
            torch.cuda.set_rng_state(s, i)


def _py_state(s):
    version, internal, gauss = s
    return {"version": version, "internal": list(internal), "gauss": gauss}


def _py_unstate(d):
    return d["version"], tuple(d["internal"]), d["gauss"]


# ------------------------------------------------------------------ checkpoint
def resume_path(path: str) -> str:
    return os.path.join(path, RESUME_FILE) if not path.endswith(".pt") else path


def save_resume(path: str, model, optimizer, epoch: int, history=None, callbacks=(), extra: Optional[dict] = None):
    """Atomic full-state checkpoint (rank 0 writes; other ranks return)."""
    if not D.is_main():
        return None
    f = resume_path(path)
    os.makedirs(os.path.dirname(f) or ".", exist_ok=True)
    cb_states = {}
    for i, cb in enumerate(callbacks):
        if hasattr(cb, "state_dict"):
            cb_states[f"{i}:{type(cb).__name__}"] = cb.state_dict()
    state = {
        "format": 1,
        "epoch": int(epoch),
        "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "optimizer": optimizer.state_dict(),
        "callbacks": cb_states,
        "history": {"epoch": list(history.epoch), "history": {k: list(v) for k, v in history.history.items()}}
        if history is not None else None,
        "rng": rng_state(),
        "world_size": D.world_size(),
        "extra": extra or {},
    }
    tmp = f + f".tmp{os.getpid()}"
    torch.save(state, tmp)
    os.replace(tmp, f)
    return f


def load_resume(path: str) -> Optional[dict]:
    """Full-state checkpoint or None if absent. Loaded with ``weights_only=True``."""
    f = resume_path(path)
    if not os.path.exists(f):
        return None
    return torch.load(f, map_location="cpu", weights_only=True)


def restore(state: dict, model, optimizer, history=None, callbacks=()) -> int:
    """Apply a :func:`load_resume` state; returns the first epoch still to run."""
    dev_state = {k: v for k, v in state["model"].items()}
    model.load_state_dict(dev_state)
    optimizer.load_state_dict(state["optimizer"])
    for i, cb in enumerate(callbacks):
        key = f"{i}:{type(cb).__name__}"
        if key in state.get("callbacks", {}) and hasattr(cb, "load_state_dict"):
            cb.load_state_dict(state["callbacks"][key])
    if history is not None and state.get("history"):
        history.epoch = list(state["history"]["epoch"])
        history.history = {k: list(v) for k, v in state["history"]["history"].items()}
    set_rng_state(state["rng"])
    return int(state["epoch"]) + 1


# ------------------------------------------------------------------ fault injection
class FaultInjector:
    def __init__(self, kill_rank: Optional[int] = None, kill_step: Optional[int] = None, nan_steps=()):
        self.kill_rank, self.kill_step = kill_rank, kill_step
        self.nan_steps = set(int(s) for s in nan_steps)

    @classmethod
    def from_env(cls) -> Optional["FaultInjector"]:
        k = os.environ.get("GNNQC_FI_KILL_RANK_AT_STEP", "").strip()
        n = os.environ.get("GNNQC_FI_NAN_AT_STEP", "").strip()
        if not k and not n:
            return None
        kr = ks = None
        if k:
            if ":" in k:
                a, b = k.split(":", 1)
                kr, ks = int(a), int(b)
            else:
                kr, ks = 0, int(k)
        nans = [int(s) for s in n.split(",") if s.strip()] if n else []
        return cls(kr, ks, nans)

    @property
    def poisons(self) -> bool:
        return bool(self.nan_steps)

    def nan_now(self, step: int) -> bool:
        return step in self.nan_steps

    def after_step(self, step: int):
        if self.kill_step is not None and step == self.kill_step and D.rank() == self.kill_rank:
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                torch.cuda.synchronize()
            sys.stdout.flush()
            sys.stderr.flush()
            print(f"[fault-injection] rank {D.rank()} exits after step {step}", file=sys.stderr, flush=True)
            os._exit(FI_EXIT_CODE)


__all__ = ["FI_EXIT_CODE", "FaultInjector", "save_resume", "load_resume", "restore", "rng_state", "set_rng_state",
           "resume_path"]
