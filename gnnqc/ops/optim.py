"""Flat-buffer optimisers.

All trainable parameters of a model are re-homed into ONE contiguous fp32
buffer (each ``Parameter.data`` becomes a view), and their ``.grad`` tensors into
a second one. Consequences on MI355X:

* the data-parallel gradient all-reduce is a single RCCL collective on one
  753 KB buffer (no per-tensor launches, no bucketing metadata);
* the Adam update is one HIP kernel over the whole buffer;
* lr / step live on the device, so the optimiser launch can be captured in a HIP
  graph and replayed while the LR schedule changes;
* non-finite guard (on by default): one extra kernel checks the
  (all-reduced) gradient buffer; a step with NaN/Inf gradients is skipped on the
  device - parameters, slots and the bias-correction step stay untouched - and
  counted in ``skipped_steps``. It lives inside the captured graph, so it costs no
  host synchronisation. In DP the all-reduce spreads a NaN to every rank, so all
  ranks skip the same step. The same guard rejects a step in which an LSTM chain kernel's
  bounded spin timed out (``gnnqc.ops.lstm.check_chain`` raises on it at epoch end).

Optimisers by name like ``libs/fit_model.py:71-74``: adam (Keras eps 1e-7,
"epsilon-hat" update), sgd, rmsprop (Keras defaults rho .9, eps 1e-7).
"""
from __future__ import annotations

from typing import Optional, Iterable, List

import torch


def flatten_parameters(params: Iterable[torch.nn.Parameter], align: int = 4):
    """Move params (and grads) into contiguous buffers; returns (flat_p, flat_g, slices)."""
    params = [p for p in params if p.requires_grad]
    if not params:
        raise ValueError("no trainable parameters")
    dev, dt = params[0].device, params[0].dtype
    sizes = []
    off = 0
    for p in params:
        n = p.numel()
        sizes.append((off, n))
        off += (n + align - 1) // align * align
    flat_p = torch.zeros(off, device=dev, dtype=dt)
    flat_g = torch.zeros(off, device=dev, dtype=dt)
    for p, (o, n) in zip(params, sizes):
        flat_p[o:o + n].copy_(p.data.reshape(-1))
        p.data = flat_p[o:o + n].view_as(p.data)
        p.grad = flat_g[o:o + n].view_as(p.data)
    return flat_p, flat_g, params


class FlatOptimizer:
    """Base: owns the flat buffers of a module's trainables."""

    grad_zeroed_by_step = False        # subclasses whose update clears flat_g override this

    def __init__(self, params, lr: float, guard: bool = True):
        self.flat_p, self.flat_g, self.params = flatten_parameters(params)
        dev = self.flat_p.device
        self.lr_t = torch.tensor([float(lr)], device=dev, dtype=torch.float32)
        self.step_t = torch.zeros(1, device=dev, dtype=torch.float32)   # applied steps (bias correction)
        self.iterations = 0                                              # attempted steps (host)
        self.guard = bool(guard)
        # [nonfinite count, ticket, ok flag, skipped steps, decision generation, overflowed elements
        # (adam_flagged), decision-wait timeouts (adam_guarded), -] (adam.hip grad_guard /
        # adam_guarded / adam_flagged)
        self.guard_state = torch.zeros(8, device=dev, dtype=torch.int32)
        self.guard_state[2] = 1
        # multi-step graphs (gnnqc.train.engine): a device batch cursor the update advances
        self.cursor: Optional[torch.Tensor] = None
        self.cursor_mod = 1
        from . import use_hip
        if use_hip(self.flat_p):
            # the chain control words the guard reads are allocated now: a first use inside a
            # graph capture (a model without the chain kernels) would be refused
            from .lstm import chain_ctl
            chain_ctl(dev)

    @property
    def skipped_steps(self) -> int:
        return int(self.guard_state[3].item())

    def check_update(self):
        """Raise if a workgroup of the one-launch guarded update gave up waiting for the step
        decision (adam.hip adam_guarded_kernel counts it in guard_state[6]): that step may have
        updated only part of the parameters. Synchronises."""
        n = int(self.guard_state[6].item())
        if n:
            self.guard_state[6:7].zero_()
            raise RuntimeError(f"guarded Adam: {n} workgroup(s) never saw the step decision (grid not co-resident: "
                               "another kernel held the CUs?); the parameters may be partially updated")

    def _begin_step(self, need_flag: bool = True):
        """Advance the step counter; with the guard, only if the gradients are finite.
        Returns the device ok flag (bool tensor) for eager updates (``need_flag``), or None."""
        self.iterations += 1
        if not self.guard:
            self.step_t.add_(1.0)
            return None
        from . import use_hip
        if use_hip(self.flat_g):
            from ..utils.native import hip_ops
            from .lstm import chain_ctl
            # a step whose LSTM chain kernel timed out (stale hand-off data) is rejected too
            hip_ops().grad_guard(self.flat_g, self.guard_state, self.step_t, chain_ctl(self.flat_g.device))
            # (a HIP update kernel reads the guard state itself: no bool conversion launch)
            return self.guard_state[2:3].bool() if need_flag else None
        ok = torch.isfinite(self.flat_g).all().reshape(1)
        self.step_t.add_(ok.float())
        self.guard_state[2:3].copy_(ok.int())
        self.guard_state[3:4].add_((~ok).int())
        return ok

    @property
    def lr(self) -> float:
        return float(self.lr_t.item())

    @lr.setter
    def lr(self, value: float):
        self.lr_t.fill_(float(value))

    def zero_grad(self):
        # grads are views into flat_g: never set them to None
        self.flat_g.zero_()

    def relink_grads(self):
        """Re-attach grads as views (autograd may have replaced .grad)."""
        off = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None or p.grad.data_ptr() != self.flat_g[off:off + n].data_ptr():
                g = self.flat_g[off:off + n].view_as(p.data)
                if p.grad is not None:
                    g.copy_(p.grad)
                p.grad = g
            off += (n + 3) // 4 * 4

    def views(self, flat: torch.Tensor) -> List[torch.Tensor]:
        """Per-parameter views of a flat buffer laid out like ``flat_p`` (slots, grads)."""
        out, off = [], 0
        for p in self.params:
            n = p.numel()
            out.append(flat[off:off + n].view_as(p.data))
            off += (n + 3) // 4 * 4
        return out

    def state_dict(self):
        return {"lr": self.lr, "iterations": self.iterations, "step": float(self.step_t.item()),
                "skipped_steps": self.skipped_steps}

    def load_state_dict(self, sd):
        self.lr = sd["lr"]
        self.iterations = int(sd["iterations"])
        self.step_t.fill_(float(sd.get("step", self.iterations)))
        self.guard_state[3] = int(sd.get("skipped_steps", 0))


class FlatAdam(FlatOptimizer):
    def __init__(self, params, lr: float = 1e-3, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-7,
                 weight_decay: float = 0.0, guard: bool = True):
        super().__init__(params, lr, guard)
        self.beta1, self.beta2, self.eps, self.wd = beta1, beta2, eps, weight_decay
        self.m = torch.zeros_like(self.flat_p)
        self.v = torch.zeros_like(self.flat_p)
        # the HIP update clears the gradient buffer once it has read it (no separate zero-fill
        # launch per training step); the trainer then skips zero_grad (grad_zeroed_by_step)
        self.zero_grad_in_step = self.flat_p.is_cuda
        # set by the trainer when EVERY kernel writing this model's gradients flags non-finite
        # values (chain control word 7): the update then decides from the flags (adam_flagged, no
        # grid-wide scan of the gradient buffer)
        self.flagged_producers = False
        # data parallel with the one-shot peer all-reduce (gnnqc.parallel.peer): a flag-driven step
        # reduces the gradients INSIDE the update launch (peer_allreduce.hip adam_peer); the trainer
        # then issues no separate collective
        self.peer = None

    @property
    def grad_zeroed_by_step(self) -> bool:
        from . import use_hip
        return self.zero_grad_in_step and use_hip(self.flat_p)

    def step(self, grad_scale: float = 1.0):
        from . import use_hip
        hip = use_hip(self.flat_p)
        if hip and self.guard and self.zero_grad_in_step:
            # guard + update (+ batch cursor) as ONE launch when the buffer fits a co-resident grid
            from ..utils.native import hip_ops
            from .lstm import chain_ctl
            if self.flagged_producers and self.peer is not None:
                pa = self.peer
                if hip_ops().adam_peer(self.flat_p, self.flat_g, self.m, self.v, self.lr_t, self.step_t, self.beta1,
                                       self.beta2, self.eps, float(grad_scale), self.wd, self.guard_state, self.cursor,
                                       int(self.cursor_mod), pa.bases, pa.region, pa.rank, pa.cap):
                    self.iterations += 1
                    return
                # more slices than the fused kernel's flag table: the two separate launches (the
                # trainer issued no collective for this step, so reduce here, reject bits first)
                hip_ops().chain_poison(self.flat_g, chain_ctl(self.flat_g.device))
                pa(self.flat_g)
            if self.flagged_producers:
                hip_ops().adam_flagged(self.flat_p, self.flat_g, self.m, self.v, self.lr_t, self.step_t, self.beta1,
                                       self.beta2, self.eps, float(grad_scale), self.wd, self.guard_state,
                                       chain_ctl(self.flat_g.device), self.cursor, int(self.cursor_mod))
                self.iterations += 1
                return
            if hip_ops().adam_guarded(self.flat_p, self.flat_g, self.m, self.v, self.lr_t, self.step_t, self.beta1,
                                      self.beta2, self.eps, float(grad_scale), self.wd, self.guard_state,
                                      chain_ctl(self.flat_g.device), self.cursor, int(self.cursor_mod)):
                self.iterations += 1
                return
        if self.cursor is not None:
            raise RuntimeError("a device batch cursor needs the single-launch HIP Adam")
        ok = self._begin_step(need_flag=not hip)
        if hip:
            from ..utils.native import hip_ops
            hip_ops().adam_step(self.flat_p, self.flat_g, self.m, self.v, self.lr_t, self.step_t, self.beta1,
                                self.beta2, self.eps, float(grad_scale), self.wd,
                                self.guard_state if self.guard else None, self.zero_grad_in_step)
            return
        with torch.no_grad():
            g = self.flat_g * grad_scale
            if self.wd:
                g = g + self.wd * self.flat_p
            m = self.m * self.beta1 + g * (1 - self.beta1)
            v = self.v * self.beta2 + g * g * (1 - self.beta2)
            t = self.step_t
            alpha = self.lr_t * torch.sqrt(1 - self.beta2 ** t) / (1 - self.beta1 ** t)
            p = self.flat_p - alpha * m / (torch.sqrt(v) + self.eps)
            _commit(ok, (self.m, m), (self.v, v), (self.flat_p, p))

    def state_dict(self):
        sd = super().state_dict()
        sd.update(m=self.m.detach().cpu(), v=self.v.detach().cpu())
        return sd

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        self.m.copy_(sd["m"].to(self.m.device))
        self.v.copy_(sd["v"].to(self.v.device))

    def slots(self) -> List[torch.Tensor]:
        return [self.m, self.v]


class FlatSGD(FlatOptimizer):
    def __init__(self, params, lr: float = 0.01, momentum: float = 0.0):
        super().__init__(params, lr)
        self.momentum = momentum
        self.buf = torch.zeros_like(self.flat_p) if momentum else None

    def step(self, grad_scale: float = 1.0):
        ok = self._begin_step()
        with torch.no_grad():
            g = self.flat_g * grad_scale
            if self.buf is not None:
                buf = self.buf * self.momentum - self.lr_t * g
                _commit(ok, (self.buf, buf), (self.flat_p, self.flat_p + buf))
            else:
                _commit(ok, (self.flat_p, self.flat_p - self.lr_t * g))

    def slots(self):
        return [self.buf] if self.buf is not None else []


class FlatRMSprop(FlatOptimizer):
    def __init__(self, params, lr: float = 1e-3, rho: float = 0.9, eps: float = 1e-7):
        super().__init__(params, lr)
        self.rho, self.eps = rho, eps
        self.ms = torch.zeros_like(self.flat_p)

    def step(self, grad_scale: float = 1.0):
        ok = self._begin_step()
        with torch.no_grad():
            g = self.flat_g * grad_scale
            ms = self.ms * self.rho + g * g * (1 - self.rho)
            _commit(ok, (self.ms, ms), (self.flat_p, self.flat_p - self.lr_t * g / (torch.sqrt(ms) + self.eps)))

    def slots(self):
        return [self.ms]


def _commit(ok, *pairs):
    """dst <- new for each (dst, new) pair, unless the device flag ``ok`` is False."""
    for dst, new in pairs:
        if ok is None:
            dst.copy_(new)
        else:
            dst.copy_(torch.where(ok, new, dst))


def make_optimizer(name: str, params, lr: float, guard: bool = True):
    name = (name or "adam").lower()
    if name == "adam":
        return FlatAdam(params, lr, guard=guard)
    if name == "sgd":
        o = FlatSGD(params, lr)
    elif name == "rmsprop":
        o = FlatRMSprop(params, lr)
    else:
        raise ValueError(f"unknown optimizer {name}")
    o.guard = bool(guard)
    return o


__all__ = ["flatten_parameters", "FlatAdam", "FlatSGD", "FlatRMSprop", "make_optimizer"]
