"""Training / evaluation engine: device-resident, HIP-graph captured steps.

One training step = gather batch from HBM by window id -> forward -> weighted BCE
-> backward into the flat gradient buffer -> (DP) one RCCL all-reduce -> one Adam
kernel. On GPU the gather+forward+backward(+optimizer when world == 1) is
captured once into a HIP graph (``torch.cuda.CUDAGraph``) and replayed with new
window ids, so a step costs a handful of host calls regardless of the ~100 kernels
inside. Metric accumulators (loss sums, confusion counts, score histograms) live
on the device and are only read at epoch end - no host sync per step.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, Optional

import numpy as np
import torch

from ..eval import metrics as M
from ..ops.head import fused_head_loss
from ..ops.lstm import direct_grad_accumulation
from ..ops.metrics import score_histogram
from ..parallel import dist as D
from .loss import weighted_bce_with_logits
from .resilience import FaultInjector

_rf = torch.autograd.profiler.record_function

HIST_BINS = 1001


class MetricAccumulator:
    """Device-side running sums for the Keras compile metrics of ``libs/fit_model.py:79-86``."""

    def __init__(self, device):
        self.device = device
        self.sums = torch.zeros(6, device=device, dtype=torch.float64)   # loss*n, n, tp, tn, fp, fn
        self.hist = torch.zeros(2, HIST_BINS, device=device, dtype=torch.float32)

    def reset(self):
        self.sums.zero_()
        self.hist.zero_()

    @torch.no_grad()
    def update(self, loss, logits, y, mask):
        self.update_buffers(self.sums, self.hist, loss, logits, y, mask)

    @staticmethod
    @torch.no_grad()
    def update_buffers(sums, hist, loss, logits, y, mask):
        p = torch.sigmoid(logits.float()).reshape(-1)
        m = mask.float().reshape(-1)
        n = m.sum()
        pred = (p > 0.5).float()
        yy = (y.reshape(-1) > 0.5).float()
        vals = torch.stack([loss.detach().double() * n.double(), n.double(), (pred * yy * m).sum().double(),
                            ((1 - pred) * (1 - yy) * m).sum().double(), (pred * (1 - yy) * m).sum().double(),
                            ((1 - pred) * yy * m).sum().double()])
        sums.add_(vals)
        if hist is not None:
            hist.add_(score_histogram(p, yy, m, hist.shape[1]))

    def result(self, prefix: str = "") -> Dict[str, float]:
        sums = self.sums.clone()
        hist = self.hist.clone()
        D.all_reduce_(sums)
        D.all_reduce_(hist)
        s = sums.cpu().numpy()
        out = {"loss": float(s[0] / max(s[1], 1.0))}
        out.update(M.keras_metrics_from_counts(s[2], s[3], s[4], s[5]))
        out["auc"] = M.auc_from_hist(hist.cpu().numpy())
        return {prefix + k: v for k, v in out.items()}


def _graph_upload(graph) -> bool:
    """hipGraphUpload of a captured graph's executable on the current stream: the first replay of a
    graph otherwise pays the upload of its command buffers (done here, outside any timed region).
    False when the runtime or the executable handle is not available (no effect then)."""
    if graph is None or not torch.cuda.is_available():
        return False
    try:
        import ctypes
        exe = graph.raw_cuda_graph_exec()
        lib = ctypes.CDLL("libamdhip64.so")
        rc = lib.hipGraphUpload(ctypes.c_void_p(int(exe)), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        return rc == 0
    except Exception:         # (older torch / no HIP runtime: the first replay uploads instead)
        return False


class Trainer:
    def __init__(self, model, store, optimizer, class_weights: Optional[Dict[int, float]], baseline: bool = False,
                 use_graph: bool = True, batch_size: int = 128):
        self.model = model
        self.store = store
        self.opt = optimizer
        self.ds_type = store.ds_type
        self.baseline = baseline
        cw = class_weights or {0: 1.0, 1: 1.0}
        self.w0, self.w1 = float(cw[0]), float(cw[1])
        self.device = store.device
        self.world = D.world_size()
        self.use_graph = bool(use_graph) and self.device.type == "cuda"
        self.batch_size = int(batch_size)
        self.train_metrics = MetricAccumulator(self.device)
        self.graph = None
        # the step's gradient collective: with more than one rank, or forced on a one-rank process
        # group (GNNQC_DP_FORCE_COLLECTIVE=1: exercises the captured RCCL path on one GPU)
        self.collective = self.world > 1 or (os.environ.get("GNNQC_DP_FORCE_COLLECTIVE", "0") == "1"
                                             and D.is_initialized())
        # DP (or GNNQC_SPLIT_OPT_GRAPH=1): the optimizer runs after the all-reduce, so it
        # is captured as a second small graph instead of being launched eagerly each step
        self.split_opt = self.collective or os.environ.get("GNNQC_SPLIT_OPT_GRAPH", "0") == "1"
        # DP over RCCL: the all-reduce is captured INSIDE the multi-step graph (gather -> forward ->
        # backward -> chain-timeout poison -> all-reduce -> guarded Adam, graph_steps times per
        # replay): no host round trip per step. gloo (host collectives) stays eager per step.
        # opt-in one-shot peer all-reduce over xGMI (GNNQC_PEER_ALLREDUCE=1, gnnqc.parallel.peer):
        # a plain kernel, so it is captured in the step graph under any process-group backend
        self.peer = None
        if self.collective and self.device.type == "cuda":
            from ..parallel.peer import make_peer_allreduce
            self.peer = make_peer_allreduce(self.opt.flat_g.numel(), self.device)
        self.dp_graph = (self.collective and self.use_graph and (D.backend() == "nccl" or self.peer is not None)
                         and os.environ.get("GNNQC_DP_GRAPH", "1") == "1")
        # flag-driven steps reduce over the peers inside the Adam launch (one launch, one pass over the
        # gradients; GNNQC_PEER_FUSED_ADAM=0 keeps the separate all-reduce kernel)
        # (only after the fused kernel passed its own setup check against the two separate launches)
        if self.peer is not None and hasattr(self.opt, "peer") and os.environ.get("GNNQC_PEER_FUSED_ADAM", "1") == "1":
            from ..parallel.peer import check_fused_adam
            if check_fused_adam(self.peer, self.opt.flat_g.numel(), self.device, self.opt.beta1, self.opt.beta2,
                                self.opt.eps):
                self.opt.peer = self.peer
        self.opt_graph = None
        self.static_wids = torch.full((self.batch_size,), -1, dtype=torch.long, device=self.device)
        self.last_loss = torch.zeros((), device=self.device)
        self._one = torch.ones((), device=self.device)
        self.global_step = 0
        self.fault = FaultInjector.from_env()
        # NaN poisoning of the gradient (fault injection only: no extra kernel otherwise)
        self.poison = torch.zeros(1, device=self.device) if (self.fault and self.fault.poisons) else None
        # HIP-event timing of the DP all-reduce (read once per epoch)
        self._comm_events = []
        # multi-step graphs (train_steps): GNNQC_GRAPH_STEPS training steps per replay, walking a
        # device batch table with a device cursor the Adam launch advances (no host work, no id
        # copy and no graph-launch gap between those steps)
        self.graph_steps = max(1, int(os.environ.get("GNNQC_GRAPH_STEPS", "8")))
        self.multi_graph = None
        self._multi_key = None
        self.multi_graph1 = None            # (one-step graph of the same form: leftover steps)
        self._multi_key1 = None
        self._table = None
        self._cursor = torch.zeros(1, dtype=torch.long, device=self.device)
        self._graph_loss = None
        self._multi_loss = None
        # the store-fused CML step's gradient kernels all flag non-finite values: the update can
        # decide from those flags (one pass, no grid-wide barrier; gnnqc.ops.optim.FlatAdam). This is
        # the mode's eligibility; every step (and so every captured graph) re-checks that its backward
        # really wrote all gradients through flagging kernels (_body)
        self._flag_base = False
        if hasattr(self.opt, "flagged_producers"):
            was = self.model.training
            self.model.train()
            self._flag_base = bool(
                self.device.type == "cuda" and self._store_fused() and self.model.regularization_loss() is None
                and os.environ.get("GNNQC_FLAGGED_ADAM", "1") == "1")
            self.opt.flagged_producers = self._flag_base
            self.model.train(was)

    # ---------------------------------------------------------------- body
    def _loss(self, wids, metrics: Optional["MetricAccumulator"] = None):
        """(total, loss, logits, batch). With a fused-head model the loss, logits and
        the metric update come out of one HIP kernel (``gnnqc.ops.head``)."""
        if self._store_fused():
            # the gather is fused into the GCN kernel: no Batch is materialised
            loss, z = self.model.fused_store_loss(self.store, wids, self.w0, self.w1,
                                                  metrics.sums if metrics else None, metrics.hist if metrics else None)
            reg = self.model.regularization_loss()
            return (loss + reg if reg is not None else loss), loss, z, None
        with _rf("gnnqc.gather"):
            b = self.store.gather(wids)
            inputs = b.model_inputs(self.ds_type, self.baseline)
        fused = None
        if hasattr(self.model, "fused_loss") and not self.baseline:
            fused = self.model.fused_loss(inputs, b.y, b.y_mask, self.w0, self.w1, metrics.sums if metrics else None,
                                          metrics.hist if metrics else None)
        spec = self.model.head_spec() if (fused is None and hasattr(self.model, "head_spec")) else None
        if fused is not None:
            loss, z = fused
        elif spec is not None:
            dense, dense2, dense_out, a1, a2 = spec
            loss, z = fused_head_loss(self.model.features(inputs), dense, dense2, dense_out, a1, a2, b.y, b.y_mask,
                                      self.w0, self.w1, metrics.sums if metrics else None,
                                      metrics.hist if metrics else None)
        else:
            z = self.model.logits(inputs)
            loss = weighted_bce_with_logits(z, b.y, b.y_mask, self.w0, self.w1)
            if metrics is not None:
                metrics.update(loss, z, b.y, b.y_mask)
        reg = self.model.regularization_loss() if hasattr(self.model, "regularization_loss") else None
        total = loss + reg if reg is not None else loss
        return total, loss, z, b

    def _store_fused(self) -> bool:
        """The CML headed-chain model reads its batches straight from the store (one launch for
        gather + GCN + pooling, ``gnnqc.ops.gcn.gcn_pool_from_store``). Decided once per mode;
        ``GNNQC_STORE_GCN=0`` keeps the gather + generic GCN kernels (A/B measurements)."""
        key = bool(self.model.training)
        cache = self.__dict__.setdefault("_store_fused_cache", {})
        if key not in cache:
            cache[key] = (not self.baseline and os.environ.get("GNNQC_STORE_GCN", "1") == "1"
                          and hasattr(self.model, "store_fused_ok") and self.model.store_fused_ok(self.store))
        return cache[key]

    def _body(self, wids, with_opt: bool):
        # every training step ends with the optimizer update (here, or after the DP all-reduce);
        # a HIP Adam clears the gradient buffer as it reads it, so no zero-fill launch here
        # (the graph-capture warm-up, which runs no update, zeroes explicitly afterwards)
        if not self.opt.grad_zeroed_by_step:
            self.opt.zero_grad()
        with _rf("gnnqc.forward"):
            total, loss, z, b = self._loss(wids, self.train_metrics)
        from ..ops.lstm import unflagged_grad_writes
        n_unflagged = unflagged_grad_writes()
        with _rf("gnnqc.backward"), direct_grad_accumulation(True):
            total.backward(self._one)          # (a kept seed: no ones_like fill launch per step)
        if self._flag_base:
            # a gradient summed by autograd itself raised no flag: this step takes the scanning update
            self.opt.flagged_producers = unflagged_grad_writes() == n_unflagged
        if self.poison is not None:
            self.opt.flat_g[:1].add_(self.poison)
        self.last_loss = loss.detach()       # (a reference, not a copy launch: graph replays refresh it)
        if with_opt:
            with _rf("gnnqc.optimizer"):
                self.opt.step(grad_scale=1.0)

    def _capture(self):
        # warm up on a side stream (allocator + lazy init), then capture
        snap = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        with_opt = not self.split_opt
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._body(self.static_wids, with_opt=False)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        it0 = self.opt.iterations
        with torch.cuda.graph(self.graph):
            self._body(self.static_wids, with_opt=with_opt)
        if self.split_opt:
            self.opt_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.opt_graph):
                self.opt.step(grad_scale=1.0 / self.world)
        self.opt.iterations = it0          # capture runs nothing; replays count steps
        self._graph_loss = self.last_loss
        # undo warm-up side effects (BN running stats, metric sums)
        with torch.no_grad():
            for k, v in self.model.state_dict().items():
                v.copy_(snap[k])
        self.train_metrics.reset()
        self.opt.zero_grad()

    def _multi_ok(self) -> bool:
        return (self.use_graph and (not self.split_opt or self.dp_graph) and self.fault is None
                and self.graph_steps > 1 and getattr(self.opt, "zero_grad_in_step", False) and self.opt.guard)

    def _reduce_grads(self):
        """The DP gradient collective: a rank whose LSTM chain timed out this step poisons its
        gradient first (so every rank's guard rejects the step), then ONE SUM all-reduce of the
        flat 753 KB buffer. Not bucketed and not overlapped with the backward on purpose: the
        cross-CU chain kernels assume no other kernel shares the device while they run, and a
        single small collective is latency-bound on xGMI, so splitting it only adds latency."""
        if self.peer_fused():
            return                # the update launch reduces (and carries the reject bits) itself
        if self.device.type == "cuda":
            from ..ops.lstm import chain_ctl
            from ..utils.native import hip_ops
            hip_ops().chain_poison(self.opt.flat_g, chain_ctl(self.device))
        self._all_reduce_flat()

    def peer_fused(self) -> bool:
        """Whether this step's gradient reduction runs inside the Adam launch (adam_peer)."""
        return getattr(self.opt, "peer", None) is not None and bool(getattr(self.opt, "flagged_producers", False))

    def _all_reduce_flat(self):
        if self.peer is not None:
            self.peer(self.opt.flat_g)
        else:
            D.all_reduce_(self.opt.flat_g, force=True)

    @torch.no_grad()
    def measure_allreduce(self, n: int = 20) -> Optional[float]:
        """Mean time (us) of the step's gradient all-reduce run on its own (HIP events around each
        of ``n`` eager collectives); for the in-graph DP layout, whose collectives cannot be timed
        one by one. The gradient buffer is zero between steps (Adam clears it), so this changes
        nothing."""
        if not self.collective or self.device.type != "cuda":
            return None
        self._all_reduce_flat()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for a, b in ev:
            a.record()
            self._all_reduce_flat()
            b.record()
        torch.cuda.synchronize()
        self.opt.zero_grad()
        return 1e3 * sum(a.elapsed_time(b) for a, b in ev) / n

    def _capture_multi(self, nrows: int, steps: int = 0):
        """Capture ``graph_steps`` full training steps (gather -> forward -> backward -> guarded
        Adam, which advances the device cursor) as ONE graph over the static table [nrows, B].
        ``steps=1``: the one-step graph of the same form (``multi_graph1``), which replays the
        leftover steps of a run that is not a multiple of ``graph_steps`` from the same table and
        cursor (the single-step graph's host id copy and launch gap cost ~10 us a step)."""
        one = steps == 1
        from ..data.store import CursorIds
        snap = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        ids = CursorIds(self._table, self._cursor)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._body(ids, with_opt=False)
                if self.dp_graph:
                    self._reduce_grads()          # (communicator + RCCL state warm before capture)
        torch.cuda.current_stream().wait_stream(s)
        self.opt.zero_grad()
        graph = torch.cuda.CUDAGraph()
        it0 = self.opt.iterations
        self.opt.cursor, self.opt.cursor_mod = self._cursor, nrows
        # (thread-local capture mode: the process group's watchdog thread keeps polling its own
        # events while this thread captures)
        kw = {"capture_error_mode": "thread_local"} if self.dp_graph else {}
        try:
            with torch.cuda.graph(graph, **kw):
                for _ in range(1 if one else self.graph_steps):
                    if self.dp_graph:
                        self._body(ids, with_opt=False)
                        self._reduce_grads()
                        self.opt.step(grad_scale=1.0 / self.world)
                    else:
                        self._body(ids, with_opt=True)
        finally:
            self.opt.cursor, self.opt.cursor_mod = None, 1
        self.opt.iterations = it0
        if one:
            self.multi_graph1, self._multi_loss1 = graph, self.last_loss
            self._multi_key1 = (nrows, self._table.shape[1])
        else:
            self.multi_graph, self._multi_loss = graph, self.last_loss
            self._multi_key = (nrows, self._table.shape[1])
        with torch.no_grad():
            for k, v in self.model.state_dict().items():
                v.copy_(snap[k])
        self.train_metrics.reset()
        self.opt.zero_grad()

    def prepare_graphs(self, rows: torch.Tensor):
        """Capture the step graphs for batches drawn from ``rows`` now (outside any timed region):
        the single-step graph and, when multi-step replay applies, the multi-step graph."""
        if not self.use_graph:
            return
        if self.graph is None:
            self._capture()
        if self._multi_ok():
            if self._table is None or tuple(self._table.shape) != tuple(rows.shape):
                self._table, self._table_src = torch.empty_like(rows, dtype=torch.long), None
                self.multi_graph = self.multi_graph1 = None
            self._load_table(rows)
            if self.multi_graph is None or self._multi_key != (int(rows.shape[0]), rows.shape[1]):
                self._capture_multi(int(rows.shape[0]))
            if self.multi_graph1 is None or self._multi_key1 != (int(rows.shape[0]), rows.shape[1]):
                self._capture_multi(int(rows.shape[0]), steps=1)
        for g in (self.graph, self.multi_graph, self.multi_graph1):
            _graph_upload(g)

    def _load_table(self, rows: torch.Tensor):
        """Copy the batch-id rows into the graphs' device table, unless the table already holds
        exactly these rows (same tensor, unmodified since): a copy launch and its gap less per call."""
        # (the source is kept referenced, so no other tensor can take its memory and pass as it)
        src = getattr(self, "_table_src", None)
        if src is not None and src[0] is rows and src[1] == rows._version:
            return
        self._table.copy_(rows, non_blocking=True)
        self._table_src = (rows, rows._version)

    def train_steps(self, rows: torch.Tensor, start: int, k: int):
        """``k`` training steps on batches ``rows[(start + i) % len(rows)]`` (rows: [n, B] device
        ids). With graphs, full chunks of ``graph_steps`` steps replay one multi-step graph each;
        the rest (and every step when fault injection or DP is on) go through :meth:`train_step`."""
        nb = int(rows.shape[0])
        S = self.graph_steps
        one_ok = (self.multi_graph1 is not None and self._multi_ok() and self._table is not None
                  and tuple(self._table.shape) == tuple(rows.shape) and self._multi_key1 == (nb, rows.shape[1]))
        if k < S and one_ok:                 # (prepare_graphs captured the one-step form)
            self.model.train()
            self._load_table(rows)
            self._cursor.fill_(start % nb)
            for _ in range(k):
                self.multi_graph1.replay()
            self.opt.iterations += k
            self.global_step += k
            self.last_loss = self._multi_loss1
            return self.last_loss
        if not self._multi_ok() or k < S:
            for i in range(k):
                self.train_step(rows[(start + i) % nb])
            return self.last_loss
        self.model.train()
        if self._table is None or tuple(self._table.shape) != tuple(rows.shape):
            self._table, self._table_src = torch.empty_like(rows, dtype=torch.long), None
            self.multi_graph = self.multi_graph1 = None
            one_ok = False
        if self.multi_graph is not None and self._multi_key != (nb, rows.shape[1]):
            self.multi_graph = None
        self._load_table(rows)
        if self.multi_graph is None:
            if self.graph is None:
                self._capture()              # the single-step graph shares the warm allocator state
            self._capture_multi(nb)
        self._cursor.fill_(start % nb)
        n = k // S
        for _ in range(n):
            self.multi_graph.replay()
        self.opt.iterations += n * S
        self.global_step += n * S
        self.last_loss = self._multi_loss
        if k > n * S and one_ok:             # leftover steps: the one-step graph, same table and cursor
            for _ in range(k - n * S):
                self.multi_graph1.replay()
            self.opt.iterations += k - n * S
            self.global_step += k - n * S
            self.last_loss = self._multi_loss1
            return self.last_loss
        for i in range(n * S, k):
            self.train_step(rows[(start + i) % nb])
        return self.last_loss

    def train_step(self, wids: torch.Tensor):
        self.model.train()
        step = self.global_step + 1
        if self.poison is not None:
            self.poison.fill_(float("nan") if self.fault.nan_now(step) else 0.0)
        self._step(wids)
        self.global_step = step
        if self.fault is not None:
            self.fault.after_step(step)
        return self.last_loss

    def _step(self, wids):
        if self.use_graph:
            if self.graph is None:
                self._capture()
            self.static_wids.copy_(wids, non_blocking=True)
            self.graph.replay()
            self.last_loss = self._graph_loss
        else:
            self._body(wids.to(self.device), with_opt=not self.split_opt)
        if not self.split_opt:
            self.opt.iterations += int(self.use_graph)
            return
        # data parallel: one all-reduce of the flat gradient buffer, then Adam
        if self.collective:
            with _rf("gnnqc.allreduce"):
                if self.device.type == "cuda":
                    if len(self._comm_events) < 64:      # sample the first steps of an epoch
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        self._reduce_grads()
                        e1.record()
                        self._comm_events.append((e0, e1))
                    else:
                        self._reduce_grads()
                else:
                    D.all_reduce_(self.opt.flat_g)
        with _rf("gnnqc.optimizer"):
            if self.opt_graph is not None:
                self.opt_graph.replay()
                self.opt.iterations += 1
            else:
                self.opt.step(grad_scale=1.0 / self.world)

    # ---------------------------------------------------------------- epoch helpers
    def train_epoch(self, loader, epoch: int) -> Dict[str, float]:
        import time
        loader.set_epoch(epoch)
        self.train_metrics.reset()
        self._comm_events = []
        skipped0 = self.opt.skipped_steps
        upd_state = getattr(self.opt, "guard_state", None)
        partial0 = int(upd_state[5].item()) if upd_state is not None else 0
        rejected0 = self._chain_rejected()
        steps0 = self.global_step
        t0 = time.perf_counter()
        rows = loader.batch_ids()
        if torch.is_tensor(rows) and rows.dim() == 2 and rows.shape[0] > 0 and rows.shape[1] == self.batch_size:
            self.train_steps(rows, 0, int(rows.shape[0]))
        else:
            for row in rows:
                self.train_step(row)
        if self.world > 1:
            # a peer all-reduce timeout or a partial guarded update on ANY rank is fatal on EVERY
            # rank (the ranks' parameters may differ): agree before any other collective
            upd = getattr(self.opt, "guard_state", None)
            flag = torch.tensor([1.0 if self.peer is not None and self.peer.timed_out() else 0.0,
                                 float(upd[6].item()) if upd is not None else 0.0],
                                device=self.device if D.backend() == "nccl" else "cpu")
            D.all_reduce_(flag, force=True)
            if float(flag[0].item()) != 0.0:
                raise RuntimeError("peer all-reduce: a rank never arrived (spin timeout); training stopped on "
                                   "every rank")
            if float(flag[1].item()) != 0.0:
                raise RuntimeError("guarded Adam: a workgroup never saw the step decision on some rank (partial "
                                   "update); training stopped on every rank")
        D.average_buffers(self.model)                 # DP: BN moving statistics agree on every rank
        logs = self.train_metrics.result()            # device -> host: synchronises the epoch
        dt = time.perf_counter() - t0
        nsteps = self.global_step - steps0
        logs["skipped_steps"] = float(self.opt.skipped_steps - skipped0)
        if upd_state is not None:
            # gradient elements the flag-driven Adam left untouched because they were not finite
            # although no producer flagged them (an fp32 overflow of a sum of finite parts)
            logs["nonfinite_grad_elements"] = float(int(upd_state[5].item()) - partial0)
            if logs["nonfinite_grad_elements"]:
                import warnings
                warnings.warn(f"{int(logs['nonfinite_grad_elements'])} non-finite gradient element(s) were "
                              "skipped by the update this epoch (their parameters were not changed)")
        if hasattr(self.opt, "check_update"):
            self.opt.check_update()
        if rejected0 is not None:
            # steps rejected on the device after an LSTM chain spin timeout: fail loudly
            from ..ops.lstm import check_chain
            check_chain(self.device, rejected0)
        logs["windows_per_sec"] = nsteps * loader.batch_size * self.world / max(dt, 1e-9)
        if self._comm_events:
            logs["allreduce_us"] = 1e3 * sum(a.elapsed_time(b) for a, b in self._comm_events) / len(self._comm_events)
        return logs

    def _chain_rejected(self) -> Optional[int]:
        """Training steps rejected so far for an LSTM chain spin timeout (None off the GPU)."""
        if self.device.type != "cuda":
            return None
        from ..ops.lstm import chain_ctl
        return int(chain_ctl(self.device)[3].item())

    @torch.no_grad()
    def evaluate(self, loader, prefix: str = "val_") -> Dict[str, float]:
        acc = MetricAccumulator(self.device)
        self.model.eval()
        for row in loader.batch_ids():
            self._loss(row, acc)
        self.model.train()
        out = acc.result(prefix)
        if self.device.type == "cuda":
            from ..ops.lstm import check_chain
            check_chain(self.device)
        return out


@torch.no_grad()
def predict(model, store, loader, baseline: bool = False, gather_all: bool = True):
    """Probabilities, labels and label mask for every window in ``loader`` (host numpy).

    CML: one value per window; SoilNet: one per (window, node) with mask.
    Returns dict with ``p``, ``y``, ``mask``, ``wid`` (window id per row) and, for
    SoilNet, ``node`` (node position).
    """
    was_training = model.training
    model.eval()
    ps, ys, ms, ws = [], [], [], []
    for row in loader.batch_ids():
        b = store.gather(row)
        p = model(b.model_inputs(store.ds_type, baseline))
        ps.append(p.float())
        ys.append(b.y.float())
        ms.append(b.y_mask.float())
        ws.append(b.wid)
    if was_training:
        model.train()
    if store.device.type == "cuda":
        from ..ops.lstm import check_chain
        check_chain(store.device)
    if not ps:                          # no batch on this rank (e.g. a tiny held-out fold)
        N = () if store.per_sensor else (store.n_nodes,)
        ps = ys = ms = [torch.zeros((0, *N), device=store.device)]
        ws = [torch.zeros(0, dtype=torch.long, device=store.device)]
    p = torch.cat(ps)
    y = torch.cat(ys)
    m = torch.cat(ms)
    w = torch.cat(ws)
    if gather_all:
        p, y, m, w = (D.all_gather_var(t) for t in (p, y, m, w))
    out = {"p": p.cpu().numpy(), "y": y.cpu().numpy(), "mask": m.cpu().numpy(), "wid": w.cpu().numpy()}
    if not store.per_sensor:
        N = out["p"].shape[1]
        out["node"] = np.broadcast_to(np.arange(N), out["p"].shape).copy()
    return out


def flatten_predictions(pred: dict):
    """Drop padding / unlabelled rows -> (p, y, wid[, node]) 1-D arrays."""
    keep = pred["mask"].reshape(-1) > 0
    res = {"p": pred["p"].reshape(-1)[keep], "y": pred["y"].reshape(-1)[keep]}
    wid = pred["wid"]
    if pred["p"].ndim == 2:
        wid = np.repeat(wid, pred["p"].shape[1])
        res["node"] = pred["node"].reshape(-1)[keep]
    res["wid"] = wid.reshape(-1)[keep]
    return res


__all__ = ["Trainer", "MetricAccumulator", "predict", "flatten_predictions"]
