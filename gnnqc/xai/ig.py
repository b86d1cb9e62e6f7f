"""Integrated Gradients.

Reference: ``xai/libs/integrated_gradients.py`` - ``IntegratedGradientsExplainer``
(``:91-2044``): zero baseline (``:898-917``), ``m_steps + 1`` linearly interpolated
inputs (``:919-942``), one forward + ``GradientTape`` backward per interpolation
step on the whole batch (``:955-1004``), trapezoidal Riemann average (``:1006-1015``),
optional input scaling and negative-value policy (``:1180-1208``), threshold
classification and TP/TN/FP/FN sample selection (``:495-546``, ``:1226-1262``),
per-sample ``.npy`` outputs in ``<out>/integrated_gradients/<project>/<ds>/<dataset>/
<sensor>/<sensor>_<YYYYmmdd_HHMMSS>_<true>_<pred>/`` (``:221-384``, ``:1248-1400``) and
SLURM array sharding (``:190-199``, ``:432-448``).

MI355X design: the reference runs 101 sequential forward/backward passes over a
batch of 128 windows - each pass uses a sliver of the GPU. Here the alpha axis is
folded into the batch: ``k`` interpolation steps x ``B`` windows go through ONE
forward + ONE input-gradient backward (frozen weights: the LSTM backward skips the
weight-gradient kernel, the fused GCN backward skips its reduction), so the
persistent LSTM kernels get ``k*B`` sequences to spread over 256 CUs. The
trapezoid weights are applied while accumulating on the device; nothing goes to the
host until a batch is finished. Batches are sharded across ranks (one process per
GPU, ``torch.distributed``) or SLURM array tasks exactly like the reference's
``_split_work``.
"""
from __future__ import annotations

import os
import shutil
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import config as C

CONFUSION = {(0, 0): "TN", (0, 1): "FP", (1, 0): "FN", (1, 1): "TP"}


def trapezoid_weights(m_steps: int, device=None) -> torch.Tensor:
    """Weights w_i with sum_i w_i g_i == mean_i (g_i + g_{i+1}) / 2 over m_steps intervals.
    (Built on the host and copied once: element assignment of a Python scalar into a GPU tensor
    is a synchronising pageable copy, which stalled every attribute() call.)"""
    w = torch.full((m_steps + 1,), 1.0 / m_steps, dtype=torch.float32)
    w[0] = w[-1] = 0.5 / m_steps
    return w.to(device) if device is not None else w


def _frozen(model):
    """Context: weights do not require grad (input gradients only), restored afterwards."""
    class _Ctx:
        def __enter__(self):
            self.flags = [(p, p.requires_grad) for p in model.parameters()]
            for p, _ in self.flags:
                p.requires_grad_(False)

        def __exit__(self, *a):
            for p, f in self.flags:
                p.requires_grad_(f)
    return _Ctx()


def _ig_hip(t: torch.Tensor) -> bool:
    """The HIP interpolation / accumulation / finalize kernels (csrc/kernels/ig.hip) run for fp32
    inputs on the GPU; a missing extension on a GPU box fails loudly in hip_ops()."""
    from ..ops import use_hip
    return bool(use_hip(t) and t.dtype == torch.float32)


def _ops():
    from ..utils.native import hip_ops
    return hip_ops()


class IntegratedGradients:
    """Alpha-batched IG engine for the GCN / baseline classifiers.

    ``attribute(batch)`` returns device tensors:

    * ``grad_x``    [B, T, N, C] node-feature attributions (GCN models),
    * ``grad_anom`` [B, T, C] flagged-sensor series attributions (CML),
    * ``pred``      [B] model output at alpha = 1 (the actual prediction),
    * ``path_pred`` [m+1, B] outputs along the path (gradient-saturation plots).

    SoilNet models emit one score per node; ``target`` [B] picks the node whose score
    is explained (default: the highest-scoring valid node).
    """

    def __init__(self, model, ds_type: str, m_steps: int = 100, baseline: str = "zero",
                 max_rows: int = 16384, scale_gradients: bool = True, negative_values: str = "keep",
                 use_graph: bool = True):
        if baseline != "zero":
            raise NotImplementedError("only the zero baseline is implemented (as in the reference, :901-917)")
        if negative_values not in ("keep", "clip", "abs"):
            raise ValueError(f"negative_values must be keep/clip/abs, got {negative_values!r}")
        self.model = model
        self.ds_type = ds_type
        self.m_steps = int(m_steps)
        self.max_rows = int(max_rows)
        self.scale_gradients = scale_gradients
        self.negative_values = negative_values
        self.is_baseline = type(model).__name__ == "BaselineClassifier"
        # flagged-sensor inputs (CML, XAI SoilNet) vs network-wide SoilNet
        self.per_sensor = bool(getattr(model, "per_sensor", ds_type == "cml"))
        # the CML GCN's path-folded attribution replays as ONE HIP graph per input shape (about 85
        # launches: the host, not the GPU, bounded the eager loop)
        self.use_graph = bool(use_graph)
        self._graph = None

    # -- inputs that are interpolated ------------------------------------------------
    def _split(self, batch):
        """(interpolated tensors, static tensors, rebuild fn)."""
        if self.per_sensor:
            if self.is_baseline:
                return [batch.anom], [], lambda v, s: (v[0],)
            return ([batch.x, batch.anom], [batch.adj, batch.node_mask, batch.anom_pos],
                    lambda v, s: (v[0], v[1], s[0], s[1], s[2]))
        if self.is_baseline:
            return [batch.x], [batch.node_mask], lambda v, s: (v[0], s[0])
        return [batch.x], [batch.adj, batch.node_mask], lambda v, s: (v[0], s[0], s[1])

    def _select(self, out: torch.Tensor, B: int, k: int, target: Optional[torch.Tensor]):
        out = out.reshape(k * B, -1)
        if out.shape[1] == 1:
            return out[:, 0]
        t = target.repeat(k)
        return out.gather(1, t[:, None])[:, 0]

    def attribute(self, batch, target: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        model = self.model
        was_training = model.training
        model.eval()
        try:
            if (self.use_graph and target is None and batch.x.is_cuda and _ig_hip(batch.x)
                    and self._cml_path_folded_ok(batch)):
                return self._attribute_graphed(batch)
            return self._attribute(batch, target)
        finally:
            model.train(was_training)

    _GRAPH_FIELDS = ("x", "anom", "adj", "node_mask", "anom_pos")

    def _attribute_graphed(self, batch) -> Dict[str, torch.Tensor]:
        """:meth:`_attribute` captured once per input shape as a HIP graph over static copies of
        the batch's input tensors, then replayed (inputs copied in, results cloned out)."""
        import dataclasses
        ts = [getattr(batch, f) for f in self._GRAPH_FIELDS]
        key = tuple((None if t is None else (tuple(t.shape), t.dtype, str(t.device))) for t in ts)
        # the graph reads the weights and buffers by address: a model whose tensors were replaced
        # (moved, re-created) must be captured again (in-place updates such as load_state_dict or
        # an optimizer step keep the addresses and are seen by the replay)
        key += tuple(t.data_ptr() for t in list(self.model.parameters()) + list(self.model.buffers()))
        if self._graph is None or self._graph[0] != key:
            self._graph = None
            static = dataclasses.replace(batch, **{f: (None if t is None else t.clone())
                                                   for f, t in zip(self._GRAPH_FIELDS, ts)})
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):                    # allocator + lazy init outside the capture
                    self._attribute(static, None)
            torch.cuda.current_stream().wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = self._attribute(static, None)
            self._graph = (key, g, static, out)
        _, g, static, out = self._graph
        for f, t in zip(self._GRAPH_FIELDS, ts):
            if t is not None:
                getattr(static, f).copy_(t, non_blocking=True)
        g.replay()
        return {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}

    def _attribute(self, batch, target: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        model = self.model
        vals, static, build = self._split(batch)
        B = vals[0].shape[0]
        hip = _ig_hip(vals[0])
        fused = hip and self._cml_path_folded_ok(batch)
        if fused:
            # the prediction is the path's last point (alpha = 1: the unscaled inputs), read off
            # path_pred below instead of a separate forward pass
            pred_full = None
        else:
            with torch.no_grad():
                pred_full = model(build(vals, static)).reshape(B, -1).float()
        if pred_full is None:
            pred = None
        elif pred_full.shape[1] > 1:
            if target is None:
                masked = pred_full.masked_fill(batch.node_mask <= 0, -1.0)
                target = masked.argmax(1)
            pred = pred_full.gather(1, target[:, None])[:, 0]
        else:
            pred = pred_full[:, 0]
        dev = vals[0].device
        dt = torch.float64 if vals[0].dtype == torch.float64 else torch.float32
        key = (str(dev), dt)
        if getattr(self, "_path_key", None) != key:       # path points + weights: once per device
            self._alphas = torch.linspace(0.0, 1.0, self.m_steps + 1, device=dev, dtype=dt)
            self._wts = trapezoid_weights(self.m_steps, dev).to(dt)
            self._path_key = key
        alphas, wts = self._alphas, self._wts
        # (GNNQC_IG_LEAN=0: zero-filled accumulators and a sum() seed, the pre-round-6-close form, for A/B)
        lean = fused and os.environ.get("GNNQC_IG_LEAN", "1") == "1"
        acc = [(torch.empty_like if lean else torch.zeros_like)(v, dtype=dt) for v in vals]
        k = max(1, min(self.m_steps + 1, self.max_rows // max(B, 1)))
        # (one fused chunk covering the whole path: its output rows are the path predictions, no copy)
        whole = lean and k >= self.m_steps + 1 and dt == torch.float32
        path_pred = None if whole else torch.empty(self.m_steps + 1, B, device=dev, dtype=dt)
        vf = [v.to(dt).contiguous() for v in vals]
        with _frozen(model), torch.enable_grad():
            for s in (range(0, self.m_steps + 1, k) if fused else ()):
                # (the first chunk's gradient launch writes the accumulators: no zero fill)
                self._cml_path_folded_chunk(batch, alphas[s:s + k].contiguous(), wts[s:s + k].contiguous(),
                                            acc, None if whole else path_pred[s:s + k], target, first=(s == 0 and lean))
                if whole:
                    path_pred = self._last_y.reshape(self.m_steps + 1, B)
            for s in (range(0, self.m_steps + 1, k) if not fused else ()):
                a = alphas[s:s + k]
                kk = a.numel()
                # zero baseline: x_alpha = alpha * x, folded into the batch dimension (HIP: one
                # ig_interp launch per input tensor for all kk path points)
                xs = []
                for v in vf:
                    if hip:
                        xi = _ops().ig_interp(v, a.contiguous())
                    else:
                        shp = (kk,) + (1,) * v.dim()
                        xi = (a.view(shp) * v.unsqueeze(0)).reshape((kk * B,) + tuple(v.shape[1:]))
                    xs.append(xi.requires_grad_(True))
                st = [t.repeat((kk,) + (1,) * (t.dim() - 1)) for t in static]
                out = model(build(xs, st))
                y = self._select(out, B, kk, target)
                grads = torch.autograd.grad(y.sum(), xs)
                path_pred[s:s + kk] = y.detach().view(kk, B).to(dt)
                w = wts[s:s + kk].contiguous()
                for j, g in enumerate(grads):
                    if hip and g.is_contiguous() and g.dtype == torch.float32 and g.data_ptr() % 16 == 0:
                        _ops().ig_accum(acc[j], g, w)      # trapezoid-weighted sum, one launch
                    else:
                        g = g.view((kk, B) + tuple(g.shape[1:]))
                        acc[j] += torch.tensordot(w, g.to(dt), dims=1)
        mode = {"keep": 0, "clip": 1, "abs": 2}[self.negative_values]
        if hip:
            e = vf[0].new_zeros(0)
            acc = [_ops().ig_finalize(g, v if self.scale_gradients else e, mode) for g, v in zip(acc, vf)]
        else:
            if self.scale_gradients:
                acc = [g * v for g, v in zip(acc, vf)]       # (x - baseline) * avg grad
            if self.negative_values == "abs":
                acc = [g.abs() for g in acc]
            elif self.negative_values == "clip":
                acc = [g.clamp(min=0) for g in acc]
        if pred is None:
            pred = path_pred[-1].float()
        res = {"pred": pred, "path_pred": path_pred, "target": target}
        if self.per_sensor:
            if self.is_baseline:
                res["grad_anom"] = acc[0]
            else:
                res["grad_x"], res["grad_anom"] = acc
        else:
            res["grad_x"] = acc[0]
        return res


    # -- CML GCN on the GPU: the alpha scaling folded into the GCN kernels ---------------
    def _cml_path_folded_ok(self, batch) -> bool:
        """The CML GCN's path-folded IG (``ig_gcn_pool_fwd`` / ``ig_gcn_pool_bwd``): the path
        points' GCN + pooling computed from the un-replicated batch, their input gradients
        trapezoid-summed in the same backward launch (no kk x B copies of x, anom, adj, mask)."""
        m = self.model
        if self.is_baseline or not self.per_sensor or type(m).__name__ != "GCNClassifier" or m.training:
            return False
        if getattr(m, "sensors_time_layer", None) is not None or getattr(m, "spatial_transformer", None) is not None:
            return False
        x, anom = batch.x, batch.anom
        if x.dtype != torch.float32 or anom is None or not m._fused_ok():
            return False
        inputs = (x, anom, batch.adj, batch.node_mask, batch.anom_pos)
        if not m._cml_time_major(inputs):
            return False
        g = m.gcn_layer
        cin, F, N = x.shape[-1], g.kernel.shape[1], x.shape[2]
        shape_ok = N <= 32 and ((cin == 2 and F in (8, 16, 32)) or (cin in (1, 3) and F == 16))
        return bool(shape_ok and anom.shape[-1] <= min(F, 4) and not (g.dropout and m.training))

    def _cml_path_folded_chunk(self, batch, a: torch.Tensor, wt: torch.Tensor, acc, path_pred_rows,
                               target: Optional[torch.Tensor], first: bool = False):
        """One chunk of path points: GCN forward of all of them (one launch), the TimeLayer + head
        on the path batch, one backward to the LSTM input, then one launch that turns that gradient
        into the trapezoid-weighted input gradients of x and anom (accumulated into ``acc``)."""
        m = self.model
        ops = _ops()
        g = m.gcn_layer
        x = batch.x.contiguous()
        anom = batch.anom.float().contiguous()
        mask = batch.node_mask.float().contiguous()
        B = x.shape[0]
        kk = a.numel()
        pooling = "selection" if m.pooling_type == "selection" else m.aggregation_type
        ap = (batch.anom_pos.long().contiguous() if (pooling == "selection" and batch.anom_pos is not None)
              else x.new_zeros(0))
        with torch.no_grad():
            w, _S, st = ops.gcn_prep(x, batch.adj.float().contiguous(), mask, ap, g.aggregate == "mean",
                                     {"mean": 0, "sum": 1, "selection": 2}[pooling], g.kernel.contiguous(),
                                     g.bias.contiguous(), g.bn_gamma.contiguous(), g.bn_beta.contiguous(),
                                     g.bn_moving_mean, g.bn_moving_variance, False, float(g.momentum), float(g.eps))
            Cp = g.kernel.shape[1] + anom.shape[-1]
            Cp += (-Cp) % 4
            h0 = ops.ig_gcn_pool_fwd(x, w, anom, g.kernel.contiguous(), g.bias.contiguous(), st[2].contiguous(),
                                     st[3].contiguous(), g.prelu_alpha.contiguous(), a, int(Cp))
        h0.requires_grad_(True)
        spec = m.head_spec()
        taken = []
        last = None
        if (spec is not None and os.environ.get("GNNQC_IG_T4_HEAD", "1") == "1"
                and tuple(spec[0].kernel.shape) == (128, 64) and tuple(spec[1].kernel.shape) == (64, 64)
                and tuple(spec[2].kernel.shape) == (64, 1) and all(d.bias is not None for d in spec[:3])):
            # time4 + the frozen head in one launch (time4_prob_fwd: sigmoid outputs and d p / d h_{T-1}),
            # the recurrence backward seeded with it (no head launches)
            from ..ops.lstm import lstm_last128_prob_tm
            head_w = [spec[0].kernel, spec[0].bias, spec[1].kernel, spec[1].bias, spec[2].kernel, spec[2].bias]

            def last(hin, mod):
                taken.append(True)
                return lstm_last128_prob_tm(hin, mod, head_w, (spec[3], spec[4]), kk * B)

        feat = m.time_layer.forward_time_major(h0, kk * B, last=last)
        if taken:
            y = feat
            # d sum(y) / d h0 with a cached ones seed (no reduction + fill launches per call)
            if os.environ.get("GNNQC_IG_LEAN", "1") == "1":
                ones = getattr(self, "_ones", None)
                if ones is None or ones.shape != y.shape or ones.device != y.device:
                    ones = self._ones = torch.ones_like(y)
                (gh,) = torch.autograd.grad(y, h0, ones)
            else:
                (gh,) = torch.autograd.grad(y.sum(), h0)
        elif (spec is not None and feat.dim() == 2 and feat.shape[1] in (32, 64, 128) and feat.dtype == torch.float32
                and spec[0].kernel.shape[1] == 64 and tuple(spec[1].kernel.shape) == (64, 64)
                and tuple(spec[2].kernel.shape) == (64, 1) and os.environ.get("GNNQC_IG_HEAD_HIP", "1") == "1"):
            # the frozen head on HIP (head.hip, PROB mode): sigmoid outputs, then d sum(sigmoid) / d feat
            # in one more launch; autograd only carries that gradient back through the LSTM stack
            d1, d2, d3, a1, a2 = spec
            ff = feat.detach()
            if not (ff.stride(1) == 1 and ff.stride(0) % 4 == 0 and ff.data_ptr() % 16 == 0):
                ff = ff.contiguous()
            W1, W2, W3 = d1.kernel.contiguous(), d2.kernel.contiguous(), d3.kernel.contiguous()
            z1, z2, prob = ops.head_prob_fwd(ff, W1, d1.bias.contiguous(), W2, d2.bias.contiguous(), W3,
                                             d3.bias.contiguous(), float(a1), float(a2))
            dfeat = ops.head_prob_bwd(ff, W1, W2, W3, z1, z2, prob, float(a1), float(a2))
            (gh,) = torch.autograd.grad(feat, h0, dfeat)
            y = prob
        else:
            out = torch.sigmoid(m.head(feat))
            y = self._select(out, B, kk, target)
            (gh,) = torch.autograd.grad(y.sum(), h0)
        if path_pred_rows is None:
            self._last_y = y.detach()
        else:
            path_pred_rows.copy_(y.detach().view(kk, B).to(path_pred_rows.dtype))
        ops.ig_gcn_pool_bwd(x, w, mask, gh.contiguous(), g.kernel.contiguous(), g.bias.contiguous(),
                            st[2].contiguous(), st[3].contiguous(), g.prelu_alpha.contiguous(), a, wt.float(),
                            acc[0], acc[1], bool(first))


def completeness_gap(ig_res: Dict[str, torch.Tensor]) -> torch.Tensor:
    """IG axiom check: sum of (input-scaled) attributions ~= f(x) - f(baseline)."""
    tot = 0
    for k in ("grad_x", "grad_anom"):
        if k in ig_res:
            g = ig_res[k]
            tot = tot + g.reshape(g.shape[0], -1).sum(1)
    return tot - (ig_res["path_pred"][-1] - ig_res["path_pred"][0])


# ====================================================================================
class IntegratedGradientsExplainer:
    """Config-driven explainer with the reference's output layout.

    ``IntegratedGradientsExplainer(preproc_config, model_config, xai_config)`` - paths
    or Config objects. ``prepare_data()`` builds the window store; ``get_gradients()``
    runs IG over the selected batches and writes per-sample files.
    """

    def __init__(self, preproc_config, model_config, xai_config, model=None, windows=None, device=None,
                 raw=None, shard: Optional[str] = None):
        load = lambda c: C.load(c) if isinstance(c, str) else c  # noqa: E731
        self.preproc_config = C.normalize_preproc(load(preproc_config))
        self.model_config = load(model_config)
        self.xai_config = load(xai_config) if xai_config is not None else C.default("xai_ig")
        self.ig_cfg = self.xai_config.integrated_gradients
        self.ds_type = self.preproc_config.ds_type
        from ..parallel import dist as D
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        # explicit shard ("i/n"), SLURM array job sharding (``:190-199``) or one rank per GPU
        shard = shard or os.environ.get("GNNQC_IG_SHARD")
        if shard:
            i, n = (int(v) for v in str(shard).split("/"))
            if not 0 <= i < n:
                raise ValueError(f"shard {shard!r}: need 0 <= i < n")
            self.workerid, self.n_worker = i, n
        elif "SLURM_ARRAY_TASK_ID" in os.environ:
            self.workerid = int(os.environ["SLURM_ARRAY_TASK_ID"])
            self.n_worker = int(os.environ["SLURM_ARRAY_TASK_COUNT"])
        elif D.world_size() > 1:
            self.workerid, self.n_worker = D.rank(), D.world_size()
        else:
            self.workerid = self.n_worker = None
        self.output_dir = self._save_path()
        os.makedirs(self.output_dir, exist_ok=True)
        torch.manual_seed(int(self.ig_cfg.get("random_seed", 42)))
        np.random.seed(int(self.ig_cfg.get("random_seed", 42)))
        self.model = model if model is not None else self._load_model()
        self.model.to(self.device).eval()
        self.is_baseline = type(self.model).__name__ == "BaselineClassifier"
        self.windows = windows
        self.raw = raw
        self.store = None
        self.sample_ids = None
        self.results: List[dict] = []

    # -- paths (``:221-384``) ----------------------------------------------------------
    def _save_path(self, sensor: str = "", date: str = "", true="", pred="") -> str:
        base = os.path.join(self.xai_config.output_dir, "integrated_gradients", self.xai_config.project,
                            self.ds_type, self.ig_cfg.dataset)
        if sensor == "" and date == "":
            return base
        return os.path.join(base, sensor, f"{sensor}_{date}_{true}_{pred}")

    def _file_name(self, sensor: str = "", date: str = "", true="", pred="") -> str:
        stem = f"{self.xai_config.project}_{self.ds_type}_{self.ig_cfg.dataset}"
        if sensor == "" and date == "":
            return stem
        return f"{stem}_{sensor}_{date}_{true}_{pred}"

    def log_file(self, batch_id: int, index: int, sensor: str, date: str):
        d = os.path.join(self.output_dir, "log")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "log.txt" if self.workerid is None else f"log_{self.workerid}.txt"), "a") as f:
            f.write(f"{self.xai_config.project},{self.ds_type},{self.ig_cfg.dataset},{batch_id},{index},{sensor},"
                    f"{date}\n")

    @staticmethod
    def _split_work(items: Sequence, workerid: int, n_worker: int) -> list:
        return [it for i, it in enumerate(items) if i % n_worker == workerid]

    def copy_config_files(self, paths: Sequence[str]):
        for p in paths:
            if isinstance(p, str) and os.path.exists(p):
                shutil.copy(p, self.output_dir)

    # -- model / data ----------------------------------------------------------------
    def _load_model(self):
        path = self.model_config.get("model_path")
        if path and os.path.exists(os.path.join(path, "gnnqc_state.pt")):
            from ..ckpt import load_model
            return load_model(path, device=self.device)
        if path and os.path.exists(os.path.join(path, "variables", "variables.index")):
            from ..ckpt.keras_layout import build_from_keras
            return build_from_keras(path, ds_type=self.ds_type, device=self.device)[0]
        raise FileNotFoundError(f"no model at {path!r}")

    def prepare_data(self):
        """Window store + the id list of the configured dataset split (``:590-703``)."""
        from ..data.preprocessing import create_windows_dataset, load_dataset
        from ..data.store import DeviceStore
        if self.windows is None:
            self.windows = create_windows_dataset(self.preproc_config, raw=self.raw)
        norm = getattr(self.model, "model_normalization", getattr(self.model, "normalization", None))
        self.store = DeviceStore(self.windows, norm, self.preproc_config.graph, device=self.device)
        tr, va, te = load_dataset(self.preproc_config, self.windows)
        which = self.ig_cfg.dataset
        ids = {"train": tr, "val": va, "test": te}.get(which)
        if ids is None or which == "all":
            ids = np.arange(self.windows.n_windows)
        self.sample_ids = np.asarray(ids, np.int64)
        if self.ig_cfg.get("evaluate_model", False):
            self.evaluate()
        return self.sample_ids

    def evaluate(self) -> dict:
        from ..eval.metrics import roc_auc_score
        preds, ys = [], []
        for b in self._batches(range(self.n_batches)):
            with torch.no_grad():
                p = self.model(b[1].model_inputs(self.ds_type, self.is_baseline)).reshape(b[1].y.shape)
            keep = b[1].y_mask > 0
            preds.append(p[keep].float().cpu().numpy())
            ys.append(b[1].y[keep].cpu().numpy())
        y, p = np.concatenate(ys), np.concatenate(preds)
        res = {"auc": float(roc_auc_score(y, p)) if 0 < y.sum() < len(y) else float("nan"), "n": int(len(y))}
        print(res)
        return res

    @property
    def batch_size(self) -> int:
        return int(self.preproc_config.batch_size)

    @property
    def n_batches(self) -> int:
        return -(-len(self.sample_ids) // self.batch_size)

    def _batches(self, batch_ids):
        for bid in batch_ids:
            ids = self.sample_ids[bid * self.batch_size:(bid + 1) * self.batch_size]
            if len(ids) == 0:
                raise ValueError(f"Batch {bid} not found. The dataset has fewer batches.")
            yield bid, self.store.gather(torch.as_tensor(ids, device=self.device)), ids

    # -- IG over batches ---------------------------------------------------------------
    def get_gradients(self, max_batches: Optional[int] = None):
        if self.store is None:
            self.prepare_data()
        sel = self.ig_cfg.batch_ids
        bids = list(range(self.n_batches)) if sel in ("all", None) else [int(b) for b in sel]
        if self.workerid is not None:
            bids = self._split_work(bids, self.workerid, self.n_worker)
        if max_batches is not None:
            bids = bids[:max_batches]
        engine = IntegratedGradients(self.model, self.ds_type, m_steps=int(self.ig_cfg.m_steps),
                                     baseline=self.ig_cfg.get("baseline", "zero"),
                                     scale_gradients=bool(self.ig_cfg.get("scale_gradients", True)),
                                     negative_values=self.ig_cfg.get("negative_values", "keep"),
                                     max_rows=int(self.ig_cfg.get("max_rows", 16384)))
        for bid, batch, ids in self._batches(bids):
            res = None
            if not self.ig_cfg.get("load_gradients_from_sample_file", False):
                res = engine.attribute(batch)
                if self.ig_cfg.get("plot_interpolated_data_element_series", False):
                    self._plot_interpolated(batch, bid, int(self.ig_cfg.m_steps))
            else:
                with torch.no_grad():
                    res = {"pred": self.model(batch.model_inputs(self.ds_type, self.is_baseline)).reshape(
                        len(batch.wid), -1)[:, 0].float()}
            self._unwrap_and_save(bid, batch, ids, res)
        return self.results

    def _plot_interpolated(self, batch, bid: int, m: int):
        """The batch's first sample along the zero-baseline path x_a = a x (``_interpolate`` +
        ``_plot_interpolated_data_element_series``, ``integrated_gradients.py:919-942,1415-1466``):
        ``interpolated_data_element_1_batch_<id>.png`` (flagged series) and ``..._2_..`` (node
        features) in the output directory."""
        from ..viz.ig import plot_interpolated_series
        alphas = np.linspace(0.0, 1.0, m + 1)
        out = []
        if batch.anom is not None:
            a0 = batch.anom[0].detach().float().cpu().numpy()
            out.append(plot_interpolated_series(alphas[:, None, None] * a0[None], alphas,
                                                os.path.join(self.output_dir,
                                                             f"interpolated_data_element_1_batch_{bid}.png")))
        x0 = batch.x[0].detach().float().cpu().numpy().transpose(1, 0, 2)          # [N, T, C]
        out.append(plot_interpolated_series(alphas[:, None, None, None] * x0[None], alphas,
                                            os.path.join(self.output_dir, f"interpolated_data_element_2_batch_{bid}.png")))
        return out

    def _sample_dates(self, wid: int) -> np.ndarray:
        """Time stamps of window ``wid`` (``timestep_before`` steps before its centre ... after)."""
        ws = self.windows
        g_of, l_of = self._flat if hasattr(self, "_flat") else ws.flat()
        self._flat = (g_of, l_of)
        g = ws.groups[int(g_of[wid])]
        c = int(ws.indices[int(g_of[wid])].center[int(l_of[wid])])
        tb = int(round(ws.timestep_before / ws.freq))
        return np.asarray(g.time[c - tb: c - tb + ws.seq_len])

    def _sample_info(self, wid: int):
        ws = self.windows
        g_of, l_of = ws.flat() if not hasattr(self, "_flat") else self._flat
        self._flat = (g_of, l_of)
        g = ws.groups[int(g_of[wid])]
        ix = ws.indices[int(g_of[wid])]
        c = int(ix.center[int(l_of[wid])])
        date = np.datetime64(g.time[c], "s").astype(object).strftime("%Y%m%d_%H%M%S")
        return str(g.group_id), date

    def _unwrap_and_save(self, bid: int, batch, ids, res):
        thr = float(self.ig_cfg.threshold)
        pred = res["pred"].detach().float().cpu().numpy()
        pred_cls = (pred > thr).astype(int)
        if batch.y.dim() == 1:                   # one label per window (per-sensor data)
            true = batch.y.detach().cpu().numpy().astype(int)
        else:
            t = res.get("target")
            yv = batch.y.detach().cpu().numpy()
            true = (yv[np.arange(len(ids)), t.cpu().numpy()] if t is not None else yv.max(1)).astype(int)
        which = list(self.ig_cfg.which_samples)
        keep = [i for i in range(len(ids)) if CONFUSION[(int(true[i]), int(pred_cls[i]))] in which]
        x = batch.x.detach().float().cpu().numpy()
        mask = batch.node_mask.detach().cpu().numpy() > 0
        anom = batch.anom.detach().float().cpu().numpy() if batch.anom is not None else None
        gx = res["grad_x"].detach().cpu().numpy() if "grad_x" in res else None
        ga = res["grad_anom"].detach().cpu().numpy() if "grad_anom" in res else None
        for i in keep:
            sensor, date = self._sample_info(int(ids[i]))
            tr, pr = int(true[i]), int(pred_cls[i])
            out = self._save_path(sensor, date, tr, pr)
            os.makedirs(out, exist_ok=True)
            fn = self._file_name(sensor, date, tr, pr)
            nodes = np.nonzero(mask[i])[0]
            feats = x[i][:, nodes].transpose(1, 0, 2)                      # [n, T, C] like ``_unwrap_features``
            files = {"features_unwrapped": feats, "predictions_unwrapped": np.array([pred[i]], np.float32),
                     "anomaly_flag_true_unwrapped": np.array(tr)}
            if anom is not None:
                files["anom_ts_unwrapped"] = anom[i]
            if gx is not None:
                files["gradients_features_unwrapped"] = gx[i][:, nodes].transpose(1, 0, 2)
            if ga is not None:
                files["gradients_anom_ts_unwrapped"] = ga[i]
            if "path_pred" in res:
                files["path_predictions_unwrapped"] = res["path_pred"][:, i].detach().cpu().numpy()
            if self.ig_cfg.get("load_gradients_from_sample_file", False):
                for k in ("gradients_features_unwrapped", "gradients_anom_ts_unwrapped"):
                    p = os.path.join(out, f"{k}_{fn}.npy")
                    if os.path.exists(p):
                        files[k] = np.load(p)
            for k, v in files.items():
                np.save(os.path.join(out, f"{k}_{fn}.npy"), v)
            self.log_file(bid, i, sensor, date)
            rec = {"batch": bid, "index": i, "sensor": sensor, "date": date, "true": tr, "pred": pr,
                   "score": float(pred[i]), "dir": out, "file_stem": fn,
                   "timestep_before_steps": int(round(self.windows.timestep_before / self.windows.freq))}
            self.results.append(rec)
            if self.ig_cfg.get("plot_classified_timeseries_sample", False) and anom is not None:
                # the flagged series of the window, the centre step shaded by outcome
                # (``plot_classified_timeseries_sample``, ``integrated_gradients.py:1468-1514``)
                from ..viz.results import timeseries_figure
                timeseries_figure(pr, tr, anom[i], sensor, self._sample_dates(int(ids[i])),
                                  os.path.join(out, f"anomalous_ts_{fn}.png"), rec["timestep_before_steps"],
                                  self.model_config, ds_type=self.ds_type)
            if self.ig_cfg.get("plot_heatmap", False):
                from ..viz.ig import plot_ig_heatmap
                plot_ig_heatmap(files, rec, self.xai_config, out_path=os.path.join(out, f"ig_heatmap_{fn}.png"),
                                batch_id=bid)
            if self.ig_cfg.get("plot_gradient_saturation", False) and "path_pred" in res:
                from ..viz.ig import plot_gradient_saturation
                plot_gradient_saturation(files["path_predictions_unwrapped"],
                                         os.path.join(out, f"gradient_saturation_{fn}.png"))

    def plot_ig_heatmap_from_directory(self, overwrite: bool = False, sensors=None, time_from=None, time_to=None,
                                       directory: Optional[str] = None):
        """Heatmaps of the saved samples of ``sensors`` whose centre time lies in
        [time_from, time_to], this worker's round-robin share (``integrated_gradients.py:1893-2044``;
        the paper's script calls it once per sensor and range,
        ``xai/notebooks/run_integrated_gradients_20240318.py:22-31``)."""
        from ..viz.ig import plot_ig_heatmap_from_directory
        return plot_ig_heatmap_from_directory(directory or self.output_dir, self.xai_config, overwrite=overwrite,
                                              sensors=sensors, time_from=time_from, time_to=time_to,
                                              workerid=self.workerid, n_worker=self.n_worker,
                                              stem=self._file_name())


def run_explainer(args):
    """CLI: ``python -m gnnqc.cli explain --model-dir ... [--xai-config ...]``."""
    import json
    from ..cli.common import load_configs, make_raw, resolve_device
    pc, mc = load_configs(args)
    dev = resolve_device(args.device)
    xc = C.load(args.xai_config) if args.xai_config else C.default("xai_ig")
    if args.out_dir:
        xc["output_dir"] = args.out_dir
    mc["model_path"] = args.model_dir
    raw = make_raw(args, pc)
    ex = IntegratedGradientsExplainer(pc, mc, xc, device=dev, raw=raw, shard=getattr(args, "shard", None))
    ex.prepare_data()
    res = ex.get_gradients(max_batches=args.max_batches)
    print(json.dumps({"samples": len(res), "output_dir": ex.output_dir}))


__all__ = ["IntegratedGradients", "IntegratedGradientsExplainer", "trapezoid_weights", "completeness_gap",
           "run_explainer", "CONFUSION"]
