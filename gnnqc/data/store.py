"""Device-resident window store and static-shape batches.

The reference parses ragged ``SequenceExample`` records on host threads and
builds a block-diagonal SparseTensor with one copy of the edge list per
(sample, time step) (``libs/preprocessing_functions.py:566-666``). Here:

* every group's series live in HBM as ``series[G, Ttot, Nmax, C]`` (time-major, so a
  window is one contiguous slab per node block), with the normalisation shift/scale
  next to them;
* a batch is gathered **on the device** from window ids - no host parsing;
* the graph of a sample is ONE dense ``[Nmax, Nmax]`` adjacency shared by all T
  steps (no B*T*E index blow-up); node padding + masks keep every batch at a
  static shape so the whole train step can be captured in a HIP graph.

Normalisations (``parse_*_tfrecord_fn``, ``:566-634,771-857``): ``rolling_median``
(CML default), ``rolling_median_fractional``, ``rolling_mean``, ``standarization``,
``scale``, ``median`` and SoilNet's ``scale_range``.
"""
from __future__ import annotations

import dataclasses
from typing import NamedTuple, Optional

import numpy as np
import torch

from .graph import build_adjacency
from .windows import WindowSet

_SOIL_SCALE_RANGE = {"moisture": (0.0, 1 / 60.0), "temp": (-20.0, 1 / 60.0), "battv": (2800.0, 1 / 800.0)}


@dataclasses.dataclass
class Batch:
    x: torch.Tensor                   # [B, T, N, C] normalised node features (0 for invalid nodes)
    adj: torch.Tensor                 # [B, N, N] 0/1 adjacency restricted to valid nodes
    node_mask: torch.Tensor           # [B, N] float
    anom: Optional[torch.Tensor]      # [B, T, C] flagged-sensor series (CML)
    anom_pos: torch.Tensor            # [B] position of the flagged node (CML) / -1
    y: torch.Tensor                   # [B] (CML) or [B, N] (SoilNet) float labels
    y_mask: torch.Tensor              # [B] or [B, N] float: which labels count
    wid: torch.Tensor                 # [B] window ids (-1 = padding)
    per_sensor: Optional[bool] = None  # flagged-sensor neighbourhoods (CML, XAI SoilNet); None: CML only

    def to(self, device, non_blocking=True):
        return Batch(**{k: (v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v)
                        for k, v in dataclasses.asdict(self).items()})

    def model_inputs(self, ds_type: str, baseline: bool = False):
        """Input tuple in the spirit of the reference's wrapper functions (``:743-768``; XAI
        SoilNet per-sensor batches: ``xai/libs/preprocessing_functions.py:667-707, 791-802``)."""
        per_sensor = self.per_sensor if self.per_sensor is not None else ds_type == "cml"
        if per_sensor:
            if baseline:
                return (self.anom,)
            return (self.x, self.anom, self.adj, self.node_mask, self.anom_pos)
        if baseline:
            return (self.x, self.node_mask)
        return (self.x, self.adj, self.node_mask)


def _norm_arrays(group, normalization: str):
    """Per-group (shift, scale) arrays shaped [Tn, N, C] (Tn = Ttot or 1)."""
    names = group.feature_names
    st = group.stats
    N, C, T = group.features.shape

    def stack(suffix):
        return np.stack([st[f"{n}_{suffix}"] for n in names], axis=-1)  # [N, C] or [N, T, C]

    if normalization == "scale_range":
        shift = np.array([_SOIL_SCALE_RANGE.get(n, (0.0, 1.0))[0] for n in names], np.float32)
        scale = np.array([_SOIL_SCALE_RANGE.get(n, (0.0, 1.0))[1] for n in names], np.float32)
        return np.broadcast_to(shift, (1, N, C)).copy(), np.broadcast_to(scale, (1, N, C)).copy()
    if normalization in ("rolling_median", "rolling_median_fractional", "rolling_mean"):
        if normalization == "rolling_mean":
            shift = stack("rolling_mean")
            sd = stack("rolling_std")
            with np.errstate(divide="ignore"):
                scale = 1.0 / sd
        else:
            shift = stack("rolling_median")
            if normalization == "rolling_median":
                scale = np.ones_like(shift)
            else:
                with np.errstate(divide="ignore"):
                    scale = 1.0 / shift
        # [N, T, C] -> [T, N, C]
        return np.ascontiguousarray(shift.transpose(1, 0, 2)), np.ascontiguousarray(scale.transpose(1, 0, 2))
    if normalization == "standarization":
        shift, scale = stack("mean"), 1.0 / stack("std")
    elif normalization == "scale":
        mn, mx = stack("min"), stack("max")
        shift, scale = mn, 1.0 / (mx - mn)
    elif normalization == "median":
        med = stack("median")
        shift = med
        # CML 'median' is fractional (``:138-140``); SoilNet's keeps the division commented out (``:358-361``)
        scale = 1.0 / med if group.ds_type == "cml" else np.ones_like(med)
    elif normalization in (None, "none"):
        shift, scale = np.zeros((N, C)), np.ones((N, C))
    else:
        raise ValueError(f"unknown normalization {normalization!r}")
    return shift[None].astype(np.float32), scale[None].astype(np.float32)


class CursorIds(NamedTuple):
    """Batch ids read on the device: row ``cursor[0] % table.shape[0]`` of ``table`` [rows, B]
    (int64). The optimiser's update advances the cursor, so a HIP graph of several training steps
    walks the table without any host work between them."""
    table: torch.Tensor
    cursor: torch.Tensor


class DeviceStore:
    """All windows of a :class:`WindowSet`, resident on one device."""

    def __init__(self, windows: WindowSet, normalization: str, graph_cfg, device="cpu",
                 feature_dtype=torch.float32):
        self.windows = windows
        self.ds_type = windows.ds_type
        self.per_sensor = windows.per_sensor
        self.normalization = normalization
        self.device = torch.device(device)
        G = len(windows.groups)
        N = windows.max_nodes
        T_tot = max(g.n_time for g in windows.groups)
        C = windows.groups[0].features.shape[1]
        self.n_nodes, self.n_feat, self.seq_len = N, C, windows.seq_len
        self.tb = int(round(windows.timestep_before / windows.freq))
        series = np.zeros((G, T_tot, N, C), np.float32)
        shifts, scales = [], []
        adj = np.zeros((G, N, N), np.float32)
        anom_pos = np.full(G, -1, np.int64)
        t_var = normalization in ("rolling_median", "rolling_median_fractional", "rolling_mean")
        Tn = T_tot if t_var else 1
        shift_all = np.zeros((G, Tn, N, C), np.float32)
        scale_all = np.ones((G, Tn, N, C), np.float32)
        for gi, g in enumerate(windows.groups):
            n = g.n_nodes
            series[gi, : g.n_time, :n] = np.nan_to_num(g.features.transpose(2, 0, 1), nan=0.0)
            sh, sc = _norm_arrays(g, normalization)
            shift_all[gi, : sh.shape[0], :n] = np.nan_to_num(sh, nan=0.0, posinf=0.0, neginf=0.0)
            scale_all[gi, : sc.shape[0], :n] = np.nan_to_num(sc, nan=0.0, posinf=0.0, neginf=0.0)
            adj[gi, :n, :n] = build_adjacency(graph_cfg, g.distances, g.depths, g.ds_type)
            anom_pos[gi] = g.anomalous_pos
        dev = self.device
        self.series = torch.from_numpy(series).to(dev, feature_dtype)
        self.shift = torch.from_numpy(shift_all).to(dev)
        self.scale = torch.from_numpy(scale_all).to(dev)
        self.time_varying_norm = t_var
        self.group_adj = torch.from_numpy(adj).to(dev)
        self.group_anom_pos = torch.from_numpy(anom_pos).to(dev)
        # per-window tables
        wg, wl = windows.flat()
        centers = np.concatenate([ix.center for ix in windows.indices])
        valid = np.zeros((len(centers), N), bool)
        off = 0
        for ix in windows.indices:
            valid[off: off + ix.size, : ix.node_valid.shape[1]] = ix.node_valid
            off += ix.size
        self.win_group = torch.from_numpy(wg).to(dev)
        self.win_center = torch.from_numpy(centers).to(dev)
        self.win_valid = torch.from_numpy(valid).to(dev)
        self.win_valid_u8 = self.win_valid.to(torch.uint8).contiguous()
        if self.per_sensor:
            lab = np.concatenate([ix.labels for ix in windows.indices]).astype(np.float32)
            self.win_label = torch.from_numpy(lab).to(dev)
            self.win_label_valid = None
        else:
            lab = np.zeros((len(centers), N), np.float32)
            lv = np.zeros((len(centers), N), np.float32)
            off = 0
            for ix in windows.indices:
                n = ix.labels.shape[1]
                lab[off: off + ix.size, :n] = ix.labels
                lv[off: off + ix.size, :n] = ix.label_valid
                off += ix.size
            self.win_label = torch.from_numpy(lab).to(dev)
            self.win_label_valid = torch.from_numpy(lv).to(dev)
        self.t_offsets = torch.arange(-self.tb, self.seq_len - self.tb, device=dev)

    def gcn_fused_data(self, agg_mean: bool, pool: int) -> dict:
        """Operands of the fused gather + GCN kernels (``gcn_fused.hip``): the store tensors plus
        the per-window tables that depend only on the data (fp64 moments of each window's
        normalised values, the node pooling weights of each window for this aggregation / pooling),
        computed once per (aggregation, pooling) on first use - never inside a graph capture."""
        key = (bool(agg_mean), int(pool))
        cache = self.__dict__.setdefault("_gcn_fused", {})
        d = cache.get(key)
        if d is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("DeviceStore.gcn_fused_data: first use inside a HIP graph capture; call it "
                                   "(or run one eager step) before capturing")
            from ..utils.native import hip_ops
            mom, pw = hip_ops().gcn_window_prep(self.series, self.shift, self.scale, self.win_group, self.win_center,
                                                self.win_valid_u8, self.group_adj, self.group_anom_pos, self.tb,
                                                self.seq_len, self.time_varying_norm, bool(agg_mean), int(pool))
            d = {"fwd": (self.series, self.shift, self.scale, self.win_group, self.win_center, self.win_valid_u8,
                         self.win_label, self.group_anom_pos, mom, pw),
                 "bwd": (self.series, self.shift, self.scale, self.win_group, self.win_center, self.win_valid_u8,
                         self.group_anom_pos, pw),
                 "dims": (self.tb, self.seq_len, self.time_varying_norm),
                 "ca": self.n_feat, "mom": mom, "pw": pw}
            cache[key] = d
        return d

    @property
    def n_windows(self) -> int:
        return int(self.win_center.shape[0])

    def labels(self, ids=None) -> torch.Tensor:
        return self.win_label if ids is None else self.win_label[ids]

    def gather(self, wids, valid_sample: Optional[torch.Tensor] = None) -> Batch:
        """Cut a batch of windows out of the resident series (all on device).

        ``wids`` may contain -1 for padding slots; those samples get all-zero
        inputs and zero label masks. ``wids`` may also be a :class:`CursorIds` (multi-step
        graphs): the batch is row ``cursor % rows`` of a device id table, read on the device.
        """
        dev = self.device
        cur = wids if isinstance(wids, CursorIds) else None
        from ..ops import use_hip
        if use_hip(self.series) and self.series.dtype == torch.float32 and self.group_adj.dtype == torch.float32:
            # ONE launch: the normalised window cut + masks, adjacency, labels, flagged series
            from ..utils.native import hip_ops
            ops = hip_ops()
            e = self.series.new_zeros(0)
            el = e.long()
            vs = valid_sample.to(dev, torch.float32).contiguous() if valid_sample is not None else e
            lv = self.win_label_valid if self.win_label_valid is not None else e
            if cur is not None:
                args = (el, cur.table, cur.cursor)
            else:
                args = (wids.to(dev).long().contiguous(), el, None)
            x, vm, adj, ap, y, y_mask, anom, wid = ops.batch_gather(
                self.series, self.shift, self.scale, self.win_group, self.win_center, self.win_valid_u8, *args,
                self.group_adj, self.group_anom_pos, self.win_label, lv, vs, self.tb, self.seq_len,
                self.time_varying_norm)
            return Batch(x=x, adj=adj, node_mask=vm, anom=anom if self.per_sensor else None, anom_pos=ap,
                         y=y, y_mask=y_mask, wid=wid, per_sensor=self.per_sensor)
        if cur is not None:
            wids = cur.table[cur.cursor[0] % cur.table.shape[0]]
        wids = wids.to(dev)
        pad = wids < 0
        w = wids.clamp(min=0)
        g = self.win_group[w]
        c = self.win_center[w]
        valid = self.win_valid[w] & ~pad[:, None]                    # [B, N]
        vm = valid.to(torch.float32)
        t = c[:, None] + self.t_offsets[None, :]                     # [B, T]
        x = self.series[g[:, None], t].float()                       # [B, T, N, C]
        tc = c if self.time_varying_norm else torch.zeros_like(c)
        sh = self.shift[g, tc]                                       # [B, N, C]
        sc = self.scale[g, tc]
        x = (x - sh[:, None]) * sc[:, None] * vm[:, None, :, None]
        adj = self.group_adj[g] * vm[:, :, None] * vm[:, None, :]
        ap = self.group_anom_pos[g]
        sample_ok = (~pad).to(x.dtype)
        if valid_sample is not None:
            sample_ok = sample_ok * valid_sample.to(x.dtype)
        if self.per_sensor:
            idx = ap.clamp(min=0)
            anom = x[torch.arange(x.shape[0], device=dev), :, idx]   # [B, T, C]
            y = self.win_label[w] * sample_ok
            y_mask = sample_ok
        else:
            anom = None
            y = self.win_label[w] * vm
            y_mask = self.win_label_valid[w] * sample_ok[:, None]
        return Batch(x=x, adj=adj, node_mask=vm, anom=anom, anom_pos=ap, y=y, y_mask=y_mask, wid=wids,
                     per_sensor=self.per_sensor)


class DeviceLoader:
    """Shuffling, rank-sharded batch iterator over window ids (all on device).

    Replaces tf.data ``shuffle(shuffle_size, seed, reshuffle_each_iteration=True)
    .batch(batch_size)`` (``libs/preprocessing_functions.py:959-962``) with a full
    per-epoch permutation. Each rank reads a disjoint strided shard of the global
    permutation; batches are padded to ``batch_size`` (pad id -1) so shapes are static.
    """

    def __init__(self, store: DeviceStore, window_ids, batch_size: int, shuffle: bool = True,
                 seed: int = 44, rank: int = 0, world_size: int = 1, drop_last: bool = False):
        self.store = store
        self.ids = torch.as_tensor(np.asarray(window_ids, dtype=np.int64)).to(store.device)
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.seed = int(seed)
        self.rank, self.world = int(rank), int(world_size)
        self.drop_last = drop_last
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def _order(self):
        n = self.ids.numel()
        if self.shuffle:
            gen = torch.Generator(device="cpu")
            gen.manual_seed(self.seed + 1000003 * self.epoch)
            perm = torch.randperm(n, generator=gen).to(self.ids.device)
            ids = self.ids[perm]
        else:
            ids = self.ids
        # shard: global batch = batch_size * world; rank r takes slots r::world
        gb = self.batch_size * self.world
        n_batches = (n // gb) if self.drop_last else -(-n // gb)
        total = n_batches * gb
        if total > n:
            ids = torch.cat([ids, torch.full((total - n,), -1, dtype=ids.dtype, device=ids.device)])
        else:
            ids = ids[:total]
        return ids.view(n_batches, self.batch_size, self.world)[:, :, self.rank]

    def __len__(self):
        gb = self.batch_size * self.world
        n = self.ids.numel()
        return (n // gb) if self.drop_last else -(-n // gb)

    def batch_ids(self):
        return self._order()

    def __iter__(self):
        for row in self._order():
            yield self.store.gather(row)


__all__ = ["Batch", "CursorIds", "DeviceStore", "DeviceLoader"]
