"""TimeLayer: stacked temporal encoder (``libs/create_model.py:43-136``).

LSTM branch: ``LSTM(f) -> LSTM(f) -> MaxPool(p)``, then ``n_stacks`` x
[``LSTM(f*2^(i+1)) x 2 -> MaxPool(p)``], then ``LSTM(f*2^(n+1))`` returning the last
state. CNN branch: the same pattern with ``Conv1D(same) + LeakyReLU(alpha)`` and a
final ``GlobalAveragePooling1D``. (The reference's TimeLayer hard-codes pool size 3
for the CNN stack pools, ``:99``; the baseline uses ``pool_size``, ``:320``.)

Attribute names mirror the reference (``time1, time2, time_layers, pooling_layers,
time4``) so checkpoint variable paths line up.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn

from .layers import LSTM, Conv1D, GlobalAveragePooling1D, LeakyReLU, MaxPooling1D


def _pair_fusion() -> bool:
    """Layer-pair forward fusion (``lstm_tm2_fwd``); ``GNNQC_NO_PAIR=1`` disables it."""
    return os.environ.get("GNNQC_NO_PAIR", "0") != "1"


class TimeLayer(nn.Module):
    def __init__(self, in_features: int, filter_1_size: int = 8, n_stacks: int = 2, layer_type: str = "lstm",
                 activation: str = "tanh", kernel_size: Optional[int] = 5, regularizer: Optional[float] = None,
                 pool_size: int = 3, alpha: float = 0.3, cnn_stack_pool: Optional[int] = 3,
                 compute_bf16: bool = True):
        super().__init__()
        self.layer_type = layer_type
        self.filter_1_size, self.n_stacks, self.pool_size, self.alpha = filter_1_size, n_stacks, pool_size, alpha
        f = filter_1_size
        self.time_layers = nn.ModuleList()
        self.pooling_layers = nn.ModuleList()
        if layer_type == "lstm":
            mk = lambda i, o, seq=True: LSTM(i, o, activation, seq, regularizer, compute_bf16)  # noqa: E731
            self.time1 = mk(in_features, f)
            self.time2 = mk(f, f)
            self.max_pooling = MaxPooling1D(pool_size)
            prev = f
            for i in range(n_stacks):
                u = f * 2 ** (i + 1)
                self.time_layers.append(mk(prev, u))
                self.time_layers.append(mk(u, u))
                self.pooling_layers.append(MaxPooling1D(pool_size))
                prev = u
            self.time4 = mk(prev, f * 2 ** (n_stacks + 1), False)
        else:
            if kernel_size is None:
                raise ValueError("CNN TimeLayer needs kernel_size")
            self.time1 = Conv1D(in_features, f, kernel_size, regularizer=regularizer, compute_bf16=compute_bf16)
            self.time2 = Conv1D(f, f, kernel_size, regularizer=regularizer, compute_bf16=compute_bf16)
            self.leakyrelu1 = LeakyReLU(alpha)
            self.leakyrelu2 = LeakyReLU(alpha)
            self.max_pooling = MaxPooling1D(pool_size)
            self.leakyrelu_layers = nn.ModuleList()
            prev = f
            for i in range(n_stacks):
                u = f * 2 ** (i + 1)
                self.time_layers.append(Conv1D(prev, u, kernel_size, regularizer=regularizer, compute_bf16=compute_bf16))
                self.leakyrelu_layers.append(LeakyReLU(alpha))
                self.time_layers.append(Conv1D(u, u, kernel_size, regularizer=regularizer, compute_bf16=compute_bf16))
                self.leakyrelu_layers.append(LeakyReLU(alpha))
                self.pooling_layers.append(MaxPooling1D(cnn_stack_pool or pool_size))
                prev = u
            self.time4 = Conv1D(prev, f * 2 ** (n_stacks + 1), kernel_size, regularizer=regularizer,
                               compute_bf16=compute_bf16)
            self.leakyrelu3 = LeakyReLU(alpha)
            self.global_pooling = GlobalAveragePooling1D()

    @property
    def out_features(self) -> int:
        return self.filter_1_size * 2 ** (self.n_stacks + 1)

    def _sequence(self):
        """The layer/pool sequence of the LSTM branch, in execution order."""
        seq = [self.time1, self.time2, self.max_pooling]
        for i in range(len(self.pooling_layers)):
            seq += [self.time_layers[2 * i], self.time_layers[2 * i + 1], self.pooling_layers[i]]
        return seq + [self.time4]

    def _forward_tm(self, x: torch.Tensor) -> torch.Tensor:
        """GPU LSTM branch: the leading H <= 32 layers (and their pools) run time-major
        ([T, Mp, C], fused-backward kernels); the rest continues sequence-major."""
        import torch.nn.functional as F
        M = x.shape[0]
        Mp = (M + 15) // 16 * 16
        cpad = (-x.shape[-1]) % 4          # float4 loader granules: zero channels up to a multiple of 4
        h = x.float().transpose(0, 1)
        if Mp != M or cpad:
            h = F.pad(h, (0, cpad, 0, Mp - M))
        return self.forward_time_major(h.contiguous(), M)

    def forward_time_major(self, h: torch.Tensor, M: int, last=None) -> torch.Tensor:
        """LSTM branch on a time-major input ``[T, Mp, C]`` (Mp = M rounded up to 16, zero
        rows past M; C may carry zero channels past the first layer's input width).
        Returns ``[M, out_features]``. Producers that can write this layout directly (the
        SoilNet GCN kernel) skip the transpose/pad copy of :meth:`_forward_tm`."""
        from ..ops.lstm import (_chain_on, last128_eligible, lstm_chain_tm, lstm_last128_tm, lstm_layer_tm,
                                lstm_pair_tm, pool_fusion, tm_eligible)
        from ..ops.pool import max_pool1d_tm
        if self.layer_type != "lstm":
            # CNN branch behind a time-major producer (the store-fused CML GCN front end): [M, T, Cin]
            cin = self.time1.kernel.shape[1]
            return self._forward_cnn(h.transpose(0, 1)[:M, :, :cin].contiguous())
        tm = True
        seq = self._sequence()
        i = 0
        plan = self._chain_plan(seq, h) if _chain_on() else None
        if plan is not None:                      # leading layers + pools: one pipelined launch
            mods, pools, i = plan
            h = lstm_chain_tm(h, mods, pools)
        while i < len(seq):
            mod = seq[i]
            i += 1
            if isinstance(mod, MaxPooling1D):
                h = max_pool1d_tm(h, mod.pool_size) if tm else mod(h)
                continue
            nxt = seq[i] if i < len(seq) else None

            def fused_pool(j, units):
                # a MaxPooling1D right after the layer(s): pooled inside their autograd node, and the
                # backward recurrence un-pools the pooled gradient on load (no maxpool1d_bwd pass)
                p = seq[j] if j < len(seq) else None
                if (isinstance(p, MaxPooling1D) and pool_fusion() and units % 4 == 0 and h.shape[-1] % 4 == 0
                        and 1 <= p.pool_size <= 255 and h.shape[0] // p.pool_size >= 1):
                    return p.pool_size
                return 0

            if (tm and isinstance(nxt, LSTM) and mod.return_sequences and nxt.return_sequences
                    and mod.units <= 32 and nxt.units == mod.units and nxt.kernel.shape[0] == mod.units and _pair_fusion()
                    and tm_eligible(h, mod.units, h.shape[-1], mod.activation, mod.compute_bf16)
                    and nxt.activation == mod.activation and nxt.compute_bf16 == mod.compute_bf16):
                i += 1
                P = fused_pool(i, mod.units)
                h = lstm_pair_tm(h, mod, nxt, P)   # two layers, one pipelined forward kernel
                i += 1 if P else 0
                continue
            if tm and tm_eligible(h, mod.units, h.shape[-1], mod.activation, mod.compute_bf16):
                P = fused_pool(i, mod.units) if mod.return_sequences else 0
                h = lstm_layer_tm(h, mod.kernel, mod.recurrent_kernel, mod.bias, mod.return_sequences, P)
                i += 1 if P else 0
                if not mod.return_sequences:
                    return h[:M]
                continue
            if tm and last128_eligible(h, mod):      # time4 (H = 128, last state) on the time-major input
                # (``last(h, mod)``: the caller takes this layer over, e.g. fused with a frozen head)
                return last(h, mod) if last is not None else lstm_last128_tm(h, mod)[:M]
            if tm:                                   # leave time-major: [T, Mp, C] -> [M, T, C]
                h = h.transpose(0, 1)
                if h.shape[0] != M:                  # (a no-op slice would still cost a zero-fill + copy in backward)
                    h = h[:M]
                if h.shape[-1] != mod.kernel.shape[0]:   # (only if the first layer is not time-major)
                    h = h[..., : mod.kernel.shape[0]]
                h = h.contiguous()
                tm = False
            h = mod(h)
        return h

    def head_chain_ok(self, h: torch.Tensor) -> bool:
        """Whether the whole LSTM branch of a time-major input ``h`` [T, Mp, C] runs as the chain +
        time4/head kernels (:func:`gnnqc.ops.lstm.lstm_chain_head_tm`): every layer but the last in
        the chain plan, the last one H = 128 returning its last state after <= 16 steps."""
        from ..ops.lstm import _chain_on
        if self.layer_type != "lstm" or not _chain_on() or os.environ.get("GNNQC_HEAD_CHAIN", "1") != "1":
            return False
        seq = self._sequence()
        plan = self._chain_plan(seq, h)
        if plan is None or plan[2] != len(seq) - 1:
            return False
        last = seq[-1]
        mods, pools, _ = plan
        T = h.shape[0]
        for p in pools:
            T = T // p if p else T
        return (isinstance(last, LSTM) and not last.return_sequences and last.units == 128
                and last.activation == "tanh" and last.compute_bf16 and 1 <= T <= 16
                and mods[-1].units % 4 == 0 and mods[-1].units <= 64 and last.kernel.shape[0] == mods[-1].units)

    def forward_time_major_head(self, h: torch.Tensor, M: int, head, alphas, y: torch.Tensor, mask: torch.Tensor,
                                w0: float, w1: float, sums=None, hist=None):
        """(loss, logits) of the LSTM branch + classifier head + weighted BCE on a time-major
        input (see :meth:`head_chain_ok`), one launch forward and one backward."""
        from ..ops.lstm import lstm_chain_head_tm
        mods, pools, _ = self._chain_plan(self._sequence(), h)
        return lstm_chain_head_tm(h, list(mods) + [self.time4], list(pools), head, y, mask, M,
                                  alphas[0], alphas[1], w0, w1, sums, hist)

    @staticmethod
    def _chain_plan(seq, h: torch.Tensor):
        """Leading run of time-major LSTM layers (returning sequences, each optionally followed
        by a MaxPooling1D) that the cross-CU chain kernel takes: ``(modules, pools, next index)``
        or None. Constraints of ``lstm_chain.hip``: H in {16, 32, 64}, inputs <= 64 channels and
        no wider than the layer, all workgroups co-resident (``chain_fits``)."""
        from ..ops import use_hip
        from ..ops.lstm import chain_fits
        T, Mp, din = h.shape
        if not use_hip(h) or din % 4 or h.data_ptr() % 16:
            return None
        mods, pools = [], []
        i = 0
        while i < len(seq):
            mod = seq[i]
            if not (isinstance(mod, LSTM) and mod.return_sequences and mod.activation == "tanh" and mod.compute_bf16
                    and mod.units in (16, 32, 64)):
                break
            Dw = mod.kernel.shape[0]
            if din > 64 or Dw > din or (mods and din > mod.units) or T >= 4096:
                break
            j, pool = i + 1, 0
            if j < len(seq) and isinstance(seq[j], MaxPooling1D):
                P = seq[j].pool_size
                if not (1 <= P <= 255 and T // P >= 1):
                    break
                pool, j = P, j + 1
            mods.append(mod)
            pools.append(pool)
            T = T // pool if pool else T
            din = mod.units
            i = j
            if pool not in (0, 3):       # consumer-side pooling takes 3; others end the chain
                break
        if not chain_fits(Mp, len(mods), h.device):
            return None
        return mods, pools, i

    def _forward_cnn(self, x: torch.Tensor) -> torch.Tensor:
        """CNN branch (``create_model.py:80-101``): every Conv1D + LeakyReLU pair is one fused
        kernel on the GPU, and the last one also folds in the GlobalAveragePooling1D."""
        x1 = self.time1.forward_act(x, self.leakyrelu1.alpha)
        x1 = self.time2.forward_act(x1, self.leakyrelu2.alpha)
        x1 = self.max_pooling(x1)
        for i in range(len(self.pooling_layers)):
            x1 = self.time_layers[2 * i].forward_act(x1, self.leakyrelu_layers[2 * i].alpha)
            x1 = self.time_layers[2 * i + 1].forward_act(x1, self.leakyrelu_layers[2 * i + 1].alpha)
            x1 = self.pooling_layers[i](x1)
        return self.time4.forward_act(x1, self.leakyrelu3.alpha, gap=True)

    def time_major_ok(self, x: torch.Tensor, channels: int) -> bool:
        """Whether :meth:`forward_time_major` can take a ``channels``-wide input on x's device."""
        return self._tm_ok(x, channels)

    def _tm_ok(self, x: torch.Tensor, channels: Optional[int] = None) -> bool:
        from ..ops.lstm import tm_eligible
        c = x.shape[-1] if channels is None else int(channels)
        return (self.layer_type == "lstm" and self.time1.activation == "tanh"
                and tm_eligible(x, self.time1.units, c + (-c) % 4, self.time1.activation,
                                self.time1.compute_bf16)
                and os.environ.get("GNNQC_NO_TM", "0") != "1")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._tm_ok(x):
            return self._forward_tm(x)
        if self.layer_type != "lstm":
            return self._forward_cnn(x)
        x1 = self.time1(x)
        x1 = self.time2(x1)
        x1 = self.max_pooling(x1)
        for i in range(len(self.pooling_layers)):
            x1 = self.time_layers[2 * i](x1)
            x1 = self.time_layers[2 * i + 1](x1)
            x1 = self.pooling_layers[i](x1)
        x1 = self.time4(x1)
        return x1


__all__ = ["TimeLayer"]
