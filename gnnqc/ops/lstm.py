"""Keras-semantics LSTM layer.

Gate order i, f, c(g), o; ``z_t = x_t W + h_{t-1} U + b``; recurrent activation
sigmoid; ``activation`` (tanh by default) for g and the cell output; zero initial
state (Keras ``LSTM`` as built by ``libs/create_model.py:61-79``).

GPU path: one library GEMM for the input projection of all T steps, then the
persistent HIP recurrence (``lstm_fwd``); backward = persistent BPTT kernel
(``lstm_bwd``) producing dz for all steps, then the weight/input gradients as
plain GEMMs over all (sequence, step) rows.
"""
from __future__ import annotations

import contextlib
from typing import Optional

import torch

_ACT = {
    "tanh": torch.tanh,
    "relu": torch.relu,
    "sigmoid": torch.sigmoid,
    "linear": lambda x: x,
    None: lambda x: x,
}


def lstm_eager(x: torch.Tensor, W: torch.Tensor, U: torch.Tensor, b: torch.Tensor,
               return_sequences: bool = True, activation: str = "tanh") -> torch.Tensor:
    """Reference implementation: x [M,T,Din], W [Din,4H], U [H,4H], b [4H]. Inside
    :func:`gnnqc.ops.lstm_ref.kernel_rounding` it rounds where the HIP kernels do (numerics tests)."""
    from .lstm_ref import KernelLSTM, kernel_rounding_on
    if kernel_rounding_on() and activation == "tanh":
        return KernelLSTM.apply(x, W, U, b, bool(return_sequences), True)
    act = _ACT[activation]
    M, T, _ = x.shape
    H = U.shape[0]
    xp = torch.matmul(x, W) + b
    h = x.new_zeros(M, H)
    c = x.new_zeros(M, H)
    outs = []
    for t in range(T):
        z = xp[:, t] + h @ U
        i, f, g, o = z.split(H, dim=-1)
        i, f, o = torch.sigmoid(i), torch.sigmoid(f), torch.sigmoid(o)
        c = f * c + i * act(g)
        h = o * act(c)
        if return_sequences:
            outs.append(h)
    return torch.stack(outs, 1) if return_sequences else h


class _DirectGrad:
    """When enabled (by the training engine), LSTM weight gradients are accumulated by the
    ``lstm_grads`` kernels straight into ``param.grad`` (the optimiser's flat gradient
    buffer views) instead of being returned to autograd - no separate AccumulateGrad add
    per parameter. Off by default so that ``torch.autograd.grad`` (e.g. integrated
    gradients) never touches ``.grad``. In this mode the weight-gradient passes are deferred
    and batched (:class:`_Pipe`).

    (Measured on MI355X and removed: dW/dU/db on a side stream behind a dx-only kernel -
    0.885 vs 0.757 ms/step, cross-stream event waits cost more than the overlap won - and the
    chain's weight-gradient batch on a side stream concurrent with the GCN backward, 0.3812 vs
    0.3788 ms/step.)"""

    enabled = False


class _Pipe:
    """Pipelined backward (direct-accumulation mode only; measured 0.667 vs 0.709 ms/step for
    one weight-gradient kernel per layer behind its recurrence, the fallback for layers the pipe
    does not take).

    A layer's weight-gradient pass does not feed any later recurrence, so it is deferred:
    each time-major backward recurrence launches ONE kernel (``lstm_tm_bwd_pipe``) whose
    first workgroups run the recurrence (a handful of tiles - most CUs idle) while the
    remaining workgroups run the weight-gradient pass of the previously finished layer and
    the split reduction of the one before. dx of the layer is a separate small kernel
    (the next recurrence's input). Leftover work is flushed when the direct-accumulation
    context exits. Single stream: ordering is plain stream order, no events."""

    enabled = True  # (tests switch it off to compare with the per-layer fused backward)
    job = None      # layer whose weight-gradient pass has not run yet
    red = None      # layer whose gradient pass ran; its split reduction has not
    batch = []      # jobs of a chain backward: all gradient passes in one launch at the flush
    gcn = None      # (gcn_t, gcn_i): the fused GCN backward, run as extra workgroups of that launch


# Largest sequence count (rows of 16-sequence tiles) a recurrence may have for its layer to
# join the pipe: the gradient workgroups only help when the recurrence leaves most CUs idle
# (CML: 8 tiles). With hundreds of tiles (SoilNet: 418) they compete with the recurrence
# for the CUs and the step got slower (6.11 vs 5.15 ms), so such layers keep the fused path.
PIPE_MAX_SEQ = 2048


_MULTI_MAX = 12        # jobs per lstm_grads_multi launch (lstm_tm.hip MULTI_MAX)


def _pipe_on(sinks, n_seq: int) -> bool:
    return _Pipe.enabled and _DirectGrad.enabled and all(d for _, d in sinks) and n_seq <= PIPE_MAX_SEQ


def _pipe_job(dz, x, h, W, sinks, period: int, hshift: int):
    from ..utils.native import hip_ops
    H = W.shape[1] // 4
    return dict(dz=dz, x=x, h=h, W=W, period=int(period), hshift=int(hshift),
                ws=hip_ops().lstm_grads_job_ws(dz, x, W, H), g=[s for s, _ in sinks])


def _pipe_launch(dh=None, g=None, c=None, W=None, U=None, T: int = 0, job=None, red=None):
    """One pipe kernel: [recurrence] + [grads of ``job``] + [reduce of ``red``]. Returns dz."""
    from ..utils.native import hip_ops
    ref = dh if dh is not None else (job or red)["dz"]
    e = ref.new_zeros(0)
    rec = (dh, g, c, W, U) if dh is not None else (e, e, e, e, e)
    jb = (job["dz"], job["x"], job["h"], job["W"], job["period"], job["hshift"], job["ws"]) if job else \
        (e, e, e, e, 1, 1, e)
    rd = (red["ws"], red["W"], *red["g"]) if red else (e, e, e, e, e)
    return hip_ops().lstm_tm_bwd_pipe(*rec, int(T), *jb, *rd)


def _pipe_drain_one():
    """Advance the pending jobs by one stage without a recurrence."""
    job, red = _Pipe.job, _Pipe.red
    if job is None and red is None:
        return
    _pipe_launch(job=job, red=red)
    _Pipe.job, _Pipe.red = None, job


def defer_to_grads_launch(gcn_lists) -> bool:
    """Queue the fused GCN backward (``lstm_grads_multi``'s gcn_t / gcn_i lists) onto the pending
    batched weight-gradient launch of this backward: the two are independent, and one launch
    overlaps them on the CUs the recurrences left idle. False (the caller launches it itself) when
    no batch is pending or ``GNNQC_GCN_DEFER=0``."""
    import os
    if not (_DirectGrad.enabled and _Pipe.batch and _Pipe.gcn is None and os.environ.get("GNNQC_GCN_DEFER", "1") == "1"):
        return False
    _Pipe.gcn = gcn_lists
    return True


def pipe_flush():
    """Run all pending weight-gradient / reduction work (end of the backward). With a chain
    backward's batch: every pending gradient pass in ONE launch, every reduction in one more."""
    if _Pipe.batch:
        from ..utils.native import hip_ops
        grads = ([_Pipe.job] if _Pipe.job is not None else []) + _Pipe.batch
        reds = ([_Pipe.red] if _Pipe.red is not None else []) + grads
        gt, gi = _Pipe.gcn if _Pipe.gcn is not None else ([], [])
        hip_ops().lstm_grads_multi([j["dz"] for j in grads], [j["x"] for j in grads], [j["h"] for j in grads],
                                   [j["W"] for j in grads], [j["period"] for j in grads],
                                   [j["hshift"] for j in grads], [j["ws"] for j in grads],
                                   [r["ws"] for r in reds], [r["W"] for r in reds], [r["g"][0] for r in reds],
                                   [r["g"][1] for r in reds], [r["g"][2] for r in reds], gt, gi)
        _Pipe.job, _Pipe.red, _Pipe.batch, _Pipe.gcn = None, None, [], None
    while _Pipe.job is not None or _Pipe.red is not None:
        _pipe_drain_one()


def _pipe_push(job):
    """Queue ``job``: if a job is still pending (no recurrence consumed it), advance first."""
    if _Pipe.job is not None:
        _pipe_drain_one()
    _Pipe.job = job


def _pipe_tm_backward(dh, g, c, x, h, W, U, sinks, need_dx):
    """Time-major layer backward in pipe mode: one pipe launch (recurrence + pending grads +
    pending reduce), dx = dz W^T, then this layer's own weight-gradient job is queued."""
    from ..utils.native import hip_ops
    T, Mp = x.shape[0], x.shape[1]
    HR = U.shape[0]
    if dh.dim() == 2:        # gradient only at the last step
        dh = torch.nn.functional.pad(dh.unsqueeze(0), (0, 0, 0, 0, T - 1, 0))
    job, red = _Pipe.job, _Pipe.red
    if job is not None and job["W"].shape[1] // 4 not in (HR, 2 * HR):
        _pipe_drain_one()              # shape the fused kernel does not take: run it alone
        job, red = _Pipe.job, _Pipe.red
    dz = _pipe_launch(dh, g, c, W, U, T, job, red)
    _Pipe.job, _Pipe.red = None, job
    dx = hip_ops().lstm_dx(dz, W, x) if need_dx else None
    _pipe_push(_pipe_job(dz, x, h, W, sinks, T * Mp, Mp))
    return dx


def _pipe_x_ok(x: torch.Tensor, Dw: int) -> bool:
    return (x.stride(-1) == 1 and x.stride(-2) % 4 == 0 and x.data_ptr() % 16 == 0 and (Dw + 16) // 16 <= 5
            and x.shape[-1] % 4 == 0)


@contextlib.contextmanager
def _deferred_reduce(on: bool):
    """Queue the split reductions of the weight-gradient launches issued inside (direct
    accumulation into the optimiser's gradient buffers only: nothing reads those before the
    step's optimizer update) for :func:`direct_grad_accumulation`'s exit, which runs all of them
    in one launch (``lstm_reduce_flush``) instead of one reduce launch per layer."""
    import os
    if not (on and _DirectGrad.enabled and os.environ.get("GNNQC_DEFER_REDUCE", "1") == "1"):
        yield
        return
    from ..utils.native import hip_ops
    ops = hip_ops()
    prev = ops.lstm_defer_reduce(True)
    _Deferred.pending = True
    try:
        yield
    finally:
        ops.lstm_defer_reduce(prev)


class _Deferred:
    pending = False     # split reductions queued in the native library (lstm_reduce_flush)


@contextlib.contextmanager
def direct_grad_accumulation(flag: bool = True):
    prev = _DirectGrad.enabled
    _DirectGrad.enabled = flag
    try:
        yield
    finally:
        _DirectGrad.enabled = prev
        if _Pipe.job is not None or _Pipe.red is not None or _Pipe.batch:
            pipe_flush()
        _Pipe.gcn = None
        if _Deferred.pending:
            from ..utils.native import hip_ops
            _Deferred.pending = False
            hip_ops().lstm_reduce_flush()


class _Unflagged:
    count = 0     # gradients handed back to autograd (summed into .grad by PyTorch: no non-finite flag)


def unflagged_grad_writes() -> int:
    """How many weight gradients so far went through autograd's own accumulation instead of a HIP
    kernel that raises the non-finite flag (chain control word 7). The trainer takes the flag-driven
    Adam only for steps whose backward added none (``gnnqc.train.engine.Trainer._body``)."""
    return _Unflagged.count


def _grad_sink(p: torch.Tensor):
    g = p.grad if _DirectGrad.enabled and isinstance(p, torch.nn.Parameter) else None
    if g is not None and g.is_contiguous() and g.dtype == torch.float32 and g.device == p.device:
        return g, True
    _Unflagged.count += 1
    return torch.zeros_like(p), False


class _HipLSTM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, U, b, bf16: bool, return_sequences: bool):
        from ..utils.native import hip_ops
        ops = hip_ops()
        # rows may be padded (e.g. a channel-padded producer): only unit inner stride needed
        if not (x.stride(2) == 1 and x.stride(0) == x.shape[1] * x.stride(1)):
            # (.contiguous() keeps odd strides on size-1 dims, e.g. T = 1 cut from a time-major view)
            x = x.clone(memory_format=torch.contiguous_format)
        need = any(ctx.needs_input_grad[:4])
        h, c, g = ops.lstm_fwd(x, W.contiguous(), U.contiguous(), b.contiguous(), need, bf16)
        ctx.bf16 = bf16
        ctx.return_sequences = return_sequences
        ctx.params = (W, U, b)       # leaf Parameters (for direct gradient accumulation)
        if need:
            ctx.save_for_backward(x, W, U, h, c, g)
        return h if return_sequences else h[:, -1]

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        ops = hip_ops()
        x, W, U, h, c, g = ctx.saved_tensors
        M, T, Din = x.shape
        H = U.shape[0]
        if ctx.return_sequences:
            dh = dout.contiguous()
        else:
            # gradient only at the last step: one constant-pad launch (not zeros + slice copy)
            dh = torch.nn.functional.pad(dout.unsqueeze(1), (0, 0, T - 1, 0))
        dz = ops.lstm_bwd(dh, g, c, U.contiguous(), ctx.bf16)
        if not ctx.bf16:
            # fp32 numerics-reference mode: exact fp32 GEMMs for the weight gradients
            dz2 = dz.reshape(M * T, 4 * H)
            dx = (dz2 @ W.t()).view(M, T, Din) if ctx.needs_input_grad[0] else None
            dW = torch.einsum("mtd,mtg->dg", x, dz) if ctx.needs_input_grad[1] else None
            dU = None
            if ctx.needs_input_grad[2]:
                dU = torch.einsum("mth,mtg->hg", h[:, :-1], dz[:, 1:]) if T > 1 else torch.zeros_like(U)
            db = dz2.sum(0) if ctx.needs_input_grad[3] else None
            return dx, dW, dU, db, None, None
        if not any(ctx.needs_input_grad[1:4]):
            # frozen weights (integrated gradients): only dx = dz W^T (bf16 dz: one HIP pass)
            dx = None
            if ctx.needs_input_grad[0]:
                if Din % 4 == 0 and Din <= 128:
                    dx = ops.lstm_dx(dz, W.contiguous(), x)
                else:
                    dx = (dz.reshape(M * T, 4 * H).float() @ W.t()).view(M, T, Din)
            return dx, None, None, None, None, None
        Wp, Up, bp = ctx.params
        gW, dW_in = _grad_sink(Wp)
        gU, dU_in = _grad_sink(Up)
        gb, db_in = _grad_sink(bp)
        need_dx = bool(ctx.needs_input_grad[0])
        Wc = W.contiguous()
        if (dW_in and dU_in and db_in and _pipe_on(((gW, True),), M) and _pipe_x_ok(x, W.shape[0])):
            # sequence-major recurrence (H = 128); the weight-gradient job joins the pipe
            dx = ops.lstm_dx(dz, Wc, x) if need_dx else None
            _pipe_push(_pipe_job(dz, x, h, Wc, ((gW, True), (gU, True), (gb, True)), T, 1))
            return dx, None, None, None, None, None
        with _deferred_reduce(dW_in and dU_in and db_in):
            dx = ops.lstm_grads(dz, x, h, Wc, gW, gU, gb, need_dx)
        return (dx if need_dx else None,
                None if dW_in or not ctx.needs_input_grad[1] else gW,
                None if dU_in or not ctx.needs_input_grad[2] else gU,
                None if db_in or not ctx.needs_input_grad[3] else gb,
                None, None)


def _tm_layer_backward(dout, x, W, U, b, h, g, c, params, need_w, need_dx):
    """Backward of one time-major layer (the pipe when it takes the layer, else one fused kernel).
    Returns dx (or None) and the three weight gradients to hand to autograd (None where they
    were accumulated directly into ``.grad``)."""
    from ..utils.native import hip_ops
    wgrad = any(need_w)
    if not wgrad and not need_dx:
        return None, [None, None, None]
    if wgrad:
        sinks = [_grad_sink(p) for p in params]
    else:
        e = x.new_zeros(0)
        sinks = [(e, True)] * 3
    Wc, Uc = W.contiguous(), U.contiguous()
    if wgrad and g.numel() > 0 and _pipe_on(sinks, x.shape[1]) and _pipe_x_ok(x, W.shape[0]):
        dx = _pipe_tm_backward(dout.contiguous(), g, c, x, h, Wc, Uc, sinks, need_dx)
    else:
        with _deferred_reduce(wgrad and all(d for _, d in sinks)):
            dx = hip_ops().lstm_tm_bwd(dout.contiguous(), g, c, x, h, Wc, Uc, b.contiguous(), sinks[0][0],
                                       sinks[1][0], sinks[2][0], need_dx)
    grads = [None if (direct or not n) else buf for (buf, direct), n in zip(sinks, need_w)]
    return (dx if need_dx else None), grads


class _HipLSTMChain(torch.autograd.Function):
    """A stack of time-major layers (with MaxPooling1D between some of them) whose forward
    runs as ONE cross-CU pipelined kernel (``lstm_chain.hip``: every layer of a 16-sequence
    tile on its own CU, consuming the previous layer's output as it is produced). The
    backward runs the per-layer backward kernels in reverse, un-pooling between them."""

    @staticmethod
    def forward(ctx, x, pools, *params):
        from ..utils.native import hip_ops
        ns = len(pools)
        Ws = [params[3 * i].contiguous() for i in range(ns)]
        Us = [params[3 * i + 1].contiguous() for i in range(ns)]
        bs = [params[3 * i + 2].contiguous() for i in range(ns)]
        need = any(ctx.needs_input_grad)
        outs = hip_ops().lstm_chain_fwd(x, Ws, Us, bs, [int(p) for p in pools], need)
        ctx.pools = tuple(int(p) for p in pools)
        ctx.params = params
        if need:
            ctx.save_for_backward(x, *Ws, *Us, *outs)
        last = outs[5 * (ns - 1):]
        return last[3] if pools[-1] else last[0]

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        ops = hip_ops()
        pools = ctx.pools
        ns = len(pools)
        saved = ctx.saved_tensors
        x, Ws, Us, outs = saved[0], saved[1:1 + ns], saved[1 + ns:1 + 2 * ns], saved[1 + 2 * ns:]
        need = ctx.needs_input_grad
        grads = [None] * (3 * ns)
        dh = dout.contiguous()
        dx = None

        def layer_x(i):
            if i == 0:
                return x
            return outs[5 * (i - 1) + 3] if pools[i - 1] else outs[5 * (i - 1)]

        if _chain_bwd_on() and chain_fits(dh.shape[1], ns, dh.device) and all(layer_x(i).shape[-1] % 4 == 0 for i in range(ns)):
            # all reverse recurrences in ONE cross-CU pipelined launch (dz of every layer + dx
            # of the bottom one), then the weight-gradient passes
            order = list(reversed(range(ns)))
            e8 = x.new_zeros(0, dtype=torch.uint8)
            res = ops.lstm_chain_bwd(dh, [outs[5 * i + 1] for i in order], [outs[5 * i + 2] for i in order],
                                     [Ws[i] for i in order], [Us[i] for i in order],
                                     [outs[5 * i + 4] if pools[i] else e8 for i in order],
                                     [pools[i] for i in order], [layer_x(i).shape[-1] for i in order],
                                     [outs[5 * i].shape[0] for i in order])
            for k, i in enumerate(order):
                nw = need[2 + 3 * i:5 + 3 * i]
                if not any(nw):
                    continue
                h = outs[5 * i]
                xi = layer_x(i)
                sinks = [_grad_sink(p) for p in ctx.params[3 * i:3 * i + 3]]
                if (_pipe_on(sinks, h.shape[1]) and _pipe_x_ok(xi, Ws[i].shape[0])
                        and len(_Pipe.batch) < _MULTI_MAX - 2):
                    _Pipe.batch.append(_pipe_job(res[k], xi, h, Ws[i], sinks, h.shape[0] * h.shape[1], h.shape[1]))
                else:
                    ops.lstm_tm_grads(res[k], xi, h, Ws[i], sinks[0][0], sinks[1][0], sinks[2][0], False)
                grads[3 * i:3 * i + 3] = [None if (direct or not n) else buf for (buf, direct), n in zip(sinks, nw)]
            dx = res[ns]
            return (dx if need[0] else None, None, *grads)
        for i in reversed(range(ns)):
            h, g, c, _, idx = outs[5 * i:5 * i + 5]
            T, Mp, H = h.shape
            if pools[i]:
                dh = ops.maxpool1d_bwd(dh.view(1, -1, Mp * H), idx.view(1, -1, Mp * H), T, pools[i]).view(T, Mp, H)
            if i == 0:
                xi = x
            else:
                xi = outs[5 * (i - 1) + 3] if pools[i - 1] else outs[5 * (i - 1)]
            need_dx = i > 0 or bool(need[0])
            dx, gr = _tm_layer_backward(dh, xi, Ws[i], Us[i], ctx.params[3 * i + 2], h, g, c,
                                        ctx.params[3 * i:3 * i + 3], need[2 + 3 * i:5 + 3 * i], need_dx)
            grads[3 * i:3 * i + 3] = gr
            dh = dx
        return (dx if need[0] else None, None, *grads)


class _HipLSTMChainHead(torch.autograd.Function):
    """CML TimeLayer + classifier head + weighted BCE in two forward and two backward launches:
    the six pipelined time-major layers as ONE chain kernel (``lstm_chain.hip``), then time4
    (H = 128, last state) with the Dense head, the loss and the metric accumulation as ONE
    kernel (``time4_head.hip``); backward: the head backward + time4's reverse recurrence as ONE
    kernel, whose dx (gradient of the chain's pooled output) feeds ONE chain backward. The
    weight-gradient passes of all seven layers then run as one ``lstm_grads_multi`` launch.

    Inputs: x [T, Mp, C] time-major, y / mask [M]; ``consts`` = (alpha1, alpha2, w0, w1);
    params = 7 x (W, U, b) then the head's (W1, b1, W2, b2, W3, b3). Returns (loss, logits [M])."""

    @staticmethod
    def forward(ctx, x, y, mask, sums, hist, consts, pools, M, *params):
        from ..utils.native import hip_ops
        ops = hip_ops()
        ns = len(pools)                    # chain stages (time4 follows)
        Ws = [params[3 * i].contiguous() for i in range(ns + 1)]
        Us = [params[3 * i + 1].contiguous() for i in range(ns + 1)]
        bs = [params[3 * i + 2].contiguous() for i in range(ns + 1)]
        head = [p.contiguous() for p in params[3 * (ns + 1):]]
        need = any(ctx.needs_input_grad)
        e = x.new_zeros(0)
        sums_ = sums if sums is not None else e.double()
        hist_ = hist if hist is not None else e
        if _t4_chain_on() and pools[-1] == 3:
            # time4 + head + loss as one more stage of the chain launch (it consumes the last
            # stage's output as it is produced); spare workgroups build time4's backward fragments
            outs = ops.lstm_chain_head_fwd(x, Ws[:ns], Us[:ns], bs[:ns], [int(p) for p in pools], need, Ws[ns],
                                           Us[ns], bs[ns], head, y, mask, int(M), *[float(c) for c in consts],
                                           sums_, hist_)
            h4, g4, c4, logits, loss = outs[-5:]
            del outs[-5:]
            hb = outs.pop()       # the head backward precomputed by the launch (dL/dloss = 1), or empty
            pk = outs.pop()
        else:
            # (the chain's spare workgroups build time4's weight-fragment image on the way)
            outs = ops.lstm_chain_fwd_pack(x, Ws[:ns], Us[:ns], bs[:ns], [int(p) for p in pools], need, Ws[ns],
                                           Us[ns])
            pk = outs.pop()
            hb = e
            xt = outs[5 * (ns - 1) + 3] if pools[-1] else outs[5 * (ns - 1)]      # time4's input [T4, Mp, C]
            h4, g4, c4, logits, loss = ops.time4_head_fwd(xt, Ws[ns], Us[ns], bs[ns], pk, need, head, y, mask, int(M),
                                                          *[float(c) for c in consts], sums_, hist_)
        ctx.pools, ctx.consts, ctx.M = tuple(int(p) for p in pools), tuple(float(c) for c in consts), int(M)
        ctx.params = params
        ctx.set_materialize_grads(False)     # (no zeros tensor for the non-differentiable logits)
        if need:
            ctx.save_for_backward(x, y, mask, *Ws, *Us, *head, *outs, h4, g4, c4, pk, hb)
        ctx.mark_non_differentiable(logits)
        return loss.reshape(()), logits

    @staticmethod
    def backward(ctx, dloss, _dlogits):
        from ..utils.native import hip_ops
        ops = hip_ops()
        pools = ctx.pools
        ns = len(pools)
        saved = ctx.saved_tensors
        x, y, mask = saved[:3]
        Ws, Us = saved[3:4 + ns], saved[4 + ns:5 + 2 * ns]
        head = saved[5 + 2 * ns:11 + 2 * ns]
        outs = saved[11 + 2 * ns:11 + 7 * ns]
        h4, g4, c4, pk, hb = saved[11 + 7 * ns:]
        need = ctx.needs_input_grad
        npar = 3 * (ns + 1)

        def layer_x(i):
            if i == 0:
                return x
            return outs[5 * (i - 1) + 3] if pools[i - 1] else outs[5 * (i - 1)]

        g = dloss.reshape(1).float()
        if not g.is_contiguous():
            g = g.contiguous()
        hsinks = [_grad_sink(p) for p in ctx.params[npar:]]
        xt = layer_x(ns)
        order = list(reversed(range(ns)))
        e8 = x.new_zeros(0, dtype=torch.uint8)
        chain_args = ([outs[5 * i + 1] for i in order], [outs[5 * i + 2] for i in order],
                      [Ws[i] for i in order], [Us[i] for i in order],
                      [outs[5 * i + 4] if pools[i] else e8 for i in order],
                      [pools[i] for i in order], [layer_x(i).shape[-1] for i in order],
                      [outs[5 * i].shape[0] for i in order])
        grads = [None] * npar
        sinks = {i: [_grad_sink(p) for p in ctx.params[3 * i:3 * i + 3]] for i in range(ns + 1)}
        if _t4_chain_on() and pools[-1] == 3 and xt.is_contiguous():
            # time4 + head backward as the first stage of the chain backward launch: the top
            # chain stage consumes time4's dx as it is produced
            res = ops.lstm_chain_head_bwd(g, xt, h4, g4, c4, Ws[ns], Us[ns], pk, hb, list(head), y, mask, ctx.M, *ctx.consts,
                                          [s for s, _ in hsinks], *chain_args)
            dz4 = res.pop(0)
        else:
            dz4, dxt = ops.time4_head_bwd(g, xt, h4, g4, c4, Ws[ns], Us[ns], pk, list(head), y, mask, ctx.M,
                                          *ctx.consts, [s for s, _ in hsinks])
            res = ops.lstm_chain_bwd(dxt, *chain_args)
        dzs = {ns: dz4}
        hs = {ns: h4}
        for k, i in enumerate(order):
            dzs[i] = res[k]
            hs[i] = outs[5 * i]
        for i in [ns] + order:
            nw = need[8 + 3 * i:11 + 3 * i]
            if not any(nw):
                continue
            h = hs[i]
            xi = layer_x(i)
            sk = sinks[i]
            if (_pipe_on(sk, h.shape[1]) and _pipe_x_ok(xi, Ws[i].shape[0])
                    and len(_Pipe.batch) < _MULTI_MAX - 2):
                _Pipe.batch.append(_pipe_job(dzs[i], xi, h, Ws[i], sk, h.shape[0] * h.shape[1], h.shape[1]))
            else:
                ops.lstm_tm_grads(dzs[i], xi, h, Ws[i], sk[0][0], sk[1][0], sk[2][0], False)
            grads[3 * i:3 * i + 3] = [None if (direct or not n) else buf for (buf, direct), n in zip(sk, nw)]
        hgrads = [None if (direct or not n) else buf for (buf, direct), n in zip(hsinks, need[8 + npar:])]
        dx = res[ns]
        return (dx if need[0] else None, None, None, None, None, None, None, None, *grads, *hgrads)


def lstm_chain_head_tm(x_tm: torch.Tensor, mods, pools, head, y: torch.Tensor, mask: torch.Tensor, M: int,
                       alpha1: float, alpha2: float, w0: float, w1: float, sums=None, hist=None):
    """(loss, logits) of ``mods`` (LSTM modules: the chain layers, then time4 - H = 128 returning its
    last state) followed by the Dense head ``head`` = (dense, dense2, dense_out) and the weighted
    BCE. ``pools``: the chain layers' pools (time4 has none)."""
    params = []
    for m in mods:
        params += [m.kernel, m.recurrent_kernel, m.bias]
    for d in head:
        params += [d.kernel, d.bias]
    return _HipLSTMChainHead.apply(x_tm, y, mask, sums, hist, (alpha1, alpha2, w0, w1), tuple(int(p) for p in pools),
                                   int(M), *params)


def _chain_bwd_on() -> bool:
    """Cross-CU pipelined backward of the chain (``GNNQC_CHAIN_BWD``, default on)."""
    import os
    return os.environ.get("GNNQC_CHAIN_BWD", "1") == "1"


def _t4_chain_on() -> bool:
    """time4 + head as a stage of the chain launches (``lstm_chain_head_fwd`` / ``_bwd``;
    ``GNNQC_T4_CHAIN``, default on) instead of their own launches after / before the chain."""
    import os
    return os.environ.get("GNNQC_T4_CHAIN", "1") == "1"


def _chain_on() -> bool:
    """Cross-CU pipelined forward of the time-major LSTM stack (``GNNQC_CHAIN``, default on)."""
    import os
    return os.environ.get("GNNQC_CHAIN", "1") == "1"


def lstm_chain_tm(x_tm: torch.Tensor, mods, pools) -> torch.Tensor:
    """Forward of stacked LSTM modules (``gnnqc.models.layers.LSTM``, all returning sequences)
    with ``pools[i]`` > 0 a MaxPooling1D after module i; returns the last stage's output."""
    params = []
    for m in mods:
        params += [m.kernel, m.recurrent_kernel, m.bias]
    return _HipLSTMChain.apply(x_tm, tuple(int(p) for p in pools), *params)


_CHAIN_CAP = {}


def chain_capacity(device) -> int:
    """Chain workgroups that can be resident at once on ``device``: its CU count (queried: a
    partitioned MI355X exposes 32 or 64) times the occupancy of the 1024-thread chain kernels."""
    device = torch.device(device)
    if device.type != "cuda":
        return 0
    idx = device.index if device.index is not None else torch.cuda.current_device()
    cap = _CHAIN_CAP.get(idx)
    if cap is None:
        from ..utils.native import hip_ops
        cap = int(hip_ops().lstm_chain_capacity(torch.empty(0, device=torch.device("cuda", idx))))
        _CHAIN_CAP[idx] = cap
    return cap


def chain_fits(Mp: int, n_stages: int, device=None, spare: int = 0) -> bool:
    """All workgroups of a chain launch must be co-resident (one 1024-thread workgroup per CU);
    ``spare``: workgroups needed besides the stages' (the weight-gradient role of the backward)."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    return (2 <= n_stages <= 8 and n_stages * ((Mp // 16 + 7) // 8 * 8) + spare <= chain_capacity(device))


_CHAIN_CTL = {}


def chain_ctl(device) -> Optional[torch.Tensor]:
    """The device's chain control words ``[epoch, finished, timeout flag, rejected steps, fwd / bwd
    head tickets, debug spin limit, non-finite gradient flag, head backward arrivals, 0 ...]`` as an
    int32[16] view (``lstm_chain.hip``); None off the GPU. The optimiser's update reads and clears
    the timeout / non-finite flags inside the captured step."""
    device = torch.device(device)
    if device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    t = _CHAIN_CTL.get(idx)
    if t is None:
        from ..utils.native import hip_ops
        t = hip_ops().lstm_chain_ctl(torch.empty(0, device=torch.device("cuda", idx)))
        _CHAIN_CTL[idx] = t
    return t


class ChainTimeoutError(RuntimeError):
    """A chain consumer gave up waiting for its producer (not all workgroups were resident, or
    another kernel held the CUs): the affected results were computed from stale data."""


def check_chain(device, rejected_before: Optional[int] = None) -> int:
    """Raise :class:`ChainTimeoutError` if a chain spin timed out since the last check (forward-only
    use: evaluation, prediction) or if training steps were rejected for it since
    ``rejected_before``. Synchronises. Returns the current rejected-step count."""
    ctl = chain_ctl(device)
    if ctl is None:
        return 0
    v = ctl.cpu().tolist()
    if v[2]:
        ctl[2:3].zero_()
        raise ChainTimeoutError("LSTM chain kernel: a consumer spin timed out; results of this pass are invalid "
                                "(is another kernel sharing the GPU, or is the device partitioned?)")
    if rejected_before is not None and v[3] > rejected_before:
        raise ChainTimeoutError(f"LSTM chain kernel: {v[3] - rejected_before} training step(s) rejected after a "
                                "consumer spin timeout (skipped on the device, parameters untouched)")
    return int(v[3])


class _HipLSTMTM(torch.autograd.Function):
    """Time-major LSTM layer (``lstm_tm.hip``): x [T, Mp, Din] -> h [T, Mp, H] (or the last
    step [Mp, H]). The backward is ONE fused kernel: recurrence, dx, and dW/dU/db
    accumulated straight into the gradient buffers (direct mode) or returned."""

    @staticmethod
    def forward(ctx, x, W, U, b, return_sequences: bool, pool: int = 0):
        from ..utils.native import hip_ops
        x = x.contiguous()
        need = any(ctx.needs_input_grad[:4])
        sg = not recompute_gates(x, U.shape[0], any(ctx.needs_input_grad[1:4]))
        h, g, c = hip_ops().lstm_tm_fwd(x, W.contiguous(), U.contiguous(), b.contiguous(), need, sg)
        ctx.params = (W, U, b)
        ctx.return_sequences = return_sequences
        out, idx = _pool_out(h, pool) if (pool and return_sequences) else (h, x.new_zeros(0, dtype=torch.uint8))
        ctx.pool = int(pool) if return_sequences else 0
        if need:
            ctx.save_for_backward(x, W, U, b, h, g, c, idx)
        return out if return_sequences else h[-1]

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        x, W, U, b, h, g, c, idx = ctx.saved_tensors
        need = ctx.needs_input_grad
        wgrad = any(need[1:4])
        need_dx = bool(need[0])
        if not wgrad and not need_dx:
            return None, None, None, None, None
        if wgrad:
            sinks = [_grad_sink(p) for p in ctx.params]
        else:
            e = x.new_zeros(0)
            sinks = [(e, True)] * 3
        if wgrad and g.numel() > 0 and _pipe_on(sinks, x.shape[1]) and _pipe_x_ok(x, W.shape[0]):
            dout = _unpool(dout, idx, ctx.pool, h.shape[0])
            dx = _pipe_tm_backward(dout.contiguous(), g, c, x, h, W.contiguous(), U.contiguous(), sinks, need_dx)
        else:
            with _deferred_reduce(wgrad and all(d for _, d in sinks)):
                dx = hip_ops().lstm_tm_bwd(dout.contiguous(), g, c, x, h, W.contiguous(), U.contiguous(),
                                           b.contiguous(), sinks[0][0], sinks[1][0], sinks[2][0], need_dx,
                                           idx if ctx.pool else None, ctx.pool)
        grads = [None if (direct or not n) else buf for (buf, direct), n in zip(sinks, need[1:4])]
        return (dx if need_dx else None, *grads, None, None)


class _HipLSTMTMPair(torch.autograd.Function):
    """Two stacked time-major layers A (Din -> H) and B (H -> H), both returning sequences:
    ONE wavefront-pipelined forward kernel (``lstm_tm2_fwd``); the backward runs the
    per-layer kernels (B first, its dx is A's dh). (A pipelined pair backward was measured
    slower - 148 vs 118 us for the CML H=16 pair: B's in-loop dx MFMAs and A's waves share each
    SIMD's MFMA pipe - and removed.)"""

    @staticmethod
    def forward(ctx, x, WA, UA, bA, WB, UB, bB, pool: int = 0):
        from ..utils.native import hip_ops
        x = x.contiguous()
        need = any(ctx.needs_input_grad[:7])
        sg = not recompute_gates(x, UA.shape[0], any(ctx.needs_input_grad[1:7]))
        import os
        # (pooling by layer B's storer lanes in the same launch measured slower than the separate
        # maxpool pass - SoilNet 3.21 vs 3.11 ms, IG 4.84 vs 4.74 ms per call, profiles/r6_pool_in_fwd_ab.txt,
        # as in round 3 - so it is opt-in)
        kp = int(pool) if (pool and os.environ.get("GNNQC_TM_POOL_IN_FWD", "0") == "1") else 0
        hA, gA, cA, hB, gB, cB, pooled, pidx = hip_ops().lstm_tm2_fwd(
            x, WA.contiguous(), UA.contiguous(), bA.contiguous(), WB.contiguous(), UB.contiguous(), bB.contiguous(),
            need, sg, kp)
        ctx.params = (WA, UA, bA, WB, UB, bB)
        if kp:                            # pooled by layer B's storer lanes in the same launch
            out, idx = pooled, pidx
        else:
            out, idx = _pool_out(hB, pool) if pool else (hB, x.new_zeros(0, dtype=torch.uint8))
        ctx.pool = int(pool)
        if need:
            ctx.save_for_backward(x, WA, UA, bA, hA, gA, cA, WB, UB, bB, hB, gB, cB, idx)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        ops = hip_ops()
        x, WA, UA, bA, hA, gA, cA, WB, UB, bB, hB, gB, cB, idx = ctx.saved_tensors
        need = ctx.needs_input_grad
        e = x.new_zeros(0)
        dout = dout.contiguous()

        def sinks(params, flags):
            if any(flags):
                return [_grad_sink(p) for p in params]
            return [(e, True)] * 3

        sB = sinks(ctx.params[3:], need[4:7])
        sA = sinks(ctx.params[:3], need[1:4])
        need_dx = bool(need[0])
        dx = None
        if (any(need[4:7]) and any(need[1:4]) and gA.numel() > 0 and _pipe_on(sB, x.shape[1])
                and _pipe_on(sA, x.shape[1])
                and _pipe_x_ok(x, WA.shape[0]) and _pipe_x_ok(hA, WB.shape[0])):
            dout = _unpool(dout, idx, ctx.pool, hB.shape[0])
            dhA = _pipe_tm_backward(dout, gB, cB, hA, hB, WB.contiguous(), UB.contiguous(), sB, True)
            dx = _pipe_tm_backward(dhA, gA, cA, x, hA, WA.contiguous(), UA.contiguous(), sA, need_dx)
        else:
            with _deferred_reduce(all(d for _, d in sB) and all(d for _, d in sA)):
                dhA = ops.lstm_tm_bwd(dout, gB, cB, hA, hB, WB.contiguous(), UB.contiguous(), bB.contiguous(),
                                      sB[0][0], sB[1][0], sB[2][0], True, idx if ctx.pool else None, ctx.pool)
                if need_dx or any(need[1:4]):
                    dx = ops.lstm_tm_bwd(dhA, gA, cA, x, hA, WA.contiguous(), UA.contiguous(), bA.contiguous(),
                                         sA[0][0], sA[1][0], sA[2][0], need_dx)
        gA_ = [None if (direct or not n) else buf for (buf, direct), n in zip(sA, need[1:4])]
        gB_ = [None if (direct or not n) else buf for (buf, direct), n in zip(sB, need[4:7])]
        return (dx if need_dx else None, *gA_, *gB_, None)


def _pool_out(h: torch.Tensor, pool: int):
    """MaxPooling1D(pool) of a time-major [T, Mp, H] output inside a layer's autograd node: (pooled
    [T // pool, Mp, H], byte argmax). The node's backward then takes the pooled gradient and the
    recurrence un-pools it on load (``lstm_tm_bwd`` pidx)."""
    from ..utils.native import hip_ops
    T, Mp, H = h.shape
    y, idx = hip_ops().maxpool1d_fwd(h.contiguous().view(1, T, Mp * H), int(pool))
    return y.view(T // pool, Mp, H), idx.view(T // pool, Mp, H)


def _unpool(dout: torch.Tensor, idx: torch.Tensor, pool: int, T: int) -> torch.Tensor:
    """Full-resolution gradient of a fused pool (paths whose recurrence does not un-pool on load)."""
    if not pool:
        return dout
    from ..utils.native import hip_ops
    Ts, Mp, H = dout.shape
    return hip_ops().maxpool1d_bwd(dout.contiguous().view(1, Ts, Mp * H), idx.view(1, Ts, Mp * H), T,
                                   int(pool)).view(T, Mp, H)


def pool_fusion() -> bool:
    """Whether a MaxPooling1D after a time-major layer (pair) runs inside that layer's autograd node
    with the un-pooling done by the recurrence's dh loads (``GNNQC_TM_POOL_FUSE=0``: separate pool)."""
    import os
    return os.environ.get("GNNQC_TM_POOL_FUSE", "1") == "1"


def lstm_pair_tm(x_tm, A, B, pool: int = 0) -> torch.Tensor:
    """Fused forward of two stacked LSTM modules (``gnnqc.models.layers.LSTM``), optionally followed
    by MaxPooling1D(``pool``) in the same autograd node."""
    return _HipLSTMTMPair.apply(x_tm, A.kernel, A.recurrent_kernel, A.bias, B.kernel, B.recurrent_kernel, B.bias,
                                int(pool))


def recompute_gates(x: torch.Tensor, H: int, weight_grads: bool) -> bool:
    """Whether a time-major layer's forward saves no gates and its backward recomputes them from
    x_t and h_{t-1} (``lstm_tm.hip`` RG: bitwise the forward's pre-activations; halves the forward's
    state stream). H in {16, 32}, 16-byte x granules, and the backward must take the fused kernel:
    frozen weights (integrated gradients), or too many sequences for the pipelined backward
    (``PIPE_MAX_SEQ``). ``GNNQC_TM_RG=0`` keeps the saved gates."""
    import os
    if os.environ.get("GNNQC_TM_RG", "1") != "1" or H not in (16, 32):
        return False
    Din = x.shape[-1]
    if Din % 4 or Din > 64 or x.data_ptr() % 16 or not x.is_contiguous():
        return False
    return (not weight_grads) or x.shape[1] > PIPE_MAX_SEQ or not _Pipe.enabled


def tm_eligible(x: torch.Tensor, H: int, Din: int, activation: str = "tanh", bf16: bool = True) -> bool:
    """Whether the time-major kernels handle this layer (GPU, bf16, tanh, H in {16, 32, 64})."""
    from . import use_hip
    return (use_hip(x) and bf16 and activation == "tanh" and H in (16, 32, 64) and 1 <= Din <= 127
            and (16 * Din) // (4 if Din % 4 == 0 else (2 if Din % 2 == 0 else 1)) <= 16 * H)


def lstm_layer_tm(x_tm: torch.Tensor, W: torch.Tensor, U: torch.Tensor, b: torch.Tensor,
                  return_sequences: bool = True, pool: int = 0) -> torch.Tensor:
    """Time-major layer ``[T, Mp, Din] -> [T, Mp, H]`` (or the last step), optionally followed by
    MaxPooling1D(``pool``) in the same autograd node."""
    return _HipLSTMTM.apply(x_tm, W, U, b, bool(return_sequences), int(pool))


class _HipLSTMLast128(torch.autograd.Function):
    """An H = 128 layer returning its last state on a time-major input [T, Mp, Din] (T <= 16):
    ``time4_head.hip`` in its standalone mode (``time4_fwd`` / ``time4_bwd``: no head, compact
    saved state, workgroups looping over 16-sequence tiles). Replaces, for the time layer's last
    LSTM (time4, ``libs/create_model.py:61-79``), the sequence-major lstm_fwd<128> / lstm_bwd /
    lstm_dx kernels and the [T, Mp, C] <-> [M, T, C] copies around them. Weight gradients: the
    backward's dz through ``lstm_tm_grads`` (the training chain-head path's weight pass)."""

    @staticmethod
    def forward(ctx, x, W, U, b):
        from ..utils.native import hip_ops
        x = x.contiguous()
        need = any(ctx.needs_input_grad[:4])
        wgrad = any(ctx.needs_input_grad[1:4])
        h, g, c = hip_ops().time4_fwd(x, W.contiguous(), U.contiguous(), b.contiguous(), need, wgrad)
        ctx.params = (W, U, b)
        if need:
            ctx.save_for_backward(x, W, U, g, c, h if wgrad else x.new_zeros(0))
        return h[-1] if wgrad else h

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        ops = hip_ops()
        x, W, U, g, c, h = ctx.saved_tensors
        need = ctx.needs_input_grad
        wgrad = any(need[1:4])
        Wc = W.contiguous()
        dz, dx = ops.time4_bwd(dout.contiguous(), x, g, c, Wc, U.contiguous(), wgrad)
        grads = [None, None, None]
        if wgrad:
            sinks = [_grad_sink(p) for p in ctx.params]
            with _deferred_reduce(all(d for _, d in sinks)):
                ops.lstm_tm_grads(dz, x, h, Wc, sinks[0][0], sinks[1][0], sinks[2][0], False)
            grads = [None if (direct or not n) else buf for (buf, direct), n in zip(sinks, need[1:4])]
        return (dx if need[0] else None, *grads)


class _HipLSTMLast128Prob(torch.autograd.Function):
    """time4 (as :class:`_HipLSTMLast128`) + the FROZEN Dense head for integrated gradients:
    ``time4_prob_fwd`` returns the head's sigmoid outputs and, from the same launch,
    d prob / d h_{T-1}; the backward scales those rows by d loss / d prob and runs the time4
    recurrence (``time4_bwd`` row_scale): input gradient only (weights and head frozen)."""

    @staticmethod
    def forward(ctx, x, W, U, b, head, alphas, M):
        from ..utils.native import hip_ops
        x = x.contiguous()
        need = bool(ctx.needs_input_grad[0])
        prob, dh, g, c = hip_ops().time4_prob_fwd(x, W.contiguous(), U.contiguous(), b.contiguous(),
                                                  [t.contiguous() for t in head], float(alphas[0]),
                                                  float(alphas[1]), int(M), need)
        if need:
            ctx.save_for_backward(x, W, U, g, c, dh)
        ctx.M = int(M)
        return prob[:M]

    @staticmethod
    def backward(ctx, dprob):
        from ..utils.native import hip_ops
        x, W, U, g, c, dh = ctx.saved_tensors
        scale = dprob.float().contiguous()          # [M]: the rows past M get no gradient
        _, dx = hip_ops().time4_bwd(dh, x, g, c, W.contiguous(), U.contiguous(), False, 0, scale)
        return dx, None, None, None, None, None, None


def lstm_last128_prob_tm(x_tm: torch.Tensor, mod, head, alphas, M: int) -> torch.Tensor:
    """Sigmoid outputs [M] of LSTM module ``mod`` (H = 128, last state; see ``last128_eligible``) and
    the frozen head ``head`` = [W1, b1, W2, b2, W3, b3] with LeakyReLU slopes ``alphas``."""
    if any(t.requires_grad for t in [mod.kernel, mod.recurrent_kernel, mod.bias, *head]):
        raise ValueError("lstm_last128_prob_tm: weights must be frozen (integrated gradients)")
    return _HipLSTMLast128Prob.apply(x_tm, mod.kernel, mod.recurrent_kernel, mod.bias, tuple(head), tuple(alphas), int(M))


def last128_eligible(x: torch.Tensor, mod) -> bool:
    """Whether :class:`_HipLSTMLast128` takes LSTM module ``mod`` on time-major ``x`` [T, Mp, Din]
    (``GNNQC_T4_TM=0``: the sequence-major kernels)."""
    import os
    from . import use_hip
    if os.environ.get("GNNQC_T4_TM", "1") != "1" or not use_hip(x) or x.dim() != 3:
        return False
    T, Mp, Din = x.shape
    return (mod.units == 128 and not mod.return_sequences and mod.activation == "tanh" and mod.compute_bf16
            and 1 <= T <= 16 and Mp % 16 == 0 and Din % 4 == 0 and 4 <= Din <= 64
            and mod.kernel.shape[0] <= Din and x.dtype == torch.float32)


def lstm_last128_tm(x_tm: torch.Tensor, mod) -> torch.Tensor:
    """Last state [Mp, 128] of LSTM module ``mod`` on time-major ``x_tm`` (see ``last128_eligible``)."""
    return _HipLSTMLast128.apply(x_tm, mod.kernel, mod.recurrent_kernel, mod.bias)


def lstm_layer(x: torch.Tensor, W: torch.Tensor, U: torch.Tensor, b: torch.Tensor,
               return_sequences: bool = True, activation: str = "tanh", bf16: bool = True) -> torch.Tensor:
    """Dispatch: HIP persistent kernel on GPU (tanh, H multiple of 16), eager otherwise."""
    from . import use_hip
    H = U.shape[0]
    if use_hip(x) and activation == "tanh" and H % 16 == 0 and H in (16, 32, 64, 128) and x.shape[-1] <= 128:
        return _HipLSTM.apply(x, W, U, b, bool(bf16), bool(return_sequences))
    return lstm_eager(x, W, U, b, return_sequences, activation)


__all__ = ["unflagged_grad_writes", "lstm_layer", "lstm_eager", "lstm_layer_tm", "lstm_pair_tm", "lstm_chain_tm", "chain_fits", "tm_eligible",
           "chain_capacity", "chain_ctl", "check_chain", "ChainTimeoutError", "lstm_chain_head_tm",
           "lstm_last128_tm", "lstm_last128_prob_tm", "last128_eligible",
           "direct_grad_accumulation"]
