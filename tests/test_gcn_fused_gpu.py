"""Store-fused CML front end (``gcn_fused.hip``: window gather + GeneralConv + BatchNorm + PReLU +
node pooling in one launch, parameter gradients with float atomics in one launch) against the
generic path (batch_gather -> gcn_prep -> gcn_pool_fwd; gcn_pool_bwd -> gcn_bwd_finalize), and the
whole training step through both paths."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda_device, cml_windows, seed=0):
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    pc, ws = cml_windows
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    torch.manual_seed(seed)
    mc = C.default("model_cml")
    model = GCNClassifier(mc, pc).to(cuda_device)
    with torch.no_grad():
        g = model.gcn_layer
        g.bn_gamma.uniform_(0.5, 1.5)
        g.bn_beta.normal_(0, 0.2)
        g.prelu_alpha.uniform_(0.0, 0.4)
        g.bias.normal_(0, 0.1)
    return pc, st, model


def _ids(st, B, cuda_device, pad=0):
    ids = torch.randperm(st.n_windows, generator=torch.Generator().manual_seed(3))[:B].to(cuda_device)
    if pad:
        ids[-pad:] = -1
    return ids


@pytest.mark.parametrize("pooling", ["mean", "selection"])
@pytest.mark.parametrize("training", [True, False])
def test_fused_front_end_matches_generic(cuda_device, cml_windows, pooling, training):
    from gnnqc.ops.gcn import gcn_pool, gcn_pool_from_store, store_gcn_ok
    _, st, model = _setup(cuda_device, cml_windows)
    g = model.gcn_layer
    ids = _ids(st, 100, cuda_device, pad=4)
    assert store_gcn_ok(st, g, training, pooling)
    b = st.gather(ids)
    rm0, rv0 = g.bn_moving_mean.clone(), g.bn_moving_variance.clone()
    x, anom, adj, mask, ap = b.model_inputs("cml")
    h0, M0 = gcn_pool(x, adj, mask, anom, ap, g.kernel, g.bias, g.bn_gamma, g.bn_beta, g.prelu_alpha,
                      g.bn_moving_mean, g.bn_moving_variance, training, g.aggregate, pooling, g.momentum, g.eps,
                      0.0, time_major=True)
    rm_generic, rv_generic = g.bn_moving_mean.clone(), g.bn_moving_variance.clone()
    with torch.no_grad():
        g.bn_moving_mean.copy_(rm0)
        g.bn_moving_variance.copy_(rv0)
    h1, M1, y, ym, wid = gcn_pool_from_store(st, ids, g, training, pooling)
    torch.cuda.synchronize()
    assert M1 == M0 and h1.shape == h0.shape
    torch.testing.assert_close(h1, h0, atol=2e-5, rtol=2e-5)
    torch.testing.assert_close(y, b.y)
    torch.testing.assert_close(ym, b.y_mask)
    assert torch.equal(wid, ids)
    torch.testing.assert_close(g.bn_moving_mean, rm_generic, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(g.bn_moving_variance, rv_generic, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("coef", ["1", "0"])
def test_fused_front_end_gradients_match_generic(cuda_device, cml_windows, monkeypatch, coef):
    """Parameter gradients of the fused backward (per-workgroup closed form + atomics) equal the
    generic two-launch backward on the same upstream gradient - both in the coefficient form
    (GNNQC_GCN_COEF=1: the forward writes per-(t, sample, feature) coefficients, the backward is
    dh x coef) and in the recomputing form."""
    from gnnqc.ops.gcn import gcn_pool, gcn_pool_from_store
    from gnnqc.ops.lstm import direct_grad_accumulation
    monkeypatch.setenv("GNNQC_GCN_COEF", coef)
    _, st, model = _setup(cuda_device, cml_windows)
    g = model.gcn_layer
    ids = _ids(st, 128, cuda_device, pad=3)
    b = st.gather(ids)
    x, anom, adj, mask, ap = b.model_inputs("cml")
    params = [g.kernel, g.bias, g.bn_gamma, g.bn_beta, g.prelu_alpha]
    torch.manual_seed(5)
    T = st.seq_len
    dh = None
    out = {}
    for name in ("generic", "fused"):
        for p in params:
            p.grad = torch.zeros_like(p)
        with direct_grad_accumulation(True):
            if name == "generic":
                h, _ = gcn_pool(x, adj, mask, anom, ap, g.kernel, g.bias, g.bn_gamma, g.bn_beta, g.prelu_alpha,
                                g.bn_moving_mean, g.bn_moving_variance, True, g.aggregate, "mean", g.momentum, g.eps,
                                0.0, time_major=True)
            else:
                h = gcn_pool_from_store(st, ids, g, True, "mean")[0]
            if dh is None:
                dh = torch.randn_like(h)
                dh[:, 128:] = 0
            h.backward(dh)
        torch.cuda.synchronize()
        out[name] = [p.grad.clone() for p in params]
    assert T == h.shape[0]
    for n, a, r in zip(["W", "b", "gamma", "beta", "alpha"], out["fused"], out["generic"]):
        torch.testing.assert_close(a, r, atol=1e-4 * (r.abs().max().item() + 1e-3), rtol=1e-4, msg=n)


def test_two_forwards_before_backward_coef_side_job(cuda_device, cml_windows, monkeypatch):
    """Gradient accumulation over micro-batches: two store-fused forwards, then the backward of
    both. In the coefficient side mode the first forward's coefficient job is still pending when the
    second forward installs its own (no chain forward in between took it); it must be flushed, not
    dropped (dropped, the first backward would read an unwritten coefficient tensor). Parameter
    gradients equal the recomputing backward (GNNQC_GCN_COEF=0)."""
    from gnnqc.ops.gcn import gcn_pool_from_store
    from gnnqc.ops.lstm import direct_grad_accumulation
    _, st, model = _setup(cuda_device, cml_windows)
    g = model.gcn_layer
    params = [g.kernel, g.bias, g.bn_gamma, g.bn_beta, g.prelu_alpha]
    ids = [_ids(st, 128, cuda_device, pad=3), _ids(st, 128, cuda_device)[32:].contiguous()]
    gen = torch.Generator(device="cpu").manual_seed(11)
    dhs = None
    out = {}
    rm0, rv0 = g.bn_moving_mean.clone(), g.bn_moving_variance.clone()
    for coef in ("0", "1"):
        monkeypatch.setenv("GNNQC_GCN_COEF", coef)
        with torch.no_grad():
            g.bn_moving_mean.copy_(rm0)
            g.bn_moving_variance.copy_(rv0)
        for p in params:
            p.grad = torch.zeros_like(p)
        with direct_grad_accumulation(True):
            hs = [gcn_pool_from_store(st, i, g, True, "mean")[0] for i in ids]
            if dhs is None:
                dhs = [torch.randn(h.shape, generator=gen).to(cuda_device) for h in hs]
                dhs[0][:, 128:] = 0
                dhs[1][:, 96:] = 0
            for h, dh in zip(hs, dhs):
                h.backward(dh)
        torch.cuda.synchronize()
        out[coef] = [p.grad.clone() for p in params]
    for n, a, r in zip(["W", "b", "gamma", "beta", "alpha"], out["1"], out["0"]):
        torch.testing.assert_close(a, r, atol=1e-4 * (r.abs().max().item() + 1e-3), rtol=1e-4, msg=n)


def test_training_step_store_path_matches_gather_path(cuda_device, cml_windows, monkeypatch):
    """Two full training steps (forward, backward, guarded Adam) through the Trainer with the
    store-fused front end and with the generic gather path: same loss and parameters."""
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    _, st, model = _setup(cuda_device, cml_windows)
    ids = _ids(st, 128, cuda_device)
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("GNNQC_STORE_GCN", flag)
        m = copy.deepcopy(model)
        opt = make_optimizer("adam", m.parameters(), 1e-3)
        tr = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, use_graph=False, batch_size=128)
        assert tr._store_fused() == (flag == "1")
        losses = [float(tr.train_step(ids).item()) for _ in range(2)]
        torch.cuda.synchronize()
        res[flag] = (losses, {n: p.detach().clone() for n, p in m.named_parameters()})
    l1, p1 = res["1"]
    l0, p0 = res["0"]
    assert abs(l1[0] - l0[0]) <= 1e-4 * abs(l0[0]) + 1e-6, (l1, l0)
    assert abs(l1[1] - l0[1]) <= 2e-3 * abs(l0[1]) + 1e-5, (l1, l0)
    init = dict(model.named_parameters())
    for n in p0:
        d0 = p0[n] - init[n].detach()
        d1 = p1[n] - init[n].detach()
        # Adam turns a near-zero gradient into a +-lr step, so elements whose gradient is rounding
        # noise may flip: compare the update as a whole
        assert (d1 - d0).norm().item() <= 0.05 * d0.norm().item() + 1e-6, (n, (d1 - d0).norm().item(),
                                                                           d0.norm().item())


def test_gcn_backward_inside_grads_launch_matches_own_launch(cuda_device, cml_windows, monkeypatch):
    """The fused GCN backward run as extra workgroups of the batched LSTM weight-gradient launch
    (GNNQC_GCN_DEFER=1, the training default) == its own launch: every parameter gradient of a full
    CML loss backward (float atomics: equal up to summation order)."""
    from gnnqc.data.store import CursorIds
    from gnnqc.ops import lstm as L
    from gnnqc.ops.lstm import direct_grad_accumulation
    _, st, model = _setup(cuda_device, cml_windows)
    ids = _ids(st, 128, cuda_device)
    assert model.store_fused_ok(st)
    deferred = []
    real = L.defer_to_grads_launch

    def spy(lists):
        ok = real(lists)
        deferred.append(ok)
        return ok

    monkeypatch.setattr(L, "defer_to_grads_launch", spy)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("GNNQC_GCN_DEFER", flag)
        for p in model.parameters():
            p.grad = torch.zeros_like(p)
        with direct_grad_accumulation(True):
            loss = model.fused_store_loss(st, ids, 1.0, 5.0, None, None)[0]
            loss.backward()
        torch.cuda.synchronize()
        out[flag] = {n: p.grad.clone() for n, p in model.named_parameters()}
    assert deferred == [True, False], deferred
    for n in out["0"]:
        a, r = out["1"][n], out["0"][n]
        # (float atomics: the GCN parameter gradients are sums with strong cancellation - bn_gamma's
        # norm is ~1e-4 - so their run-to-run ordering noise reaches ~3e-3 of the norm; a wrong or
        # missing contribution is an O(1) relative error)
        assert (a - r).norm().item() <= 1e-2 * (r.norm().item() + 1e-6), (n, (a - r).norm().item())


def test_adam_flagged_matches_guarded_and_honours_flags(cuda_device):
    """adam_flagged (decision from producer flags, no grid-wide scan) == adam_guarded on finite
    gradients; a raised producer flag, a chain timeout or a NaN in g[0] skips the whole step (g
    cleared, flags re-armed); an unflagged overflow leaves only that element untouched."""
    from gnnqc.ops.lstm import chain_ctl
    from gnnqc.ops.optim import FlatAdam
    torch.manual_seed(0)
    shapes = [(37, 5), (11,), (64, 64), (3,)]
    mk = lambda: [torch.nn.Parameter(torch.randn(*s, generator=torch.Generator().manual_seed(i)).to(cuda_device))
                  for i, s in enumerate(shapes)]
    a, b = FlatAdam(mk(), 1e-2), FlatAdam(mk(), 1e-2)
    b.flagged_producers = True
    ctl = chain_ctl(cuda_device)
    for _ in range(3):
        g = torch.randn_like(a.flat_g)
        a.flat_g.copy_(g)
        b.flat_g.copy_(g)
        a.step(0.5)
        b.step(0.5)
    torch.cuda.synchronize()
    assert torch.equal(a.flat_p, b.flat_p) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
    assert torch.count_nonzero(b.flat_g) == 0 and b.step_t.item() == 3
    for how in ("flag", "timeout", "g0"):
        before = b.flat_p.clone()
        skipped = b.skipped_steps
        rej = int(ctl[3].item())
        b.flat_g.copy_(torch.randn_like(b.flat_g))
        if how == "flag":
            ctl[7] = 1
        elif how == "timeout":
            ctl[2] = 1
        else:
            b.flat_g[0] = float("nan")
        b.step(1.0)
        torch.cuda.synchronize()
        assert torch.equal(b.flat_p, before), how
        assert b.skipped_steps == skipped + 1 and b.step_t.item() == 3, how
        assert torch.count_nonzero(b.flat_g) == 0, how
        assert int(ctl[2].item()) == 0 and int(ctl[7].item()) == 0, how
        assert int(ctl[3].item()) == rej + (1 if how == "timeout" else 0), how
    before = b.flat_p.clone()
    g = torch.randn_like(b.flat_g)
    g[5] = float("inf")
    b.flat_g.copy_(g)
    b.step(1.0)
    torch.cuda.synchronize()
    assert b.flat_p[5] == before[5] and int(b.guard_state[5].item()) == 1
    assert torch.count_nonzero(b.flat_p != before) == b.flat_p.numel() - 1

def test_deferred_forward_flushed_matches_own_launch(cuda_device, cml_windows, monkeypatch):
    """gcn_fused_fwd(defer): the producer body (gcn_fused.h gcn_prod_body), here run on its own by
    gcn_prod_flush, writes the same time-major input, labels, ids and running statistics as the
    forward kernel (the batch moments are summed in another fixed order: equal to rounding)."""
    from gnnqc.ops.gcn import gcn_pool_from_store
    from gnnqc.utils.native import hip_ops
    monkeypatch.setenv("GNNQC_GCN_PROD", "1")
    _, st, model = _setup(cuda_device, cml_windows)
    g = model.gcn_layer
    ids = _ids(st, 100, cuda_device, pad=5)
    rm0, rv0 = g.bn_moving_mean.clone(), g.bn_moving_variance.clone()
    out = {}
    for defer in (False, True):
        with torch.no_grad():
            g.bn_moving_mean.copy_(rm0)
            g.bn_moving_variance.copy_(rv0)
        h, M, y, ym, wid = gcn_pool_from_store(st, ids, g, True, "mean", defer=defer)
        assert bool(hip_ops().gcn_prod_flush(h)) == defer
        assert not hip_ops().gcn_prod_flush(h)
        torch.cuda.synchronize()
        out[defer] = (h.detach().clone(), y.clone(), ym.clone(), wid.clone(), g.bn_moving_mean.clone(),
                      g.bn_moving_variance.clone())
    a, r = out[True], out[False]
    torch.testing.assert_close(a[0], r[0], atol=2e-5, rtol=2e-5)
    torch.testing.assert_close(a[1], r[1])
    torch.testing.assert_close(a[2], r[2])
    assert torch.equal(a[3], r[3])
    torch.testing.assert_close(a[4], r[4], atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(a[5], r[5], atol=1e-6, rtol=1e-5)


def test_gcn_producers_in_chain_forward_match_own_launch(cuda_device, cml_windows, monkeypatch):
    """The CML loss with the GCN forward run as producer workgroups of the chain forward launch (its
    first stage streams their granules, the head waits for their labels; GNNQC_GCN_PROD=1,
    opt-in) == the GCN forward's own launch: loss, logits and every parameter gradient."""
    from gnnqc.ops.lstm import direct_grad_accumulation
    from gnnqc.utils.native import hip_ops
    _, st, model = _setup(cuda_device, cml_windows)
    ids = _ids(st, 128, cuda_device, pad=2)
    assert model.store_fused_ok(st)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("GNNQC_GCN_PROD", flag)
        m = copy.deepcopy(model)
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
        with direct_grad_accumulation(True):
            loss, logits = m.fused_store_loss(st, ids, 1.0, 5.0, None, None)
            assert not hip_ops().gcn_prod_flush(logits)      # (the chain launch took the job)
            loss.backward()
        torch.cuda.synchronize()
        out[flag] = (float(loss), logits.clone(), {n: p.grad.clone() for n, p in m.named_parameters()},
                     m.gcn_layer.bn_moving_mean.clone())
    a, r = out["1"], out["0"]
    assert abs(a[0] - r[0]) <= 1e-5 * abs(r[0]) + 1e-6, (a[0], r[0])
    torch.testing.assert_close(a[1], r[1], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(a[3], r[3], atol=1e-6, rtol=1e-5)
    for n in r[2]:
        x, y = a[2][n], r[2][n]
        assert (x - y).norm().item() <= 1e-2 * (y.norm().item() + 1e-6), (n, (x - y).norm().item())
