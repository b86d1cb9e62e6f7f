"""CML GCN benched path (GCN kernel -> headed LSTM chain -> head + BCE in the chain) on the GPU:
whole-model numerics against a float64 eager oracle, against the separate-kernel path, and the
chain's fail-loudly guarantees (a timed-out step is rejected, never applied)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda_device, cml_windows, B=128, seed=0):
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    pc, ws = cml_windows
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    torch.manual_seed(seed)
    mc = C.default("model_cml")
    model = GCNClassifier(mc, pc).to(cuda_device)
    with torch.no_grad():                  # non-trivial head biases / BN parameters
        for p in (model.dense.bias, model.dense2.bias, model.dense_out.bias):
            p.normal_(0, 0.1)
    n = min(B, st.n_windows)
    b = st.gather(torch.arange(n, device=cuda_device))
    return pc, mc, st, model, b


def _grads(model, fn):
    from gnnqc.ops.lstm import direct_grad_accumulation
    for p in model.parameters():
        p.grad = torch.zeros_like(p)
    with direct_grad_accumulation(True):
        loss, z = fn()
        loss.backward(torch.ones((), device=loss.device))
    torch.cuda.synchronize()
    return loss.detach(), z.detach(), {n: p.grad.clone() for n, p in model.named_parameters()}


def test_headed_chain_is_the_default_cml_path(cuda_device, cml_windows):
    _, _, _, model, b = _setup(cuda_device, cml_windows)
    inputs = b.model_inputs("cml")
    x_tm_ok = model._cml_time_major(inputs)
    assert x_tm_ok
    from gnnqc.ops.gcn import gcn_pool
    g = model.gcn_layer
    x, anom, adj, mask, anom_pos = inputs[:5]
    h, M = gcn_pool(x, adj, mask, anom, anom_pos, g.kernel, g.bias, g.bn_gamma, g.bn_beta, g.prelu_alpha, g.bn_moving_mean,
                    g.bn_moving_variance, False, g.aggregate, "mean", g.momentum, g.eps, g.dropout, time_major=True)
    assert model.time_layer.head_chain_ok(h)


def test_headed_chain_matches_separate_kernels(cuda_device, cml_windows, monkeypatch):
    """One launch for TimeLayer + head + loss (fwd) and one for their backward == the chain of six
    layers + separate time4 / head kernels: loss, logits and every parameter gradient."""
    _, _, _, model, b = _setup(cuda_device, cml_windows)
    inputs = b.model_inputs("cml")

    def run(head_chain):
        monkeypatch.setenv("GNNQC_HEAD_CHAIN", "1" if head_chain else "0")
        return _grads(model, lambda: model.fused_loss(inputs, b.y, b.y_mask, 1.0, 5.0))

    l1, z1, g1 = run(True)
    l0, z0, g0 = run(False)
    torch.testing.assert_close(z1, z0, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(l1, l0, atol=1e-4, rtol=1e-3)
    for n in g0:
        err = (g1[n] - g0[n]).norm().item()
        assert err <= 5e-3 * (g0[n].norm().item() + 1e-6), (n, err, g0[n].norm().item())


def test_cml_default_path_matches_kernel_rounding_reference(cuda_device, cml_windows):
    """The benched CML step (fused GCN, headed chain, bf16 MFMA recurrences) against the same
    model in float64 on the CPU with the LSTM rounded where the kernels round (bf16 MFMA operands,
    bf16 saved gates and dz: gnnqc/ops/lstm_ref.py): logits, loss and every parameter gradient
    within 5e-3 - rounding explains the rest, so a logic error at the percent level fails."""
    from gnnqc.data.store import DeviceStore
    from gnnqc.ops.lstm_ref import kernel_rounding
    from gnnqc.train.loss import weighted_bce_with_logits
    pc, _, _, model, b = _setup(cuda_device, cml_windows, B=96)
    inputs = b.model_inputs("cml")
    assert model.time_layer.head_chain_ok is not None
    loss, z, g = _grads(model, lambda: model.fused_loss(inputs, b.y, b.y_mask, 1.0, 5.0))

    ref = __import__("copy").deepcopy(model).cpu().double()
    for p in ref.parameters():
        p.grad = None
    _, ws = cml_windows
    st = DeviceStore(ws, "rolling_median", pc.graph, device="cpu")
    bc = st.gather(torch.arange(b.y.shape[0]))
    ri = [t.double() if torch.is_tensor(t) and t.is_floating_point() else t for t in bc.model_inputs("cml")]
    with kernel_rounding():
        zr = ref.logits(ri)
        lr = weighted_bce_with_logits(zr, bc.y.double(), bc.y_mask.double(), 1.0, 5.0)
        lr.backward()
    assert abs(loss.item() - lr.item()) <= 2e-3 * abs(lr.item()) + 1e-5, (loss.item(), lr.item())
    zerr = (z.cpu().double() - zr.detach()).abs().max().item()
    assert zerr <= 5e-3 * zr.detach().abs().max().item() + 1e-6, (zerr, zr.abs().max().item())
    worst = {}
    for n, p in ref.named_parameters():
        if p.grad is None:
            continue
        err = (g[n].cpu().double() - p.grad).norm().item()
        scale = p.grad.norm().item()
        worst[n] = err / (scale + 1e-12)
        assert err <= 5e-3 * scale + 1e-6, (n, err, scale)
    print("max relative gradient error", max(worst.values()), max(worst, key=worst.get))


def test_chain_timeout_rejects_the_step(cuda_device, cml_windows):
    """A consumer spin that times out (forced with the debug spin limit) makes the guard skip the
    step on the device (parameters untouched) and the epoch end raise ChainTimeoutError."""
    from gnnqc.data.store import DeviceLoader
    from gnnqc.ops.lstm import ChainTimeoutError, chain_ctl, check_chain
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    _, _, st, model, _ = _setup(cuda_device, cml_windows)
    opt = make_optimizer("adam", model.parameters(), 1e-3)
    tr = Trainer(model, st, opt, {0: 1.0, 1: 5.0}, use_graph=False, batch_size=64)
    loader = DeviceLoader(st, list(range(st.n_windows)), 64, shuffle=False)
    row = next(iter(loader.batch_ids()))
    ctl = chain_ctl(cuda_device)
    rejected0 = check_chain(cuda_device)
    tr.train_step(row)                                  # a normal step first
    torch.cuda.synchronize()
    before = opt.flat_p.clone()
    skipped0 = opt.skipped_steps
    try:
        ctl[6] = 1                                      # spin limit 1: consumers give up at once
        tr.train_step(row)
        torch.cuda.synchronize()
    finally:
        ctl[6] = 0
    assert opt.skipped_steps == skipped0 + 1
    assert torch.equal(opt.flat_p, before), "a timed-out step must not change the parameters"
    with pytest.raises(ChainTimeoutError):
        check_chain(cuda_device, rejected0)
    tr.train_step(row)                                  # and training continues normally
    torch.cuda.synchronize()
    assert opt.skipped_steps == skipped0 + 1
    assert not torch.equal(opt.flat_p, before)


def test_headed_chain_eval_metrics_match(cuda_device, cml_windows, monkeypatch):
    """Evaluation through the headed chain (no-grad, TRAIN=false kernels) == separate kernels."""
    from gnnqc.data.store import DeviceLoader
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    _, _, st, model, _ = _setup(cuda_device, cml_windows)
    opt = make_optimizer("adam", model.parameters(), 1e-3)
    tr = Trainer(model, st, opt, {0: 1.0, 1: 5.0}, use_graph=False, batch_size=64)
    loader = DeviceLoader(st, list(range(st.n_windows)), 64, shuffle=False)
    monkeypatch.setenv("GNNQC_HEAD_CHAIN", "1")
    a = tr.evaluate(loader)
    monkeypatch.setenv("GNNQC_HEAD_CHAIN", "0")
    r = tr.evaluate(loader)
    for k in r:
        assert abs(a[k] - r[k]) <= 2e-3 * abs(r[k]) + 2e-3, (k, a[k], r[k])


@pytest.mark.parametrize("B", [128, 40])
def test_t4_chain_stage_matches_separate_launch(cuda_device, cml_windows, monkeypatch, B):
    """time4 + head + loss as stages of the chain launches (lstm_chain_head_fwd: the stage pools the
    last chain stage's granules itself; lstm_chain_head_bwd: the head backward + time4's reverse
    recurrence publish dx granules to the top chain stage; two cells per lane) == the separate
    time4_head_fwd / _bwd launches: loss and logits (same bf16 operands and accumulation order per
    cell), every gradient (the backward's partial sums are split differently), no spin timed out."""
    from gnnqc.utils.native import hip_ops
    _, _, _, model, b = _setup(cuda_device, cml_windows, B=B)
    inputs = b.model_inputs("cml")

    def run(on):
        monkeypatch.setenv("GNNQC_T4_CHAIN", "1" if on else "0")
        return _grads(model, lambda: model.fused_loss(inputs, b.y, b.y_mask, 1.0, 5.0))

    l0, z0, g0 = run(False)
    l1, z1, g1 = run(True)
    st = hip_ops().lstm_chain_status(z1).cpu()
    assert int(st[2]) == 0, "a consumer spin timed out"
    torch.testing.assert_close(z1, z0, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(l1, l0, atol=1e-6, rtol=1e-5)
    for n in g0:
        err = (g1[n] - g0[n]).norm().item()
        assert err <= 1e-3 * (g0[n].norm().item() + 1e-6), (n, err, g0[n].norm().item())
    with torch.no_grad():                      # evaluation (TRAIN = false kernels)
        monkeypatch.setenv("GNNQC_T4_CHAIN", "1")
        le1, ze1 = model.fused_loss(inputs, b.y, b.y_mask, 1.0, 5.0)
        monkeypatch.setenv("GNNQC_T4_CHAIN", "0")
        le0, ze0 = model.fused_loss(inputs, b.y, b.y_mask, 1.0, 5.0)
    torch.testing.assert_close(ze1, ze0, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(le1, le0, atol=1e-6, rtol=1e-5)


def test_head_backward_precomputed_by_forward_launch(cuda_device, cml_windows, monkeypatch):
    """The head backward run by the chain FORWARD launch (dL/dloss = 1, the backward scales dh_{T-1}
    and the reduced head-gradient records by the real dL/dloss) == the head backward run at the start
    of the backward launch: same code on the same values, so every gradient matches tightly; an
    upstream gradient of 2.5 scales every gradient by 2.5 on the precomputed path."""
    from gnnqc.ops.lstm import direct_grad_accumulation
    from gnnqc.utils.native import hip_ops
    _, _, _, model, b = _setup(cuda_device, cml_windows)
    inputs = b.model_inputs("cml")
    monkeypatch.setenv("GNNQC_T4_CHAIN", "1")

    def run(pre, scale=1.0):
        monkeypatch.setenv("GNNQC_HEAD_BWD_IN_FWD", "1" if pre else "0")
        for p in model.parameters():
            p.grad = torch.zeros_like(p)
        with direct_grad_accumulation(True):
            loss, _ = model.fused_loss(inputs, b.y, b.y_mask, 1.0, 5.0)
            loss.backward(torch.full((), scale, device=loss.device))
        torch.cuda.synchronize()
        return {n: p.grad.clone() for n, p in model.named_parameters()}

    g0 = run(False)
    g1 = run(True)
    assert int(hip_ops().lstm_chain_status(b.y)[2].item()) == 0
    for n in g0:
        torch.testing.assert_close(g1[n], g0[n], atol=1e-7, rtol=1e-5, msg=n)
    # dL/dloss = 2.5: the scaled dh_{T-1} / records vs the head backward with gl = 2.5 (fp32 products
    # in a different order, then the same bf16 dz roundings: near-identical, compared by norm)
    h0 = run(False, 2.5)
    h1 = run(True, 2.5)
    for n in h0:
        err = (h1[n] - h0[n]).norm().item()
        assert err <= 1e-4 * (h0[n].norm().item() + 1e-9), (n, err, h0[n].norm().item())
        assert abs(h0[n].norm().item() - 2.5 * g0[n].norm().item()) <= 1e-2 * h0[n].norm().item() + 1e-9, n
