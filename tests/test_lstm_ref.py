"""The kernel-rounding LSTM reference (gnnqc/ops/lstm_ref.py): without rounding its hand-written
backward is the exact float64 gradient (== autograd through the eager recurrence); with rounding
it differs from float64 by bf16-sized amounts only."""
import pytest
import torch


@pytest.mark.parametrize("H,ret", [(16, True), (64, True), (128, False)])
def test_kernel_lstm_backward_is_exact_without_rounding(H, ret):
    from gnnqc.ops.lstm import lstm_eager
    from gnnqc.ops.lstm_ref import KernelLSTM
    g = torch.Generator().manual_seed(H)
    M, T, D = 5, 9, 7
    x = torch.randn(M, T, D, generator=g, dtype=torch.float64, requires_grad=True)
    W = (torch.randn(D, 4 * H, generator=g, dtype=torch.float64) * 0.3).requires_grad_()
    U = (torch.randn(H, 4 * H, generator=g, dtype=torch.float64) * 0.3).requires_grad_()
    b = (torch.randn(4 * H, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    gout = torch.randn((M, T, H) if ret else (M, H), generator=g, dtype=torch.float64)
    ref = torch.autograd.grad((lstm_eager(x, W, U, b, ret) * gout).sum(), (x, W, U, b))
    out = KernelLSTM.apply(x, W, U, b, ret, False)
    torch.testing.assert_close(out, lstm_eager(x, W, U, b, ret), rtol=1e-12, atol=1e-12)
    got = torch.autograd.grad((out * gout).sum(), (x, W, U, b))
    for a, r in zip(got, ref):
        torch.testing.assert_close(a, r, rtol=1e-10, atol=1e-10)


def test_kernel_rounding_context_switches_the_eager_lstm():
    from gnnqc.ops.lstm import lstm_eager
    from gnnqc.ops.lstm_ref import kernel_rounding
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 6, 4, generator=g, dtype=torch.float64)
    W = torch.randn(4, 64, generator=g, dtype=torch.float64) * 0.3
    U = torch.randn(16, 64, generator=g, dtype=torch.float64) * 0.3
    b = torch.zeros(64, dtype=torch.float64)
    full = lstm_eager(x, W, U, b)
    with kernel_rounding():
        rounded = lstm_eager(x, W, U, b)
    assert not torch.equal(full, rounded)
    assert (full - rounded).abs().max().item() < 3e-2       # bf16-sized differences only
