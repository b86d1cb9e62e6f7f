"""Every opt-in backward layout of the LSTM TimeLayer (kept for A/B measurements, see
profiles/README.md) against the default layout on the same weights and input: outputs and every
gradient. SoilNet-like stack (20 input channels, 16/16/32/32/64/64/128 units with pooling)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

LAYOUTS = [
    # (switches of the variant, switches of both runs)
    ({"GNNQC_TM_RECDX": "0"}, {"GNNQC_CHAIN": "0"}),          # dx from weight-gradient slabs + sum
]


@pytest.mark.parametrize("variant,base", LAYOUTS, ids=[next(iter(v)) + "=" + next(iter(v.values())) for v, _ in LAYOUTS])
def test_timelayer_backward_layouts_agree(cuda_device, monkeypatch, variant, base):
    from gnnqc.models.timelayer import TimeLayer
    from gnnqc.ops.lstm import direct_grad_accumulation
    torch.manual_seed(1)
    tl = TimeLayer(20, 16, 2, "lstm", pool_size=3).to(cuda_device)
    x = torch.randn(160, 120, 20, device=cuda_device)
    for k, v in base.items():
        monkeypatch.setenv(k, v)

    def run(env):
        for k in variant:
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        xi = x.clone().requires_grad_(True)
        for p in tl.parameters():
            p.grad = None
        with direct_grad_accumulation(True):
            out = tl(xi)
            (out * torch.linspace(-1, 1, out.shape[-1], device=cuda_device)).pow(2).sum().backward()
        torch.cuda.synchronize()
        return out.detach(), [xi.grad.clone()] + [p.grad.clone() for p in tl.parameters()]

    o0, g0 = run({})
    o1, g1 = run(variant)
    torch.testing.assert_close(o1, o0, atol=2e-3, rtol=1e-2)
    assert len(g0) == len(g1)
    for a, b in zip(g1, g0):
        assert torch.isfinite(a).all()
        assert (a - b).norm().item() <= 2e-2 * (b.norm().item() + 1e-6)
