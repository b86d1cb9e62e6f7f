"""Deferred weight-gradient reductions (``lstm_defer_reduce`` / ``lstm_reduce_flush``): under direct
gradient accumulation the per-layer backward of a wide TimeLayer (more sequences than the
pipelined backward takes, as SoilNet's 6,688 node sequences) queues every layer's split
reduction and runs them in one launch at the end of the backward. The gradients must equal those
autograd receives from the per-layer reductions (same split records; the per-layer reduce sums
the splits in groups first, so equality is to fp32 rounding, not bitwise)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_deferred_reduce_matches_per_layer(cuda_device, monkeypatch):
    from gnnqc.models.timelayer import TimeLayer
    from gnnqc.ops import lstm as L
    monkeypatch.setenv("GNNQC_CHAIN", "0")          # the per-layer kernels, as on the SoilNet step
    torch.manual_seed(0)
    tl = TimeLayer(20, 16, 2).to(cuda_device)
    x = torch.randn(L.PIPE_MAX_SEQ + 160, 45, 20, device=cuda_device)
    w = torch.randn(tl.out_features, device=cuda_device)

    def run(direct):
        for p in tl.parameters():
            p.grad = torch.zeros_like(p) if direct else None
        out = tl(x)
        loss = (out * w).sum()
        with L.direct_grad_accumulation(direct):
            loss.backward()
            if direct:
                assert L._Deferred.pending, "no split reduction was deferred"
        assert not L._Deferred.pending
        torch.cuda.synchronize()
        return {n: p.grad.detach().clone() for n, p in tl.named_parameters()}

    ref = run(False)
    got = run(True)
    for n in ref:
        scale = ref[n].abs().max().item() + 1e-12
        err = (got[n] - ref[n]).abs().max().item()
        assert err <= 1e-5 * scale, (n, err, scale)
