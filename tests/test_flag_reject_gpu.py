"""Whole-step rejection by the flag-driven Adam (adam.hip adam_flagged): every HIP kernel that writes
weight gradients raises the non-finite flag (chain control word 7), so a NaN that reaches ONE
producer's sums rejects the entire step (no parameter changes, one skipped step) instead of the
element-wise skip of unflagged values. A NaN is injected into one saved activation between the
forward and the backward (``torch.autograd.graph.saved_tensors_hooks``): it reaches only the weight
gradients computed from it, through the producer path the switches select."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (switches, predicate on a saved fp32 tensor to poison)
H32 = lambda t: t.dim() == 3 and t.shape[-1] == 32 and t.shape[0] > 8          # noqa: E731  (layer 2/3 h)
FEAT = lambda t: t.dim() == 2 and t.shape[-1] == 128                            # noqa: E731  (head features)
CASES = {
    "chain_multi_reduce": ({}, H32),                                          # lstm_grads_multi reductions
    "per_layer_pipe": ({"GNNQC_CHAIN_BWD": "0"}, H32),                        # pipe / flush reductions
    "per_layer_no_defer": ({"GNNQC_CHAIN_BWD": "0", "GNNQC_DEFER_REDUCE": "0", "pipe": False}, H32),
    "head_hip": ({"GNNQC_HEAD_CHAIN": "0"}, FEAT),                            # head.hip backward
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_nan_in_one_producer_rejects_whole_step(case, cuda_device, cml_windows, monkeypatch):
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    env, pred = CASES[case]
    import gnnqc.ops.lstm as L
    for k, v in env.items():
        if k == "pipe":
            monkeypatch.setattr(L._Pipe, "enabled", v)       # per-layer fused backward + lstm_grads reduce
        else:
            monkeypatch.setenv(k, v)
    pc, ws = cml_windows
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    torch.manual_seed(0)
    model = GCNClassifier(C.default("model_cml"), pc).to(cuda_device)
    opt = make_optimizer("adam", model.parameters(), 1e-3)
    tr = Trainer(model, st, opt, {0: 1.0, 1: 5.0}, use_graph=False, batch_size=32)
    assert tr._flag_base, "the CML store-fused step takes the flag-driven update"
    ids = torch.arange(32, device=cuda_device)
    tr.train_step(ids)                                      # a clean step updates
    torch.cuda.synchronize()
    assert opt.skipped_steps == 0 and opt.flagged_producers
    hit = []

    def pack(t):
        if not hit and t.dtype == torch.float32 and t.is_cuda and pred(t):
            t = t.clone()
            t.view(-1)[t.numel() // 2] = float("nan")
            hit.append(tuple(t.shape))
        return t

    before = opt.flat_p.clone()
    with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
        tr.train_step(ids)
    torch.cuda.synchronize()
    assert hit, "no saved tensor matched the injection predicate"
    assert opt.flagged_producers, "the step must still take the flag-driven update"
    assert opt.skipped_steps == 1, f"{case}: the poisoned step must be rejected as a whole"
    assert torch.equal(opt.flat_p, before), f"{case}: a rejected step changes no parameter"
    assert int(opt.guard_state[5].item()) == 0, "no element-wise partial update"
    assert float(opt.flat_g.abs().max()) == 0.0, "the gradient buffer is cleared either way"
    tr.train_step(ids)                                      # and training goes on
    torch.cuda.synchronize()
    assert opt.skipped_steps == 1 and not torch.equal(opt.flat_p, before)
