"""Plumbing of the deferred weight-gradient reductions (no GPU needed: the switch and the flush are
tensor-less catch-all ops of the native library). The GPU numerics are in
tests/test_deferred_reduce_gpu.py."""
import os

import pytest

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gnnqc", "_lib", "libgnnqc_hip.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="HIP extension not built")
def test_deferred_reduce_switch_scoped_to_direct_accumulation():
    import torch
    from gnnqc.ops import lstm as L
    torch.ops.load_library(LIB)
    ops = torch.ops.gnnqc
    assert ops.lstm_defer_reduce(False) is False
    # outside direct accumulation nothing is deferred (autograd would read the buffers at once)
    with L._deferred_reduce(True):
        assert ops.lstm_defer_reduce(False) is False
    assert not L._Deferred.pending
    with L.direct_grad_accumulation(True):
        with L._deferred_reduce(False):               # a non-direct sink: not deferred
            assert ops.lstm_defer_reduce(False) is False
        with L._deferred_reduce(True):
            assert ops.lstm_defer_reduce(True) is True     # on inside; restore it for the exit
        assert ops.lstm_defer_reduce(False) is False       # restored after the call
        assert L._Deferred.pending
    # the context's exit flushed the (empty) queue and cleared the pending mark
    assert not L._Deferred.pending
    assert ops.lstm_reduce_flush() == 0


def test_deferred_reduce_kill_switch(monkeypatch):
    from gnnqc.ops import lstm as L
    monkeypatch.setenv("GNNQC_DEFER_REDUCE", "0")
    with L.direct_grad_accumulation(True):
        with L._deferred_reduce(True):
            pass
        assert not L._Deferred.pending
