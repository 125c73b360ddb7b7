"""CPU tests of the side-stream weight-gradient bookkeeping in ``ops/_grad.py`` (the stream
objects are stand-ins: no GPU needed)."""
import types

import torch

from determined_clone_amd.ops import _grad


class _Param:
    is_cuda = True
    device = types.SimpleNamespace(index=0)


def test_main_tail_keeps_the_last_weight_gradients_of_a_pass_on_the_current_stream(monkeypatch):
    """DCA_WGRAD_MAIN_TAIL=N: with no history every weight gradient goes to the side stream; after
    a join the last N calls of the next pass (by the previous pass's count) stay on the current
    stream."""
    monkeypatch.setattr(_grad, "SIDE_STREAM", True)
    monkeypatch.setattr(_grad, "MAIN_TAIL", 2)
    monkeypatch.setattr(_grad, "target", lambda p: object())
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    monkeypatch.setitem(_grad._streams, 0, "side")
    monkeypatch.setattr(_grad, "_calls", 0)
    monkeypatch.setattr(_grad, "_last_total", 0)
    assert [_grad.side_stream_for(_Param()) for _ in range(5)] == ["side"] * 5
    _grad.join()  # end of the step: records the pass length
    assert [_grad.side_stream_for(_Param()) for _ in range(5)] == ["side"] * 3 + [None] * 2
    _grad.join()
    assert _grad._last_total == 5 and _grad._calls == 0


def test_main_tail_off_by_default(monkeypatch):
    monkeypatch.setattr(_grad, "SIDE_STREAM", True)
    monkeypatch.setattr(_grad, "MAIN_TAIL", 0)
    monkeypatch.setattr(_grad, "target", lambda p: object())
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    monkeypatch.setitem(_grad._streams, 0, "side")
    monkeypatch.setattr(_grad, "_calls", 0)
    monkeypatch.setattr(_grad, "_last_total", 3)
    assert [_grad.side_stream_for(_Param()) for _ in range(3)] == ["side"] * 3
