"""ops._grad.step_stream: a no-op off the GPU / when not requested; on a GPU the training loop runs
on a high-priority stream joined back into the caller's stream (GPU test)."""
import pytest
import torch

from determined_clone_amd.ops import _grad


def test_step_stream_noop_on_cpu(monkeypatch):
    monkeypatch.setattr(_grad, "STEP_PRIORITY", "high")
    with _grad.step_stream(torch.device("cpu")) as s:
        assert s is None
    monkeypatch.setattr(_grad, "STEP_PRIORITY", "normal")
    with _grad.step_stream() as s:
        assert s is None


@pytest.mark.gpu
def test_step_stream_high_priority_gpu(monkeypatch):
    monkeypatch.setattr(_grad, "STEP_PRIORITY", "high")
    x = torch.randn(1 << 20, device="cuda")
    prev = torch.cuda.current_stream()
    with _grad.step_stream(torch.device("cuda")) as s:
        assert s is not None and torch.cuda.current_stream() == s
        assert s.priority == torch.cuda.Stream.priority_range()[1]
        y = x * 2  # ordered after x's creation on the previous stream
    assert torch.cuda.current_stream() == prev
    torch.testing.assert_close(y, x * 2)  # the caller's stream waited for the step stream
