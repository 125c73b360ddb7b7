"""Async torch.distributed collectives that complete only when waited for.

gloo runs host collectives inside the call, so a code path that reads a collective's output
before waiting on it -- or never waits -- still passes on CPU, while on RCCL (where
``async_op=True`` really returns before the data moved) it would read stale data. Tests patch the
collectives with :func:`install` so such bugs show on gloo too."""
import torch


class LazyWork:
    def __init__(self, fn, args, kwargs):
        self.fn, self.args, self.kwargs, self.done = fn, args, kwargs, False

    def wait(self, *_a, **_k):
        if not self.done:
            self.fn(*self.args, **self.kwargs)
            self.done = True
        return True

    def is_completed(self):
        return self.done


def install(names=("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor")):
    """Make every ``async_op=True`` call of the named collectives lazy (call inside the worker)."""
    dist = torch.distributed
    for name in names:
        real = getattr(dist, name)

        def lazy(*a, __real=real, async_op=False, **k):
            if not async_op:
                return __real(*a, **k)
            return LazyWork(__real, a, k)
        setattr(dist, name, lazy)
