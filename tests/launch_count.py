"""Count device launches in a code region: every ATen op that launches work on a CUDA tensor (views and allocations
excluded) plus every native HIP entry point (dxa.ops.native.call).  Used by tests that pin launch budgets."""
import contextlib

import torch
from torch.utils._python_dispatch import TorchDispatchMode

_NO_LAUNCH = {"view", "_unsafe_view", "slice", "select", "as_strided", "expand", "unsqueeze", "squeeze", "permute",
              "t", "transpose", "alias", "detach", "_reshape_alias", "empty", "new_empty", "empty_strided", "set_",
              "resize_", "unbind", "split", "narrow", "lift_fresh", "reshape", "unfold", "is_pinned", "_pin_memory",
              "split_with_sizes", "chunk", "_local_scalar_dense", "empty_like"}


class _Mode(TorchDispatchMode):
    def __init__(self, log):
        super().__init__()
        self.log = log

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__.split(".")[0]
        ts = [a for a in list(args) + list((kwargs or {}).values()) if torch.is_tensor(a)]
        if name not in _NO_LAUNCH and (any(t.is_cuda for t in ts) or (torch.is_tensor(out) and out.is_cuda)):
            self.log.append(func.__name__)
        return out


@contextlib.contextmanager
def count_launches():
    """``with count_launches() as log: ...`` → ``log`` lists the launches (ATen op names / native entry points)."""
    from dxa.ops import native as N
    log = []
    real = N.call

    def call(name, *a):
        log.append(name)
        return real(name, *a)
    N.call = call
    try:
        with _Mode(log):
            yield log
    finally:
        N.call = real
