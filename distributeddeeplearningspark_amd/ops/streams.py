"""Weight-gradient side stream: parameter-gradient GEMMs run beside the backward critical path.

In a convolution's backward only the data-gradient feeds the next (earlier) layer; the
weight-gradient GEMM feeds nothing but the optimizer and the data-parallel all-reduce.  On one
in-order stream the two alternate with the HBM-bound BatchNorm backward sweeps, so the chip runs
an MFMA-bound GEMM, then a bandwidth-bound sweep, then a GEMM...  Issuing every weight gradient on
a second HIP stream (ordered after the data it reads by a stream wait, never by a host sync) lets
the hardware co-schedule the weight-gradient workgroups with the sweeps and data-gradients of the
following layers.

Protocol:
  * ``with on_grad_stream(device, *tensors):`` — launches inside run on the side stream, after
    everything already issued on the current stream; the listed tensors (allocated on the current
    stream) are recorded on the side stream so the caching allocator keeps them alive;
  * ``join(device)`` — the current stream waits for the side stream (end of backward: before the
    optimizer reads the gradient arena).  ``Model.backward_unit`` and the data-parallel engine call it;
  * collectives of gradient buckets are launched with :func:`on_grad_stream` too, so RCCL orders
    them after the side-stream weight gradients AND the main-stream BatchNorm parameter gradients.

Where it pays is measured per model (interleaved A/B on one box,
``profiles/r3/ab_wgrad_stream.jsonl``): BERT-base +2.5-2.8 % tokens/s (the wgrad GEMMs overlap the
attention / LayerNorm backward); ResNet-50 unchanged (every bottleneck kernel already fills the chip,
so the side stream's workgroups only take slots the main stream frees); VGG-16 slower (its step is
host-bound and the per-layer stream waits add host work).  So the call sites pass ``default``:
transformer weight gradients use the side stream, convolution / Dense ones do not, and
``DDL_WGRAD_STREAM=1`` / ``0`` forces it on / off everywhere.  HIP-graph capture follows the same
fork / join through events, so a captured step keeps the overlap.
"""
from __future__ import annotations

from contextlib import contextmanager

import torch

_STREAMS: dict = {}
_PENDING: dict = {}


def enabled(default: bool = True) -> bool:
    from . import scope as _scope

    if _scope.tag():  # replica-group steps run on their own streams: no shared side stream
        return False
    return default


def _key(device) -> int:
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


def grad_stream(device, default: bool = True):
    """The side stream of ``device`` (None on the CPU or when disabled)."""
    d = torch.device(device)
    if d.type != "cuda" or not enabled(default):
        return None
    k = _key(d)
    s = _STREAMS.get(k)
    if s is None:
        s = _STREAMS[k] = torch.cuda.Stream(torch.device("cuda", k))
    return s


@contextmanager
def on_grad_stream(device, *tensors, default: bool = True):
    s = grad_stream(device, default)
    if s is None:
        yield None
        return
    k = _key(device)
    cur = torch.cuda.current_stream(torch.device("cuda", k))
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        yield s
    for t in tensors:
        if t is not None and t.is_cuda:
            t.record_stream(s)
    _PENDING[k] = True


def join(device):
    """Current stream waits for the side-stream work issued so far (no host sync)."""
    d = torch.device(device)
    if d.type != "cuda":
        return
    k = _key(d)
    if not _PENDING.get(k):
        return
    s = _STREAMS.get(k)
    if s is not None:
        torch.cuda.current_stream(torch.device("cuda", k)).wait_stream(s)
    _PENDING[k] = False
