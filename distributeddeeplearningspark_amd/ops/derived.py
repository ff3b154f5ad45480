"""Weight-derived filters of a training step, computed in ONE launch.

The backward pass needs re-laid-out copies of many weights: the flipped filter of every stride-1 conv
data-gradient run as a forward conv (``conv.flip_filter``), the per-class filters of strided data-gradients
(``conv.class_filter``) and the transposed weights of the large Linear / 1x1 data-gradients
(``gemm.transpose``).  Computed one by one they were 44 launches per ResNet-50 step (12 per VGG-16 step,
48 per BERT-base step), each a few microseconds of a mostly idle GPU.  The weights do not change between the
forward pass and the optimizer, so here every such copy of the model being trained is computed by a single
``taps_batch`` launch (csrc/kernels/layer_ops.hip) at the first request of the step, from a job table built
from the previous step's requests; later requests of the step return the already-computed copies.

Only copies of the training model's own arena storage (``ParamArena.compute``) are batched: their addresses
are stable across steps, so the device job table stays valid (and a captured hipGraph replays the launch).
Anything else, or a model outside ``begin_step``, takes the one-launch-per-copy path.
"""
from __future__ import annotations

import weakref

import torch

from ._native import C


class _Registry:
    def __init__(self, storage_ptr: int):
        self.storage_ptr = storage_ptr
        self.jobs: list = []  # (src, dst, taps)
        self.index: dict = {}
        self.table = None  # (device table, njobs, blocks) of self.jobs
        self.ran = -1  # step stamp of the last batched launch

    def launch(self):
        if self.table is None or self.table[1] != len(self.jobs):
            t, blocks = C().taps_batch_table([j[0] for j in self.jobs], [j[1] for j in self.jobs],
                                             [list(j[2]) for j in self.jobs])
            self.table = (t.to(self.jobs[0][0].device), len(self.jobs), int(blocks))
        C().taps_batch(*self.table)


ENABLED = True  # tests switch the batching off to compare with the one-launch-per-copy path
_REGS = weakref.WeakKeyDictionary()  # arena -> registry (dies with its model)
_CUR: list = [None]
_STEP = [0]


def begin_step(model) -> None:
    """Called by Model.backward_step: the arena's weights are fixed until the optimizer runs."""
    a = getattr(model, "arena", None)
    if not ENABLED or a is None or not a.compute.is_cuda or a.compute.dtype != torch.bfloat16:
        _CUR[0] = None
        return
    ptr = a.compute.untyped_storage().data_ptr()
    reg = _REGS.get(a)
    if reg is None or reg.storage_ptr != ptr:  # new arena or a re-homed one (ParamArena.rebind)
        reg = _REGS[a] = _Registry(ptr)
    _CUR[0] = reg
    _STEP[0] += 1


def end_step() -> None:
    _CUR[0] = None


def taps_transpose(w: torch.Tensor, taps, out_shape) -> torch.Tensor:
    """out[ci][t][co] = w[co][taps[t]][ci] (``w`` [Co][KH][KW][Ci] or [N][K] bf16, contiguous)."""
    reg = _CUR[0]
    taps = tuple(int(t) for t in taps)
    if reg is None or not w.is_contiguous() or w.untyped_storage().data_ptr() != reg.storage_ptr:
        out = torch.empty(out_shape, dtype=w.dtype, device=w.device)
        _one(w, out, taps)
        return out
    key = (w.data_ptr(), tuple(w.shape), taps)
    j = reg.index.get(key)
    if j is not None:
        if reg.ran != _STEP[0]:
            stale = reg.table is None or reg.table[1] != len(reg.jobs)
            if stale and torch.cuda.is_current_stream_capturing():
                _one(w, reg.jobs[j][1], taps)  # no table upload inside a capture: this copy alone
                return reg.jobs[j][1]
            reg.launch()  # every registered copy of this step's weights, one launch
            reg.ran = _STEP[0]
        return reg.jobs[j][1]
    out = torch.empty(out_shape, dtype=w.dtype, device=w.device)  # persistent: reused every step
    _one(w, out, taps)
    reg.index[key] = len(reg.jobs)
    reg.jobs.append((w.detach(), out, taps))
    return out


def _one(w, out, taps):
    if w.dim() == 2:
        C().transpose_bf16(w, out)
    else:
        C().filter_taps_transpose(w, out, list(taps))
