"""Multi-view data-parallel training step: the one exchange on the path.

The reference trains on one GPU, one view per step (train.py:67-125); SURVEY
§8(e) shards views across the GPUs of a node instead: every rank holds a full
replica of the Gaussians, renders and back-propagates its own view through
the MI355X rasterizer, and the parameter gradients -- 59 floats per Gaussian
(means3D 3, SH 48, opacity 1, scales 3, rotations 4) -- are summed across
ranks with ONE RCCL all-reduce over xGMI (``torch.distributed`` backend
"nccl" is RCCL on ROCm).  Densification statistics use per-view
||dL/dmeans2D[:, :2]|| (scene/gaussian_model.py:405-407), so they are summed
(accum, denom) and max-reduced (radii) separately.

Gradients are written into one flat HBM buffer that is all-reduced in
place: no per-tensor launches, no concatenation copy after the backward,
and replicas stay bit-identical because the ring all-reduce hands every rank
the same bits.  The same code runs on ``gloo`` for the CPU tests.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

PARAM_ORDER: Tuple[str, ...] = ("means3D", "shs", "opacities", "scales", "rotations")


class FlatGrads:
    """One contiguous buffer holding the gradients of `params` (views)."""

    def __init__(self, params: Dict[str, torch.Tensor], order: Sequence[str] = PARAM_ORDER):
        self.order = tuple(order)
        numel = sum(params[k].numel() for k in self.order)
        dev = params[self.order[0]].device
        self.flat = torch.zeros(numel, dtype=torch.float32, device=dev)
        self.views: Dict[str, torch.Tensor] = {}
        off = 0
        for k in self.order:
            n = params[k].numel()
            self.views[k] = self.flat[off:off + n].view_as(params[k])
            off += n

    def load(self, grads: Dict[str, torch.Tensor]) -> None:
        for k in self.order:
            self.views[k].copy_(grads[k])

    def attach(self, params: Dict[str, torch.Tensor]) -> None:
        """Make params[k].grad alias the flat buffer, so autograd's first
        accumulation writes straight into it (torch copies into an existing
        .grad of matching layout)."""
        for k in self.order:
            params[k].grad = self.views[k]


def allreduce_(flat: torch.Tensor, group=None, average: bool = False) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        if average:
            flat.div_(dist.get_world_size(group))
    return flat


def densification_stats_allreduce_(grad_norm_accum: torch.Tensor, denom: torch.Tensor, max_radii2D: torch.Tensor,
                                   group=None) -> None:
    """scene/gaussian_model.py:400-407 statistics across views: sums and a max."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(grad_norm_accum, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(denom, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(max_radii2D, op=dist.ReduceOp.MAX, group=group)


def grads_of(params: Dict[str, torch.Tensor], order: Iterable[str] = PARAM_ORDER) -> List[torch.Tensor]:
    return [params[k].grad for k in order]


def flat_numel_per_gaussian(sh_coeffs: int = 16) -> int:
    return 3 + 3 * sh_coeffs + 1 + 3 + 4  # 59 at SH degree 3
