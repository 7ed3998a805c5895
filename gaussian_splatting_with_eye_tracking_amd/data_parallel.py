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

The default exchange ("views") moves less: the per-Gaussian backward
(base/cr/backward.cu:20-396) is linear in the 9 screen-space sums the blend
backward produces, given the view's camera, radius and SH clamp bits.  Each
rank therefore runs only the blend backward of its view and packs a VIEW
RECORD (10 words per Gaussian + the 40-word camera, gsplat_amd.h); one
all-gather hands every rank all N records, and one multi-view kernel forms
the sum over the N views of the parameter gradients (and, for training,
the per-view densification statistics), reading the parameters once.  Per
rank that is (N-1) x 40 B per Gaussian received instead of a ring
all-reduce's 2 (N-1)/N x 236 B -- 6x less at N = 2, 1.5x less at N = 8 --
and every rank computes the same sum in the same view order, so replicas
stay bit-identical.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

PARAM_ORDER: Tuple[str, ...] = ("means3D", "shs", "opacities", "scales", "rotations")
VIEW_ROW = 10    # words per Gaussian in a view record
CAM_WORDS = 40   # camera words closing a view record


def view_record_numel(P: int) -> int:
    return P * VIEW_ROW + CAM_WORDS


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


# ------------------------------------------------------------ view exchange ---
def gather_view_records(record: torch.Tensor, group=None) -> torch.Tensor:
    """All ranks' view records in rank order: record is this rank's [P * 10 +
    40] record or its [v, P * 10 + 40] records (v views per rank); returns
    [world * v, P * 10 + 40] (one RCCL all-gather; on gloo the list form)."""
    recs = record if record.dim() == 2 else record.unsqueeze(0)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return recs
    world = dist.get_world_size(group)
    v, n = recs.shape
    out = torch.empty((world, v * n), dtype=recs.dtype, device=recs.device)
    src = recs.contiguous().view(-1)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, src, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), src, group=group)
    return out.view(world * v, n)


def view_record(settings, radii: torch.Tensor, geom: torch.Tensor, num_rendered: int, binning: torch.Tensor,
                img: torch.Tensor, dL_dpix: torch.Tensor, colors_precomp: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Stage 1: the blend backward of one rendered view -> its view record."""
    from . import _C
    e = torch.empty(0, device=dL_dpix.device) if colors_precomp is None else colors_precomp
    return _C.rasterize_gaussians_backward_view_grads(
        settings.bg, radii, e, settings.viewmatrix, settings.projmatrix, settings.tanfovx, settings.tanfovy,
        settings.campos, dL_dpix, geom, num_rendered, binning, img, settings.debug)


def multiview_param_grads(views: torch.Tensor, means3D: torch.Tensor, shs: torch.Tensor, sh_degree: int,
                          scales: torch.Tensor, rotations: torch.Tensor, scale_modifier: float = 1.0,
                          stats: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None):
    """Stage 2: sum over the gathered views of the parameter gradients:
    (dL_dmeans3D, dL_dshs, dL_dopacities, dL_dscales, dL_drotations).  With
    stats = (xyz_gradient_accum, denom, max_radii2D) the densification
    statistics of every view are accumulated in place (train.py:111-113)."""
    from . import _C
    e = torch.empty(0, device=means3D.device)
    st = stats if stats is not None else (e, e, e)
    return _C.backward_gaussians_multiview(views, means3D, shs if shs is not None else e, int(sh_degree), scales,
                                           rotations, float(scale_modifier), st[0], st[1], st[2])


def exchange_view_grads(settings, fwd, dL_dpix: torch.Tensor, means3D: torch.Tensor, shs: torch.Tensor,
                        scales: torch.Tensor, rotations: torch.Tensor, group=None, stats=None, chunks: int = 4):
    """The data-parallel backward of one step: this rank's view record,
    all-gathered, then the multi-view parameter gradients (identical bits on
    every rank).  fwd = (num_rendered, color, radii, geom, binning, img) as
    returned by _C.rasterize_gaussians.

    With more than one rank the gather is split into `chunks` ranges of
    Gaussians, all issued asynchronously up front: the RCCL stream moves
    chunk c + 1 while the compute stream runs the multi-view backward of
    chunk c (each chunk's work waits only for its own collective), so at
    most one chunk's backward is exposed after the last transfer."""
    num_rendered, _color, radii, geom, binning, img = fwd
    rec = view_record(settings, radii, geom, num_rendered, binning, img, dL_dpix)
    return exchange_view_records(rec, settings, means3D, shs, scales, rotations, group, stats, chunks)


class ViewExchange:
    """The "views" exchange pipelined behind the rendering of a rank's views.

    A rank with v views per step hands each view record to `add` as soon as
    its blend backward has produced it: the record is all-gathered at once
    (asynchronously, on the collective stream), so the transfer of view j
    overlaps the forward + blend backward of views j + 1 ... v - 1 on the
    compute stream.  The last view -- whose transfer has nothing left to hide
    behind -- is gathered in `chunks` Gaussian ranges, each released to the
    multi-view backward as it lands (exchange_view_records' overlap).  The
    gathered records sit in rank-then-view order, so `finish` computes the
    same sums in the same order as exchange_view_records: bit-identical
    results.  Over one rank it just keeps the records."""

    def __init__(self, P: int, views_per_rank: int, device, group=None, chunks: int = 4):
        self.P, self.v, self.group, self.chunks = int(P), int(views_per_rank), group, max(1, int(chunks))
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.nccl = self.world > 1 and dist.get_backend(group) == "nccl"
        self.RL = view_record_numel(self.P)
        self.device = device
        if self.world == 1:
            self.buf = torch.empty((self.v, self.RL), dtype=torch.float32, device=device)
        # every gather lands in its own contiguous [world, n] buffer (one
        # all_gather_into_tensor on RCCL, no flatten copy); the multi-view
        # kernel then reads view (r, j) through a per-view row pointer
        self.full: List[torch.Tensor] = [None] * max(0, self.v - 1)  # views 0 .. v-2: [world, RL], by index
        self.pending: List[object] = []
        self.last: List[Tuple[int, int, torch.Tensor, object]] = []  # (a, b, [world, (b-a)*10], work)
        self.cam_stage = None
        self.cam_work = None

    def _gather(self, src: torch.Tensor):
        src = src.contiguous()
        out = torch.empty((self.world, src.numel()), dtype=src.dtype, device=src.device)
        if self.nccl:
            w = dist.all_gather_into_tensor(out, src, group=self.group, async_op=True)
        else:
            w = dist.all_gather(list(out.unbind(0)), src, group=self.group, async_op=True)
        return out, w

    def add(self, j: int, rec: torch.Tensor) -> None:
        """View j's record; each j in [0, v) exactly once.

        Every rank must add its views in the SAME order of j: add() issues
        the step's collectives as it goes (a full-record all-gather for
        j < v - 1; the cameras and the chunked row gathers for j = v - 1), and
        collectives of different shapes issued in different orders on two
        ranks mismatch (a hang or corrupted records).  With one rank any order
        works."""
        if not 0 <= j < self.v:
            raise ValueError(f"ViewExchange.add: view {j} outside [0, {self.v})")
        if self.world == 1:
            self.buf[j].copy_(rec)
            return
        P = self.P
        if j < self.v - 1 or P == 0:
            if j < self.v - 1 and self.full[j] is not None:
                raise ValueError(f"ViewExchange.add: view {j} added twice")
            out, w = self._gather(rec)
            if j < self.v - 1:
                self.full[j] = out
            self.pending.append(w)
            return
        if self.cam_stage is not None:
            raise ValueError(f"ViewExchange.add: view {j} added twice")
        self.cam_stage, self.cam_work = self._gather(rec[P * VIEW_ROW:])
        step = max(1, -(-P // self.chunks))
        for a in range(0, P, step):
            b = min(P, a + step)
            out, w = self._gather(rec[a * VIEW_ROW:b * VIEW_ROW])
            self.last.append((a, b, out, w))

    # views in rank-then-view order (the order exchange_view_records sums in)
    def _cams(self) -> List[torch.Tensor]:
        P = self.P
        return [self.full[j][r, P * VIEW_ROW:] if j < self.v - 1 else self.cam_stage[r]
                for r in range(self.world) for j in range(self.v)]

    def _rows(self, a: int, b: int, chunk: torch.Tensor) -> List[torch.Tensor]:
        return [self.full[j][r, a * VIEW_ROW:b * VIEW_ROW] if j < self.v - 1 else chunk[r]
                for r in range(self.world) for j in range(self.v)]

    def wait(self) -> None:
        for w in self.pending:
            w.wait()
        if self.cam_work is not None:
            self.cam_work.wait()
        for _a, _b, _c, w in self.last:
            w.wait()

    def records(self) -> torch.Tensor:
        """The gathered records as one [world * v, RL] tensor in summation
        order (a copy, for checks; finish() reads them in place)."""
        if self.world == 1:
            return self.buf.clone()
        self.wait()
        pieces = [self._rows(a, b, ch) for a, b, ch, _w in self.last]  # per chunk: one slice per view
        return torch.stack([torch.cat([p[i] for p in pieces] + [c]) for i, c in enumerate(self._cams())])

    def finish(self, settings, means3D: torch.Tensor, shs: torch.Tensor, scales: torch.Tensor,
               rotations: torch.Tensor, stats=None):
        P = self.P
        if P == 0:
            for w in self.pending:
                w.wait()
            return _empty_param_grads(means3D, shs)
        if self.world == 1:
            return multiview_param_grads(self.buf, means3D, shs, settings.sh_degree, scales, rotations,
                                         settings.scale_modifier, stats)
        from . import _C
        if self.cam_work is None or any(f is None for f in self.full):
            raise ValueError("ViewExchange.finish: not every view was added")
        for w in self.pending:
            w.wait()
        self.cam_work.wait()
        cams = self._cams()
        dev = means3D.device
        M = shs.shape[1] if shs is not None and shs.numel() else 0
        outs = (torch.empty((P, 3), device=dev), torch.empty((P, M, 3), device=dev), torch.empty((P, 1), device=dev),
                torch.empty((P, 3), device=dev), torch.empty((P, 4), device=dev))
        e = torch.empty(0, device=dev)
        st = stats if stats is not None else (e, e, e)
        for a, b, chunk, w in self.last:
            w.wait()
            _C.backward_gaussians_multiview_views(self._rows(a, b, chunk), cams, a, means3D,
                                                  shs if shs is not None else e,
                                                  int(settings.sh_degree), scales, rotations,
                                                  float(settings.scale_modifier), *outs, st[0], st[1], st[2])
        return outs


_SIDE_STREAMS: Dict[Tuple[int, int], List[torch.cuda.Stream]] = {}


def run_views_on_streams(n_views: int, render_one, n_streams: int = 3, device=None) -> None:
    """render_one(j) for j in [0, n_views), view j enqueued on stream
    j % n_streams (stream 0 = the current stream, the others cached side
    streams), so the independent per-view forward + blend backward of one
    step overlap on the GPU: view j + 1's preprocess and binning (HBM- and
    latency-bound) run beside view j's blends (VALU-bound).  The host still
    enqueues in view order -- each forward waits on the host for its own
    instance count -- so every view's collectives (ViewExchange.add inside
    render_one) are issued in the same order on every rank.  The side streams
    start after the work already on the current stream, and the current
    stream continues after all of them."""
    if n_views <= 0:
        return
    if n_streams <= 1 or not torch.cuda.is_available():
        for j in range(n_views):
            render_one(j)
        return
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), n_streams)
    side = _SIDE_STREAMS.get(key)
    if side is None:
        side = [torch.cuda.Stream(device=dev) for _ in range(n_streams - 1)]
        _SIDE_STREAMS[key] = side
    cur = torch.cuda.current_stream(dev)
    streams = [cur] + side
    for s in side:
        s.wait_stream(cur)
    try:
        for j in range(n_views):
            s = streams[j % n_streams]
            if s is cur:
                render_one(j)
            else:
                with torch.cuda.stream(s):
                    render_one(j)
    finally:
        # joined back even when a view raises: the caller's stream (and the
        # caching allocator's reuse of its blocks) must not run ahead of
        # side-stream work still reading or writing them
        for s in side:
            cur.wait_stream(s)


def _empty_param_grads(means3D: torch.Tensor, shs: Optional[torch.Tensor]):
    dev = means3D.device
    P = means3D.shape[0]
    M = shs.shape[1] if shs is not None and shs.dim() == 3 else 0
    return (torch.zeros((P, 3), device=dev), torch.zeros((P, M, 3), device=dev), torch.zeros((P, 1), device=dev),
            torch.zeros((P, 3), device=dev), torch.zeros((P, 4), device=dev))


def exchange_view_records(rec: torch.Tensor, settings, means3D: torch.Tensor, shs: torch.Tensor,
                          scales: torch.Tensor, rotations: torch.Tensor, group=None, stats=None, chunks: int = 4):
    """exchange_view_grads from this rank's view record(s) on -- rec is one
    [P * 10 + 40] record or [v, P * 10 + 40] (v views per rank, the same v on
    every rank): the (chunked) all-gather and the multi-view parameter
    backward over all world * v views, in rank-then-view order."""
    recs = rec if rec.dim() == 2 else rec.unsqueeze(0)
    P = means3D.shape[0]
    if P == 0:  # every Gaussian pruned: nothing to exchange, empty gradients
        return _empty_param_grads(means3D, shs)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1 or chunks <= 1:
        views = gather_view_records(recs, group)
        return multiview_param_grads(views, means3D, shs, settings.sh_degree, scales, rotations,
                                     settings.scale_modifier, stats)
    from . import _C
    world = dist.get_world_size(group)
    v = recs.shape[0]
    nccl = dist.get_backend(group) == "nccl"

    def gather_async(src: torch.Tensor, width: int) -> Tuple[torch.Tensor, object]:
        # src: [v, width] -> [world * v, width] in rank-then-view order
        src = src.contiguous().view(-1)
        out = torch.empty((world, src.numel()), dtype=src.dtype, device=src.device)
        if nccl:
            w = dist.all_gather_into_tensor(out, src, group=group, async_op=True)
        else:
            w = dist.all_gather(list(out.unbind(0)), src, group=group, async_op=True)
        return out.view(world * v, width), w

    cams, w_cam = gather_async(recs[:, P * VIEW_ROW:], CAM_WORDS)
    step = max(1, -(-P // max(1, chunks)))
    bounds = [(a, min(P, a + step)) for a in range(0, P, step)]
    pending = [(a, b) + gather_async(recs[:, a * VIEW_ROW:b * VIEW_ROW], (b - a) * VIEW_ROW) for a, b in bounds]
    dev = means3D.device
    M = shs.shape[1] if shs is not None and shs.numel() else 0
    outs = (torch.empty((P, 3), device=dev), torch.empty((P, M, 3), device=dev), torch.empty((P, 1), device=dev),
            torch.empty((P, 3), device=dev), torch.empty((P, 4), device=dev))
    e = torch.empty(0, device=dev)
    st = stats if stats is not None else (e, e, e)
    w_cam.wait()
    for a, b, rows, w in pending:
        w.wait()
        _C.backward_gaussians_multiview_range(rows, cams, a, means3D, shs if shs is not None else e,
                                              int(settings.sh_degree), scales, rotations,
                                              float(settings.scale_modifier), *outs, st[0], st[1], st[2])
    return outs
