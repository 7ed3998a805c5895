"""gloo tests (CPU) of the multi-view data-parallel exchange at world sizes 2,
3, 4 and 8 -- the driver's N = 2, 4, 8 scaling runs rehearsed rank for rank.

Each rank renders + back-propagates its own view (the CPU oracle stands in
for the GPU backward here), writes its gradients into the flat buffer, and
the all-reduce must deliver sum-over-views on every rank, bit-identically
("the 8-GPU summed grad equals the sum of the single-GPU
per-view grads").  The densification statistics are summed / max-reduced.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _view_grads(rank, world=2):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    W, H = 64, 48
    cam0 = S.make_camera(W, H)
    sc = S.make_scene(800, cam0, seed=0)
    cam = S.make_orbit_camera(W, H, yaw_deg=(rank - (world - 1) / 2.0) * 5.0)
    s = O.settings_from_camera(cam)
    kw = dict(shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    r = O.forward(s, sc.means3D, sc.opacities, **kw)
    g = O.backward(s, r, sc.means3D, S.make_cotangent(H, W, 100 + rank), **kw)
    return sc, g, r


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
        sc, g, r = _view_grads(rank, world)
        params = {"means3D": torch.from_numpy(sc.means3D), "shs": torch.from_numpy(sc.shs),
                  "opacities": torch.from_numpy(sc.opacities), "scales": torch.from_numpy(sc.scales),
                  "rotations": torch.from_numpy(sc.rotations)}
        fg = DP.FlatGrads(params)
        assert fg.flat.numel() == sc.P * DP.flat_numel_per_gaussian()
        fg.load({"means3D": torch.from_numpy(g["dL_dmeans3D"]), "shs": torch.from_numpy(g["dL_dsh"]),
                 "opacities": torch.from_numpy(g["dL_dopacity"]), "scales": torch.from_numpy(g["dL_dscales"]),
                 "rotations": torch.from_numpy(g["dL_drotations"])})
        DP.allreduce_(fg.flat)
        acc = torch.from_numpy(np.linalg.norm(g["dL_dmeans2D"][:, :2], axis=1)).float()
        denom = torch.from_numpy((r.radii > 0).astype(np.float32))
        radii = torch.from_numpy(r.radii.astype(np.float32))
        DP.densification_stats_allreduce_(acc, denom, radii)
        q.put((rank, fg.flat.numpy().copy(), acc.numpy(), denom.numpy(), radii.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_gradient_allreduce(world):
    """The north_star exchange: one flat all-reduce of every rank's view
    gradients (59 floats per Gaussian) and the densification statistics --
    every rank ends bit-identical, equal to the sum over the views."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = {}
    for _ in range(world):
        rank, flat, acc, denom, radii = q.get(timeout=240)
        outs[rank] = (flat, acc, denom, radii)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # replicas bit-identical
    for r in range(1, world):
        for i in range(4):
            np.testing.assert_array_equal(outs[0][i], outs[r][i])
    # == sum over views computed locally
    exp = []
    accs, dens, rads = [], [], []
    for rank in range(world):
        sc, g, r = _view_grads(rank, world)
        exp.append(np.concatenate([g["dL_dmeans3D"].ravel(), g["dL_dsh"].ravel(), g["dL_dopacity"].ravel(),
                                   g["dL_dscales"].ravel(), g["dL_drotations"].ravel()]))
        accs.append(np.linalg.norm(g["dL_dmeans2D"][:, :2], axis=1).astype(np.float32))
        dens.append((r.radii > 0).astype(np.float32))
        rads.append(r.radii.astype(np.float32))
    np.testing.assert_allclose(outs[0][0], np.sum(exp, 0), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(outs[0][1], np.sum(accs, 0), rtol=1e-5)
    np.testing.assert_array_equal(outs[0][2], np.sum(dens, 0))
    np.testing.assert_array_equal(outs[0][3], np.max(rads, 0))


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
        P = 1000
        rec = torch.arange(DP.view_record_numel(P), dtype=torch.float32) * (rank + 1) + 0.25 * rank
        views = DP.gather_view_records(rec)
        q.put((rank, views.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_view_record_all_gather_rank_order():
    """The "views" exchange: every rank receives all ranks' view records, in
    rank order, bit-identically (the multi-view backward then sums the views
    in that order on every rank, test_gpu_multiview.py)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = {}
    for _ in range(world):
        rank, views = q.get(timeout=240)
        outs[rank] = views
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, ROOT)
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    n = DP.view_record_numel(1000)
    exp = np.stack([np.arange(n, dtype=np.float32) * (r + 1) + np.float32(0.25 * r) for r in range(world)])
    for r in range(world):
        assert outs[r].shape == (world, n)
        np.testing.assert_array_equal(outs[r], exp)


def _multi_view_gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
        P = 700
        n = DP.view_record_numel(P)
        # two views per rank: view v = 2 * rank + i
        rec = torch.stack([torch.arange(n, dtype=torch.float32) + 1000.0 * (2 * rank + i) for i in range(2)])
        views = DP.gather_view_records(rec)
        # zero Gaussians (everything pruned): empty gradients, no collective needed
        z = torch.zeros((0, 3))

        class _S:
            sh_degree, scale_modifier = 3, 1.0

        g = DP.exchange_view_records(torch.zeros(DP.view_record_numel(0)), _S, z, torch.zeros((0, 16, 3)),
                                     z, torch.zeros((0, 4)))
        q.put((rank, views.numpy().copy(), [tuple(t.shape) for t in g]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_view_record_gather_several_views_per_rank_and_empty_model():
    """Config 5 at N < 8 ranks: each rank packs 8 / N view records; the
    gather returns [world * v, record] in rank-then-view order on every rank.
    A model with zero Gaussians yields empty gradients instead of failing."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_multi_view_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = {}
    for _ in range(world):
        rank, views, shapes = q.get(timeout=240)
        outs[rank] = (views, shapes)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, ROOT)
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    n = DP.view_record_numel(700)
    exp = np.stack([np.arange(n, dtype=np.float32) + np.float32(1000.0 * v) for v in range(4)])
    for r in range(world):
        np.testing.assert_array_equal(outs[r][0], exp)
        assert outs[r][1] == [(0, 3), (0, 16, 3), (0, 1), (0, 3), (0, 4)]


def _pipelined_worker(rank, world, port, q, order=(0, 1, 2), v=3):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
        P = 37
        n = DP.view_record_numel(P)
        ex = DP.ViewExchange(P, v, "cpu", chunks=4)
        for j in order:  # record of (rank, view j): its values say whose it is
            ex.add(j, torch.arange(n, dtype=torch.float32) + 1000.0 * (rank * v + j))
        try:
            ex.add(0, torch.zeros(n))
            dup = False
        except ValueError:
            dup = True
        q.put((rank, ex.records().numpy().copy(), dup))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,order", [(2, (0, 1, 2)), (2, (1, 2, 0)), (4, (0, 1)), (4, (1, 0)), (8, (0,))])
def test_pipelined_view_gather_order(world, order):
    """data_parallel.ViewExchange (per-view asynchronous gathers, the last view
    in Gaussian chunks) lands every record in rank-then-view order, the order
    exchange_view_records sums in, on every rank, whatever order the views are
    added in (every rank adding in the same order: the gathers are
    collectives); a view added twice is refused.  Config 5's schedules: world
    2 with 3 views each, world 4 with 2 (8 / 4), world 8 with one view per
    rank -- the chunked last-view path alone."""
    v = len(order)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, world, port, q, order, v)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    outs = {r: rec for r, rec, _dup in got}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(dup for _r, _rec, dup in got)
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    n = DP.view_record_numel(37)
    want = np.stack([np.arange(n, dtype=np.float32) + 1000.0 * k for k in range(world * v)])
    for r in range(world):
        np.testing.assert_array_equal(outs[r], want)
