"""Two ranks on one GPU (gloo; the one-GPU box's stand-in for RCCL over
xGMI): the "views" exchange end to end (data_parallel.exchange_view_grads).

* every rank ends with bit-identical parameter gradients and statistics;
* the chunked, asynchronous gather (chunks > 1: the transfer of chunk c + 1
  overlapping the backward of chunk c) gives the same bits as one gather;
* the result equals the per-view reference backwards summed (atomic-order
  noise, 1e-5 relative), i.e. the "8-GPU summed grad equals the sum of the
  single-GPU per-view grads" bar of SURVEY §8(e).
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P, W, H = 12000, 192, 128


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank):
    import sys
    for p in (ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import gs_helpers as G
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    sc = S.make_scene(P, S.make_camera(W, H), seed=3)
    cam = S.make_orbit_camera(W, H, (rank - 0.5) * 8.0)
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc)
    dpix = torch.from_numpy(S.make_cotangent(H, W, 50 + rank)).cuda()
    return G, s, t, dpix


def _fwd(C, s, t):
    e = torch.Tensor([])
    return C.rasterize_gaussians(s.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], 1.0, e,
                                 s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width,
                                 t["shs"], 3, s.campos, False, False)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        import gaussian_splatting_with_eye_tracking_amd._C as C
        from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
        G, s, t, dpix = _setup(rank)
        fwd = _fwd(C, s, t)
        # one record (the blend backward's float atomics add in a run-dependent
        # order), exchanged with one gather and with 3 asynchronous chunks
        rec = DP.view_record(s, fwd[2], fwd[3], fwd[0], fwd[4], fwd[5], dpix)
        res = {}
        for chunks in (1, 3):
            stats = tuple(torch.zeros(P, device="cuda") for _ in range(3))
            g = DP.exchange_view_records(rec, s, t["means3D"], t["shs"], t["scales"], t["rotations"],
                                         stats=stats, chunks=chunks)
            torch.cuda.synchronize()
            res[chunks] = [x.cpu().numpy() for x in g] + [x.cpu().numpy() for x in stats]
        # two views per rank: the stacked exchange vs the pipelined one (each
        # record gathered as it is produced, the last one in chunks)
        rec2 = DP.view_record(s, fwd[2], fwd[3], fwd[0], fwd[4], fwd[5], dpix * 0.5 + 0.25)
        stats = tuple(torch.zeros(P, device="cuda") for _ in range(3))
        g = DP.exchange_view_records(torch.stack([rec, rec2]), s, t["means3D"], t["shs"], t["scales"],
                                     t["rotations"], stats=stats, chunks=3)
        res["stacked"] = [x.cpu().numpy() for x in g] + [x.cpu().numpy() for x in stats]
        ex = DP.ViewExchange(P, 2, "cuda", chunks=3)
        ex.add(0, rec)
        ex.add(1, rec2)
        stats = tuple(torch.zeros(P, device="cuda") for _ in range(3))
        g = ex.finish(s, t["means3D"], t["shs"], t["scales"], t["rotations"], stats=stats)
        torch.cuda.synchronize()
        res["pipelined"] = [x.cpu().numpy() for x in g] + [x.cpu().numpy() for x in stats]
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_view_exchange():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = {}
    import queue
    import time
    t0 = time.time()
    while len(outs) < world:  # (a worker that dies fails the test at once, not after the queue's timeout)
        try:
            rank, res = q.get(timeout=5)
            outs[rank] = res
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"a rank exited with {dead}"
            assert time.time() - t0 < 150, "ranks did not finish"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i in range(8):
        np.testing.assert_array_equal(outs[0][1][i], outs[1][1][i])   # replicas bit-identical
        np.testing.assert_array_equal(outs[0][3][i], outs[1][3][i])
        np.testing.assert_array_equal(outs[0][1][i], outs[0][3][i])   # chunked == one gather
        np.testing.assert_array_equal(outs[0]["stacked"][i], outs[0]["pipelined"][i])  # pipelined == stacked
        np.testing.assert_array_equal(outs[1]["stacked"][i], outs[1]["pipelined"][i])
        np.testing.assert_array_equal(outs[0]["pipelined"][i], outs[1]["pipelined"][i])
    # == sum over the two views of the reference-API backward
    import gaussian_splatting_with_eye_tracking_amd._C as C
    want = None
    for rank in range(world):
        G, s, t, dpix = _setup(rank)
        fwd = _fwd(C, s, t)
        K, color, radii, geom, binning, img = fwd
        e = torch.Tensor([])
        g = C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"], 1.0, e,
                                           s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, dpix, t["shs"], 3,
                                           s.campos, geom, K, binning, img, False)
        per = [g[3], g[5], g[2], g[6], g[7]]
        want = [x.double().cpu().numpy() for x in per] if want is None else \
            [a + x.double().cpu().numpy() for a, x in zip(want, per)]
    for i in range(5):
        assert G.rel_err(outs[0][1][i], want[i]) < 1e-5, i
