"""The multi-GPU frame behind the C ABI (include/gsm_multigpu.h, csrc/gsm_multigpu.hip) on one MI355X:
a world-size-1 RCCL communicator from torch.distributed drives the whole protocol -- partition
projection, counts all-gather, peer-write exchange (to itself), ordering all-reduce, slab render
from the device-side count -- and the frame equals the single-GPU frame and the oracle bit for bit.
The N > 1 runs are the driver's (8-GPU node); the exchange order across ranks is covered on CPU by
tests/test_exchange_distributed.py and the composition of slabs by
tests/test_gpu_parity.py::test_partitioned_frame_matches_single_gpu."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_world1(cuda):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=cuda.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


@pytest.mark.parametrize("n,w,h,sh,prec", [(60_000, 640, 360, 16, 1), (30_000, 1280, 720, 4, 0)])
def test_world1_rccl_frame_matches_single_gpu_and_oracle(gsm, cuda, oracle, nccl_world1, n, w, h, sh, prec):
    from gsm_amd import scenes
    world, harm, cam = scenes.gen_scene(n, w, h, sh, prec, seed=5)
    wt = cuda.from_numpy(world.view(np.uint8).reshape(-1).copy()).cuda()
    ht = cuda.from_numpy(harm.view(np.uint8).reshape(-1).copy()).cuda()
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cp = gsm.CameraParams.from_dict(cam)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rend = gsm.GlobalRenderer(device=0, config=cfg)
    mg = gsm.MultiGpuRenderer(rend, gsm.MultiGpuRenderer.torch_comm(0), 0, 1)
    color = cuda.full((h, w, 4), float("nan"), dtype=cuda.float16, device="cuda")
    depth = cuda.full((h, w), float("nan"), dtype=cuda.float16, device="cuda")
    for _ in range(2):  # a second frame reuses the exchange buffers and the IPC mapping
        mg.render(color, depth, inp, cp, w, h)
    cuda.cuda.synchronize()
    ref = oracle.render(world, harm, sh, cam, w, h, max_gaussians=n)
    got = color.view(cuda.int16).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, ref["color"])
    assert np.array_equal(depth.view(cuda.int16).cpu().numpy().view(np.uint16), ref["depth"])
    counts = mg.counts()
    with_tiles = int(np.count_nonzero(ref["tile_counts"]))
    assert counts.shape == (1, 1) and with_tiles <= counts[0, 0] <= n
    assert rend.debug_read_total_assignments() == ref["total_assignments"]
    mg.close()
    rend.close()


def test_create_rejects_a_mismatched_world(gsm, cuda, nccl_world1):
    rend = gsm.GlobalRenderer(device=0, config=gsm.RendererConfig(max_gaussians=16, max_width=64, max_height=32))
    with pytest.raises(gsm.RendererError) as e:
        gsm.MultiGpuRenderer(rend, gsm.MultiGpuRenderer.torch_comm(0), 0, 2)
    assert e.value.status == gsm.Status.INVALID_ARGUMENT
    rend.close()


@pytest.mark.parametrize("world,n,w,h,prec", [(2, 40_000, 640, 360, 1), (3, 60_000, 1280, 720, 1),
                                              (8, 50_000, 640, 360, 0)])
def test_native_exchange_virtual_ranks(gsm, cuda, oracle, world, n, w, h, prec):
    """The device steps of gsm_multigpu_render for world > 1 without RCCL (include/gsm_debug.h): W
    renderers on one GPU play the ranks -- each projects its id range and counts its records per slab
    (k_project_part), the count matrix is stacked on the device (the all-gather), every rank's
    k_part_copy writes its records straight into every slab owner's receive buffer at the matrix's
    offsets, and each owner renders its rows from the count read on the device.  Ids and slab rows
    are split as gsm_multigpu.hip splits them.  The composed frame equals the oracle bit for bit:
    the push offsets, the receive counts and the rank-ordered ties of world > 1 (the world-1 RCCL
    test above cannot reach them)."""
    import math
    from gsm_amd import scenes
    sh = 16 if prec else 4
    world_np, harm_np, cam_d = scenes.gen_scene(n, w, h, sh, prec, seed=78)
    ref = oracle.render(world_np, harm_np, sh, cam_d, w, h, max_gaussians=n)
    wt = cuda.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).cuda()
    ht = cuda.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).cuda()
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cam = gsm.CameraParams.from_dict(cam_d)
    tiles_y = (h + 15) // 16
    per_rows = math.ceil(tiles_y / world)
    rows = [min(i * per_rows, tiles_y) for i in range(world + 1)]
    per_ids = math.ceil(n / world)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    ranks = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
    send = [cuda.zeros(world, dtype=cuda.int32, device="cuda") for _ in range(world)]
    for rk in range(world):
        first = min(rk * per_ids, n)
        ranks[rk].debug_partition_counts(inp, cam, w, h, first, min(per_ids, n - first), rows, send[rk])
    counts = cuda.stack(send).contiguous()  # row r = rank r's records per slab (the all-gather)
    recv = [cuda.zeros(n * gsm.SPLAT_RECORD_BYTES, dtype=cuda.uint8, device="cuda") for _ in range(world)]
    recv_count = [cuda.full((1,), -1, dtype=cuda.int32, device="cuda") for _ in range(world)]
    for rk in range(world):
        ranks[rk].debug_partition_push(world, rk, counts, recv, recv_count[rk])
    color = cuda.full((h, w, 4), float("nan"), dtype=cuda.float16, device="cuda")
    depth = cuda.full((h, w), float("nan"), dtype=cuda.float16, device="cuda")
    for d in range(world):
        if rows[d] == rows[d + 1]:
            continue
        ranks[d].set_tile_rows(rows[d], rows[d + 1])
        ranks[d].debug_render_records_device_count(color, depth, recv[d], n, recv_count[d], w, h)
    cuda.cuda.synchronize()
    cm = counts.cpu().numpy().astype(np.int64)
    assert [int(c.item()) for c in recv_count] == [int(x) for x in cm.sum(axis=0)]
    with_tiles = int(np.count_nonzero(ref["tile_counts"]))
    assert with_tiles <= cm.sum() <= with_tiles * world
    got = color.view(cuda.int16).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, ref["color"])
    assert np.array_equal(depth.view(cuda.int16).cpu().numpy().view(np.uint16), ref["depth"])
    for rend in ranks:
        rend.close()


@pytest.mark.parametrize("rows,gather", [("contiguous", True), ("interleaved", True), ("contiguous", False)])
def test_world1_rccl_transport_frame(gsm, cuda, oracle, nccl_world1, rows, gather):
    """GSM_MG_TRANSPORT_RCCL (gsm_multigpu_options, r06): the same per-slab runs moved by
    RCCL inside the library -- count rows all-gathered and read on the host, the records by grouped
    ncclSend / ncclRecv (a device copy for the rank's own slab), the slab pixels by send / recv to rank 0 --
    over a world-1 communicator from torch.distributed.  Two frames, gathered into the caller's tensors (or
    rendered into them directly), equal the oracle bit for bit, and the counts the frame read are the
    single-GPU frame's."""
    from gsm_amd import scenes
    n, w, h, sh, prec = 60_000, 640, 360, 16, 1
    world, harm, cam = scenes.gen_scene(n, w, h, sh, prec, seed=5)
    wt = cuda.from_numpy(world.view(np.uint8).reshape(-1).copy()).cuda()
    ht = cuda.from_numpy(harm.view(np.uint8).reshape(-1).copy()).cuda()
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cams = [cam, scenes.orbit_camera(w, h, 5.0)]
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rend = gsm.GlobalRenderer(device=0, config=cfg)
    opts = gsm.MultiGpuOptions(rows=rows, transport="rccl")
    mg = gsm.MultiGpuRenderer(rend, gsm.MultiGpuRenderer.torch_comm(0), 0, 1, options=opts)
    for c in cams:
        color = cuda.full((h, w, 4), float("nan"), dtype=cuda.float16, device="cuda")
        depth = cuda.full((h, w), float("nan"), dtype=cuda.float16, device="cuda")
        mg.render(color, depth, inp, gsm.CameraParams.from_dict(c), w, h, gather=gather)
        cuda.cuda.synchronize()
        ref = oracle.render(world, harm, sh, c, w, h, max_gaussians=n)
        assert np.array_equal(color.view(cuda.int16).cpu().numpy().view(np.uint16), ref["color"])
        assert np.array_equal(depth.view(cuda.int16).cpu().numpy().view(np.uint16), ref["depth"])
        counts = mg.counts()
        assert counts.shape == (1, 1) and int(np.count_nonzero(ref["tile_counts"])) <= counts[0, 0] <= n
    assert mg.status() == 0
    mg.close()
    rend.close()
