"""Multi-rank path on CPU (gloo, world_size 2 and 3): stripe partition + gather to rank 0 +
un-permute reproduce the single-rank frame bit-exactly.  The per-rank render here is the
oracle (CPU); on the GPU box bench.py runs the same partition with libpt.so and RCCL."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, w, h, stripe, spp, q, rgba8=False):
    sys.path[:0] = [os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"), os.path.join(REPO, "oracle"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    import ptamd
    import ptdist
    p = ptamd.Preset("rtiow", w, h)
    nodes = oracle.build_lbvh(p.objects, oracle.morton_keys(p.objects))
    rows = ptdist.stripe_rows(h, stripe, world, rank)
    states = oracle.film_states(11, w, rows)
    rgb, st = oracle.render(p.objects, p.materials, nodes, ptamd.camera_to_array(p.camera), w, h, rows, spp, 50,
                            states, 1)
    mr = ptdist.max_rows(h, stripe, world)
    if rgba8:   # the device-quantised frame (PT_OUT_RGBA8), as bench.py sends it by default
        px = oracle.quantize_png(rgb)
        buf = torch.zeros((mr * w * 4,), dtype=torch.uint8)
    else:
        px = rgb
        buf = torch.zeros((mr * w * 3,), dtype=torch.float32)      # flat
    buf[: px.size] = torch.from_numpy(px.reshape(-1))
    out = ptdist.gather_to_root(buf, world, rank)
    total = torch.tensor([float(st.rays)], dtype=torch.float64)
    dist.all_reduce(total)
    if rank == 0:
        q.put((ptdist.assemble(out.numpy(), h, w, stripe, world, 4 if rgba8 else 3), total.item()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,stripe,rgba8", [(2, 8, False), (3, 5, False), (2, 4, True)])
def test_stripes_gather_equals_single_rank(world, stripe, rgba8):
    sys.path[:0] = [os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"), os.path.join(REPO, "oracle")]
    import oracle
    import ptamd
    w, h, spp = 40, 27, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, stripe, spp, q, rgba8)) for r in range(world)]
    for pr in procs:
        pr.start()
    try:
        img, rays = q.get(timeout=120)
    finally:
        for pr in procs:
            pr.join(timeout=5)
            if pr.is_alive():
                pr.kill()
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p = ptamd.Preset("rtiow", w, h)
    nodes = oracle.build_lbvh(p.objects, oracle.morton_keys(p.objects))
    rows = np.arange(h, dtype=np.int32)
    ref, st = oracle.render(p.objects, p.materials, nodes, ptamd.camera_to_array(p.camera), w, h, rows, spp, 50,
                            oracle.film_states(11, w, rows), 1)
    if rgba8:
        np.testing.assert_array_equal(img.reshape(-1, 4), oracle.quantize_png(ref))
    else:
        np.testing.assert_array_equal(img.reshape(-1, 3).view(np.uint32), ref.view(np.uint32))
    assert rays == st.rays


def test_stripe_partition_covers_frame():
    sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
    import ptdist
    for h, stripe, world in ((1080, 8, 8), (1080, 8, 3), (7, 4, 5), (800, 8, 2)):
        parts = [ptdist.stripe_rows(h, stripe, world, r) for r in range(world)]
        allr = np.sort(np.concatenate(parts))
        np.testing.assert_array_equal(allr, np.arange(h))
        assert max(len(p) for p in parts) <= ptdist.max_rows(h, stripe, world)
