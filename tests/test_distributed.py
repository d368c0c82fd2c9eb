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


@pytest.mark.timeout(240)
@pytest.mark.parametrize("mode", ["none", "raise", "mismatch", "hang"])
def test_one_failing_rank_ends_every_rank(mode, tmp_path):
    """bench.py's fail-fast path (ptdist.init / phase / guarded / agree) with 3 gloo ranks: when rank 1
    fails in phase "frame check" -- an exception, a failed frame check, or a hang -- EVERY rank exits
    non-zero within the collective timeout (plus process start-up), and the failing rank's stderr
    names its rank and phase.  With no failure all ranks exit 0 and the gather is complete."""
    import subprocess
    import time
    world, timeout_s, watchdog_s = 3, 8.0, 12.0
    port = str(_free_port())
    procs, logs = [], []
    t0 = time.perf_counter()
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, GLOO_SOCKET_IFNAME="lo")
        log = open(tmp_path / f"rank{r}.log", "w+")
        logs.append(log)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "failfast_worker.py"), mode, str(timeout_s),
                                       str(watchdog_s)], env=env, stdout=log, stderr=subprocess.STDOUT,
                                      start_new_session=True))
    limit = 150.0   # start-up (import torch) + the timeout / watchdog, far below this test's own timeout
    try:
        for p in procs:
            p.wait(timeout=max(1.0, limit - (time.perf_counter() - t0)))
    except subprocess.TimeoutExpired:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
        tails = []
        for r, log in enumerate(logs):
            log.seek(0)
            tails.append(f"--- rank {r} (exit {procs[r].poll()}):\n" + log.read()[-1500:])
        pytest.fail("ranks still running after %.0f s:\n%s" % (limit, "\n".join(tails)))
    elapsed = time.perf_counter() - t0
    out = []
    for log in logs:
        log.seek(0)
        out.append(log.read())
        log.close()
    codes = [p.returncode for p in procs]
    if mode == "none":
        assert codes == [0] * world, out
        return
    assert all(c != 0 for c in codes), (codes, out)
    assert "[rank 1/3] FAILED in phase 'frame check'" in out[1] or mode == "hang", out[1]
    if mode == "hang":   # the hung rank's watchdog dumps its stack (faulthandler) and ends it
        assert "time.sleep" in out[1] or "Timeout" in out[1], out[1]
    # every rank ends within the timeout (the hung rank: its watchdog) after start-up
    assert elapsed < 120.0, elapsed


def test_bench_method_is_the_same_at_every_n(monkeypatch):
    """The driver divides bench.py's N = 1 and N = 8 ms_per_step: both lines must measure the same
    method.  With the default flags every N renders one frame at a time (frames_in_flight 1) on the
    host-built wide tree; the two-frames-in-flight figure is a separate `pipelined` field at every N."""
    import bench
    monkeypatch.delenv("PT_BENCH_WIDE_DEVICE", raising=False)
    args = bench.make_parser().parse_args([])
    got = {n: bench.run_settings(args, n) for n in (1, 2, 4, 8)}
    assert all(v == {"frames_in_flight": 1, "wide_tree": "host"} for v in got.values()), got
    assert not args.no_pipelined
    monkeypatch.setenv("PT_BENCH_WIDE_DEVICE", "1")   # an override applies to every N alike
    assert {bench.run_settings(args, n)["wide_tree"] for n in (1, 8)} == {"device"}
    two = bench.make_parser().parse_args(["--frames-in-flight", "2"])
    assert {bench.run_settings(two, n)["frames_in_flight"] for n in (1, 8)} == {2}
