"""GPU tests: bench.py's multi-rank flow run as separate processes: row stripes
over ranks, the gather to rank 0 and the un-permuted PNG equal to the 1-rank PNG (gloo ranks sharing
the box's one GPU, and RCCL with the one rank a one-GPU box allows), the fail-fast of a failing
rank, and the C4 8-rank rehearsal.

These tests start their own GPU processes (up to 8 ranks).  The file sorts LAST among the GPU
tests (round 6; in round 5 it ran first): the ranks then share the GPU with the suite process, which
by then holds its own GPU context, streams and device memory -- the order in which the 8-rank
rehearsal once failed (round 5, gpurun_out/r05h).  Each run's log records whether the parent holds
GPU state and the box's load, and with PT_TEST_LOG_DIR set every log is kept (helpers.run_logged).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _quiet_parent():
    """Before the multi-process tests: the suite process's own GPU work finished and its freed memory
    returned (a parent with frames still in flight or large caches is the one difference between these
    tests late in the suite and alone; each run's log records the parent's state, helpers.run_logged)."""
    import gc
    import sys
    gc.collect()
    t = sys.modules.get("torch")
    if t is not None and t.cuda.is_initialized():
        t.cuda.synchronize()
        t.cuda.empty_cache()
    yield


def free_port() -> str:
    """A free TCP port on 127.0.0.1 for a torch.distributed.run rendezvous (a fixed port can still be
    held by an earlier run on a shared box)."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return str(sk.getsockname()[1])


def _torchrun(n, port=None):
    import sys
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", port or free_port()]


def _rank_env(**kw):
    """Multi-rank runs of bench.py: phases traced to stderr (PT_DIST_TRACE), gloo bound to the
    loopback interface (the rendezvous is 127.0.0.1; gloo would otherwise pick the interface the
    host name resolves to), a collective timeout and a watchdog well below the subprocess timeout."""
    import os
    env = dict(os.environ, PT_DIST_TRACE="1", GLOO_SOCKET_IFNAME="lo", PT_DIST_TIMEOUT="60", PT_BENCH_WATCHDOG="150")
    env.update(kw)
    return env


@pytest.mark.timeout(400)
def test_bench_two_ranks_reassemble_one_rank_frame(tmp_path):
    """bench.py's multi-rank flow (stripe partition, per-rank RGBA8 frames, gather, un-permute,
    PNG) rehearsed with two ranks sharing the GPU over gloo: the PNG equals the 1-rank PNG, and the
    N > 1 line carries the per-rank kernel / gather figures and one frame's latency beside the
    pipelined (two frames in flight) rate; both lines report the same method (one frame at a time,
    the host-built wide tree)."""
    import os
    import sys
    from helpers import failure_digest, last_json, read_png, run_logged
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["bench.py", "--config", "c2", "--spp", "4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
              "--no-compat"]
    one, two = str(tmp_path / "one.png"), str(tmp_path / "two.png")
    rc, log1, _ = run_logged([sys.executable] + common + ["--png", one], 150, cwd=repo, log_path=tmp_path / "r1.log")
    assert rc == 0, log1[-3000:]
    rc, log2, _ = run_logged(_torchrun(2) + common[:1] + ["--gpus", "2"] + common[1:] + ["--png", two], 200, cwd=repo,
                             env=_rank_env(PT_DIST_BACKEND="gloo"), log_path=tmp_path / "r2.log")
    assert rc == 0, failure_digest(log2)
    np.testing.assert_array_equal(read_png(one), read_png(two))
    b = last_json(log2)
    assert [r["rank"] for r in b["per_rank"]] == [0, 1]
    assert all(r["kernel_ms"] > 0 and r["gather_ms"] >= 0 and r["rays_per_frame"] > 0 for r in b["per_rank"])
    assert sum(r["rays_per_frame"] for r in b["per_rank"]) == b["config"]["rays_per_frame"]
    a = last_json(log1)
    for k in ("frames_in_flight", "wide_tree"):   # the same method at N = 1 and N = 2
        assert a["config"][k] == b["config"][k], (k, a["config"][k], b["config"][k])
    assert b["config"]["frames_in_flight"] == 1 and b["config"]["wide_tree"] == "host"
    assert a["pipelined"]["frames_in_flight"] == b["pipelined"]["frames_in_flight"] == 2
    assert b["pipelined"]["ms_per_step"] > 0 and b["pipelined"]["value"] > 0
    assert "[rank 1/2] phase: timed frames" in log2 and "[rank 1/2] phase: pipelined frames" in log2


@pytest.mark.timeout(400)
@pytest.mark.parametrize("kind", ["raise", "mismatch", "hang"])
def test_bench_failing_rank_ends_every_rank(tmp_path, kind):
    """Fail-fast of bench.py's multi-rank flow (two gloo ranks sharing the GPU): rank 1 fails just
    before the timed frames (PT_BENCH_INJECT: an exception, a frame that differs from the
    reference-order frame, or a hang) and BOTH ranks exit non-zero, well within the collective
    timeout + watchdog, with the failure named by rank and phase."""
    import os
    import sys
    from helpers import run_logged
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    where = "timed frames" if kind == "mismatch" else "timed"
    cmd = _torchrun(2) + ["bench.py", "--gpus", "2", "--config", "c2", "--spp", "4", "--steps", "2", "--warmup", "1",
                          "--no-cpu-baseline", "--no-compat"]
    env = _rank_env(PT_DIST_BACKEND="gloo", PT_BENCH_INJECT=f"1:{where}:{kind}", PT_DIST_TIMEOUT="20",
                    PT_BENCH_WATCHDOG="40", TORCHELASTIC_ERROR_FILE=str(tmp_path / "err.json"))
    rc, log, wall = run_logged(cmd, 240, cwd=repo, env=env, log_path=tmp_path / "fail.log")
    assert rc != 0, log[-3000:]
    if kind == "raise":
        assert "[rank 1/2] FAILED in phase 'timed frames'" in log and "injected failure" in log, log[-3000:]
    elif kind == "mismatch":   # every rank learns of it (agree) and exits with it
        assert log.count("frame differs from the reference-order frame on rank(s) [1]") == 2, log[-3000:]
    else:   # the peer's collective times out (20 s) or the hung rank's watchdog (40 s) fires first
        assert "Timed out" in log or "Timeout (0:00:40)" in log or "FAILED" in log, log[-3000:]
    assert wall < 200, wall


@pytest.mark.timeout(400)
@pytest.mark.parametrize("fif", [1, 2])
def test_bench_rccl_gather_one_rank(tmp_path, fif):
    """bench.py's multi-rank flow over RCCL (backend "nccl": process group, dist.gather of the
    RGBA8 stripes, barriers, max / sum reductions) with the one rank a one-GPU box allows
    (PT_DIST_FORCE=1): the PNG equals the plain 1-rank PNG and the reported rays are the frame's.
    fif 2: frames in flight as N > 1 runs them (two films on two streams, each frame's gather
    enqueued on its own stream, three timed frames so both films alternate)."""
    import os
    import sys
    from helpers import last_json, read_png, run_logged
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["bench.py", "--config", "c2", "--spp", "4", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
              "--no-compat", "--no-interactive"]
    one, forced = str(tmp_path / "one.png"), str(tmp_path / "rccl.png")
    rc, log1, _ = run_logged([sys.executable] + common + ["--png", one], 150, cwd=repo, log_path=tmp_path / "r1.log")
    assert rc == 0, log1[-3000:]
    rc, log2, _ = run_logged(_torchrun(1) + common[:1] + ["--gpus", "1"] + common[1:] +
                             ["--png", forced, "--frames-in-flight", str(fif), "--steps", "3"], 200, cwd=repo,
                             env=_rank_env(PT_DIST_FORCE="1", PT_DIST_BACKEND="nccl"), log_path=tmp_path / "r2.log")
    assert rc == 0, log2[-3000:]
    np.testing.assert_array_equal(read_png(one), read_png(forced))
    a, b = last_json(log1), last_json(log2)
    assert a["config"]["rays_per_frame"] == b["config"]["rays_per_frame"] > 0
    assert b["config"]["frames_in_flight"] == fif and b["steps"] == 3
    # the RCCL gather's own time, from HIP events on the frame's stream
    assert len(b["per_rank"]) == 1 and b["per_rank"][0]["gather_ms"] > 0
    assert (b.get("single_frame_ms") is not None) == (fif == 2)


@pytest.mark.timeout(780)
def test_bench_c4_eight_ranks_rehearsal(tmp_path):
    """C4 (BASELINE.json configs[3]: the C3 scene at 1920x1080, 4096 spp, row-tiled over 8 GPUs)
    through bench.py's own multi-rank flow: 8 ranks over gloo sharing this one GPU (a rehearsal,
    never a reported number), each rendering its 1/8 of the stripes at the full sample count on the
    wide tree it built (host SAH, as at N = 1); the gathered, un-permuted PNG equals the 1-rank PNG
    byte for byte and the rank-0 line reports the whole frame's rays and all eight ranks' figures."""
    import os
    import sys
    from helpers import failure_digest, last_json, read_png, run_logged
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["bench.py", "--config", "c4", "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-compat",
              "--no-interactive"]
    one, eight = str(tmp_path / "one.png"), str(tmp_path / "eight.png")
    rc, log1, _ = run_logged([sys.executable] + common + ["--png", one], 240, cwd=repo, log_path=tmp_path / "r1.log")
    assert rc == 0, failure_digest(log1)
    # eight processes share one GPU and the box's CPU share here, so the rehearsal's collective
    # timeout is wider than the other tests' (a phase takes a few seconds: 28-46 s for the whole run);
    # the per-phase watchdog fires before the collective timeout, so a rank stuck in a phase dumps its
    # own stack (faulthandler) before the others give up on it, and both fire inside the GPU box's
    # 180-s silence limit; the rank log streams into gpurun_out/test_logs/ as the ranks trace phases
    env = _rank_env(PT_DIST_BACKEND="gloo", PT_DIST_TIMEOUT="170", PT_BENCH_WATCHDOG="150")
    rc, log8, wall = run_logged(_torchrun(8) + common[:1] + ["--gpus", "8"] + common[1:] + ["--png", eight], 480,
                                cwd=repo, env=env, log_path=tmp_path / "r8.log")
    assert rc == 0, f"8 ranks failed after {wall:.0f} s\n" + failure_digest(log8)
    np.testing.assert_array_equal(read_png(one), read_png(eight))
    l1, l8 = last_json(log1), last_json(log8)
    assert l1["config"]["spp"] == l8["config"]["spp"] == 4096 and l8["n_gpus"] == 8
    assert l1["config"]["rays_per_frame"] == l8["config"]["rays_per_frame"] > 4 * 1920 * 1080 * 4096
    assert len(l8["per_rank"]) == 8 and "wide_tree_host_ms" in l8["scene_build"]
    assert l1["config"]["wide_tree"] == l8["config"]["wide_tree"] == "host"   # one method at N = 1 and N = 8
    assert l1["config"]["frames_in_flight"] == l8["config"]["frames_in_flight"] == 1


@pytest.mark.timeout(200)
def test_binding_before_torch_shares_one_hip_runtime(tmp_path):
    """A process that imports the binding before torch: torch must still see the GPU (the binding
    loads torch first, so libpt.so binds torch's HIP runtime instead of a second one), and a
    device tensor and a libpt call work side by side.  Its own process: the suite's has torch."""
    import os
    import sys
    from helpers import run_logged
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, 'path-tracer-cuda-opengl_amd/python'); import ptamd; import torch; "
            "x = torch.ones(64, device='cuda:0'); n = ptamd.device_count(); "
            "print('ok', float(x.sum()), n, torch.cuda.device_count())")
    rc, log, _ = run_logged([sys.executable, "-c", code], 150, cwd=repo, log_path=tmp_path / "bind.log")
    assert rc == 0, log[-3000:]
    line = [ln for ln in log.splitlines() if ln.startswith("ok ")][-1].split()
    assert float(line[1]) == 64.0 and int(line[2]) > 0 and int(line[3]) > 0, line
