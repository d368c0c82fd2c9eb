"""One rank of the fail-fast test (tests/test_distributed.py::test_one_failing_rank_ends_every_rank).

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python failfast_worker.py <mode> <timeout_s> <watchdog_s>

The ranks run bench.py's multi-rank sequence in miniature through ptdist (init with a collective
timeout, phases, guarded work, agreed checks, the frame gather to rank 0); rank 1 fails in phase
"frame check" as `mode` says: `raise` (an exception), `mismatch` (a failed check, agreed by all
ranks), `hang` (stops responding), or `none` (no failure)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "path-tracer-cuda-opengl_amd", "python"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ptdist  # noqa: E402


def main() -> None:
    mode, timeout_s, watchdog_s = sys.argv[1], float(sys.argv[2]), float(sys.argv[3])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ptdist.init("gloo", rank, world, timeout_s=timeout_s, watchdog_s=watchdog_s)
    with ptdist.guarded():
        ptdist.phase("frame check")
        ok = True
        if rank == 1:
            if mode == "raise":
                raise RuntimeError("frame differs from the reference-order frame")
            if mode == "hang":
                time.sleep(10 ** 6)
            ok = mode != "mismatch"
        bad = ptdist.agree(ok)
        if bad:
            raise SystemExit(3)
        ptdist.phase("gather")
        buf = torch.full((64,), float(rank))
        out = ptdist.gather_to_root(buf, world, rank)
        if rank == 0:
            assert out.view(world, -1)[:, 0].tolist() == [float(r) for r in range(world)]
        dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank} ok", flush=True)


if __name__ == "__main__":
    main()
