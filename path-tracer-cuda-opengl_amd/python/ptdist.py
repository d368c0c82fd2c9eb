"""Row-stripe partition of a frame across ranks and the gather that reassembles it.

Stripe s (rows [s*stripe, (s+1)*stripe)) belongs to rank s % world, which interleaves cheap
(sky) and expensive (geometry) rows across GPUs.  Every rank renders its rows packed in
order into a buffer padded to `max_rows(...)` rows (fp32 RGB, or RGBA8 quantised on the device:
4 instead of 12 bytes per pixel on the wire), one gather to rank 0 (`gather_to_root`: RCCL over
xGMI on the GPU box, gloo in the CPU tests; SURVEY §8(e)'s ncclGather) concatenates the buffers
there, and `assemble` un-permutes them.
The RNG is keyed by the GLOBAL pixel index (curand_init(seed, pixel, 0), main.cu:268), so
the assembled frame is bit-identical to a single-GPU render.

Fail-fast (the reference runs one process, so it has no counterpart): `init` gives every
collective a timeout, `phase` names what a rank is doing (and re-arms an optional stack-dump
watchdog), `guarded` turns any exception on a rank into a one-line report naming the rank and
phase plus an immediate non-zero exit, and `agree` lets all ranks learn that some rank's check
failed so that all of them exit with the same status.  A rank that dies leaves its peers blocked
in a collective at most `timeout_s`: gloo raises at once when the peer's sockets close (or at the
timeout), RCCL's watchdog aborts the communicator and ends the process at the timeout.
"""
from __future__ import annotations

import datetime
import faulthandler
import os
import sys
import time
import traceback
from contextlib import contextmanager

import numpy as np

_STATE = {"rank": 0, "world": 1, "phase": "start", "watchdog_s": 0.0, "backend": None, "t0": time.monotonic()}


def init(backend: str, rank: int, world: int, device=None, timeout_s: float = 120.0, watchdog_s: float = 0.0) -> None:
    """init_process_group with a collective timeout (`timeout_s`) and, if watchdog_s > 0, a
    per-phase watchdog: a rank that spends longer than watchdog_s in one phase dumps every
    thread's Python stack to stderr and exits 1 (faulthandler), so a hang names its rank and phase."""
    import torch.distributed as dist
    _STATE.update(rank=rank, world=world, watchdog_s=float(watchdog_s), backend=backend)
    kw = {"timeout": datetime.timedelta(seconds=timeout_s)}
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    phase("init_process_group")
    dist.init_process_group(backend, **kw)


def tag() -> str:
    return f"[rank {_STATE['rank']}/{_STATE['world']}]"


def phase(name: str) -> None:
    """Record the rank's current phase (reported on failure; PT_DIST_TRACE=1 prints each one) and
    re-arm the watchdog for it."""
    _STATE["phase"] = name
    if os.environ.get("PT_DIST_TRACE") == "1":
        sys.stderr.write(f"{tag()} phase: {name} (t = {time.monotonic() - _STATE['t0']:.1f} s)\n")
        sys.stderr.flush()
    if _STATE["watchdog_s"] > 0:
        sys.stderr.flush()
        faulthandler.dump_traceback_later(_STATE["watchdog_s"], exit=True)


def fail(msg: str, code: int = 1) -> None:
    """Report `msg` with the rank and phase on stderr and end the process NOW (os._exit: no
    interpreter shutdown, no process-group teardown that could wait on the peers)."""
    try:
        faulthandler.cancel_dump_traceback_later()
        sys.stderr.write(f"{tag()} FAILED in phase '{_STATE['phase']}': {msg}\n")
        sys.stderr.flush()
        sys.stdout.flush()
    finally:
        os._exit(code)


@contextmanager
def guarded(code: int = 1):
    """Run a rank's work; any exception (or a non-zero SystemExit) ends this rank at once with a
    non-zero status and a report naming the rank and phase, instead of leaving it to unwind while
    its peers wait in a collective."""
    try:
        yield
    except SystemExit as e:
        if e.code in (0, None):
            raise
        # (SystemExit("message"): a failed check, status 3)
        fail(f"exit {e.code}" if isinstance(e.code, int) else str(e.code), e.code if isinstance(e.code, int) else 3)
    except BaseException as e:   # noqa: BLE001 (every failure must end the rank)
        fail("".join(traceback.format_exception(type(e), e, e.__traceback__)).rstrip(), code)
    finally:
        if _STATE["watchdog_s"] > 0:
            faulthandler.cancel_dump_traceback_later()


def agree(ok: bool, device="cpu") -> list:
    """Collective: every rank passes its own check result and gets the sorted list of ranks whose
    check failed (empty: all passed).  One all_reduce of a world-sized flag vector."""
    import torch
    import torch.distributed as dist
    flags = torch.zeros(_STATE["world"], dtype=torch.int32, device=device)
    flags[_STATE["rank"]] = 0 if ok else 1
    dist.all_reduce(flags)
    return [int(r) for r in torch.nonzero(flags.cpu()).flatten()]


def stripe_rows(height: int, stripe: int, world: int, rank: int) -> np.ndarray:
    r = np.arange(height)
    return r[(r // stripe) % world == rank].astype(np.int32)


def max_rows(height: int, stripe: int, world: int) -> int:
    stripes = (height + stripe - 1) // stripe
    return ((stripes + world - 1) // world) * stripe


def gather_to_root(local, world: int, rank: int, out=None):
    """Gather every rank's padded stripe buffer (a flat tensor, same shape on every rank) into
    `out` on rank 0 -- shape (world * local.numel(),), allocated if None -- and return it there
    (None on the other ranks).  One collective per frame; only rank 0 receives (the frame is
    written by rank 0), unlike an all-gather that would send every frame to every rank."""
    import torch
    import torch.distributed as dist
    if rank == 0:
        if out is None:
            out = torch.empty((world * local.numel(),), dtype=local.dtype, device=local.device)
        dist.gather(local, list(out.view(world, -1).unbind(0)), dst=0)
        return out
    dist.gather(local, None, dst=0)
    return None


def assemble(gathered, height: int, width: int, stripe: int, world: int, channels: int = 3):
    """gathered: array/tensor of shape (world, max_rows, width, channels) -> (height, width, channels).
    channels = 3 for fp32 RGB frames, 4 for device-quantised RGBA8 frames (PT_OUT_RGBA8)."""
    mr = max_rows(height, stripe, world)
    g = gathered.reshape(world, mr, width, channels)
    try:  # torch tensor
        import torch
        if isinstance(g, torch.Tensor):
            img = torch.empty((height, width, channels), dtype=g.dtype, device=g.device)
            for r in range(world):
                rows = torch.as_tensor(stripe_rows(height, stripe, world, r), device=g.device, dtype=torch.long)
                img[rows] = g[r, : len(rows)]
            return img
    except ImportError:
        pass
    img = np.empty((height, width, channels), dtype=g.dtype)
    for r in range(world):
        rows = stripe_rows(height, stripe, world, r)
        img[rows] = g[r, : len(rows)]
    return img
