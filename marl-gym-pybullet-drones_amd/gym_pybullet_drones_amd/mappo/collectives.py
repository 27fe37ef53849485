"""Process groups for the learner's collectives.

Collectives captured in HIP graphs (the update's gradient all-reduce, the
rollout's normaliser moments) run on a process group of their own, so the
RCCL watchdog never polls an eager collective's event while a capture is open
(capture_collectives); eager collectives stay on the default group.
"""
import contextlib

import torch
import torch.distributed as tdist

_CAPTURE_GROUPS = {}   # id(default group) → (the default group, the group of the captured collectives)
_capturing = 0


def collective_group():
    """The process group of a collective issued now: the capture group inside a
    graph capture (capture_collectives), otherwise the default group (None)."""
    if not _capturing:
        return None
    hit = _CAPTURE_GROUPS.get(id(tdist.group.WORLD))
    return hit[1] if hit is not None and hit[0] is tdist.group.WORLD else None


@contextlib.contextmanager
def capture_collectives():
    """Wrap a HIP-graph capture whose collectives must be captured.

    The RCCL watchdog thread of a process group polls the HIP event of every
    eager collective it has not yet retired (a ~100 ms loop), and a poll of an
    event whose stream is capturing aborts the process.  So collectives issued
    inside a capture go to a process group of their own (same ranks, created
    once, its communicator connected eagerly): that group never runs an eager
    collective, captured works are never enqueued to a watchdog, and its
    watchdog has nothing to poll — whatever the default group issued just
    before the capture.  No timing assumption about the watchdog's loop.
    Other backends (gloo) are not graph-capturable: the default group stays."""
    global _capturing
    if tdist.is_available() and tdist.is_initialized() and tdist.get_backend() == "nccl":
        world = tdist.group.WORLD
        hit = _CAPTURE_GROUPS.get(id(world))
        if hit is None or hit[0] is not world:   # (a re-initialised default group: a new capture group)
            # a device id connects the new communicator now, not at its first (captured) collective
            bound = getattr(tdist.group.WORLD, "bound_device_id", None)
            dev = None if bound is not None else torch.device("cuda", torch.cuda.current_device())
            _CAPTURE_GROUPS[id(world)] = (world, tdist.new_group(backend="nccl", device_id=dev))
    _capturing += 1
    try:
        yield
    finally:
        _capturing -= 1
