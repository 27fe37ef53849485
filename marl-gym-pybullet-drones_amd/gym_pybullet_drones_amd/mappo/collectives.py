"""Process groups for the learner's collectives.

The RCCL watchdog thread of a process group polls the HIP end event of every
eager collective it has not yet retired (a ~100 ms loop); a poll of an event
last recorded in a stream that is capturing aborts the process
(hipErrorCapturedEvent).  Two rules keep every such poll off capturing streams,
with no timing assumption:
* collectives captured in HIP graphs (the update's gradient all-reduce, the
  rollout's normaliser moments) run on a process group of their own
  (capture_collectives): captured works are never enqueued to a watchdog, and
  that group never runs an eager collective;
* eager collectives (all_reduce / broadcast below) are issued async and waited
  for: their events are recorded on the default group's internal stream, which
  no capture ever joins — not on the caller's current stream, which may be a
  pooled side stream that a later capture reuses (a synchronous collective
  records its event there; the round-6 bench aborted so).
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


def all_reduce(t):
    """Sum-all-reduce of t as the learner issues it: inside a capture on the
    capture group (captured), otherwise async on the default group and waited
    for (see the module docstring)."""
    if _capturing:
        tdist.all_reduce(t, group=collective_group())
    else:
        tdist.all_reduce(t, async_op=True).wait()


def broadcast(t, src=0):
    """Eager broadcast from rank src (async + wait: the event on the group's own stream)."""
    tdist.broadcast(t, src, async_op=True).wait()
