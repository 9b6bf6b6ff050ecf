"""Samples-per-pixel sharding over ranks.

Frames (kdpt_render_frames, bench.py): frame f covers global iterations f*spp + 1 .. (f+1)*spp; rank r of N
renders those with (iteration - 1 - f*spp) % N == r (frame_share), and one reduce per frame combines the
ranks' frame images -- weak scaling keeps spp = (per-GPU spp) * N, strong scaling a fixed spp.

One process per GPU.  Rank r of N renders the global iterations 1 + k*N + r (k = 0, 1, ...), so every
iteration-dependent behaviour of the reference -- the RNG seed makeSeededRandomEngine(iter, ...), the
iteration-2 sort, cacherays -- sees the same global iteration number it would on one GPU.  Each rank
accumulates its own float3 sum; the only exchange is one reduce of the W*H*3 sums to rank 0 (RCCL over xGMI
with the "nccl" backend, gloo on CPU).  No data-path collective: the shards are independent.
"""
from __future__ import annotations


def global_iteration(step: int, world: int, rank: int) -> int:
    """1-based global iteration rendered by `rank` at its local step `step`."""
    return 1 + step * world + rank


def shard_iterations(first_step: int, steps: int, world: int, rank: int) -> list:
    """The global iterations of local steps [first_step, first_step + steps) on `rank`."""
    return [global_iteration(s, world, rank) for s in range(first_step, first_step + steps)]


def frame_share(frame: int, spp: int, world: int, rank: int):
    """(first global iteration, count) of `rank`'s share of frame `frame` (stride `world`), as
    kdpt_render_frames renders it."""
    count = (spp - rank + world - 1) // world if rank < spp else 0
    return frame * spp + 1 + rank, count


def frame_iterations(frame: int, spp: int, world: int, rank: int) -> list:
    first, count = frame_share(frame, spp, world, rank)
    return [first + k * world for k in range(count)]


def reduce_image(image, dist, dst: int = 0):
    """Sum the ranks' accumulation buffers into `dst` (in place on `image`, a torch tensor).

    With the "nccl" backend (RCCL) the device buffer is reduced in place over xGMI.  The "gloo" backend
    (CPU rehearsals, and several ranks sharing one GPU, which RCCL refuses) reduces a host copy, which
    is written back into the device buffer on `dst`."""
    if dist is None or not dist.is_initialized():
        return image
    # (one rank: the reduce is a no-op that still runs through the backend, e.g. bench.py --force-dist)
    if image.is_cuda and dist.get_backend() == "gloo":
        host = image.cpu()
        dist.reduce(host, dst=dst, op=dist.ReduceOp.SUM)
        if dist.get_rank() == dst:
            image.copy_(host)
        return image
    dist.reduce(image, dst=dst, op=dist.ReduceOp.SUM)
    return image


def render_shard(tracer, first_step: int, steps: int, world: int, rank: int) -> int:
    """Trace this rank's iterations with a PathTracer (accumulating into its image); returns segments."""
    seg = 0
    for it in shard_iterations(first_step, steps, world, rank):
        tracer.trace_iteration(it)
        seg += tracer.stats().segments
    return seg
