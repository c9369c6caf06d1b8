"""Face sharding across ranks (one process per GPU) and the single result exchange.

SURVEY.md §8(e): faces are independent (the reference loops them, src/FaceForest.cpp:175-180) and
the only shared state is the read-only model, so each rank owns a contiguous block of
ceil(N / world) faces, runs the whole path on it with no data-path collective, and the
`ffd_face` records (FACE_RECORD_BYTES each) are gathered to one rank in one collective.
With the "nccl" backend (RCCL over xGMI on ROCm) the gather moves device buffers; with "gloo"
(tests, CPU) host buffers.
"""
import torch
import torch.distributed as dist

from . import FACE_RECORD_BYTES


def shard_bounds(n_faces, world, rank):
    """Contiguous block [lo, hi) of rank `rank` among `world` (ceil(N/world) faces each; the
    last ranks may be short or empty)."""
    if world < 1 or not 0 <= rank < world or n_faces < 0:
        raise ValueError("bad shard arguments")
    per = -(-n_faces // world)
    lo = min(n_faces, rank * per)
    return lo, min(n_faces, lo + per)


def gather_records(local, n_faces, dst=0, group=None):
    """Gather every rank's face records (uint8 tensor of n_local * FACE_RECORD_BYTES, the shard
    of shard_bounds order) into one uint8 tensor of n_faces * FACE_RECORD_BYTES on `dst`
    (None on other ranks).  Shards are padded to the common ceil(N/world) size so one
    fixed-size gather serves ragged splits."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = -(-n_faces // world)
    rec = FACE_RECORD_BYTES
    lo, hi = shard_bounds(n_faces, world, rank)
    if local.dtype != torch.uint8 or local.numel() != (hi - lo) * rec:
        raise ValueError("local records do not match this rank's shard")
    buf = torch.zeros(per * rec, dtype=torch.uint8, device=local.device)
    buf[: local.numel()] = local
    if rank == dst:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.gather(buf, gather_list=parts, dst=dst, group=group)
        out = torch.cat([p[: (shard_bounds(n_faces, world, r)[1] - shard_bounds(n_faces, world, r)[0]) * rec]
                         for r, p in enumerate(parts)])
        return out
    dist.gather(buf, dst=dst, group=group)
    return None
