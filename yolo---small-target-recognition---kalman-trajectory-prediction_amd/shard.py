"""Stream sharding across GPUs and the end-of-run exchange.

Independent video streams shard one group per GPU: rank r owns streams
[r * S, (r + 1) * S) with their own detector replica and tracker state, so the data path has
no collective at all (weak scaling).  The only exchange is at the end of the run: one
all_reduce(SUM) of the run counters (the tracker's get_statistics() fields,
kalman/enhanced_multi_target_tracker.py:288-304, plus frames processed) and one
all_reduce(MAX) of the wall time, over RCCL ("nccl" backend on ROCm) on the GPU box or gloo
on CPU.  Messages are tens of bytes: latency-bound, not xGMI-bandwidth-bound.
"""
from __future__ import annotations

import numpy as np
import torch

COUNTERS = ("frames", "frame_count", "total_tracks_created", "total_tracks_terminated", "current_active_tracks",
            "long_term_predictions", "successful_recoveries", "overflow")


def stream_ids(rank: int, world: int, streams_per_rank: int) -> list[int]:
    """Global stream indices owned by `rank` (contiguous block, disjoint across ranks)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return [rank * streams_per_rank + s for s in range(streams_per_rank)]


def stream_seed(stream_id: int, streams_per_rank: int) -> int:
    """Scene seed of a global stream: numpy default_rng(seed) per stream; rank 0's
    streams get seeds 0..S-1 (seed 0 = the training run's seed, args.yaml)."""
    rank, s = divmod(stream_id, streams_per_rank)
    return 1000 * rank + s


def local_counters(frames_done: int, stats: np.ndarray) -> dict:
    """Run counters of this rank from the per-stream tracker stats (yk_tracker_stats rows)."""
    out = {"frames": float(frames_done)}
    for k in COUNTERS[1:]:
        out[k] = float(np.asarray(stats[k]).sum())
    return out


def device_identity(device=None) -> str:
    """This rank's physical device: the GPU's PCI address (domain:bus:device) and uuid, read
    from the HIP device properties; ``cpu:<pid>`` for a CPU (gloo) rank."""
    if device is None or torch.device(device).type != "cuda":
        import os

        return f"cpu:{os.getpid()}"
    p = torch.cuda.get_device_properties(torch.device(device))
    return f"pci {p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x} uuid {p.uuid}"


def gather_devices(ident: str) -> list[str]:
    """Every rank's device_identity(), in rank order, checked to be pairwise distinct (one
    process per GPU: two ranks on one device would share its CUs and HBM, and a scaling line
    measured that way is not an N-GPU number).  Raises RuntimeError naming the ranks that
    collide.  [ident] when torch.distributed is not initialised."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [ident]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, ident)
    seen = {}
    for r, d in enumerate(out):
        if d in seen:
            raise RuntimeError(f"ranks {seen[d]} and {r} run on the same device ({d}): launch one process per GPU")
        seen[d] = r
    return out


def reduce_run(counters: dict, elapsed: float, device=None) -> tuple[dict, float]:
    """End-of-run exchange: SUM of the counters and MAX of the wall time over all ranks.
    Identity when torch.distributed is not initialised (single process)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return dict(counters), float(elapsed)
    dev = device if device is not None else torch.device("cpu")
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    keys = list(counters)
    c = torch.tensor([float(counters[k]) for k in keys], dtype=torch.float64, device=dev)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    vals = c.cpu().tolist()
    return {k: v for k, v in zip(keys, vals)}, float(t.item())
