"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 path: stream sharding and the
end-of-run counter / wall-time exchange that bench.py runs over RCCL on the GPU box."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import pkg


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, S=8):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard = pkg().shard
        ids = shard.stream_ids(rank, world, S)
        stats = np.zeros(S, dtype=[(k, np.int64) for k in shard.COUNTERS[1:]])
        stats["current_active_tracks"] = np.arange(S) + 10 * rank
        stats["total_tracks_created"] = 3 + rank
        stats["overflow"] = rank  # bench.py fails the run when the reduced overflow is non-zero
        c = shard.local_counters(100 * S, stats)
        c["live_min_start"] = float(stats["current_active_tracks"].min())  # bench.py's extra key
        out, el = shard.reduce_run(c, 1.0 + rank)
        devs = shard.gather_devices(shard.device_identity(None))
        assert len(devs) == world and len(set(devs)) == world
        # two ranks reporting one device: every rank raises, naming the pair
        try:
            shard.gather_devices("pci 0000:75:00 uuid same" if rank < 2 else f"pci 0000:{rank:02x}:00")
            clash = None
        except RuntimeError as e:
            clash = str(e)
        assert clash is not None and "ranks 0 and 1" in clash
        q.put((rank, ids, [shard.stream_seed(i, S) for i in ids], out, el))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_shard_and_reduce():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    all_ids = [i for r in res for i in r[1]]
    assert sorted(all_ids) == list(range(16)) and len(set(all_ids)) == 16  # disjoint, complete
    assert res[0][2] == list(range(8)) and res[1][2] == [1000 + s for s in range(8)]
    for _, _, _, out, el in res:
        assert el == 2.0  # MAX of the ranks' wall times
        assert out["frames"] == 1600.0
        assert out["current_active_tracks"] == sum(range(8)) * 2 + 10 * 8
        assert out["total_tracks_created"] == 8 * 3 + 8 * 4


def test_single_process_reduce_is_identity():
    shard = pkg().shard
    c = {"frames": 5.0}
    assert shard.reduce_run(c, 0.5) == ({"frames": 5.0}, 0.5)
    with pytest.raises(ValueError):
        shard.stream_ids(2, 2, 8)


def test_config4_one_stream_per_rank_four_ranks():
    """bench.py --config 4: one stream per GPU; 4 gloo ranks stand in for 4 GPUs."""
    world, port = 4, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, 1)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [[0], [1], [2], [3]]
    assert [r[2] for r in res] == [[0], [1000], [2000], [3000]]
    for _, _, _, out, el in res:
        assert el == 4.0 and out["frames"] == 400.0
        assert out["overflow"] == 0 + 1 + 2 + 3
        assert out["current_active_tracks"] == 0 + 10 + 20 + 30
