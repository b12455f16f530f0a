"""Multi-process host plumbing on CPU (gloo, world_size 2) and the TSDF shard ownership map."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from bundlefusion_amd.dist import HostGroup, chunk_owner


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    g = HostGroup(rank, world)
    g.barrier()
    q.put((rank, g.max(1.5 + rank), g.sum(rank + 1.0)))
    g.barrier()
    g.close()


def test_gloo_world2_barrier_max_sum():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, 2.5, 3.0), (1, 2.5, 3.0)]


def test_single_process_group_is_a_noop():
    g = HostGroup(0, 1)
    g.barrier()
    assert g.max(3.0) == 3.0 and g.sum(2.0) == 2.0


@pytest.mark.parametrize("shards", [2, 4, 8])
def test_chunk_ownership_partitions_and_groups_chunks(shards):
    """Every block has exactly one owner; the 8^3-block x 4 mm blocks of one 1 m chunk share it."""
    rng = np.random.default_rng(0)
    owners = [chunk_owner(*rng.integers(-400, 400, 3), 0.004, shards) for _ in range(2000)]
    assert set(owners) <= set(range(shards))
    assert len(set(owners)) == shards  # all shards get work
    # blocks whose corners round to the same chunk centre share an owner
    a = chunk_owner(100, 100, 100, 0.004, shards)  # 3.2 m -> chunk 3
    b = chunk_owner(104, 96, 102, 0.004, shards)  # 3.33 m, 3.07 m, 3.26 m -> same chunk
    assert a == b
