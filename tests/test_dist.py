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


def _id_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    g = HostGroup(rank, world)
    uid = bytes(np.random.default_rng(7).integers(0, 256, 128, dtype=np.uint8)) if rank == 0 else None
    got = g.broadcast_bytes(uid, 128)
    q.put((rank, got))
    g.close()


def test_gloo_world2_unique_id_handoff():
    """The RCCL unique id drawn on rank 0 reaches every rank unchanged (dist.Comm's hand-off)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_id_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = bytes(np.random.default_rng(7).integers(0, 256, 128, dtype=np.uint8))
    assert res[0] == res[1] == expect


def _pair_worker(rank, world, port, q):
    """One rank of the sharded global solve's exchange, on CPU: build the statistics of the pairs
    p % world == rank (zeros elsewhere, k_pair_stats' partition), sum over ranks (gloo standing in
    for the RCCL all-reduce) and report the result."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import torch
    import torch.distributed as dist
    from ba_problem import make_problem
    from oracle_ba import pose_to_matrix
    from oracle_pairs import pair_stats
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    g = HostGroup(rank, world)
    prob = make_problem(K=8, max_per_pair=10, outliers=0.02, seed=3)
    T = np.stack([pose_to_matrix(prob["rot"][k], prob["trans"][k]) for k in range(8)])
    full = pair_stats(prob["corr"], T)
    keys = sorted(full)
    mine = np.stack([full[k] + 0.0 if p % world == rank else np.zeros(28) for p, k in enumerate(keys)])
    t = torch.from_numpy(mine.copy())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    q.put((rank, t.numpy().copy(), np.stack([full[k] for k in keys])))
    g.close()


def test_gloo_world2_pair_shard_exchange_is_exact():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_pair_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        np.testing.assert_array_equal(res[r][0], res[r][1])


def test_chunk_owner_array_matches_scalar_mirror():
    from bundlefusion_amd.dist import chunk_owner_array
    rng = np.random.default_rng(1)
    b = rng.integers(-2000, 2000, (3000, 3))
    for G in (2, 4, 8):
        got = chunk_owner_array(b, 0.004, G)
        want = [chunk_owner(int(x), int(y), int(z), 0.004, G) for x, y, z in b]
        np.testing.assert_array_equal(got, want)


def test_shard_balance_report_shape():
    from types import SimpleNamespace
    from bundlefusion_amd.dist import shard_balance
    rng = np.random.default_rng(2)
    b = rng.integers(-100, 100, (5000, 3))
    cam = SimpleNamespace(fx=577.87, fy=577.87, mx=319.5, my=239.5, imageWidth=640, imageHeight=480,
                          sensorDepthWorldMin=0.1, sensorDepthWorldMax=4.0)
    T = np.eye(4)
    r = shard_balance(b, 0.004, [T], cam, (2, 4))
    assert r["blocks"] == 5000 and sum(r["G2"]["stored"]) == 5000 and sum(r["G4"]["stored"]) == 5000
    assert r["G2"]["stored_max_over_mean"] >= 1.0


def _agree_worker(rank, world, port, paths, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from bundlefusion_amd.dist import input_digest
    g = HostGroup(rank, world)
    try:
        g.agree("the .sens and parameter files", input_digest(paths[rank]))
        q.put((rank, "ok"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    g.close()


@pytest.mark.parametrize("same", [True, False])
def test_app_ranks_agree_on_their_inputs(tmp_path, same):
    """bench.py --sens under torchrun: every rank opens the same .sens and parameter files (the replicated
    bundle adjustment and the collectives' sizes depend on them). The ranks compare input digests over gloo;
    a rank with a different file fails the job on every rank."""
    files = []
    for r in range(2):
        p = tmp_path / f"rank{r}.sens"
        p.write_bytes(b"SENS" + bytes(range(256)) * 64 + (b"" if same or r == 0 else b"x"))
        prm = tmp_path / f"params{r}.txt"
        prm.write_text("s_SDFVoxelSize = 0.004f;\n")
        files.append([str(p), str(prm)])
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, files, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if same:
        assert res == [(0, "ok"), (1, "ok")]
    else:
        assert all("ranks disagree" in m for _, m in res)
        assert "differs from rank 0" in res[1][1] and "differs" not in res[0][1]
