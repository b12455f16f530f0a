"""GPU: the multi-rank reconstruction loop with its communicator, 2 and 3 ranks on one GPU.

Each rank is a bf_recon with TSDF shard r of G and a communicator of one in-process loopback group
(bf_comm_create_loopback), driven from its own host thread, as one process per GPU drives its loop. With
the communicator the ranks take the multi-GPU code paths: local solves round-robin by submap with the
solved poses broadcast from the owner, the global solve's image-pair statistics built on the owning rank
and summed over ranks once per GN iteration, cache frames only for the rank's own submaps and the
keyframes. The ranks must issue the identical re-integration queue and end with the trajectory of the
unsharded loop without a communicator, bit for bit (the all-reduce adds each pair's blocks to exact
zeros; the broadcast copies the owner's poses), and their scenes must partition the unsharded scene.
RCCL itself needs one GPU per rank: its calls are the same two collectives (comm.cpp), covered on one
rank by test_rccl_single_rank_exchange and across ranks by the driver's multi-GPU run."""
import threading

import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd.abi import BFSceneOptions
from bundlefusion_amd.dist import LoopbackComm, chunk_owner_array
from bundlefusion_amd.recon import FIX_DEINTEGRATE, Recon, recon_options
from bundlefusion_amd.stream import SyntheticStream
from oracle_lib import blocks_of

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]


@pytest.mark.parametrize("world,async_bundling,lag", [(2, 0, 0), (2, 1, 20), (3, 1, 20)])
def test_rank_loops_with_communicator_match_the_unsharded_loop(world, async_bundling, lag):
    F, VOX, CHUNK = 80, 0.01, 0.5
    streams = [SyntheticStream(F, width=160, height=120, cache_source="loop") for _ in range(world + 1)]
    st = streams[0]
    params = bfa.hash_params(voxel_size=VOX, num_buckets=1 << 16, num_blocks=1 << 15)
    K = st.K
    loops = []
    for (count, index), sti in zip([(1, 0)] + [(world, r) for r in range(world)], streams):
        opts = recon_options(F, recordOps=1, cacheWidth=80, cacheHeight=60, cacheIntrinsics=st.cache_intrinsics,
                             maxGlobalCorr=max(1000, 25 * K * (K - 1) // 2), maxKeyframes=K + 1,
                             asyncBundling=async_bundling, resultLag=lag)
        so = BFSceneOptions()
        so.shardCount, so.shardIndex, so.shardChunk = count, index, CHUNK
        rc = Recon(params, st.cam, opts, so)
        sti.attach(rc)
        loops.append(rc)
    full, ranks = loops[0], loops[1:]
    comms = LoopbackComm.group(world)
    for rc, c in zip(ranks, comms):
        rc.set_comm(c)

    for f in range(F):  # the reference: one loop, no communicator
        full.process_frame(f)
    end_full = full.end_sequence()
    full.synchronize()

    results, errors = {}, []

    def rank(i, rc):
        try:
            for f in range(F):
                rc.process_frame(f)
            results[i] = rc.end_sequence()
            rc.synchronize()
        except Exception as e:  # noqa: BLE001 — re-raised below with its rank
            errors.append((i, repr(e)))

    threads = [threading.Thread(target=rank, args=(i, rc)) for i, rc in enumerate(ranks)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=540)
    assert not any(t.is_alive() for t in threads), "a rank did not finish"
    assert not errors, errors

    keys = ("pastEndFrames", "globalSolves", "localSolved", "denseSolve", "queueDrained")
    assert end_full["denseSolve"] == 1
    for i in range(world):
        assert [results[i][k] for k in keys] == [end_full[k] for k in keys]
    ref = full.op_log()
    assert sum(1 for k, *_ in ref if k == FIX_DEINTEGRATE) > 0
    for rc in ranks:
        log = rc.op_log()
        assert len(log) == len(ref)
        for (k0, f0, o0, n0), (k1, f1, o1, n1) in zip(ref, log):
            assert (k0, f0) == (k1, f1)
            np.testing.assert_array_equal(o0, o1)
            np.testing.assert_array_equal(n0, n1)
        np.testing.assert_array_equal(rc.trajectory(F), full.trajectory(F))
    # each rank solved only its own local submaps (round-robin), together all of them
    s_full, s_ranks = full.stats(), [rc.stats() for rc in ranks]
    assert all(s["localSolves"] > 0 for s in s_ranks)
    assert sum(s["localSolves"] for s in s_ranks) == s_full["localSolves"]
    assert all(s["globalSolves"] == s_full["globalSolves"] for s in s_ranks)

    fh, _, _, fv = full.export()
    fb = blocks_of(fh)
    union = {}
    for i, rc in enumerate(ranks):
        h, _, _, v = rc.export()
        b = blocks_of(h)
        assert b and not (set(b) & set(union)), "a block is owned by two ranks"
        assert np.all(chunk_owner_array(np.array(sorted(b)), VOX, world, chunk=CHUNK) == i)
        for k, ptr in b.items():
            union[k] = v[ptr:ptr + 512]
    assert set(union) == set(fb) and len(fb) > 500
    for k, ptr in fb.items():
        a, b = fv[ptr:ptr + 512], union[k]
        assert np.array_equal(a["sdf"].view(np.uint32), b["sdf"].view(np.uint32)), k
        assert np.array_equal(a["weight"], b["weight"]), k
        assert np.array_equal(a["color"], b["color"]), k
    for rc in loops:
        rc.close()
    for c in comms:
        c.close()


def test_loopback_collective_a_rank_skips_fails_loudly():
    """A collective that one rank never joins must not hand back sums: its wait ends at the group's timeout
    and the call that synchronises it fails (bf_comm_allreduce_sum_f64 checks the group's error word after
    the stream), as does every later collective of the group; the ranks that did join get no success either."""
    comms = LoopbackComm.group(2, timeout_ms=300)
    try:
        d = bfa.DeviceArray.from_host(np.arange(8, dtype=np.float64))
        with pytest.raises(bfa.BFError, match="did not reach a collective"):
            comms[0].allreduce_sum_f64(d)  # rank 1 never arrives
        with pytest.raises(bfa.BFError, match="did not reach a collective"):
            comms[1].allreduce_sum_f64(d)  # the group stays failed
    finally:
        for c in comms:
            c.close()
