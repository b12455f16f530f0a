"""GPU: the reconstruction loop with the TSDF sharded over two ranks, both ranks
in one process on one GPU (bf_recon instances with shardCount 2, shardIndex 0 / 1, bundling
replicated).

Every rank sees every frame and runs the same bundle adjustment, so the ranks must issue the
identical re-integration queue (the same op list: kind, frame, old and new transform, in order) and
end with the identical trajectory; their scenes must own disjoint block sets whose union, blocks
and voxel payload, is the unsharded loop's scene. This is the multi-GPU TSDF path minus the
process boundary (one process per GPU adds only the host barrier, tests/test_dist.py).
"""
import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd.abi import BFSceneOptions
from bundlefusion_amd.dist import chunk_owner_array
from bundlefusion_amd.recon import FIX_DEINTEGRATE, Recon, recon_options
from bundlefusion_amd.stream import SyntheticStream
from oracle_lib import blocks_of

pytestmark = pytest.mark.gpu


def test_two_shard_loops_partition_the_unsharded_loop():
    F, VOX, CHUNK = 60, 0.01, 0.5
    # one seeded stream per rank, as each GPU holds its own copy of the inputs: the loop edits its
    # correspondences in place (max-residual removal, invalid-submap marking)
    streams = [SyntheticStream(F, width=160, height=120) for _ in range(3)]
    st = streams[0]
    params = bfa.hash_params(voxel_size=VOX, num_buckets=1 << 16, num_blocks=1 << 15)
    K = st.K
    loops = []
    for (count, index), sti in zip([(1, 0), (2, 0), (2, 1)], streams):
        # the default bundling config, dense local term included: every BA reduction is a fixed-order sum
        # (no float atomics), so replicated solves on every rank are bit-identical
        opts = recon_options(F, recordOps=1, cacheWidth=80, cacheHeight=60, cacheIntrinsics=st.cache_intrinsics,
                             maxGlobalCorr=max(1000, 25 * K * (K - 1) // 2), maxKeyframes=K + 1, asyncBundling=0)
        so = BFSceneOptions()
        so.shardCount, so.shardIndex, so.shardChunk = count, index, CHUNK
        rc = Recon(params, st.cam, opts, so)
        sti.attach(rc)
        loops.append(rc)
    for f in range(F):
        for rc in loops:
            rc.process_frame(f)
    ends = [rc.end_sequence() for rc in loops]  # the past-the-end phase, dense solve included
    keys = ("pastEndFrames", "globalSolves", "localSolved", "denseSolve", "queueDrained")
    assert ends[0]["denseSolve"] == 1 and all([e[k] for k in keys] == [ends[0][k] for k in keys] for e in ends[1:])
    for rc in loops:
        rc.synchronize()
    full, s0, s1 = loops
    # identical queue op lists and trajectories on every rank
    ref = full.op_log()
    assert sum(1 for k, *_ in ref if k == FIX_DEINTEGRATE) > 0  # some de-integrations happened
    for rc in (s0, s1):
        log = rc.op_log()
        assert len(log) == len(ref)
        for (k0, f0, o0, n0), (k1, f1, o1, n1) in zip(ref, log):
            assert (k0, f0) == (k1, f1)
            np.testing.assert_array_equal(o0, o1)
            np.testing.assert_array_equal(n0, n1)
        np.testing.assert_array_equal(rc.trajectory(F), full.trajectory(F))
    # disjoint block sets whose union is the unsharded scene, voxel payload bit-identical
    fh, _, _, fv = full.export()
    fb = blocks_of(fh)
    union = {}
    for i, rc in enumerate((s0, s1)):
        h, _, _, v = rc.export()
        b = blocks_of(h)
        assert b and not (set(b) & set(union)), "a block is owned by both ranks"
        owners = chunk_owner_array(np.array(sorted(b)), VOX, 2, chunk=CHUNK)
        assert np.all(owners == i)  # the host mirror of owned() agrees with the device
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
