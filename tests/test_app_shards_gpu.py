"""GPU: the FriedLiver application with its TSDF sharded over two ranks (BFAppOptions.shardCount 2, shardIndex
0 / 1), both ranks in one process on one GPU, bundling replicated (no communicator), next to the unsharded
application on the same `.sens` and parameter files.

Every rank decodes and preprocesses every frame and runs the same bundle adjustment, so the ranks must issue
the identical re-integration queue and end with the identical optimized trajectory; their scenes must own
disjoint block sets whose union, blocks and voxels, is the unsharded application's scene, through the
end-of-sequence phase. Outputs: each rank writes the mesh of its own blocks (<stem>.shard<i>of2.ply), shard 0
alone the trajectory .sens and processed.txt. The multi-process form (one app per GPU, RCCL round-robin local
solves + pair-stat all-reduce) is bench.py --sens under torchrun; its host plumbing is tests/test_dist.py."""
import os
import threading

import numpy as np
import pytest

from bundlefusion_amd.app import FriedLiver
from bundlefusion_amd.dist import LoopbackComm, chunk_owner_array
from bundlefusion_amd.params import NORTH_STAR_APP, write_parameter_files
from bundlefusion_amd.recon import FIX_DEINTEGRATE
from bundlefusion_amd.stream import write_synthetic_sens
from oracle_lib import blocks_of

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

F = 105
CHUNK = 0.5
APP = dict(NORTH_STAR_APP, s_hashNumBuckets=1 << 20, s_hashNumSDFBlocks=1 << 18)


@pytest.mark.parametrize("with_comm", [False, True])
def test_two_shard_apps_partition_the_unsharded_app(tmp_path, with_comm):
    """with_comm: the shard apps also share an in-process loopback communicator (bf_comm_create_loopback)
    and run from their own threads, so they take the multi-GPU bundling paths (round-robin local solves
    with the broadcast, the pair-stat all-reduce, own-submap cache frames) and must still match."""
    d = str(tmp_path)
    sens = os.path.join(d, "synthetic.sens")
    write_synthetic_sens(sens, F, 640, 480)
    pa, pb = write_parameter_files(d, APP, {}, sens=sens)
    apps, outs = [], []
    for count, index in ((1, 0), (2, 0), (2, 1)):
        out = os.path.join(d, f"out{count}{index}")
        os.makedirs(out)
        outs.append(out)
        apps.append(FriedLiver(pa, pb, output_dir=out, async_bundling=0, record_ops=True, shard=(count, index),
                               shard_chunk=CHUNK))
    if not with_comm:
        for f in range(F):
            for a in apps:
                assert a.step()
        res = [a.finish() for a in apps]
    else:
        comms = LoopbackComm.group(2)
        apps[1].set_comm(comms[0])
        apps[2].set_comm(comms[1])
        for f in range(F):
            assert apps[0].step()
        res = [apps[0].finish(), None, None]
        errors = []

        def rank(i):
            try:
                for f in range(F):
                    assert apps[i].step()
                res[i] = apps[i].finish()
            except Exception as e:  # noqa: BLE001 — reported below with its rank
                errors.append((i, repr(e)))

        threads = [threading.Thread(target=rank, args=(i,)) for i in (1, 2)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=500)
        assert not any(t.is_alive() for t in threads), "a rank did not finish"
        assert not errors, errors
    for k in ("pastEndFrames", "globalSolves", "localSolved", "denseSolve", "queueDrained"):
        assert res[1]["end"][k] == res[2]["end"][k] == res[0]["end"][k], k
    assert res[0]["end"]["denseSolve"] == 1
    full, s0, s1 = (a.recon for a in apps)
    ref = full.op_log()
    assert sum(1 for k, *_ in ref if k == FIX_DEINTEGRATE) > 0
    for rc in (s0, s1):
        log = rc.op_log()
        assert len(log) == len(ref)
        for (k0, f0, o0, n0), (k1, f1, o1, n1) in zip(ref, log):
            assert (k0, f0) == (k1, f1)
            np.testing.assert_array_equal(o0, o1)
            np.testing.assert_array_equal(n0, n1)
        np.testing.assert_array_equal(rc.optimized_trajectory(), full.optimized_trajectory())
        np.testing.assert_array_equal(rc.trajectory(F), full.trajectory(F))
    fh, _, _, fv = full.export()
    fb = blocks_of(fh)
    union = {}
    for i, rc in enumerate((s0, s1)):
        h, _, _, v = rc.export()
        b = blocks_of(h)
        assert b and not (set(b) & set(union)), "a block is owned by both ranks"
        assert np.all(chunk_owner_array(np.array(sorted(b)), APP["s_SDFVoxelSize"], 2, chunk=CHUNK) == i)
        for k, ptr in b.items():
            union[k] = v[ptr:ptr + 512]
    assert set(union) == set(fb) and len(fb) > 1000
    for k, ptr in fb.items():
        a, b = fv[ptr:ptr + 512], union[k]
        assert np.array_equal(a["sdf"].view(np.uint32), b["sdf"].view(np.uint32)), k
        assert np.array_equal(a["weight"], b["weight"]), k
        assert np.array_equal(a["color"], b["color"]), k
    # outputs: a mesh per shard (their triangles add up to the unsharded mesh's within the shard seams),
    # the trajectory .sens and processed.txt from shard 0 only
    assert os.path.exists(os.path.join(outs[0], "synthetic.ply"))
    assert os.path.exists(os.path.join(outs[1], "synthetic.shard0of2.ply"))
    assert os.path.exists(os.path.join(outs[2], "synthetic.shard1of2.ply"))
    assert os.path.exists(os.path.join(outs[1], "synthetic.optimized.sens"))
    assert os.path.exists(os.path.join(outs[1], "processed.txt"))
    assert not os.path.exists(os.path.join(outs[2], "synthetic.optimized.sens"))
    assert not os.path.exists(os.path.join(outs[2], "processed.txt"))
    assert res[1]["meshTriangles"] > 0 and res[2]["meshTriangles"] > 0
    for a in apps:
        a.close()
    if with_comm:
        for c in comms:
            c.close()
