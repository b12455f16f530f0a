"""GPU parity of the HIP voxel-hash TSDF against the CPU oracle (bit-exact).

Integer state (block set, computeHashPos bucket of every entry, heap free count) and the
voxel payload (sdf bits, weight, colour) must be identical; slot placement and heap
pointers are compared through the block coordinates (the reference assigns them in a
racy order, CUDASceneRepHashSDF.h:335-348)."""
import numpy as np
import pytest

import bundlefusion_amd as bfa
from tsdf_compare import Pair, render_frames

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scene():
    return bfa.synth_scene(0)


def small_cam():
    return bfa.depth_camera(160, 120, fx=577.87 / 4, fy=577.87 / 4)


def test_single_frame_parity(scene):
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 17, num_blocks=1 << 16)
    pair = Pair(p, cam)
    (T, d, c), = render_frames(scene, cam, [0])
    pair.integrate(0, T, d, c)
    n = pair.compare()
    assert n > 500
    assert pair.gpu.getHeapFreeCount() == pair.ora.getHeapFreeCount()
    assert pair.gpu.numVisible() == pair.ora.numOccupied()
    assert pair.gpu.errorFlags() == 0


def test_sequence_integrate_deintegrate_gc(scene):
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 17, num_blocks=1 << 16)
    pair = Pair(p, cam)
    frames = render_frames(scene, cam, [0, 7, 14, 21, 28])
    for k, (T, d, c) in enumerate(frames):
        pair.integrate(k, T, d, c)
        pair.gc()
        pair.compare()
    # re-integration: de-integrate frames 1 and 3 with their old pose, integrate with a moved pose
    for k in (1, 3):
        T, d, c = frames[k]
        pair.integrate(k, T, d, c, deint=True)
        T2 = T.copy()
        T2[0, 3] += 0.01
        pair.integrate(k, T2, d, c)
        pair.gc()
        pair.compare()
    # de-integrate everything: all voxels return to weight 0 and GC frees every block
    for k, (T, d, c) in enumerate(frames):
        if k in (1, 3):
            T = T.copy()
            T[0, 3] += 0.01
        pair.integrate(k, T, d, c, deint=True)
        pair.gc()
    pair.compare()


def _off_bucket_entries(params, h):
    from oracle_lib import bucket_of
    occ = np.nonzero(h["ptr"] != -2)[0]
    return sum(1 for i in occ if i // 4 != bucket_of((h[i]["x"], h[i]["y"], h[i]["z"]), params.hashNumBuckets))


def test_collision_lists(scene):
    """~1 block per bucket: full buckets spill into collision lists (serial overflow insert)
    and GC deletes list entries; every block stays reachable, so the sets must match exactly."""
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.02, num_buckets=1021, num_blocks=4096, max_list=7)
    pair = Pair(p, cam)
    frames = render_frames(scene, cam, [0, 20])
    for k, (T, d, c) in enumerate(frames):
        pair.integrate(k, T, d, c)
        pair.gc()
        pair.compare()
    gh, _, _, _ = pair.gpu.export()
    assert _off_bucket_entries(p, gh) > 0, "no collision list was exercised"
    T, d, c = frames[0]
    pair.integrate(0, T, d, c, deint=True)
    pair.gc()
    pair.compare()


def test_overloaded_hash_keeps_invariants(scene):
    """4x overload: which blocks fit in the 7-probe window is order-dependent (in the reference
    too), so only the debugHash invariants and the DDA block superset are checked."""
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.02, num_buckets=257, num_blocks=4096, max_list=7)
    big = bfa.hash_params(voxel_size=0.02, num_buckets=1 << 16, num_blocks=4096)
    from oracle_lib import OracleScene, blocks_of, check_hash_invariants
    g = bfa.SceneRepHashSDF(p)
    ref = OracleScene(big)
    (T, d, c), = render_frames(scene, cam, [0])
    g.integrate(T, bfa.DeviceArray.from_host(d), bfa.DeviceArray.from_host(c), cam)
    ref.integrate(T, d, c, cam)
    h, heap, hc, _ = g.export()
    check_hash_invariants(p, h, heap, hc)
    assert set(blocks_of(h)) <= set(blocks_of(ref.export()[0]))
    assert _off_bucket_entries(p, h) > 0


def test_no_color_allocates_but_does_not_update(scene):
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 16, num_blocks=1 << 15)
    pair = Pair(p, cam)
    (T, d, c), = render_frames(scene, cam, [3])
    pair.integrate(0, T, d, None)
    pair.compare()
    _, _, _, vox = pair.gpu.export()
    assert np.all(vox["weight"] == 0)


def test_empty_frame(scene):
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 14, num_blocks=1 << 12)
    pair = Pair(p, cam)
    d = np.full((cam.imageHeight, cam.imageWidth), -np.inf, np.float32)
    c = np.zeros((cam.imageHeight, cam.imageWidth, 4), np.uint8)
    pair.integrate(0, np.eye(4, dtype=np.float32), d, c)
    pair.gc()
    assert pair.compare() == 0
    assert pair.gpu.getHeapFreeCount() == p.numSDFBlocks


def test_heap_exhaustion_flags_error(scene):
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 14, num_blocks=64)
    g = bfa.SceneRepHashSDF(p)
    (T, d, c), = render_frames(scene, cam, [0])
    dd, cc = bfa.DeviceArray.from_host(d), bfa.DeviceArray.from_host(c)
    g.integrate(T, dd, cc, cam)
    assert g.errorFlags() & 2
    assert g.getHeapFreeCount() == 0
    from oracle_lib import check_hash_invariants
    h, heap, hc, _ = g.export()
    check_hash_invariants(p, h, heap, hc)


def test_full_resolution_frame(scene):
    """640x480 @ 4 mm: the bench configuration's per-frame shape."""
    cam = bfa.depth_camera(640, 480)
    p = bfa.hash_params(voxel_size=0.004, num_buckets=1 << 20, num_blocks=1 << 18)
    pair = Pair(p, cam)
    frames = render_frames(scene, cam, [0, 5])
    for k, (T, d, c) in enumerate(frames):
        pair.integrate(k, T, d, c)
    pair.gc()
    assert pair.compare() > 10000


@pytest.mark.parametrize("shift", [0.0, 0.004, 0.03, 0.15])
def test_fused_reintegrate_parity(scene, shift):
    """Scene::reintegrate (one fused voxel pass) == deIntegrate(old) + integrate(new) in the oracle,
    for pose changes from none (identical lists) to 15 cm (largely disjoint lists, new blocks)."""
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 17, num_blocks=1 << 16)
    pair = Pair(p, cam)
    frames = render_frames(scene, cam, [0, 5, 10, 15])
    for k, (T, d, c) in enumerate(frames):
        pair.integrate(k, T, d, c)
    pair.gc()
    rng = np.random.default_rng(7)
    for k in (1, 2):
        T, d, c = frames[k]
        T2 = T.copy()
        T2[:3, 3] += rng.normal(size=3) * shift
        dd, cc = pair._upload(k, d, c)
        pair.gpu.reintegrate(T, T2, dd, cc, cam)
        pair.ora.integrate(T, d, c, cam, deintegrate=True)
        pair.ora.integrate(T2, d, c, cam)
        pair.compare()
        pair.gc()
        pair.compare()
    assert pair.gpu.errorFlags() == 0


def _perturbed(T, rng, shift, rot_deg=0.0):
    T2 = T.copy()
    T2[:3, 3] += rng.normal(size=3) * shift
    if rot_deg:
        w = rng.normal(size=3)
        w *= np.deg2rad(rot_deg) / np.linalg.norm(w)
        K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
        th = np.linalg.norm(w)
        R = np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K
        T2[:3, :3] = (R @ T2[:3, :3].astype(np.float64)).astype(np.float32)
    return T2.astype(np.float32)


@pytest.mark.parametrize("shift", [0.004, 0.05])
def test_op_batch_parity(scene, shift):
    """Scene::applyOps (a frame's fixes as one voxel pass: per-block op masks, voxels loaded once and
    updated in op order) == the same integrate / deIntegrate calls one by one in the oracle, then GC
    on both (the GC list is the last op's frustum list in both). Mixed batch: re-integrations of
    several frames (de-integrate + integrate), a de-integration only, an integration of a frame that
    was not in the volume, and two ops touching the same frame twice."""
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 17, num_blocks=1 << 16)
    pair = Pair(p, cam)
    frames = render_frames(scene, cam, [0, 4, 8, 12, 16, 20])
    for k in range(5):
        T, d, c = frames[k]
        pair.integrate(k, T, d, c)
    pair.gc()
    rng = np.random.default_rng(11)
    cur = {k: frames[k][0] for k in range(5)}
    for rnd in range(2):
        ops = []
        for k in (1, 3, 0):  # re-integrations
            T2 = _perturbed(cur[k], rng, shift, rot_deg=0.3)
            ops += [(cur[k], k, True), (T2, k, False)]
            cur[k] = T2
        if rnd == 0:
            ops.append((cur[4], 4, True))       # de-integration only
            del cur[4]
            ops.append((frames[5][0], 5, False))  # integration of a new frame
            cur[5] = frames[5][0]
        else:
            T2 = _perturbed(cur[5], rng, shift)
            ops += [(cur[5], 5, True), (T2, 5, False)]
            cur[5] = T2
        dev = []
        for T, k, deint in ops:
            dd, cc = pair._upload(k, frames[k][1], frames[k][2])
            dev.append((T, dd, cc, deint))
            pair.ora.integrate(T, frames[k][1], frames[k][2], cam, deintegrate=deint)
        pair.gpu.apply_ops(dev, cam)
        assert pair.compare() > 1000
        pair.gc()
        pair.compare()
    assert pair.gpu.errorFlags() == 0


def test_op_batch_alloc_congested_path(scene):
    """The alloc walk's congested-tile path (a tile whose keys overflow its LDS set and overflow list walks
    again and emits every block directly; never taken at the bench workloads) forced on for every tile
    (BFSceneOptions.testFlags = BF_SCENE_TEST_ALLOC_DIRECT): its candidates duplicate phase 2's, the global
    dedup removes them, and the scene stays bit-exact with the oracle through single integrations and an op
    batch."""
    from bundlefusion_amd.abi import BF_SCENE_TEST_ALLOC_DIRECT
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 17, num_blocks=1 << 16)
    pair = Pair(p, cam, test_flags=BF_SCENE_TEST_ALLOC_DIRECT)
    frames = render_frames(scene, cam, [0, 5, 10, 15])
    for k in range(3):
        T, d, c = frames[k]
        pair.integrate(k, T, d, c)
        pair.compare()
    pair.gc()
    rng = np.random.default_rng(7)
    ops = []
    for k in (0, 2):
        T2 = _perturbed(frames[k][0], rng, 0.02, rot_deg=0.3)
        ops += [(frames[k][0], k, True), (T2, k, False)]
    ops.append((frames[3][0], 3, False))
    dev = []
    for T, k, deint in ops:
        dd, cc = pair._upload(k, frames[k][1], frames[k][2])
        dev.append((T, dd, cc, deint))
        pair.ora.integrate(T, frames[k][1], frames[k][2], cam, deintegrate=deint)
    pair.gpu.apply_ops(dev, cam)
    assert pair.compare() > 1000
    pair.gc()
    pair.compare()
    assert pair.gpu.getHeapFreeCount() == pair.ora.getHeapFreeCount()
    assert pair.gpu.errorFlags() == 0


def test_op_batch_full_resolution(scene):
    """A full 10-fix batch (20 ops) at 640x480 / 4 mm against the oracle."""
    cam = bfa.depth_camera(640, 480)
    p = bfa.hash_params(voxel_size=0.004, num_buckets=1 << 20, num_blocks=1 << 18)
    pair = Pair(p, cam)
    ids = list(range(0, 40, 4))
    frames = render_frames(scene, cam, ids)
    for k, (T, d, c) in enumerate(frames):
        pair.integrate(k, T, d, c)
    rng = np.random.default_rng(5)
    ops = []
    for k, (T, d, c) in enumerate(frames):
        T2 = _perturbed(T, rng, 0.01, rot_deg=0.2)
        ops += [(T, k, True), (T2, k, False)]
    dev = []
    for T, k, deint in ops:
        dd, cc = pair._upload(k, frames[k][1], frames[k][2])
        dev.append((T, dd, cc, deint))
        pair.ora.integrate(T, frames[k][1], frames[k][2], cam, deintegrate=deint)
    pair.gpu.apply_ops(dev, cam)
    pair.gc()
    assert pair.compare() > 10000
    assert pair.gpu.errorFlags() == 0


def test_chunk_sharding_partitions_the_scene(scene):
    """Multi-GPU TSDF sharding: scenes with shardCount 2, shardIndex 0 / 1 fed the
    same frames own disjoint block sets whose union — blocks and voxel payload — is the unsharded
    scene (each block's voxels depend only on the frames, not on which GPU owns it)."""
    cam = small_cam()
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 16, num_blocks=1 << 15)
    full = bfa.SceneRepHashSDF(p)
    shards = [bfa.SceneRepHashSDF(p, shard_count=2, shard_index=i, shard_chunk=0.5) for i in range(2)]
    frames = render_frames(scene, cam, [0, 6, 12])
    dev = []
    for T, d, c in frames:
        dd, cc = bfa.DeviceArray.from_host(d), bfa.DeviceArray.from_host(c)
        dev.append((dd, cc))
        for s in [full] + shards:
            s.integrate(T, dd, cc, cam)
    T, d, c = frames[1]
    for s in [full] + shards:
        s.deIntegrate(T, dev[1][0], dev[1][1], cam)
        s.garbageCollect()
    from oracle_lib import blocks_of
    fh, _, _, fv = full.export()
    fb = blocks_of(fh)
    from bundlefusion_amd.dist import chunk_owner
    union = {}
    for i, s in enumerate(shards):
        h, _, _, v = s.export()
        b = blocks_of(h)
        assert not (set(b) & set(union)), "a block is owned by both shards"
        for k in list(b)[:300]:  # the host mirror of owned() agrees with the device
            assert chunk_owner(*k, 0.01, 2, chunk=0.5) == i
        for k, ptr in b.items():
            union[k] = v[ptr:ptr + 512]
    assert set(union) == set(fb)
    assert len(union) > 200 and 0 < len(blocks_of(shards[0].export()[0])) < len(fb)
    for k, ptr in fb.items():
        a, b = fv[ptr:ptr + 512], union[k]
        np.testing.assert_array_equal(a["sdf"].view(np.uint32), b["sdf"].view(np.uint32))
        np.testing.assert_array_equal(a["weight"], b["weight"])
        np.testing.assert_array_equal(a["color"], b["color"])
