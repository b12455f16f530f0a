"""CPU tests of the TSDF oracle: analytic known-answer tests written from the cited reference
lines, structural invariants (debugHash), and the committed golden fixture."""
import os

import numpy as np
import pytest

import bundlefusion_amd as bfa
from oracle_lib import (OracleScene, block_voxels, blocks_of, bucket_of, check_hash_invariants,
                        dense_integrate, matrix_inverse)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_compute_hash_pos_kat():
    # VoxelUtilHashSDF.h:225-234: ((x*p0) ^ (y*p1) ^ (z*p2)) % n, wrapping int32, negatives + n
    n = 800000
    assert bucket_of((0, 0, 0), n) == 0
    assert bucket_of((1, 0, 0), n) == 73856093 % n == 256093
    assert bucket_of((-1, 0, 0), n) == n - 256093
    assert bucket_of((0, 1, 0), n) == 19349669 % n
    # int32 wrap: 83492791 * 30 overflows
    v = (83492791 * 30) & 0xFFFFFFFF
    v = v - (1 << 32) if v >= 1 << 31 else v
    expect = (abs(v) % n) * (1 if v >= 0 else -1)
    expect = expect + n if expect < 0 else expect
    assert bucket_of((0, 0, 30), n) == expect


def test_matrix_inverse_matches_numpy():
    rng = np.random.default_rng(0)
    for _ in range(20):
        T = bfa.synth_pose(int(rng.integers(0, 1000)))
        inv = matrix_inverse(T)
        np.testing.assert_allclose(inv @ T, np.eye(4), atol=2e-6)


def plane_frame(cam, z=1.0, rgb=(100, 150, 200)):
    d = np.full((cam.imageHeight, cam.imageWidth), z, np.float32)
    c = np.zeros((cam.imageHeight, cam.imageWidth, 4), np.uint8)
    c[..., 0], c[..., 1], c[..., 2], c[..., 3] = rgb[0], rgb[1], rgb[2], 255
    return d, c


def test_plane_known_answer():
    """Fronto-parallel plane at 1 m, identity pose: every in-band voxel that projects on screen
    gets sdf = depth - z (float32), weight 1 and the input colour
    (integrateDepthMapKernel, CUDASceneRepHashSDF.cu:450-499)."""
    cam = bfa.depth_camera(64, 48, fx=50.0, fy=50.0)
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 14, num_blocks=1 << 13)
    o = OracleScene(p)
    d, c = plane_frame(cam)
    o.integrate(np.eye(4, dtype=np.float32), d, c, cam)
    h, heap, hc, vox = o.export()
    check_hash_invariants(p, h, heap, hc)
    blocks = blocks_of(h)
    assert blocks
    vs = np.float32(p.virtualVoxelSize)
    trunc = np.float32(p.truncation) + np.float32(p.truncScale) * np.float32(1.0)
    zs = set()
    n_upd = 0
    for (bx, by, bz), ptr in blocks.items():
        v = block_voxels(vox, ptr)
        for i in range(512):
            x, y, z = bx * 8 + i % 8, by * 8 + (i % 64) // 8, bz * 8 + i // 64
            wx, wy, wz = np.float32(x) * vs, np.float32(y) * vs, np.float32(z) * vs
            u = np.float32(wx * np.float32(cam.fx) / wz + np.float32(cam.mx))
            w = np.float32(wy * np.float32(cam.fy) / wz + np.float32(cam.my))
            ux, uy = int(u + np.float32(0.5)), int(w + np.float32(0.5))
            sdf = np.float32(1.0) - wz
            inside = 0 <= ux < cam.imageWidth and 0 <= uy < cam.imageHeight and (u + 0.5) > -1 and (w + 0.5) > -1
            if inside and abs(sdf) < trunc:
                assert v[i]["weight"] == 1.0
                assert v[i]["sdf"] == sdf
                assert tuple(v[i]["color"]) == (100, 150, 200, 255)
                n_upd += 1
                zs.add(z)
            else:
                assert v[i]["weight"] == 0.0
    assert n_upd > 1000
    # the band is +-8 cm around 1 m: voxel z indices 93..107
    assert min(zs) >= 92 and max(zs) <= 108


def test_integrate_weight_and_colour_running_average():
    """Second observation: sdf averaged with weight, colour 0.2*new + 0.8*old rounded (.cu:486-499)."""
    cam = bfa.depth_camera(32, 24, fx=25.0, fy=25.0)
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 12, num_blocks=1 << 11)
    o = OracleScene(p)
    d1, c1 = plane_frame(cam, 1.0, (100, 100, 100))
    d2, c2 = plane_frame(cam, 1.02, (200, 50, 0))
    o.integrate(np.eye(4, dtype=np.float32), d1, c1, cam)
    o.integrate(np.eye(4, dtype=np.float32), d2, c2, cam)
    h, heap, hc, vox = o.export()
    v = vox[vox["weight"] == 2.0]
    assert len(v) > 100
    assert np.all(v["color"][:, 0] == 120) and np.all(v["color"][:, 1] == 90) and np.all(v["color"][:, 2] == 80)
    assert np.all(v["color"][:, 3] == 255)


def test_deintegrate_restores_weights_and_gc_frees_all():
    scene = bfa.synth_scene(0)
    cam = bfa.depth_camera(80, 60, fx=577.87 / 8, fy=577.87 / 8)
    p = bfa.hash_params(voxel_size=0.02, num_buckets=1 << 14, num_blocks=1 << 13)
    o = OracleScene(p)
    frames = []
    for f in (0, 15):
        T = bfa.synth_pose(f)
        d, c = bfa.synth_render_host(scene, T, cam, 1, f)
        frames.append((T, d, c))
    o.integrate(*frames[0][:1], frames[0][1], frames[0][2], cam)
    _, _, _, v0 = o.export()
    o.integrate(frames[1][0], frames[1][1], frames[1][2], cam)
    o.deIntegrate(frames[1][0], frames[1][1], frames[1][2], cam)
    h, heap, hc, v1 = o.export()
    check_hash_invariants(p, h, heap, hc)
    np.testing.assert_array_equal(v0["weight"], v1["weight"])
    np.testing.assert_allclose(v0["sdf"], v1["sdf"], atol=1e-5)
    # colour is not restored: integrate blends 0.2*new + 0.8*old but de-integrate divides a
    # weighted sum by (w-1) (CUDASceneRepHashSDF.cu:491 vs :502), so they are not inverses
    o.deIntegrate(frames[0][0], frames[0][1], frames[0][2], cam)
    o.garbageCollect()
    h, heap, hc, v2 = o.export()
    check_hash_invariants(p, h, heap, hc)
    assert np.all(v2["weight"] == 0)
    # every block visible from frame 0 was freed; what remains was only visible from frame 1
    assert o.getHeapFreeCount() > p.numSDFBlocks - len(blocks_of(h)) - 1


def test_collision_list_invariants_oracle():
    scene = bfa.synth_scene(0)
    cam = bfa.depth_camera(80, 60, fx=577.87 / 8, fy=577.87 / 8)
    p = bfa.hash_params(voxel_size=0.02, num_buckets=97, num_blocks=2048)
    o = OracleScene(p)
    for f in (0, 40, 80):
        T = bfa.synth_pose(f)
        d, c = bfa.synth_render_host(scene, T, cam, 1, f)
        o.integrate(T, d, c, cam)
        o.garbageCollect()
        h, heap, hc, vox = o.export()
        check_hash_invariants(p, h, heap, hc)
    # some entries live off their bucket (collision lists were exercised)
    occ = np.nonzero(h["ptr"] != -2)[0]
    off_bucket = sum(1 for i in occ if i // 4 != bucket_of((h[i]["x"], h[i]["y"], h[i]["z"]), p.hashNumBuckets))
    assert off_bucket > 0


def test_dense_grid_matches_hash_on_allocated_blocks():
    """Config 1 (dense 128^3 grid) and the hash path share the per-voxel arithmetic."""
    scene = bfa.synth_scene(0)
    cam = bfa.depth_camera(160, 120, fx=577.87 / 4, fy=577.87 / 4)
    p = bfa.hash_params(voxel_size=0.004, num_buckets=1 << 16, num_blocks=1 << 15)
    T = bfa.synth_pose(0)
    d, c = bfa.synth_render_host(scene, T, cam, 1, 0)
    origin = (-64, -448, 448)  # 128^3 voxels around the camera's view of the far wall
    n = 128
    grid = dense_integrate(T, d, c, cam, p, origin, n)
    o = OracleScene(p)
    o.integrate(T, d, c, cam)
    h, _, _, vox = o.export()
    checked = 0
    for (bx, by, bz), ptr in blocks_of(h).items():
        ox, oy, oz = bx * 8 - origin[0], by * 8 - origin[1], bz * 8 - origin[2]
        if 0 <= ox < n and 0 <= oy < n and 0 <= oz < n:
            v = block_voxels(vox, ptr)
            g = grid[oz:oz + 8, oy:oy + 8, ox:ox + 8].reshape(512)
            assert np.array_equal(v["sdf"].view(np.uint32), g["sdf"].view(np.uint32))
            assert np.array_equal(v["weight"], g["weight"])
            checked += 1
    assert checked > 50
    assert (grid["weight"] > 0).sum() > 10000


def test_golden_fixture():
    """Regression pin: tests/golden/tsdf_frame0_80x60.npz was produced by this oracle
    (tests/golden/make_golden.py); the reference itself cannot run here."""
    path = os.path.join(GOLDEN, "tsdf_frame0_80x60.npz")
    if not os.path.exists(path):
        pytest.skip("golden fixture not generated")
    g = np.load(path, allow_pickle=False)
    from golden.make_golden import tsdf_frame0
    keys, sdf, weight, color, heap_free = tsdf_frame0()
    np.testing.assert_array_equal(keys, g["keys"])
    np.testing.assert_array_equal(sdf.view(np.uint32), g["sdf"].view(np.uint32))
    np.testing.assert_array_equal(weight, g["weight"])
    np.testing.assert_array_equal(color, g["color"])
    assert heap_free == int(g["heap_free"])


def test_integer_colour_blend_is_exact():
    """csrc/tsdf.hip blend_channel: the integrate colour update u8(clamp(roundf(0.2f cu + 0.8f oc),
    0, 254.5)) (CUDASceneRepHashSDF.cu:486-496, float32, no contraction) equals the integer form
    min(((2 cu + 8 oc + 5) * 6554) >> 16, 254) for all 65536 (cu, oc)."""
    import numpy as np
    cu = np.arange(256, dtype=np.float32)[:, None]
    oc = np.arange(256, dtype=np.float32)[None, :]
    r = (np.float32(0.2) * cu).astype(np.float32) + (np.float32(0.8) * oc).astype(np.float32)
    assert r.dtype == np.float32
    t = np.trunc(r)
    rf = t + ((r - t) >= np.float32(0.5))  # roundf for r >= 0
    ref = np.minimum(np.maximum(rf, 0), 254.5).astype(np.uint8)
    ci, oi = np.arange(256)[:, None], np.arange(256)[None, :]
    alt = np.minimum(((2 * ci + 8 * oi + 5) * 6554) >> 16, 254)
    np.testing.assert_array_equal(ref, alt)


def test_packed_float_colour_blend_is_exact():
    """csrc/tsdf.hip blend_color_f (the batch pass's integrate colour): min(rint((4 oc + cu) * 0.2f), 254)
    in float32 (4 oc + cu an exact integer, one rounded multiply, round-to-nearest-even; v_cvt_pk_u8_f32
    then converts an integral value) equals the reference byte for all 65536 (cu, oc), and an empty voxel
    (oc := cu) gives min(cu, 254) as the reference's new-colour branch clamped like blend_channel."""
    import numpy as np
    f32 = np.float32
    cu = np.arange(256, dtype=f32)[:, None]
    oc = np.arange(256, dtype=f32)[None, :]
    r = (np.float32(0.2) * cu).astype(f32) + (np.float32(0.8) * oc).astype(f32)
    t = np.trunc(r)
    ref = np.minimum(np.maximum(t + ((r - t) >= f32(0.5)), 0), 254.5).astype(np.uint8)
    a = (oc * f32(4.0) + cu).astype(f32)
    q = (a * f32(0.2)).astype(f32)
    assert q.dtype == f32
    packed = np.minimum(np.rint(q), f32(254.0)).astype(np.uint8)
    np.testing.assert_array_equal(packed, ref)
    c1 = np.arange(256, dtype=f32)
    empty = np.minimum(np.rint((c1 * f32(4.0) + c1).astype(f32) * f32(0.2)), f32(254.0)).astype(np.uint8)
    np.testing.assert_array_equal(empty, np.minimum(np.arange(256), 254).astype(np.uint8))


def test_deintegrate_colour_shortcut_is_exact():
    """csrc/tsdf.hip deint_channel: the de-integrate colour update u8(clamp(roundf((oc w - cu) / (w - 1)),
    0, 254.5)) (float32, CUDASceneRepHashSDF.cu:420-521) equals med3(oc + floor((2 (oc - cu) + d) * rcp(2 d)
    + 5e-4), 0, 254), d = w - 1, rcp forced to 0 for d > 510 — for every (oc, cu), every integral weight
    2..700 with the rcp exactly rounded and 1 ulp either side (v_rcp_f32's bound), and sampled weights up to
    the default weightMax (tools/check_deint_color.c runs the 9.3e9-case sweep)."""
    import numpy as np
    f32 = np.float32
    o = np.arange(256, dtype=f32)[:, None]
    c = np.arange(256, dtype=f32)[None, :]

    def ref(w):
        x = (o * w).astype(f32) - c
        q = (x / (w - f32(1))).astype(f32)
        a = np.abs(q)
        t = np.floor(a)
        r = np.copysign(t + ((a - t) >= f32(0.5)), q)
        return np.maximum(f32(0), np.minimum(r, f32(254.5))).astype(np.uint8)

    def fast(w, rc):
        d = w - f32(1)
        num = ((o - c) * f32(2)).astype(f32) + d  # exact: small integers
        k = np.floor((num * rc).astype(f32) + f32(5e-4))
        return np.minimum(np.maximum(o + k, f32(0)), f32(254)).astype(np.uint8)

    with np.errstate(all="ignore"):
        for wi in list(range(2, 701)) + [int(x) for x in np.geomspace(701, 99999999, 300)]:
            w = f32(wi)
            d = w - f32(1)
            r0 = ref(w)
            rcs = [f32(0)] if d > 510 else [f32(1) / (f32(2) * d)]
            if d <= 510:
                rcs += [np.nextafter(rcs[0], f32(np.inf)), np.nextafter(rcs[0], f32(0))]
            for rc in rcs:
                np.testing.assert_array_equal(fast(w, rc), r0, err_msg=f"w={wi} rc={rc!r}")


def test_oracle_shards_partition_the_scene():
    """The oracle scene with a multi-GPU shard's ownership (or_scene_set_shard, the restatement the sharded
    GPU window replays run on): each shard stores exactly the blocks whose 0.25 m chunk it owns
    (dist.chunk_owner_array, the host mirror of tsdf.hip's owned()), the shards are disjoint, and their union
    is the unsharded scene with bit-identical voxels."""
    from bundlefusion_amd.dist import chunk_owner_array
    scene = bfa.synth_scene(0)
    cam = bfa.depth_camera(160, 120, fx=577.87 / 4, fy=577.87 / 4)
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 15, num_blocks=1 << 14)
    frames = []
    for f in (0, 8):
        T = bfa.synth_pose(f)
        d, c = bfa.synth_render_host(scene, T, cam, 1, f)
        frames.append((T, d, c))
    full = OracleScene(p)
    shards = [OracleScene(p, shard=(2, r, 0.25)) for r in range(2)]
    for sc in [full] + shards:
        for T, d, c in frames:
            sc.integrate(T, d, c, cam)
        sc.garbageCollect()
    fh, _, _, fv = full.export()
    fb = blocks_of(fh)
    union = {}
    for r, sc in enumerate(shards):
        h, heap, hc, v = sc.export()
        check_hash_invariants(p, h, heap, hc)
        b = blocks_of(h)
        assert b and not (set(b) & set(union))
        assert np.all(chunk_owner_array(np.array(sorted(b)), 0.01, 2, chunk=0.25) == r)
        for k, ptr in b.items():
            union[k] = block_voxels(v, ptr)
    assert set(union) == set(fb) and len(fb) > 200
    for k, ptr in fb.items():
        assert block_voxels(fv, ptr).tobytes() == union[k].tobytes(), k


def test_band_cull_rectangle_covers_truncated_pixels():
    """csrc/tsdf.hip RECT_HI: the band cull's screen rectangle [floor(lo - 0.5), floor(hi + 1.5 + 1/64)] must hold
    every column the voxel pass (and integrateDepthMapKernel, CUDASceneRepHashSDF.cu:453-457) gives a voxel whose
    projection lies within the corners' range, with the pixel taken as (int)(x + 0.5), truncated toward zero (so
    x in (-1.5, -0.5] is column 0), while the corner projections themselves carry rounding of ~1e-4 px. Without the
    1/64 the left / top edge has no margin: a corner computed 7.5e-5 px below -1.5 dropped column 0 (the round-6
    end-phase failure, profiles/r11_cull_margin_fix.txt)."""
    f32 = np.float32
    rect_hi = f32(1.5) + f32(2.0 ** -6)
    rng = np.random.default_rng(3)
    W = 640
    # corner ranges around both edges; the true voxel projection may exceed the computed hi by the rounding
    lo = np.concatenate([rng.uniform(-30, 2, 20000), rng.uniform(W - 30, W + 2, 20000)]).astype(f32)
    hi = (lo + rng.uniform(0, 25, lo.size)).astype(f32)
    hi[:5000] = f32(-1.5) - rng.uniform(0, 1e-4, 5000).astype(f32)  # the failing case's neighbourhood
    lo[:5000] = np.minimum(lo[:5000], hi[:5000] - f32(3))
    err = f32(1e-4)
    for x in (hi + err, lo - err, (lo + hi) / 2):  # projections of voxels at the extremes / inside
        x = x.astype(f32)
        col = np.trunc(x + f32(0.5)).astype(np.int64)  # C float -> int conversion
        on = (col >= 0) & (col < W)
        c0 = np.floor(lo - f32(0.5)).astype(np.int64)
        c1 = np.floor(hi + rect_hi).astype(np.int64)
        # the cull rejects when c1 < 0 or c0 > W - 1, else it reads columns [max(c0, 0), min(c1, W - 1)]
        kept = ~((c1 < 0) | (c0 > W - 1))
        covered = kept & (np.maximum(c0, 0) <= col) & (col <= np.minimum(c1, W - 1))
        assert np.all(covered[on]), np.nonzero(on & ~covered)[0][:5]
    # and the old bound, hi + 1.5, misses the failing case
    x = (f32(-1.5) - f32(7.5e-5) + f32(1e-4)).astype(f32)
    assert int(np.trunc(x + f32(0.5))) == 0 and np.floor(f32(-1.5) - f32(7.5e-5) + f32(1.5)) < 0


def test_uniform_divisor_division_is_exact(tmp_path):
    """csrc/tsdf.hip div_by_uniform (the alloc walk's divisions by fx, fy and the voxel size): a * RN(1/b) plus
    two fma residual corrections equals the IEEE quotient a / b for b in [2^-20, 2^20] and 2^-100 <= |a| <= 2^100,
    and stays a tiny number of a's sign below that. tools/check_uniform_div.c, reduced sample (2^13 numerators per
    divisor, 4 113 divisors; the full 2^21 run is the 8.6e9-case sweep DESIGN.md cites)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    src = os.path.join(os.path.dirname(__file__), "..", "tools", "check_uniform_div.c")
    exe = str(tmp_path / "check_uniform_div")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", src, "-lm", "-o", exe], check=True)
    out = subprocess.run([exe, "13"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:]
    assert " 0 disagreements" in out.stdout
