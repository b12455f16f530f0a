"""GPU parity of the raycaster (Scene::raycast: interval splat + renderKernel + computeNormals)
against the oracle's restatement of CUDARayCastSDF::render on identical volumes.

Both sides evaluate the same float32 expressions in the same order (-ffp-contract=off), so the
rendered depth / depth4 / colour / normal bits are expected to be identical; the stated bar
(>= 99.5 % validity agreement, |d depth| <= 1 mm) is asserted as the fallback
and the exact-match fraction is required to be >= 99.9 %."""
import numpy as np
import pytest

import bundlefusion_amd as bfa
from tsdf_compare import Pair, render_frames

pytestmark = pytest.mark.gpu


def build(W=160, H=120, vs=0.01, frames=(0, 3, 6, 9), noise=1, **scene_opts):
    sc = bfa.synth_scene(0)
    f = 577.87 * W / 640.0
    cam = bfa.depth_camera(W, H, fx=f, fy=f)
    p = bfa.hash_params(voxel_size=vs, num_buckets=1 << 16, num_blocks=1 << 15)
    pair = Pair(p, cam, **scene_opts)
    for k, (T, d, c) in enumerate(render_frames(sc, cam, list(frames), noise_seed=noise)):
        pair.integrate(k, T, d, c)
    pair.gc()
    return sc, cam, pair, f


def compare(g, o, min_exact=0.999):
    gd, g4, gn, gc = g[:4]
    od, o4, on, oc = o[:4]
    gv, ov = np.isfinite(gd), np.isfinite(od)
    agree = np.mean(gv == ov)
    assert agree >= 0.995, agree
    both = gv & ov
    assert both.sum() > 0
    assert np.max(np.abs(gd[both] - od[both])) <= 1e-3
    exact = np.mean((gd.view(np.uint32) == od.view(np.uint32)))
    assert exact >= min_exact, exact
    for a, b in ((g4, o4), (gc, oc), (gn, on)):
        same = np.all(a.view(np.uint32) == b.view(np.uint32), axis=-1)
        assert np.mean(same) >= min_exact
    return gv.mean()


@pytest.mark.parametrize("pose_frame", [3, 7])
def test_raycast_parity(pose_frame):
    sc, cam, pair, f = build()
    rp = bfa.raycast_params(cam.imageWidth, cam.imageHeight, fx=f, fy=f)
    T = bfa.synth_pose(pose_frame)
    g = pair.gpu.raycast(T, cam, rp, want_intervals=True)
    o = pair.ora.raycast(T, cam, rp, want_intervals=True)
    hit = compare(g, o)
    assert hit > 0.5
    # intervals: identical wherever the depth test cannot tie on a clamped NDC z
    gmin, omin = g[4], o[4]
    sel = np.isfinite(omin) & (omin >= rp.minDepth) & (omin < rp.maxDepth)
    np.testing.assert_array_equal(gmin[sel], omin[sel])


def test_raycast_gradients_parity():
    sc, cam, pair, f = build()
    rp = bfa.raycast_params(cam.imageWidth, cam.imageHeight, fx=f, fy=f, use_gradients=True)
    T = bfa.synth_pose(5)
    compare(pair.gpu.raycast(T, cam, rp), pair.ora.raycast(T, cam, rp))


def test_raycast_full_resolution_4mm():
    """640x480 render of a 4 mm volume (the bench configuration), parity + sanity vs the input."""
    W, H = 640, 480
    sc = bfa.synth_scene(0)
    cam = bfa.depth_camera(W, H)
    p = bfa.hash_params(voxel_size=0.004, num_buckets=1 << 20, num_blocks=1 << 17)
    pair = Pair(p, cam)
    for k, (T, d, c) in enumerate(render_frames(sc, cam, [0, 2], noise_seed=1)):
        pair.integrate(k, T, d, c)
    rp = bfa.raycast_params(W, H)
    T = bfa.synth_pose(1)
    g = pair.gpu.raycast(T, cam, rp)
    o = pair.ora.raycast(T, cam, rp)
    compare(g, o)
    ref, _ = bfa.synth_render_host(sc, T, cam, 0, 1)
    both = np.isfinite(g[0]) & np.isfinite(ref)
    assert both.mean() > 0.5
    assert np.median(np.abs(g[0][both] - ref[both])) < 0.003


def test_raycast_empty_and_outside():
    sc, cam, pair, f = build(frames=())
    rp = bfa.raycast_params(cam.imageWidth, cam.imageHeight, fx=f, fy=f)
    g = pair.gpu.raycast(bfa.synth_pose(0), cam, rp)
    assert np.all(g[0] == -np.inf) and np.all(g[2] == -np.inf)


@pytest.mark.parametrize("row_cap", [1, 0], ids=["row-lists-overflow", "row-lists"])
def test_splat_paths_give_the_same_intervals(row_cap):
    """Both forms of the tiled interval splat agree with the oracle bit for bit: the tile-row lists (the
    default), and the full scan a tile falls back to when the row lists overflow their capacity (forced with a
    capacity of one entry, BFSceneOptions.splatRowCap)."""
    sc, cam, pair, f = build(splat_row_cap=row_cap)
    rp = bfa.raycast_params(cam.imageWidth, cam.imageHeight, fx=f, fy=f)
    T = bfa.synth_pose(5)
    g = pair.gpu.raycast(T, cam, rp, want_intervals=True)
    o = pair.ora.raycast(T, cam, rp, want_intervals=True)
    compare(g, o)
    gmin, omin = g[4], o[4]
    sel = np.isfinite(omin) & (omin >= rp.minDepth) & (omin < rp.maxDepth)
    np.testing.assert_array_equal(gmin[sel], omin[sel])
