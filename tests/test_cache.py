"""Dense-term frame cache (CUDACache::storeFrame, /root/reference/FriedLiver/Source/CUDACache.cpp:45-94;
copyCacheFrameFrom / incrementCache, CUDACache.h:24-43).

CPU: known-answer tests of the oracle restatement (a fronto-parallel wall: constant depth, exact
camera-space positions, normal (0, 0, 1), uchar4 normal (128, 128, 255, 0), constant intensity, zero
derivatives; the cache intrinsics scaling of CUDACache::CUDACache).
GPU: bf_cache_* (one fused geometry pass + one LDS intensity pass) against the oracle, which stages the
reference's ten full-image passes, bit for bit on rendered frames; slot bookkeeping."""
import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd.cache import CUDACache, cache_options
from oracle_lib import cache_store_frame

FX = 577.87


def wall(W=640, H=480, d=2.0, rgb=(90, 160, 30)):
    depth = np.full((H, W), d, np.float32)
    color = np.zeros((H, W, 4), np.uint8)
    color[..., 0], color[..., 1], color[..., 2], color[..., 3] = rgb[0], rgb[1], rgb[2], 255
    return depth, color


def test_oracle_cache_wall_known_answer():
    o = cache_options(640, 480, FX, FX, 319.5, 239.5, 4)
    depth, color = wall()
    r = cache_store_frame(o, depth, color)
    K = r["K"]
    assert np.allclose([K[0, 0], K[1, 1], K[0, 2], K[1, 2]],
                       [FX * 80 / 640, FX * 60 / 480, 319.5 * 79 / 639, 239.5 * 59 / 479], rtol=1e-6)
    assert np.allclose(r["Kinv"] @ K, np.eye(4), atol=1e-5)
    assert np.all(r["depth"] == 2.0)
    # campos of cache pixel (x, y) = input pixel (xi, yi) back-projected at 2 m
    xi = (np.arange(80, dtype=np.float32) * np.float32(639 / 79) + np.float32(0.5)).astype(np.int64)
    yi = (np.arange(60, dtype=np.float32) * np.float32(479 / 59) + np.float32(0.5)).astype(np.int64)
    assert np.allclose(r["campos"][0, :, 0], (xi - 319.5) / FX * 2.0, atol=1e-5)
    assert np.allclose(r["campos"][:, 0, 1], (yi - 239.5) / FX * 2.0, atol=1e-5)
    assert np.all(r["campos"][..., 2] == 2.0) and np.all(r["campos"][..., 3] == 1.0)
    inner = r["normals"][1:-1, 1:-1]   # input pixels 8..631 are interior
    assert np.allclose(inner[..., :3], [0, 0, 1], atol=1e-5) and np.all(inner[..., 3] == 0)
    assert np.all(np.isneginf(r["normals"][0, :, 0])) and np.all(r["normalsU8"][0] == 0)
    assert np.all(r["normalsU8"][1:-1, 1:-1] == [128, 128, 255, 0])
    ival = np.float32((np.float32(0.299) * 90 + np.float32(0.587) * 160 + np.float32(0.114) * 30) / np.float32(255))
    assert np.allclose(r["intensity"], ival, rtol=1e-6)
    assert np.allclose(r["intensityDeriv"][1:-1, 1:-1], 0, atol=1e-6)
    assert np.all(np.isneginf(r["intensityDeriv"][0]))


def test_oracle_cache_invalid_depth_propagates():
    o = cache_options(640, 480, FX, FX, 319.5, 239.5, 4)
    depth, color = wall()
    depth[200:280, 300:340] = -np.inf
    r = cache_store_frame(o, depth, color)
    bad = ~np.isfinite(r["depth"])
    assert bad.any() and np.all(np.isneginf(r["campos"][bad][:, 0])) and np.all(r["normalsU8"][bad] == 0)


@pytest.mark.gpu
def test_cache_gpu_matches_oracle_bitwise():
    sc = bfa.synth_scene(0)
    cam = bfa.depth_camera(640, 480, fx=FX, fy=FX)
    o = cache_options(640, 480, FX, FX, cam.mx, cam.my, 8)
    cache = CUDACache(o)
    frames = []
    for f in (0, 7, 19):
        T = bfa.synth_pose(f)
        d, c = bfa.synth_render_host(sc, T, cam, 1, f)
        dd, cc = bfa.DeviceArray.from_host(d), bfa.DeviceArray.from_host(c)
        assert cache.storeFrame(dd, cc, 640, 480) == len(frames)
        frames.append((d, c, dd, cc))
    for i, (d, c, _, _) in enumerate(frames):
        g = cache.download(i)
        r = cache_store_frame(o, d, c)
        for k in ("depth", "campos", "normals", "normalsU8", "intensity", "intensityDeriv"):
            assert np.array_equal(g[k].view(np.uint8), r[k].view(np.uint8)), (i, k)
        assert np.isfinite(g["depth"]).mean() > 0.5
    K, Ki = cache.intrinsics()
    assert np.array_equal(K, r["K"]) and np.array_equal(Ki, r["Kinv"])
    # the global keyframe cache: copy of a local frame (Bundler::fuseToGlobal), skipped slots
    glob = CUDACache(o)
    glob.incrementCache()
    assert glob.copyCacheFrameFrom(cache, 2) == 1 and glob.getNumFrames() == 2
    g2 = glob.download(1)
    for k in g2:
        assert np.array_equal(g2[k].view(np.uint8), cache.download(2)[k].view(np.uint8))
    with pytest.raises(bfa.BFError):
        glob.copyCacheFrameFrom(cache, 5)  # not stored


@pytest.mark.gpu
def test_cache_half_resolution_input_and_no_filters():
    sc = bfa.synth_scene(0)
    cam = bfa.depth_camera(320, 240, fx=FX / 2, fy=FX / 2)
    o = cache_options(320, 240, FX / 2, FX / 2, cam.mx, cam.my, 2, width=160, height=120, color_sigma=0.0,
                      depth_sigma_d=0.0)
    cache = CUDACache(o)
    T = bfa.synth_pose(3)
    d, c = bfa.synth_render_host(sc, T, cam, 1, 3)
    cache.storeFrame(bfa.DeviceArray.from_host(d), bfa.DeviceArray.from_host(c), 320, 240)
    g, r = cache.download(0), cache_store_frame(o, d, c)
    for k in ("depth", "campos", "normals", "normalsU8", "intensity", "intensityDeriv"):
        assert np.array_equal(g[k].view(np.uint8), r[k].view(np.uint8)), k
