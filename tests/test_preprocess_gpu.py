"""GPU parity of the input preprocessing (CUDAImageManager::process, CUDAImageManager.cpp:22-158)
against the oracle's serial restatement (oracle/frames.cpp): ushort -> metres, erodeDepthMap x2,
gaussFilterDepthMap, nearest resampling. Same float expressions in the same order and the same
host-tabulated Gaussian weights, so the bar is bit-exact."""
import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd import io as bio
from oracle_lib import preprocess

pytestmark = pytest.mark.gpu


def frame(W=640, H=480, f=3, seed=1):
    sc = bfa.synth_scene(0)
    cam = bfa.depth_camera(W, H, fx=577.87 * W / 640, fy=577.87 * W / 640)
    d, c = bfa.synth_render_host(sc, bfa.synth_pose(f), cam, seed, f)
    u16 = np.where(np.isfinite(d) & (d > 0), np.round(d * 1000.0), 0).astype(np.uint16)
    rng = np.random.default_rng(seed)
    u16[rng.random(u16.shape) < 0.02] = 0          # sensor dropouts
    u16[200:230, 300:340] = 0                       # a hole
    return u16, np.ascontiguousarray(c, np.uint8)


def run_gpu(opts, u16, rgbx, iwh):
    H, W = u16.shape
    ch, cw = rgbx.shape[:2]
    pp = bio.Preprocessor((W, H), (cw, ch), iwh, opts)
    dd = bfa.DeviceArray.from_host(u16)
    dc = bfa.DeviceArray.from_host(rgbx)
    od = bfa.DeviceArray((iwh[1], iwh[0]), np.float32)
    oc = bfa.DeviceArray((iwh[1], iwh[0], 4), np.uint8)
    pp.run(dd, dc, od, oc)
    return od.download(), oc.download()


@pytest.mark.parametrize("iwh", [(640, 480), (320, 240)])
@pytest.mark.parametrize("erode,filt", [(True, True), (False, True), (True, False), (False, False)])
def test_preprocess_parity(iwh, erode, filt):
    u16, rgbx = frame()
    opts = bio.preprocess_options(erode=erode, depth_filter=filt)
    gd, gc = run_gpu(opts, u16, rgbx, iwh)
    od, oc = preprocess(opts, u16, rgbx, iwh)
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
    np.testing.assert_array_equal(gc, oc)
    valid = np.isfinite(gd)
    assert 0.5 < valid.mean() < 1.0


@pytest.mark.parametrize("structure,sigma_d", [(1, 1.0), (5, 3.0)])
def test_preprocess_other_radii(structure, sigma_d):
    u16, rgbx = frame(W=320, H=240, f=9, seed=3)
    opts = bio.preprocess_options(structure=structure, sigma_d=sigma_d, sigma_r=0.1)
    gd, gc = run_gpu(opts, u16, rgbx, (160, 120))
    od, oc = preprocess(opts, u16, rgbx, (160, 120))
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
    np.testing.assert_array_equal(gc, oc)


def test_preprocess_sens_round_trip(tmp_path):
    """A .sens written from synthetic frames, read back, preprocessed on the GPU: equals the oracle
    run on the same decoded frames (the path a .sens input takes into the integrator)."""
    u16, rgbx = frame(W=320, H=240, f=5)
    K = np.eye(4, dtype=np.float32)
    K[0, 0] = K[1, 1] = 288.935
    K[0, 2], K[1, 2] = 159.5, 119.5
    p = str(tmp_path / "s.sens")
    bio.write_sens(p, u16[None], rgbx[None], np.eye(4, dtype=np.float32)[None], K)
    s = bio.SensorData(p)
    d16, col = s.depth_u16(0), s.color(0)
    opts = bio.preprocess_options()
    gd, gc = run_gpu(opts, d16, col, (320, 240))
    od, oc = preprocess(opts, u16, col, (320, 240))
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
    np.testing.assert_array_equal(gc, oc)
