"""The FriedLiver application layer on CPU (bf_app_* needs a GPU; see test_app_gpu.py): the stand-in
front end's estimate against the oracle restatement (bit for bit), the .sens writer's pre-compressed
frames and the trajectory save (SensorDataReader::saveToFile, SensorDataReader.cpp:153-166), and the
past-the-end phase of the oracle loop (OnlineBundler.cpp:167-196, DepthSensing.cpp:1114-1126)."""
import ctypes as C
import math
import zlib

import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd import io as bio
from oracle_lib import lib as olib


def _tinc_product(prev, cur, f, seed, dr, dm):
    out = (C.c_float * 16)()
    bfa.check(bfa.lib().bf_front_end_tinc(bfa.abi.mat(prev), bfa.abi.mat(cur), C.c_uint32(f), C.c_uint32(seed),
                                          C.c_float(dr), C.c_float(dm), out))
    return np.array(out, np.float32).reshape(4, 4)


def _tinc_oracle(prev, cur, f, seed, dr, dm):
    L = olib()
    L.or_front_end_tinc.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_float, C.c_float, C.c_void_p]
    p = np.ascontiguousarray(prev, np.float32)
    c = np.ascontiguousarray(cur, np.float32)
    out = np.zeros(16, np.float32)
    L.or_front_end_tinc(p.ctypes.data, c.ctypes.data, f, seed, dr, dm, out.ctypes.data)
    return out.reshape(4, 4)


def test_front_end_estimate_matches_oracle_bitwise():
    poses = np.stack([bfa.synth_pose(f) for f in range(0, 400, 7)]).astype(np.float32)
    for k in range(1, len(poses)):
        for seed, dr, dm in ((1, math.radians(0.05), 0.002), (9, 0.01, 0.03), (1, 0.0, 0.0)):
            a = _tinc_product(poses[k - 1], poses[k], k, seed, dr, dm)
            b = _tinc_oracle(poses[k - 1], poses[k], k, seed, dr, dm)
            assert a.tobytes() == b.tobytes(), (k, seed)
    # no drift: the exact relative motion (to float rounding)
    rel = np.linalg.inv(poses[0].astype(np.float64)) @ poses[1].astype(np.float64)
    np.testing.assert_allclose(_tinc_product(poses[0], poses[1], 1, 1, 0.0, 0.0), rel, atol=2e-7)
    # the error step has the requested spread (rotation angle ~ sigma * sqrt(3))
    ang = []
    for f in range(1, 2000):
        T = _tinc_product(np.eye(4), np.eye(4), f, 3, 0.01, 0.0)
        ang.append(np.arccos(np.clip((np.trace(T[:3, :3]) - 1) / 2, -1, 1)))
    assert 0.0145 < np.sqrt(np.mean(np.square(ang))) < 0.0200
    bad = np.full((4, 4), -np.inf, np.float32)
    np.testing.assert_array_equal(_tinc_product(bad, poses[1], 1, 1, 0.01, 0.01), np.eye(4, dtype=np.float32))


def test_compressed_frames_and_trajectory_save(tmp_path):
    """A JPEG-colour / zlib-depth .sens written with pre-compressed streams reads back; saving a trajectory
    into it changes the poses (-inf past its end) and no other byte."""
    Image = pytest.importorskip("PIL.Image")
    import io as _io
    rng = np.random.default_rng(0)
    W, H, F = 64, 48, 5
    K = np.eye(4, dtype=np.float32)
    K[0, 0] = K[1, 1] = 60.0
    K[0, 2], K[1, 2] = (W - 1) / 2, (H - 1) / 2
    info = bio.sens_info((W, H), (W, H), K, color_compression=2, depth_compression=1)
    p = str(tmp_path / "in.sens")
    depth = rng.integers(0, 4000, (F, H, W)).astype(np.uint16)
    rgb = rng.integers(0, 255, (F, H, W, 3)).astype(np.uint8)
    jpg = []
    with bio.SensWriter(p, info) as w:
        for f in range(F):
            b = _io.BytesIO()
            Image.fromarray(rgb[f]).save(b, "JPEG", quality=90)
            jpg.append(b.getvalue())
            w.add_compressed_frame(np.eye(4) * (f + 1), jpg[-1], zlib.compress(depth[f].tobytes()), ts=(f, 10 * f))
    s = bio.SensorData(p)
    assert len(s) == F and s.info.colorCompression == 2
    for f in range(F):
        np.testing.assert_array_equal(s.depth_u16(f), depth[f])
        ref = np.asarray(Image.open(_io.BytesIO(jpg[f])).convert("RGB"))
        np.testing.assert_array_equal(s.color(f)[..., :3], ref)
        assert s.timestamps(f) == (f, 10 * f)
    s.close()
    T = np.stack([bfa.synth_pose(f) for f in range(3)]).astype(np.float32)
    out = str(tmp_path / "out.sens")
    bfa.check(bfa.lib().bf_sens_save_trajectory(p.encode(), out.encode(), T.ctypes.data_as(C.c_void_p), C.c_uint64(3)))
    a, b = open(p, "rb").read(), open(out, "rb").read()
    assert len(a) == len(b)
    s2 = bio.SensorData(out)
    for f in range(F):
        want = T[f] if f < 3 else np.full((4, 4), -np.inf, np.float32)
        np.testing.assert_array_equal(s2.pose(f), want)
        np.testing.assert_array_equal(s2.depth_u16(f), depth[f])
    diff = np.flatnonzero(np.frombuffer(a, np.uint8) != np.frombuffer(b, np.uint8))
    assert len(diff) <= 64 * F  # only pose bytes differ
