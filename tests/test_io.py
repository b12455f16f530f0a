"""§8(f)1 input formats (CPU): `.sens` (mLib SensorData v4) and
`zParameters*.txt`. Parity unpinned against mLib (absent here): the reader is checked against an
independent Python encoder written from Appendix B, the writer by round trips and against the same
encoder byte for byte, and both against the committed fixture tests/golden/sens_3x40x30.sens."""
import os
import struct
import zlib

import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd import io as bio

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def synth_frames(F=3, w=40, h=30, seed=0):
    rng = np.random.default_rng(seed)
    depth = rng.integers(400, 4000, size=(F, h, w)).astype(np.uint16)
    depth[:, ::7, ::5] = 0  # holes
    rgbx = rng.integers(0, 256, size=(F, h, w, 4)).astype(np.uint8)
    rgbx[..., 3] = 255
    poses = np.stack([np.eye(4, dtype=np.float32) for _ in range(F)])
    for f in range(F):
        poses[f, :3, 3] = [0.1 * f, -0.05 * f, 0.02 * f]
    K = np.eye(4, dtype=np.float32)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = 36.1, 36.2, 19.5, 14.5
    return depth, rgbx, poses, K


def encode_sens(depth, rgbx, poses, K, name=b"py-encoder", zlib_depth=True, shift=1000.0, color_codec=None,
                jpeg_quality=90):
    """Independent encoder of the v4 layout (Appendix B), used to pin the C++ reader. color_codec:
    None = raw RGB (colorCompression 0), "png" (1) or "jpeg" (2) through PIL (build container only)."""
    F, h, w = depth.shape
    out = [struct.pack("<IQ", 4, len(name)), name]
    ident = np.eye(4, dtype=np.float32)
    for m in (K, ident, K, ident):
        out.append(np.asarray(m, "<f4").tobytes())
    cc = {None: 0, "png": 1, "jpeg": 2}[color_codec]
    out.append(struct.pack("<ii", cc, 1 if zlib_depth else 0))
    out.append(struct.pack("<IIIIfQ", w, h, w, h, shift, F))
    for f in range(F):
        col = np.ascontiguousarray(rgbx[f, ..., :3]).tobytes()
        if color_codec is not None:
            import io as _io

            from PIL import Image
            b = _io.BytesIO()
            im = Image.fromarray(np.ascontiguousarray(rgbx[f, ..., :3]))
            im.save(b, "JPEG", quality=jpeg_quality) if color_codec == "jpeg" else im.save(b, "PNG")
            col = b.getvalue()
        dep = depth[f].astype("<u2").tobytes()
        if zlib_depth:
            dep = zlib.compress(dep)
        out.append(np.asarray(poses[f], "<f4").tobytes())
        out.append(struct.pack("<QQQQ", f, f, len(col), len(dep)))
        out += [col, dep]
    out.append(struct.pack("<Q", 0))
    return b"".join(out)


@pytest.mark.parametrize("zl", [True, False])
def test_reader_against_independent_encoder(tmp_path, zl):
    depth, rgbx, poses, K = synth_frames()
    p = str(tmp_path / "a.sens")
    open(p, "wb").write(encode_sens(depth, rgbx, poses, K, zlib_depth=zl))
    s = bio.SensorData(p)
    assert len(s) == 3 and s.info.version == 4 and s.sensor_name == "py-encoder"
    assert s.info.depthCompression == (1 if zl else 0) and s.info.colorCompression == 0
    np.testing.assert_array_equal(s.intrinsics("depth"), K)
    for f in range(3):
        np.testing.assert_array_equal(s.pose(f), poses[f])
        assert s.timestamps(f) == (f, f)
        np.testing.assert_array_equal(s.depth_u16(f), depth[f])
        np.testing.assert_array_equal(s.color(f), rgbx[f])
        d = s.depth(f)  # SensorDataReader.cpp:104-107
        ref = np.where(depth[f] == 0, -np.inf, depth[f].astype(np.float32) / np.float32(1000.0)).astype(np.float32)
        np.testing.assert_array_equal(d, ref)


def test_writer_matches_encoder_bytes(tmp_path):
    depth, rgbx, poses, K = synth_frames(seed=4)
    p = str(tmp_path / "w.sens")
    bio.write_sens(p, depth, rgbx, poses, K, zlib_depth=False, name="py-encoder")
    assert open(p, "rb").read() == encode_sens(depth, rgbx, poses, K, zlib_depth=False)


def test_writer_reader_round_trip_zlib(tmp_path):
    depth, rgbx, poses, K = synth_frames(F=5, w=64, h=48, seed=7)
    p = str(tmp_path / "r.sens")
    bio.write_sens(p, depth, rgbx, poses, K, zlib_depth=True)
    s = bio.SensorData(p)
    assert len(s) == 5
    for f in range(5):
        np.testing.assert_array_equal(s.depth_u16(f), depth[f])
        np.testing.assert_array_equal(s.color(f), rgbx[f])
        np.testing.assert_array_equal(s.pose(f), poses[f])


def test_committed_fixture():
    """tests/golden/sens_3x40x30.sens (written by tests/golden/make_golden.py with the encoder above)."""
    s = bio.SensorData(os.path.join(GOLDEN, "sens_3x40x30.sens"))
    exp = np.load(os.path.join(GOLDEN, "sens_3x40x30.npz"))
    for f in range(3):
        np.testing.assert_array_equal(s.depth_u16(f), exp["depth"][f])
        np.testing.assert_array_equal(s.color(f), exp["rgbx"][f])
        np.testing.assert_array_equal(s.pose(f), exp["poses"][f])


def test_errors(tmp_path):
    with pytest.raises(bfa.BFError):
        bio.SensorData(str(tmp_path / "missing.sens"))
    p = tmp_path / "bad.sens"
    p.write_bytes(struct.pack("<IQ", 3, 0))
    with pytest.raises(bfa.BFError):
        bio.SensorData(str(p))
    depth, rgbx, poses, K = synth_frames(F=1)
    raw = bytearray(encode_sens(depth, rgbx, poses, K))
    p2 = tmp_path / "trunc.sens"
    p2.write_bytes(bytes(raw[:-40]))
    with pytest.raises(bfa.BFError):
        bio.SensorData(str(p2))


def test_parameter_file():
    pf = bio.ParameterFile(os.path.join(GOLDEN, "zParameters_fixture.txt"))
    assert pf.number("s_sensorIdx") == 8
    assert pf.boolean("s_erodeSIFTdepth") and not pf.boolean("s_SDFUseGradients")
    assert pf.floats("s_SDFVoxelSize")[0] == np.float32(0.004)
    assert pf.string("s_binaryDumpSensorFile") == "../data//sequence.sens"
    np.testing.assert_array_equal(pf.floats("s_topVideoTransformWorld"), np.eye(4, dtype=np.float32).reshape(16))
    assert "s_missing" not in pf
    with pytest.raises(bfa.BFError):
        pf.number("s_missing")
    hp = pf.hash_params()  # CUDASceneRepHashSDF::parametersFromGlobalAppState
    assert hp.hashNumBuckets == 8388608 and hp.numSDFBlocks == 2097152 and hp.hashBucketSize == 4
    assert hp.virtualVoxelSize == np.float32(0.004) and hp.truncation == np.float32(0.06)
    assert hp.integrationWeightMax == 99999999 and hp.streamingMinGridPos.x == -128
    rp = pf.raycast_params(288.935, 288.935, 159.5, 119.5)  # CUDARayCastSDF::parametersFromGlobalAppState
    assert (rp.width, rp.height) == (640, 480)
    assert rp.fx == pytest.approx(288.935 * 2, rel=1e-6) and rp.mx == pytest.approx(159.5 * 639 / 319, rel=1e-6)
    assert rp.rayIncrement == np.float32(np.float32(0.8) * np.float32(0.06))
    assert rp.maxNumVertices == 2097152 * 6
    o = pf.preprocess_options()
    assert o.erode == 1 and o.depthFilter == 1 and o.erodeStructureSize == 3
    assert o.sigmaD == np.float32(2.0) and o.sigmaR == np.float32(0.05)


def test_parameter_override(tmp_path):
    a = tmp_path / "a.txt"
    b = tmp_path / "b.txt"
    a.write_text("s_x = 1;\ns_y = 2.5f;\n")
    b.write_text("s_x = 3; // later file wins\n")
    pf = bio.ParameterFile(str(a), str(b))
    assert pf.number("s_x") == 3 and pf.number("s_y") == 2.5
