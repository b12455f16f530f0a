"""The `.sens` colour-stream decoders (bundlefusion_amd/csrc/image_codec.cpp, through the C ABI's
bf_image_decode and bf_sens_read_color). The reference decodes JPEG / PNG colour through the
un-vendored mLib (SensorDataReader.cpp:98-116); the decoders are pinned byte for byte against PIL
(libjpeg-turbo, zlib) on the committed fixtures of tests/golden/make_image_fixtures.py, and — where
PIL is importable — on a seeded sweep of sizes, subsamplings, qualities and restart intervals.
Tolerance: 0 (the IJG islow IDCT, fancy upsampling and fixed-point YCbCr tables are reproduced)."""
import io
import os
import struct

import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd import io as bio

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fixtures():
    d = np.load(os.path.join(GOLDEN, "image_codec.npz"))
    return d, sorted(k[:-7] for k in d.files if k.endswith("__bytes"))


@pytest.mark.parametrize("name", _fixtures()[1])
def test_golden_streams_bit_exact(name):
    d, _ = _fixtures()
    data = d[name + "__bytes"].tobytes()
    got = bio.decode_image(data, 2 if name.startswith("jpeg") else 1)
    assert got.shape[:2] == d[name + "__rgb"].shape[:2]
    np.testing.assert_array_equal(got[..., :3], d[name + "__rgb"])
    assert (got[..., 3] == 255).all()


def test_jpeg_sens_reads_like_pil():
    """A JPEG-colour .sens (colorCompression 2, zlib depth), the copyroom / apt0 layout."""
    d, _ = _fixtures()
    s = bio.SensorData(os.path.join(GOLDEN, "sens_jpeg_3x64x48.sens"))
    assert len(s) == 3 and s.info.colorCompression == 2 and s.info.depthCompression == 1
    for f in range(3):
        np.testing.assert_array_equal(s.color(f)[..., :3], d["sens_jpeg__rgb"][f])
        np.testing.assert_array_equal(s.depth_u16(f), d["sens_jpeg__depth"][f])
        np.testing.assert_array_equal(s.pose(f), d["sens_jpeg__poses"][f])


def test_png_sens_round_trip(tmp_path):
    """PNG colour (colorCompression 1) is lossless: the frames read back exactly."""
    pytest.importorskip("PIL")
    from test_io import encode_sens, synth_frames
    depth, rgbx, poses, K = synth_frames(F=2, w=40, h=30, seed=3)
    p = str(tmp_path / "png.sens")
    open(p, "wb").write(encode_sens(depth, rgbx, poses, K, color_codec="png"))
    s = bio.SensorData(p)
    assert s.info.colorCompression == 1
    for f in range(2):
        np.testing.assert_array_equal(s.color(f)[..., :3], rgbx[f, ..., :3])


def _pattern(w, h, rng):
    y, x = np.mgrid[0:h, 0:w]
    a = np.stack([x * 255 // max(1, w - 1), y * 255 // max(1, h - 1), ((x + y) * 7) % 256], -1)
    return (a + rng.integers(-40, 40, a.shape)).clip(0, 255).astype(np.uint8)


def test_jpeg_sweep_against_pil():
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(0)
    for (w, h) in [(1, 1), (2, 2), (5, 3), (23, 17), (101, 77), (640, 480)]:
        for sub in (0, 1, 2):
            for q, rst in ((30, 0), (75, 1), (95, 7), (100, 0)):
                b = io.BytesIO()
                Image.fromarray(_pattern(w, h, rng)).save(b, "JPEG", quality=q, subsampling=sub,
                                                          restart_marker_blocks=rst)
                data = b.getvalue()
                ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
                got = bio.decode_image(data, 2)[..., :3]
                np.testing.assert_array_equal(got, ref, err_msg=f"{w}x{h} sub={sub} q={q} rst={rst}")


def test_unsupported_and_corrupt_streams():
    d, _ = _fixtures()
    good = d["jpeg_64x48_s2_q90_r0__bytes"].tobytes()
    with pytest.raises(bfa.BFError):
        bio.decode_image(good[:2] + b"\x00" * 8, 2)  # no marker after SOI
    with pytest.raises(bfa.BFError):
        bio.decode_image(good[: len(good) // 3], 2)  # truncated inside a segment / the scan
    # a progressive stream (SOF2) is refused with BF_ERR_ARG, not misdecoded
    Image = pytest.importorskip("PIL.Image")
    b = io.BytesIO()
    Image.fromarray(_pattern(16, 16, np.random.default_rng(1))).save(b, "JPEG", progressive=True)
    with pytest.raises(bfa.BFError, match="progressive"):
        bio.decode_image(b.getvalue(), 2)
    png = d["png_45x31_RGB__bytes"].tobytes()
    with pytest.raises(bfa.BFError):
        bio.decode_image(b"\x89PNG\r\n\x1a\n" + struct.pack(">I", 13) + b"IHDR" + b"\x00" * 17, 1)
    with pytest.raises(bfa.BFError):
        bio.decode_image(png[:40], 1)


def _png_chunk(kind: bytes, body: bytes) -> bytes:
    import zlib
    return struct.pack(">I", len(body)) + kind + body + struct.pack(">I", zlib.crc32(kind + body) & 0xFFFFFFFF)


def test_hostile_headers_refused_before_allocation():
    """Crafted headers: a PNG whose IHDR claims 2^16 x 2^16 or 2^31 x 1 pixels (so that
    (stride + 1) * H or W * H * 4 would wrap a small zlib stream past the size check), and a JPEG SOS
    segment of length 0 at the end of the buffer, are rejected with an error, never decoded."""
    import zlib
    for w, h in ((1 << 16, 1 << 16), (1 << 31, 1), (0xFFFFFFFF, 0xFFFFFFFF)):
        ihdr = struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)
        png = (b"\x89PNG\r\n\x1a\n" + _png_chunk(b"IHDR", ihdr) + _png_chunk(b"IDAT", zlib.compress(b"\x00" * 64))
               + _png_chunk(b"IEND", b""))
        with pytest.raises(bfa.BFError, match="limit"):
            bio.decode_image(png, 1)
    d, _ = _fixtures()
    good = d["jpeg_64x48_s2_q90_r0__bytes"].tobytes()
    sos = good.index(b"\xff\xda")
    with pytest.raises(bfa.BFError):
        bio.decode_image(good[:sos] + b"\xff\xda\x00\x02", 2)  # SOS with an empty body at the buffer's end
    # a SOF0 claiming 65535 x 65535 (4.3 G pixels) is refused before its planes are allocated
    sof = good.index(b"\xff\xc0")
    big = bytearray(good)
    big[sof + 5:sof + 9] = b"\xff\xff\xff\xff"
    with pytest.raises(bfa.BFError, match="limit"):
        bio.decode_image(bytes(big), 2)
