"""Generates tests/golden/image_codec.npz and tests/golden/sens_jpeg_3x64x48.sens with PIL (present in
the build container only; run: python tests/golden/make_image_fixtures.py).

The `.sens` colour stream of the BundleFusion datasets is JPEG (colorCompression 2) or PNG (1); the
reference decodes it through the un-vendored mLib (SensorDataReader.cpp:98-116), so the decoders in
bundlefusion_amd/csrc/image_codec.cpp are pinned against PIL (libjpeg-turbo / zlib) decodes of
streams PIL encoded: every fixture holds the encoded bytes and PIL's RGB output."""
import io
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(os.path.dirname(HERE)), os.path.dirname(HERE)]


def pattern(w, h, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    a = np.stack([x * 255 // max(1, w - 1), y * 255 // max(1, h - 1), ((x + y) * 7) % 256], -1)
    return (a + rng.integers(-40, 40, a.shape)).clip(0, 255).astype(np.uint8)


def main():
    cases = {}
    k = 0
    # JPEG: 4:4:4 / 4:2:2 / 4:2:0, odd sizes, restart intervals, high / low quality, greyscale
    for (w, h) in [(64, 48), (37, 29), (3, 5), (17, 9)]:
        for sub in (0, 1, 2):
            for q, rst in ((90, 0), (50, 3)):
                b = io.BytesIO()
                Image.fromarray(pattern(w, h, k)).save(b, "JPEG", quality=q, subsampling=sub, restart_marker_blocks=rst)
                cases[f"jpeg_{w}x{h}_s{sub}_q{q}_r{rst}"] = b.getvalue()
                k += 1
    b = io.BytesIO()
    Image.fromarray(pattern(33, 21, 99)[..., 0]).save(b, "JPEG", quality=85)
    cases["jpeg_33x21_grey"] = b.getvalue()
    for mode in ("RGB", "RGBA", "L", "P"):
        b = io.BytesIO()
        im = Image.fromarray(pattern(45, 31, 7))
        (im if mode == "RGB" else im.convert(mode)).save(b, "PNG")
        cases[f"png_45x31_{mode}"] = b.getvalue()
    arrays = {}
    for name, data in cases.items():
        arrays[name + "__bytes"] = np.frombuffer(data, np.uint8)
        arrays[name + "__rgb"] = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    # a JPEG-colour .sens (zlib depth), the layout of the copyroom / apt0 recordings
    from test_io import encode_sens, synth_frames
    depth, rgbx, poses, K = synth_frames(F=3, w=64, h=48, seed=1)
    sens = encode_sens(depth, rgbx, poses, K, color_codec="jpeg", jpeg_quality=90)
    open(os.path.join(HERE, "sens_jpeg_3x64x48.sens"), "wb").write(sens)
    # expected colour = PIL's decode of the same JPEG bytes the encoder wrote
    exp = []
    for f in range(3):
        b = io.BytesIO()
        Image.fromarray(np.ascontiguousarray(rgbx[f, ..., :3])).save(b, "JPEG", quality=90)
        exp.append(np.asarray(Image.open(io.BytesIO(b.getvalue())).convert("RGB")))
    arrays["sens_jpeg__rgb"] = np.stack(exp)
    arrays["sens_jpeg__depth"] = depth
    arrays["sens_jpeg__poses"] = poses
    np.savez_compressed(os.path.join(HERE, "image_codec.npz"), **arrays)


if __name__ == "__main__":
    main()
