"""Runs one deterministic 20-op batch at 640x480 / 4 mm (tests/test_tsdf_gpu.py's full-resolution case)
and prints the scene's counters and a voxel checksum: compares library builds (BF_HIP_LIB=...)."""
import os
import sys
import zlib

import numpy as np

_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [_R, os.path.join(_R, "tests")]
import bundlefusion_amd as bfa  # noqa: E402
from tsdf_compare import Pair, render_frames  # noqa: E402
from test_tsdf_gpu import _perturbed  # noqa: E402

scene = bfa.synth_scene(0)
cam = bfa.depth_camera(640, 480)
p = bfa.hash_params(voxel_size=0.004, num_buckets=1 << 20, num_blocks=1 << 18)
pair = Pair(p, cam)
frames = render_frames(scene, cam, list(range(0, 40, 4)))
for k, (T, d, c) in enumerate(frames):
    dd, cc = pair._upload(k, d, c)
    pair.gpu.integrate(T, dd, cc, cam)  # the GPU side only
rng = np.random.default_rng(5)
dev = []
for k, (T, d, c) in enumerate(frames):
    T2 = _perturbed(T, rng, 0.01, rot_deg=0.2)
    for TT, deint in ((T, True), (T2, False)):
        dd, cc = pair._upload(k, d, c)
        dev.append((TT, dd, cc, deint))
s0 = pair.gpu.stats()
pair.gpu.apply_ops(dev, cam)
s1 = pair.gpu.stats()
print({k: s1[k] - s0[k] for k in s1 if k.startswith("batch")})
h, heap, hc, vox = pair.gpu.export()
# order-independent fingerprints of the voxels
w = vox["weight"].astype(np.float64) if "weight" in vox.dtype.names else None
print("heap", hc, "weight>0", int((vox["weight"] > 0).sum()), "sum w", float(vox["weight"].astype(np.float64).sum()),
      "sum sdf", float(vox["sdf"].astype(np.float64).sum()), "sum colour", int(vox["color"].astype(np.int64).sum()))
