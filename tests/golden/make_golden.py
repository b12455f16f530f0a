"""Generates tests/golden/*.npz from the CPU oracle (run: python tests/golden/make_golden.py).

The reference cannot be built or run in this environment ("Oracle"), so these
fixtures are regression pins of the oracle's own output on seeded synthetic input, not
reference outputs."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import bundlefusion_amd as bfa  # noqa: E402
from oracle_lib import OracleScene, blocks_of  # noqa: E402


def tsdf_frame0():
    scene = bfa.synth_scene(0)
    cam = bfa.depth_camera(80, 60, fx=577.87 / 8, fy=577.87 / 8)
    p = bfa.hash_params(voxel_size=0.02, num_buckets=1 << 14, num_blocks=1 << 13)
    T = bfa.synth_pose(0)
    d, c = bfa.synth_render_host(scene, T, cam, 1, 0)
    o = OracleScene(p)
    o.integrate(T, d, c, cam)
    h, _, _, vox = o.export()
    b = blocks_of(h)
    keys = np.array(sorted(b), np.int32)
    idx = np.array([b[tuple(k)] for k in keys.tolist()])[:, None] + np.arange(512)[None, :]
    v = vox[idx.ravel()]
    return keys, v["sdf"].copy(), v["weight"].copy(), v["color"].copy(), o.getHeapFreeCount()


def sens_fixture():
    """tests/golden/sens_3x40x30.sens + .npz: the independent Appendix-B encoder of tests/test_io.py on
    seeded frames (a layout pin for the C++ reader, not a reference output)."""
    from test_io import encode_sens, synth_frames
    depth, rgbx, poses, K = synth_frames(F=3, w=40, h=30, seed=0)
    open(os.path.join(HERE, "sens_3x40x30.sens"), "wb").write(encode_sens(depth, rgbx, poses, K))
    np.savez_compressed(os.path.join(HERE, "sens_3x40x30.npz"), depth=depth, rgbx=rgbx, poses=poses)


if __name__ == "__main__":
    sens_fixture()
    keys, sdf, weight, color, heap_free = tsdf_frame0()
    np.savez_compressed(os.path.join(HERE, "tsdf_frame0_80x60.npz"), keys=keys, sdf=sdf, weight=weight,
                        color=color, heap_free=np.int64(heap_free))
    print("wrote", len(keys), "blocks")
