"""Standalone global-solve timing at the bench's final problem (development tool)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import bundlefusion_amd as bfa  # noqa: E402
from bundlefusion_amd import solver as bs  # noqa: E402

sys.path.insert(0, os.path.join(REPO))
from bench import global_solve_timing  # noqa: E402


class _S:  # minimal stream stand-in: GT keyframes + global correspondences
    def __init__(self, K, S=10):
        self.S = S
        self.gt = np.stack([bfa.synth_pose(i) for i in range(K * S)]).astype(np.float32)
        sc = bfa.synth_scene(0)
        g = bs.synth_correspondences(sc, self.gt[::S][:K], bfa.depth_camera(640, 480), max_per_pair=25,
                                     outlier_frac=0.02, seed=2)
        order = np.argsort(np.maximum(g["i"], g["j"]), kind="stable")
        self.global_host = g[order]
        mx = np.maximum(self.global_host["i"], self.global_host["j"])
        self.global_prefix = np.searchsorted(mx, np.arange(K), side="right").astype(np.uint32)


if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    st = _S(K)
    print(global_solve_timing(st, K, reps=3))
