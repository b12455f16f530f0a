"""Standalone per-frame input work on one GPU: CUDAImageManager::process (erode x2, bilateral filter)
and CUDACache::storeFrame at the north-star 640x480 with the bundling defaults, on a synthetic
depth image (slanted planes with holes). Run under `rocprofv3 --kernel-trace --stats` for the
per-kernel times; prints the wall time per frame of each stage (synchronized, launch included).
Usage: python tools/time_preproc.py [frames]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bundlefusion_amd as bfa  # noqa: E402
from bundlefusion_amd import DeviceArray  # noqa: E402
from bundlefusion_amd.cache import CUDACache, cache_options  # noqa: E402
from bundlefusion_amd.io import Preprocessor, preprocess_options  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    W, H = 640, 480
    rng = np.random.default_rng(7)
    yy, xx = np.mgrid[0:H, 0:W]
    depth = (800 + 2.0 * xx + 1.5 * yy + rng.normal(0, 3, (H, W))).astype(np.float64)
    depth[(xx // 80 + yy // 60) % 5 == 0] += 400  # depth edges
    depth[rng.random((H, W)) < 0.03] = 0  # holes
    d16 = DeviceArray.from_host(depth.clip(0, 65535).astype(np.uint16))
    rgbx = DeviceArray.from_host(rng.integers(0, 256, (H, W, 4), dtype=np.uint8))
    dout = DeviceArray((H, W), np.float32)
    cout = DeviceArray((H, W, 4), np.uint8)
    pre = Preprocessor((W, H), (W, H), (W, H), preprocess_options())
    cache = CUDACache(cache_options(W, H, 525.0, 525.0, 319.5, 239.5, n + 10))
    for _ in range(10):
        pre.run(d16, rgbx, dout, cout)
        cache.storeFrame(dout, cout, W, H)
    bfa.check(bfa.lib().bf_device_synchronize())
    t = time.perf_counter()
    for _ in range(n):
        pre.run(d16, rgbx, dout, cout)
    t_pre = (time.perf_counter() - t) / n
    t = time.perf_counter()
    for _ in range(n):
        cache.storeFrame(dout, cout, W, H)
    bfa.check(bfa.lib().bf_device_synchronize())
    t_cache = (time.perf_counter() - t) / n
    print(f"preprocess {1e6 * t_pre:.1f} us/frame (synchronized), cache store {1e6 * t_cache:.1f} us/frame (queued)")


if __name__ == "__main__":
    main()
