"""Python binding of the dense-term frame cache (bf_cache_*): mirror of CUDACache
(/root/reference/FriedLiver/Source/CUDACache.h/.cpp)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import DeviceArray, check, lib
from .abi import BFCachedFrame, BFCacheOptions


def cache_options(input_width, input_height, fx, fy, cx, cy, max_frames, width=80, height=60, color_sigma=2.5,
                  depth_sigma_d=1.0, depth_sigma_r=0.05) -> BFCacheOptions:
    """Bundler.cpp:33-38 with zParametersBundlingDefault.txt (s_downsampledWidth/Height 80x60,
    s_colorDownSigma 2.5, s_depthDownSigmaD 1.0, s_depthDownSigmaR 0.05)."""
    o = BFCacheOptions()
    o.inputWidth, o.inputHeight, o.width, o.height, o.maxFrames = input_width, input_height, width, height, max_frames
    K = np.eye(4, dtype=np.float32)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = fx, fy, cx, cy
    o.inputIntrinsics[:] = K.ravel().tolist()
    o.colorSigma, o.depthSigmaD, o.depthSigmaR = color_sigma, depth_sigma_d, depth_sigma_r
    return o


class CUDACache:
    """CUDACache over bf_cache_* (frames stay on the device; frame(i) hands out BFCachedFrame pointers)."""

    def __init__(self, opts: BFCacheOptions):
        self.opts = opts
        self.h = C.c_void_p()
        check(lib().bf_cache_create(C.byref(opts), C.byref(self.h)))

    def close(self):
        if self.h:
            lib().bf_cache_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def storeFrame(self, depth, color, color_width: int, color_height: int) -> int:
        """depth / color: DeviceArray or raw device addresses (int)."""
        def ptr(a):
            return a.ptr if isinstance(a, DeviceArray) else C.c_void_p(int(a))
        i = C.c_uint32()
        check(lib().bf_cache_store_frame(self.h, ptr(depth), ptr(color), C.c_uint32(color_width),
                                         C.c_uint32(color_height), C.byref(i)))
        return i.value

    def copyCacheFrameFrom(self, other: "CUDACache", frame: int) -> int:
        i = C.c_uint32()
        check(lib().bf_cache_copy_frame_from(self.h, other.h, C.c_uint32(frame), C.byref(i)))
        return i.value

    def incrementCache(self):
        check(lib().bf_cache_increment(self.h))

    def getNumFrames(self) -> int:
        n = C.c_uint32()
        check(lib().bf_cache_num_frames(self.h, C.byref(n)))
        return n.value

    def frame(self, i: int) -> BFCachedFrame:
        f = BFCachedFrame()
        check(lib().bf_cache_frame(self.h, C.c_uint32(i), C.byref(f)))
        return f

    def intrinsics(self):
        K = (C.c_float * 16)()
        Ki = (C.c_float * 16)()
        check(lib().bf_cache_intrinsics(self.h, K, Ki))
        return np.array(K[:], np.float32).reshape(4, 4), np.array(Ki[:], np.float32).reshape(4, 4)

    def synchronize(self):
        check(lib().bf_cache_synchronize(self.h))

    def download(self, i: int) -> dict:
        """One cache frame to host numpy arrays (tests)."""
        self.synchronize()
        f = self.frame(i)
        W, H = self.opts.width, self.opts.height
        out = {}
        for name, shape, dt in (("depth", (H, W), np.float32), ("campos", (H, W, 4), np.float32),
                                ("normals", (H, W, 4), np.float32), ("normalsU8", (H, W, 4), np.uint8),
                                ("intensity", (H, W), np.float32), ("intensityDeriv", (H, W, 2), np.float32)):
            a = np.empty(shape, dt)
            check(lib().bf_memcpy_d2h(a.ctypes.data_as(C.c_void_p), C.c_void_p(getattr(f, name)), C.c_size_t(a.nbytes)))
            out[name] = a
        return out
