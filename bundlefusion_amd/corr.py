"""EntryJ correspondences: the saveSparseCorrsToFile dump format (bf_corr_save / bf_corr_load) and the
depth + pose producer that stands in for the SiftGPU front end (bf_corr_from_depth)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import DeviceArray, check, lib
from .abi import ENTRYJ_DTYPE, BFCorrOptions


def corr_options(width, height, fx, fy, cx, cy, stride=16, max_per_pair=25, min_depth=0.1, max_depth=3.0,
                 depth_thresh=0.02, min_per_pair=1) -> BFCorrOptions:
    o = BFCorrOptions()
    o.intrinsics[:] = [fx, fy, cx, cy]
    K = np.eye(4, dtype=np.float64)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = fx, fy, cx, cy
    o.intrinsicsInv[:] = np.linalg.inv(K).astype(np.float32).ravel().tolist()
    o.width, o.height, o.stride, o.maxPerPair = width, height, stride, max_per_pair
    o.minDepth, o.maxDepth, o.depthThresh = min_depth, max_depth, depth_thresh
    o.minPerPair = min_per_pair
    return o


def corr_from_depth(depth_ptrs, transforms: DeviceArray, transforms_inv: DeviceArray, cur: int, start: int,
                    opts: BFCorrOptions, cap: int):
    """depth_ptrs: sequence of device addresses (one per image). Returns (host EntryJ array, total found)."""
    ptrs = DeviceArray.from_host(np.asarray([int(p) for p in depth_ptrs], np.uint64))
    out = DeviceArray((max(cap, 1),), ENTRYJ_DTYPE)
    n, total = C.c_uint32(), C.c_uint32()
    check(lib().bf_corr_from_depth(ptrs.ptr, transforms.ptr, transforms_inv.ptr, C.c_uint32(cur), C.c_uint32(start),
                                   C.byref(opts), out.ptr, C.c_uint32(cap), C.byref(n), C.byref(total)))
    res = out.download_range(0, 32 * n.value).view(ENTRYJ_DTYPE).copy() if n.value else np.zeros(0, ENTRYJ_DTYPE)
    return res, total.value


def corr_save(path: str, corr: np.ndarray) -> None:
    """Bundler::saveSparseCorrsToFile: uint64 count + raw EntryJ records."""
    c = np.ascontiguousarray(corr, ENTRYJ_DTYPE)
    check(lib().bf_corr_save(os.fsencode(path), c.ctypes.data_as(C.c_void_p), C.c_uint64(len(c))))


def corr_load(path: str) -> np.ndarray:
    n = C.c_uint64()
    check(lib().bf_corr_load(os.fsencode(path), None, C.c_uint64(0), C.byref(n)))
    out = np.zeros(n.value, ENTRYJ_DTYPE)
    check(lib().bf_corr_load(os.fsencode(path), out.ctypes.data_as(C.c_void_p), C.c_uint64(n.value), C.byref(n)))
    return out
