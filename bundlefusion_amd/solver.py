"""Python binding of the bundle adjuster (bf_solver_*): mirror of CUDASolverBundling
(Source/Solver/CUDASolverBundling.h) plus the synthetic BA-input generators."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import DeviceArray, abi, check, lib
from .abi import ENTRYJ_DTYPE, BFCachedFrame, BFSolveResult, BFSolverOptions, BFVerifyOptions

# SBA weight schedules (Source/SBA.cpp:28-39), indexed by GN iteration
LOCAL_WEIGHTS = dict(sparse=[1.0, 1.0, 1.0], dense_depth=[1.0, 2.0, 3.0], dense_color=[0.0, 0.0, 0.0])
GLOBAL_WEIGHTS_SPARSE_ONLY = dict(sparse=[1.0, 1.0, 1.0], dense_depth=[0.0, 0.0, 0.0], dense_color=[0.0, 0.0, 0.0])
GLOBAL_WEIGHTS_DENSE = dict(sparse=[1.0, 1.0, 1.0], dense_depth=[1.0, 1.0, 2.0], dense_color=[0.1, 0.1, 0.1])


class SolverBundling:
    """CUDASolverBundling over bf_solver_* (all buffers device-resident)."""

    def __init__(self, max_images: int, max_corr: int, opts: BFSolverOptions | None = None,
                 normal_equations: int | None = None, early_out: bool = True, pcg_launch: int = 0,
                 pcg_spin_limit_us: int = 0):
        if normal_equations is not None or not early_out or pcg_launch or pcg_spin_limit_us:
            opts = opts if opts is not None else BFSolverOptions()
            if normal_equations is not None:
                opts.normalEquations = normal_equations
            opts.disableEarlyOut = 0 if early_out else 1
            if pcg_launch:
                opts.pcgLaunch = pcg_launch
            opts.pcgSpinLimitUs = pcg_spin_limit_us
        self.h = C.c_void_p()
        check(lib().bf_solver_create(C.c_uint32(max_images), C.c_uint32(max_corr),
                                     C.byref(opts) if opts is not None else None, C.byref(self.h)))
        self.max_images, self.max_corr = max_images, max_corr

    def close(self):
        if self.h:
            lib().bf_solver_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, corr: DeviceArray, n_corr: int, valid: DeviceArray, n_images: int, n_nonlin: int, n_lin: int,
              w_sparse, w_dense_depth=None, w_dense_color=None, cache: DeviceArray | None = None, cache_w=0, cache_h=0,
              intrinsics=(0, 0, 0, 0), rot: DeviceArray = None, trans: DeviceArray = None, rebuild_jt=True,
              find_max_residual=True):
        ws = (C.c_float * n_nonlin)(*[float(x) for x in w_sparse[:n_nonlin]])
        wd = (C.c_float * n_nonlin)(*[float(x) for x in (w_dense_depth or [0.0] * n_nonlin)[:n_nonlin]])
        wc = (C.c_float * n_nonlin)(*[float(x) for x in (w_dense_color or [0.0] * n_nonlin)[:n_nonlin]])
        intr = (C.c_float * 4)(*[float(x) for x in intrinsics])
        check(lib().bf_solver_solve(self.h, corr.ptr if corr is not None else None, C.c_uint32(n_corr), valid.ptr,
                                    C.c_uint32(n_images), C.c_uint32(n_nonlin), C.c_uint32(n_lin), ws, wd, wc,
                                    cache.ptr if cache is not None else None, C.c_uint32(cache_w), C.c_uint32(cache_h),
                                    intr, rot.ptr, trans.ptr, int(rebuild_jt), int(find_max_residual)))

    def result(self) -> dict:
        r = BFSolveResult()
        check(lib().bf_solver_result(self.h, C.byref(r)))
        return {k: getattr(r, k) for k, _ in BFSolveResult._fields_}

    def synchronize(self):
        check(lib().bf_solver_synchronize(self.h))

    def verify_trajectory(self, T: DeviceArray, valid: DeviceArray, n_images: int, n_corr: int, cache: DeviceArray,
                          cache_w: int, cache_h: int, intrinsics, always=False, pair_stats: DeviceArray | None = None,
                          **thresholds) -> bool:
        """useVerification + VerifyTrajectoryCU after the last solve (CUDASolverBundling.cpp:454-476,
        Bundler.cpp:259-274): True when the submap is accepted."""
        o = BFVerifyOptions()
        for k, v in thresholds.items():
            setattr(o, k, v)
        o.always = int(always)
        intr = (C.c_float * 4)(*[float(x) for x in intrinsics])
        ok = C.c_int()
        check(lib().bf_solver_verify_trajectory(self.h, T.ptr, valid.ptr, C.c_uint32(n_images), C.c_uint32(n_corr),
                                                cache.ptr, C.c_uint32(cache_w), C.c_uint32(cache_h), intr, C.byref(o),
                                                pair_stats.ptr if pair_stats is not None else None, C.byref(ok)))
        return bool(ok.value)

    def set_shard(self, count: int, index: int, comm=None):
        """Build only the pair blocks p % count == index; comm (bundlefusion_amd.dist.Comm) sums them."""
        check(lib().bf_solver_set_shard(self.h, C.c_uint32(count), C.c_uint32(index), comm.h if comm else None))

    def export_pairs(self):
        """(stats float64[P, 28], pairs int32[P, 2]) of the last solve's assembled normal equations."""
        total = C.c_uint32(0)
        check(lib().bf_solver_export_pairs(self.h, None, None, C.c_uint32(0), C.byref(total)))
        n = total.value
        stats = np.zeros((max(n, 1), abi.PAIR_STATS), np.float64)
        ab = np.zeros((max(n, 1), 2), np.int32)
        check(lib().bf_solver_export_pairs(self.h, stats.ctypes.data_as(C.c_void_p), ab.ctypes.data_as(C.c_void_p),
                                           C.c_uint32(n), C.byref(total)))
        return stats[:n], ab[:n]

    def matrices_to_poses(self, T: DeviceArray, n: int, rot: DeviceArray, trans: DeviceArray, valid: DeviceArray):
        check(lib().bf_solver_matrices_to_poses(self.h, T.ptr, C.c_uint32(n), rot.ptr, trans.ptr, valid.ptr))

    def poses_to_matrices(self, rot: DeviceArray, trans: DeviceArray, n: int, T: DeviceArray, valid: DeviceArray):
        check(lib().bf_solver_poses_to_matrices(self.h, rot.ptr, trans.ptr, C.c_uint32(n), T.ptr, valid.ptr))

    def invalidate_image_pair(self, corr: DeviceArray, n: int, i: int, j: int):
        check(lib().bf_solver_invalidate_image_pair(self.h, corr.ptr, C.c_uint32(n), C.c_uint32(i), C.c_uint32(j)))

    def check_invalid_frames(self, valid: DeviceArray, n_images: int, corr: DeviceArray, n_corr: int, comprehensive=True):
        check(lib().bf_solver_check_invalid_frames(self.h, valid.ptr, C.c_uint32(n_images), corr.ptr,
                                                   C.c_uint32(n_corr), int(comprehensive)))


def synth_correspondences(scene, poses: np.ndarray, cam, max_per_pair=25, min_covis=0.3, noise=0.0015,
                          outlier_frac=0.02, seed=2, cap=None) -> np.ndarray:
    poses = np.ascontiguousarray(np.asarray(poses, np.float32).reshape(-1, 16))
    K = poses.shape[0]
    cap = cap or max(1, K * (K - 1) // 2 * max_per_pair)
    out = np.zeros(cap, ENTRYJ_DTYPE)
    n = C.c_uint32()
    check(lib().bf_synth_correspondences(C.byref(scene), poses.ctypes.data_as(C.c_void_p), C.c_uint32(K), C.byref(cam),
                                         C.c_uint32(max_per_pair), C.c_float(min_covis), C.c_float(noise),
                                         C.c_float(outlier_frac), C.c_uint32(seed), out.ctypes.data_as(C.c_void_p),
                                         C.c_uint32(cap), C.byref(n)))
    return out[: n.value].copy()


def synth_cache_frames(scene, poses: np.ndarray, cam) -> dict:
    """Host dense-term cache frames (CUDACache::storeFrame semantics) for every pose."""
    poses = np.asarray(poses, np.float32).reshape(-1, 4, 4)
    K, W, H = poses.shape[0], cam.imageWidth, cam.imageHeight
    out = dict(depth=np.empty((K, H, W), np.float32), campos=np.empty((K, H, W, 4), np.float32),
               normals=np.empty((K, H, W, 4), np.float32), normalsU8=np.empty((K, H, W, 4), np.uint8),
               intensity=np.empty((K, H, W), np.float32), intensityDeriv=np.empty((K, H, W, 2), np.float32))
    for k in range(K):
        check(lib().bf_synth_cache_frame(C.byref(scene), abi.mat(poses[k]), C.byref(cam),
                                         *[out[f][k].ctypes.data_as(C.c_void_p) for f in
                                           ("depth", "campos", "normals", "normalsU8", "intensity", "intensityDeriv")]))
    return out


class DeviceCache:
    """Uploads host cache frames and builds the device BFCachedFrame[] table."""

    FIELDS = ("depth", "campos", "normals", "normalsU8", "intensity", "intensityDeriv")

    def __init__(self, frames: dict):
        self.arrays = {f: DeviceArray.from_host(frames[f]) for f in self.FIELDS}
        K = frames["depth"].shape[0]
        table = (BFCachedFrame * K)()
        for k in range(K):
            for f in self.FIELDS:
                a = frames[f]
                per = a[0].nbytes
                setattr(table[k], f, self.arrays[f].ptr.value + k * per)
        raw = np.frombuffer(bytes(table), dtype=np.uint8)
        self.table = DeviceArray.from_host(raw)
        self.ptr = self.table.ptr
        self.W, self.H = frames["depth"].shape[2], frames["depth"].shape[1]
