"""ctypes binding of the oracle's bundle adjuster (oracle/ba.cpp) + BA test-problem helpers —
test infrastructure only."""
from __future__ import annotations

import ctypes as C

import numpy as np

from bundlefusion_amd.abi import ENTRYJ_DTYPE, BFCachedFrame
from oracle_lib import lib as _olib


class ORSolveParams(C.Structure):
    _fields_ = [("numImages", C.c_uint32), ("numCorr", C.c_uint32), ("nNonLin", C.c_uint32), ("nLin", C.c_uint32),
                ("maxCorrPerImage", C.c_uint32),
                ("weightsSparse", C.POINTER(C.c_float)), ("weightsDenseDepth", C.POINTER(C.c_float)),
                ("weightsDenseColor", C.POINTER(C.c_float)),
                ("cache", C.c_void_p), ("cacheW", C.c_uint32), ("cacheH", C.c_uint32), ("intrinsics", C.c_float * 4),
                ("denseDistThresh", C.c_float), ("denseNormalThresh", C.c_float), ("denseColorThresh", C.c_float),
                ("denseColorGradientMin", C.c_float), ("denseDepthMin", C.c_float), ("denseDepthMax", C.c_float),
                ("denseOverlapSubsample", C.c_uint32), ("disableEarlyOut", C.c_uint32)]


class ORSolveResult(C.Structure):
    _fields_ = [("gnIterations", C.c_uint32), ("pcgIterations", C.c_uint32), ("maxResidual", C.c_float),
                ("maxResidualIndex", C.c_int32), ("finalEnergy", C.c_float)]


def _lib():
    L = _olib()
    if not getattr(L, "_ba_ready", False):
        L.or_ba_solve.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_ba_solve.restype = None
        L.or_pose_to_matrix.argtypes = [C.c_void_p] * 3
        L.or_pose_to_matrix.restype = None
        L.or_matrix_to_pose.argtypes = [C.c_void_p] * 3
        L.or_matrix_to_pose.restype = None
        L._ba_ready = True
    return L


def pose_to_matrix(rot, trans) -> np.ndarray:
    r = np.ascontiguousarray(rot, np.float32)
    t = np.ascontiguousarray(trans, np.float32)
    M = np.empty(16, np.float32)
    _lib().or_pose_to_matrix(r.ctypes.data, t.ctypes.data, M.ctypes.data)
    return M.reshape(4, 4)


def matrix_to_pose(M):
    M = np.ascontiguousarray(np.asarray(M, np.float32).reshape(16))
    r = np.empty(3, np.float32)
    t = np.empty(3, np.float32)
    _lib().or_matrix_to_pose(M.ctypes.data, r.ctypes.data, t.ctypes.data)
    return r, t


def max_corr_per_image(max_images: int, max_corr: int) -> int:
    """clamp(maxRes / maxImages, 1000, 4000), CUDASolverBundling.cpp:37"""
    return int(min(4000, max(1000, max_corr // max_images)))


def _params(N, n_corr, n_nonlin, n_lin, w_sparse, w_depth, w_color, cache, intrinsics, max_corr_per_img, dense, keep):
    p = ORSolveParams()
    p.numImages, p.numCorr, p.nNonLin, p.nLin, p.maxCorrPerImage = N, n_corr, n_nonlin, n_lin, max_corr_per_img
    ws = (C.c_float * n_nonlin)(*w_sparse[:n_nonlin])
    wd = (C.c_float * n_nonlin)(*(w_depth or [0.0] * n_nonlin)[:n_nonlin])
    wc = (C.c_float * n_nonlin)(*(w_color or [0.0] * n_nonlin)[:n_nonlin])
    keep += [ws, wd, wc]
    p.weightsSparse, p.weightsDenseDepth, p.weightsDenseColor = ws, wd, wc
    d = dict(distT=0.15, normT=0.97, colT=0.1, gradMin=0.005, dmin=0.5, dmax=4.0, sub=4)
    if dense:
        d.update(dense)
    p.denseDistThresh, p.denseNormalThresh, p.denseColorThresh = d["distT"], d["normT"], d["colT"]
    p.denseColorGradientMin, p.denseDepthMin, p.denseDepthMax, p.denseOverlapSubsample = d["gradMin"], d["dmin"], d["dmax"], d["sub"]
    if cache is not None:
        K = cache["depth"].shape[0]
        table = (BFCachedFrame * K)()
        for k in range(K):
            for f in ("depth", "campos", "normals", "normalsU8", "intensity", "intensityDeriv"):
                a = np.ascontiguousarray(cache[f][k])
                keep.append(a)
                setattr(table[k], f, a.ctypes.data)
        keep.append(table)
        p.cache = C.addressof(table)
        p.cacheW, p.cacheH = cache["depth"].shape[2], cache["depth"].shape[1]
        p.intrinsics[:] = [float(x) for x in intrinsics]
    return p


def solve(corr: np.ndarray, valid: np.ndarray, rot: np.ndarray, trans: np.ndarray, n_nonlin: int, n_lin: int,
          w_sparse, w_depth=None, w_color=None, cache: dict | None = None, intrinsics=(0, 0, 0, 0),
          max_corr_per_img=4000, dense=None, early_out=True):
    """Oracle solve; returns (rot, trans, corr_after, result dict). Inputs are not modified.
    early_out=False: the reference built without ENABLE_EARLY_OUT (fixed schedule)."""
    corr = np.ascontiguousarray(corr.copy())
    valid = np.ascontiguousarray(valid, np.int32)
    rot = np.ascontiguousarray(rot, np.float32).copy()
    trans = np.ascontiguousarray(trans, np.float32).copy()
    keep = []
    p = _params(valid.shape[0], len(corr), n_nonlin, n_lin, w_sparse, w_depth, w_color, cache, intrinsics,
                max_corr_per_img, dense, keep)
    p.disableEarlyOut = 0 if early_out else 1
    res = ORSolveResult()
    _lib().or_ba_solve(corr.ctypes.data, valid.ctypes.data, C.addressof(p), rot.ctypes.data, trans.ctypes.data,
                       C.addressof(res))
    return rot, trans, corr, {k: getattr(res, k) for k, _ in ORSolveResult._fields_}


def dense_system(valid, rot, trans, cache, intrinsics, w_depth=1.0, w_color=0.0, dense=None):
    """Dense JtJ (6N x 6N, [trans|rot] per image), Jtr, energy sum w r^2 and #overlapping pairs."""
    valid = np.ascontiguousarray(valid, np.int32)
    rot = np.ascontiguousarray(rot, np.float32)
    trans = np.ascontiguousarray(trans, np.float32)
    N = valid.shape[0]
    keep = []
    p = _params(N, 0, 1, 1, [1.0], [w_depth], [w_color], cache, intrinsics, 4000, dense, keep)
    jtj = np.zeros((6 * N, 6 * N), np.float32)
    jtr = np.zeros(6 * N, np.float32)
    e = C.c_double()
    npairs = C.c_uint32()
    L = _lib()
    L.or_ba_dense_system.argtypes = [C.c_void_p] * 8
    L.or_ba_dense_system(valid.ctypes.data, C.addressof(p), rot.ctypes.data, trans.ctypes.data, jtj.ctypes.data,
                         jtr.ctypes.data, C.addressof(e), C.addressof(npairs))
    return jtj, jtr, e.value, npairs.value


class ORVerifyParams(C.Structure):
    _fields_ = [("numImages", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32), ("intrinsics", C.c_float * 4),
                ("distThresh", C.c_float), ("normalThresh", C.c_float), ("errThresh", C.c_float),
                ("corrThresh", C.c_float), ("depthMin", C.c_float), ("depthMax", C.c_float)]


def verify_trajectory(valid, T, cache: dict, intrinsics, dist=0.15, normal=0.97, err=0.05, corr=0.001, dmin=0.1, dmax=3.0):
    """Oracle VerifyTrajectoryCU: (valid flag, pair stats float32[N, N, 3])."""
    valid = np.ascontiguousarray(valid, np.int32)
    N = valid.shape[0]
    T = np.ascontiguousarray(np.asarray(T, np.float32).reshape(N, 16))
    keep = []
    p = _params(N, 0, 1, 1, [1.0], None, None, cache, intrinsics, 4000, None, keep)
    v = ORVerifyParams()
    v.numImages, v.width, v.height = N, p.cacheW, p.cacheH
    v.intrinsics[:] = [float(x) for x in intrinsics]
    v.distThresh, v.normalThresh, v.errThresh, v.corrThresh, v.depthMin, v.depthMax = dist, normal, err, corr, dmin, dmax
    stats = np.zeros((N, N, 3), np.float32)
    L = _lib()
    L.or_verify_trajectory.argtypes = [C.c_void_p] * 5
    L.or_verify_trajectory.restype = C.c_int
    ok = L.or_verify_trajectory(valid.ctypes.data, T.ctypes.data, p.cache, C.addressof(v), stats.ctypes.data)
    return bool(ok), stats


def count_high_residuals(corr: np.ndarray, rot, trans, w=1.0, thresh=0.02) -> int:
    corr = np.ascontiguousarray(corr)
    rot = np.ascontiguousarray(rot, np.float32)
    trans = np.ascontiguousarray(trans, np.float32)
    L = _lib()
    L.or_ba_count_high_residuals.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_float, C.c_float]
    L.or_ba_count_high_residuals.restype = C.c_uint32
    return int(L.or_ba_count_high_residuals(corr.ctypes.data, len(corr), rot.ctypes.data, trans.ctypes.data, w, thresh))


def rotation_angle(R1: np.ndarray, R2: np.ndarray) -> float:
    c = (np.trace(R1[:3, :3].T @ R2[:3, :3]) - 1.0) / 2.0
    return float(np.arccos(np.clip(c, -1.0, 1.0)))
