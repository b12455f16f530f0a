"""ctypes binding of the oracle's reconstruction-loop restatement (oracle/recon.cpp: OnlineBundler's
local -> global state machine + TrajectoryManager, synchronous order) — test infrastructure only."""
from __future__ import annotations

import ctypes as C

import numpy as np

from bundlefusion_amd.abi import BFCachedFrame, BFFixOp
from oracle_lib import lib as _olib


class ORReconParams(C.Structure):
    _fields_ = [("maxFrames", C.c_uint32), ("submapSize", C.c_uint32), ("maxFrameFixes", C.c_uint32),
                ("topNActive", C.c_uint32), ("minPoseDistSqrt", C.c_float), ("localNonLin", C.c_uint32),
                ("localLin", C.c_uint32), ("globalNonLin", C.c_uint32), ("globalLin", C.c_uint32),
                ("maxKeyframes", C.c_uint32), ("maxCorrPerImageLocal", C.c_uint32),
                ("maxCorrPerImageGlobal", C.c_uint32), ("maxResidualThresh", C.c_float), ("useLocalDense", C.c_int32),
                ("cacheWidth", C.c_uint32), ("cacheHeight", C.c_uint32), ("cacheIntrinsics", C.c_float * 4),
                ("disableEarlyOut", C.c_uint32), ("disableLocalVerify", C.c_int32),
                ("verifyOptDistThresh", C.c_float), ("verifyOptPercentThresh", C.c_float),
                ("projCorrDistThresh", C.c_float), ("projCorrNormalThresh", C.c_float),
                ("verifyOptErrThresh", C.c_float), ("verifyOptCorrThresh", C.c_float)]


class ORReconStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("localSolves", "globalSolves", "localPcgIterations", "globalPcgIterations",
                                          "removedPairs", "localVerifications", "invalidLocals", "endSolves")]


def _cap(max_corr, max_images):
    """clamp(maxRes / maxImages, 1000, 4000), CUDASolverBundling.cpp:37"""
    return int(min(4000, max(1000, max_corr // max_images)))


class OracleRecon:
    def __init__(self, F, T0, cache_intrinsics, S=10, max_keyframes=None, max_local_corr=None, max_global_corr=None,
                 cache_w=80, cache_h=60, use_local_dense=True, verify=True):
        L = _olib()
        for name, res, args in (
                ("or_recon_create", C.c_void_p, [C.c_void_p, C.c_void_p]), ("or_recon_destroy", None, [C.c_void_p]),
                ("or_recon_set_frame", None, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
                ("or_recon_set_local_corr", None, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
                ("or_recon_set_global_corr", None, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
                ("or_recon_process_frame", None, [C.c_void_p, C.c_uint32]), ("or_recon_finish", None, [C.c_void_p]),
                ("or_recon_append_global_corr", None, [C.c_void_p, C.c_void_p, C.c_uint32]),
                ("or_recon_reintegrate", None, [C.c_void_p]), ("or_recon_end_solve", None, [C.c_void_p, C.c_float]),
                ("or_recon_op_log", C.c_uint32, [C.c_void_p, C.c_void_p, C.c_uint32]),
                ("or_recon_submap_poses", C.c_int, [C.c_void_p, C.c_uint32] + [C.c_void_p] * 6),
                ("or_recon_trajectory", None, [C.c_void_p, C.c_void_p, C.c_uint32]),
                ("or_recon_stats", None, [C.c_void_p, C.c_void_p]),
                ("or_recon_end_sequence", None, [C.c_void_p, C.c_int32, C.c_int32, C.c_uint32, C.c_float, C.c_uint32,
                                                 C.c_void_p])):
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        self.L = L
        self.S = S
        num_submaps = (F + S - 1) // S
        K = max_keyframes or num_submaps + 1
        self.K = K
        p = ORReconParams()
        p.maxFrames, p.submapSize, p.maxFrameFixes, p.topNActive = F, S, 10, 30
        p.localNonLin, p.localLin, p.globalNonLin, p.globalLin = 2, 100, 3, 150
        p.maxKeyframes = K
        p.maxCorrPerImageLocal = _cap(max_local_corr or (S + 1) * S // 2 * 25, S + 1)
        p.maxCorrPerImageGlobal = _cap(max_global_corr or K * 1000, K)
        p.maxResidualThresh = 0.08
        p.useLocalDense = int(use_local_dense)
        p.cacheWidth, p.cacheHeight = cache_w, cache_h
        p.cacheIntrinsics[:] = [float(x) for x in cache_intrinsics]
        p.disableLocalVerify = 0 if verify else 1
        p.verifyOptDistThresh, p.verifyOptPercentThresh = 0.02, 0.05
        p.projCorrDistThresh, p.projCorrNormalThresh, p.verifyOptErrThresh, p.verifyOptCorrThresh = 0.15, 0.97, 0.05, 0.001
        T0 = np.ascontiguousarray(np.asarray(T0, np.float32).reshape(16))
        self.h = L.or_recon_create(C.addressof(p), T0.ctypes.data)
        self._keep = []

    def close(self):
        if self.h:
            self.L.or_recon_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_frame(self, f, Tinc, cache: dict | None):
        t = np.ascontiguousarray(np.asarray(Tinc, np.float32).reshape(16))
        if cache is None:
            self.L.or_recon_set_frame(self.h, f, t.ctypes.data, None)
            return
        cf = BFCachedFrame()
        for k in ("depth", "campos", "normals", "normalsU8", "intensity", "intensityDeriv"):
            a = np.ascontiguousarray(cache[k])
            self._keep.append(a)
            setattr(cf, k, a.ctypes.data)
        self._keep.append(cf)
        self.L.or_recon_set_frame(self.h, f, t.ctypes.data, C.addressof(cf))

    def set_local_corr(self, s, corr: np.ndarray):
        corr = np.ascontiguousarray(corr)
        self.L.or_recon_set_local_corr(self.h, s, corr.ctypes.data, len(corr))

    def set_global_corr(self, corr: np.ndarray, prefix: np.ndarray):
        corr = np.ascontiguousarray(corr)
        prefix = np.ascontiguousarray(prefix, np.uint32)
        self.L.or_recon_set_global_corr(self.h, corr.ctypes.data, len(corr), prefix.ctypes.data, len(prefix))

    def append_global_corr(self, corr: np.ndarray):
        """keyframe k's entries appended; prefix[k] = the new total (the app's incremental list)"""
        corr = np.ascontiguousarray(corr)
        self.L.or_recon_append_global_corr(self.h, corr.ctypes.data if len(corr) else None, len(corr))

    def process_frame(self, f):
        self.L.or_recon_process_frame(self.h, f)

    def finish(self):
        self.L.or_recon_finish(self.h)

    def reintegrate(self):
        self.L.or_recon_reintegrate(self.h)

    def end_solve(self, dense_depth_weight=0.0):
        self.L.or_recon_end_solve(self.h, dense_depth_weight)

    def end_sequence(self, num_solve_frames_before_exit=30, dense_at_end=True, dense_frame_limit=10000,
                     dense_depth_weight=15.0, max_past_end_frames=0):
        out = np.zeros(5, np.uint32)
        self.L.or_recon_end_sequence(self.h, num_solve_frames_before_exit, 0 if dense_at_end else 1, dense_frame_limit,
                                     dense_depth_weight, max_past_end_frames, out.ctypes.data)
        return dict(zip(("pastEndFrames", "globalSolves", "localSolved", "denseSolve", "queueDrained"), map(int, out)))

    def op_log(self):
        n = self.L.or_recon_op_log(self.h, None, 0)
        ops = (BFFixOp * max(1, n))()
        self.L.or_recon_op_log(self.h, ops, n)
        return [(ops[i].kind, ops[i].frame, np.array(ops[i].oldT[:], np.float32), np.array(ops[i].newT[:], np.float32))
                for i in range(n)]

    def submap_poses(self, s):
        loc = np.zeros((self.S + 1, 4, 4), np.float32)
        glo = np.zeros((self.K, 4, 4), np.float32)
        val = np.zeros(self.K, np.int32)
        nl, nk, ok = C.c_uint32(), C.c_uint32(), C.c_int32()
        r = self.L.or_recon_submap_poses(self.h, s, loc.ctypes.data, glo.ctypes.data, val.ctypes.data, C.addressof(nl),
                                         C.addressof(nk), C.addressof(ok))
        assert r == 0, f"no oracle record of submap {s}"
        return loc[:nl.value], glo[:nk.value], val[:nk.value], bool(ok.value)

    def trajectory(self, n):
        T = np.zeros((n, 4, 4), np.float32)
        self.L.or_recon_trajectory(self.h, T.ctypes.data, n)
        return T

    def stats(self) -> dict:
        s = ORReconStats()
        self.L.or_recon_stats(self.h, C.addressof(s))
        return {k: getattr(s, k) for k, _ in ORReconStats._fields_}
