"""Python binding of the reconstruction loop (bf_recon_*) and of the re-integration queue
(bf_traj_*): mirrors of DepthSensing.cpp's frame loop and TrajectoryManager
(Source/TrajectoryManager.h:6-118)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import check, lib
from .abi import (ENTRYJ_DTYPE, BFEndSequenceOptions, BFEndSequenceResult, BFFixOp, BFQueueEvent, BFReconOptions, BFReconStats,
                  BFSolveResult, BFTsdfStats)

FIX_DEINTEGRATE, FIX_INTEGRATE, FIX_REINTEGRATE, OP_GC = 1, 2, 3, 4


def _mat(T):
    a = np.ascontiguousarray(np.asarray(T, np.float32).reshape(16))
    return (C.c_float * 16)(*a.tolist())


class TrajectoryManager:
    """bf_traj_*: addFrame / updateOptimizedTransform / reintegrate() list logic."""

    INTEGRATED, NOT_INTEGRATED_NO_TRANSFORM = 0, 1

    def __init__(self, max_frames: int, top_n_active: int = 30, min_pose_dist_sqrt: float = 0.0):
        self.h = C.c_void_p()
        check(lib().bf_traj_create(C.c_uint32(max_frames), C.c_uint32(top_n_active), C.c_float(min_pose_dist_sqrt),
                                   C.byref(self.h)))

    def __del__(self):
        try:
            if self.h:
                lib().bf_traj_destroy(self.h)
        except Exception:
            pass

    def add_frame(self, typ: int, T, idx: int):
        check(lib().bf_traj_add_frame(self.h, C.c_int32(typ), _mat(T if T is not None else np.zeros(16)), C.c_uint32(idx)))

    def update_optimized(self, T: np.ndarray):
        T = np.ascontiguousarray(np.asarray(T, np.float32).reshape(-1, 16))
        check(lib().bf_traj_update_optimized(self.h, T.ctypes.data_as(C.c_void_p), C.c_uint32(T.shape[0])))

    def next_fixes(self, max_fixes: int = 10):
        ops = (BFFixOp * max(1, max_fixes))()
        n = C.c_uint32()
        check(lib().bf_traj_next_fixes(self.h, C.c_uint32(max_fixes), ops, C.byref(n)))
        return [(ops[i].kind, ops[i].frame, np.array(ops[i].oldT[:], np.float32), np.array(ops[i].newT[:], np.float32))
                for i in range(n.value)]

    def frame_info(self, idx: int):
        t = C.c_int32()
        d = C.c_float()
        check(lib().bf_traj_frame_info(self.h, C.c_uint32(idx), C.byref(t), C.byref(d)))
        return t.value, d.value


def pose_helper_matrix_to_pose(T) -> np.ndarray:
    out = (C.c_float * 6)()
    check(lib().bf_pose_helper_matrix_to_pose(_mat(T), out))
    return np.array(out[:], np.float32)


def recon_options(max_frames: int, **kw) -> BFReconOptions:
    o = BFReconOptions()
    o.maxFrames = max_frames
    o.useLocalDense = 1
    for k, v in kw.items():
        if k == "cacheIntrinsics":
            o.cacheIntrinsics[:] = [float(x) for x in v]
        else:
            setattr(o, k, v)
    return o


class Recon:
    """bf_recon_*: frame loop with on-the-fly re-integration and local/global BA."""

    def __init__(self, params, cam, opts: BFReconOptions, scene_opts=None):
        self.h = C.c_void_p()
        self.cam = cam
        self.params = params
        check(lib().bf_recon_create(C.byref(params), C.byref(scene_opts) if scene_opts is not None else None,
                                    C.byref(cam), C.byref(opts), C.byref(self.h)))

    @classmethod
    def borrowed(cls, handle: C.c_void_p, params, cam, owner=None):
        """A view of a loop owned elsewhere (bf_app_recon): never destroyed through this object."""
        r = cls.__new__(cls)
        r.h, r.params, r.cam, r._borrowed, r._owner = handle, params, cam, True, owner
        return r

    def close(self):
        if self.h and not getattr(self, "_borrowed", False):
            lib().bf_recon_destroy(self.h)
        self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_frame(self, f: int, depth_ptr: int, color_ptr: int, cache=None, Tinc=None):
        Tinc = np.eye(4, dtype=np.float32) if Tinc is None else Tinc
        check(lib().bf_recon_set_frame(self.h, C.c_uint32(f), C.c_void_p(depth_ptr), C.c_void_p(color_ptr),
                                       C.byref(cache) if cache is not None else None, _mat(Tinc)))

    def set_local_correspondences(self, submap: int, corr_ptr: int, n: int):
        check(lib().bf_recon_set_local_correspondences(self.h, C.c_uint32(submap), C.c_void_p(corr_ptr), C.c_uint32(n)))

    def set_global_correspondences(self, corr_ptr: int, n: int, prefix: np.ndarray):
        prefix = np.ascontiguousarray(prefix, np.uint32)
        self._prefix = prefix
        check(lib().bf_recon_set_global_correspondences(self.h, C.c_void_p(corr_ptr), C.c_uint32(n),
                                                        prefix.ctypes.data_as(C.c_void_p), C.c_uint32(len(prefix))))

    def set_comm(self, comm):
        """Shard the global solve's normal equations over comm's ranks (bundlefusion_amd.dist.Comm)."""
        check(lib().bf_recon_set_comm(self.h, comm.h if comm is not None else None))

    def set_initial_pose(self, T0):
        check(lib().bf_recon_set_initial_pose(self.h, _mat(T0)))

    def process_frame(self, f: int):
        check(lib().bf_recon_process_frame(self.h, C.c_uint32(f)))

    def finish(self):
        check(lib().bf_recon_finish(self.h))

    def reintegrate(self):
        check(lib().bf_recon_reintegrate(self.h))

    def end_solve(self, dense_depth_weight: float = 0.0):
        """One end-of-sequence global solve (OnlineBundler.cpp:171-197, 373-398); 15 = the
        USE_GLOBAL_DENSE_AT_END solve. Returns (result dict, device ms)."""
        r = BFSolveResult()
        ms = C.c_float()
        check(lib().bf_recon_end_solve(self.h, C.c_float(dense_depth_weight), C.byref(r), C.byref(ms)))
        return {k: getattr(r, k) for k, _ in BFSolveResult._fields_}, ms.value

    def end_sequence(self, num_solve_frames_before_exit: int = 30, dense_at_end: bool = True,
                     dense_frame_limit: int = 10000, dense_depth_weight: float = 15.0, max_past_end_frames: int = 0):
        """The render loop past the last frame (bf_recon_end_sequence: OnlineBundler.cpp:167-196, 373-408;
        DepthSensing.cpp:1114-1126): the last submap, s_numSolveFramesBeforeExit global solves (the last with
        the dense term), then re-integration until the queue is empty. Returns the result as a dict."""
        o = BFEndSequenceOptions(int(num_solve_frames_before_exit), 0 if dense_at_end else 1, int(dense_frame_limit),
                                 float(dense_depth_weight), int(max_past_end_frames))
        r = BFEndSequenceResult()
        check(lib().bf_recon_end_sequence(self.h, C.byref(o), C.byref(r)))
        out = {k: getattr(r, k) for k, _ in BFEndSequenceResult._fields_ if k != "last"}
        out["last"] = {k: getattr(r.last, k) for k, _ in BFSolveResult._fields_}
        return out

    def attach_cache(self, cache):
        """CUDACache::storeFrame per processed frame (OnlineBundler.cpp:199-204); cache: cache.CUDACache."""
        self._cache = cache
        check(lib().bf_recon_attach_cache(self.h, cache.h if cache is not None else None))

    def attach_preproc(self, pre):
        """CUDAImageManager::process per processed frame (DepthSensing.cpp:986); pre: io.Preprocessor."""
        self._preproc = pre
        check(lib().bf_recon_attach_preproc(self.h, pre.h if pre is not None else None))

    def set_frame_raw(self, f: int, depth_u16_ptr: int, rgbx_ptr: int):
        check(lib().bf_recon_set_frame_raw(self.h, C.c_uint32(f), C.c_void_p(depth_u16_ptr), C.c_void_p(rgbx_ptr)))

    def frame_ready(self, f: int, stream: int):
        """bf_recon_frame_ready: frame f's frame-store images are being written on `stream` (a hipStream_t);
        the loop's scene stream waits for that work on the device"""
        check(lib().bf_recon_frame_ready(self.h, C.c_uint32(f), C.c_void_p(stream)))

    def set_frame_source(self, f: int, depth_ptr: int, color_ptr: int, color_w: int, color_h: int):
        check(lib().bf_recon_set_frame_source(self.h, C.c_uint32(f), C.c_void_p(depth_ptr), C.c_void_p(color_ptr),
                                              C.c_uint32(color_w), C.c_uint32(color_h)))

    def optimized_trajectory(self) -> np.ndarray:
        """TrajectoryManager::getOptimizedTransforms: the trajectory StopScanningAndExit saves."""
        n = C.c_uint32()
        check(lib().bf_recon_optimized_trajectory(self.h, None, C.c_uint32(0), C.byref(n)))
        T = np.zeros((max(1, n.value), 4, 4), np.float32)
        check(lib().bf_recon_optimized_trajectory(self.h, T.ctypes.data_as(C.c_void_p), C.c_uint32(n.value), C.byref(n)))
        return T[:n.value]

    def queue_trace(self):
        """recordOps: the TrajectoryManager call sequence as a list of (kind, frame, payload):
        0 addFrame -> 4x4 T; 1 updateOptimizedTransform -> [count,4,4]; 2 fix loop -> list of
        (kind, frame, oldT, newT); 3 exit check -> active op count."""
        ne, nt, nf = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(lib().bf_recon_queue_trace(self.h, None, 0, C.byref(ne), None, 0, C.byref(nt), None, 0, C.byref(nf)))
        ev = (BFQueueEvent * max(1, ne.value))()
        T = np.zeros((max(1, nt.value), 4, 4), np.float32)
        fx = (BFFixOp * max(1, nf.value))()
        check(lib().bf_recon_queue_trace(self.h, ev, ne.value, C.byref(ne), T.ctypes.data_as(C.c_void_p), nt.value,
                                         C.byref(nt), fx, nf.value, C.byref(nf)))
        out = []
        for e in ev[:ne.value]:
            if e.kind == 0:
                out.append((0, e.frame, T[e.offset]))
            elif e.kind == 1:
                out.append((1, e.count, T[e.offset:e.offset + e.count]))
            elif e.kind == 2:
                out.append((2, e.count, [(fx[i].kind, fx[i].frame, np.array(fx[i].oldT[:], np.float32),
                                          np.array(fx[i].newT[:], np.float32)) for i in range(e.offset, e.offset + e.count)]))
            else:
                out.append((3, e.count, None))
        return out

    def submap_poses(self, s: int, max_keyframes: int, submap_size: int = 10):
        """recordOps history of submap s: (local float32[n,4,4], global float32[k,4,4], valid int32[k], local_ok)."""
        loc = np.zeros((submap_size + 1, 4, 4), np.float32)
        glo = np.zeros((max_keyframes, 4, 4), np.float32)
        val = np.zeros(max_keyframes, np.int32)
        nl, nk, ok = C.c_uint32(), C.c_uint32(), C.c_int32()
        check(lib().bf_recon_submap_poses(self.h, C.c_uint32(s), loc.ctypes.data_as(C.c_void_p),
                                          glo.ctypes.data_as(C.c_void_p), val.ctypes.data_as(C.c_void_p), C.byref(nl),
                                          C.byref(nk), C.byref(ok)))
        return loc[:nl.value], glo[:nk.value], val[:nk.value], bool(ok.value)

    def synchronize(self):
        check(lib().bf_recon_synchronize(self.h))

    def stats(self) -> dict:
        s = BFReconStats()
        check(lib().bf_recon_stats(self.h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in BFReconStats._fields_}

    def reset_stats(self):
        check(lib().bf_recon_reset_stats(self.h))

    def scene_stats(self) -> dict:
        s = BFTsdfStats()
        check(lib().bf_recon_scene_stats(self.h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in BFTsdfStats._fields_}

    def scene_capacity(self) -> dict:
        """bf_recon_scene_capacity: the scene's error bits, peak alloc candidates against the capacity, heap."""
        from .abi import BFSceneCapacity
        c = BFSceneCapacity()
        check(lib().bf_recon_scene_capacity(self.h, C.byref(c)))
        return {k: getattr(c, k) for k, _ in BFSceneCapacity._fields_}

    def capture_global_solve(self, submap: int) -> None:
        """Test hook: keep the inputs / outcome of submap's in-loop global solve (bf_recon_capture_global_solve)."""
        check(lib().bf_recon_capture_global_solve(self.h, C.c_uint32(submap)))

    def captured_global_solve(self) -> dict:
        """{corr_in, corr_out (EntryJ), rot_in, trans_in, rot_out, trans_out [k, 3], valid [k]} of the capture."""
        n, k = C.c_uint32(), C.c_uint32()
        check(lib().bf_recon_captured_global_solve(self.h, None, None, 0, C.byref(n), None, None, None, 0, C.byref(k)))
        ci, co = np.zeros(n.value, ENTRYJ_DTYPE), np.zeros(n.value, ENTRYJ_DTYPE)
        pi, po = np.zeros(6 * k.value, np.float32), np.zeros(6 * k.value, np.float32)
        val = np.zeros(k.value, np.int32)
        check(lib().bf_recon_captured_global_solve(self.h, ci.ctypes.data_as(C.c_void_p), co.ctypes.data_as(C.c_void_p),
                                                   C.c_uint32(n.value), C.byref(n), pi.ctypes.data_as(C.c_void_p),
                                                   po.ctypes.data_as(C.c_void_p), val.ctypes.data_as(C.c_void_p),
                                                   C.c_uint32(k.value), C.byref(k)))
        K = k.value
        return dict(corr_in=ci, corr_out=co, rot_in=pi[:3 * K].reshape(K, 3), trans_in=pi[3 * K:].reshape(K, 3),
                    rot_out=po[:3 * K].reshape(K, 3), trans_out=po[3 * K:].reshape(K, 3), valid=val)

    def set_render(self, rp) -> None:
        """visualizeFrame's render after every frame's integration (bf_recon_set_render); None stops."""
        check(lib().bf_recon_set_render(self.h, C.byref(rp) if rp is not None else None))

    def render_output(self):
        """The loop's last per-frame render: device pointers (depth, depth4, normals, colors)."""
        p = [C.c_void_p() for _ in range(4)]
        check(lib().bf_recon_render_output(self.h, *[C.byref(x) for x in p]))
        return tuple(x.value for x in p)

    def heap_free_count(self) -> int:
        c = C.c_uint32()
        check(lib().bf_recon_heap_free_count(self.h, C.byref(c)))
        return c.value

    def trajectory(self, n: int) -> np.ndarray:
        T = np.zeros((n, 4, 4), np.float32)
        check(lib().bf_recon_trajectory(self.h, T.ctypes.data_as(C.c_void_p), C.c_uint32(n)))
        return T

    def raycast_device(self, T, rp, outs):
        """render into preallocated DeviceArrays (depth, depth4, normals, colors)"""
        check(lib().bf_recon_raycast(self.h, _mat(T), C.byref(rp), *[o.ptr for o in outs]))

    def extract_mesh_device(self, mc, out):
        """StopScanningAndExtractIsoSurfaceMC into a preallocated DeviceArray of mc.maxNumTriangles x 72 B;
        returns (written, total)."""
        n, total = C.c_uint32(), C.c_uint32()
        check(lib().bf_recon_extract_mesh(self.h, C.byref(mc), out.ptr, C.byref(n), C.byref(total)))
        return n.value, total.value

    def render_stats(self) -> dict:
        from .abi import BFRenderStats
        r = BFRenderStats()
        check(lib().bf_recon_render_stats(self.h, C.byref(r)))
        return {k: getattr(r, k) for k, _ in BFRenderStats._fields_}

    def render_time(self):
        ms = C.c_double()
        n = C.c_uint64()
        check(lib().bf_recon_render_time(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def export(self):
        """(hash entries, heap, heapCounter, voxels) of the loop's scene, as SceneRepHashSDF.export."""
        from .abi import HASH_ENTRY_DTYPE, VOXEL_DTYPE
        E = self.params.hashNumBuckets * 4
        B = self.params.numSDFBlocks
        hash_ = np.empty(E, HASH_ENTRY_DTYPE)
        heap = np.empty(B, np.uint32)
        hc = C.c_uint32()
        vox = np.empty(B * 512, VOXEL_DTYPE)
        check(lib().bf_recon_export(self.h, hash_.ctypes.data_as(C.c_void_p), heap.ctypes.data_as(C.c_void_p),
                                    C.byref(hc), vox.ctypes.data_as(C.c_void_p)))
        return hash_, heap, hc.value, vox

    def export_blocks(self) -> np.ndarray:
        """int32 [n, 4] {x, y, z, allocated} of heap blocks [0, highWater) (bf_recon_export_blocks)."""
        n = C.c_uint32()
        check(lib().bf_recon_export_blocks(self.h, None, C.c_uint32(0), C.byref(n)))
        out = np.zeros((max(1, n.value), 4), np.int32)
        check(lib().bf_recon_export_blocks(self.h, out.ctypes.data_as(C.c_void_p), C.c_uint32(n.value), C.byref(n)))
        return out[:n.value]

    def op_log(self):
        n = C.c_uint32()
        check(lib().bf_recon_op_log(self.h, None, C.c_uint32(0), C.byref(n)))
        ops = (BFFixOp * max(1, n.value))()
        check(lib().bf_recon_op_log(self.h, ops, C.c_uint32(n.value), C.byref(n)))
        return [(ops[i].kind, ops[i].frame, np.array(ops[i].oldT[:], np.float32), np.array(ops[i].newT[:], np.float32))
                for i in range(n.value)]
