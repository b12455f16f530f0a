"""bundlefusion_amd — MI355X-native BundleFusion hot path (voxel-hash TSDF + bundle adjuster).

The product is the gfx950 HIP library `libbf_hip.so` behind the C ABI in
include/bf/bf.h. This package is the Python binding used by tests and bench.py:
it loads the in-tree library and fails loudly when it is missing — there is no
CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi
from .abi import (BFDepthCameraParams, BFHashParams, BFMarchingCubesParams, BFRayCastParams, BFSceneOptions,
                  BFSynthScene, BFTsdfStats, HASH_ENTRY_DTYPE, VOXEL_DTYPE)

__all__ = ["lib", "BFError", "DeviceArray", "SceneRepHashSDF", "hash_params", "depth_camera",
           "synth_scene", "synth_pose", "synth_render", "synth_render_host", "mc_params", "mesh_merge", "mesh_save_ply"]

_lib = None


class BFError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"bf error {code}: {msg}")
        self.code = code


def lib() -> C.CDLL:
    """Load bundlefusion_amd/libbf_hip.so (built by __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(abi.LIB_PATH):
            raise ImportError(f"{abi.LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(abi.LIB_PATH)
        for name in abi.header_functions():
            fn = getattr(L, name)
            fn.restype = C.c_char_p if name == "bf_last_error" else C.c_int
        if L.bf_abi_version() != abi.ABI_VERSION:
            raise ImportError(f"{abi.LIB_PATH}: ABI version {L.bf_abi_version()}, the binding expects {abi.ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        raise BFError(rc, lib().bf_last_error().decode(errors="replace"))


def device_count() -> int:
    n = C.c_int(0)
    check(lib().bf_device_count(C.byref(n)))
    return n.value


class DeviceArray:
    """A device allocation (bf_malloc) with numpy-shaped host transfers."""

    def __init__(self, shape, dtype):
        self.shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        self.ptr = C.c_void_p()
        check(lib().bf_malloc(C.byref(self.ptr), C.c_size_t(self.nbytes)))

    @classmethod
    def from_host(cls, a: np.ndarray) -> "DeviceArray":
        a = np.ascontiguousarray(a)
        d = cls(a.shape, a.dtype)
        d.upload(a)
        return d

    def upload(self, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a, dtype=self.dtype)
        assert a.nbytes == self.nbytes
        check(lib().bf_memcpy_h2d(self.ptr, a.ctypes.data_as(C.c_void_p), C.c_size_t(self.nbytes)))

    def download(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        check(lib().bf_memcpy_d2h(out.ctypes.data_as(C.c_void_p), self.ptr, C.c_size_t(self.nbytes)))
        return out

    def download_range(self, offset: int, nbytes: int) -> np.ndarray:
        """nbytes starting at byte offset, as uint8."""
        assert 0 <= offset and offset + nbytes <= self.nbytes
        out = np.empty(nbytes, np.uint8)
        check(lib().bf_memcpy_d2h(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr.value + offset), C.c_size_t(nbytes)))
        return out

    def zero(self) -> None:
        check(lib().bf_memset(self.ptr, 0, C.c_size_t(self.nbytes)))

    def __del__(self):
        try:
            if self.ptr and _lib is not None:
                _lib.bf_free(self.ptr)
                self.ptr = C.c_void_p()
        except Exception:
            pass


# ---- configuration (CUDASceneRepHashSDF::parametersFromGlobalAppState, .h:39-59) ----------
def hash_params(voxel_size=0.010, num_buckets=800000, num_blocks=200000, max_list=7, truncation=0.06,
                trunc_scale=0.02, max_integration_distance=3.0, weight_sample=1, weight_max=99999999) -> BFHashParams:
    """Defaults are zParametersDefault.txt:39-50."""
    p = BFHashParams()
    for i in (0, 5, 10, 15):
        p.rigidTransform.m[i] = 1.0
        p.rigidTransformInverse.m[i] = 1.0
    p.hashNumBuckets = num_buckets
    p.hashBucketSize = 4
    p.hashMaxCollisionLinkedListSize = max_list
    p.numSDFBlocks = num_blocks
    p.SDFBlockSize = 8
    p.virtualVoxelSize = voxel_size
    p.numOccupiedBlocks = 0
    p.maxIntegrationDistance = max_integration_distance
    p.truncScale = trunc_scale
    p.truncation = truncation
    p.integrationWeightSample = weight_sample
    p.integrationWeightMax = weight_max
    p.streamingVoxelExtents.x = p.streamingVoxelExtents.y = p.streamingVoxelExtents.z = 1.0
    p.streamingGridDimensions.x = p.streamingGridDimensions.y = p.streamingGridDimensions.z = 257
    p.streamingMinGridPos.x = p.streamingMinGridPos.y = p.streamingMinGridPos.z = -128
    p.streamingInitialChunkListSize = 2000
    return p


def depth_camera(width=640, height=480, fx=577.87, fy=577.87, mx=None, my=None, zmin=0.1, zmax=4.0) -> BFDepthCameraParams:
    """DepthCameraParams as DepthSensing.cpp:614-644 fills it (render depth range 0.1..4 m)."""
    c = BFDepthCameraParams()
    c.fx, c.fy = fx, fy
    c.mx = (width - 1) / 2.0 if mx is None else mx
    c.my = (height - 1) / 2.0 if my is None else my
    c.imageWidth, c.imageHeight = width, height
    c.sensorDepthWorldMin, c.sensorDepthWorldMax = zmin, zmax
    return c


class SceneRepHashSDF:
    """Mirror of CUDASceneRepHashSDF (DepthSensing/CUDASceneRepHashSDF.h:29-423) over bf_scene_*."""

    def __init__(self, params: BFHashParams, candidate_capacity=0, shard_count=1, shard_index=0, shard_chunk=1.0,
                 test_flags=0, splat_row_cap=0):
        self.params = params
        opts = BFSceneOptions(candidate_capacity, shard_count, shard_index, shard_chunk)
        opts.testFlags, opts.splatRowCap = test_flags, splat_row_cap
        self.h = C.c_void_p()
        check(lib().bf_scene_create(C.byref(params), C.byref(opts), C.byref(self.h)))

    def close(self):
        if self.h:
            lib().bf_scene_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        check(lib().bf_scene_reset(self.h))

    def integrate(self, T, depth: DeviceArray, color: DeviceArray | None, cam: BFDepthCameraParams, bitmask=None):
        check(lib().bf_scene_integrate(self.h, abi.mat(T), depth.ptr, color.ptr if color is not None else None,
                                       C.byref(cam), bitmask.ptr if bitmask is not None else None))

    def deIntegrate(self, T, depth: DeviceArray, color: DeviceArray | None, cam: BFDepthCameraParams, bitmask=None):
        check(lib().bf_scene_deintegrate(self.h, abi.mat(T), depth.ptr, color.ptr if color is not None else None,
                                         C.byref(cam), bitmask.ptr if bitmask is not None else None))

    def reintegrate(self, Told, Tnew, depth: DeviceArray, color: DeviceArray | None, cam: BFDepthCameraParams):
        """deIntegrate(Told) + integrate(Tnew) of one frame as one fused voxel pass."""
        check(lib().bf_scene_reintegrate(self.h, abi.mat(Told), abi.mat(Tnew), depth.ptr,
                                         color.ptr if color is not None else None, C.byref(cam)))

    def apply_ops(self, ops, cam: BFDepthCameraParams):
        """A sequence of (T, depth, color, deintegrate) voxel ops as one pass (bf_scene_apply_ops):
        the scene equals the one the sequential integrate / deIntegrate calls produce."""
        arr = (abi.BFVoxelOp * max(1, len(ops)))()
        for k, (T, depth, color, deint) in enumerate(ops):
            arr[k].T = abi.mat(T)
            arr[k].depth = depth.ptr
            arr[k].color = color.ptr if color is not None else None
            arr[k].deintegrate = 1 if deint else 0
        check(lib().bf_scene_apply_ops(self.h, arr, len(ops), C.byref(cam)))

    def garbageCollect(self):
        check(lib().bf_scene_garbage_collect(self.h))

    def setLastRigidTransformAndCompactify(self, T, cam) -> int:
        n = C.c_uint32()
        check(lib().bf_scene_compactify(self.h, abi.mat(T), C.byref(cam), C.byref(n)))
        return n.value

    def getHeapFreeCount(self) -> int:
        n = C.c_uint32()
        check(lib().bf_scene_heap_free_count(self.h, C.byref(n)))
        return n.value

    def numVisible(self) -> int:
        n = C.c_uint32()
        check(lib().bf_scene_num_visible(self.h, C.byref(n)))
        return n.value

    def capacity(self) -> dict:
        """BFSceneCapacity: sticky error bits, peak alloc candidates vs capacity, heap (bf_scene_capacity)."""
        from .abi import BFSceneCapacity
        c = BFSceneCapacity()
        check(lib().bf_scene_capacity(self.h, C.byref(c)))
        return {k: getattr(c, k) for k, _ in BFSceneCapacity._fields_}

    def errorFlags(self) -> int:
        n = C.c_uint32()
        check(lib().bf_scene_error_flags(self.h, C.byref(n)))
        return n.value

    def stats(self) -> dict:
        s = BFTsdfStats()
        check(lib().bf_scene_get_stats(self.h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in BFTsdfStats._fields_}

    def resetStats(self):
        check(lib().bf_scene_reset_stats(self.h))

    def synchronize(self):
        check(lib().bf_scene_synchronize(self.h))

    def export(self):
        """debugHash-style dump: (hash entries, heap, heapCounter, voxels) as numpy arrays."""
        E = self.params.hashNumBuckets * 4
        B = self.params.numSDFBlocks
        hash_ = np.empty(E, HASH_ENTRY_DTYPE)
        heap = np.empty(B, np.uint32)
        hc = C.c_uint32()
        vox = np.empty(B * 512, VOXEL_DTYPE)
        check(lib().bf_scene_export(self.h, hash_.ctypes.data_as(C.c_void_p), abi.u32p(heap), C.byref(hc),
                                    vox.ctypes.data_as(C.c_void_p)))
        return hash_, heap, hc.value, vox

    def raycast(self, T, cam: BFDepthCameraParams, rp, want_intervals=False):
        """CUDARayCastSDF::render from camera->world T; returns host (depth, depth4, normals, colors
        [, rayMin, rayMax])."""
        W, H = rp.width, rp.height
        outs = [DeviceArray((H, W), np.float32), DeviceArray((H, W, 4), np.float32), DeviceArray((H, W, 4), np.float32),
                DeviceArray((H, W, 4), np.float32)]
        iv = [DeviceArray((H, W), np.float32), DeviceArray((H, W), np.float32)] if want_intervals else [None, None]
        check(lib().bf_scene_raycast(self.h, abi.mat(T), C.byref(cam), C.byref(rp), *[o.ptr for o in outs],
                                     *[(a.ptr if a is not None else None) for a in iv]))
        res = [o.download() for o in outs]
        if want_intervals:
            res += [a.download() for a in iv]
        return tuple(res)

    def extract_mesh(self, mc: BFMarchingCubesParams):
        """CUDAMarchingCubesHashSDF::extractIsoSurface: float32 triangles [n, 3 vertices, 6] (x, y, z, r, g, b)
        in the fixed (heap block, voxel, triTable) order, and the count before the maxNumTriangles cap."""
        cap = int(mc.maxNumTriangles)
        buf = DeviceArray((max(cap, 1), 3, 6), np.float32)
        n, total = C.c_uint32(), C.c_uint32()
        check(lib().bf_scene_extract_mesh(self.h, C.byref(mc), buf.ptr if cap else None, C.byref(n), C.byref(total)))
        tris = buf.download_range(0, n.value * 72).view(np.float32).reshape(n.value, 3, 6) if n.value else \
            np.zeros((0, 3, 6), np.float32)
        return tris, total.value

    def export_blocks(self) -> np.ndarray:
        """int32 [n, 4] {x, y, z, allocated} of heap blocks [0, highWater) (bf_scene_export_blocks)."""
        n = C.c_uint32()
        check(lib().bf_scene_export_blocks(self.h, None, C.c_uint32(0), C.byref(n)))
        out = np.empty((max(n.value, 1), 4), np.int32)
        check(lib().bf_scene_export_blocks(self.h, out.ctypes.data_as(C.POINTER(C.c_int32)), C.c_uint32(n.value), C.byref(n)))
        return out[: n.value].copy()

    def export_block_voxels(self, first: int, count: int) -> np.ndarray:
        """voxels of heap blocks [first, first + count): VOXEL_DTYPE [count, 512] (bf_scene_export_block_voxels)."""
        out = np.empty((max(count, 1), 512), VOXEL_DTYPE)
        check(lib().bf_scene_export_block_voxels(self.h, C.c_uint32(first), C.c_uint32(count), out.ctypes.data_as(C.c_void_p)))
        return out[:count]

    def export_visible(self) -> np.ndarray:
        cap = self.params.numSDFBlocks
        out = np.empty((cap, 4), np.int32)
        n = C.c_uint32()
        check(lib().bf_scene_export_visible(self.h, out.ctypes.data_as(C.POINTER(C.c_int32)), cap, C.byref(n)))
        return out[: n.value].copy()


# ---- mesh output ---------------------------------------------------------------------------
def mc_params(voxel_size: float, thresh_factor: float = 10.0, max_triangles: int = 3000000, box=None) -> BFMarchingCubesParams:
    """CUDAMarchingCubesHashSDF::parametersFromGlobalAppState (CUDAMarchingCubesHashSDF.h:19-28):
    both thresholds = s_SDFMarchingCubeThreshFactor * s_SDFVoxelSize; box = (minCorner, maxCorner) or None."""
    p = BFMarchingCubesParams()
    t = float(np.float32(thresh_factor) * np.float32(voxel_size))
    p.threshMarchingCubes = p.threshMarchingCubes2 = t
    p.maxNumTriangles = max_triangles
    if box is not None:
        p.boxEnabled = 1
        p.minCorner[:] = [float(v) for v in box[0]]
        p.maxCorner[:] = [float(v) for v in box[1]]
    return p


def _tri_ptr(tris: np.ndarray):
    t = np.ascontiguousarray(tris, np.float32)
    assert t.size % 18 == 0
    return t, t.ctypes.data_as(C.c_void_p), t.size // 18


def mesh_merge(tris: np.ndarray, transform=None):
    """saveMesh's indexed mesh (bf_mesh_merge): (vertices [nv,3], colors [nv,4], faces [nf,3])."""
    t, ptr, n = _tri_ptr(tris)
    v = np.empty((3 * n, 3), np.float32)
    c = np.empty((3 * n, 4), np.float32)
    f = np.empty((n, 3), np.uint32)
    nv, nf = C.c_uint32(), C.c_uint32()
    check(lib().bf_mesh_merge(ptr, C.c_uint32(n), abi.mat(transform) if transform is not None else None,
                              abi.vp(v), abi.vp(c), abi.vp(f), C.byref(nv), C.byref(nf)))
    return v[: nv.value].copy(), c[: nv.value].copy(), f[: nf.value].copy()


def mesh_save_ply(path: str, tris: np.ndarray, transform=None):
    """CUDAMarchingCubesHashSDF::saveMesh (bf_mesh_save_ply); returns (vertices, faces) written."""
    t, ptr, n = _tri_ptr(tris)
    nv, nf = C.c_uint32(), C.c_uint32()
    check(lib().bf_mesh_save_ply(os.fsencode(path), ptr, C.c_uint32(n),
                                 abi.mat(transform) if transform is not None else None, C.byref(nv), C.byref(nf)))
    return nv.value, nf.value


# ---- synthetic stream ----------------------------------------------------------------------
def raycast_params(width=640, height=480, fx=577.87, fy=577.87, mx=None, my=None, min_depth=0.1, max_depth=4.0,
                   truncation=0.06, ray_increment_factor=0.8, thres_sample_dist_factor=50.5, thres_dist_factor=50.0,
                   use_gradients=False) -> BFRayCastParams:
    """CUDARayCastSDF::parametersFromGlobalAppState (CUDARayCastSDF.h:24-51), zParametersDefault.txt:35-56."""
    p = BFRayCastParams()
    p.width, p.height = width, height
    p.fx, p.fy = fx, fy
    p.mx = (width - 1) / 2.0 if mx is None else mx
    p.my = (height - 1) / 2.0 if my is None else my
    p.minDepth, p.maxDepth = min_depth, max_depth
    inc = np.float32(ray_increment_factor) * np.float32(truncation)
    p.rayIncrement = float(inc)
    p.thresSampleDist = float(np.float32(thres_sample_dist_factor) * inc)
    p.thresDist = float(np.float32(thres_dist_factor) * inc)
    p.useGradients = 1 if use_gradients else 0
    return p


def synth_scene(seed=0) -> BFSynthScene:
    s = BFSynthScene()
    check(lib().bf_synth_scene_default(C.c_uint32(seed), C.byref(s)))
    return s


def synth_pose(frame: int) -> np.ndarray:
    T = (C.c_float * 16)()
    check(lib().bf_synth_pose(C.c_uint32(frame), T))
    return np.array(T[:], dtype=np.float32).reshape(4, 4)


def synth_render(scene: BFSynthScene, T, cam: BFDepthCameraParams, noise_seed: int, frame: int,
                 depth: DeviceArray, color: DeviceArray | None):
    check(lib().bf_synth_render(C.byref(scene), abi.mat(T), C.byref(cam), C.c_uint32(noise_seed), C.c_uint32(frame),
                                depth.ptr, color.ptr if color is not None else None))


def synth_render_host(scene: BFSynthScene, T, cam: BFDepthCameraParams, noise_seed: int = 1, frame: int = 0):
    d = np.empty((cam.imageHeight, cam.imageWidth), np.float32)
    c = np.empty((cam.imageHeight, cam.imageWidth, 4), np.uint8)
    check(lib().bf_synth_render_host(C.byref(scene), abi.mat(T), C.byref(cam), C.c_uint32(noise_seed),
                                     C.c_uint32(frame), abi.f32p(d), abi.u8p(c)))
    return d, c
