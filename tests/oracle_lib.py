"""ctypes binding of the CPU oracle (oracle/_build/libbf_oracle.so) — test infrastructure only."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from bundlefusion_amd import abi

REPO = abi.REPO
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "_build", "libbf_oracle.so")
_lib = None


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "-j8"], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            build_oracle()
        L = C.CDLL(ORACLE_LIB)
        L.or_preprocess.restype = None
        L.or_preprocess.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                                    C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]
        L.or_scene_create.restype = C.c_void_p
        L.or_scene_create.argtypes = [C.c_void_p]
        for n in ("or_scene_destroy", "or_scene_reset", "or_scene_garbage_collect"):
            getattr(L, n).argtypes = [C.c_void_p]
            getattr(L, n).restype = None
        L.or_scene_integrate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.or_scene_integrate.restype = None
        L.or_scene_compactify.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_scene_compactify.restype = C.c_uint32
        L.or_scene_heap_free_count.argtypes = [C.c_void_p]
        L.or_scene_heap_free_count.restype = C.c_uint32
        L.or_scene_num_occupied.argtypes = [C.c_void_p]
        L.or_scene_num_occupied.restype = C.c_uint32
        L.or_scene_export.argtypes = [C.c_void_p] * 5
        L.or_scene_export.restype = None
        L.or_scene_export_visible.argtypes = [C.c_void_p, C.c_void_p]
        L.or_scene_import.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]
        L.or_scene_import.restype = None
        L.or_scene_export_visible.restype = None
        L.or_scene_get_stats.argtypes = [C.c_void_p, C.c_void_p]
        L.or_scene_get_stats.restype = None
        L.or_matrix_inverse.argtypes = [C.c_void_p, C.c_void_p]
        L.or_matrix_inverse.restype = None
        L.or_dense_integrate.argtypes = [C.c_void_p] * 6 + [C.c_int, C.c_void_p]
        L.or_dense_integrate.restype = None
        L.or_raycast.argtypes = [C.c_void_p] * 10
        L.or_raycast.restype = None
        L.or_extract_mesh.argtypes = [C.c_void_p] * 6
        L.or_extract_mesh.restype = None
        L.or_cache_store_frame.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32] + [C.c_void_p] * 8
        L.or_cache_store_frame.restype = None
        L.or_corr_from_depth.argtypes = [C.c_void_p] * 3 + [C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                                                             C.c_uint32, C.c_void_p, C.c_void_p]
        L.or_corr_from_depth.restype = None
        L.or_mc_tables.argtypes = [C.c_void_p] * 3
        L.or_mc_tables.restype = None
        _lib = L
    return _lib


def _m(T) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(T, np.float32).reshape(16))


def cache_store_frame(opts, depth: np.ndarray, color: np.ndarray):
    """CUDACache::storeFrame restated (oracle/frames.cpp or_cache_store_frame): dict like CUDACache.download,
    plus the cache intrinsics K / Kinv."""
    W, H = opts.width, opts.height
    d = np.ascontiguousarray(depth, np.float32)
    c = np.ascontiguousarray(color, np.uint8)
    out = {"depth": np.empty((H, W), np.float32), "campos": np.empty((H, W, 4), np.float32),
           "normals": np.empty((H, W, 4), np.float32), "normalsU8": np.empty((H, W, 4), np.uint8),
           "intensity": np.empty((H, W), np.float32), "intensityDeriv": np.empty((H, W, 2), np.float32),
           "K": np.empty(16, np.float32), "Kinv": np.empty(16, np.float32)}
    lib().or_cache_store_frame(C.addressof(opts), d.ctypes.data, c.ctypes.data, c.shape[1], c.shape[0],
                               *[out[k].ctypes.data for k in ("depth", "campos", "normals", "normalsU8", "intensity",
                                                              "intensityDeriv", "K", "Kinv")])
    out["K"], out["Kinv"] = out["K"].reshape(4, 4), out["Kinv"].reshape(4, 4)
    return out


def corr_from_depth(depths, T: np.ndarray, Tinv: np.ndarray, cur: int, start: int, opts, cap: int):
    """EntryJ producer restated (oracle/frames.cpp or_corr_from_depth); depths: list of host float arrays."""
    from bundlefusion_amd.abi import ENTRYJ_DTYPE
    ds = [np.ascontiguousarray(d, np.float32) for d in depths]
    ptrs = (C.c_void_p * len(ds))(*[d.ctypes.data for d in ds])
    T = np.ascontiguousarray(T, np.float32)
    Ti = np.ascontiguousarray(Tinv, np.float32)
    out = np.zeros(max(cap, 1), ENTRYJ_DTYPE)
    n, total = C.c_uint32(), C.c_uint32()
    lib().or_corr_from_depth(C.cast(ptrs, C.c_void_p), T.ctypes.data, Ti.ctypes.data, cur, start, C.addressof(opts),
                             out.ctypes.data, cap, C.addressof(n), C.addressof(total))
    return out[: n.value].copy(), total.value


def mc_tables():
    """The compiled marching-cubes case tables (mc_tables.h, shared by the kernel and the oracle)."""
    edges = np.zeros(256, np.uint16)
    ntri = np.zeros(256, np.uint8)
    tri = np.zeros((256, 15), np.uint8)
    lib().or_mc_tables(edges.ctypes.data, ntri.ctypes.data, tri.ctypes.data)
    return edges, ntri, tri


class OracleScene:
    """Serial CPU restatement of CUDASceneRepHashSDF (oracle/tsdf.cpp)."""

    def __init__(self, params: abi.BFHashParams, shard=None):
        self.params = params
        self.h = lib().or_scene_create(C.byref(params))
        if shard is not None:  # (count, index, chunk): a multi-GPU TSDF shard's ownership
            lib().or_scene_set_shard(C.c_void_p(self.h), C.c_uint32(shard[0]), C.c_uint32(shard[1]), C.c_float(shard[2]))

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_scene_destroy(self.h)
            self.h = None

    def integrate(self, T, depth: np.ndarray, color: np.ndarray | None, cam, deintegrate=False):
        depth = np.ascontiguousarray(depth, np.float32)
        col = None if color is None else np.ascontiguousarray(color, np.uint8)
        T = _m(T)
        lib().or_scene_integrate(self.h, T.ctypes.data, depth.ctypes.data, None if col is None else col.ctypes.data,
                                 C.byref(cam), int(deintegrate), None)

    def deIntegrate(self, T, depth, color, cam):
        self.integrate(T, depth, color, cam, deintegrate=True)

    def garbageCollect(self):
        lib().or_scene_garbage_collect(self.h)

    def compactify(self, T, cam) -> int:
        return lib().or_scene_compactify(self.h, _m(T).ctypes.data, C.byref(cam))

    def raycast(self, T, cam, rp, want_intervals=False):
        """CUDARayCastSDF::render restated (oracle/tsdf.cpp or_raycast)."""
        W, H = rp.width, rp.height
        depth = np.empty((H, W), np.float32)
        d4 = np.empty((H, W, 4), np.float32)
        nrm = np.empty((H, W, 4), np.float32)
        col = np.empty((H, W, 4), np.float32)
        rmin = np.empty((H, W), np.float32)
        rmax = np.empty((H, W), np.float32)
        lib().or_raycast(self.h, C.addressof(rp), C.addressof(cam), _m(T).ctypes.data, depth.ctypes.data, d4.ctypes.data,
                         nrm.ctypes.data, col.ctypes.data, rmin.ctypes.data, rmax.ctypes.data)
        res = (depth, d4, nrm, col)
        return res + (rmin, rmax) if want_intervals else res

    def extract_mesh(self, mc):
        """extractIsoSurface restated (oracle/tsdf.cpp or_extract_mesh): float32 [n, 3, 6], total."""
        cap = int(mc.maxNumTriangles)
        out = np.empty((max(cap, 1), 3, 6), np.float32)
        n, total = C.c_uint32(), C.c_uint32()
        lib().or_extract_mesh(self.h, C.addressof(mc), out.ctypes.data, cap, C.addressof(n), C.addressof(total))
        return out[: n.value].copy(), total.value

    def getHeapFreeCount(self) -> int:
        return lib().or_scene_heap_free_count(self.h)

    def numOccupied(self) -> int:
        return lib().or_scene_num_occupied(self.h)

    def export(self):
        E = self.params.hashNumBuckets * 4
        B = self.params.numSDFBlocks
        h = np.empty(E, abi.HASH_ENTRY_DTYPE)
        heap = np.empty(B, np.uint32)
        hc = C.c_uint32()
        vox = np.empty(B * 512, abi.VOXEL_DTYPE)
        lib().or_scene_export(self.h, h.ctypes.data, heap.ctypes.data, C.addressof(hc), vox.ctypes.data)
        return h, heap, hc.value, vox

    def import_state(self, hash_, heap, heap_counter, voxels):
        """Continue from a dumped state (e.g. the GPU loop's, bf_recon_export); compactify before a GC."""
        h = np.ascontiguousarray(hash_)
        hp = np.ascontiguousarray(heap, np.uint32)
        v = np.ascontiguousarray(voxels)
        assert len(h) == self.params.hashNumBuckets * 4 and len(hp) == self.params.numSDFBlocks
        assert len(v) == self.params.numSDFBlocks * 512
        lib().or_scene_import(self.h, h.ctypes.data, hp.ctypes.data, C.c_uint32(heap_counter), v.ctypes.data)

    def export_visible(self) -> np.ndarray:
        n = self.numOccupied()
        out = np.empty(n, abi.HASH_ENTRY_DTYPE)
        if n:
            lib().or_scene_export_visible(self.h, out.ctypes.data)
        return out

    def stats(self) -> dict:
        s = abi.BFTsdfStats()
        lib().or_scene_get_stats(self.h, C.byref(s))
        return {k: getattr(s, k) for k, _ in abi.BFTsdfStats._fields_}


def matrix_inverse(T) -> np.ndarray:
    out = np.empty(16, np.float32)
    lib().or_matrix_inverse(_m(T).ctypes.data, out.ctypes.data)
    return out.reshape(4, 4)


def dense_integrate(T, depth, color, cam, params, origin, n) -> np.ndarray:
    grid = np.empty(n * n * n, abi.VOXEL_DTYPE)
    depth = np.ascontiguousarray(depth, np.float32)
    color = np.ascontiguousarray(color, np.uint8)
    org = np.asarray(origin, np.int32)
    lib().or_dense_integrate(_m(T).ctypes.data, depth.ctypes.data, color.ctypes.data, C.byref(cam), C.byref(params),
                             org.ctypes.data, n, grid.ctypes.data)
    return grid.reshape(n, n, n)


# ---- hash-state comparison helpers (shared by CPU and GPU tests) ----------------------------
def blocks_of(hash_entries: np.ndarray) -> dict:
    """{(x,y,z): ptr} of every allocated entry."""
    occ = hash_entries[hash_entries["ptr"] != abi.FREE_ENTRY]
    return {(int(e["x"]), int(e["y"]), int(e["z"])): int(e["ptr"]) for e in occ}


def block_voxels(vox: np.ndarray, ptr: int) -> np.ndarray:
    return vox[ptr: ptr + 512]


def check_hash_invariants(params, hash_entries, heap, heap_counter):
    """debugHash (CUDASceneRepHashSDF.h:179-314): no duplicate positions, heap/pool partition,
    every entry reachable from its own bucket (slot or collision list)."""
    B = params.numSDFBlocks
    nb = params.hashNumBuckets
    E = nb * 4
    free = heap[: heap_counter + 1] if heap_counter != 0xFFFFFFFF else heap[:0]
    assert len(set(free.tolist())) == len(free), "duplicate free pointers in heap"
    occ_idx = np.nonzero(hash_entries["ptr"] != abi.FREE_ENTRY)[0]
    assert not np.any(hash_entries["ptr"][occ_idx] == abi.LOCK_ENTRY), "entry left locked"
    ptrs = hash_entries["ptr"][occ_idx] // 512
    assert len(set(ptrs.tolist())) == len(ptrs), "two entries share a block"
    assert not (set(ptrs.tolist()) & set(free.tolist())), "ptr both free and allocated"
    assert len(ptrs) + len(free) == B, f"leak: {len(ptrs)} allocated + {len(free)} free != {B}"
    pos = set()
    for i in occ_idx:
        e = hash_entries[i]
        key = (int(e["x"]), int(e["y"]), int(e["z"]))
        assert key not in pos, f"duplicate block {key}"
        pos.add(key)
        h = bucket_of(key, nb)
        if i // 4 == h:
            continue
        # must be on bucket h's collision list
        last = h * 4 + 3
        j = last
        found = False
        for _ in range(params.hashMaxCollisionLinkedListSize + 1):
            off = int(hash_entries[j]["offset"])
            if off == 0:
                break
            j = (last + off) % E
            if j == i:
                found = True
                break
        assert found, f"entry {key} at {i} unreachable from bucket {h}"


def bucket_of(key, num_buckets: int) -> int:
    """computeHashPos (VoxelUtilHashSDF.h:225-234) in int32 wrapping arithmetic."""
    def i32(v: int) -> int:
        v &= 0xFFFFFFFF
        return v - (1 << 32) if v >= (1 << 31) else v

    x, y, z = (int(v) for v in key)
    r = i32(i32(x * 73856093) ^ i32(y * 19349669) ^ i32(z * 83492791))
    res = (abs(r) % num_buckets) * (1 if r >= 0 else -1)  # C % truncates toward zero
    if res < 0:
        res += num_buckets
    return res


def preprocess(opts, depth_u16, rgbx, integration_wh):
    """Oracle of CUDAImageManager::process (oracle/frames.cpp)."""
    import numpy as np
    depth_u16 = np.ascontiguousarray(depth_u16, np.uint16)
    dh, dw = depth_u16.shape
    iw, ih = integration_wh
    out_d = np.zeros((ih, iw), np.float32)
    out_c = np.zeros((ih, iw, 4), np.uint8)
    cp = None
    ch = cw = 0
    if rgbx is not None:
        rgbx = np.ascontiguousarray(rgbx, np.uint8)
        ch, cw = rgbx.shape[:2]
        cp = rgbx.ctypes.data_as(C.c_void_p)
    lib().or_preprocess(C.byref(opts), depth_u16.ctypes.data_as(C.c_void_p), dw, dh, cp, cw, ch, iw, ih,
                        out_d.ctypes.data_as(C.c_void_p), out_c.ctypes.data_as(C.c_void_p))
    return out_d, (out_c if rgbx is not None else None)
