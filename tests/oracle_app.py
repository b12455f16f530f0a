"""CPU oracle of the FriedLiver application (bundlefusion_amd/csrc/app.cpp, bf_app_*) — TEST
INFRASTRUCTURE, composed from the oracle's restatements only:

  .sens parsing         here, in Python (format: SURVEY.md Appendix B), zlib depth, colour through PIL
                        (libjpeg / libpng, not the product's decoders)
  CUDAImageManager      oracle/frames.cpp or_preprocess2 (integration images + the sensor-size raw and
                        filtered depth that copyToBundling hands the bundler, CUDAImageManager.h:223-227)
  CUDACache::storeFrame oracle/frames.cpp or_cache_store_frame
  SiftGPU stand-in      oracle/frames.cpp or_corr_from_depth (submap pairs, keyframe pairs) and
                        or_front_end_tinc (the frame-to-frame estimate)
  the loop              oracle/recon.cpp (OnlineBundler + TrajectoryManager, synchronous order), including
                        the end-of-sequence phase (or_recon_end_sequence)

Parameters are derived here from the same settings dicts the test wrote into the zParameters files, with
the float32 arithmetic of CUDAImageManager.h:160-166 / CUDACache.cpp:14-21."""
from __future__ import annotations

import ctypes as C
import io as _io
import struct
import zlib

import numpy as np

from bundlefusion_amd import abi
from bundlefusion_amd.abi import ENTRYJ_DTYPE
from oracle_lib import cache_store_frame, corr_from_depth, lib, matrix_inverse
from oracle_recon import OracleRecon

F32 = np.float32


def read_sens(path):
    """(header dict, per-frame list of (pose, colour bytes, depth bytes)) of a v4 .sens."""
    b = open(path, "rb").read()
    o = 0

    def take(fmt):
        nonlocal o
        v = struct.unpack_from(fmt, b, o)
        o += struct.calcsize(fmt)
        return v

    version, nlen = take("<IQ")
    assert version == 4
    o += nlen
    mats = [np.frombuffer(b, "<f4", 16, o + 64 * k).reshape(4, 4).copy() for k in range(4)]
    o += 256
    cc, dc = take("<ii")
    cw, ch, dw, dh, shift, n = take("<IIIIfQ")
    frames = []
    for _ in range(n):
        pose = np.frombuffer(b, "<f4", 16, o).reshape(4, 4).copy()
        o += 64
        _, _, cb, db = take("<QQQQ")
        frames.append((pose, b[o:o + cb], b[o + cb:o + cb + db]))
        o += cb + db
    hdr = dict(colorIntrinsic=mats[0], depthIntrinsic=mats[2], colorCompression=cc, depthCompression=dc, colorWidth=cw,
               colorHeight=ch, depthWidth=dw, depthHeight=dh, depthShift=shift, numFrames=n)
    return hdr, frames


def decode_frame(hdr, frame):
    from PIL import Image
    _, col, dep = frame
    d = np.frombuffer(zlib.decompress(dep) if hdr["depthCompression"] == 1 else dep, "<u2")
    d = d.reshape(hdr["depthHeight"], hdr["depthWidth"])
    if hdr["colorCompression"] == 0:
        rgb = np.frombuffer(col, np.uint8).reshape(hdr["colorHeight"], hdr["colorWidth"], 3)
    else:
        rgb = np.asarray(Image.open(_io.BytesIO(col)).convert("RGB"))
    rgbx = np.empty(rgb.shape[:2] + (4,), np.uint8)
    rgbx[..., :3] = rgb
    rgbx[..., 3] = 255
    return d, rgbx


def front_end_tinc(prev, cur, f, seed, dr, dm):
    L = lib()
    L.or_front_end_tinc.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_float, C.c_float, C.c_void_p]
    L.or_front_end_tinc.restype = None
    p = np.ascontiguousarray(prev, F32)
    c = np.ascontiguousarray(cur, F32)
    out = np.zeros(16, F32)
    L.or_front_end_tinc(p.ctypes.data, c.ctypes.data, f, seed, dr, dm, out.ctypes.data)
    return out.reshape(4, 4)


def preprocess2(opts, depth_u16, rgbx, iw, ih):
    L = lib()
    L.or_preprocess2.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                                 C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.or_preprocess2.restype = None
    d = np.ascontiguousarray(depth_u16, np.uint16)
    c = np.ascontiguousarray(rgbx, np.uint8)
    dh, dw = d.shape
    ch, cw = c.shape[:2]
    od = np.zeros((ih, iw), F32)
    oc = np.zeros((ih, iw, 4), np.uint8)
    raw = np.zeros((dh, dw), F32)
    filt = np.zeros((dh, dw), F32)
    L.or_preprocess2(C.addressof(opts), d.ctypes.data, dw, dh, c.ctypes.data, cw, ch, iw, ih, od.ctypes.data,
                     oc.ctypes.data, raw.ctypes.data, filt.ctypes.data)
    return od, oc, raw, filt


class OracleFriedLiver:
    """The app restated: .sens + settings -> the oracle loop's inputs, frame by frame."""

    def __init__(self, sens_path, app: dict, bundling: dict, drift=(np.deg2rad(0.05), 0.002), seed=1, corr_stride=16,
                 corr_depth_thresh=0.02):
        self.hdr, self.frames = read_sens(sens_path)
        h = self.hdr
        self.F = h["numFrames"]
        self.S = int(bundling["s_submapSize"])
        self.L = self.S + 1
        K = h["depthIntrinsic"].astype(F32)
        dw, dh = h["depthWidth"], h["depthHeight"]
        iw, ih = int(app["s_integrationWidth"]), int(app["s_integrationHeight"])
        self.iw, self.ih = iw, ih
        # CUDAImageManager.h:160-166 in float32
        cam = abi.BFDepthCameraParams()
        cam.fx = F32(K[0, 0]) * (F32(iw) / F32(dw))
        cam.fy = F32(K[1, 1]) * (F32(ih) / F32(dh))
        cam.mx = F32(K[0, 2]) * (F32(iw - 1) / F32(dw - 1))
        cam.my = F32(K[1, 2]) * (F32(ih - 1) / F32(dh - 1))
        cam.imageWidth, cam.imageHeight = iw, ih
        cam.sensorDepthWorldMin, cam.sensorDepthWorldMax = app["s_renderDepthMin"], app["s_renderDepthMax"]
        self.cam = cam
        self.pre = abi.BFPreprocessOptions(1 if bundling["s_erodeSIFTdepth"] else 0, 3, 0.05, 0.3,
                                           1 if bundling["s_depthFilter"] else 0, bundling["s_depthSigmaD"],
                                           bundling["s_depthSigmaR"], h["depthShift"])
        co = abi.BFCacheOptions()
        co.inputWidth, co.inputHeight = dw, dh
        co.width, co.height = int(bundling["s_downsampledWidth"]), int(bundling["s_downsampledHeight"])
        co.maxFrames = self.F
        co.inputIntrinsics[:] = K.ravel().tolist()
        co.colorSigma, co.depthSigmaD, co.depthSigmaR = (bundling["s_colorDownSigma"], bundling["s_depthDownSigmaD"],
                                                         bundling["s_depthDownSigmaR"])
        self.cache_opts = co
        self.cache_intrinsics = (F32(K[0, 0]) * (F32(co.width) / F32(dw)), F32(K[1, 1]) * (F32(co.height) / F32(dh)),
                                 F32(K[0, 2]) * (F32(co.width - 1) / F32(dw - 1)),
                                 F32(K[1, 2]) * (F32(co.height - 1) / F32(dh - 1)))
        cr = abi.BFCorrOptions()
        cr.intrinsics[:] = [float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])]
        cr.intrinsicsInv[:] = matrix_inverse(K).ravel().tolist()
        cr.width, cr.height, cr.stride, cr.maxPerPair = dw, dh, corr_stride, 25
        cr.minDepth, cr.maxDepth, cr.depthThresh = app["s_sensorDepthMin"], app["s_SDFMaxIntegrationDistance"], corr_depth_thresh
        cr.minPerPair = int(bundling["s_minNumMatchesGlobal"])
        self.corr_opts = cr
        self.local_min = int(bundling["s_minNumMatchesLocal"])
        nsub = (self.F + self.S - 1) // self.S
        self.K = nsub + 1
        self.max_local = 25 * self.L * (self.L - 1) // 2
        self.max_global = max(1000, 25 * self.K * (self.K - 1) // 2)
        self.poses = [fr[0] for fr in self.frames]
        self.drift, self.seed = drift, seed
        self.ora = OracleRecon(self.F, self.poses[0], self.cache_intrinsics, S=self.S, max_keyframes=self.K,
                               max_local_corr=self.max_local, max_global_corr=self.max_global,
                               cache_w=co.width, cache_h=co.height, use_local_dense=bool(bundling["s_useLocalDense"]),
                               verify=bool(bundling["s_useLocalVerify"]))
        self.filtered = {}     # sensor-size filtered depth of the frames still needed
        self.kf_depth = []     # ... of each keyframe
        self.images = {}       # integration images recomputed for TSDF replays
        self.tinc = []
        self.n_global = 0
        self.next = 0

    def _local_corr(self, s, n):
        base = s * self.S
        d = [self.filtered[base + i] for i in range(n)]
        T = np.stack([self.poses[base + i] for i in range(n)]).astype(F32)
        Ti = np.stack([matrix_inverse(t) for t in T])
        o = abi.BFCorrOptions.from_buffer_copy(self.corr_opts)
        o.minPerPair = self.local_min
        parts = []
        for cur in range(1, n):
            e, _ = corr_from_depth(d, T, Ti, cur, 0, o, self.max_local)
            parts.append(e)
        c = np.concatenate(parts) if parts else np.zeros(0, ENTRYJ_DTYPE)
        if len(c):
            self.ora.set_local_corr(s, c)
        return c

    def _keyframe_corr(self, k):
        if k == 0:
            e = np.zeros(0, ENTRYJ_DTYPE)
        else:
            T = np.stack([self.poses[i * self.S] for i in range(k + 1)]).astype(F32)
            Ti = np.stack([matrix_inverse(t) for t in T])
            e, _ = corr_from_depth(self.kf_depth[:k + 1], T, Ti, k, 0, self.corr_opts, self.max_global - self.n_global)
        self.n_global += len(e)
        self.ora.append_global_corr(e)
        return e

    def step(self):
        f = self.next
        du, rgbx = decode_frame(self.hdr, self.frames[f])
        od, oc, raw, filt = preprocess2(self.pre, du, rgbx, self.iw, self.ih)
        self.filtered[f] = filt
        if f % self.S == 0:
            self.kf_depth.append(filt)
        cache = cache_store_frame(self.cache_opts, raw, rgbx)
        dr, dm = self.drift
        t = np.eye(4, dtype=F32) if f == 0 else front_end_tinc(self.poses[f - 1], self.poses[f], f, self.seed, dr, dm)
        self.tinc.append(t)
        self.ora.set_frame(f, t, cache)
        if f % self.S == 0 and f > 0:
            s = f // self.S - 1
            self._local_corr(s, self.L)
            self._keyframe_corr(s)
            for g in [g for g in self.filtered if g < f - self.S]:
                del self.filtered[g]
        self.ora.process_frame(f)
        self.next += 1

    def integration_image(self, f):
        """(depth, colour) the loop integrates frame f with (CUDAImageManager's frame store), recomputed."""
        if f not in self.images:
            du, rgbx = decode_frame(self.hdr, self.frames[f])
            od, oc, _, _ = preprocess2(self.pre, du, rgbx, self.iw, self.ih)
            self.images[f] = (od, oc)
        return self.images[f]

    def finish(self, num_solve_frames_before_exit=30):
        last = (self.next - 1) // self.S
        n = self.next - last * self.S
        if n >= 2 and len(self.kf_depth) == last + 1:
            self._local_corr(last, n)
            self._keyframe_corr(last)
        return self.ora.end_sequence(num_solve_frames_before_exit)
