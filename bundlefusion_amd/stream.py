"""Seeded synthetic RGB-D stream for the reconstruction loop (SURVEY.md §8(d) "Concrete synthetic
inputs"): GT trajectory, device-resident depth/colour frames (the CUDAImageManager frame store),
80x60 dense-term cache frames, per-submap local and global keyframe EntryJ correspondences, and the
front end's drifted per-frame pose estimates. Everything the loop reads is resident in HBM before
the first frame is processed."""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import DeviceArray, abi, check, depth_camera, lib, synth_pose, synth_scene
from .abi import ENTRYJ_DTYPE, BFCachedFrame
from .solver import synth_cache_frames, synth_correspondences


def _rodrigues(w):
    th = float(np.linalg.norm(w))
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


class SyntheticStream:
    def __init__(self, num_frames: int, width=640, height=480, submap=10, seed=0, drift=(0.05, 0.002),
                 max_per_pair=25, outliers=0.02, cache_w=80, cache_h=60, cache_source="frames", log=None,
                 raw_input=False):
        t0 = time.perf_counter()
        self.F, self.S = num_frames, submap
        self.log = log or (lambda *a: None)
        self.scene = synth_scene(seed)
        f = 577.87 * width / 640.0
        self.cam = depth_camera(width, height, fx=f, fy=f)
        self.cache_cam = depth_camera(cache_w, cache_h, fx=f * cache_w / width, fy=f * cache_h / height)
        self.cache_intrinsics = (self.cache_cam.fx, self.cache_cam.fy, self.cache_cam.mx, self.cache_cam.my)
        self.gt = np.stack([synth_pose(i) for i in range(num_frames)]).astype(np.float32)
        self.num_submaps = (num_frames + submap - 1) // submap
        self.K = self.num_submaps  # keyframe = first frame of each submap

        # device frame store (depth f32, colour uchar4), rendered on the GPU with the noise model
        P = width * height
        self.depth = DeviceArray((num_frames, height, width), np.float32)
        self.color = DeviceArray((num_frames, height, width, 4), np.uint8)
        for i in range(num_frames):
            check(lib().bf_synth_render(C.byref(self.scene), abi.mat(self.gt[i]), C.byref(self.cam), C.c_uint32(1),
                                        C.c_uint32(i), C.c_void_p(self.depth.ptr.value + 4 * P * i),
                                        C.c_void_p(self.color.ptr.value + 4 * P * i)))
        check(lib().bf_device_synchronize())
        self.log(f"rendered {num_frames} frames {width}x{height} in {time.perf_counter() - t0:.1f}s")
        # raw_input: the frames as the sensor delivers them (ushort depth in mm, RGBX), preprocessed inside the
        # loop into the frame store above (CUDAImageManager::process per frame, Recon.attach_preproc)
        self.raw_input = raw_input
        if raw_input:
            self.depth_u16 = DeviceArray((num_frames, height, width), np.uint16)
            self.rgbx = DeviceArray((num_frames, height, width, 4), np.uint8)
            for i in range(num_frames):
                check(lib().bf_synth_to_raw(C.c_void_p(self.depth.ptr.value + 4 * P * i),
                                            C.c_void_p(self.color.ptr.value + 4 * P * i), C.c_uint32(P), C.c_float(1000.0),
                                            C.c_void_p(self.depth_u16.ptr.value + 2 * P * i),
                                            C.c_void_p(self.rgbx.ptr.value + 4 * P * i)))

        # front-end frame-to-frame estimates (stand-in for computeSiftTransformCU): GT motion with a
        # random-walk error per frame, so both the local and the global solve have drift to remove
        rng = np.random.default_rng(seed + 3)
        self.tinc = np.zeros((num_frames, 4, 4), np.float32)
        self.tinc[0] = np.eye(4)
        for i in range(1, num_frames):
            step = np.eye(4)
            step[:3, :3] = _rodrigues(rng.normal(size=3) * np.deg2rad(drift[0]))
            step[:3, 3] = rng.normal(size=3) * drift[1]
            rel = np.linalg.inv(self.gt[i - 1].astype(np.float64)) @ self.gt[i].astype(np.float64)
            self.tinc[i] = (rel @ step).astype(np.float32)

        # dense-term cache frames (80x60): "frames" builds them from the rendered frames with the
        # reference's pipeline (CUDACache::storeFrame, called by Bundler::storeCachedFrame per input
        # frame); "loop": the same, but inside the loop as each frame is processed (attach_cache);
        # "synth" renders them analytically at 80x60 (no filtering)
        t1 = time.perf_counter()
        self.cache = []
        self.cache_source = cache_source
        self._cache_args = (width, height, f, f, self.cam.mx, self.cam.my, num_frames, cache_w, cache_h)
        if cache_source == "loop":
            self.cache_store = self.loop_cache()
            self.cache = [None] * num_frames
        elif cache_source == "frames":
            from .cache import CUDACache, cache_options
            self.cache_store = CUDACache(cache_options(width, height, f, f, self.cam.mx, self.cam.my, num_frames,
                                                       width=cache_w, height=cache_h))
            for i in range(num_frames):
                self.cache_store.storeFrame(self.depth.ptr.value + 4 * P * i, self.color.ptr.value + 4 * P * i,
                                            width, height)
            self.cache_store.synchronize()
            self.cache = [self.cache_store.frame(i) for i in range(num_frames)]
        else:
            cf = synth_cache_frames(self.scene, self.gt, self.cache_cam)
            self.cache_arrays = {k: DeviceArray.from_host(v) for k, v in cf.items()}
            for i in range(num_frames):
                c = BFCachedFrame()
                for k, v in cf.items():
                    setattr(c, k, self.cache_arrays[k].ptr.value + i * v[0].nbytes)
                self.cache.append(c)
        self.log(f"cache frames ({cache_source}) in {time.perf_counter() - t1:.1f}s")

        # local correspondences per submap (frames base..base+S, local indices)
        t2 = time.perf_counter()
        locs, self.local_off, self.local_n = [], [], []
        off = 0
        for s in range(self.num_submaps):
            base = s * submap
            poses = self.gt[base:min(base + submap + 1, num_frames)]
            c = synth_correspondences(self.scene, poses, self.cam, max_per_pair=max_per_pair, min_covis=0.3,
                                      noise=0.0015, outlier_frac=0.0, seed=1000 + s) if len(poses) > 1 else \
                np.zeros(0, ENTRYJ_DTYPE)
            locs.append(c)
            self.local_off.append(off)
            self.local_n.append(len(c))
            off += len(c)
        allloc = np.concatenate(locs) if off else np.zeros(1, ENTRYJ_DTYPE)
        self.local_host = allloc
        self.local_corr = DeviceArray.from_host(allloc)
        # global keyframe correspondences, ordered by max(i, j) as keyframes arrive
        kf = self.gt[::submap][: self.K]
        g = synth_correspondences(self.scene, kf, self.cam, max_per_pair=max_per_pair, min_covis=0.3, noise=0.0015,
                                  outlier_frac=outliers, seed=2)
        order = np.argsort(np.maximum(g["i"], g["j"]), kind="stable")
        g = g[order]
        self.global_host = g
        self.global_corr = DeviceArray.from_host(g if len(g) else np.zeros(1, ENTRYJ_DTYPE))
        mx = np.maximum(g["i"], g["j"])
        self.global_prefix = np.searchsorted(mx, np.arange(self.K), side="right").astype(np.uint32)
        self.log(f"correspondences: {off} local, {len(g)} global in {time.perf_counter() - t2:.1f}s")

    def loop_cache(self):
        """A fresh CUDACache for one more loop over this stream (cache_source "loop": each loop builds its own)."""
        from .cache import CUDACache, cache_options
        w, h, fx, fy, mx, my, n, cw, ch = self._cache_args
        return CUDACache(cache_options(w, h, fx, fy, mx, my, n, width=cw, height=ch))

    def attach(self, recon, frames=None, cache_store=None, own_corr=False):
        """Register every frame, correspondence list and the initial pose with a Recon (cache_store: the loop's own
        cache for cache_source "loop", default the stream's). own_corr: the loop gets its own device copies of the
        correspondence lists — the solves invalidate entries in place (per-image cap, max-residual removal), so
        loops that run side by side (the ranks of a multi-GPU job, each with its own copy on its GPU) must not
        share them."""
        P4 = 4 * self.cam.imageWidth * self.cam.imageHeight
        for i in range(self.F if frames is None else frames):
            recon.set_frame(i, self.depth.ptr.value + P4 * i, self.color.ptr.value + P4 * i, self.cache[i], self.tinc[i])
        local_corr, global_corr = self.local_corr, self.global_corr
        if own_corr:
            local_corr = DeviceArray.from_host(self.local_host)
            global_corr = DeviceArray.from_host(self.global_host if len(self.global_host) else np.zeros(1, ENTRYJ_DTYPE))
            recon._keep = getattr(recon, "_keep", []) + [local_corr, global_corr]  # alive as long as the loop
        for s in range(self.num_submaps):
            if self.local_n[s]:
                recon.set_local_correspondences(s, local_corr.ptr.value + 32 * self.local_off[s], self.local_n[s])
        recon.set_global_correspondences(global_corr.ptr.value, len(self.global_host), self.global_prefix)
        recon.set_initial_pose(self.gt[0])
        if self.raw_input:  # CUDAImageManager::process of every frame inside process_frame
            from .io import Preprocessor, preprocess_options
            W, H = self.cam.imageWidth, self.cam.imageHeight
            self.preproc = Preprocessor((W, H), (W, H), (W, H), preprocess_options())
            for i in range(self.F if frames is None else frames):
                recon.set_frame_raw(i, self.depth_u16.ptr.value + 2 * W * H * i, self.rgbx.ptr.value + 4 * W * H * i)
            recon.attach_preproc(self.preproc)
        if self.cache_source == "loop":  # storeFrame of every frame inside process_frame (the frame store is the source)
            recon.attach_cache(cache_store or self.cache_store)


def write_synthetic_sens(path: str, num_frames: int, width: int = 640, height: int = 480, seed: int = 0,
                         color_codec: str = "jpeg", jpeg_quality: int = 90, device: bool = True, log=None,
                         threads: int = 8):
    """A `.sens` of the seeded synthetic room (SURVEY.md §8(d) inputs) in the copyroom / apt0 layout: JPEG
    (or PNG / raw) colour, zlib ushort depth in millimetres, the ground-truth camera trajectory, the depth
    camera's intrinsics. Frames are rendered on the GPU (device=True) or with the host renderer, and the
    colour is compressed with PIL (the image library mLib's SensorData uses for its colour streams). The
    compression of a frame runs on a thread pool (PIL and zlib release the GIL) while the next ones render;
    frames are written in order, so the file does not depend on `threads`."""
    import io as _io
    import zlib
    from collections import deque
    from concurrent.futures import ThreadPoolExecutor

    from .io import SensWriter, sens_info
    f = 577.87 * width / 640.0
    cam = depth_camera(width, height, fx=f, fy=f)
    K = np.eye(4, dtype=np.float32)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = cam.fx, cam.fy, cam.mx, cam.my
    cc = {"raw": 0, "png": 1, "jpeg": 2}[color_codec]
    scene = synth_scene(seed)
    if color_codec != "raw":
        from PIL import Image
    if device:
        dd = DeviceArray((height, width), np.float32)
        dc = DeviceArray((height, width, 4), np.uint8)

    def compress(d, c):
        # the renderer quantises to 1 mm (the .sens convention, SensorDataReader.cpp:104-107)
        du = np.where(np.isfinite(d) & (d > 0), np.rint(d * 1000.0), 0).astype(np.uint16)
        rgb = np.ascontiguousarray(c[..., :3])
        if cc == 0:
            col = rgb.tobytes()
        else:
            b = _io.BytesIO()
            Image.fromarray(rgb).save(b, "JPEG", quality=jpeg_quality) if cc == 2 else Image.fromarray(rgb).save(b, "PNG")
            col = b.getvalue()
        return col, zlib.compress(du.tobytes(), 1)

    t0 = time.perf_counter()
    last = t0
    pending = deque()
    with SensWriter(path, sens_info((width, height), (width, height), K, color_compression=cc)) as w, \
            ThreadPoolExecutor(max(1, threads)) as pool:
        def drain(limit):
            while len(pending) > limit:
                i, T, fut = pending.popleft()
                col, dep = fut.result()
                w.add_compressed_frame(T, col, dep, ts=(i, i))

        for i in range(num_frames):
            T = synth_pose(i)
            if device:
                check(lib().bf_synth_render(C.byref(scene), abi.mat(T), C.byref(cam), C.c_uint32(1), C.c_uint32(i),
                                            dd.ptr, dc.ptr))
                d, c = dd.download(), dc.download()
            else:
                from . import synth_render_host
                d, c = synth_render_host(scene, T, cam, 1, i)
            pending.append((i, T, pool.submit(compress, d, c)))
            drain(4 * max(1, threads))
            if log and time.perf_counter() - last > 20.0:
                log(f"  .sens frame {i}")
                last = time.perf_counter()
        drain(0)
    if log:
        log(f"wrote {num_frames} frames {width}x{height} ({color_codec}) to {path} in {time.perf_counter() - t0:.1f}s")
    return cam
