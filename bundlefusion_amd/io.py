"""Input formats and preprocessing over the C ABI: `.sens` reading / writing
(mLib SensorData v4, SensorDataReader.cpp:38-116), `zParameters*.txt` (mLib ParameterFile behind
GlobalAppState / GlobalBundlingState) and CUDAImageManager::process's preprocessing on the GPU."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import DeviceArray, abi, check, lib
from .abi import BFHashParams, BFPreprocessOptions, BFRayCastParams, BFSensInfo


def _mat(a) -> C.Array:
    return abi.mat(np.asarray(a, np.float32).reshape(4, 4))


class SensorData:
    """Reader of a .sens file; frames are decoded on demand."""

    def __init__(self, path: str):
        self.h = C.c_void_p()
        check(lib().bf_sens_open(path.encode(), C.byref(self.h)))
        self.info = BFSensInfo()
        check(lib().bf_sens_info(self.h, C.byref(self.info)))

    def close(self):
        if self.h:
            lib().bf_sens_close(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        return int(self.info.numFrames)

    @property
    def sensor_name(self) -> str:
        return self.info.sensorName.decode()

    def intrinsics(self, which="depth") -> np.ndarray:
        return np.array(getattr(self.info, which + "Intrinsic"), np.float32).reshape(4, 4)

    def pose(self, f: int) -> np.ndarray:
        T = (C.c_float * 16)()
        check(lib().bf_sens_frame_pose(self.h, C.c_uint64(f), T))
        return np.array(T, np.float32).reshape(4, 4)

    def timestamps(self, f: int):
        a, b = C.c_uint64(), C.c_uint64()
        check(lib().bf_sens_frame_timestamps(self.h, C.c_uint64(f), C.byref(a), C.byref(b)))
        return a.value, b.value

    def depth_u16(self, f: int) -> np.ndarray:
        out = np.empty((self.info.depthHeight, self.info.depthWidth), np.uint16)
        check(lib().bf_sens_read_depth_u16(self.h, C.c_uint64(f), out.ctypes.data_as(C.c_void_p)))
        return out

    def depth(self, f: int) -> np.ndarray:
        """SensorDataReader::processDepth: d / depthShift, 0 -> -inf."""
        out = np.empty((self.info.depthHeight, self.info.depthWidth), np.float32)
        check(lib().bf_sens_read_depth(self.h, C.c_uint64(f), out.ctypes.data_as(C.c_void_p)))
        return out

    def color(self, f: int) -> np.ndarray:
        out = np.empty((self.info.colorHeight, self.info.colorWidth, 4), np.uint8)
        check(lib().bf_sens_read_color(self.h, C.c_uint64(f), out.ctypes.data_as(C.c_void_p)))
        return out


def decode_image(data: bytes, compression: int) -> np.ndarray:
    """The .sens colour-stream decoders (compression 1 = PNG, 2 = JPEG) -> H x W x 4 RGBX."""
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
    w, h = C.c_uint32(), C.c_uint32()
    check(lib().bf_image_decode(buf, C.c_uint64(len(data)), C.c_int(compression), C.byref(w), C.byref(h), None,
                                C.c_uint64(0)))
    out = np.empty((h.value, w.value, 4), np.uint8)
    check(lib().bf_image_decode(buf, C.c_uint64(len(data)), C.c_int(compression), C.byref(w), C.byref(h),
                                out.ctypes.data_as(C.c_void_p), C.c_uint64(out.nbytes)))
    return out


def write_sens(path: str, depth_u16, rgbx, poses, depth_intrinsic, color_intrinsic=None, depth_shift=1000.0,
               zlib_depth=True, name="bundlefusion_amd synthetic", timestamps=None):
    """SensorData::saveToFile layout: raw RGB colour, zlib (or raw) ushort depth."""
    depth_u16 = np.ascontiguousarray(depth_u16, np.uint16)
    rgbx = np.ascontiguousarray(rgbx, np.uint8)
    F, dh, dw = depth_u16.shape
    ch, cw = rgbx.shape[1:3]
    info = BFSensInfo()
    info.version = 4
    info.sensorName = name.encode()[:255]
    ident = np.eye(4, dtype=np.float32).reshape(16)
    info.depthIntrinsic[:] = np.asarray(depth_intrinsic, np.float32).reshape(16)
    info.colorIntrinsic[:] = np.asarray(color_intrinsic if color_intrinsic is not None else depth_intrinsic,
                                        np.float32).reshape(16)
    info.depthExtrinsic[:] = ident
    info.colorExtrinsic[:] = ident
    info.colorCompression = 0
    info.depthCompression = 1 if zlib_depth else 0
    info.colorWidth, info.colorHeight, info.depthWidth, info.depthHeight = cw, ch, dw, dh
    info.depthShift = depth_shift
    w = C.c_void_p()
    check(lib().bf_sens_writer_create(path.encode(), C.byref(info), C.byref(w)))
    try:
        for f in range(F):
            tc, td = (timestamps[f] if timestamps is not None else (f, f))
            check(lib().bf_sens_writer_add_frame(w, _mat(poses[f]), C.c_uint64(tc), C.c_uint64(td),
                                                 depth_u16[f].ctypes.data_as(C.c_void_p),
                                                 rgbx[f].ctypes.data_as(C.c_void_p)))
    finally:
        check(lib().bf_sens_writer_close(w))


class SensWriter:
    """bf_sens_writer_*: frames encoded here (raw RGB, raw / zlib depth) or passed pre-compressed (e.g. JPEG
    colour + zlib depth: the copyroom / apt0 layout)."""

    def __init__(self, path: str, info: BFSensInfo):
        self.h = C.c_void_p()
        check(lib().bf_sens_writer_create(path.encode(), C.byref(info), C.byref(self.h)))

    def add_frame(self, pose, depth_u16: np.ndarray, rgbx: np.ndarray, ts=(0, 0)):
        d = np.ascontiguousarray(depth_u16, np.uint16)
        c = np.ascontiguousarray(rgbx, np.uint8)
        check(lib().bf_sens_writer_add_frame(self.h, _mat(pose), C.c_uint64(ts[0]), C.c_uint64(ts[1]),
                                             d.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p)))

    def add_compressed_frame(self, pose, color: bytes, depth: bytes, ts=(0, 0)):
        cb = (C.c_uint8 * max(1, len(color))).from_buffer_copy(color or b"\0")
        db = (C.c_uint8 * max(1, len(depth))).from_buffer_copy(depth or b"\0")
        check(lib().bf_sens_writer_add_compressed_frame(self.h, _mat(pose), C.c_uint64(ts[0]), C.c_uint64(ts[1]), cb,
                                                        C.c_uint64(len(color)), db, C.c_uint64(len(depth))))

    def close(self):
        if self.h:
            check(lib().bf_sens_writer_close(self.h))
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def sens_info(depth_wh, color_wh, depth_intrinsic, color_intrinsic=None, color_compression=0, depth_compression=1,
              depth_shift=1000.0, name="bundlefusion_amd synthetic") -> BFSensInfo:
    info = BFSensInfo()
    info.version = 4
    info.sensorName = name.encode()[:255]
    ident = np.eye(4, dtype=np.float32).reshape(16)
    info.depthIntrinsic[:] = np.asarray(depth_intrinsic, np.float32).reshape(16)
    info.colorIntrinsic[:] = np.asarray(color_intrinsic if color_intrinsic is not None else depth_intrinsic,
                                        np.float32).reshape(16)
    info.depthExtrinsic[:] = ident
    info.colorExtrinsic[:] = ident
    info.colorCompression, info.depthCompression = color_compression, depth_compression
    info.depthWidth, info.depthHeight = depth_wh
    info.colorWidth, info.colorHeight = color_wh
    info.depthShift = depth_shift
    return info


class ParameterFile:
    """zParameters*.txt; later loads override earlier keys."""

    def __init__(self, *paths: str):
        self.h = C.c_void_p()
        check(lib().bf_params_create(C.byref(self.h)))
        for p in paths:
            self.load(p)

    def load(self, path: str):
        check(lib().bf_params_load(self.h, path.encode()))

    def __del__(self):
        try:
            lib().bf_params_destroy(self.h)
        except Exception:
            pass

    def __contains__(self, key: str) -> bool:
        f = C.c_int()
        check(lib().bf_params_has(self.h, key.encode(), C.byref(f)))
        return bool(f.value)

    def string(self, key: str) -> str:
        buf = C.create_string_buffer(4096)
        check(lib().bf_params_get_string(self.h, key.encode(), buf, C.c_size_t(4096)))
        return buf.value.decode()

    def floats(self, key: str) -> np.ndarray:
        n = C.c_uint32()
        check(lib().bf_params_get_floats(self.h, key.encode(), None, 0, C.byref(n)))
        out = (C.c_float * max(1, n.value))()
        check(lib().bf_params_get_floats(self.h, key.encode(), out, n.value, C.byref(n)))
        return np.array(out[:n.value], np.float32)

    def number(self, key: str) -> float:
        v = C.c_double()
        check(lib().bf_params_get_number(self.h, key.encode(), C.byref(v)))
        return v.value

    def boolean(self, key: str) -> bool:
        v = C.c_int()
        check(lib().bf_params_get_bool(self.h, key.encode(), C.byref(v)))
        return bool(v.value)

    def hash_params(self) -> BFHashParams:
        p = BFHashParams()
        check(lib().bf_params_hash_params(self.h, C.byref(p)))
        return p

    def raycast_params(self, fx, fy, mx, my) -> BFRayCastParams:
        p = BFRayCastParams()
        check(lib().bf_params_raycast_params(self.h, C.c_float(fx), C.c_float(fy), C.c_float(mx), C.c_float(my),
                                             C.byref(p)))
        return p

    def preprocess_options(self, depth_shift=1000.0) -> BFPreprocessOptions:
        o = BFPreprocessOptions()
        check(lib().bf_params_preprocess_options(self.h, C.c_float(depth_shift), C.byref(o)))
        return o


def preprocess_options(erode=True, structure=3, erode_thresh=0.05, erode_fraction=0.3, depth_filter=True,
                       sigma_d=2.0, sigma_r=0.05, depth_shift=1000.0) -> BFPreprocessOptions:
    """zParametersBundlingDefault.txt values (s_erodeSIFTdepth, s_depthFilter, s_depthSigmaD/R)."""
    return BFPreprocessOptions(1 if erode else 0, structure, erode_thresh, erode_fraction, 1 if depth_filter else 0,
                               sigma_d, sigma_r, depth_shift)


class Preprocessor:
    """CUDAImageManager::process on the GPU: device in, device out."""

    def __init__(self, depth_wh, color_wh, integration_wh, opts: BFPreprocessOptions):
        self.h = C.c_void_p()
        check(lib().bf_preproc_create(depth_wh[0], depth_wh[1], color_wh[0], color_wh[1], integration_wh[0],
                                      integration_wh[1], C.byref(opts), C.byref(self.h)))
        self.iw, self.ih = integration_wh

    def __del__(self):
        try:
            lib().bf_preproc_destroy(self.h)
        except Exception:
            pass

    def run(self, depth_u16: DeviceArray, rgbx: DeviceArray | None, depth_out: DeviceArray, color_out: DeviceArray | None):
        check(lib().bf_preproc_run(self.h, depth_u16.ptr, rgbx.ptr if rgbx is not None else None, depth_out.ptr,
                                   color_out.ptr if color_out is not None else None))
        check(lib().bf_preproc_synchronize(self.h))

    def run_async(self, depth_u16_ptr: int, rgbx_ptr: int, depth_out_ptr: int, color_out_ptr: int):
        """bf_preproc_run without the wait: queued on self.stream"""
        check(lib().bf_preproc_run(self.h, C.c_void_p(depth_u16_ptr), C.c_void_p(rgbx_ptr), C.c_void_p(depth_out_ptr),
                                   C.c_void_p(color_out_ptr)))

    @property
    def stream(self) -> int:
        s = C.c_void_p()
        check(lib().bf_preproc_stream(self.h, C.byref(s)))
        return s.value or 0
