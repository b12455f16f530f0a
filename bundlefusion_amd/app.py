"""The FriedLiver application over the north-star path (bf_app_*, include/bf/bf.h): the mirror of
Source/FriedLiver.cpp's main() (:184-320) and the DepthSensing render loop (DepthSensing.cpp:966-1129,
StopScanningAndExit :904-953) for a `.sens` input.

    python -m bundlefusion_amd.app zParametersDefault.txt zParametersBundlingDefault.txt [file.sens]

reads the two parameter files (GlobalAppState / GlobalBundlingState; argv[3] overrides
s_binaryDumpSensorFile as FriedLiver.cpp:230-245 does), runs every frame through the loop, the
end-of-sequence phase, and writes the optimized trajectory (.sens), the mesh (.ply) and processed.txt.
The work is native (csrc/app.cpp); this module only marshals arguments."""
from __future__ import annotations

import argparse
import ctypes as C
import math
import os
import sys

import numpy as np

from . import check, lib
from .abi import BFAppInfo, BFAppOptions, BFAppResult, BFAppTiming, BFReconOptions


def _struct_dict(s):
    out = {}
    for k, _ in s._fields_:
        v = getattr(s, k)
        if isinstance(v, C.Structure):
            v = _struct_dict(v)
        elif isinstance(v, C.Array):
            v = list(v)
        out[k] = v
    return out


def resolve(app_params: str, bundling_params: str, sens_file: str | None = None, max_frames: int = 0):
    """Host only: what bf_app_create derives from the two zParameters files and the .sens header
    (bf_app_resolve; FriedLiver.cpp:228-250) -> (BFAppInfo, BFReconOptions of the loop)."""
    o = BFAppOptions()
    keep = os.fsencode(sens_file) if sens_file else None
    o.sensFile, o.maxFrames = keep, int(max_frames)
    info, loop = BFAppInfo(), BFReconOptions()
    check(lib().bf_app_resolve(os.fsencode(app_params), os.fsencode(bundling_params), C.byref(o), C.byref(info),
                               C.byref(loop)))
    return info, loop


class FriedLiver:
    """One run of the application: FriedLiver(app_params, bundling_params, sens_file).run()."""

    def __init__(self, app_params: str, bundling_params: str, sens_file: str | None = None, output_dir: str | None = None,
                 overwrite_sens: bool = False, skip_outputs: bool = False, async_bundling: int = 1,
                 record_ops: bool = False, enable_timing: bool = False, max_frames: int = 0,
                 front_end_drift=(math.radians(0.05), 0.002), front_end_seed: int = 1, corr_stride: int = 16,
                 corr_depth_thresh: float = 0.02, prefetch_frames: int = 16, decode_threads: int = 8,
                 num_solve_frames_before_exit: int = 0, shard=(1, 0), shard_chunk: float = 0.0, result_lag: int = 0):
        """shard = (count, index): this rank's TSDF chunk-ownership shard of a multi-GPU run (attach the ranks'
        communicator with set_comm before the first step)."""
        o = BFAppOptions()
        self._keep = [os.fsencode(sens_file) if sens_file else None, os.fsencode(output_dir) if output_dir else None]
        o.sensFile, o.outputDir = self._keep
        o.overwriteSens, o.skipOutputs = int(overwrite_sens), int(skip_outputs)
        o.asyncBundling, o.recordOps, o.enableTiming = int(async_bundling), int(record_ops), int(enable_timing)
        o.maxFrames = int(max_frames)
        if front_end_drift is None or (front_end_drift[0] == 0 and front_end_drift[1] == 0):
            o.noFrontEndDrift = 1
        else:
            o.frontEndDriftRad, o.frontEndDriftM = float(front_end_drift[0]), float(front_end_drift[1])
        o.frontEndSeed = int(front_end_seed)
        o.corrStride, o.corrDepthThresh = int(corr_stride), float(corr_depth_thresh)
        o.prefetchFrames, o.decodeThreads = int(prefetch_frames), int(decode_threads)
        o.numSolveFramesBeforeExit = int(num_solve_frames_before_exit)
        o.shardCount, o.shardIndex = int(shard[0]), int(shard[1])
        o.shardChunk, o.resultLag = float(shard_chunk), int(result_lag)
        self.h = C.c_void_p()
        check(lib().bf_app_create(os.fsencode(app_params), os.fsencode(bundling_params), C.byref(o), C.byref(self.h)))
        self._info = BFAppInfo()
        check(lib().bf_app_info(self.h, C.byref(self._info)))

    def close(self):
        if self.h:
            lib().bf_app_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def info(self) -> BFAppInfo:
        return self._info

    @property
    def num_frames(self) -> int:
        return int(self._info.numFrames)

    def step(self) -> bool:
        """One input frame (CUDAImageManager::process + processInput + OnD3D11FrameRender)."""
        got = C.c_int()
        check(lib().bf_app_step(self.h, C.byref(got)))
        return bool(got.value)

    def finish(self) -> dict:
        r = BFAppResult()
        check(lib().bf_app_finish(self.h, C.byref(r)))
        return _struct_dict(r)

    def run(self) -> dict:
        r = BFAppResult()
        check(lib().bf_app_run(self.h, C.byref(r)))
        return _struct_dict(r)

    @property
    def recon(self):
        """The app's loop (bundlefusion_amd.recon.Recon view) for op logs, submap poses, trajectories."""
        from .recon import Recon
        h = C.c_void_p()
        check(lib().bf_app_recon(self.h, C.byref(h)))
        return Recon.borrowed(h, self._info.hashParams, self._info.integrationCamera, owner=self)

    def set_comm(self, comm):
        """The ranks' RCCL communicator (dist.Comm): round-robin local solves + the global solve's pair-stat
        all-reduce (bf_recon_set_comm on the app's loop); before the first step."""
        self._comm = comm
        self.recon.set_comm(comm)

    def timing(self) -> dict:
        """Host time per section of the frame loop so far (decode wait, upload + preprocessing, EntryJ, loop)."""
        t = BFAppTiming()
        check(lib().bf_app_timing(self.h, C.byref(t)))
        return _struct_dict(t)

    def front_end_pose(self, f: int) -> np.ndarray:
        T = (C.c_float * 16)()
        check(lib().bf_app_front_end_pose(self.h, C.c_uint32(f), T))
        return np.array(T, np.float32).reshape(4, 4)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="FriedLiver over the MI355X path: zParameters + .sens -> trajectory, mesh")
    ap.add_argument("app_params", nargs="?", default="zParametersDefault.txt")
    ap.add_argument("bundling_params", nargs="?", default="zParametersBundlingDefault.txt")
    ap.add_argument("sens", nargs="?", default=None, help="overrides s_binaryDumpSensorFile (FriedLiver argv[3])")
    ap.add_argument("--output-dir", default=None)
    ap.add_argument("--overwrite-sens", action="store_true",
                    help="write the trajectory into the input .sens, as the reference does")
    ap.add_argument("--max-frames", type=int, default=0)
    a = ap.parse_args(argv)
    app = FriedLiver(a.app_params, a.bundling_params, a.sens, output_dir=a.output_dir, overwrite_sens=a.overwrite_sens,
                     max_frames=a.max_frames)
    r = app.run()
    print(f"[ stop scanning and exit ] {r['frames']} frames in {r['loopSeconds']:.1f} s "
          f"({r['frames'] / max(r['loopSeconds'], 1e-9):.1f} frames/s), end phase {r['endSeconds']:.1f} s, "
          f"#VALID TRANSFORMS = {r['numValidTransforms']} of {r['numTransforms']}, heap free {r['heapFreeCount']}, "
          f"{r['meshTriangles']} triangles, valid = {bool(r['valid'])}")
    app.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
