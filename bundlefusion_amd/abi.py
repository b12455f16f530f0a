"""ctypes mirror of include/bf/types.h and include/bf/bf.h.

This is binding plumbing for tests and bench.py: the product is the C ABI in
libbf_hip.so. Struct layouts are asserted against the sizes the C header
static_asserts (HashEntry 32 B, Voxel 12 B, HashParams 224 B, ...).
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(_HERE)
# BF_HIP_LIB: an alternative build of the same library (A/B timing of kernel variants: the ab: step of tools/gpu.sh)
LIB_PATH = os.environ.get("BF_HIP_LIB") or os.path.join(_HERE, "libbf_hip.so")
HEADER_PATH = os.path.join(REPO, "include", "bf", "bf.h")

FREE_ENTRY = -2
LOCK_ENTRY = -1
SDF_BLOCK_SIZE = 8
HASH_BUCKET_SIZE = 4


class BFMat4(C.Structure):
    _fields_ = [("m", C.c_float * 16)]


class BFFloat3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class BFInt3(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("z", C.c_int32)]


class BFHashParams(C.Structure):
    _fields_ = [
        ("rigidTransform", BFMat4),
        ("rigidTransformInverse", BFMat4),
        ("hashNumBuckets", C.c_uint32),
        ("hashBucketSize", C.c_uint32),
        ("hashMaxCollisionLinkedListSize", C.c_uint32),
        ("numSDFBlocks", C.c_uint32),
        ("SDFBlockSize", C.c_int32),
        ("virtualVoxelSize", C.c_float),
        ("numOccupiedBlocks", C.c_uint32),
        ("maxIntegrationDistance", C.c_float),
        ("truncScale", C.c_float),
        ("truncation", C.c_float),
        ("integrationWeightSample", C.c_uint32),
        ("integrationWeightMax", C.c_uint32),
        ("streamingVoxelExtents", BFFloat3),
        ("streamingGridDimensions", BFInt3),
        ("streamingMinGridPos", BFInt3),
        ("streamingInitialChunkListSize", C.c_uint32),
        ("dummy", C.c_uint32 * 2),
    ]


class BFDepthCameraParams(C.Structure):
    _fields_ = [
        ("fx", C.c_float), ("fy", C.c_float), ("mx", C.c_float), ("my", C.c_float),
        ("imageWidth", C.c_uint32), ("imageHeight", C.c_uint32),
        ("sensorDepthWorldMin", C.c_float), ("sensorDepthWorldMax", C.c_float),
    ]


class BFRayCastParams(C.Structure):
    _fields_ = [
        ("viewMatrix", BFMat4), ("viewMatrixInverse", BFMat4),
        ("mx", C.c_float), ("my", C.c_float), ("fx", C.c_float), ("fy", C.c_float),
        ("width", C.c_uint32), ("height", C.c_uint32),
        ("numOccupiedSDFBlocks", C.c_uint32), ("maxNumVertices", C.c_uint32), ("splatMinimum", C.c_int32),
        ("minDepth", C.c_float), ("maxDepth", C.c_float), ("rayIncrement", C.c_float),
        ("thresSampleDist", C.c_float), ("thresDist", C.c_float),
        ("useGradients", C.c_uint8), ("pad_", C.c_uint8 * 3), ("dummy0", C.c_uint32),
    ]


class BFMarchingCubesParams(C.Structure):
    _fields_ = [("threshMarchingCubes", C.c_float), ("threshMarchingCubes2", C.c_float),
                ("boxEnabled", C.c_uint32), ("maxNumTriangles", C.c_uint32),
                ("minCorner", C.c_float * 3), ("maxCorner", C.c_float * 3)]


class BFTsdfStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "pixels", "candidates", "allocated", "scanned", "visible", "voxelsUpdated",
        "gcBlocks", "gcFreed", "allocOverflow", "integrateOps", "bandBlocks", "voxelsRMW",
        "batchOps", "batchBlocks", "batchVoxelsRMW", "batchUpdates", "batchEvals", "batchHalves")]


class BFSceneOptions(C.Structure):
    _fields_ = [("candidateCapacity", C.c_uint32), ("shardCount", C.c_uint32),
                ("shardIndex", C.c_uint32), ("shardChunk", C.c_float),
                ("applyXcdRun", C.c_uint32), ("applyRounds", C.c_uint32), ("testFlags", C.c_uint32),
                ("splatRowCap", C.c_uint32)]


BF_SCENE_TEST_ALLOC_DIRECT = 1


class BFSceneCapacity(C.Structure):  # include/bf/types.h
    _fields_ = [(n, C.c_uint32) for n in ("errorFlags", "peakCandidates", "candidateCapacity", "heapFree",
                                          "numSDFBlocks", "highWater")]


class BFSynthScene(C.Structure):
    _fields_ = [("seed", C.c_uint32), ("numPrimitives", C.c_uint32),
                ("roomMin", C.c_float * 3), ("roomMax", C.c_float * 3),
                ("prims", (C.c_float * 8) * 64)]


# numpy views of the POD arrays
HASH_ENTRY_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("z", "<i4"), ("ptr", "<i4"),
                             ("offset", "<u4"), ("pad", "<i4", (3,))])
VOXEL_DTYPE = np.dtype([("sdf", "<f4"), ("weight", "<f4"), ("color", "u1", (4,))])
ENTRYJ_DTYPE = np.dtype([("i", "<u4"), ("j", "<u4"), ("pos_i", "<f4", (3,)), ("pos_j", "<f4", (3,))])

assert C.sizeof(BFMat4) == 64
assert C.sizeof(BFHashParams) == 224, C.sizeof(BFHashParams)
assert C.sizeof(BFDepthCameraParams) == 32
assert C.sizeof(BFRayCastParams) == 192, C.sizeof(BFRayCastParams)
assert BFRayCastParams.useGradients.offset == 184
assert HASH_ENTRY_DTYPE.itemsize == 32 and VOXEL_DTYPE.itemsize == 12 and ENTRYJ_DTYPE.itemsize == 32


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Every `bf_*` function declared in include/bf/bf.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(?:int|const char\s*\*)\s+(bf_[a-z0-9_]+)\s*\(", text)))


def mat(T) -> C.Array:
    a = np.ascontiguousarray(np.asarray(T, dtype=np.float32).reshape(16))
    return (C.c_float * 16)(*a.tolist())


def f32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def u8p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def u32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def vp(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class BFCachedFrame(C.Structure):
    _fields_ = [("depth", C.c_void_p), ("campos", C.c_void_p), ("normals", C.c_void_p), ("normalsU8", C.c_void_p),
                ("intensity", C.c_void_p), ("intensityDeriv", C.c_void_p)]


class BFSolverOptions(C.Structure):
    _fields_ = [("denseDistThresh", C.c_float), ("denseNormalThresh", C.c_float), ("denseColorThresh", C.c_float),
                ("denseColorGradientMin", C.c_float), ("denseDepthMin", C.c_float), ("denseDepthMax", C.c_float),
                ("denseOverlapSubsample", C.c_uint32), ("verifyOptDistThresh", C.c_float),
                ("normalEquations", C.c_int32), ("disableEarlyOut", C.c_int32),
                ("pcgLaunch", C.c_int32), ("pcgSpinLimitUs", C.c_uint32)]

ABI_VERSION = 4  # include/bf/bf.h BF_ABI_VERSION: the struct layouts above
SOLVE_ERR_PAIR_BOUND, SOLVE_ERR_PCG_TIMEOUT, SOLVE_PCG_RECOVERED = 4, 8, 16  # BFSolveResult.error bits
SOLVE_ERR_FATAL = 0xFFFFFFFF & ~SOLVE_PCG_RECOVERED

NORMAL_EQ_AUTO, NORMAL_EQ_MATRIX_FREE, NORMAL_EQ_ASSEMBLED = 0, 1, 2
PAIR_STATS = 28  # doubles per image pair of the assembled normal equations (bf_solver_export_pairs)


class BFSolveResult(C.Structure):
    _fields_ = [("gnIterations", C.c_uint32), ("pcgIterations", C.c_uint32), ("maxResidual", C.c_float),
                ("maxResidualIndex", C.c_int32), ("energy", C.c_float), ("highResidualCount", C.c_uint32),
                ("numDensePairs", C.c_uint32), ("error", C.c_uint32), ("skipped", C.c_uint32),
                ("verifyUsed", C.c_uint32), ("verifyOk", C.c_uint32)]


class BFVerifyOptions(C.Structure):  # include/bf/bf.h: local-submap verification thresholds (0 = default)
    _fields_ = [("projCorrDistThresh", C.c_float), ("projCorrNormalThresh", C.c_float),
                ("verifyOptErrThresh", C.c_float), ("verifyOptCorrThresh", C.c_float),
                ("verifyOptPercentThresh", C.c_float), ("sensorDepthMin", C.c_float), ("sensorDepthMax", C.c_float),
                ("always", C.c_int32)]


class BFSensInfo(C.Structure):  # include/bf/types.h, mLib SensorData v4 header
    _fields_ = [("version", C.c_uint32), ("sensorName", C.c_char * 256),
                ("colorIntrinsic", C.c_float * 16), ("colorExtrinsic", C.c_float * 16),
                ("depthIntrinsic", C.c_float * 16), ("depthExtrinsic", C.c_float * 16),
                ("colorCompression", C.c_int32), ("depthCompression", C.c_int32),
                ("colorWidth", C.c_uint32), ("colorHeight", C.c_uint32), ("depthWidth", C.c_uint32),
                ("depthHeight", C.c_uint32), ("depthShift", C.c_float), ("reserved", C.c_uint32),
                ("numFrames", C.c_uint64)]


class BFPreprocessOptions(C.Structure):  # include/bf/types.h
    _fields_ = [("erode", C.c_int32), ("erodeStructureSize", C.c_int32), ("erodeDepthThresh", C.c_float),
                ("erodeFraction", C.c_float), ("depthFilter", C.c_int32), ("sigmaD", C.c_float),
                ("sigmaR", C.c_float), ("depthShift", C.c_float)]


class BFCacheOptions(C.Structure):  # include/bf/types.h
    _fields_ = [("inputWidth", C.c_uint32), ("inputHeight", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("maxFrames", C.c_uint32), ("inputIntrinsics", C.c_float * 16), ("colorSigma", C.c_float),
                ("depthSigmaD", C.c_float), ("depthSigmaR", C.c_float)]


class BFCorrOptions(C.Structure):  # include/bf/types.h
    _fields_ = [("intrinsics", C.c_float * 4), ("intrinsicsInv", C.c_float * 16), ("width", C.c_uint32),
                ("height", C.c_uint32), ("stride", C.c_uint32), ("maxPerPair", C.c_uint32), ("minDepth", C.c_float),
                ("maxDepth", C.c_float), ("depthThresh", C.c_float),
                ("minPerPair", C.c_uint32)]


class BFVoxelOp(C.Structure):  # include/bf/bf.h
    _fields_ = [("T", C.c_float * 16), ("depth", C.c_void_p), ("color", C.c_void_p), ("deintegrate", C.c_uint32),
                ("reserved", C.c_uint32)]


MAX_VOXEL_OPS = 24


class BFFixOp(C.Structure):
    _fields_ = [("kind", C.c_int32), ("frame", C.c_uint32), ("oldT", C.c_float * 16), ("newT", C.c_float * 16)]


class BFReconOptions(C.Structure):
    _fields_ = [("maxFrames", C.c_uint32), ("submapSize", C.c_uint32), ("maxFrameFixes", C.c_uint32),
                ("topNActive", C.c_uint32), ("minPoseDistSqrt", C.c_float),
                ("localNonLin", C.c_uint32), ("localLin", C.c_uint32), ("globalNonLin", C.c_uint32),
                ("globalLin", C.c_uint32), ("maxKeyframes", C.c_uint32), ("maxLocalCorr", C.c_uint32),
                ("maxGlobalCorr", C.c_uint32), ("maxResidualThresh", C.c_float), ("useLocalDense", C.c_int32),
                ("cacheWidth", C.c_uint32), ("cacheHeight", C.c_uint32), ("cacheIntrinsics", C.c_float * 4),
                ("enableTiming", C.c_int32), ("recordOps", C.c_int32), ("asyncBundling", C.c_int32),
                ("solver", BFSolverOptions), ("disableLocalVerify", C.c_int32), ("verify", BFVerifyOptions),
                ("resultLag", C.c_uint32), ("bundlingPriority", C.c_int32)]


class BFRenderStats(C.Structure):  # include/bf/bf.h
    _fields_ = [(n, C.c_uint64) for n in ("samples", "voxelLoads", "hashProbes", "rays", "splatBlocks", "splatAtomics",
                                          "renders", "pixels", "timedRenders")] + [
        ("renderMs", C.c_double), ("splatMs", C.c_double), ("waveSamples", C.c_uint64),
        ("waveSamplesMax", C.c_uint64), ("longWaves", C.c_uint64)]


class BFEndSequenceOptions(C.Structure):  # include/bf/bf.h: the render loop past the last frame
    _fields_ = [("numSolveFramesBeforeExit", C.c_int32), ("disableDenseAtEnd", C.c_int32),
                ("denseFrameLimit", C.c_uint32), ("denseDepthWeight", C.c_float), ("maxPastEndFrames", C.c_uint32)]


class BFEndSequenceResult(C.Structure):
    _fields_ = [("pastEndFrames", C.c_uint32), ("globalSolves", C.c_uint32), ("localSolved", C.c_uint32),
                ("denseSolve", C.c_uint32), ("queueDrained", C.c_uint32), ("denseSolveMs", C.c_float),
                ("last", BFSolveResult)]


class BFQueueEvent(C.Structure):  # include/bf/bf.h: one TrajectoryManager call of the loop (recordOps)
    _fields_ = [("kind", C.c_int32), ("frame", C.c_uint32), ("count", C.c_uint32), ("offset", C.c_uint32)]


class BFAppOptions(C.Structure):  # include/bf/bf.h: the FriedLiver application (bf_app_*)
    _fields_ = [("sensFile", C.c_char_p), ("outputDir", C.c_char_p), ("overwriteSens", C.c_int32),
                ("skipOutputs", C.c_int32), ("asyncBundling", C.c_int32), ("recordOps", C.c_int32),
                ("enableTiming", C.c_int32), ("maxFrames", C.c_uint32), ("frontEndDriftRad", C.c_float),
                ("frontEndDriftM", C.c_float), ("frontEndSeed", C.c_uint32), ("noFrontEndDrift", C.c_int32),
                ("corrStride", C.c_uint32), ("corrDepthThresh", C.c_float), ("prefetchFrames", C.c_uint32),
                ("decodeThreads", C.c_uint32), ("numSolveFramesBeforeExit", C.c_int32),
                ("shardCount", C.c_uint32), ("shardIndex", C.c_uint32), ("shardChunk", C.c_float),
                ("resultLag", C.c_uint32), ("bundlingPriority", C.c_int32)]


class BFAppInfo(C.Structure):
    _fields_ = [("hashParams", BFHashParams), ("integrationCamera", BFDepthCameraParams), ("numFrames", C.c_uint32),
                ("sensorDepthWidth", C.c_uint32), ("sensorDepthHeight", C.c_uint32), ("sensorColorWidth", C.c_uint32),
                ("sensorColorHeight", C.c_uint32),
                ("preprocess", BFPreprocessOptions), ("cache", BFCacheOptions), ("corr", BFCorrOptions),
                ("cacheIntrinsics", C.c_float * 4), ("submapSize", C.c_uint32), ("maxKeyframes", C.c_uint32),
                ("maxLocalCorr", C.c_uint32), ("maxGlobalCorr", C.c_uint32), ("numSolveFramesBeforeExit", C.c_int32),
                ("reserved", C.c_uint32 * 2)]


class BFAppResult(C.Structure):
    _fields_ = [("frames", C.c_uint32), ("loopSeconds", C.c_double), ("endSeconds", C.c_double),
                ("end", BFEndSequenceResult), ("heapFreeCount", C.c_uint32), ("numTransforms", C.c_uint32),
                ("numValidTransforms", C.c_uint32), ("valid", C.c_int32), ("meshTriangles", C.c_uint32),
                ("meshVertices", C.c_uint32), ("meshFaces", C.c_uint32)]


class BFAppTiming(C.Structure):  # include/bf/bf.h: the app's host time per section (bf_app_timing)
    _fields_ = [("frames", C.c_uint32), ("decodeThreads", C.c_uint32)] + [
        (n, C.c_double) for n in ("stepSeconds", "decodeWaitSeconds", "uploadSeconds", "corrSeconds", "loopSeconds",
                                  "decodeSeconds", "uploadBytes")]


class BFReconStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "frames", "integrations", "deintegrations", "fixOps", "localSolves", "globalSolves",
        "globalGnIterations", "globalPcgIterations", "localGnIterations", "localPcgIterations",
        "removedPairs", "integrateLaunches")] + [
        ("integrateKernelMs", C.c_double), ("localSolveMs", C.c_double), ("globalSolveMs", C.c_double),
        ("reintegrateLaunches", C.c_uint64), ("reintegrateKernelMs", C.c_double),
        ("localVerifications", C.c_uint64), ("invalidLocals", C.c_uint64), ("endSolves", C.c_uint64),
        ("pcgRecoveries", C.c_uint64), ("hostMs", C.c_double), ("hostWaitMs", C.c_double),
        ("globalPcgLaunches", C.c_uint64), ("globalPcgKernelMs", C.c_double), ("renders", C.c_uint64)]
