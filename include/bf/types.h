/*
 * bf/types.h — plain-old-data layouts shared by the HIP library, the C ABI,
 * the CPU oracle and the ctypes binding.
 *
 * Every struct mirrors the byte layout of the reference structure it replaces
 * so a FriedLiver-shaped host can hand its buffers over unchanged:
 *
 *   BFMat4              <- float4x4        Source/SiftGPU/cuda_SimpleMatrixUtil.h:855-875 (row-major m11..m44)
 *   BFHashEntry         <- HashEntry       Source/DepthSensing/VoxelUtilHashSDF.h:56-74   (32 B, __align__(16))
 *   BFVoxel             <- Voxel           Source/DepthSensing/VoxelUtilHashSDF.h:77-98   (12 B)
 *   BFHashParams        <- HashParams      Source/DepthSensing/CUDAHashParams.h:10-36     (224 B)
 *   BFDepthCameraParams <- DepthCameraParams Source/DepthSensing/CUDADepthCameraParams.h:7-19 (32 B)
 *   BFRayCastParams     <- RayCastParams   Source/DepthSensing/CUDARayCastParams.h:8-27   (192 B)
 *   BFEntryJ            <- EntryJ          Source/SiftGPU/SIFTImageManager.h:45-60        (32 B)
 *
 * C99/C++ compatible; no HIP or torch types.
 */
#ifndef BF_TYPES_H
#define BF_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BF_SDF_BLOCK_SIZE 8            /* VoxelUtilHashSDF.h:40 */
#define BF_HASH_BUCKET_SIZE 4          /* VoxelUtilHashSDF.h:41 */
#define BF_VOXELS_PER_BLOCK 512
#define BF_LOCK_ENTRY (-1)             /* VoxelUtilHashSDF.h:52 */
#define BF_FREE_ENTRY (-2)             /* VoxelUtilHashSDF.h:53 */
#define BF_INVALID_IMAGE 0xFFFFFFFFu   /* EntryJ::setInvalid, SIFTImageManager.h:51-54 */

typedef struct BFMat4 {
    float m[16]; /* row-major: m[r*4+c] */
} BFMat4;

typedef struct BFFloat3 { float x, y, z; } BFFloat3;
typedef struct BFInt3 { int32_t x, y, z; } BFInt3;

typedef struct __attribute__((aligned(16))) BFHashEntry {
    int32_t x, y, z;   /* SDF block coordinate (lower-left corner / 8) */
    int32_t ptr;       /* dumps: voxel index of the block's first voxel (= heap block * 512, the reference's
                          unit), or FREE/LOCK; on the device the scene keeps the heap block index here so
                          that more than 2^22 blocks fit (bf_scene_export converts) */
    uint32_t offset;   /* collision-list offset relative to the bucket's last slot */
    int32_t pad[3];
} BFHashEntry;

typedef struct BFVoxel {
    float sdf;
    float weight;
    uint8_t color[4];
} BFVoxel;

typedef struct __attribute__((aligned(16))) BFHashParams {
    BFMat4 rigidTransform;          /* camera -> world */
    BFMat4 rigidTransformInverse;   /* world -> camera */
    uint32_t hashNumBuckets;
    uint32_t hashBucketSize;
    uint32_t hashMaxCollisionLinkedListSize;
    uint32_t numSDFBlocks;
    int32_t SDFBlockSize;
    float virtualVoxelSize;
    uint32_t numOccupiedBlocks;
    float maxIntegrationDistance;
    float truncScale;
    float truncation;
    uint32_t integrationWeightSample;
    uint32_t integrationWeightMax;
    BFFloat3 streamingVoxelExtents;
    BFInt3 streamingGridDimensions;
    BFInt3 streamingMinGridPos;
    uint32_t streamingInitialChunkListSize;
    uint32_t dummy[2];
} BFHashParams;

typedef struct __attribute__((aligned(16))) BFDepthCameraParams {
    float fx, fy, mx, my;
    uint32_t imageWidth, imageHeight;
    float sensorDepthWorldMin;  /* render depth min (frustum) */
    float sensorDepthWorldMax;  /* render depth max (frustum) */
} BFDepthCameraParams;

typedef struct __attribute__((aligned(16))) BFRayCastParams {
    BFMat4 viewMatrix;          /* world -> camera */
    BFMat4 viewMatrixInverse;   /* camera -> world */
    float mx, my, fx, fy;
    uint32_t width, height;
    uint32_t numOccupiedSDFBlocks;
    uint32_t maxNumVertices;
    int32_t splatMinimum;
    float minDepth, maxDepth;
    float rayIncrement;
    float thresSampleDist;
    float thresDist;
    uint8_t useGradients;
    uint8_t pad_[3];
    uint32_t dummy0;
} BFRayCastParams;

typedef struct BFEntryJ {
    uint32_t imgIdx_i;
    uint32_t imgIdx_j;
    BFFloat3 pos_i;   /* camera-space point in frame i */
    BFFloat3 pos_j;   /* camera-space point in frame j */
} BFEntryJ;

/* Per-frame dense-term cache (CUDACachedFrame, Source/CUDACacheUtil.h:10-53), as a
 * struct of device pointers, one per cached frame. All images are W*H (80x60 default). */
typedef struct BFCachedFrame {
    const float* depth;          /* d_depthDownsampled */
    const float* campos;         /* d_cameraposDownsampled, float4 per pixel (x,y,z,w) */
    const float* normals;        /* d_normalsDownsampled, float4 per pixel */
    const uint8_t* normalsU8;    /* d_normalsDownsampledUCHAR4, uchar4 per pixel */
    const float* intensity;      /* d_intensityDownsampled */
    const float* intensityDeriv; /* d_intensityDerivsDownsampled, float2 per pixel */
} BFCachedFrame;

/* One scene call of the re-integration queue / reconstruction loop log (reintegrate(),
 * DepthSensing.cpp:854-902). */
typedef struct BFFixOp {
    int32_t kind;     /* 1 de-integrate (oldT), 2 integrate (newT), 3 re-integrate (oldT -> newT) */
    uint32_t frame;
    float oldT[16];
    float newT[16];
} BFFixOp;

/* Outcome of one bundle-adjustment solve (CUDASolverBundling::solve + computeMaxResidual). */
/* BFSolveResult.error bits */
#define BF_SOLVE_ERR_PAIR_BOUND 4u   /* more image pairs than the all-reduce's pair bound (sharded solves) */
#define BF_SOLVE_ERR_PCG_TIMEOUT 8u  /* a persistent PCG launch timed out and was not redone */
#define BF_SOLVE_PCG_RECOVERED 16u   /* a persistent PCG launch timed out and its GN step was redone with the
                                        per-iteration arithmetic: the result is valid (bit-identical to
                                        BFSolverOptions.pcgLaunch = 1) */
#define BF_SOLVE_ERR_FATAL (~BF_SOLVE_PCG_RECOVERED)

typedef struct BFSolveResult {
    uint32_t gnIterations;       /* Gauss-Newton iterations executed (early exit at max|delta| < 0.005) */
    uint32_t pcgIterations;      /* PCG iterations executed over all GN iterations */
    float maxResidual;           /* max_c max_k w*|r_c,k| (EvalMaxResidual + host max) */
    int32_t maxResidualIndex;    /* its correspondence index (lowest on ties) */
    float energy;                /* sum_c w |r_c|^2 (EvalResidual) */
    uint32_t highResidualCount;  /* correspondences with max residual > verifyOptDistThresh */
    uint32_t numDensePairs;      /* overlapping image pairs found by the dense term (last GN iter) */
    uint32_t error;              /* BF_SOLVE_ERR_* bits: nonzero under BF_SOLVE_ERR_FATAL means the poses
                                    are not a valid solve (the loop fails the call with BF_ERR_INTERNAL) */
    uint32_t skipped;            /* the solve was gated off (an invalidated local submap's global solve) */
    uint32_t verifyUsed;         /* the last verification ran its dense pair check (useVerification) */
    uint32_t verifyOk;           /* ... and passed (VerifyTrajectoryCU's d_validOpt) */
} BFSolveResult;

/* Ray-caster counters summed over renders (bf_recon_render_stats). */
typedef struct BFRenderStats {
    uint64_t samples;      /* trilinear SDF samples (traversal, bisection, gradients) */
    uint64_t voxelLoads;   /* 12-B voxel reads (a sample stops at its first zero-weight corner) */
    uint64_t hashProbes;   /* hash lookups (a per-ray one-block cache skips repeats) */
    uint64_t rays;         /* pixels with a splatted interval (marched) */
    uint64_t splatBlocks;  /* visible blocks rasterised by the interval splat */
    uint64_t splatAtomics; /* min / max depth updates of the splat (one per covered pixel and pass) */
    uint64_t renders;      /* renderKernel launches */
    uint64_t pixels;       /* pixels over those launches */
    uint64_t timedRenders; /* renders timed by the clocks below (enabled by the first bf_recon_render_time) */
    double renderMs;       /* summed renderKernel device time of the timed renders */
    double splatMs;        /* summed interval-splat device time of the timed renders */
    uint64_t waveSamples;  /* per renderKernel wave, 64 x its largest per-lane sample count: samples / waveSamples
                              is the fraction of the wave's march steps its lanes spend on samples */
    uint64_t waveSamplesMax; /* the largest per-lane sample count of any renderKernel wave (since the scene's creation) */
    uint64_t longWaves;    /* renderKernel waves whose largest per-lane sample count exceeds 32 */
} BFRenderStats;

/* Device-side counters used by the bench to compute algorithmic bytes. */
typedef struct BFTsdfStats {
    uint64_t pixels;          /* P: pixels read by alloc (valid or not) */
    uint64_t candidates;      /* U: candidate (absent, in-frustum) block lookups emitted by alloc */
    uint64_t allocated;       /* A: new hash entries written */
    uint64_t scanned;         /* blocks scanned by compactify (allocated blocks read) */
    uint64_t visible;         /* Nv summed over compactify calls */
    uint64_t voxelsUpdated;   /* V: voxels read-modify-written inside the truncation band */
    uint64_t gcBlocks;        /* blocks whose weights were scanned by GC */
    uint64_t gcFreed;         /* blocks freed by GC */
    uint64_t allocOverflow;   /* candidates dropped: candidate buffer / heap exhausted */
    uint64_t integrateOps;    /* integrate + de-integrate calls */
    uint64_t bandBlocks;      /* blocks on the voxel-update work lists (band-culled) */
    uint64_t voxelsRMW;       /* voxels read-modify-written by the update passes (a fused re-integration
                                 applies two updates to a voxel in one read + write) */
    /* the op-batch pass alone (bf_scene_apply_ops / k_apply_ops), also counted in the totals above */
    uint64_t batchOps;        /* voxel ops applied through batches */
    uint64_t batchBlocks;     /* work-list blocks of the batch passes */
    uint64_t batchVoxelsRMW;  /* voxels read + written once by a batch pass */
    uint64_t batchUpdates;    /* voxel-op updates inside the truncation band applied by batch passes */
    uint64_t batchEvals;      /* voxel-op evaluations (projection + band test) of the batch passes */
    uint64_t batchHalves;     /* block z-halves (256 voxels) a batch pass loaded: those some op's mask reaches */
} BFTsdfStats;

/* Capacity state of a scene (bf_scene_capacity / bf_recon_scene_capacity). The reference drops allocations
 * silently when its heap runs out (VoxelUtilHashSDF.h:535-540); here every dropped block sets a sticky error
 * bit, and the loop (bf_recon_*, bf_app_step) fails with BF_ERR_CAPACITY once one is set. */
typedef struct BFSceneCapacity {
    uint32_t errorFlags;         /* since the last reset: 1 alloc candidate buffer overflow, 2 heap exhausted,
                                    4 candidate dedup set congested (each drops blocks that should exist) */
    uint32_t peakCandidates;     /* largest alloc candidate count of one integrate / op batch since the reset
                                    (it may exceed candidateCapacity: the excess is what bit 1 dropped) */
    uint32_t candidateCapacity;  /* BFSceneOptions.candidateCapacity in effect */
    uint32_t heapFree;           /* getHeapFreeCount */
    uint32_t numSDFBlocks;       /* heap size */
    uint32_t highWater;          /* 1 + highest heap block index ever handed out */
} BFSceneCapacity;

/* mLib SensorData v4 header (SensorDataReader.cpp:45-60 reads these fields) */
typedef struct BFSensInfo {
    uint32_t version;              /* 4 */
    char sensorName[256];          /* truncated to 255 chars */
    float colorIntrinsic[16];      /* row-major mat4f */
    float colorExtrinsic[16];
    float depthIntrinsic[16];
    float depthExtrinsic[16];
    int32_t colorCompression;      /* -1 unknown, 0 raw (RGB, 3 B per pixel), 1 png, 2 jpeg */
    int32_t depthCompression;      /* -1 unknown, 0 raw ushort, 1 zlib ushort, 2 occi */
    uint32_t colorWidth, colorHeight, depthWidth, depthHeight;
    float depthShift;              /* ushort / depthShift = metres (1000) */
    uint32_t reserved;
    uint64_t numFrames;
} BFSensInfo;

/* CUDAImageManager::process (CUDAImageManager.cpp:22-158) input preprocessing; defaults in
 * brackets are zParametersBundlingDefault.txt's. */
typedef struct BFPreprocessOptions {
    int32_t erode;                 /* s_erodeSIFTdepth [1]: 2 passes of erodeDepthMap */
    int32_t erodeStructureSize;    /* [3] */
    float erodeDepthThresh;        /* [0.05] */
    float erodeFraction;           /* [0.3] */
    int32_t depthFilter;           /* s_depthFilter [1]: gaussFilterDepthMap */
    float sigmaD;                  /* s_depthSigmaD [2.0] */
    float sigmaR;                  /* s_depthSigmaR [0.05] */
    float depthShift;              /* ushort -> metres divisor [1000] */
} BFPreprocessOptions;

/* MarchingCubesParams (Source/DepthSensing/MarchingCubesSDFUtil.h:9-22), filled as
 * CUDAMarchingCubesHashSDF::parametersFromGlobalAppState (CUDAMarchingCubesHashSDF.h:19-28) does:
 * both thresholds = s_SDFMarchingCubeThreshFactor [10] * s_SDFVoxelSize; maxNumTriangles =
 * s_marchingCubesMaxNumTriangles [3 000 000]. */
typedef struct BFMarchingCubesParams {
    float threshMarchingCubes;     /* m_threshMarchingCubes: corner-pair sdf consistency bound */
    float threshMarchingCubes2;    /* m_threshMarchingCubes2: per-corner |sdf| bound */
    uint32_t boxEnabled;           /* m_boxEnabled: only voxels inside [minCorner, maxCorner] */
    uint32_t maxNumTriangles;      /* m_maxNumTriangles: output capacity (extra triangles dropped) */
    float minCorner[3];
    float maxCorner[3];
} BFMarchingCubesParams;

/* MarchingCubesData::Vertex / Triangle (MarchingCubesSDFUtil.h:32-43): float3 position, float3
 * colour in [0, 1]; 72 B per triangle. */
typedef struct BFMcVertex { float p[3]; float c[3]; } BFMcVertex;
typedef struct BFMcTriangle { BFMcVertex v[3]; } BFMcTriangle;

/* CUDACache construction parameters (CUDACache::CUDACache, CUDACache.cpp:15-42, as Bundler.cpp:33-38
 * creates it); zParametersBundlingDefault.txt values in brackets. A sigma <= 0 turns its filter off. */
typedef struct BFCacheOptions {
    uint32_t inputWidth, inputHeight;  /* depth input size (the SIFT depth size) */
    uint32_t width, height;            /* s_downsampledWidth / s_downsampledHeight [80 x 60] */
    uint32_t maxFrames;                /* m_maxNumImages */
    float inputIntrinsics[16];         /* row-major mat4f of the input depth camera */
    float colorSigma;                  /* s_colorDownSigma [2.5] */
    float depthSigmaD;                 /* s_depthDownSigmaD [1.0] */
    float depthSigmaR;                 /* s_depthDownSigmaR [0.05] */
} BFCacheOptions;

/* EntryJ producer from depth maps + poses (bf_corr_from_depth, the SiftGPU stand-in). */
typedef struct BFCorrOptions {
    float intrinsics[4];       /* fx, fy, cx, cy of the depth maps (projection into frame cur) */
    float intrinsicsInv[16];   /* row-major inverse intrinsics (AddCurrToResidualsCU's colorIntrinsicsInv) */
    uint32_t width, height;    /* depth map size */
    uint32_t stride;           /* sampling grid spacing in pixels */
    uint32_t maxPerPair;       /* MAX_MATCHES_PER_IMAGE_PAIR_FILTERED [25], <= 64 */
    float minDepth, maxDepth;  /* accepted depth range (metres) */
    float depthThresh;         /* |depth_cur - z| agreement (metres) */
    uint32_t minPerPair;       /* a pair with fewer matches keeps none (s_minNumMatchesLocal / Global [5]); 0 = 1 */
} BFCorrOptions;

#ifdef __cplusplus
} /* extern "C" */

static_assert(sizeof(BFMcTriangle) == 72, "MarchingCubesData::Triangle is 72 B");
static_assert(sizeof(BFMat4) == 64, "float4x4 is 64 B");
static_assert(sizeof(BFHashEntry) == 32, "HashEntry is 32 B");
static_assert(sizeof(BFVoxel) == 12, "Voxel is 12 B");
static_assert(sizeof(BFHashParams) == 224, "HashParams is 224 B");
static_assert(sizeof(BFDepthCameraParams) == 32, "DepthCameraParams is 32 B");
static_assert(sizeof(BFRayCastParams) == 192, "RayCastParams is 192 B");
static_assert(__builtin_offsetof(BFRayCastParams, useGradients) == 184, "m_useGradients at 184");
static_assert(sizeof(BFEntryJ) == 32, "EntryJ is 32 B");
#endif

#endif /* BF_TYPES_H */
