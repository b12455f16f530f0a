/*
 * bf/bf.h — C ABI of the MI355X-native BundleFusion hot path (libbf_hip.so).
 *
 * Plain C: opaque handles, POD structs from bf/types.h, raw pointers and sizes. No HIP,
 * torch or C++ types cross this boundary. Every function returns an int status
 * (0 = ok, < 0 = error) and bf_last_error() returns the message of the last failure
 * on the calling thread. Handles are bound to the device current at creation and
 * carry their own HIP stream; there is no global constant state (the reference kept
 * HashParams / DepthCameraParams / RayCastParams in __constant__ memory,
 * Source/DepthSensing/CUDAConstant.cu:6-48, which made it one scene per device).
 *
 * Which reference entry point each function replaces is given beside it
 * (paths relative to /root/reference/FriedLiver/Source/).
 */
#ifndef BF_BF_H
#define BF_BF_H

#include <stddef.h>
#include <stdint.h>
#include "types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define BF_ABI_VERSION 4  /* 2: BFSolverOptions.pcgSpinLimitUs, BFCorrOptions.minPerPair; 3: BFReconStats.globalPcgLaunches /
                             globalPcgKernelMs, BFTsdfStats.batchHalves, BFRenderStats.waveSamples / waveSamplesMax / longWaves, BFAppTiming;
                             4: configuration through the ABI only (BFSceneOptions.applyXcdRun / applyRounds / testFlags /
                             splatRowCap, BFReconOptions.bundlingPriority, bf_set_host_threads; no environment switches),
                             BFSceneCapacity + bf_scene_capacity / bf_recon_scene_capacity (scene errors fail the loop),
                             bf_recon_set_render (visualizeFrame's render per frame) */

/* ---- runtime ------------------------------------------------------------- */
int bf_abi_version(void);
/* sizeof of a struct of types.h / bf.h by name (bindings check their layouts against it) */
int bf_abi_struct_size(const char* name, size_t* out);
const char* bf_last_error(void);
int bf_device_count(int* count);
int bf_set_device(int device);
int bf_device_synchronize(void);
/* threads of the host pool the loop uses for its per-submap loops over every frame, counting the calling thread
 * (default 4; results do not depend on it); takes effect before the pool's first use */
int bf_set_host_threads(int n);
/* device memory helpers (so hosts need no HIP headers) */
int bf_malloc(void** dptr, size_t bytes);
int bf_free(void* dptr);
/* Blocking copies: device-synchronize first, so they are ordered after all work queued on the
 * scene and solver streams (host plumbing, never inside a timed region). */
int bf_memcpy_h2d(void* dst, const void* src, size_t bytes);
int bf_memcpy_d2h(void* dst, const void* src, size_t bytes);
int bf_memcpy_d2d(void* dst, const void* src, size_t bytes);
int bf_memset(void* dptr, int value, size_t bytes);
/* events for timing a handle's stream (hipEvent pairs) */
typedef struct bf_timer bf_timer;
int bf_timer_create(bf_timer** out);
int bf_timer_destroy(bf_timer* t);

/* ---- TSDF scene: CUDASceneRepHashSDF (DepthSensing/CUDASceneRepHashSDF.h:29-423) ---- */
typedef struct bf_scene bf_scene;

typedef struct BFSceneOptions {
    uint32_t candidateCapacity; /* alloc candidates per integrate (0 = default 2^21) */
    uint32_t shardCount;        /* multi-GPU spatial ownership: number of shards (0/1 = off) */
    uint32_t shardIndex;        /* this handle's shard */
    float shardChunk;           /* ownership chunk edge in metres (0 = 1.0) */
    /* v4: the voxel pass's scheduling (environment switches up to v3); 0 = the measured defaults */
    uint32_t applyXcdRun;       /* work-list positions handed to one XCD per run, a power of two (0 = 64) */
    uint32_t applyRounds;       /* grid of the voxel pass in rounds of resident workgroups (0 = 4) */
    uint32_t testFlags;         /* test switches (0 in production): BF_SCENE_TEST_ALLOC_DIRECT */
    uint32_t splatRowCap;       /* test switch: capacity of the ray-interval splat's row lists (0 = 4 per heap block) */
} BFSceneOptions;
#define BF_SCENE_TEST_ALLOC_DIRECT 1u  /* every walking alloc tile also takes the walk's congested path */

/* ctor + reset (CUDASceneRepHashSDF.h:32-34, :147-155 -> resetCUDA, CUDASceneRepHashSDF.cu:67) */
int bf_scene_create(const BFHashParams* params, const BFSceneOptions* opts, bf_scene** out);
int bf_scene_destroy(bf_scene* s);
int bf_scene_reset(bf_scene* s);
/* integrate / deIntegrate (CUDASceneRepHashSDF.h:65-108 -> allocCUDA, compactifyHashAllInOneCUDA,
 * integrateDepthMapCUDA / deIntegrateDepthMapCUDA, CUDASceneRepHashSDF.cu:253,368,524,538).
 * T: camera->world row-major 4x4. depth: device float[W*H] metres (-inf = invalid).
 * color: device uchar4[W*H] RGBA, or NULL (then no voxel updates, as in the reference).
 * bitMask: reference chunk-streaming mask (device) or NULL. */
int bf_scene_integrate(bf_scene* s, const float T[16], const float* depth, const uint8_t* color,
                       const BFDepthCameraParams* cam, const uint32_t* bitMask);
int bf_scene_deintegrate(bf_scene* s, const float T[16], const float* depth, const uint8_t* color,
                         const BFDepthCameraParams* cam, const uint32_t* bitMask);
/* One re-integration fix (DepthSensing.cpp:890-895): bf_scene_deintegrate(Told) followed by
 * bf_scene_integrate(Tnew) of the same frame, fused into one voxel pass; the resulting scene is
 * identical to the two calls. */
int bf_scene_reintegrate(bf_scene* s, const float Told[16], const float Tnew[16], const float* depth, const uint8_t* color,
                         const BFDepthCameraParams* cam);
/* A frame's re-integration fixes (reintegrate(), DepthSensing.cpp:854-902, the loop body's
 * deIntegrate / integrate calls): n <= BF_MAX_VOXEL_OPS ops, each de-integrating (deintegrate != 0)
 * or integrating one frame at pose T (camera -> world), applied in order as ONE voxel pass. Voxel
 * values and the allocated block set equal those of the sequence of bf_scene_deintegrate /
 * bf_scene_integrate calls; the visible list afterwards is the last op's frustum list (what the
 * reference's garbageCollect after the loop walks). */
#define BF_MAX_VOXEL_OPS 24
typedef struct BFVoxelOp {
    float T[16];
    const float* depth;   /* device, W*H float */
    const uint8_t* color; /* device, W*H uchar4 */
    uint32_t deintegrate;
    uint32_t reserved;
} BFVoxelOp;
int bf_scene_apply_ops(bf_scene* s, const BFVoxelOp* ops, uint32_t n, const BFDepthCameraParams* cam);
/* garbageCollect (CUDASceneRepHashSDF.h:110-126 -> garbageCollectIdentifyCUDA,
 * resetHashBucketMutexCUDA, garbageCollectFreeCUDA, CUDASceneRepHashSDF.cu:113,633,671) */
int bf_scene_garbage_collect(bf_scene* s);
/* setLastRigidTransformAndCompactify (CUDASceneRepHashSDF.h:136-139); nVisible may be NULL
 * (otherwise this call synchronizes to read it back) */
int bf_scene_compactify(bf_scene* s, const float T[16], const BFDepthCameraParams* cam, uint32_t* nVisible);
/* getHeapFreeCount (CUDASceneRepHashSDF.h:168-172) — synchronizes */
int bf_scene_heap_free_count(bf_scene* s, uint32_t* count);
int bf_scene_num_visible(bf_scene* s, uint32_t* count);
/* error bits: 1 candidate buffer overflow, 2 heap exhausted, 4 dedup set congested */
int bf_scene_error_flags(bf_scene* s, uint32_t* flags);
/* capacity state (types.h BFSceneCapacity): the sticky error bits, the peak alloc candidates of one call against
 * candidateCapacity, heap free count and high water — synchronizes */
int bf_scene_capacity(bf_scene* s, BFSceneCapacity* out);
int bf_scene_get_stats(bf_scene* s, BFTsdfStats* out);
int bf_scene_reset_stats(bf_scene* s);
/* debugHash-style dump to HOST memory (CUDASceneRepHashSDF.h:179-314): any pointer may be NULL.
 * hash: BFHashEntry[4*numBuckets], heap: uint32[numSDFBlocks], voxels: BFVoxel[numSDFBlocks*512].
 * Entries carry the reference's ptr (heap block * 512), so a hash dump needs numSDFBlocks <= 2^22
 * (BF_ERR_CAPACITY otherwise); larger scenes dump with bf_scene_export_blocks / _block_voxels. */
int bf_scene_export(bf_scene* s, BFHashEntry* hash, uint32_t* heap, uint32_t* heapCounter, BFVoxel* voxels);
/* heap blocks [0, highWater) to HOST: int32 {x, y, z, allocated} per block (heap order); min(cap, n) written,
 * *n = highWater (the allocated prefix compactify streams) */
int bf_scene_export_blocks(bf_scene* s, int32_t* out4, uint32_t cap, uint32_t* n);
/* visible list of the last compactify to HOST: int32 {x,y,z,ptr} x n */
int bf_scene_export_visible(bf_scene* s, int32_t* out4, uint32_t cap, uint32_t* n);
/* voxels of heap blocks [first, first + count) to HOST: BFVoxel[count * 512] (block i's run is the
 * voxels at voxel index i * 512, VoxelUtilHashSDF.h:609); the dump of scenes above 2^22 blocks */
int bf_scene_export_block_voxels(bf_scene* s, uint32_t first, uint32_t count, BFVoxel* out);
/* CUDARayCastSDF::render (CUDARayCastSDF.cpp:38-72) preceded by setLastRigidTransformAndCompactify
 * (CUDASceneRepHashSDF.h:128-139): camera->world T, frustum camera params cam (render depth range),
 * ray-cast params rp (intrinsics, size, minDepth/maxDepth, rayIncrement, thresholds, useGradients;
 * the view matrices are derived from T). Device outputs of rp->width*rp->height: depth f32, depth4 /
 * normals / colors float4 (MINF where no surface); rayMin / rayMax (optional) receive the splatted
 * ray intervals (rayIntervalSplatCUDA + the D3D11 min/max passes). */
int bf_scene_raycast(bf_scene* s, const float T[16], const BFDepthCameraParams* cam, const BFRayCastParams* rp, float* depth,
                     float* depth4, float* normals, float* colors, float* rayMin, float* rayMax);
int bf_scene_synchronize(bf_scene* s);
/* CUDAMarchingCubesHashSDF::extractIsoSurface (CUDAMarchingCubesHashSDF.cpp:107-118 ->
 * resetMarchingCubesCUDA + extractIsoSurfaceCUDA, CUDAMarchingCubesSDF.cu:29-53) over every allocated
 * block (the s_streamingEnabled = 0 path of StopScanningAndExtractIsoSurfaceMC, DepthSensing.cpp:348-352).
 * tris: DEVICE BFMcTriangle[p->maxNumTriangles]; *numTriangles = triangles written (at most
 * maxNumTriangles, extra ones dropped as the reference's appendTriangle does); *totalTriangles (may be
 * NULL) = the count before that cap. Output order is fixed: heap block, voxel (z*64 + y*8 + x),
 * triTable order (the reference's atomic append order varies run to run). Synchronizes. */
int bf_scene_extract_mesh(bf_scene* s, const BFMarchingCubesParams* p, BFMcTriangle* tris, uint32_t* numTriangles,
                          uint32_t* totalTriangles);
int bf_scene_device_bytes(bf_scene* s, uint64_t* bytes);
/* time the next operations on the scene's stream */
int bf_scene_timer_start(bf_scene* s, bf_timer* t);
int bf_scene_timer_stop(bf_scene* s, bf_timer* t, float* ms); /* synchronizes */

/* ---- bundle adjustment: CUDASolverBundling (Solver/CUDASolverBundling.h/.cpp) ---------- */
typedef struct bf_solver bf_solver;

typedef struct BFSolverOptions {   /* zParametersBundlingDefault.txt defaults when 0 */
    float denseDistThresh;         /* s_denseDistThresh = 0.15 */
    float denseNormalThresh;       /* s_denseNormalThresh = 0.97 */
    float denseColorThresh;        /* s_denseColorThresh = 0.1 */
    float denseColorGradientMin;   /* s_denseColorGradientMin = 0.005 */
    float denseDepthMin;           /* s_denseDepthMin = 0.5 */
    float denseDepthMax;           /* s_denseDepthMax = 4.0 */
    uint32_t denseOverlapSubsample;/* s_denseOverlapCheckSubsampleFactor = 4 */
    float verifyOptDistThresh;     /* 0.02 (CUDASolverBundling.cpp:34) */
    int32_t normalEquations;       /* 0 auto: sparse-only solves assemble the normal equations per image
                                      pair (fp64 statistics, one exchange per GN iteration when sharded);
                                      1 matrix-free (the reference's applyJ/applyJT); 2 assembled */
    int32_t disableEarlyOut;       /* 0: the reference build (#define ENABLE_EARLY_OUT, SolverBundling.cu:7:
                                      a PCG step with |p.Ap| < 5e-7 is the last, and the GN loop stops when
                                      max|delta| < 0.005, :1088-1093, :1204-1210); 1: built without it, fixed
                                      nNonLin x nLin schedules */
    int32_t pcgLaunch;             /* 0 auto: a pair-mode GN step of 65..513 images runs its whole PCG loop in
                                      one persistent launch (when the grid fits co-resident); 1: one launch
                                      per PCG iteration. Bit-identical results either way */
    uint32_t pcgSpinLimitUs;       /* bound of every wait inside the persistent PCG launch, in microseconds
                                      (0: 2 s). A launch that times out is redone in stream order with the
                                      per-iteration arithmetic (result error bit BF_SOLVE_PCG_RECOVERED);
                                      a small value forces that path (tests) */
} BFSolverOptions;

/* ctor (CUDASolverBundling.cpp:24-136): capacity maxImages x maxCorr residuals */
int bf_solver_create(uint32_t maxImages, uint32_t maxCorr, const BFSolverOptions* opts, bf_solver** out);
int bf_solver_destroy(bf_solver* s);
/* CUDASolverBundling::solve (CUDASolverBundling.cpp:187-284) -> solveBundlingStub
 * (SolverBundling.cu:1137). Device pointers: corr EntryJ[nCorr] (may be invalidated in place by
 * the per-image cap), valid int[nImages], rot/trans float3[nImages] (in/out, se(3) [omega|t]),
 * cache BFCachedFrame[nImages] (device array of device pointers) or NULL. Host pointers: the
 * per-GN-iteration weights [nNonLin]. Enqueued asynchronously on the solver's stream; no host
 * round trip until bf_solver_result. */
int bf_solver_solve(bf_solver* s, BFEntryJ* corr, uint32_t nCorr, const int* valid, uint32_t nImages,
                    uint32_t nNonLin, uint32_t nLin, const float* wSparse, const float* wDenseDepth,
                    const float* wDenseColor, const BFCachedFrame* cache, uint32_t cacheW, uint32_t cacheH,
                    const float intrinsics[4], float* rot, float* trans, int rebuildJT, int findMaxResidual);
/* synchronizes; getMaxResidual inputs, iteration counts (CUDASolverBundling.cpp:429-476) */
int bf_solver_result(bf_solver* s, BFSolveResult* out);
/* getVarToCorrNumEntriesPerRow: device int[nImages] of the last table build */
int bf_solver_num_entries_per_row(bf_solver* s, const int** dptr);
int bf_solver_synchronize(bf_solver* s);
int bf_solver_timer_start(bf_solver* s, bf_timer* t);
int bf_solver_timer_stop(bf_solver* s, bf_timer* t, float* ms); /* synchronizes */
/* device time of the persistent PCG launches (one per GN step, dispatch-stamped events): enable != 0 starts
 * (or keeps) timing them, enable == 0 stops; *ms / *launches: totals since timing started (synchronizes) */
int bf_solver_pcg_time(bf_solver* s, int enable, double* ms, uint64_t* launches);
/* convertMatricesToPosesCU / convertPosesToMatricesCU (SBA.cu:75-119), on the solver's stream */
int bf_solver_matrices_to_poses(bf_solver* s, const float* T, uint32_t n, float* rot, float* trans, const int* valid);
int bf_solver_poses_to_matrices(bf_solver* s, const float* rot, const float* trans, uint32_t n, float* T, const int* valid);
/* SIFTImageManager::InvalidateImageToImageCU (SIFTImageManager.cu:692-719) */
int bf_solver_invalidate_image_pair(bf_solver* s, BFEntryJ* corr, uint32_t nCorr, uint32_t i, uint32_t j);
/* CheckForInvalidFrames[Simple]CU (SIFTImageManager.cu:725-793), using the last table build */
int bf_solver_check_invalid_frames(bf_solver* s, int* valid, uint32_t nImages, BFEntryJ* corr, uint32_t nCorr,
                                   int comprehensive);

/* Local-submap verification after a solve (SBA::align, SBA.cpp:106-109):
 * CUDASolverBundling::useVerification (Solver/CUDASolverBundling.cpp:454-476) — the dense check runs only
 * when >= percentThresh of the last solve's nCorr correspondences kept a max-norm residual above
 * verifyOptDistThresh (the solve must have run with findMaxResidual, which counts them) or when
 * `always` is set — then SIFTImageManager::VerifyTrajectoryCU (SiftGPU/SIFTImageManager.cu:1036-1159) over
 * every valid image pair i < j of the trajectory T (DEVICE float4x4[nImages], camera -> world) with the
 * cache frames (DEVICE BFCachedFrame[nImages]). Fields left 0 take the defaults of
 * zParametersBundlingDefault.txt:55-64 / Bundler.cpp:267. *valid (may be NULL; synchronizes) = 1 when the
 * submap is accepted; pairStats (DEVICE float[nImages^2 * 3] or NULL) receives {sum residual, sum
 * weight, #correspondences} per pair (i * nImages + j). The outcome is also in bf_solver_result. */
typedef struct BFVerifyOptions {
    float projCorrDistThresh;      /* s_projCorrDistThres = 0.15 */
    float projCorrNormalThresh;    /* s_projCorrNormalThres = 0.97 */
    float verifyOptErrThresh;      /* s_verifyOptErrThresh = 0.05 */
    float verifyOptCorrThresh;     /* s_verifyOptCorrThresh = 0.001 */
    float verifyOptPercentThresh;  /* m_verifyOptPercentThresh = 0.05 (CUDASolverBundling.cpp:36) */
    float sensorDepthMin, sensorDepthMax;  /* 0.1 / 3.0 (Bundler.cpp:267) */
    int32_t always;                /* 1: skip useVerification, check every pair */
} BFVerifyOptions;
int bf_solver_verify_trajectory(bf_solver* s, const float* T, const int* valid, uint32_t nImages, uint32_t nCorr,
                                const BFCachedFrame* cache, uint32_t cacheW, uint32_t cacheH, const float intrinsics[4],
                                const BFVerifyOptions* opts, float* pairStats, int* validOut);

/* ---- multi-GPU: RCCL communicator for the global normal equations ----------
 * One process per GPU. Rank 0 draws the id (bf_comm_unique_id), the host hands it to every rank,
 * every rank calls bf_comm_create (collective). A sharded solver builds the normal-equation blocks
 * of the image pairs p with p % nranks == rank and sums them over ranks with one RCCL all-reduce per
 * GN iteration; the PCG that follows runs replicated, so every rank ends with the same poses (bit-
 * identical to a single-GPU solve). */
typedef struct bf_comm bf_comm;
int bf_comm_unique_id(uint8_t id[128]);
int bf_comm_create(const uint8_t id[128], int nranks, int rank, bf_comm** out);
int bf_comm_destroy(bf_comm* c);
/* In-process loopback group (tests): out[0..nranks-1] are communicators of one group for ranks driven from
 * their own host threads in this process, sharing the current GPU. A collective is a one-workgroup kernel
 * enqueued on the caller's stream (as RCCL's are: asynchronous, stream-ordered, no host wait) that waits on
 * the device for every rank's contribution and sums in rank order; a rank that never arrives within
 * timeoutMs (0: 60 s) ends the wait and the next collective call fails. capacityBytes: the largest collective
 * (0: 16 MiB; the global solve's pair statistics are 224 B per image pair, 83 MB at config 4's 2 001 keyframes).
 * Lets the multi-rank loop run on one GPU with RCCL's ordering semantics; RCCL is not involved. */
int bf_comm_create_loopback(int nranks, int timeoutMs, size_t capacityBytes, bf_comm** out);
/* in-place sum over ranks of n doubles (device pointer); synchronizes (tests) */
int bf_comm_allreduce_sum_f64(bf_comm* c, double* d, size_t n);
/* shard the solver's pairs: count shards, this is shard index; comm (count ranks) or NULL (no
 * exchange: each shard keeps only its own blocks, for tests of the partition) */
int bf_solver_set_shard(bf_solver* s, uint32_t count, uint32_t index, bf_comm* comm);
/* assembled normal equations of the last GN iteration of the last solve: per image pair (a < b),
 * 28 doubles {M = sum P_b P_a^T (row-major 9), s_a (3), s_b (3), n, Q_a (xx xy xz yy yz zz), Q_b};
 * copies min(cap, total) pairs to host stats / pairAB (2 ints each), *total = pair count */
int bf_solver_export_pairs(bf_solver* s, double* stats, int32_t* pairAB, uint32_t cap, uint32_t* total);

/* ---- synthetic RGB-D stream (seeded analytic room) ------------ */
typedef struct BFSynthScene {
    uint32_t seed;
    uint32_t numPrimitives;   /* boxes + spheres inside the room (<= 64) */
    float roomMin[3], roomMax[3];
    float prims[64][8];       /* {type(0 box,1 sphere), cx, cy, cz, ex|r, ey, ez, hue} */
} BFSynthScene;

int bf_synth_scene_default(uint32_t seed, BFSynthScene* out);
/* camera->world pose of frame f of the default Lissajous trajectory */
int bf_synth_pose(uint32_t frame, float T[16]);
/* render one frame on the GPU into device buffers (depth float[W*H], color uchar4[W*H]).
 * noiseSeed != 0 adds the depth noise model and 1 mm quantisation. */
int bf_synth_render(const BFSynthScene* scene, const float T[16], const BFDepthCameraParams* cam,
                    uint32_t noiseSeed, uint32_t frame, float* d_depth, uint8_t* d_color);
/* device: a rendered frame as the sensor delivers it (the .sens convention, SensorDataReader.cpp:104-107):
 * depth ushort = rint(d * depthShift), 0 where d is invalid; colour RGBX bytes (alpha kept) */
int bf_synth_to_raw(const float* d_depth, const uint8_t* d_color, uint32_t numPixels, float depthShift,
                    uint16_t* d_depthU16, uint8_t* d_rgbx);
/* same arithmetic on the host (tests) into host buffers */
int bf_synth_render_host(const BFSynthScene* scene, const float T[16], const BFDepthCameraParams* cam,
                         uint32_t noiseSeed, uint32_t frame, float* depth, uint8_t* color);
/* Stand-in for the SIFT front end: for every pair of the K camera->world poses (HOST float[16*K])
 * whose views share >= minCovis of sampled surface points, up to maxPerPair EntryJ correspondences
 * (camera-space points in each frame, SIFTImageManager.cu:610-686 convention) with N(0, noise^2)
 * jitter and an outlierFrac share of 0.1-0.3 m outliers. Writes HOST EntryJ[cap]; *n = count. */
int bf_synth_correspondences(const BFSynthScene* scene, const float* poses, uint32_t K, const BFDepthCameraParams* cam,
                             uint32_t maxPerPair, float minCovis, float noise, float outlierFrac, uint32_t seed,
                             BFEntryJ* out, uint32_t cap, uint32_t* n);
/* Dense-term cache frame of one view (CUDACache::storeFrame, CUDACache.cpp:45-86, from a noiseless
 * render): HOST buffers depth[W*H], campos[4*W*H], normals[4*W*H], normalsU8[4*W*H],
 * intensity[W*H], intensityDeriv[2*W*H]; cam is the cache resolution camera. */
int bf_synth_cache_frame(const BFSynthScene* scene, const float T[16], const BFDepthCameraParams* cam, float* depth,
                         float* campos, float* normals, uint8_t* normalsU8, float* intensity, float* intensityDeriv);

/* ---- reconstruction loop: integrate + re-integration queue + local/global BA ------------
 * The frame loop of DepthSensing.cpp (integrate :1003-1056, reintegrate :854-902) driven by
 * TrajectoryManager (TrajectoryManager.cpp:8-200) and the OnlineBundler local->global
 * hierarchy (OnlineBundler.cpp:242-416). Frames are borrowed device pointers that must stay
 * resident (the CUDAImageManager frame store); correspondences are EntryJ inputs. */

typedef struct BFReconOptions {
    uint32_t maxFrames;          /* frame-store / trajectory capacity */
    uint32_t submapSize;         /* s_submapSize = 10 */
    uint32_t maxFrameFixes;      /* s_maxFrameFixes = 10 */
    uint32_t topNActive;         /* s_topNActive = 30 */
    float minPoseDistSqrt;       /* s_minPoseDistSqrt = 0 */
    uint32_t localNonLin, localLin;    /* s_numLocalNonLinIterations 2 / s_numLocalLinIterations 100 */
    uint32_t globalNonLin, globalLin;  /* s_numGlobalNonLinIterations 3 / s_numGlobalLinIterations 150 */
    uint32_t maxKeyframes;       /* global solver images */
    uint32_t maxLocalCorr;       /* per submap */
    uint32_t maxGlobalCorr;
    float maxResidualThresh;     /* s_optMaxResThresh = 0.08 */
    int32_t useLocalDense;       /* SBA::m_bUseLocalDense = true */
    uint32_t cacheWidth, cacheHeight;  /* 80 x 60 */
    float cacheIntrinsics[4];    /* fx fy mx my of the cache resolution */
    int32_t enableTiming;        /* record k_integrate / solve device times (bench) */
    int32_t recordOps;           /* keep a log of every scene call (parity replay in tests) */
    int32_t asyncBundling;       /* 1: solves run on their own stream and their poses are picked up
                                    by the frame loop when ready (the reference's bundling thread);
                                    0: the loop waits for each submap's solves (deterministic);
                                    2: as 1, with the solves issued from a separate host thread */
    BFSolverOptions solver;
    int32_t disableLocalVerify;  /* 0: s_useLocalVerify = true (zParametersBundlingDefault.txt:62): after each local
                                    solve useVerification + VerifyTrajectoryCU; a failing submap is invalidated
                                    (OnlineBundler.cpp:145-159, 255-261, 351-360, 399-405) */
    BFVerifyOptions verify;      /* its thresholds (0 = defaults) */
    uint32_t resultLag;          /* asyncBundling 1/2: 0 = a submap's poses are applied by the first frame that
                                    finds its solves done (timing-dependent, like the reference's threads);
                                    L > 0 = they are applied exactly L frames after the submap was issued
                                    (waiting for them if needed), so the run's op sequence is repeatable;
                                    L <= 8 * submapSize (the result ring), else BF_ERR_ARG */
    int32_t bundlingPriority;    /* v4. queue priority of the bundling streams: 0 normal, as the scene stream (default:
                                    the voxel pass runs in resident rounds, so a bundling launch finds slots within a
                                    round); 1 the highest; 2 keyed on the solve being issued (highest up to 1 537
                                    keyframes or when sharded, normal above: the round-4 policy) */
} BFReconOptions;

typedef struct BFReconStats {
    uint64_t frames;             /* processFrame calls */
    uint64_t integrations;       /* scene integrate calls (new frames + fixes) */
    uint64_t deintegrations;
    uint64_t fixOps;             /* re-integration queue ops (de-, re-, integrate) */
    uint64_t localSolves, globalSolves;
    uint64_t globalGnIterations, globalPcgIterations;
    uint64_t localGnIterations, localPcgIterations;
    uint64_t removedPairs;       /* max-residual removals */
    uint64_t integrateLaunches;  /* timed k_integrate launches */
    double integrateKernelMs;    /* summed device time of those launches */
    double localSolveMs, globalSolveMs;  /* summed device time of the solves */
    uint64_t reintegrateLaunches;  /* timed k_reintegrate launches (fused de-/re-integration) */
    double reintegrateKernelMs;
    uint64_t localVerifications; /* local solves whose dense verification ran (useVerification) */
    uint64_t invalidLocals;      /* local submaps invalidated by it */
    uint64_t endSolves;          /* end-of-sequence global solves (bf_recon_end_solve) */
    uint64_t pcgRecoveries;      /* solves whose persistent PCG timed out and was redone (BF_SOLVE_PCG_RECOVERED);
                                    a solve with a BF_SOLVE_ERR_FATAL bit fails the call with BF_ERR_INTERNAL */
    double hostMs;               /* host wall time inside bf_recon_process_frame (enqueueing + waits) */
    double hostWaitMs;           /* ... of it blocked on bundling results (resultLag, a full ring) */
    uint64_t globalPcgLaunches;  /* timed persistent PCG launches of the global solves (one per GN step) */
    double globalPcgKernelMs;    /* their summed device time (dispatch-stamped events) */
    uint64_t renders;            /* v4: per-frame renders (bf_recon_set_render) */
} BFReconStats;

typedef struct bf_recon bf_recon;
int bf_recon_create(const BFHashParams* params, const BFSceneOptions* sceneOpts, const BFDepthCameraParams* cam,
                    const BFReconOptions* opts, bf_recon** out);
int bf_recon_destroy(bf_recon* r);
/* frame store entry f: device depth / colour, HOST BFCachedFrame of device pointers (or NULL),
 * and the front end's frame-to-frame estimate Tinc (camera f expressed in camera f-1; the
 * stand-in for computeSiftTransformCU, OnlineBundler.cu:6-71; ignored for f = 0) */
int bf_recon_set_frame(bf_recon* r, uint32_t f, const float* depth, const uint8_t* color,
                       const BFCachedFrame* cache, const float Tinc[16]);
int bf_recon_set_local_correspondences(bf_recon* r, uint32_t submap, BFEntryJ* corr, uint32_t n);
/* global list ordered by max(i,j); prefix[k] (HOST) = number of entries with max(i,j) <= k */
int bf_recon_set_global_correspondences(bf_recon* r, BFEntryJ* corr, uint32_t n, const uint32_t* prefix,
                                        uint32_t numKeyframes);
int bf_recon_set_initial_pose(bf_recon* r, const float T0[16]);
int bf_recon_process_frame(bf_recon* r, uint32_t f);
int bf_recon_finish(bf_recon* r);
/* One end-of-sequence global solve (OnlineBundler::processInput past the last frame, OnlineBundler.cpp:171-197,
 * then optimizeGlobal with isSequenceDone, :373-398): all keyframes, every global correspondence, max-residual
 * removal; the reference's bundling thread runs s_numSolveFramesBeforeExit (30) of them and, with
 * USE_GLOBAL_DENSE_AT_END (GlobalBundlingState.h:9), the last with dense depth weight 15 (:177-189) — pass
 * denseDepthWeight 15 for that one (0: sparse only). The dense term reads each keyframe's cache frame (the
 * submap's first frame, Bundler::fuseToGlobal's copy). Waits for the solve; the new poses go to the
 * trajectory (the queue picks them up). out / ms (device time) may be NULL. */
int bf_recon_end_solve(bf_recon* r, float denseDepthWeight, BFSolveResult* out, float* ms);
/* with recordOps: submap s's local trajectory (HOST float[16 * (submapSize + 1)]) and the global keyframe poses
 * and valid flags after its global solve (HOST float[16 * maxKeyframes], int[maxKeyframes]); *numLocal /
 * *numKeyframes = entries written, *localValid = its verification outcome. Any output may be NULL. */
int bf_recon_submap_poses(bf_recon* r, uint32_t s, float* local, float* global, int32_t* valid, uint32_t* numLocal,
                          uint32_t* numKeyframes, int32_t* localValid);
/* a loop iteration without a new frame (the reference keeps calling reintegrate() from its render
 * loop after scanning ends): pick up results, run up to maxFrameFixes queue ops, GC */
int bf_recon_reintegrate(bf_recon* r);
int bf_recon_synchronize(bf_recon* r);
int bf_recon_stats(bf_recon* r, BFReconStats* out);
int bf_recon_scene_stats(bf_recon* r, BFTsdfStats* out);
int bf_recon_reset_stats(bf_recon* r);  /* zero loop + scene counters and the device clocks */
int bf_recon_heap_free_count(bf_recon* r, uint32_t* count);
/* bf_scene_capacity of the loop's scene (waits for the scene stream). The loop checks the scene's error bits
 * itself: bf_recon_process_frame / _reintegrate fail with BF_ERR_CAPACITY once a frame's batch set one (seen
 * one or two frames later: the bits reach the host through pinned memory written by the frame's GC kernel, no
 * synchronization), and bf_recon_synchronize / _finish / _end_sequence check them exactly. */
int bf_recon_scene_capacity(bf_recon* r, BFSceneCapacity* out);
/* integrated camera->world transform per frame (HOST float[16*n], -inf rows when not integrated) */
int bf_recon_trajectory(bf_recon* r, float* T, uint32_t n);
/* visualizeFrame's render (DepthSensing.cpp:790-793): bf_scene_raycast on the loop's scene with its
 * depth camera; device outputs as bf_scene_raycast */
int bf_recon_raycast(bf_recon* r, const float T[16], const BFRayCastParams* rp, float* depth, float* depth4, float* normals,
                     float* colors);
/* Test hook: capture submap `submap`'s in-loop global solve (arm before that submap is issued). The loop
 * copies, on the bundling stream, the solve's inputs as it sees them (the global EntryJ list prefix after
 * invalidate_local, the keyframes' se(3) poses, the valid flags) and its outcome before the max-residual
 * removal (poses, the list with the per-image cap's invalidations). bf_recon_captured_global_solve waits for
 * it and copies to HOST: corrIn / corrOut EntryJ[min(cap, *nCorr)], poseIn / poseOut float[6 * k] as
 * [rot 3k | trans 3k] with k = min(capImages, *nImages), valid int32[k]; any output may be NULL. */
int bf_recon_capture_global_solve(bf_recon* r, uint32_t submap);
int bf_recon_captured_global_solve(bf_recon* r, BFEntryJ* corrIn, BFEntryJ* corrOut, uint32_t cap, uint32_t* nCorr,
                                   float* poseIn, float* poseOut, int32_t* valid, uint32_t capImages, uint32_t* nImages);
/* visualizeFrame every frame (DepthSensing.cpp:766-850 -> :790-793): with rp set, each frame's re-integration
 * batch (which integrates the previous frame) is followed on the scene stream by setLastRigidTransformAndCompactify
 * + CUDARayCastSDF::render at the pose of the frame that batch integrated (the reference renders each frame right
 * after integrating it), with the loop's depth camera, into loop-owned device images of rp->width x rp->height;
 * rp = NULL stops. The render costs the frame loop what it costs the reference's (BFReconStats.renders counts
 * them). bf_recon_render_output gives the images of the last render (device pointers; read them after
 * bf_recon_synchronize): depth f32, depth4 / normals / colors float4, as bf_scene_raycast writes them. */
int bf_recon_set_render(bf_recon* r, const BFRayCastParams* rp);
int bf_recon_render_output(bf_recon* r, const float** depth, const float** depth4, const float** normals,
                           const float** colors);
/* StopScanningAndExtractIsoSurfaceMC (DepthSensing.cpp:335-365) on the loop's scene: waits for the
 * scene stream, then bf_scene_extract_mesh (tris: DEVICE BFMcTriangle[p->maxNumTriangles]) */
int bf_recon_extract_mesh(bf_recon* r, const BFMarchingCubesParams* p, BFMcTriangle* tris, uint32_t* numTriangles,
                          uint32_t* totalTriangles);
/* summed device time / count of the renderKernel launches since the first call (enables the clock) */
int bf_recon_render_time(bf_recon* r, double* ms, uint64_t* launches);
/* the ray caster's device counters, summed over every render of the loop's scene (raycast
 * bytes = 96 B per trilinear sample (8 voxels x 12 B) + 52 B of output per pixel) */
int bf_recon_render_stats(bf_recon* r, BFRenderStats* out);
/* bf_scene_export_blocks on the loop's scene */
int bf_recon_export_blocks(bf_recon* r, int32_t* out4, uint32_t cap, uint32_t* n);
/* debugHash-style dump of the loop's scene (same layout as bf_scene_export) */
int bf_recon_export(bf_recon* r, BFHashEntry* hash, uint32_t* heap, uint32_t* heapCounter, BFVoxel* voxels);
/* with recordOps: the scene calls issued so far, in order (kind 1 de-integrate with oldT,
 * 2 integrate with newT, 4 garbage collect); copies min(cap, total) entries, *n = total */
int bf_recon_op_log(bf_recon* r, BFFixOp* out, uint32_t cap, uint32_t* n);
/* multi-GPU: shard the global solve's normal equations over comm's ranks (one RCCL all-reduce per
 * GN iteration); call before the first frame. The all-reduce size comes from a host-side count of
 * the image pairs of each keyframe prefix of the global correspondences (computed when they are set). */
int bf_recon_set_comm(bf_recon* r, bf_comm* c);

/* Per-frame dense-term cache construction inside the loop (OnlineBundler::processInput ->
 * Bundler::storeCachedFrame -> CUDACache::storeFrame, OnlineBundler.cpp:199-204). With a cache attached,
 * bf_recon_process_frame(f) first stores frame f into it (slot f: the cache must hold exactly f frames at
 * that point) from the frame's source images — those of bf_recon_set_frame_source, else the frame store's
 * depth and colour at the integration size — and the local solves read those cache frames (ordered after
 * the cache's stream by an event). The cache is borrowed: it must outlive the loop. */
typedef struct bf_cache bf_cache;
int bf_recon_attach_cache(bf_recon* r, bf_cache* c);
int bf_recon_set_frame_source(bf_recon* r, uint32_t f, const float* depth, const uint8_t* color, uint32_t colorW,
                              uint32_t colorH);
/* Per-frame input preprocessing inside the loop (DepthSensing.cpp:986: CUDAImageManager::process, then the
 * frame's integration). With a preprocessor attached and raw sensor images registered for frame f,
 * bf_recon_process_frame(f) first runs bf_preproc_run(raw depth, raw RGBX -> frame f's frame-store depth and
 * colour of bf_recon_set_frame) on the preprocessor's stream; the scene stream and the attached cache are
 * ordered after it by events, and the cache takes the raw sensor depth and colour as its source (as
 * copyToBundling hands them to the bundler). The preprocessor is borrowed and must outlive the loop; its
 * output size must be the integration size. The raw images must stay valid as long as the frame store's
 * (a raw colour image of the integration size is integrated from directly, without a copy).
 * Look-ahead: bf_recon_process_frame(f) also queues frame f + 1's preprocessing when its raw images are
 * registered by then, so the raw images of frame f + 1 must hold their data before bf_recon_process_frame(f)
 * is called whenever bf_recon_set_frame_raw(f + 1) was called before it (register a frame's raw images only
 * once they are filled, or fill them all up front). */
typedef struct bf_preproc bf_preproc;
int bf_recon_attach_preproc(bf_recon* r, bf_preproc* p);
int bf_recon_set_frame_raw(bf_recon* r, uint32_t f, const uint16_t* depthU16, const uint8_t* rgbx);
/* Frame f's frame-store images (bf_recon_set_frame) are being written by work queued on `stream` (a
 * hipStream_t; the caller's own upload or preprocessing, CUDAImageManager::process outside the loop): the
 * loop's scene stream waits for that work on the device, in the batch that first reads the frame, instead
 * of the caller synchronising before bf_recon_process_frame. Call after queueing the producing work and
 * before bf_recon_process_frame(f). (The FriedLiver app does this for every frame on its input stream.) */
int bf_recon_frame_ready(bf_recon* r, uint32_t f, void* stream);

/* The end of the sequence (the render loop past the last input frame): OnlineBundler::processInput's
 * past-the-end branch (OnlineBundler.cpp:167-196), process() -> optimizeGlobal with isSequenceDone (:373-408)
 * and the exit check of OnD3D11FrameRender (DepthSensing/DepthSensing.cpp:1114-1126), in the single-threaded
 * order (the reference's bundling thread races the render loop; this is its RUN_MULTITHREADED-off schedule).
 * Past-the-end iteration p = 0, 1, ...:
 *   p = 0: the last (partial) submap's local solve + a global solve (prepareLocalSolve(curFrame, true)), or a
 *          global solve alone when the last submap was already solved;
 *   1 <= p < N: a global solve over every keyframe (sparse, max-residual removal: s_numOptPerResidualRemoval 1);
 *   p == N: the same with dense depth weight denseDepthWeight (15) when USE_GLOBAL_DENSE_AT_END applies
 *          (fewer than denseFrameLimit frames, every keyframe has a cache frame), else sparse;
 *   then reintegrate(); from p >= N on, the loop stops when generateUpdateLists leaves no active op.
 * N = numSolveFramesBeforeExit (s_numSolveFramesBeforeExit, 30). N < 0 is the reference's -1: a global solve
 * every iteration and no exit check (OnlineBundler.cpp:175, DepthSensing.cpp:1116), so only maxPastEndFrames
 * ends the phase. maxPastEndFrames caps the iterations (0 = 100000). Waits for every solve (deterministic). */
typedef struct BFEndSequenceOptions {
    int32_t numSolveFramesBeforeExit;  /* [30] */
    int32_t disableDenseAtEnd;         /* 1: no USE_GLOBAL_DENSE_AT_END switch */
    uint32_t denseFrameLimit;          /* [10000] m_lastFrameProcessed < 10000 (OnlineBundler.cpp:179); 0 = default */
    float denseDepthWeight;            /* [15] (0 = default) */
    uint32_t maxPastEndFrames;         /* [100000] */
} BFEndSequenceOptions;
typedef struct BFEndSequenceResult {
    uint32_t pastEndFrames;   /* render-loop iterations past the last frame */
    uint32_t globalSolves;    /* global solves issued past the end (incl. the last submap's) */
    uint32_t localSolved;     /* 1 if p = 0 solved a last partial submap */
    uint32_t denseSolve;      /* 1 if the USE_GLOBAL_DENSE_AT_END solve ran with the dense term */
    uint32_t queueDrained;    /* 1 if the loop stopped with no re-integration op left (0: hit the cap) */
    float denseSolveMs;       /* device time of that solve */
    BFSolveResult last;       /* the last global solve */
} BFEndSequenceResult;
int bf_recon_end_sequence(bf_recon* r, const BFEndSequenceOptions* o, BFEndSequenceResult* out);

/* TrajectoryManager::getOptimizedTransforms (TrajectoryManager.h:50-68): min(#added, #optimized) frames,
 * -inf for Invalid frames; the trajectory StopScanningAndExit writes (DepthSensing.cpp:921-934). HOST
 * T[16 * cap]; *n = frame count (min(cap, n) written). */
int bf_recon_optimized_trajectory(bf_recon* r, float* T, uint32_t cap, uint32_t* n);

/* With recordOps: every TrajectoryManager call the loop made, in order, so a test can drive a second
 * TrajectoryManager through the identical call sequence (the queue checked apart from BA float drift):
 *   kind 0 addFrame(Integrated, T, frame)            T = transforms[offset]
 *   kind 1 updateOptimizedTransform(count frames)    transforms[offset .. offset + count)
 *   kind 2 reintegrate()'s fix loop: count ops       fixes[offset .. offset + count) (kind 1/2/3 BFFixOp)
 *   kind 3 generateUpdateLists + getNumActiveOperations (the exit check), count = the result
 * Any output may be NULL with cap 0; *n* = totals. */
typedef struct BFQueueEvent {
    int32_t kind;
    uint32_t frame;
    uint32_t count;
    uint32_t offset;
} BFQueueEvent;
int bf_recon_queue_trace(bf_recon* r, BFQueueEvent* events, uint32_t capEvents, uint32_t* nEvents, float* transforms,
                         uint32_t capTransforms, uint32_t* nTransforms, BFFixOp* fixes, uint32_t capFixes, uint32_t* nFixes);

/* ---- re-integration queue alone (host; TrajectoryManager.h:6-118) ---------------------- */
typedef struct bf_traj bf_traj;

int bf_traj_create(uint32_t maxFrames, uint32_t topNActive, float minPoseDistSqrt, bf_traj** out);
int bf_traj_destroy(bf_traj* t);
/* type: 0 Integrated, 1 NotIntegrated_NoTransform (T ignored) */
int bf_traj_add_frame(bf_traj* t, int32_t type, const float T[16], uint32_t idx);
int bf_traj_update_optimized(bf_traj* t, const float* T, uint32_t numFrames);
/* reintegrate() list logic: up to maxFixes ops into ops[maxFixes]; *n = count */
int bf_traj_next_fixes(bf_traj* t, uint32_t maxFixes, BFFixOp* ops, uint32_t* n);
int bf_traj_frame_info(bf_traj* t, uint32_t idx, int32_t* type, float* dist);
/* PoseHelper::MatrixToPose (PoseHelper.h:332-362): out[6] = [translation part | omega] */
int bf_pose_helper_matrix_to_pose(const float T[16], float out[6]);

/* ---- input formats and preprocessing ------------------------------------ */
/* ---- dense-term frame cache: CUDACache (Source/CUDACache.h/.cpp/.cu) ------------------------
 * Per frame at width x height: depth, camera-space positions, float4 + uchar4 normals, intensity and
 * its Sobel derivatives (the CUDACachedFrame the dense term reads). Device storage is owned by the
 * cache; bf_cache_frame hands out a BFCachedFrame of device pointers for bf_solver_solve /
 * bf_recon_set_frame. Work is queued on the cache's own stream. */
int bf_cache_create(const BFCacheOptions* o, bf_cache** out);
int bf_cache_destroy(bf_cache* c);
/* storeFrame (CUDACache.cpp:45-94): device depth (inputWidth x inputHeight float metres, -inf invalid,
 * the raw SIFT depth Bundler::storeCachedFrame passes) and colour (device uchar4, colorW x colorH);
 * *index (may be NULL) = the frame slot written */
int bf_cache_store_frame(bf_cache* c, const float* depth, const uint8_t* color, uint32_t colorW, uint32_t colorH,
                         uint32_t* index);
/* copyCacheFrameFrom (CUDACache.h:24-39): the next slot of dst = frame of src (same size);
 * Bundler::fuseToGlobal's keyframe copy (Bundler.cpp:385-391) */
int bf_cache_copy_frame_from(bf_cache* dst, const bf_cache* src, uint32_t frame, uint32_t* index);
/* incrementCache (CUDACache.h:41-43): skip a slot (invalid keyframe) */
int bf_cache_increment(bf_cache* c);
int bf_cache_num_frames(bf_cache* c, uint32_t* n);
int bf_cache_frame(bf_cache* c, uint32_t index, BFCachedFrame* out);
/* m_intrinsics / m_intrinsicsInv: the input intrinsics scaled to the cache size (row-major) */
int bf_cache_intrinsics(bf_cache* c, float K[16], float Kinv[16]);
int bf_cache_synchronize(bf_cache* c);

/* ---- correspondences: EntryJ I/O and a producer from depth + poses ---------------------------
 * Bundler::saveSparseCorrsToFile (Bundler.cpp:396-409): mLib BinaryDataStreamFile of a uint64 count
 * followed by the raw 32-B EntryJ records (restated, unpinned). bf_corr_load reads min(cap, count)
 * records into HOST memory, *n = count in the file. */
int bf_corr_save(const char* path, const BFEntryJ* corr, uint64_t n);
int bf_corr_load(const char* path, BFEntryJ* corr, uint64_t cap, uint64_t* n);
/* The SiftGPU stand-in (feature matching is out of scope): for every image pair (i, curFrame),
 * i in [startFrame, curFrame), grid pixels of frame i carried by the poses into frame curFrame whose
 * depths agree become EntryJ {i, curFrame, pos_i, pos_j} with pos = intrinsicsInv * (d * (u, v, 1)), as
 * AddCurrToResidualsCU (SIFTImageManager.cu:610-686) appends them; at most maxPerPair per pair, in a
 * fixed order (pair, then a fixed permutation of the grid). depth: DEVICE array of device pointers
 * (float, width x height, -inf invalid); transforms / transformsInv: DEVICE float4x4[...] camera ->
 * world and its inverse. out: DEVICE EntryJ[cap]; *n = matches written (<= cap), *total (may be NULL)
 * = matches found. Runs on the null (legacy) stream, so it is ordered after the caller's work there and on
 * blocking streams; synchronizes. */
int bf_corr_from_depth(const float* const* depth, const float* transforms, const float* transformsInv, uint32_t curFrame,
                       uint32_t startFrame, const BFCorrOptions* o, BFEntryJ* out, uint32_t cap, uint32_t* n,
                       uint32_t* total);

/* ---- mesh output: CUDAMarchingCubesHashSDF::saveMesh (CUDAMarchingCubesHashSDF.cpp:48-105) ------
 * Triangle soup (HOST BFMcTriangle[n], e.g. from bf_scene_extract_mesh) -> indexed mesh as saveMesh
 * builds it: mergeCloseVertices(1e-5, approx) (vertices snapped to a 1e-5 grid, first occurrence kept,
 * faces remapped, degenerate faces dropped), removeDuplicateFaces (same vertex set), applyTransform.
 * The mLib MeshData / MeshIO these call are not vendored: restated, parity unpinned.
 * bf_mesh_merge: HOST outputs sized for the worst case (3n vertices, n faces); any may be NULL to
 * count only. transform: row-major 4x4 or NULL. */
int bf_mesh_merge(const BFMcTriangle* tris, uint32_t n, const float transform[16], float* vertices /* 3 per */,
                  float* colors /* 4 per, RGBA in [0,1] */, uint32_t* faces /* 3 per */, uint32_t* numVertices,
                  uint32_t* numFaces);
/* ... and MeshIOf::saveToFile of the result: binary little-endian PLY (float x y z, uchar red green
 * blue alpha, face list uchar/int). */
int bf_mesh_save_ply(const char* path, const BFMcTriangle* tris, uint32_t n, const float transform[16],
                     uint32_t* numVertices, uint32_t* numFaces);

/* .sens reader (mLib SensorData v4 as SensorDataReader.cpp:38-116 uses it; format restated in
 * SURVEY.md Appendix B). Frames are read on demand. Depth: raw or zlib ushort; colour: raw RGB, PNG or
 * baseline / extended-sequential Huffman JPEG (SOF0 / SOF1, 8-bit; bf_image_decode; progressive is refused); occi depth returns BF_ERR_ARG. */
typedef struct bf_sens bf_sens;
int bf_sens_open(const char* path, bf_sens** out);
int bf_sens_close(bf_sens* s);
int bf_sens_info(const bf_sens* s, BFSensInfo* out);
int bf_sens_frame_pose(const bf_sens* s, uint64_t frame, float camToWorld[16]);
int bf_sens_frame_timestamps(const bf_sens* s, uint64_t frame, uint64_t* tsColor, uint64_t* tsDepth);
int bf_sens_read_depth_u16(bf_sens* s, uint64_t frame, uint16_t* out);      /* host, depthW*depthH */
/* SensorDataReader::processDepth (:104-107): d / depthShift, 0 -> -inf */
int bf_sens_read_depth(bf_sens* s, uint64_t frame, float* out);             /* host, depthW*depthH */
int bf_sens_read_color(bf_sens* s, uint64_t frame, uint8_t* rgbx);           /* host, colorW*colorH*4, X = 255 */
/* writer (SensorData::saveToFile layout; numFrames patched on close): bf_sens_writer_add_frame encodes raw RGB
 * colour and raw or zlib depth; any compression with pre-compressed frames */
typedef struct bf_sens_writer bf_sens_writer;
int bf_sens_writer_create(const char* path, const BFSensInfo* info, bf_sens_writer** out);
int bf_sens_writer_add_frame(bf_sens_writer* w, const float camToWorld[16], uint64_t tsColor, uint64_t tsDepth,
                             const uint16_t* depth, const uint8_t* rgbx);
/* a frame whose colour / depth streams are already compressed as the header says (JPEG / PNG colour, zlib
 * depth): written as given (SensorData::saveToFile keeps the compressed streams) */
int bf_sens_writer_add_compressed_frame(bf_sens_writer* w, const float camToWorld[16], uint64_t tsColor, uint64_t tsDepth,
                                        const uint8_t* color, uint64_t colorBytes, const uint8_t* depth, uint64_t depthBytes);
int bf_sens_writer_close(bf_sens_writer* w);
/* SensorDataReader::saveToFile (SensorDataReader.cpp:153-166) as StopScanningAndExit uses it: the input .sens
 * with frame i's camToWorld = T[i] (HOST float[16 n]) for i < n and -inf after, every other byte unchanged;
 * out == in rewrites the file in place (the reference overwrites its input). */
int bf_sens_save_trajectory(const char* in, const char* out, const float* T, uint64_t n);
/* The colour-stream decoders behind bf_sens_read_color (colorCompression 1 = PNG, 2 = JPEG; the
 * reference decodes through mLib, SensorDataReader.cpp:98-116): data[n] -> RGBX (X = 255). Call with
 * rgbx = NULL to get the size; otherwise rgbx holds cap bytes (>= 4 * width * height). */
int bf_image_decode(const uint8_t* data, uint64_t n, int compression, uint32_t* width, uint32_t* height,
                    uint8_t* rgbx, uint64_t cap);

/* zParameters*.txt (mLib ParameterFile behind GlobalAppState / GlobalBundlingState): later loads
 * override earlier keys. Getters return BF_ERR_ARG for a missing key (the reference warns and
 * default-constructs, GlobalAppState.h:129-131). */
typedef struct bf_params bf_params;
int bf_params_create(bf_params** out);
int bf_params_load(bf_params* p, const char* path);
int bf_params_destroy(bf_params* p);
int bf_params_has(const bf_params* p, const char* key, int* found);
int bf_params_get_string(const bf_params* p, const char* key, char* buf, size_t cap); /* quotes stripped */
int bf_params_get_floats(const bf_params* p, const char* key, float* out, uint32_t cap, uint32_t* count);
int bf_params_get_number(const bf_params* p, const char* key, double* out);
int bf_params_get_bool(const bf_params* p, const char* key, int* out);
/* CUDASceneRepHashSDF::parametersFromGlobalAppState (CUDASceneRepHashSDF.h:39-59) */
int bf_params_hash_params(const bf_params* p, BFHashParams* out);
/* CUDARayCastSDF::parametersFromGlobalAppState (CUDARayCastSDF.h:24-51) for integration intrinsics
 * fx, fy, mx, my at s_integrationWidth x s_integrationHeight */
int bf_params_raycast_params(const bf_params* p, float fx, float fy, float mx, float my, BFRayCastParams* out);
/* CUDAImageManager's preprocessing options from the bundling parameters */
int bf_params_preprocess_options(const bf_params* p, float depthShift, BFPreprocessOptions* out);

/* CUDAImageManager::process (CUDAImageManager.cpp:22-158): ushort depth -> metres, erodeDepthMap x2,
 * gaussFilterDepthMap, nearest resampling of depth and colour to the integration size. All image
 * pointers are device pointers; work is queued on the handle's stream. */
int bf_preproc_create(uint32_t depthW, uint32_t depthH, uint32_t colorW, uint32_t colorH, uint32_t integrationW,
                      uint32_t integrationH, const BFPreprocessOptions* opt, bf_preproc** out);
int bf_preproc_destroy(bf_preproc* p);
int bf_preproc_run(bf_preproc* p, const uint16_t* depthU16, const uint8_t* rgbx, float* depthOut, uint8_t* colorOut);
int bf_preproc_synchronize(bf_preproc* p);
int bf_preproc_stream(bf_preproc* p, void** stream);  /* the hipStream_t bf_preproc_run queues on */

/* ---- the FriedLiver application over the path: main() + the render loop --------
 * FriedLiver.cpp:184-320 reads two parameter files (argv[1] zParametersDefault.txt -> GlobalAppState,
 * argv[2] zParametersBundlingDefault.txt -> GlobalBundlingState; argv[3] overrides s_binaryDumpSensorFile,
 * :228-250), opens the .sens (SensorDataReader::createFirstConnected, SensorDataReader.cpp:38-79) and runs
 * OnD3D11FrameRender per input frame (DepthSensing.cpp:966-1129). Per frame here:
 *   CUDAImageManager::process (CUDAImageManager.cpp:22-158): read + decode the frame (prefetch threads),
 *     H2D, erode x2, bilateral filter, resample into the device-resident frame store;
 *   OnlineBundler::processInput (OnlineBundler.cpp:167-227): CUDACache::storeFrame from the sensor-size
 *     eroded depth + colour; the SiftGPU stand-in: bf_corr_from_depth EntryJ between the frames of each
 *     submap and between keyframes (matched with the .sens trajectory, s_minNumMatches filter), and the
 *     front end's frame-to-frame estimate (see bundlefusion_amd/csrc/frontend.h);
 *   the loop (bf_recon_process_frame): re-integration queue + integrate, local/global BA per submap.
 * At the end of the input: bf_recon_end_sequence (s_numSolveFramesBeforeExit), then StopScanningAndExit
 * (DepthSensing.cpp:904-953): the optimized trajectory into a .sens (SensorDataReader::saveToFile,
 * SensorDataReader.cpp:153-166), marching cubes into <sens stem>.ply, processed.txt. */
typedef struct bf_app bf_app;
typedef struct BFAppOptions {
    const char* sensFile;       /* argv[3]: overrides s_binaryDumpSensorFile (NULL: the parameter) */
    const char* outputDir;      /* directory of the exit outputs (NULL: the .sens file's, as the reference) */
    int32_t overwriteSens;      /* 1: the trajectory goes into the input .sens (the reference overwrites it);
                                   0: into <outputDir>/<stem>.optimized.sens */
    int32_t skipOutputs;        /* 1: no .sens / .ply / processed.txt */
    int32_t asyncBundling;      /* BFReconOptions.asyncBundling (the app default is 1) */
    int32_t recordOps;          /* BFReconOptions.recordOps (tests) */
    int32_t enableTiming;       /* BFReconOptions.enableTiming */
    uint32_t maxFrames;         /* read at most this many frames (0: all; CUDAImageManager also stops at
                                   s_maxNumImages * s_submapSize) */
    float frontEndDriftRad;     /* front-end error per frame (rotation sigma, rad) [0.000873 = 0.05 deg] */
    float frontEndDriftM;       /* (translation sigma, m) [0.002] */
    uint32_t frontEndSeed;      /* [1] */
    int32_t noFrontEndDrift;    /* 1: the .sens relative motion exactly */
    uint32_t corrStride;        /* EntryJ producer sampling grid, pixels [16] */
    float corrDepthThresh;      /* depth agreement, m [0.02] */
    uint32_t prefetchFrames;    /* decoded frames ahead [16] */
    uint32_t decodeThreads;     /* [8] */
    int32_t numSolveFramesBeforeExit; /* overrides s_numSolveFramesBeforeExit when != 0 (-2: run no past-end phase) */
    uint32_t shardCount;        /* multi-GPU (one app per GPU, every rank on the same .sens and parameters): the
                                   TSDF is split into shardCount chunk-ownership shards (BFSceneOptions) and
                                   this app owns shard shardIndex; 0 / 1: one GPU. Attach the ranks'
                                   communicator with bf_recon_set_comm(bf_app_recon(...)) before the first step:
                                   local solves then run round-robin by submap with a broadcast, the global
                                   solve's pair statistics are all-reduced. The reference's
                                   only multi-GPU mode is its fixed reconstruction / bundling device split
                                   (DualGPU.h:108-134) */
    uint32_t shardIndex;
    float shardChunk;           /* ownership chunk edge, m (0: 1 m) */
    uint32_t resultLag;         /* BFReconOptions.resultLag (0: poll) */
} BFAppOptions;
typedef struct BFAppInfo {      /* what the app derived from the parameters and the .sens header */
    BFHashParams hashParams;    /* (the 16-byte aligned members first) */
    BFDepthCameraParams integrationCamera; /* the depth intrinsics scaled to the integration size (CUDAImageManager.h:160-166) */
    uint32_t numFrames;         /* frames it will process */
    uint32_t sensorDepthWidth, sensorDepthHeight, sensorColorWidth, sensorColorHeight;
    BFPreprocessOptions preprocess;
    BFCacheOptions cache;
    BFCorrOptions corr;         /* EntryJ producer: sensor depth size and intrinsics */
    float cacheIntrinsics[4];
    uint32_t submapSize, maxKeyframes, maxLocalCorr, maxGlobalCorr;
    int32_t numSolveFramesBeforeExit;
    uint32_t reserved[2];       /* (size a multiple of 16) */
} BFAppInfo;
typedef struct BFAppResult {
    uint32_t frames;            /* input frames processed */
    double loopSeconds;         /* wall time of the frame loop (input decode overlapped) */
    double endSeconds;          /* wall time of the end-of-sequence phase */
    BFEndSequenceResult end;
    uint32_t heapFreeCount;     /* getHeapFreeCount at exit */
    uint32_t numTransforms, numValidTransforms;  /* of the optimized trajectory (PoseHelper::countNumValidTransforms) */
    int32_t valid;              /* processed.txt's verdict: heap free >= 800 and >= half the transforms valid */
    uint32_t meshTriangles, meshVertices, meshFaces;
} BFAppResult;
/* where the app's frame loop spends its host time (bf_app_timing; cumulative over the steps so far) */
typedef struct BFAppTiming {
    uint32_t frames;            /* steps that processed a frame */
    uint32_t decodeThreads;     /* decode workers */
    double stepSeconds;         /* wall time inside bf_app_step */
    double decodeWaitSeconds;   /* ... blocked waiting for the decode workers */
    double uploadSeconds;       /* ... issuing the H2D copies + preprocessing and waiting for the copies */
    double corrSeconds;         /* ... producing EntryJ (the SiftGPU stand-in) at submap boundaries */
    double loopSeconds;         /* ... in the loop's processFrame (re-integration, integrate, solves) */
    double decodeSeconds;       /* decode work summed over the workers (read + zlib + JPEG/PNG) */
    double uploadBytes;         /* bytes copied host -> device for the input frames */
} BFAppTiming;
int bf_app_create(const char* appParams, const char* bundlingParams, const BFAppOptions* o, bf_app** out);
int bf_app_destroy(bf_app* a);
/* Host only (no device): the parameters bf_app_create derives from the two zParameters files and the .sens
 * header (FriedLiver.cpp:228-250, GlobalAppState / GlobalBundlingState), and the loop options it hands the
 * loop; the same checks and errors as bf_app_create's parameter stage. loop may be NULL. */
int bf_app_resolve(const char* appParams, const char* bundlingParams, const BFAppOptions* o, BFAppInfo* info,
                   BFReconOptions* loop);
int bf_app_info(const bf_app* a, BFAppInfo* out);
/* one input frame through the loop; *gotFrame = 0 once the input has ended (nothing done) */
int bf_app_step(bf_app* a, int* gotFrame);
/* end of sequence + StopScanningAndExit outputs (after the last step) */
int bf_app_finish(bf_app* a, BFAppResult* out);
/* FriedLiver main: every frame, then finish */
int bf_app_run(bf_app* a, BFAppResult* out);
/* the app's loop (borrowed: do not destroy) for the bf_recon_* queries (op log, submap poses, trajectory) */
int bf_app_recon(bf_app* a, bf_recon** out);
int bf_app_timing(const bf_app* a, BFAppTiming* out);
/* The stand-in front end's frame-to-frame estimate (computeSiftTransformCU's role, OnlineBundler.cu:6-71;
 * bundlefusion_amd/csrc/frontend.h): inv(prev) * cur * a seeded error step (rotation sigma driftRad, translation
 * sigma driftM; both 0: the exact relative motion), identity when a pose is not finite. Host only. */
int bf_front_end_tinc(const float prev[16], const float cur[16], uint32_t frame, uint32_t seed, float driftRad, float driftM,
                      float Tinc[16]);
/* inputs the app handed the loop for frame f (tests): Tinc (HOST float[16]) */
int bf_app_front_end_pose(const bf_app* a, uint32_t f, float Tinc[16]);

#ifdef __cplusplus
}
#endif
#endif
