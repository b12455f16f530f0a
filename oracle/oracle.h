/*
 * oracle/oracle.h — TEST INFRASTRUCTURE: the CPU restatement ("bf_cpu") of the
 * reference's TSDF / raycast / bundle-adjustment arithmetic, used as the parity
 * checker and as bench.py's cpu_baseline leg. Nothing in the product
 * (bundlefusion_amd/) links, loads or calls this library.
 *
 * Parity status: the reference cannot be compiled or run here (SURVEY.md §8(c):
 * VS2013/CUDA 7/D3D11/mLib, no nvcc) and ships no tests, fixtures or golden
 * vectors. The oracle is therefore pinned only by analytic
 * known-answer tests written from the cited reference lines (tests/test_oracle_*.py)
 * and by committed fixtures it generated itself — "parity unpinned" against a
 * running reference, as DESIGN.md states.
 */
#ifndef BF_ORACLE_H
#define BF_ORACLE_H

#include "../include/bf/types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- TSDF scene (CUDASceneRepHashSDF semantics, serial schedule) ---------- */
typedef struct ORScene ORScene;
ORScene* or_scene_create(const BFHashParams* params);
void or_scene_destroy(ORScene* s);
void or_scene_reset(ORScene* s);
/* multi-GPU TSDF shard: alloc keeps only the blocks whose chunk (edge `chunk` m) hashes onto `index` of `count` */
void or_scene_set_shard(ORScene* s, uint32_t count, uint32_t index, float chunk);
/* integrate (deintegrate=0) / de-integrate (deintegrate=1) one frame with camera->world T.
 * depth: float[W*H] metres (-inf invalid); color: uchar4[W*H] or NULL. */
void or_scene_integrate(ORScene* s, const float T[16], const float* depth, const uint8_t* color,
                        const BFDepthCameraParams* cam, int deintegrate, const uint32_t* bitMask);
void or_scene_garbage_collect(ORScene* s);
uint32_t or_scene_compactify(ORScene* s, const float T[16], const BFDepthCameraParams* cam);
uint32_t or_scene_heap_free_count(const ORScene* s);
uint32_t or_scene_num_occupied(const ORScene* s);
/* full dump (debugHash): hash[E], heap[B], voxels[B*512] */
void or_scene_export(const ORScene* s, BFHashEntry* hash, uint32_t* heap, uint32_t* heapCounter,
                     BFVoxel* voxels);
void or_scene_import(ORScene* o, const BFHashEntry* hash, const uint32_t* heap, uint32_t heapCounter, const BFVoxel* voxels);
/* occupied (visible) list of the last compactify: entries[numOccupied] */
void or_scene_export_visible(const ORScene* s, BFHashEntry* out);
void or_scene_get_stats(const ORScene* s, BFTsdfStats* out);

/* Dense-grid variant of config 1 (one frame -> dense n^3 TSDF, no hash). Restates the
 * per-voxel arithmetic of integrateDepthMapKernel over a dense volume. */
void or_dense_integrate(const float T[16], const float* depth, const uint8_t* color,
                        const BFDepthCameraParams* cam, const BFHashParams* params,
                        const int origin[3], int n, BFVoxel* grid);

/* ---- raycast (CUDARayCastSDF::render semantics) ----------------------------- */
void or_raycast(const ORScene* s, const BFRayCastParams* rp, const BFDepthCameraParams* cam,
                const float T[16], float* depth, float* depth4, float* normals, float* colors,
                float* rayMin, float* rayMax);
/* CUDAMarchingCubesHashSDF::extractIsoSurface restated: triangles of every allocated block in heap
 * order, voxel order, triTable order; first cap written, *total before the cap */
void or_mc_tables(uint16_t* edges, uint8_t* ntri, uint8_t* tri /* 256 x 15 */);
void or_extract_mesh(const ORScene* s, const BFMarchingCubesParams* p, BFMcTriangle* out, uint32_t cap, uint32_t* n,
                     uint32_t* total);

/* ---- Lie helpers (LieDerivUtil.h) ------------------------------------------ */
void or_pose_to_matrix(const float rot[3], const float trans[3], float M[16]);
void or_matrix_to_pose(const float M[16], float rot[3], float trans[3]);
void or_matrix_inverse(const float M[16], float out[16]);
/* EntryJ producer from depth + poses (see bundlefusion_amd/csrc/corr.hip): host arrays */
void or_corr_from_depth(const float* const* depth, const float* T, const float* Tinv, uint32_t cur, uint32_t start,
                        const BFCorrOptions* o, BFEntryJ* out, uint32_t cap, uint32_t* n, uint32_t* total);
/* CUDACache::storeFrame (CUDACache.cpp:45-94) staged at the input resolution as the reference runs it:
 * outputs at o->width x o->height (depth f32, campos / normals float4, normals uchar4, intensity f32,
 * derivatives float2); K / Kinv = the cache intrinsics (may be NULL) */
void or_cache_store_frame(const BFCacheOptions* o, const float* depth, const uint8_t* color, uint32_t cw, uint32_t ch,
                          float* depthOut, float* camposOut, float* normalsOut, uint8_t* nu8Out, float* intensityOut,
                          float* derivOut, float K[16], float Kinv[16]);

/* ---- bundle adjustment (CUDASolverBundling::solve semantics) --------------- */
typedef struct ORSolveParams {
    uint32_t numImages;
    uint32_t numCorr;
    uint32_t nNonLin;
    uint32_t nLin;
    uint32_t maxCorrPerImage;
    const float* weightsSparse;     /* [nNonLin] */
    const float* weightsDenseDepth; /* [nNonLin] */
    const float* weightsDenseColor; /* [nNonLin] */
    /* dense term inputs (may be NULL when weights are 0) */
    const BFCachedFrame* cache;     /* host pointers */
    uint32_t cacheW, cacheH;
    float intrinsics[4];            /* fx, fy, mx, my of the cache frames */
    float denseDistThresh, denseNormalThresh, denseColorThresh, denseColorGradientMin;
    float denseDepthMin, denseDepthMax;
    uint32_t denseOverlapSubsample;
    uint32_t disableEarlyOut;       /* 1: built without ENABLE_EARLY_OUT (SolverBundling.cu:7) */
} ORSolveParams;

typedef struct ORSolveResult {
    uint32_t gnIterations;      /* GN iterations executed */
    uint32_t pcgIterations;     /* total PCG iterations executed */
    float maxResidual;          /* computeMaxResidual */
    int32_t maxResidualIndex;
    float finalEnergy;          /* EvalResidual with the last weightSparse */
} ORSolveResult;

/* corr: EntryJ[numCorr] (entries may be invalidated in place by the row cap);
 * validImages: int[numImages]; rot/trans: float3[numImages] in/out. */
void or_ba_solve(BFEntryJ* corr, const int* validImages, const ORSolveParams* p, float* rot,
                 float* trans, ORSolveResult* res);
void or_ba_dense_system(const int* validImages, const ORSolveParams* p, const float* rot, const float* trans,
                        float* jtjOut, float* jtrOut, double* energyOut, uint32_t* pairsOut);

/* CountHighResidualsDevice (SolverBundling.cu:657-687) at poses rot/trans with weight w: correspondences
 * whose evalAbsMaxResidualDevice (SolverBundlingEquationsLie.h:27-40) exceeds thresh */
uint32_t or_ba_count_high_residuals(const BFEntryJ* corr, uint32_t n, const float* rot, const float* trans, float w,
                                    float thresh);
/* VerifyTrajectoryCU (SiftGPU/SIFTImageManager.cu:1036-1159) with computeProjError's float-normal branch
 * (:418-487): T = camera->world float4x4[numImages] (host), cache = host frames; returns 1 (valid) / 0.
 * Sums in the order of the gfx950 kernel (thread t of 256 takes pixels t, t+256, ...; a tree per 64
 * threads; the 4 partials in order). pairStats (may be NULL): float[numImages^2 * 3]. */
typedef struct ORVerifyParams {
    uint32_t numImages, width, height;
    float intrinsics[4];
    float distThresh, normalThresh, errThresh, corrThresh, depthMin, depthMax;
} ORVerifyParams;
int or_verify_trajectory(const int* valid, const float* T, const BFCachedFrame* cache, const ORVerifyParams* p,
                         float* pairStats);

/* TrajectoryManager + reintegrate() list logic (traj.cpp) */
void or_pose_helper_matrix_to_pose(const float* T, float out[6]);
void* or_traj_create(unsigned maxFrames, unsigned topN, float minDist);
void or_traj_destroy(void* h);
void or_traj_add_frame(void* h, int type, const float* T, unsigned idx);
void or_traj_update_optimized(void* h, const float* T, unsigned numFrames);
unsigned or_traj_next_fixes(void* h, unsigned maxFixes, int* kinds, unsigned* frames, float* oldT, float* newT);
void or_traj_frame_info(void* h, unsigned idx, int* type, float* dist);

void or_traj_integrated(void* h, unsigned idx, float* T);
/* generateUpdateLists + getNumActiveOperations (the past-the-end exit check, DepthSensing.cpp:1116-1123) */
unsigned or_traj_generate_and_count(void* h);

/* ---- bundling side of the reconstruction loop (recon.cpp): OnlineBundler local -> global state
 * machine + TrajectoryManager, in the order of the product's synchronous mode ----------------- */
typedef struct ORReconParams {
    uint32_t maxFrames, submapSize, maxFrameFixes, topNActive;
    float minPoseDistSqrt;
    uint32_t localNonLin, localLin, globalNonLin, globalLin;
    uint32_t maxKeyframes;
    uint32_t maxCorrPerImageLocal, maxCorrPerImageGlobal;  /* clamp(maxCorr / maxImages, 1000, 4000) */
    float maxResidualThresh;
    int32_t useLocalDense;
    uint32_t cacheWidth, cacheHeight;
    float cacheIntrinsics[4];
    uint32_t disableEarlyOut;
    int32_t disableLocalVerify;
    float verifyOptDistThresh, verifyOptPercentThresh;
    float projCorrDistThresh, projCorrNormalThresh, verifyOptErrThresh, verifyOptCorrThresh;
} ORReconParams;
typedef struct ORReconStats {
    uint64_t localSolves, globalSolves, localPcgIterations, globalPcgIterations, removedPairs;
    uint64_t localVerifications, invalidLocals, endSolves;
} ORReconStats;
typedef struct ORRecon ORRecon;
ORRecon* or_recon_create(const ORReconParams* p, const float T0[16]);
void or_recon_destroy(ORRecon* r);
/* cache: HOST BFCachedFrame of host pointers (or NULL) */
void or_recon_set_frame(ORRecon* r, uint32_t f, const float Tinc[16], const BFCachedFrame* cache);
void or_recon_set_local_corr(ORRecon* r, uint32_t s, const BFEntryJ* corr, uint32_t n);
void or_recon_set_global_corr(ORRecon* r, const BFEntryJ* corr, uint32_t n, const uint32_t* prefix, uint32_t numKeyframes);
void or_recon_append_global_corr(ORRecon* r, const BFEntryJ* corr, uint32_t n);
void or_recon_process_frame(ORRecon* r, uint32_t f);
void or_recon_finish(ORRecon* r);
void or_recon_reintegrate(ORRecon* r);
void or_recon_end_solve(ORRecon* r, float denseDepthWeight);
void or_recon_end_sequence(ORRecon* r, int32_t numSolveFramesBeforeExit, int32_t disableDense, uint32_t denseFrameLimit,
                           float denseDepthWeight, uint32_t maxPastEndFrames, uint32_t* out5);
uint32_t or_recon_op_log(const ORRecon* r, BFFixOp* out, uint32_t cap);
int or_recon_submap_poses(const ORRecon* r, uint32_t s, float* local, float* global, int32_t* valid, uint32_t* numLocal,
                          uint32_t* numKeyframes, int32_t* localValid);
void or_recon_trajectory(const ORRecon* r, float* T, uint32_t n);
void or_recon_stats(const ORRecon* r, ORReconStats* out);

/* ---- input preprocessing (CUDAImageManager::process) ---------------------- */
void or_preprocess(const BFPreprocessOptions* o, const uint16_t* depthU16, uint32_t dw, uint32_t dh,
                   const uint8_t* rgbx, uint32_t cw, uint32_t ch, uint32_t iw, uint32_t ih, float* depthOut,
                   uint8_t* colorOut);
/* ... also returning the sensor-size raw (eroded) and filtered depth (CUDAImageManager::copyToBundling) */
void or_preprocess2(const BFPreprocessOptions* o, const uint16_t* depthU16, uint32_t dw, uint32_t dh, const uint8_t* rgbx,
                    uint32_t cw, uint32_t ch, uint32_t iw, uint32_t ih, float* depthOut, uint8_t* colorOut, float* rawOut,
                    float* filteredOut);

/* the app's front-end estimate (bundlefusion_amd/csrc/frontend.h), restated */
void or_front_end_tinc(const float* prev, const float* cur, uint32_t frame, uint32_t seed, float driftRad, float driftM,
                       float* out);

#ifdef __cplusplus
}
#endif
#endif
