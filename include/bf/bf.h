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

#define BF_ABI_VERSION 1

/* ---- runtime ------------------------------------------------------------- */
int bf_abi_version(void);
const char* bf_last_error(void);
int bf_device_count(int* count);
int bf_set_device(int device);
int bf_device_synchronize(void);
/* device memory helpers (so hosts need no HIP headers) */
int bf_malloc(void** dptr, size_t bytes);
int bf_free(void* dptr);
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
} BFSceneOptions;

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
int bf_scene_get_stats(bf_scene* s, BFTsdfStats* out);
int bf_scene_reset_stats(bf_scene* s);
/* debugHash-style dump to HOST memory (CUDASceneRepHashSDF.h:179-314): any pointer may be NULL.
 * hash: BFHashEntry[4*numBuckets], heap: uint32[numSDFBlocks], voxels: BFVoxel[numSDFBlocks*512] */
int bf_scene_export(bf_scene* s, BFHashEntry* hash, uint32_t* heap, uint32_t* heapCounter, BFVoxel* voxels);
/* visible list of the last compactify to HOST: int32 {x,y,z,ptr} x n */
int bf_scene_export_visible(bf_scene* s, int32_t* out4, uint32_t cap, uint32_t* n);
int bf_scene_synchronize(bf_scene* s);
int bf_scene_device_bytes(bf_scene* s, uint64_t* bytes);
/* time the next operations on the scene's stream */
int bf_scene_timer_start(bf_scene* s, bf_timer* t);
int bf_scene_timer_stop(bf_scene* s, bf_timer* t, float* ms); /* synchronizes */

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
/* same arithmetic on the host (tests) into host buffers */
int bf_synth_render_host(const BFSynthScene* scene, const float T[16], const BFDepthCameraParams* cam,
                         uint32_t noiseSeed, uint32_t frame, float* depth, uint8_t* color);

#ifdef __cplusplus
}
#endif
#endif
