// api.cpp — the C ABI (include/bf/bf.h). Catches every C++ exception at the boundary and
// turns it into a status code + bf_last_error() message.
#include "../../include/bf/bf.h"
#include "ba.h"
#include "recon.h"
#include "host_pool.h"
#include "trajectory.h"
#include "bf_runtime.h"
#include "synth.h"
#include "tsdf.h"
#include "image_codec.h"
#include "io.h"
#include "cache.h"
#include "frames.h"
#include "app.h"
#include "frontend.h"

#include <cstring>
#include <memory>
#include <limits>
#include <string>

namespace bf {

static thread_local std::string g_lastError;
void set_last_error(const std::string& msg) { g_lastError = msg; }

void synth_render_device(const BFSynthScene& sc, const BFMat4& T, const BFDepthCameraParams& cam, uint32_t noiseSeed,
                         uint32_t frame, float* depth, uint8_t* color, hipStream_t stream);
void synth_render_host(const BFSynthScene& sc, const BFMat4& T, const BFDepthCameraParams& cam, uint32_t noiseSeed,
                       uint32_t frame, float* depth, uint8_t* color);
void synth_scene_default(uint32_t seed, BFSynthScene* out);
void synth_to_raw(const float* depth, const uint8_t* color, uint32_t n, float shift, uint16_t* du, uint8_t* rgbx,
                  hipStream_t stream);
uint32_t synth_correspondences(const BFSynthScene& sc, const float* poses, uint32_t K, const BFDepthCameraParams& cam,
                               uint32_t maxPerPair, float minCovis, float noise, float outlierFrac, uint32_t seed,
                               BFEntryJ* out, uint32_t cap);
void synth_cache_frame(const BFSynthScene& sc, const BFMat4& T, const BFDepthCameraParams& cam, float* depth, float* campos,
                       float* normals, uint8_t* normalsU8, float* intensity, float* intensityDeriv);

// General cofactor inverse, cuda_SimpleMatrixUtil.h:980-1090 (host side of setLastRigidTransform,
// CUDASceneRepHashSDF.h:128-134).
BFMat4 mat4_inverse(const BFMat4& M) {
    const float* e = M.m;
    float inv[16];
    inv[0] = e[5] * e[10] * e[15] - e[5] * e[11] * e[14] - e[9] * e[6] * e[15] + e[9] * e[7] * e[14] + e[13] * e[6] * e[11] - e[13] * e[7] * e[10];
    inv[4] = -e[4] * e[10] * e[15] + e[4] * e[11] * e[14] + e[8] * e[6] * e[15] - e[8] * e[7] * e[14] - e[12] * e[6] * e[11] + e[12] * e[7] * e[10];
    inv[8] = e[4] * e[9] * e[15] - e[4] * e[11] * e[13] - e[8] * e[5] * e[15] + e[8] * e[7] * e[13] + e[12] * e[5] * e[11] - e[12] * e[7] * e[9];
    inv[12] = -e[4] * e[9] * e[14] + e[4] * e[10] * e[13] + e[8] * e[5] * e[14] - e[8] * e[6] * e[13] - e[12] * e[5] * e[10] + e[12] * e[6] * e[9];
    inv[1] = -e[1] * e[10] * e[15] + e[1] * e[11] * e[14] + e[9] * e[2] * e[15] - e[9] * e[3] * e[14] - e[13] * e[2] * e[11] + e[13] * e[3] * e[10];
    inv[5] = e[0] * e[10] * e[15] - e[0] * e[11] * e[14] - e[8] * e[2] * e[15] + e[8] * e[3] * e[14] + e[12] * e[2] * e[11] - e[12] * e[3] * e[10];
    inv[9] = -e[0] * e[9] * e[15] + e[0] * e[11] * e[13] + e[8] * e[1] * e[15] - e[8] * e[3] * e[13] - e[12] * e[1] * e[11] + e[12] * e[3] * e[9];
    inv[13] = e[0] * e[9] * e[14] - e[0] * e[10] * e[13] - e[8] * e[1] * e[14] + e[8] * e[2] * e[13] + e[12] * e[1] * e[10] - e[12] * e[2] * e[9];
    inv[2] = e[1] * e[6] * e[15] - e[1] * e[7] * e[14] - e[5] * e[2] * e[15] + e[5] * e[3] * e[14] + e[13] * e[2] * e[7] - e[13] * e[3] * e[6];
    inv[6] = -e[0] * e[6] * e[15] + e[0] * e[7] * e[14] + e[4] * e[2] * e[15] - e[4] * e[3] * e[14] - e[12] * e[2] * e[7] + e[12] * e[3] * e[6];
    inv[10] = e[0] * e[5] * e[15] - e[0] * e[7] * e[13] - e[4] * e[1] * e[15] + e[4] * e[3] * e[13] + e[12] * e[1] * e[7] - e[12] * e[3] * e[5];
    inv[14] = -e[0] * e[5] * e[14] + e[0] * e[6] * e[13] + e[4] * e[1] * e[14] - e[4] * e[2] * e[13] - e[12] * e[1] * e[6] + e[12] * e[2] * e[5];
    inv[3] = -e[1] * e[6] * e[11] + e[1] * e[7] * e[10] + e[5] * e[2] * e[11] - e[5] * e[3] * e[10] - e[9] * e[2] * e[7] + e[9] * e[3] * e[6];
    inv[7] = e[0] * e[6] * e[11] - e[0] * e[7] * e[10] - e[4] * e[2] * e[11] + e[4] * e[3] * e[10] + e[8] * e[2] * e[7] - e[8] * e[3] * e[6];
    inv[11] = -e[0] * e[5] * e[11] + e[0] * e[7] * e[9] + e[4] * e[1] * e[11] - e[4] * e[3] * e[9] - e[8] * e[1] * e[7] + e[8] * e[3] * e[5];
    inv[15] = e[0] * e[5] * e[10] - e[0] * e[6] * e[9] - e[4] * e[1] * e[10] + e[4] * e[2] * e[9] + e[8] * e[1] * e[6] - e[8] * e[2] * e[5];
    const float det = e[0] * inv[0] + e[1] * inv[4] + e[2] * inv[8] + e[3] * inv[12];
    const float detr = 1.0f / det;
    BFMat4 r;
    for (int i = 0; i < 16; i++) r.m[i] = inv[i] * detr;
    return r;
}

// float4x4 * float4x4 (cuda_SimpleMatrixUtil.h operator*): row i . column j, k = 0..3
BFMat4 mat4_mul(const BFMat4& a, const BFMat4& b) {
    BFMat4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float s = 0.0f;
            for (int k = 0; k < 4; k++) s += a.m[i * 4 + k] * b.m[k * 4 + j];
            r.m[i * 4 + j] = s;
        }
    return r;
}

static BFMat4 to_mat(const float* T) {
    BFMat4 m;
    std::memcpy(m.m, T, 64);
    return m;
}

}  // namespace bf

using namespace bf;

#define BF_TRY try {
#define BF_CATCH                                                      \
    return 0;                                                         \
    }                                                                 \
    catch (const bf::Error& e) {                                      \
        set_last_error(e.what());                                     \
        return e.code;                                                \
    }                                                                 \
    catch (const std::bad_alloc&) {                                   \
        set_last_error("host allocation failed");                    \
        return BF_ERR_CAPACITY;                                       \
    }                                                                 \
    catch (const std::exception& e) {                                 \
        set_last_error(e.what());                                     \
        return BF_ERR_INTERNAL;                                       \
    }

struct bf_scene {
    hipStream_t stream = nullptr;
    Scene* scene = nullptr;
};

struct bf_timer {
    hipEvent_t a = nullptr, b = nullptr;
};

struct bf_solver {
    hipStream_t stream = nullptr;
    Solver* solver = nullptr;
};
struct bf_comm {
    Comm* c = nullptr;
};
struct bf_sens {
    SensReader* r = nullptr;
};
struct bf_sens_writer {
    SensWriter* w = nullptr;
};
struct bf_params {
    ParamFile f;
};
struct bf_cache {
    hipStream_t stream = nullptr;
    Cache* c = nullptr;
};
struct bf_preproc {
    hipStream_t stream = nullptr;
    Preproc* p = nullptr;
};

extern "C" {

int bf_abi_version(void) { return BF_ABI_VERSION; }
int bf_abi_struct_size(const char* name, size_t* out) {
    BF_TRY
    BF_REQUIRE(name && out, BF_ERR_ARG, "null argument");
    static const struct {
        const char* n;
        size_t s;
    } kSizes[] = {
        {"BFHashParams", sizeof(BFHashParams)},
        {"BFDepthCameraParams", sizeof(BFDepthCameraParams)},
        {"BFRayCastParams", sizeof(BFRayCastParams)},
        {"BFHashEntry", sizeof(BFHashEntry)},
        {"BFVoxel", sizeof(BFVoxel)},
        {"BFEntryJ", sizeof(BFEntryJ)},
        {"BFFixOp", sizeof(BFFixOp)},
        {"BFSolveResult", sizeof(BFSolveResult)},
        {"BFTsdfStats", sizeof(BFTsdfStats)},
        {"BFSceneCapacity", sizeof(BFSceneCapacity)},
        {"BFSensInfo", sizeof(BFSensInfo)},
        {"BFPreprocessOptions", sizeof(BFPreprocessOptions)},
        {"BFMarchingCubesParams", sizeof(BFMarchingCubesParams)},
        {"BFCacheOptions", sizeof(BFCacheOptions)},
        {"BFCorrOptions", sizeof(BFCorrOptions)},
        {"BFCachedFrame", sizeof(BFCachedFrame)},
        {"BFSceneOptions", sizeof(BFSceneOptions)},
        {"BFVoxelOp", sizeof(BFVoxelOp)},
        {"BFSolverOptions", sizeof(BFSolverOptions)},
        {"BFVerifyOptions", sizeof(BFVerifyOptions)},
        {"BFReconOptions", sizeof(BFReconOptions)},
        {"BFReconStats", sizeof(BFReconStats)},
        {"BFEndSequenceOptions", sizeof(BFEndSequenceOptions)},
        {"BFEndSequenceResult", sizeof(BFEndSequenceResult)},
        {"BFQueueEvent", sizeof(BFQueueEvent)},
        {"BFAppOptions", sizeof(BFAppOptions)},
        {"BFAppInfo", sizeof(BFAppInfo)},
        {"BFAppResult", sizeof(BFAppResult)},
        {"BFAppTiming", sizeof(BFAppTiming)},
        {"BFMcTriangle", sizeof(BFMcTriangle)},
        {"BFSynthScene", sizeof(BFSynthScene)},
        {"BFRenderStats", sizeof(BFRenderStats)}};
    for (const auto& e : kSizes)
        if (std::strcmp(e.n, name) == 0) {
            *out = e.s;
            return 0;
        }
    throw Error(BF_ERR_ARG, std::string("unknown struct ") + name);
    BF_CATCH
}
const char* bf_last_error(void) { return g_lastError.c_str(); }

int bf_device_count(int* count) {
    BF_TRY
    BF_HIP(hipGetDeviceCount(count));
    BF_CATCH
}
int bf_set_device(int device) {
    BF_TRY
    BF_HIP(hipSetDevice(device));
    BF_CATCH
}
int bf_set_host_threads(int n) {
    BF_TRY
    BF_REQUIRE(n >= 1 && n <= 256, BF_ERR_ARG, "host threads 1..256");
    HostPool::requested().store(n);
    BF_CATCH
}
int bf_device_synchronize(void) {
    BF_TRY
    BF_HIP(hipDeviceSynchronize());
    BF_CATCH
}
int bf_malloc(void** dptr, size_t bytes) {
    BF_TRY
    BF_REQUIRE(dptr != nullptr, BF_ERR_ARG, "dptr");
    BF_HIP(hipMalloc(dptr, bytes ? bytes : 1));
    BF_CATCH
}
int bf_free(void* dptr) {
    BF_TRY
    if (dptr) BF_HIP(hipFree(dptr));
    BF_CATCH
}
int bf_memcpy_h2d(void* dst, const void* src, size_t bytes) {
    BF_TRY
    BF_HIP(hipDeviceSynchronize());  // ordered after work on every scene/solver stream
    BF_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    BF_CATCH
}
int bf_memcpy_d2h(void* dst, const void* src, size_t bytes) {
    BF_TRY
    BF_HIP(hipDeviceSynchronize());  // ordered after work on every scene/solver stream
    BF_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    BF_CATCH
}
int bf_memcpy_d2d(void* dst, const void* src, size_t bytes) {
    BF_TRY
    BF_HIP(hipDeviceSynchronize());  // ordered after work on every scene/solver stream
    BF_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToDevice));
    BF_CATCH
}
int bf_memset(void* dptr, int value, size_t bytes) {
    BF_TRY
    BF_HIP(hipDeviceSynchronize());
    BF_HIP(hipMemset(dptr, value, bytes));
    BF_HIP(hipDeviceSynchronize());
    BF_CATCH
}
int bf_timer_create(bf_timer** out) {
    BF_TRY
    bf_timer* t = new bf_timer();
    BF_HIP(hipEventCreate(&t->a));
    BF_HIP(hipEventCreate(&t->b));
    *out = t;
    BF_CATCH
}
int bf_timer_destroy(bf_timer* t) {
    BF_TRY
    if (t) {
        if (t->a) (void)hipEventDestroy(t->a);
        if (t->b) (void)hipEventDestroy(t->b);
        delete t;
    }
    BF_CATCH
}

// ---- scene ------------------------------------------------------------------------------
int bf_scene_create(const BFHashParams* params, const BFSceneOptions* opts, bf_scene** out) {
    BF_TRY
    BF_REQUIRE(params && out, BF_ERR_ARG, "null argument");
    const SceneConfig cfg = scene_config(*params, opts);
    bf_scene* s = new bf_scene();
    try {
        BF_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        s->scene = new Scene(cfg, s->stream);
    } catch (...) {
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
        throw;
    }
    *out = s;
    BF_CATCH
}
int bf_scene_destroy(bf_scene* s) {
    BF_TRY
    if (s) {
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        delete s->scene;
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
    }
    BF_CATCH
}
int bf_scene_reset(bf_scene* s) {
    BF_TRY
    BF_REQUIRE(s, BF_ERR_ARG, "null scene");
    s->scene->reset();
    BF_CATCH
}
int bf_scene_integrate(bf_scene* s, const float T[16], const float* depth, const uint8_t* color,
                       const BFDepthCameraParams* cam, const uint32_t* bitMask) {
    BF_TRY
    BF_REQUIRE(s && T && cam, BF_ERR_ARG, "null argument");
    s->scene->integrate(to_mat(T), depth, color, *cam, false, bitMask);
    BF_CATCH
}
int bf_scene_deintegrate(bf_scene* s, const float T[16], const float* depth, const uint8_t* color,
                         const BFDepthCameraParams* cam, const uint32_t* bitMask) {
    BF_TRY
    BF_REQUIRE(s && T && cam, BF_ERR_ARG, "null argument");
    s->scene->integrate(to_mat(T), depth, color, *cam, true, bitMask);
    BF_CATCH
}
int bf_scene_reintegrate(bf_scene* s, const float Told[16], const float Tnew[16], const float* depth, const uint8_t* color,
                         const BFDepthCameraParams* cam) {
    BF_TRY
    BF_REQUIRE(s && Told && Tnew && cam, BF_ERR_ARG, "null argument");
    s->scene->reintegrate(to_mat(Told), to_mat(Tnew), depth, color, *cam);
    BF_CATCH
}
int bf_scene_apply_ops(bf_scene* s, const BFVoxelOp* ops, uint32_t n, const BFDepthCameraParams* cam) {
    BF_TRY
    BF_REQUIRE(s && cam && (ops || n == 0), BF_ERR_ARG, "null argument");
    BF_REQUIRE(n <= BF_MAX_VOXEL_OPS && n <= Scene::kMaxOps, BF_ERR_ARG, "too many ops");
    VoxelOp v[BF_MAX_VOXEL_OPS];
    for (uint32_t k = 0; k < n; k++) v[k] = VoxelOp{to_mat(ops[k].T), ops[k].depth, ops[k].color, ops[k].deintegrate != 0};
    s->scene->applyOps(v, n, *cam);
    BF_CATCH
}
int bf_scene_garbage_collect(bf_scene* s) {
    BF_TRY
    BF_REQUIRE(s, BF_ERR_ARG, "null scene");
    s->scene->garbageCollect();
    BF_CATCH
}
int bf_scene_compactify(bf_scene* s, const float T[16], const BFDepthCameraParams* cam, uint32_t* nVisible) {
    BF_TRY
    BF_REQUIRE(s && T && cam, BF_ERR_ARG, "null argument");
    s->scene->compactify(to_mat(T), *cam);
    if (nVisible) *nVisible = s->scene->numVisible();
    BF_CATCH
}
int bf_scene_heap_free_count(bf_scene* s, uint32_t* count) {
    BF_TRY
    BF_REQUIRE(s && count, BF_ERR_ARG, "null argument");
    *count = s->scene->heapFreeCount();
    BF_CATCH
}
int bf_scene_num_visible(bf_scene* s, uint32_t* count) {
    BF_TRY
    BF_REQUIRE(s && count, BF_ERR_ARG, "null argument");
    *count = s->scene->numVisible();
    BF_CATCH
}
int bf_scene_error_flags(bf_scene* s, uint32_t* flags) {
    BF_TRY
    BF_REQUIRE(s && flags, BF_ERR_ARG, "null argument");
    *flags = s->scene->errorFlags();
    BF_CATCH
}
int bf_scene_capacity(bf_scene* s, BFSceneCapacity* out) {
    BF_TRY
    BF_REQUIRE(s && out, BF_ERR_ARG, "null argument");
    *out = s->scene->capacity();
    BF_CATCH
}
int bf_scene_get_stats(bf_scene* s, BFTsdfStats* out) {
    BF_TRY
    BF_REQUIRE(s && out, BF_ERR_ARG, "null argument");
    *out = s->scene->stats();
    BF_CATCH
}
int bf_scene_reset_stats(bf_scene* s) {
    BF_TRY
    BF_REQUIRE(s, BF_ERR_ARG, "null scene");
    s->scene->resetStats();
    BF_CATCH
}
int bf_scene_export(bf_scene* s, BFHashEntry* hash, uint32_t* heap, uint32_t* heapCounter, BFVoxel* voxels) {
    BF_TRY
    BF_REQUIRE(s, BF_ERR_ARG, "null scene");
    s->scene->exportState(hash, heap, heapCounter, voxels);
    BF_CATCH
}
int bf_scene_export_blocks(bf_scene* s, int32_t* out4, uint32_t cap, uint32_t* n) {
    BF_TRY
    BF_REQUIRE(s && n && (out4 || cap == 0), BF_ERR_ARG, "null argument");
    *n = s->scene->exportBlocks(reinterpret_cast<int4*>(out4), cap);
    BF_CATCH
}
int bf_scene_export_visible(bf_scene* s, int32_t* out4, uint32_t cap, uint32_t* n) {
    BF_TRY
    BF_REQUIRE(s && out4 && n, BF_ERR_ARG, "null argument");
    *n = s->scene->exportVisible(reinterpret_cast<int4*>(out4), cap);
    BF_CATCH
}
int bf_scene_export_block_voxels(bf_scene* s, uint32_t first, uint32_t count, BFVoxel* out) {
    BF_TRY
    BF_REQUIRE(s && (out || count == 0), BF_ERR_ARG, "null argument");
    s->scene->exportBlockVoxels(first, count, out);
    BF_CATCH
}
int bf_scene_raycast(bf_scene* s, const float T[16], const BFDepthCameraParams* cam, const BFRayCastParams* rp, float* depth,
                     float* depth4, float* normals, float* colors, float* rayMin, float* rayMax) {
    BF_TRY
    BF_REQUIRE(s && T && cam && rp, BF_ERR_ARG, "null argument");
    s->scene->raycast(to_mat(T), *cam, *rp, depth, reinterpret_cast<float4*>(depth4), reinterpret_cast<float4*>(normals),
                      reinterpret_cast<float4*>(colors), rayMin, rayMax);
    BF_CATCH
}
int bf_scene_extract_mesh(bf_scene* s, const BFMarchingCubesParams* p, BFMcTriangle* tris, uint32_t* numTriangles,
                          uint32_t* totalTriangles) {
    BF_TRY
    BF_REQUIRE(s && p && numTriangles, BF_ERR_ARG, "null argument");
    *numTriangles = s->scene->extractMesh(*p, tris, tris ? p->maxNumTriangles : 0u, totalTriangles);
    BF_CATCH
}
int bf_scene_synchronize(bf_scene* s) {
    BF_TRY
    BF_REQUIRE(s, BF_ERR_ARG, "null scene");
    BF_HIP(hipStreamSynchronize(s->stream));
    BF_CATCH
}
int bf_scene_device_bytes(bf_scene* s, uint64_t* bytes) {
    BF_TRY
    BF_REQUIRE(s && bytes, BF_ERR_ARG, "null argument");
    *bytes = s->scene->deviceBytes();
    BF_CATCH
}
int bf_scene_timer_start(bf_scene* s, bf_timer* t) {
    BF_TRY
    BF_REQUIRE(s && t, BF_ERR_ARG, "null argument");
    BF_HIP(hipEventRecord(t->a, s->stream));
    BF_CATCH
}
int bf_scene_timer_stop(bf_scene* s, bf_timer* t, float* ms) {
    BF_TRY
    BF_REQUIRE(s && t && ms, BF_ERR_ARG, "null argument");
    BF_HIP(hipEventRecord(t->b, s->stream));
    BF_HIP(hipEventSynchronize(t->b));
    BF_HIP(hipEventElapsedTime(ms, t->a, t->b));
    BF_CATCH
}

// ---- synthetic stream ---------------------------------------------------------------------
int bf_synth_scene_default(uint32_t seed, BFSynthScene* out) {
    BF_TRY
    BF_REQUIRE(out, BF_ERR_ARG, "null argument");
    synth_scene_default(seed, out);
    BF_CATCH
}
int bf_synth_pose(uint32_t frame, float T[16]) {
    BF_TRY
    BF_REQUIRE(T, BF_ERR_ARG, "null argument");
    synth_pose(frame, T);
    BF_CATCH
}
int bf_synth_render(const BFSynthScene* scene, const float T[16], const BFDepthCameraParams* cam, uint32_t noiseSeed,
                    uint32_t frame, float* d_depth, uint8_t* d_color) {
    BF_TRY
    BF_REQUIRE(scene && T && cam && d_depth, BF_ERR_ARG, "null argument");
    synth_render_device(*scene, to_mat(T), *cam, noiseSeed, frame, d_depth, d_color, nullptr);
    BF_HIP(hipStreamSynchronize(nullptr));
    BF_CATCH
}
int bf_synth_to_raw(const float* d_depth, const uint8_t* d_color, uint32_t numPixels, float depthShift,
                    uint16_t* d_depthU16, uint8_t* d_rgbx) {
    BF_TRY
    BF_REQUIRE(d_depth && d_color && d_depthU16 && d_rgbx && depthShift > 0.0f, BF_ERR_ARG, "null argument");
    synth_to_raw(d_depth, d_color, numPixels, depthShift, d_depthU16, d_rgbx, nullptr);
    BF_HIP(hipStreamSynchronize(nullptr));
    BF_CATCH
}
int bf_synth_render_host(const BFSynthScene* scene, const float T[16], const BFDepthCameraParams* cam, uint32_t noiseSeed,
                         uint32_t frame, float* depth, uint8_t* color) {
    BF_TRY
    BF_REQUIRE(scene && T && cam && depth, BF_ERR_ARG, "null argument");
    synth_render_host(*scene, to_mat(T), *cam, noiseSeed, frame, depth, color);
    BF_CATCH
}
int bf_synth_correspondences(const BFSynthScene* scene, const float* poses, uint32_t K, const BFDepthCameraParams* cam,
                             uint32_t maxPerPair, float minCovis, float noise, float outlierFrac, uint32_t seed,
                             BFEntryJ* out, uint32_t cap, uint32_t* n) {
    BF_TRY
    BF_REQUIRE(scene && poses && cam && out && n, BF_ERR_ARG, "null argument");
    *n = synth_correspondences(*scene, poses, K, *cam, maxPerPair, minCovis, noise, outlierFrac, seed, out, cap);
    BF_CATCH
}
int bf_synth_cache_frame(const BFSynthScene* scene, const float T[16], const BFDepthCameraParams* cam, float* depth,
                         float* campos, float* normals, uint8_t* normalsU8, float* intensity, float* intensityDeriv) {
    BF_TRY
    BF_REQUIRE(scene && T && cam && depth && campos && normals && normalsU8 && intensity && intensityDeriv, BF_ERR_ARG,
               "null argument");
    synth_cache_frame(*scene, to_mat(T), *cam, depth, campos, normals, normalsU8, intensity, intensityDeriv);
    BF_CATCH
}

// ---- bundle adjustment ---------------------------------------------------------------------
int bf_solver_create(uint32_t maxImages, uint32_t maxCorr, const BFSolverOptions* o, bf_solver** out) {
    BF_TRY
    BF_REQUIRE(out, BF_ERR_ARG, "null argument");
    const SolverConfig cfg = make_solver_config(maxImages, maxCorr, o);
    bf_solver* s = new bf_solver();
    try {
        BF_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        s->solver = new Solver(cfg, s->stream);
    } catch (...) {
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
        throw;
    }
    *out = s;
    BF_CATCH
}
int bf_solver_destroy(bf_solver* s) {
    BF_TRY
    if (s) {
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        delete s->solver;
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
    }
    BF_CATCH
}
int bf_solver_solve(bf_solver* s, BFEntryJ* corr, uint32_t nCorr, const int* valid, uint32_t nImages, uint32_t nNonLin,
                    uint32_t nLin, const float* wSparse, const float* wDenseDepth, const float* wDenseColor,
                    const BFCachedFrame* cache, uint32_t cacheW, uint32_t cacheH, const float intrinsics[4], float* rot,
                    float* trans, int rebuildJT, int findMaxResidual) {
    BF_TRY
    BF_REQUIRE(s && valid && rot && trans && wSparse, BF_ERR_ARG, "null argument");
    BF_REQUIRE(nCorr == 0 || corr, BF_ERR_ARG, "null correspondences");
    SolveArgs a{};
    a.corr = corr; a.numCorr = nCorr; a.valid = valid; a.numImages = nImages; a.nNonLin = nNonLin; a.nLin = nLin;
    a.wSparse = wSparse; a.wDenseDepth = wDenseDepth; a.wDenseColor = wDenseColor;
    a.cache = cache; a.cacheW = cacheW; a.cacheH = cacheH;
    if (intrinsics) std::memcpy(a.intrinsics, intrinsics, 16);
    a.rot = rot; a.trans = trans; a.rebuildJT = rebuildJT != 0; a.findMaxResidual = findMaxResidual != 0;
    s->solver->solve(a);
    BF_CATCH
}
int bf_solver_result(bf_solver* s, BFSolveResult* out) {
    BF_TRY
    BF_REQUIRE(s && out, BF_ERR_ARG, "null argument");
    SolveResult r = s->solver->result();
    out->gnIterations = r.gnIterations;
    out->pcgIterations = r.pcgIterations;
    out->maxResidual = r.maxResidual;
    out->maxResidualIndex = r.maxResidualIndex;
    out->energy = r.energy;
    out->highResidualCount = r.highResidualCount;
    out->numDensePairs = r.numDensePairs;
    out->error = r.error;
    out->skipped = r.skipped;
    out->verifyUsed = r.verifyUsed;
    out->verifyOk = r.verifyOk;
    BF_CATCH
}
int bf_solver_verify_trajectory(bf_solver* s, const float* T, const int* valid, uint32_t nImages, uint32_t nCorr,
                                const BFCachedFrame* cache, uint32_t cacheW, uint32_t cacheH, const float intrinsics[4],
                                const BFVerifyOptions* o, float* pairStats, int* validOut) {
    BF_TRY
    BF_REQUIRE(s && T && valid && cache && intrinsics, BF_ERR_ARG, "null argument");
    VerifyParams p = verify_params(o);
    p.T = T; p.valid = valid; p.numImages = nImages; p.numCorr = nCorr; p.cache = cache;
    p.cacheW = cacheW; p.cacheH = cacheH;
    std::memcpy(p.intrinsics, intrinsics, 16);
    p.pairStats = pairStats;
    s->solver->verify(p);
    if (validOut) {
        int v = 0;
        BF_HIP(hipMemcpyAsync(&v, s->solver->verifyFlag(), 4, hipMemcpyDeviceToHost, s->stream));
        BF_HIP(hipStreamSynchronize(s->stream));
        *validOut = v;
    }
    BF_CATCH
}
int bf_solver_num_entries_per_row(bf_solver* s, const int** dptr) {
    BF_TRY
    BF_REQUIRE(s && dptr, BF_ERR_ARG, "null argument");
    *dptr = s->solver->numEntriesPerRow();
    BF_CATCH
}
int bf_solver_synchronize(bf_solver* s) {
    BF_TRY
    BF_REQUIRE(s, BF_ERR_ARG, "null solver");
    BF_HIP(hipStreamSynchronize(s->stream));
    BF_CATCH
}
int bf_solver_timer_start(bf_solver* s, bf_timer* t) {
    BF_TRY
    BF_REQUIRE(s && t, BF_ERR_ARG, "null argument");
    BF_HIP(hipEventRecord(t->a, s->stream));
    BF_CATCH
}
int bf_solver_timer_stop(bf_solver* s, bf_timer* t, float* ms) {
    BF_TRY
    BF_REQUIRE(s && t && ms, BF_ERR_ARG, "null argument");
    BF_HIP(hipEventRecord(t->b, s->stream));
    BF_HIP(hipEventSynchronize(t->b));
    BF_HIP(hipEventElapsedTime(ms, t->a, t->b));
    BF_CATCH
}
int bf_solver_pcg_time(bf_solver* s, int enable, double* ms, uint64_t* launches) {
    BF_TRY
    BF_REQUIRE(s, BF_ERR_ARG, "null solver");
    KernelClock& c = s->solver->pcgClock();
    if (ms) *ms = c.enabled() ? c.totalMs() : 0.0;
    if (launches) *launches = c.enabled() ? c.launches() : 0;
    if (enable && !c.enabled()) c.reset();
    c.enable(enable != 0);
    BF_CATCH
}
int bf_solver_matrices_to_poses(bf_solver* s, const float* T, uint32_t n, float* rot, float* trans, const int* valid) {
    BF_TRY
    BF_REQUIRE(s && T && rot && trans && valid, BF_ERR_ARG, "null argument");
    matrices_to_poses(T, n, rot, trans, valid, s->stream);
    BF_CATCH
}
int bf_solver_poses_to_matrices(bf_solver* s, const float* rot, const float* trans, uint32_t n, float* T, const int* valid) {
    BF_TRY
    BF_REQUIRE(s && T && rot && trans && valid, BF_ERR_ARG, "null argument");
    poses_to_matrices(rot, trans, n, T, valid, s->stream);
    BF_CATCH
}
int bf_solver_invalidate_image_pair(bf_solver* s, BFEntryJ* corr, uint32_t nCorr, uint32_t i, uint32_t j) {
    BF_TRY
    BF_REQUIRE(s && (corr || nCorr == 0), BF_ERR_ARG, "null argument");
    invalidate_image_pair(corr, nCorr, i, j, s->stream);
    BF_CATCH
}
int bf_solver_check_invalid_frames(bf_solver* s, int* valid, uint32_t nImages, BFEntryJ* corr, uint32_t nCorr,
                                   int comprehensive) {
    BF_TRY
    BF_REQUIRE(s && valid, BF_ERR_ARG, "null argument");
    check_invalid_frames(s->solver->numEntriesPerRow(), valid, nImages, corr, nCorr, comprehensive != 0, s->stream);
    BF_CATCH
}

int bf_solver_set_shard(bf_solver* s, uint32_t count, uint32_t index, bf_comm* comm) {
    BF_TRY
    BF_REQUIRE(s, BF_ERR_ARG, "null argument");
    s->solver->setShard(count, index, comm ? comm->c : nullptr);
    BF_CATCH
}
int bf_solver_export_pairs(bf_solver* s, double* stats, int32_t* pairAB, uint32_t cap, uint32_t* total) {
    BF_TRY
    BF_REQUIRE(s && total, BF_ERR_ARG, "null argument");
    *total = s->solver->exportPairs(stats, pairAB, cap);
    BF_CATCH
}

// ---- multi-GPU communicator (RCCL) --------------------------------------------------------
int bf_comm_unique_id(uint8_t id[128]) {
    BF_TRY
    BF_REQUIRE(id, BF_ERR_ARG, "null argument");
    Comm::uniqueId(id);
    BF_CATCH
}
int bf_comm_create(const uint8_t id[128], int nranks, int rank, bf_comm** out) {
    BF_TRY
    BF_REQUIRE(id && out, BF_ERR_ARG, "null argument");
    bf_comm* h = new bf_comm();
    try {
        h->c = new Comm(id, nranks, rank);
    } catch (...) {
        delete h;
        throw;
    }
    *out = h;
    BF_CATCH
}
int bf_comm_create_loopback(int nranks, int timeoutMs, size_t capacityBytes, bf_comm** out) {
    BF_TRY
    BF_REQUIRE(out && nranks >= 1, BF_ERR_ARG, "null argument / nranks");
    auto group = Comm::loopbackGroup(nranks, timeoutMs, capacityBytes);
    std::vector<bf_comm*> made;
    try {
        for (int r = 0; r < nranks; r++) {
            bf_comm* h = new bf_comm();
            made.push_back(h);
            h->c = new Comm(group, r);
        }
    } catch (...) {
        for (bf_comm* h : made) {
            delete h->c;
            delete h;
        }
        throw;
    }
    for (int r = 0; r < nranks; r++) out[r] = made[(size_t)r];
    BF_CATCH
}
int bf_comm_destroy(bf_comm* c) {
    BF_TRY
    if (c) {
        delete c->c;
        delete c;
    }
    BF_CATCH
}
int bf_comm_allreduce_sum_f64(bf_comm* c, double* d, size_t n) {
    BF_TRY
    BF_REQUIRE(c && (d || n == 0), BF_ERR_ARG, "null argument");
    hipStream_t st = nullptr;
    BF_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    try {
        c->c->allreduceSum(d, n, st);
        BF_HIP(hipStreamSynchronize(st));
        c->c->checkError();  // a collective that timed out waiting for a rank leaves no valid sum
    } catch (...) {
        (void)hipStreamDestroy(st);
        throw;
    }
    BF_HIP(hipStreamDestroy(st));
    BF_CATCH
}

// ---- reconstruction loop ----------------------------------------------------------------
struct bf_recon {
    Recon* r = nullptr;
};

int bf_recon_create(const BFHashParams* params, const BFSceneOptions* sceneOpts, const BFDepthCameraParams* cam,
                    const BFReconOptions* opts, bf_recon** out) {
    BF_TRY
    BF_REQUIRE(params && cam && opts && out, BF_ERR_ARG, "null argument");
    bf_recon* h = new bf_recon();
    try {
        h->r = new Recon(*params, sceneOpts, *cam, *opts);
    } catch (...) {
        delete h;
        throw;
    }
    *out = h;
    BF_CATCH
}
int bf_recon_destroy(bf_recon* r) {
    BF_TRY
    if (r) {
        delete r->r;
        delete r;
    }
    BF_CATCH
}
int bf_recon_set_frame(bf_recon* r, uint32_t f, const float* depth, const uint8_t* color, const BFCachedFrame* cache,
                       const float Tinc[16]) {
    BF_TRY
    BF_REQUIRE(r && depth && Tinc, BF_ERR_ARG, "null argument");
    r->r->setFrame(f, depth, color, cache, to_mat(Tinc));
    BF_CATCH
}
int bf_recon_set_local_correspondences(bf_recon* r, uint32_t submap, BFEntryJ* corr, uint32_t n) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->setLocalCorrespondences(submap, corr, n);
    BF_CATCH
}
int bf_recon_set_global_correspondences(bf_recon* r, BFEntryJ* corr, uint32_t n, const uint32_t* prefix,
                                        uint32_t numKeyframes) {
    BF_TRY
    BF_REQUIRE(r && (prefix || numKeyframes == 0), BF_ERR_ARG, "null argument");
    r->r->setGlobalCorrespondences(corr, n, prefix, numKeyframes);
    BF_CATCH
}
int bf_recon_set_initial_pose(bf_recon* r, const float T0[16]) {
    BF_TRY
    BF_REQUIRE(r && T0, BF_ERR_ARG, "null argument");
    r->r->setInitialPose(to_mat(T0));
    BF_CATCH
}
int bf_recon_process_frame(bf_recon* r, uint32_t f) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->processFrame(f);
    BF_CATCH
}
int bf_recon_finish(bf_recon* r) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->finish();
    BF_CATCH
}
int bf_recon_end_solve(bf_recon* r, float denseDepthWeight, BFSolveResult* out, float* ms) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    BF_REQUIRE(denseDepthWeight >= 0.0f, BF_ERR_ARG, "negative dense weight");
    const SolveResult res = r->r->endSolve(denseDepthWeight, ms);
    if (out) {
        *out = BFSolveResult{};
        out->gnIterations = res.gnIterations;
        out->pcgIterations = res.pcgIterations;
        out->maxResidual = res.maxResidual;
        out->maxResidualIndex = res.maxResidualIndex;
        out->energy = res.energy;
        out->highResidualCount = res.highResidualCount;
        out->numDensePairs = res.numDensePairs;
        out->error = res.error;
        out->skipped = res.skipped;
    }
    BF_CATCH
}
int bf_recon_submap_poses(bf_recon* r, uint32_t s, float* local, float* global, int32_t* valid, uint32_t* numLocal,
                          uint32_t* numKeyframes, int32_t* localValid) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->submapPoses(s, local, global, valid, numLocal, numKeyframes, localValid);
    BF_CATCH
}
int bf_recon_reintegrate(bf_recon* r) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->reintegrate();
    BF_CATCH
}
int bf_recon_synchronize(bf_recon* r) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->synchronize();
    BF_CATCH
}
int bf_recon_stats(bf_recon* r, BFReconStats* out) {
    BF_TRY
    BF_REQUIRE(r && out, BF_ERR_ARG, "null argument");
    *out = r->r->stats();
    BF_CATCH
}
int bf_recon_reset_stats(bf_recon* r) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->resetStats();
    BF_CATCH
}
int bf_recon_scene_stats(bf_recon* r, BFTsdfStats* out) {
    BF_TRY
    BF_REQUIRE(r && out, BF_ERR_ARG, "null argument");
    r->r->synchronize();
    *out = r->r->scene().stats();
    BF_CATCH
}
int bf_recon_heap_free_count(bf_recon* r, uint32_t* count) {
    BF_TRY
    BF_REQUIRE(r && count, BF_ERR_ARG, "null argument");
    *count = r->r->scene().heapFreeCount();
    BF_CATCH
}
int bf_recon_scene_capacity(bf_recon* r, BFSceneCapacity* out) {
    BF_TRY
    BF_REQUIRE(r && out, BF_ERR_ARG, "null argument");
    *out = r->r->sceneCapacity();
    BF_CATCH
}
int bf_recon_trajectory(bf_recon* r, float* T, uint32_t n) {
    BF_TRY
    BF_REQUIRE(r && T, BF_ERR_ARG, "null argument");
    r->r->trajectory(reinterpret_cast<BFMat4*>(T), n);
    BF_CATCH
}

int bf_recon_export(bf_recon* r, BFHashEntry* hash, uint32_t* heap, uint32_t* heapCounter, BFVoxel* voxels) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->synchronize();
    r->r->scene().exportState(hash, heap, heapCounter, voxels);
    BF_CATCH
}
int bf_recon_export_blocks(bf_recon* r, int32_t* out4, uint32_t cap, uint32_t* n) {
    BF_TRY
    BF_REQUIRE(r && n && (out4 || cap == 0), BF_ERR_ARG, "null argument");
    r->r->synchronize();
    *n = r->r->scene().exportBlocks(reinterpret_cast<int4*>(out4), cap);
    BF_CATCH
}
int bf_recon_raycast(bf_recon* r, const float T[16], const BFRayCastParams* rp, float* depth, float* depth4, float* normals,
                     float* colors) {
    BF_TRY
    BF_REQUIRE(r && T && rp, BF_ERR_ARG, "null argument");
    r->r->scene().raycast(to_mat(T), r->r->camera(), *rp, depth, reinterpret_cast<float4*>(depth4),
                          reinterpret_cast<float4*>(normals), reinterpret_cast<float4*>(colors), nullptr, nullptr);
    BF_CATCH
}
int bf_recon_capture_global_solve(bf_recon* r, uint32_t submap) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null argument");
    r->r->captureGlobalSolve(submap);
    BF_CATCH
}
int bf_recon_captured_global_solve(bf_recon* r, BFEntryJ* corrIn, BFEntryJ* corrOut, uint32_t cap, uint32_t* nCorr,
                                   float* poseIn, float* poseOut, int32_t* valid, uint32_t capImages, uint32_t* nImages) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null argument");
    r->r->capturedGlobalSolve(corrIn, corrOut, cap, nCorr, poseIn, poseOut, valid, capImages, nImages);
    BF_CATCH
}
int bf_recon_set_render(bf_recon* r, const BFRayCastParams* rp) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null argument");
    r->r->setRender(rp);
    BF_CATCH
}
int bf_recon_render_output(bf_recon* r, const float** depth, const float** depth4, const float** normals,
                           const float** colors) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null argument");
    r->r->renderOutput(depth, depth4, normals, colors);
    BF_CATCH
}
int bf_recon_extract_mesh(bf_recon* r, const BFMarchingCubesParams* p, BFMcTriangle* tris, uint32_t* numTriangles,
                          uint32_t* totalTriangles) {
    BF_TRY
    BF_REQUIRE(r && p && numTriangles, BF_ERR_ARG, "null argument");
    r->r->synchronize();
    *numTriangles = r->r->scene().extractMesh(*p, tris, tris ? p->maxNumTriangles : 0u, totalTriangles);
    BF_CATCH
}
int bf_recon_render_stats(bf_recon* r, BFRenderStats* out) {
    BF_TRY
    BF_REQUIRE(r && out, BF_ERR_ARG, "null argument");
    r->r->synchronize();
    r->r->scene().renderStats(*out);
    BF_CATCH
}
int bf_recon_render_time(bf_recon* r, double* ms, uint64_t* launches) {
    BF_TRY
    BF_REQUIRE(r && ms && launches, BF_ERR_ARG, "null argument");
    r->r->synchronize();
    auto& clk = r->r->scene().renderClock();
    if (!clk.enabled()) clk.enable(true);
    *ms = clk.totalMs();
    *launches = clk.launches();
    BF_CATCH
}
int bf_recon_set_comm(bf_recon* r, bf_comm* c) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null argument");
    r->r->setComm(c ? c->c : nullptr);
    BF_CATCH
}
int bf_recon_attach_cache(bf_recon* r, bf_cache* c) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->attachCache(c ? c->c : nullptr);
    BF_CATCH
}
int bf_recon_set_frame_source(bf_recon* r, uint32_t f, const float* depth, const uint8_t* color, uint32_t colorW,
                              uint32_t colorH) {
    BF_TRY
    BF_REQUIRE(r && depth && color, BF_ERR_ARG, "null argument");
    r->r->setFrameSource(f, depth, color, colorW, colorH);
    BF_CATCH
}
int bf_recon_attach_preproc(bf_recon* r, bf_preproc* p) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    r->r->attachPreproc(p ? p->p : nullptr);
    BF_CATCH
}
int bf_recon_set_frame_raw(bf_recon* r, uint32_t f, const uint16_t* depthU16, const uint8_t* rgbx) {
    BF_TRY
    BF_REQUIRE(r && depthU16 && rgbx, BF_ERR_ARG, "null argument");
    r->r->setFrameRaw(f, depthU16, rgbx);
    BF_CATCH
}
int bf_recon_frame_ready(bf_recon* r, uint32_t f, void* stream) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null argument");
    r->r->inputsProduced(f, static_cast<hipStream_t>(stream));
    BF_CATCH
}
int bf_recon_end_sequence(bf_recon* r, const BFEndSequenceOptions* o, BFEndSequenceResult* out) {
    BF_TRY
    BF_REQUIRE(r && o, BF_ERR_ARG, "null argument");
    const BFEndSequenceResult res = r->r->endSequence(*o);
    if (out) *out = res;
    BF_CATCH
}
int bf_recon_optimized_trajectory(bf_recon* r, float* T, uint32_t cap, uint32_t* n) {
    BF_TRY
    BF_REQUIRE(r && n && (T || cap == 0), BF_ERR_ARG, "null argument");
    r->r->synchronize();
    *n = r->r->optimizedTrajectory(reinterpret_cast<BFMat4*>(T), cap);
    BF_CATCH
}
int bf_recon_queue_trace(bf_recon* r, BFQueueEvent* events, uint32_t capEvents, uint32_t* nEvents, float* transforms,
                         uint32_t capTransforms, uint32_t* nTransforms, BFFixOp* fixes, uint32_t capFixes, uint32_t* nFixes) {
    BF_TRY
    BF_REQUIRE(r, BF_ERR_ARG, "null recon");
    BF_REQUIRE((events || capEvents == 0) && (transforms || capTransforms == 0) && (fixes || capFixes == 0), BF_ERR_ARG,
               "null output with a capacity");
    const auto& ev = r->r->queueEvents();
    const auto& tr = r->r->queueTransforms();
    const auto& fx = r->r->queueFixes();
    if (nEvents) *nEvents = (uint32_t)ev.size();
    if (nTransforms) *nTransforms = (uint32_t)tr.size();
    if (nFixes) *nFixes = (uint32_t)fx.size();
    for (uint32_t i = 0; i < capEvents && i < ev.size(); i++) events[i] = ev[i];
    for (uint32_t i = 0; i < capTransforms && i < tr.size(); i++) std::memcpy(transforms + 16 * (size_t)i, tr[i].m, 64);
    for (uint32_t i = 0; i < capFixes && i < fx.size(); i++) fixes[i] = fx[i];
    BF_CATCH
}
int bf_recon_op_log(bf_recon* r, BFFixOp* out, uint32_t cap, uint32_t* n) {
    BF_TRY
    BF_REQUIRE(r && n && (out || cap == 0), BF_ERR_ARG, "null argument");
    const auto& log = r->r->opLog();
    *n = (uint32_t)log.size();
    for (uint32_t i = 0; i < cap && i < log.size(); i++) out[i] = log[i];
    BF_CATCH
}

// ---- the FriedLiver application ---------------------------------------------------------------
struct bf_app {
    App* a = nullptr;
    bf_recon recon;  // borrowed view of the app's loop
};

int bf_app_create(const char* appParams, const char* bundlingParams, const BFAppOptions* o, bf_app** out) {
    BF_TRY
    BF_REQUIRE(appParams && bundlingParams && out, BF_ERR_ARG, "null argument");
    *out = nullptr;
    BFAppOptions def{};
    def.asyncBundling = 1;
    std::unique_ptr<bf_app> h(new bf_app);
    h->a = new App(appParams, bundlingParams, o ? *o : def);
    h->recon.r = &h->a->recon();
    *out = h.release();
    BF_CATCH
}
int bf_app_destroy(bf_app* a) {
    BF_TRY
    if (a) {
        delete a->a;
        delete a;
    }
    BF_CATCH
}
int bf_app_info(const bf_app* a, BFAppInfo* out) {
    BF_TRY
    BF_REQUIRE(a && out, BF_ERR_ARG, "null argument");
    *out = a->a->info();
    BF_CATCH
}
int bf_app_step(bf_app* a, int* gotFrame) {
    BF_TRY
    BF_REQUIRE(a, BF_ERR_ARG, "null app");
    const bool got = a->a->step();
    if (gotFrame) *gotFrame = got ? 1 : 0;
    BF_CATCH
}
int bf_app_finish(bf_app* a, BFAppResult* out) {
    BF_TRY
    BF_REQUIRE(a, BF_ERR_ARG, "null app");
    const BFAppResult r = a->a->finish();
    if (out) *out = r;
    BF_CATCH
}
int bf_app_run(bf_app* a, BFAppResult* out) {
    BF_TRY
    BF_REQUIRE(a, BF_ERR_ARG, "null app");
    const BFAppResult r = a->a->run();
    if (out) *out = r;
    BF_CATCH
}
int bf_app_recon(bf_app* a, bf_recon** out) {
    BF_TRY
    BF_REQUIRE(a && out, BF_ERR_ARG, "null argument");
    *out = &a->recon;
    BF_CATCH
}
int bf_front_end_tinc(const float prev[16], const float cur[16], uint32_t frame, uint32_t seed, float driftRad, float driftM,
                      float Tinc[16]) {
    BF_TRY
    BF_REQUIRE(prev && cur && Tinc, BF_ERR_ARG, "null argument");
    const BFMat4 T = front_end_tinc(prev, cur, frame, seed, driftRad, driftM);
    std::memcpy(Tinc, T.m, 64);
    BF_CATCH
}
int bf_app_resolve(const char* appParams, const char* bundlingParams, const BFAppOptions* o, BFAppInfo* info,
                   BFReconOptions* loop) {
    BF_TRY
    BF_REQUIRE(appParams && bundlingParams && info, BF_ERR_ARG, "null argument");
    BFAppOptions opt{};
    if (o) opt = *o;
    const AppConfig c = load_app_config(appParams, bundlingParams, opt);
    *info = c.info;
    if (loop) *loop = c.ro;
    BF_CATCH
}
int bf_app_timing(const bf_app* a, BFAppTiming* out) {
    BF_TRY
    BF_REQUIRE(a && out, BF_ERR_ARG, "null argument");
    *out = a->a->timing();
    BF_CATCH
}
int bf_app_front_end_pose(const bf_app* a, uint32_t f, float Tinc[16]) {
    BF_TRY
    BF_REQUIRE(a && Tinc, BF_ERR_ARG, "null argument");
    const BFMat4 T = a->a->frontEndPose(f);
    std::memcpy(Tinc, T.m, 64);
    BF_CATCH
}

// ---- re-integration queue (host) ----------------------------------------------------------
struct bf_traj {
    TrajectoryManager* tm = nullptr;
    std::vector<FixOp> ops;
};

int bf_traj_create(uint32_t maxFrames, uint32_t topNActive, float minPoseDistSqrt, bf_traj** out) {
    BF_TRY
    BF_REQUIRE(out && maxFrames > 0, BF_ERR_ARG, "bad argument");
    bf_traj* t = new bf_traj();
    t->tm = new TrajectoryManager(maxFrames, topNActive ? topNActive : 30u, minPoseDistSqrt);
    *out = t;
    BF_CATCH
}
int bf_traj_destroy(bf_traj* t) {
    BF_TRY
    if (t) {
        delete t->tm;
        delete t;
    }
    BF_CATCH
}
int bf_traj_add_frame(bf_traj* t, int32_t type, const float T[16], uint32_t idx) {
    BF_TRY
    BF_REQUIRE(t, BF_ERR_ARG, "null traj");
    BF_REQUIRE(type == 0 || type == 1, BF_ERR_ARG, "type must be Integrated (0) or NotIntegrated_NoTransform (1)");
    BFMat4 m;
    if (type == 0) {
        BF_REQUIRE(T, BF_ERR_ARG, "null transform");
        m = to_mat(T);
    } else {
        for (float& v : m.m) v = -std::numeric_limits<float>::infinity();
    }
    t->tm->addFrame((FrameType)type, m, idx);
    BF_CATCH
}
int bf_traj_update_optimized(bf_traj* t, const float* T, uint32_t numFrames) {
    BF_TRY
    BF_REQUIRE(t && (T || numFrames == 0), BF_ERR_ARG, "null argument");
    t->tm->updateOptimizedTransforms(reinterpret_cast<const BFMat4*>(T), numFrames);
    BF_CATCH
}
int bf_traj_next_fixes(bf_traj* t, uint32_t maxFixes, BFFixOp* ops, uint32_t* n) {
    BF_TRY
    BF_REQUIRE(t && n && (ops || maxFixes == 0), BF_ERR_ARG, "null argument");
    *n = t->tm->nextFixes(maxFixes, t->ops);
    for (uint32_t i = 0; i < *n; i++) {
        ops[i].kind = (int32_t)t->ops[i].kind;
        ops[i].frame = t->ops[i].frame;
        std::memcpy(ops[i].oldT, t->ops[i].oldT.m, 64);
        std::memcpy(ops[i].newT, t->ops[i].newT.m, 64);
    }
    BF_CATCH
}
int bf_traj_frame_info(bf_traj* t, uint32_t idx, int32_t* type, float* dist) {
    BF_TRY
    BF_REQUIRE(t, BF_ERR_ARG, "null traj");
    if (type) *type = (int32_t)t->tm->type(idx);
    if (dist) *dist = t->tm->dist(idx);
    BF_CATCH
}
int bf_pose_helper_matrix_to_pose(const float T[16], float out[6]) {
    BF_TRY
    BF_REQUIRE(T && out, BF_ERR_ARG, "null argument");
    pose_helper_matrix_to_pose(to_mat(T), out);
    BF_CATCH
}


// ---- input formats and preprocessing ------------------------------------------------------------
// ---- correspondences --------------------------------------------------------------------------------
int bf_corr_save(const char* path, const BFEntryJ* corr, uint64_t n) {
    BF_TRY
    BF_REQUIRE(path, BF_ERR_ARG, "null path");
    corr_save(path, corr, n);
    BF_CATCH
}
int bf_corr_load(const char* path, BFEntryJ* corr, uint64_t cap, uint64_t* n) {
    BF_TRY
    BF_REQUIRE(path, BF_ERR_ARG, "null path");
    const uint64_t c = corr_load(path, corr, cap);
    if (n) *n = c;
    BF_CATCH
}
int bf_corr_from_depth(const float* const* depth, const float* transforms, const float* transformsInv, uint32_t curFrame,
                       uint32_t startFrame, const BFCorrOptions* o, BFEntryJ* out, uint32_t cap, uint32_t* n,
                       uint32_t* total) {
    BF_TRY
    BF_REQUIRE(o && n, BF_ERR_ARG, "null argument");
    *n = corr_from_depth(depth, transforms, transformsInv, curFrame, startFrame, *o, out, cap, total);
    BF_CATCH
}

// ---- CUDACache ---------------------------------------------------------------------------------
int bf_cache_create(const BFCacheOptions* o, bf_cache** out) {
    BF_TRY
    BF_REQUIRE(o && out, BF_ERR_ARG, "null argument");
    *out = nullptr;
    CacheConfig cfg{};
    cfg.inputWidth = o->inputWidth; cfg.inputHeight = o->inputHeight;
    cfg.width = o->width; cfg.height = o->height; cfg.maxFrames = o->maxFrames;
    std::memcpy(cfg.inputIntrinsics, o->inputIntrinsics, 64);
    cfg.colorSigma = o->colorSigma; cfg.depthSigmaD = o->depthSigmaD; cfg.depthSigmaR = o->depthSigmaR;
    std::unique_ptr<bf_cache> h(new bf_cache);
    BF_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    try {
        h->c = new Cache(cfg, h->stream);
    } catch (...) {
        (void)hipStreamDestroy(h->stream);
        throw;
    }
    *out = h.release();
    BF_CATCH
}
int bf_cache_destroy(bf_cache* c) {
    BF_TRY
    if (!c) return 0;
    (void)hipStreamSynchronize(c->stream);
    delete c->c;
    (void)hipStreamDestroy(c->stream);
    delete c;
    BF_CATCH
}
int bf_cache_store_frame(bf_cache* c, const float* depth, const uint8_t* color, uint32_t colorW, uint32_t colorH,
                         uint32_t* index) {
    BF_TRY
    BF_REQUIRE(c, BF_ERR_ARG, "null cache");
    const uint32_t i = c->c->storeFrame(depth, color, colorW, colorH);
    if (index) *index = i;
    BF_CATCH
}
int bf_cache_copy_frame_from(bf_cache* dst, const bf_cache* src, uint32_t frame, uint32_t* index) {
    BF_TRY
    BF_REQUIRE(dst && src, BF_ERR_ARG, "null cache");
    if (src->stream != dst->stream) BF_HIP(hipStreamSynchronize(src->stream));
    const uint32_t i = dst->c->copyFrameFrom(*src->c, frame);
    if (index) *index = i;
    BF_CATCH
}
int bf_cache_increment(bf_cache* c) {
    BF_TRY
    BF_REQUIRE(c, BF_ERR_ARG, "null cache");
    c->c->increment();
    BF_CATCH
}
int bf_cache_num_frames(bf_cache* c, uint32_t* n) {
    BF_TRY
    BF_REQUIRE(c && n, BF_ERR_ARG, "null argument");
    *n = c->c->numFrames();
    BF_CATCH
}
int bf_cache_frame(bf_cache* c, uint32_t index, BFCachedFrame* out) {
    BF_TRY
    BF_REQUIRE(c && out, BF_ERR_ARG, "null argument");
    *out = c->c->frame(index);
    BF_CATCH
}
int bf_cache_intrinsics(bf_cache* c, float K[16], float Kinv[16]) {
    BF_TRY
    BF_REQUIRE(c, BF_ERR_ARG, "null cache");
    if (K) std::memcpy(K, c->c->intrinsics(), 64);
    if (Kinv) std::memcpy(Kinv, c->c->intrinsicsInv(), 64);
    BF_CATCH
}
int bf_cache_synchronize(bf_cache* c) {
    BF_TRY
    BF_REQUIRE(c, BF_ERR_ARG, "null cache");
    BF_HIP(hipStreamSynchronize(c->stream));
    BF_CATCH
}

int bf_mesh_merge(const BFMcTriangle* tris, uint32_t n, const float transform[16], float* vertices, float* colors,
                  uint32_t* faces, uint32_t* numVertices, uint32_t* numFaces) {
    BF_TRY
    BF_REQUIRE(tris || n == 0, BF_ERR_ARG, "null triangles");
    const Mesh m = mesh_from_triangles(tris, n, transform);
    if (vertices) std::memcpy(vertices, m.vertices.data(), 4 * m.vertices.size());
    if (colors) std::memcpy(colors, m.colors.data(), 4 * m.colors.size());
    if (faces) std::memcpy(faces, m.faces.data(), 4 * m.faces.size());
    if (numVertices) *numVertices = (uint32_t)(m.vertices.size() / 3);
    if (numFaces) *numFaces = (uint32_t)(m.faces.size() / 3);
    BF_CATCH
}
int bf_mesh_save_ply(const char* path, const BFMcTriangle* tris, uint32_t n, const float transform[16],
                     uint32_t* numVertices, uint32_t* numFaces) {
    BF_TRY
    BF_REQUIRE(path && (tris || n == 0), BF_ERR_ARG, "null argument");
    const Mesh m = mesh_from_triangles(tris, n, transform);
    mesh_save_ply(path, m);
    if (numVertices) *numVertices = (uint32_t)(m.vertices.size() / 3);
    if (numFaces) *numFaces = (uint32_t)(m.faces.size() / 3);
    BF_CATCH
}

int bf_sens_open(const char* path, bf_sens** out) {
    BF_TRY
    BF_REQUIRE(path && out, BF_ERR_ARG, "null argument");
    *out = nullptr;
    std::unique_ptr<SensReader> r(new SensReader(path));
    *out = new bf_sens{r.release()};
    BF_CATCH
}
int bf_sens_close(bf_sens* s) {
    BF_TRY
    if (s) {
        delete s->r;
        delete s;
    }
    BF_CATCH
}
int bf_sens_info(const bf_sens* s, BFSensInfo* out) {
    BF_TRY
    BF_REQUIRE(s && out, BF_ERR_ARG, "null argument");
    *out = s->r->info();
    BF_CATCH
}
int bf_sens_frame_pose(const bf_sens* s, uint64_t frame, float camToWorld[16]) {
    BF_TRY
    BF_REQUIRE(s && camToWorld, BF_ERR_ARG, "null argument");
    s->r->pose(frame, camToWorld);
    BF_CATCH
}
int bf_sens_frame_timestamps(const bf_sens* s, uint64_t frame, uint64_t* tsColor, uint64_t* tsDepth) {
    BF_TRY
    BF_REQUIRE(s, BF_ERR_ARG, "null argument");
    s->r->timestamps(frame, tsColor, tsDepth);
    BF_CATCH
}
int bf_sens_read_depth_u16(bf_sens* s, uint64_t frame, uint16_t* out) {
    BF_TRY
    BF_REQUIRE(s && out, BF_ERR_ARG, "null argument");
    s->r->depthU16(frame, out);
    BF_CATCH
}
int bf_sens_read_depth(bf_sens* s, uint64_t frame, float* out) {
    BF_TRY
    BF_REQUIRE(s && out, BF_ERR_ARG, "null argument");
    const BFSensInfo& in = s->r->info();
    const size_t n = (size_t)in.depthWidth * in.depthHeight;
    std::vector<uint16_t> d(n);
    s->r->depthU16(frame, d.data());
    for (size_t i = 0; i < n; i++)  // SensorDataReader.cpp:104-107
        out[i] = d[i] == 0 ? -std::numeric_limits<float>::infinity() : (float)d[i] / in.depthShift;
    BF_CATCH
}
int bf_sens_read_color(bf_sens* s, uint64_t frame, uint8_t* rgbx) {
    BF_TRY
    BF_REQUIRE(s && rgbx, BF_ERR_ARG, "null argument");
    s->r->colorRGBX(frame, rgbx);
    BF_CATCH
}
int bf_image_decode(const uint8_t* data, uint64_t n, int compression, uint32_t* width, uint32_t* height, uint8_t* rgbx,
                    uint64_t cap) {
    BF_TRY
    BF_REQUIRE(data && width && height, BF_ERR_ARG, "null argument");
    BF_REQUIRE(compression == 1 || compression == 2, BF_ERR_ARG, "compression must be 1 (PNG) or 2 (JPEG)");
    const DecodedImage img = compression == 2 ? jpeg_decode(data, n) : png_decode(data, n);
    *width = img.width;
    *height = img.height;
    if (rgbx) {
        BF_REQUIRE(cap >= img.rgbx.size(), BF_ERR_CAPACITY, "output buffer too small");
        std::memcpy(rgbx, img.rgbx.data(), img.rgbx.size());
    }
    BF_CATCH
}
int bf_sens_writer_create(const char* path, const BFSensInfo* info, bf_sens_writer** out) {
    BF_TRY
    BF_REQUIRE(path && info && out, BF_ERR_ARG, "null argument");
    *out = nullptr;
    std::unique_ptr<SensWriter> w(new SensWriter(path, *info));
    *out = new bf_sens_writer{w.release()};
    BF_CATCH
}
int bf_sens_writer_add_frame(bf_sens_writer* w, const float camToWorld[16], uint64_t tsColor, uint64_t tsDepth,
                             const uint16_t* depth, const uint8_t* rgbx) {
    BF_TRY
    BF_REQUIRE(w && camToWorld && depth, BF_ERR_ARG, "null argument");
    w->w->addFrame(camToWorld, tsColor, tsDepth, depth, rgbx);
    BF_CATCH
}
int bf_sens_save_trajectory(const char* in, const char* out, const float* T, uint64_t n) {
    BF_TRY
    BF_REQUIRE(in && out && (T || n == 0), BF_ERR_ARG, "null argument");
    sens_save_with_trajectory(in, out, reinterpret_cast<const BFMat4*>(T), n);
    BF_CATCH
}
int bf_sens_writer_add_compressed_frame(bf_sens_writer* w, const float camToWorld[16], uint64_t tsColor, uint64_t tsDepth,
                                        const uint8_t* color, uint64_t colorBytes, const uint8_t* depth, uint64_t depthBytes) {
    BF_TRY
    BF_REQUIRE(w && camToWorld, BF_ERR_ARG, "null argument");
    w->w->addCompressedFrame(camToWorld, tsColor, tsDepth, color, colorBytes, depth, depthBytes);
    BF_CATCH
}
int bf_sens_writer_close(bf_sens_writer* w) {
    BF_TRY
    if (w) {
        std::unique_ptr<SensWriter> owned(w->w);
        delete w;
        owned->close();
    }
    BF_CATCH
}

int bf_params_create(bf_params** out) {
    BF_TRY
    BF_REQUIRE(out, BF_ERR_ARG, "null argument");
    *out = new bf_params;
    BF_CATCH
}
int bf_params_load(bf_params* p, const char* path) {
    BF_TRY
    BF_REQUIRE(p && path, BF_ERR_ARG, "null argument");
    p->f.load(path);
    BF_CATCH
}
int bf_params_destroy(bf_params* p) {
    BF_TRY
    delete p;
    BF_CATCH
}
int bf_params_has(const bf_params* p, const char* key, int* found) {
    BF_TRY
    BF_REQUIRE(p && key && found, BF_ERR_ARG, "null argument");
    *found = p->f.has(key) ? 1 : 0;
    BF_CATCH
}
int bf_params_get_string(const bf_params* p, const char* key, char* buf, size_t cap) {
    BF_TRY
    BF_REQUIRE(p && key && buf && cap, BF_ERR_ARG, "null argument");
    const std::string v = p->f.str(key);
    BF_REQUIRE(v.size() < cap, BF_ERR_CAPACITY, "buffer too small for " + std::string(key));
    std::memcpy(buf, v.c_str(), v.size() + 1);
    BF_CATCH
}
int bf_params_get_floats(const bf_params* p, const char* key, float* out, uint32_t cap, uint32_t* count) {
    BF_TRY
    BF_REQUIRE(p && key, BF_ERR_ARG, "null argument");
    const std::vector<float> v = p->f.floats(key);
    if (count) *count = (uint32_t)v.size();
    for (size_t i = 0; i < v.size() && i < cap && out; i++) out[i] = v[i];
    BF_CATCH
}
int bf_params_get_number(const bf_params* p, const char* key, double* out) {
    BF_TRY
    BF_REQUIRE(p && key && out, BF_ERR_ARG, "null argument");
    *out = p->f.number(key);
    BF_CATCH
}
int bf_params_get_bool(const bf_params* p, const char* key, int* out) {
    BF_TRY
    BF_REQUIRE(p && key && out, BF_ERR_ARG, "null argument");
    *out = p->f.boolean(key) ? 1 : 0;
    BF_CATCH
}
int bf_params_hash_params(const bf_params* p, BFHashParams* o) {
    BF_TRY
    BF_REQUIRE(p && o, BF_ERR_ARG, "null argument");
    *o = hash_params_from(p->f);
    BF_CATCH
}
int bf_params_raycast_params(const bf_params* p, float fx, float fy, float mx, float my, BFRayCastParams* o) {
    BF_TRY
    BF_REQUIRE(p && o, BF_ERR_ARG, "null argument");
    *o = raycast_params_from(p->f, fx, fy, mx, my);
    BF_CATCH
}
int bf_params_preprocess_options(const bf_params* p, float depthShift, BFPreprocessOptions* o) {
    BF_TRY
    BF_REQUIRE(p && o, BF_ERR_ARG, "null argument");
    *o = preprocess_options_from(p->f, depthShift);
    BF_CATCH
}

int bf_preproc_create(uint32_t depthW, uint32_t depthH, uint32_t colorW, uint32_t colorH, uint32_t integrationW,
                      uint32_t integrationH, const BFPreprocessOptions* opt, bf_preproc** out) {
    BF_TRY
    BF_REQUIRE(opt && out, BF_ERR_ARG, "null argument");
    *out = nullptr;
    std::unique_ptr<bf_preproc> h(new bf_preproc);
    // the input work is on the frame loop's critical path (the scene stream's next batch waits for it):
    // its kernels take free slots ahead of the voxel pass's next round and of the bundling launches
    int prLeast = 0, prGreatest = 0;
    BF_HIP(hipDeviceGetStreamPriorityRange(&prLeast, &prGreatest));
    BF_HIP(hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, prGreatest));
    h->p = new Preproc(depthW, depthH, colorW, colorH, integrationW, integrationH, *opt, h->stream);
    *out = h.release();
    BF_CATCH
}
int bf_preproc_destroy(bf_preproc* p) {
    BF_TRY
    if (p) {
        delete p->p;
        if (p->stream) (void)hipStreamDestroy(p->stream);
        delete p;
    }
    BF_CATCH
}
int bf_preproc_run(bf_preproc* p, const uint16_t* depthU16, const uint8_t* rgbx, float* depthOut, uint8_t* colorOut) {
    BF_TRY
    BF_REQUIRE(p && depthU16 && depthOut, BF_ERR_ARG, "null argument");
    p->p->run(depthU16, rgbx, depthOut, colorOut);
    BF_CATCH
}
int bf_preproc_synchronize(bf_preproc* p) {
    BF_TRY
    BF_REQUIRE(p, BF_ERR_ARG, "null argument");
    BF_HIP(hipStreamSynchronize(p->stream));
    BF_CATCH
}
int bf_preproc_stream(bf_preproc* p, void** stream) {
    BF_TRY
    BF_REQUIRE(p && stream, BF_ERR_ARG, "null argument");
    *stream = static_cast<void*>(p->stream);
    BF_CATCH
}

}  // extern "C"
