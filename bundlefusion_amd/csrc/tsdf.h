// tsdf.h — MI355X voxel-hash TSDF scene (replaces CUDASceneRepHashSDF,
// Source/DepthSensing/CUDASceneRepHashSDF.h:29-423).
//
// Device layout (one allocation per array, all resident in HBM):
//   hash      BFHashEntry[E]      reference layout; E = 4 * numBuckets
//   heap      uint32[B]           free-block stack, reference semantics (VoxelUtilHashSDF.h:535-546)
//   voxels    BFVoxel[B * 512]    12-B AoS voxels, one 6 KiB run per block
//   blockPos  int4[B]             per heap block: {x, y, z, allocated} — lets compactify stream
//                                 only the allocated pool prefix instead of the whole hash table
//   visible   int4[B]             compacted frustum list {x, y, z, ptr} (16 B vs 32 B HashEntry);
//                                 GC walks this list, as the reference walks d_hashCompactified
//   band      int4[24 B]          (op batches: one bin of B entries per op count) the subset of `visible` whose voxels can reach the truncation band
//                                 of the current depth map (conservative cull against per-8x8-tile
//                                 depth bounds) — the list integrate walks
//   tiles     float2[tiles]       per-8x8-pixel-tile min/max of the valid depths of the current op(s)
//   tiles2    float2[tiles2]      the same per 32x32 pixels (footprints wider than 2x2 tiles)
//   ctrl      uint32[16]          device-resident counters (heap counter, visible count, ...)
//   cand/candSet/candSlot/ovf     alloc scratch (per-op candidate list, global dedup set)
//   victims                       GC scratch
// No host round trip inside integrate / de-integrate / GC: every count a kernel needs is
// read from `ctrl` on the device.
#pragma once
#include "bf_math.h"
#include "bf_runtime.h"

namespace bf {

enum Ctrl {
    C_HEAP = 0,        // heap counter (points at the last free block)
    C_VISIBLE = 1,     // numOccupiedBlocks of the last compactify
    C_CAND = 2,        // alloc candidates emitted
    C_OVF = 3,         // candidates whose bucket was full (collision-list path)
    C_HIGHWATER = 4,   // 1 + highest heap block index ever handed out
    C_CANDPEAK = 5,    // largest alloc candidate count of one integrate / batch since the reset (may exceed the capacity)
    C_GC_LIST = 6,     // GC victims that touch a collision list (serial path)
    C_ERR = 7,         // error bits (1: candidate buffer overflow, 2: heap exhausted, 4: dedup set full)
    C_BAND = 8,        // blocks of the visible list that may hold a voxel inside the truncation band
    C_TICKET = 9,      // last-workgroup ticket of k_alloc_insert (self-resetting)
    C_TICKET_GC = 10,  // last-workgroup ticket of k_gc (self-resetting)
    C_OPBIN = 16,      // op batches: work-list entries per op count (1..kMaxOps -> slots 16..39)
    C_COUNT = 48
};

struct SceneConfig {
    BFHashParams hp;
    uint32_t candCapacity;   // max alloc candidates per integrate
    uint32_t shardCount;     // >1: spatial ownership sharding across GPUs
    uint32_t shardIndex;
    float shardChunk;        // ownership chunk edge in metres (default 1 m, the streaming chunk)
    uint32_t allocForceDirect = 0;  // test switch (BF_SCENE_TEST_ALLOC_DIRECT): every walking tile also takes the alloc walk's congested path
    uint32_t applyXcdRun = 0;       // voxel pass: work-list positions per XCD run (0: 64)
    uint32_t applyRounds = 0;       // voxel pass: rounds of resident workgroups (0: kApplyRounds)
    uint32_t splatRowCap = 0;       // test switch: ray-interval splat row-list capacity (0: 4 per heap block)
};
}  // namespace bf
struct BFSceneOptions;  // include/bf/bf.h
namespace bf {
// the scene configuration of a BFSceneOptions (NULL: defaults)
SceneConfig scene_config(const BFHashParams& hp, const BFSceneOptions* so);

// One voxel op of a batch: integrate (deint = false) or de-integrate one frame at pose T (camera ->
// world); depth / color are device pointers (float / uchar4 per pixel).
struct VoxelOp {
    BFMat4 T;
    const float* depth;
    const uint8_t* color;
    bool deint;
    // optional per-depth-map cache of the band-cull depth tiles (Scene::tileCount(cam) float2: fine
    // level, then coarse) and of the interleaved {depth bits, colour} image (Scene::dcCount(cam) uint2, the voxel
    // pass's gather source); both computed by the batch unless tilesReady (they depend on the frame only)
    float2* tiles = nullptr;
    uint2* dc = nullptr;
    bool tilesReady = false;
};

class Scene {
public:
    // render counters (raycast.hip): kRenderStatSlots slots of kRenderStatFields, summed by renderStats()
    static constexpr int kRenderStatSlots = 64, kRenderStatFields = 16;
    // a frame's fixes (<= 10 re-integrations, 2 voxel ops each) + the deferred integration of the
    // previous frame; <= 32 (op bit masks)
    static constexpr uint32_t kMaxOps = 24;
    Scene(const SceneConfig& cfg, hipStream_t stream);
    ~Scene();

    void reset();
    // integrate (deint=false) / de-integrate (deint=true) one frame; depth/color are device
    // pointers (float / uchar4 per pixel, W*H of cam). T is camera->world.
    void integrate(const BFMat4& T, const float* depth, const uint8_t* color, const BFDepthCameraParams& cam,
                   bool deint, const uint32_t* bitMask);
    // re-integration of one frame: de-integrate with Told then integrate with Tnew as a two-op
    // applyOps batch (identical voxel results to the two calls)
    void reintegrate(const BFMat4& Told, const BFMat4& Tnew, const float* depth, const uint8_t* color,
                     const BFDepthCameraParams& cam);
    // a sequence of integrate / de-integrate ops (reintegrate(), DepthSensing.cpp:854-902) as ONE
    // voxel pass: alloc for every integrate op, one compactify scan with a per-block op mask, and
    // a kernel that applies the ops to each voxel in sequence order (one read, one write). Voxel
    // values equal the sequential calls; `visible` is the frustum list of the last op, as the
    // reference's garbageCollect after the loop sees it.
    void applyOps(const VoxelOp* ops, uint32_t n, const BFDepthCameraParams& cam);
    static size_t tileCount(const BFDepthCameraParams& cam);  // float2 per depth map of a VoxelOp tile cache
    static size_t dcCount(const BFDepthCameraParams& cam);    // uint2 per depth map of a VoxelOp dc image
    KernelClock& applyClock() { return applyClock_; }  // k_apply_ops launches
    void garbageCollect();
    void compactify(const BFMat4& T, const BFDepthCameraParams& cam);

    // synchronous queries (tests, debug)
    uint32_t heapFreeCount();
    uint32_t numVisible();
    uint32_t errorFlags();
    // capacity state (BFSceneCapacity): sticky error bits, peak candidates against the capacity, heap; synchronizes
    BFSceneCapacity capacity();
    // the error bits as of the last garbageCollect, mirrored by k_gc into pinned host memory (no synchronization;
    // enableErrorMirror first): the loop checks them once per frame without waiting for the scene stream
    void enableErrorMirror();
    uint32_t mirroredErrorFlags() const { return errMirror_ ? __atomic_load_n(errMirror_, __ATOMIC_ACQUIRE) : 0u; }
    BFTsdfStats stats();
    void resetStats();
    void exportState(BFHashEntry* hash, uint32_t* heap, uint32_t* heapCounter, BFVoxel* voxels);
    uint32_t exportVisible(int4* out, uint32_t cap);
    void exportBlockVoxels(uint32_t first, uint32_t count, BFVoxel* out);
    uint32_t exportBlocks(int4* out, uint32_t cap);  // blockPos[0, highWater): {x, y, z, allocated}

    const SceneConfig& config() const { return cfg_; }
    hipStream_t stream() const { return stream_; }
    void setStream(hipStream_t s) { stream_ = s; }
    // raw device views for the raycaster / stream runner
    const BFHashEntry* dHash() const { return hash_.p; }
    const BFVoxel* dVoxels() const { return voxels_.p; }
    const int4* dVisible() const { return visible_.p; }
    const uint32_t* dCtrl() const { return ctrl_.p; }
    uint32_t* dCtrlMut() { return ctrl_.p; }
    size_t deviceBytes() const;
    KernelClock& integrateClock() { return integrateClock_; }  // k_integrate launches (bench roofline)

    // CUDARayCastSDF::render (CUDARayCastSDF.cpp:38-72) after setLastRigidTransformAndCompactify:
    // frustum compactify for camera T (cam = depth-camera frustum params), ray-interval splat
    // (min / max target), renderKernel, computeNormals (unless rp.useGradients). Outputs are
    // device arrays of rp.width * rp.height: depth f32, depth4 / normals / colors float4.
    // rayMin / rayMax (optional, device f32) receive the splatted intervals.
    void raycast(const BFMat4& T, const BFDepthCameraParams& cam, const BFRayCastParams& rp, float* depth, float4* depth4,
                 float4* normals, float4* colors, float* rayMin, float* rayMax);
    KernelClock& renderClock() { return renderClock_; }
    // accumulated ray-cast counters (BFRenderStats order after launches / kernelMs): trilinear samples,
    // voxel loads, hash probes, marched rays, splatted blocks, splat atomics, renders, pixels
    void renderStats(BFRenderStats& out);
    // CUDAMarchingCubesHashSDF::extractIsoSurface (CUDAMarchingCubesHashSDF.cpp:107-118) over every
    // allocated block: writes min(total, cap) triangles to the device array out in (heap block,
    // voxel, case-table) order, returns that count; *total = triangles before the cap. Synchronizes.
    uint32_t extractMesh(const BFMarchingCubesParams& p, BFMcTriangle* out, uint32_t cap, uint32_t* total);

private:
    void alloc(const float* depth, const BFDepthCameraParams& cam, const uint32_t* bitMask);
    void beginOp();

    SceneConfig cfg_;
    hipStream_t stream_;
    uint32_t E_, B_;
    BFMat4 T_, Tinv_;

    DevBuf<BFHashEntry> hash_;
    DevBuf<uint32_t> heap_;
    DevBuf<BFVoxel> voxels_;
    uint64_t hostPixels_ = 0;  // BFTsdfStats.pixels: W x H per alloc walk, counted at launch
    DevBuf<int4> blockPos_;
    DevBuf<int4> visible_;
    DevBuf<int4> band_;
    DevBuf<float2> tiles_;
    size_t tilesCap_ = 0;
    DevBuf<float2> tiles2_;  // 32x32-pixel depth bounds
    size_t tiles2Cap_ = 0;
    void ensureTiles(size_t fine, size_t coarse);
    DevBuf<uint2> dc_;  // per-op {depth, colour} images of ops without a caller cache
    size_t dcCap_ = 0;
    DevBuf<uint32_t> ctrl_;
    DevBuf<unsigned long long> stats_;  // [64 slots][16]
    DevBuf<unsigned long long> cand_;
    DevBuf<unsigned long long> candSet_;
    DevBuf<int> candSlot_;
    DevBuf<unsigned long long> ovf_;
    DevBuf<unsigned long long> gcList_;
    DevBuf<uint32_t> blockCount_;
    uint32_t* errMirror_ = nullptr;  // pinned host word written by k_gc (enableErrorMirror)
    uint32_t candSetMask_;
    int numCUs_;
    unsigned integrateGrid_[2] = {0, 0};
    KernelClock integrateClock_;
    KernelClock renderClock_, splatClock_;
    DevBuf<unsigned long long> renderStats_;
    DevBuf<uint4> blockMask_;  // per work-list entry of an op batch: which ops may update each z-half (uint2) / quarter
    DevBuf<uint32_t> blockBirth_;  // per heap block: epoch << 8 | (255 - first op) of the batch that allocated it
    DevBuf<uint8_t> candOp_;       // per alloc candidate of a batch: the integrate op that emitted it
    uint32_t batchEpoch_ = 0;
    KernelClock applyClock_;
    unsigned applyGrid_ = 0, compactifyGrid_ = 0;
    int applyXcdShift_ = 6;   // log2 of the voxel pass's work-list run per XCD (BFSceneOptions.applyXcdRun)
    DevBuf<uint32_t> splatMin_, splatMax_;  // ordered-int float targets of the interval splat
    size_t splatCap_ = 0;
    DevBuf<int4> splatQuads_;
    DevBuf<uint32_t> splatBin_, splatRowIdx_;  // the splat's tile-row lists (raycast.hip)
    DevBuf<unsigned long long> waveLog_, tileLog_;  // diagnostics build (BF_RENDER_DIAG): per-wave / per-tile clocks (raycast.hip)
};

}  // namespace bf
