// oracle/tsdf.cpp — TEST INFRASTRUCTURE (CPU oracle, see oracle.h header).
//
// Serial CPU restatement of the reference voxel-hash scene: every reference kernel is
// executed as if its threads ran one after another (a legal schedule of the racy
// reference: with one thread at a time every try-lock succeeds and the host alloc
// loop of CUDASceneRepHashSDF.h:335-348 converges after one effective pass).
// Citations are to /root/reference/FriedLiver/Source/DepthSensing/.
#include "oracle.h"
#include "or_math.h"
#include "../bundlefusion_amd/csrc/mc_tables.h"  // case tables (data; checked by tests/test_mc.py)

#include <algorithm>
#include <cstring>
#include <limits>
#include <vector>

using namespace orc;

namespace {

const float MINF = -std::numeric_limits<float>::infinity();
const float PINF = std::numeric_limits<float>::infinity();

struct Scene {
    BFHashParams hp;
    std::vector<BFHashEntry> hash;      // d_hash
    std::vector<BFHashEntry> compact;   // d_hashCompactified (first numOccupied valid)
    std::vector<uint32_t> heap;         // d_heap
    uint32_t heapCounter;               // d_heapCounter
    std::vector<BFVoxel> voxels;        // d_SDFBlocks
    std::vector<int> mutex;             // d_hashBucketMutex
    std::vector<int> decision;          // d_hashDecision (GC)
    uint32_t numOccupied;
    m4 T, Tinv;
    BFDepthCameraParams cam;
    BFTsdfStats stats;
    // multi-GPU TSDF shard (or_scene_set_shard): alloc keeps only the blocks whose chunk this shard owns
    uint32_t shardCount = 1, shardIndex = 0;
    float shardChunk = 1.0f;
};

m4 toM4(const float* p) { m4 m; std::memcpy(m.e, p, 64); return m; }

// ---- VoxelUtilHashSDF.h restatements ---------------------------------------

// computeHashPos, VoxelUtilHashSDF.h:225-234 (wrapping int32 multiplies)
uint32_t hashPos(const Scene& s, i3 p) {
    int32_t a = (int32_t)((uint32_t)p.x * 73856093u);
    int32_t b = (int32_t)((uint32_t)p.y * 19349669u);
    int32_t c = (int32_t)((uint32_t)p.z * 83492791u);
    int res = (a ^ b ^ c) % (int)s.hp.hashNumBuckets;
    if (res < 0) res += (int)s.hp.hashNumBuckets;
    return (uint32_t)res;
}

float truncation(const Scene& s, float z) { return s.hp.truncation + s.hp.truncScale * z; }  // :272-274

// worldToVirtualVoxelPos :283-287 (round half away from zero via sign)
i3 worldToVirtualVoxelPos(const Scene& s, f3 pos) {
    f3 p = pos / s.hp.virtualVoxelSize;
    f3 sg = mk((float)sgn(p.x), (float)sgn(p.y), (float)sgn(p.z));
    f3 q = p + sg * 0.5f;
    return {f2i(q.x), f2i(q.y), f2i(q.z)};
}
// virtualVoxelPosToSDFBlock :290-299
i3 virtualVoxelPosToSDFBlock(i3 v) {
    if (v.x < 0) v.x -= BF_SDF_BLOCK_SIZE - 1;
    if (v.y < 0) v.y -= BF_SDF_BLOCK_SIZE - 1;
    if (v.z < 0) v.z -= BF_SDF_BLOCK_SIZE - 1;
    return {v.x / BF_SDF_BLOCK_SIZE, v.y / BF_SDF_BLOCK_SIZE, v.z / BF_SDF_BLOCK_SIZE};
}
f3 virtualVoxelPosToWorld(const Scene& s, i3 p) {  // :308-310
    return mk((float)p.x, (float)p.y, (float)p.z) * s.hp.virtualVoxelSize;
}
f3 SDFBlockToWorld(const Scene& s, i3 b) {  // :313-315
    return virtualVoxelPosToWorld(s, {b.x * BF_SDF_BLOCK_SIZE, b.y * BF_SDF_BLOCK_SIZE, b.z * BF_SDF_BLOCK_SIZE});
}
// Multi-GPU spatial ownership (the build's sharding; no reference counterpart beyond the
// d_bitMask hook of allocKernel, CUDASceneRepHashSDF.cu:227): the block's corner chunk, rounded as
// worldToChunks (:136-150), hashed with computeHashPos onto the shard count.
bool owned(const Scene& s, i3 b) {
    if (s.shardCount <= 1) return true;
    const f3 w = SDFBlockToWorld(s, b) / s.shardChunk;
    const i3 c = {f2i(w.x + (float)sgn(w.x) * 0.5f), f2i(w.y + (float)sgn(w.y) * 0.5f), f2i(w.z + (float)sgn(w.z) * 0.5f)};
    int32_t a = (int32_t)((uint32_t)c.x * 73856093u), bb = (int32_t)((uint32_t)c.y * 19349669u), cc = (int32_t)((uint32_t)c.z * 83492791u);
    int res = (a ^ bb ^ cc) % (int)s.shardCount;
    if (res < 0) res += (int)s.shardCount;
    return (uint32_t)res == s.shardIndex;
}
i3 worldToSDFBlock(const Scene& s, f3 w) { return virtualVoxelPosToSDFBlock(worldToVirtualVoxelPos(s, w)); }

// DepthCameraUtil.h:71-107 + :137-144 (frustum test against c_depthCameraParams)
f3 cameraToKinectProj(const BFDepthCameraParams& c, f3 pos) {
    float px = pos.x * c.fx / pos.z + c.mx;
    float py = pos.y * c.fy / pos.z + c.my;
    f3 r;
    r.x = (2.0f * px - ((float)c.imageWidth - 1.0f)) / ((float)c.imageWidth - 1.0f);
    r.y = (((float)c.imageHeight - 1.0f) - 2.0f * py) / ((float)c.imageHeight - 1.0f);
    r.z = (pos.z - c.sensorDepthWorldMin) / (c.sensorDepthWorldMax - c.sensorDepthWorldMin);
    return r;
}
bool isInCameraFrustumApprox(const BFDepthCameraParams& c, const m4& viewInv, f3 pos) {
    f3 pc = xform(viewInv, pos);
    f3 pp = cameraToKinectProj(c, pc);
    // pProj *= 0.95: operator*=(float3&, float) (cutil_math.h:761) takes 0.95 as 0.95f
    pp = pp * 0.95f;
    return !(pp.x < -1.0f || pp.x > 1.0f || pp.y < -1.0f || pp.y > 1.0f || pp.z < 0.0f || pp.z > 1.0f);
}
// isSDFBlockInCameraFrustumApprox :322-326
bool blockInFrustum(const Scene& s, i3 b) {
    f3 w = SDFBlockToWorld(s, b) + mk(1, 1, 1) * (s.hp.virtualVoxelSize * 0.5f * (BF_SDF_BLOCK_SIZE - 1.0f));
    return isInCameraFrustumApprox(s.cam, s.Tinv, w);
}

bool samePos(const BFHashEntry& e, i3 p) { return e.x == p.x && e.y == p.y && e.z == p.z; }

void deleteHashEntry(BFHashEntry& e) { e.x = e.y = e.z = 0; e.offset = 0; e.ptr = BF_FREE_ENTRY; }  // :382-386
void deleteVoxel(BFVoxel& v) { v.sdf = 0; v.weight = 0; v.color[0] = v.color[1] = v.color[2] = v.color[3] = 0; }

uint32_t numEntries(const Scene& s) { return s.hp.hashNumBuckets * BF_HASH_BUCKET_SIZE; }

// getHashEntryForSDFBlockPos :440-485
BFHashEntry getHashEntryForSDFBlockPos(const Scene& s, i3 b) {
    uint32_t h = hashPos(s, b), hp = h * BF_HASH_BUCKET_SIZE;
    BFHashEntry entry{};
    entry.x = b.x; entry.y = b.y; entry.z = b.z; entry.offset = 0; entry.ptr = BF_FREE_ENTRY;
    for (uint32_t j = 0; j < BF_HASH_BUCKET_SIZE; j++) {
        const BFHashEntry& curr = s.hash[j + hp];
        if (samePos(curr, b) && curr.ptr != BF_FREE_ENTRY) return curr;
    }
    const uint32_t last = (h + 1) * BF_HASH_BUCKET_SIZE - 1;
    uint32_t i = last;
    for (uint32_t it = 0; it < s.hp.hashMaxCollisionLinkedListSize; it++) {
        const BFHashEntry& curr = s.hash[i];
        if (samePos(curr, b) && curr.ptr != BF_FREE_ENTRY) return curr;
        if (curr.offset == 0) break;
        i = (last + curr.offset) % numEntries(s);
    }
    return entry;
}

// consumeHeap / appendHeap :535-546
uint32_t consumeHeap(Scene& s) { uint32_t addr = s.heapCounter--; return s.heap[addr]; }
void appendHeap(Scene& s, uint32_t ptr) { uint32_t addr = s.heapCounter++; s.heap[addr + 1] = ptr; }

// allocBlock :549-655 (serial: every atomicExch try-lock succeeds unless the bucket
// was already locked in this pass by an earlier thread)
bool allocBlock(Scene& s, i3 pos) {
    uint32_t h = hashPos(s, pos), hp = h * BF_HASH_BUCKET_SIZE;
    int firstEmpty = -1;
    for (uint32_t j = 0; j < BF_HASH_BUCKET_SIZE; j++) {
        uint32_t i = j + hp;
        const BFHashEntry& curr = s.hash[i];
        if (samePos(curr, pos) && curr.ptr != BF_FREE_ENTRY) return false;
        if (firstEmpty == -1 && curr.ptr == BF_FREE_ENTRY) firstEmpty = (int)i;
    }
    const uint32_t last = (h + 1) * BF_HASH_BUCKET_SIZE - 1;
    uint32_t i = last;
    for (uint32_t it = 0; it < s.hp.hashMaxCollisionLinkedListSize; it++) {
        const BFHashEntry& curr = s.hash[i];
        if (samePos(curr, pos) && curr.ptr != BF_FREE_ENTRY) return false;
        if (curr.offset == 0) break;
        i = (last + curr.offset) % numEntries(s);
    }
    if (s.heapCounter == 0xFFFFFFFFu || s.heapCounter >= s.hp.numSDFBlocks) {  // heap exhausted (unchecked in ref)
        s.stats.allocOverflow++;
        return false;
    }
    if (firstEmpty != -1) {
        int prev = s.mutex[h]; s.mutex[h] = BF_LOCK_ENTRY;
        if (prev != BF_LOCK_ENTRY) {
            BFHashEntry& e = s.hash[firstEmpty];
            e.x = pos.x; e.y = pos.y; e.z = pos.z; e.offset = 0;
            e.ptr = (int32_t)(consumeHeap(s) * BF_VOXELS_PER_BLOCK);
            s.stats.allocated++;
            return true;
        }
        return false;
    }
    int offset = 0;
    for (uint32_t it = 0; it < s.hp.hashMaxCollisionLinkedListSize;) {
        offset++;
        i = (last + (uint32_t)offset) % numEntries(s);
        if ((offset % BF_HASH_BUCKET_SIZE) == 0) continue;  // never a last bucket slot
        const BFHashEntry& curr = s.hash[i];
        if (curr.ptr == BF_FREE_ENTRY) {
            int prev = s.mutex[h]; s.mutex[h] = BF_LOCK_ENTRY;
            if (prev != BF_LOCK_ENTRY) {
                BFHashEntry lastEntry = s.hash[last];
                uint32_t h2 = i / BF_HASH_BUCKET_SIZE;
                prev = s.mutex[h2]; s.mutex[h2] = BF_LOCK_ENTRY;
                if (prev != BF_LOCK_ENTRY) {
                    BFHashEntry& e = s.hash[i];
                    e.x = pos.x; e.y = pos.y; e.z = pos.z;
                    e.offset = lastEntry.offset;
                    e.ptr = (int32_t)(consumeHeap(s) * BF_VOXELS_PER_BLOCK);
                    lastEntry.offset = (uint32_t)offset;
                    s.hash[last] = lastEntry;
                    s.stats.allocated++;
                    return true;
                }
            }
            return false;
        }
        it++;
    }
    return false;
}

// deleteHashEntryElement :739-826
bool deleteHashEntryElement(Scene& s, i3 b) {
    uint32_t h = hashPos(s, b), hp = h * BF_HASH_BUCKET_SIZE;
    for (uint32_t j = 0; j < BF_HASH_BUCKET_SIZE; j++) {
        uint32_t i = j + hp;
        const BFHashEntry curr = s.hash[i];
        if (samePos(curr, b) && curr.ptr != BF_FREE_ENTRY) {
            if (curr.offset != 0) {
                int prev = s.mutex[h]; s.mutex[h] = BF_LOCK_ENTRY;
                if (prev == BF_LOCK_ENTRY) return false;
                appendHeap(s, (uint32_t)curr.ptr / BF_VOXELS_PER_BLOCK);
                uint32_t nextIdx = (i + curr.offset) % numEntries(s);
                s.hash[i] = s.hash[nextIdx];
                deleteHashEntry(s.hash[nextIdx]);
                return true;
            } else {
                appendHeap(s, (uint32_t)curr.ptr / BF_VOXELS_PER_BLOCK);
                deleteHashEntry(s.hash[i]);
                return true;
            }
        }
    }
    const uint32_t last = (h + 1) * BF_HASH_BUCKET_SIZE - 1;
    uint32_t i = last;
    BFHashEntry curr = s.hash[i];
    uint32_t prevIdx = i;
    i = (last + curr.offset) % numEntries(s);
    for (uint32_t it = 0; it < s.hp.hashMaxCollisionLinkedListSize; it++) {
        curr = s.hash[i];
        if (samePos(curr, b) && curr.ptr != BF_FREE_ENTRY) {
            int prev = s.mutex[h]; s.mutex[h] = BF_LOCK_ENTRY;
            if (prev == BF_LOCK_ENTRY) return false;
            appendHeap(s, (uint32_t)curr.ptr / BF_VOXELS_PER_BLOCK);
            deleteHashEntry(s.hash[i]);
            BFHashEntry p = s.hash[prevIdx];
            p.offset = curr.offset;
            s.hash[prevIdx] = p;
            return true;
        }
        if (curr.offset == 0) return false;
        prevIdx = i;
        i = (last + curr.offset) % numEntries(s);
    }
    return false;
}

void resetMutex(Scene& s) { std::fill(s.mutex.begin(), s.mutex.end(), BF_FREE_ENTRY); }  // :58-65

// DepthCameraUtil.h:114-119 (kinectDepthToSkeleton)
f3 depthToSkeleton(const BFDepthCameraParams& c, uint32_t ux, uint32_t uy, float depth) {
    const float x = ((float)ux - c.mx) / c.fx;
    const float y = ((float)uy - c.my) / c.fy;
    return mk(depth * x, depth * y, depth);
}

// allocKernel, CUDASceneRepHashSDF.cu:165-251, one pixel: the DDA walk. The blocks it would test
// (in the frustum, in walk order) are appended to `out`; the hash lookups and inserts happen in
// allocPass, in pixel order, because their outcome depends on what earlier threads inserted.
void allocPixelWalk(const Scene& s, const float* depth, uint32_t x, uint32_t y, std::vector<i3>& out) {
    const BFDepthCameraParams& c = s.cam;
    float d = depth[y * c.imageWidth + x];
    if (d == MINF || d == 0.0f) return;
    if (d >= s.hp.maxIntegrationDistance) return;
    float t = truncation(s, d);
    float minDepth = std::min(s.hp.maxIntegrationDistance, d - t);
    float maxDepth = std::min(s.hp.maxIntegrationDistance, d + t);
    if (minDepth >= maxDepth) return;
    f3 rayMin = xform(s.T, depthToSkeleton(c, x, y, minDepth));
    f3 rayMax = xform(s.T, depthToSkeleton(c, x, y, maxDepth));
    f3 rayDir = normalize(rayMax - rayMin);
    i3 id = worldToSDFBlock(s, rayMin);
    i3 idEnd = worldToSDFBlock(s, rayMax);
    f3 step = mk((float)sgn(rayDir.x), (float)sgn(rayDir.y), (float)sgn(rayDir.z));
    auto clamp01 = [](float v) { return std::max(0.0f, std::min(v, 1.0f)); };
    i3 idc = {id.x + f2i(clamp01(step.x)), id.y + f2i(clamp01(step.y)), id.z + f2i(clamp01(step.z))};
    f3 boundaryPos = SDFBlockToWorld(s, idc) - mk(1, 1, 1) * (0.5f * s.hp.virtualVoxelSize);
    f3 tMax = (boundaryPos - rayMin) / rayDir;
    f3 tDelta = (step * (float)BF_SDF_BLOCK_SIZE * s.hp.virtualVoxelSize) / rayDir;
    i3 idBound = {f2i((float)idEnd.x + step.x), f2i((float)idEnd.y + step.y), f2i((float)idEnd.z + step.z)};
    if (rayDir.x == 0.0f) { tMax.x = PINF; tDelta.x = PINF; }
    if (boundaryPos.x - rayMin.x == 0.0f) { tMax.x = PINF; tDelta.x = PINF; }
    if (rayDir.y == 0.0f) { tMax.y = PINF; tDelta.y = PINF; }
    if (boundaryPos.y - rayMin.y == 0.0f) { tMax.y = PINF; tDelta.y = PINF; }
    if (rayDir.z == 0.0f) { tMax.z = PINF; tDelta.z = PINF; }
    if (boundaryPos.z - rayMin.z == 0.0f) { tMax.z = PINF; tDelta.z = PINF; }
    // (the chunk-streaming bitmask test is disabled with streaming, zParametersDefault.txt:100)
    for (uint32_t iter = 0; iter < 1024; iter++) {
        if (blockInFrustum(s, id) && owned(s, id)) out.push_back(id);
        if (tMax.x < tMax.y && tMax.x < tMax.z) {
            id.x = f2i((float)id.x + step.x);
            if (id.x == idBound.x) return;
            tMax.x += tDelta.x;
        } else if (tMax.z < tMax.y) {
            id.z = f2i((float)id.z + step.z);
            if (id.z == idBound.z) return;
            tMax.z += tDelta.z;
        } else {
            id.y = f2i((float)id.y + step.y);
            if (id.y == idBound.y) return;
            tMax.y += tDelta.y;
        }
    }
}

// Open-addressing set of block coordinates seen in one alloc pass, with the outcome of their first
// test (absent after it: 1).
struct SeenSet {
    std::vector<uint64_t> key;
    std::vector<uint8_t> absent;
    uint64_t mask = 0;
    void reset(size_t n) {
        size_t cap = 1024;
        while (cap < 2 * n) cap <<= 1;
        key.assign(cap, ~0ull);
        absent.assign(cap, 0);
        mask = cap - 1;
    }
    static uint64_t pack(i3 p) {
        return ((uint64_t)(uint32_t)(p.x & 0x1FFFFF) << 42) | ((uint64_t)(uint32_t)(p.y & 0x1FFFFF) << 21) |
               (uint64_t)(uint32_t)(p.z & 0x1FFFFF);
    }
    // returns the slot; *found = already present
    size_t find(uint64_t k, bool* found) const {
        size_t h = (size_t)((k * 0x9E3779B97F4A7C15ull) >> 20) & mask;
        while (key[h] != ~0ull && key[h] != k) h = (h + 1) & mask;
        *found = key[h] == k;
        return h;
    }
};

// One alloc pass over the walks' block lists in pixel order (thread order of a serial schedule). A
// repeated block inside a pass is a no-op whatever its first test did (found: found again; inserted:
// found; failed on a locked bucket / full list / empty heap: fails again, the locks stay set for the
// pass), so only its first occurrence runs; the candidate count still counts every absent test.
void allocPass(Scene& s, const std::vector<i3>& walk, SeenSet& seen, bool count) {
    seen.reset(walk.size());
    for (const i3& id : walk) {
        bool found = false;
        const size_t slot = seen.find(SeenSet::pack(id), &found);
        if (found) {
            if (count && seen.absent[slot]) s.stats.candidates++;
            continue;
        }
        seen.key[slot] = SeenSet::pack(id);
        BFHashEntry e = getHashEntryForSDFBlockPos(s, id);
        if (e.ptr == BF_FREE_ENTRY) {
            if (count) s.stats.candidates++;
            seen.absent[slot] = allocBlock(s, id) ? 0 : 1;
        }
    }
}

// compactifyHashAllInOneKernel :324-366 (order: table order; the HIP build's order differs,
// consumers are order-independent)
uint32_t compactify(Scene& s) {
    s.numOccupied = 0;
    const uint32_t E = numEntries(s);
    // table order, evaluated in parallel chunks and concatenated in chunk order
    const uint32_t chunk = 1u << 16, nChunks = (E + chunk - 1) / chunk;
    std::vector<std::vector<BFHashEntry>> part(nChunks);
    std::vector<uint64_t> scanned(nChunks, 0);
#pragma omp parallel for schedule(dynamic, 4)
    for (long c = 0; c < (long)nChunks; c++) {
        const uint32_t lo = (uint32_t)c * chunk, hi = std::min(E, lo + chunk);
        for (uint32_t i = lo; i < hi; i++) {
            const BFHashEntry& e = s.hash[i];
            if (e.ptr != BF_FREE_ENTRY) {
                scanned[c]++;
                if (blockInFrustum(s, {e.x, e.y, e.z})) part[c].push_back(e);
            }
        }
    }
    for (uint32_t c = 0; c < nChunks; c++) {
        s.stats.scanned += scanned[c];
        for (const BFHashEntry& e : part[c]) s.compact[s.numOccupied++] = e;
    }
    s.stats.visible += s.numOccupied;
    s.hp.numOccupiedBlocks = s.numOccupied;
    return s.numOccupied;
}

// integrateDepthMapKernel<deIntegrate>, CUDASceneRepHashSDF.cu:420-521
void integrateBlock(Scene& s, const BFHashEntry& entry, const float* depthImg, const uint8_t* colorImg,
                    bool deIntegrate, uint64_t& updated) {
    const BFDepthCameraParams& c = s.cam;
    i3 base = {entry.x * BF_SDF_BLOCK_SIZE, entry.y * BF_SDF_BLOCK_SIZE, entry.z * BF_SDF_BLOCK_SIZE};
    for (uint32_t i = 0; i < BF_VOXELS_PER_BLOCK; i++) {
        i3 pi = {base.x + (int)(i % 8), base.y + (int)((i % 64) / 8), base.z + (int)(i / 64)};
        f3 pf = xform(s.Tinv, virtualVoxelPosToWorld(s, pi));
        // cameraToKinectScreenInt: make_int2(pImage + 0.5) then make_uint2 (DepthCameraUtil.h:78-88)
        float sx = pf.x * c.fx / pf.z + c.mx;
        float sy = pf.y * c.fy / pf.z + c.my;
        uint32_t ux = (uint32_t)f2i(sx + 0.5f), uy = (uint32_t)f2i(sy + 0.5f);
        if (!(ux < c.imageWidth && uy < c.imageHeight)) continue;
        float depth = depthImg[uy * c.imageWidth + ux];
        if (!colorImg) continue;  // color stays MINF -> no update (:441-448)
        const uint8_t* cc = colorImg + 4 * (uy * c.imageWidth + ux);
        if (depth == MINF) continue;
        if (!(depth < s.hp.maxIntegrationDistance)) continue;
        float sdf = depth - pf.z;
        float tr = truncation(s, depth);
        if (!(std::fabs(sdf) < tr)) continue;
        if (sdf >= 0.0f) sdf = std::fmin(tr, sdf); else sdf = std::fmax(-tr, sdf);
        const float wUpd = 1.0f;  // :465-466
        BFVoxel& v = s.voxels[(size_t)entry.ptr + i];
        BFVoxel nv;
        float oc[3] = {(float)v.color[0], (float)v.color[1], (float)v.color[2]};
        float cu[3] = {(float)cc[0], (float)cc[1], (float)cc[2]};
        float res[3];
        if (!deIntegrate) {
            for (int k = 0; k < 3; k++) res[k] = (v.weight == 0.0f) ? cu[k] : 0.2f * cu[k] + 0.8f * oc[k];
            for (int k = 0; k < 3; k++) {
                float r = std::round(res[k]);
                r = std::fmax(0.0f, std::fmin(r, 254.5f));
                nv.color[k] = (uint8_t)r;
            }
            nv.color[3] = 255;
            nv.sdf = (sdf * wUpd + v.sdf * v.weight) / (wUpd + v.weight);
            nv.weight = std::min((float)s.hp.integrationWeightMax, wUpd + v.weight);
        } else {
            for (int k = 0; k < 3; k++) {
                float r = (oc[k] * v.weight - cu[k] * wUpd) / (v.weight - wUpd);
                r = std::round(r);
                r = std::fmax(0.0f, std::fmin(r, 254.5f));
                nv.color[k] = (uint8_t)r;
            }
            nv.color[3] = 255;
            nv.sdf = (v.sdf * v.weight - sdf * wUpd) / (v.weight - wUpd);
            nv.weight = std::max(0.0f, v.weight - wUpd);
            if (nv.weight <= 0.001f) { nv.sdf = 0.0f; nv.color[0] = nv.color[1] = nv.color[2] = nv.color[3] = 0; nv.weight = 0.0f; }
        }
        v = nv;
        updated++;
    }
}

void setTransform(Scene& s, const float* T, const BFDepthCameraParams* cam) {
    s.T = toM4(T);
    s.Tinv = inverse(s.T);
    std::memcpy(s.hp.rigidTransform.m, s.T.e, 64);
    std::memcpy(s.hp.rigidTransformInverse.m, s.Tinv.e, 64);
    s.cam = *cam;
}

}  // namespace

struct ORScene { Scene s; };

extern "C" {

ORScene* or_scene_create(const BFHashParams* params) {
    ORScene* o = new ORScene();
    o->s.hp = *params;
    Scene& s = o->s;
    const size_t E = (size_t)params->hashNumBuckets * BF_HASH_BUCKET_SIZE;
    s.hash.resize(E);
    s.compact.resize(E);
    s.heap.resize(params->numSDFBlocks);
    s.voxels.resize((size_t)params->numSDFBlocks * BF_VOXELS_PER_BLOCK);
    s.mutex.resize(params->hashNumBuckets);
    s.decision.resize(E);
    or_scene_reset(o);
    return o;
}

void or_scene_destroy(ORScene* o) { delete o; }

void or_scene_set_shard(ORScene* o, uint32_t count, uint32_t index, float chunk) {
    o->s.shardCount = count ? count : 1;
    o->s.shardIndex = index;
    o->s.shardChunk = chunk > 0.0f ? chunk : 1.0f;
}

// CUDASceneRepHashSDF::reset (.h:147-155) -> resetCUDA (.cu:67-111)
void or_scene_reset(ORScene* o) {
    Scene& s = o->s;
    const uint32_t B = s.hp.numSDFBlocks;
    s.heapCounter = B - 1;
    for (uint32_t i = 0; i < B; i++) s.heap[i] = B - i - 1;
    for (auto& v : s.voxels) deleteVoxel(v);
    for (auto& e : s.hash) deleteHashEntry(e);
    for (auto& e : s.compact) deleteHashEntry(e);
    resetMutex(s);
    s.numOccupied = 0;
    s.hp.numOccupiedBlocks = 0;
    std::memset(&s.stats, 0, sizeof(s.stats));
    float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    s.T = toM4(I);
    s.Tinv = toM4(I);
}

// CUDASceneRepHashSDF::integrate (.h:65-83) / deIntegrate (.h:85-108)
void or_scene_integrate(ORScene* o, const float T[16], const float* depth, const uint8_t* color,
                        const BFDepthCameraParams* cam, int deintegrate, const uint32_t* bitMask) {
    Scene& s = o->s;
    setTransform(s, T, cam);
    s.stats.integrateOps++;
    if (!deintegrate) {
        // alloc (.h:328-352): repeat {reset bucket mutex; alloc pass} until the heap free
        // count is unchanged. Serially, a pass inserts at most one block per bucket (the
        // bucket stays locked for the rest of the pass, VoxelUtilHashSDF.h:604-611).
        s.stats.pixels += (uint64_t)cam->imageWidth * cam->imageHeight;
        (void)bitMask;
        // the walks depend on the pose and the depth only: computed once, in parallel by row, and
        // concatenated in pixel order
        const uint32_t W = cam->imageWidth, H = cam->imageHeight;
        std::vector<std::vector<i3>> rows(H);
#pragma omp parallel for schedule(dynamic, 4)
        for (long y = 0; y < (long)H; y++)
            for (uint32_t x = 0; x < W; x++) allocPixelWalk(s, depth, x, (uint32_t)y, rows[y]);
        std::vector<i3> walk;
        size_t total = 0;
        for (const auto& r : rows) total += r.size();
        walk.reserve(total);
        for (const auto& r : rows) walk.insert(walk.end(), r.begin(), r.end());
        rows.clear();
        SeenSet seen;
        uint32_t prevFree = s.heapCounter + 1;
        for (int pass = 0;; pass++) {
            resetMutex(s);
            allocPass(s, walk, seen, pass == 0);
            uint32_t currFree = s.heapCounter + 1;
            if (currFree == prevFree) break;
            prevFree = currFree;
        }
        resetMutex(s);
    }
    compactify(s);
    uint64_t updated = 0;
#pragma omp parallel for reduction(+ : updated) schedule(dynamic, 64)
    for (long b = 0; b < (long)s.numOccupied; b++) integrateBlock(s, s.compact[b], depth, color, deintegrate != 0, updated);
    s.stats.voxelsUpdated += updated;
}

uint32_t or_scene_compactify(ORScene* o, const float T[16], const BFDepthCameraParams* cam) {
    setTransform(o->s, T, cam);
    return compactify(o->s);
}

// CUDASceneRepHashSDF::garbageCollect (.h:110-126): identify (.cu:584-631), mutex reset,
// free (.cu:648-668) over the last compacted list. Free threads run serially in ascending
// block-coordinate order (the canonical order the HIP build also uses for collision-list
// deletes; simple in-bucket deletes are order-independent).
void or_scene_garbage_collect(ORScene* o) {
    Scene& s = o->s;
    if (s.numOccupied == 0) return;
    std::vector<BFHashEntry> victims;
    for (uint32_t b = 0; b < s.numOccupied; b++) {
        const BFHashEntry& e = s.compact[b];
        uint32_t maxW = 0;
        for (uint32_t i = 0; i < BF_VOXELS_PER_BLOCK; i++) {
            uint32_t w = (uint32_t)s.voxels[(size_t)e.ptr + i].weight;  // max as uint (.cu:606)
            maxW = std::max(maxW, w);
        }
        s.stats.gcBlocks++;
        if (maxW == 0) victims.push_back(e);
    }
    std::sort(victims.begin(), victims.end(), [](const BFHashEntry& a, const BFHashEntry& b) {
        if (a.x != b.x) return a.x < b.x;
        if (a.y != b.y) return a.y < b.y;
        return a.z < b.z;
    });
    resetMutex(s);
    for (const BFHashEntry& e : victims) {
        if (deleteHashEntryElement(s, {e.x, e.y, e.z})) {
            for (uint32_t i = 0; i < BF_VOXELS_PER_BLOCK; i++) deleteVoxel(s.voxels[(size_t)e.ptr + i]);
            s.stats.gcFreed++;
        }
    }
}

uint32_t or_scene_heap_free_count(const ORScene* o) { return o->s.heapCounter + 1; }  // .h:168-172
uint32_t or_scene_num_occupied(const ORScene* o) { return o->s.numOccupied; }

void or_scene_export(const ORScene* o, BFHashEntry* hash, uint32_t* heap, uint32_t* heapCounter, BFVoxel* voxels) {
    const Scene& s = o->s;
    if (hash) std::memcpy(hash, s.hash.data(), s.hash.size() * sizeof(BFHashEntry));
    if (heap) std::memcpy(heap, s.heap.data(), s.heap.size() * sizeof(uint32_t));
    if (heapCounter) *heapCounter = s.heapCounter;
    if (voxels) std::memcpy(voxels, s.voxels.data(), s.voxels.size() * sizeof(BFVoxel));
}

// the inverse of or_scene_export: a scene state (e.g. a GPU dump, bf_scene_export's layout) to continue
// from; the compacted list is empty until the next compactify
void or_scene_import(ORScene* o, const BFHashEntry* hash, const uint32_t* heap, uint32_t heapCounter, const BFVoxel* voxels) {
    Scene& s = o->s;
    std::memcpy(s.hash.data(), hash, s.hash.size() * sizeof(BFHashEntry));
    std::memcpy(s.heap.data(), heap, s.heap.size() * sizeof(uint32_t));
    s.heapCounter = heapCounter;
    std::memcpy(s.voxels.data(), voxels, s.voxels.size() * sizeof(BFVoxel));
    s.numOccupied = 0;
    resetMutex(s);
}

void or_scene_export_visible(const ORScene* o, BFHashEntry* out) {
    std::memcpy(out, o->s.compact.data(), o->s.numOccupied * sizeof(BFHashEntry));
}

void or_scene_get_stats(const ORScene* o, BFTsdfStats* out) { *out = o->s.stats; }

// Config 1: one frame into a dense n^3 grid whose voxel (0,0,0) sits at virtual voxel
// `origin`; same per-voxel arithmetic as integrateDepthMapKernel<false>.
void or_dense_integrate(const float T[16], const float* depth, const uint8_t* color,
                        const BFDepthCameraParams* cam, const BFHashParams* params,
                        const int origin[3], int n, BFVoxel* grid) {
    ORScene tmp;  // only hp/cam/T are used by integrateBlock
    Scene& s = tmp.s;
    s.hp = *params;
    setTransform(s, T, cam);
    const int nb = n / BF_SDF_BLOCK_SIZE;
    s.voxels.assign((size_t)nb * nb * nb * BF_VOXELS_PER_BLOCK, BFVoxel{});
    for (auto& v : s.voxels) deleteVoxel(v);
    uint64_t upd = 0;
    for (int bz = 0; bz < nb; bz++)
        for (int by = 0; by < nb; by++)
            for (int bx = 0; bx < nb; bx++) {
                BFHashEntry e{};
                e.x = origin[0] / 8 + bx; e.y = origin[1] / 8 + by; e.z = origin[2] / 8 + bz;
                e.ptr = ((bz * nb + by) * nb + bx) * BF_VOXELS_PER_BLOCK;
                integrateBlock(s, e, depth, color, false, upd);
            }
    for (int bz = 0; bz < nb; bz++)
        for (int by = 0; by < nb; by++)
            for (int bx = 0; bx < nb; bx++)
                for (int i = 0; i < BF_VOXELS_PER_BLOCK; i++) {
                    int x = bx * 8 + i % 8, y = by * 8 + (i % 64) / 8, z = bz * 8 + i / 64;
                    grid[((size_t)z * n + y) * n + x] = s.voxels[(size_t)((bz * nb + by) * nb + bx) * 512 + i];
                }
}

}  // extern "C"

// ---- raycast: CUDARayCastSDF::render (CUDARayCastSDF.cpp:38-72) ----------------------------
namespace {

// cameraToDepthProj (RayCastSDFUtil.h:208-222)
f3 rcProj(const BFRayCastParams& p, f3 pos) {
    f3 r;
    const float px = pos.x * p.fx / pos.z + p.mx, py = pos.y * p.fy / pos.z + p.my;
    r.x = (2.0f * px - ((float)p.width - 1.0f)) / ((float)p.width - 1.0f);
    r.y = (((float)p.height - 1.0f) - 2.0f * py) / ((float)p.height - 1.0f);
    r.z = (pos.z - p.minDepth) / (p.maxDepth - p.minDepth);
    return r;
}
f3 rcDepthToCamera(const BFRayCastParams& p, uint32_t ux, uint32_t uy, float depth) {
    const float x = ((float)ux - p.mx) / p.fx, y = ((float)uy - p.my) / p.fy;
    return {depth * x, depth * y, depth};
}
f3 fmin3(f3 a, f3 b) { return {std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z)}; }
f3 fmax3(f3 a, f3 b) { return {std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)}; }

struct Quad {  // the 6 vertices of rayIntervalSplatKernel (CUDARayCastSDF.cu:170-180) as a rectangle
    float minX, maxX, minY, maxY, ndcZ, depthWorld;
};

// D3D11 raster of one pass: pixel centres inside [left, right) x [top, bottom) (top-left rule for an
// axis-aligned rectangle), depth test on the NDC z clamped to [0, 1] (depth clip disabled), the pixel
// shader writes the world depth.
void rasterPass(const std::vector<Quad>& quads, const BFRayCastParams& p, bool minPass, std::vector<float>& target) {
    const uint32_t W = p.width, H = p.height;
    std::vector<float> zbuf((size_t)W * H, minPass ? 1.0f : 0.0f);
    target.assign((size_t)W * H, minPass ? MINF : 0.0f);
    for (const Quad& q : quads) {
        const float Wf = (float)W, Hf = (float)H;
        const float left = (q.minX + 1.0f) * 0.5f * Wf, right = (q.maxX + 1.0f) * 0.5f * Wf;
        const float top = (1.0f - q.maxY) * 0.5f * Hf, bottom = (1.0f - q.minY) * 0.5f * Hf;
        if (!(left < right) || !(top < bottom)) continue;
        const float z = std::fmin(std::fmax(q.ndcZ, 0.0f), 1.0f);
        for (uint32_t py = 0; py < H; py++) {
            const float cy = (float)py + 0.5f;
            if (!(top <= cy && cy < bottom)) continue;
            for (uint32_t px = 0; px < W; px++) {
                const float cx = (float)px + 0.5f;
                if (!(left <= cx && cx < right)) continue;
                float& zb = zbuf[(size_t)py * W + px];
                if (minPass ? (z < zb) : (z > zb)) {
                    zb = z;
                    target[(size_t)py * W + px] = q.depthWorld;
                }
            }
        }
    }
}

// getVoxel(worldPos) (VoxelUtilHashSDF.h:406-417)
BFVoxel getVoxelWorld(const Scene& s, f3 pos) {
    const i3 v = worldToVirtualVoxelPos(s, pos);
    const BFHashEntry e = getHashEntryForSDFBlockPos(s, virtualVoxelPosToSDFBlock(v));
    BFVoxel out;
    if (e.ptr == BF_FREE_ENTRY) {
        deleteVoxel(out);
        return out;
    }
    int lx = v.x % BF_SDF_BLOCK_SIZE, ly = v.y % BF_SDF_BLOCK_SIZE, lz = v.z % BF_SDF_BLOCK_SIZE;
    if (lx < 0) lx += BF_SDF_BLOCK_SIZE;
    if (ly < 0) ly += BF_SDF_BLOCK_SIZE;
    if (lz < 0) lz += BF_SDF_BLOCK_SIZE;
    return s.voxels[(size_t)e.ptr + (size_t)(lz * 64 + ly * 8 + lx)];
}

float frac1(float v) { return v - std::floor(v); }

// trilinearInterpolationSimpleFastFast (RayCastSDFUtil.h:96-116), literal corner order
bool trilinear(const Scene& s, f3 pos, float& dist, uint8_t rgb[3]) {
    const float oSet = s.hp.virtualVoxelSize;
    const f3 posDual = pos - mk(oSet / 2.0f, oSet / 2.0f, oSet / 2.0f);
    const f3 vv = pos / s.hp.virtualVoxelSize;
    const f3 w = {frac1(vv.x), frac1(vv.y), frac1(vv.z)};
    dist = 0.0f;
    f3 colorFloat = {0.0f, 0.0f, 0.0f};
    auto tap = [&](f3 off, float fx, float fy, float fz) {
        const BFVoxel v = getVoxelWorld(s, posDual + off);
        if (v.weight == 0) return false;
        const f3 vColor = {(float)v.color[0], (float)v.color[1], (float)v.color[2]};
        const float wt = fx * fy * fz;
        dist += wt * v.sdf;
        colorFloat = colorFloat + wt * vColor;
        return true;
    };
    if (!tap({0.0f, 0.0f, 0.0f}, 1.0f - w.x, 1.0f - w.y, 1.0f - w.z)) return false;
    if (!tap({oSet, 0.0f, 0.0f}, w.x, 1.0f - w.y, 1.0f - w.z)) return false;
    if (!tap({0.0f, oSet, 0.0f}, 1.0f - w.x, w.y, 1.0f - w.z)) return false;
    if (!tap({0.0f, 0.0f, oSet}, 1.0f - w.x, 1.0f - w.y, w.z)) return false;
    if (!tap({oSet, oSet, 0.0f}, w.x, w.y, 1.0f - w.z)) return false;
    if (!tap({0.0f, oSet, oSet}, 1.0f - w.x, w.y, w.z)) return false;
    if (!tap({oSet, 0.0f, oSet}, w.x, 1.0f - w.y, w.z)) return false;
    if (!tap({oSet, oSet, oSet}, w.x, w.y, w.z)) return false;
    rgb[0] = (uint8_t)colorFloat.x;
    rgb[1] = (uint8_t)colorFloat.y;
    rgb[2] = (uint8_t)colorFloat.z;
    return true;
}

f3 gradientForPoint(const Scene& s, f3 pos) {  // RayCastSDFUtil.h:172-194
    const float vs = s.hp.virtualVoxelSize;
    const f3 off = {vs, vs, vs};
    float dp00, d0p0, d00p, d100, d010, d001;
    uint8_t c[3];
    trilinear(s, pos - mk(0.5f * off.x, 0.0f, 0.0f), dp00, c);
    trilinear(s, pos - mk(0.0f, 0.5f * off.y, 0.0f), d0p0, c);
    trilinear(s, pos - mk(0.0f, 0.0f, 0.5f * off.z), d00p, c);
    trilinear(s, pos + mk(0.5f * off.x, 0.0f, 0.0f), d100, c);
    trilinear(s, pos + mk(0.0f, 0.5f * off.y, 0.0f), d010, c);
    trilinear(s, pos + mk(0.0f, 0.0f, 0.5f * off.z), d001, c);
    const f3 g = {(dp00 - d100) / off.x, (d0p0 - d010) / off.y, (d00p - d001) / off.z};
    const float l = length(g);
    if (l == 0.0f) return {0.0f, 0.0f, 0.0f};
    return mk(-g.x, -g.y, -g.z) / l;
}

}  // namespace

extern "C" void or_raycast(const ORScene* o, const BFRayCastParams* rpIn, const BFDepthCameraParams* cam, const float T[16],
                           float* depth, float* depth4, float* normals, float* colors, float* rayMin, float* rayMax) {
    Scene& s = const_cast<ORScene*>(o)->s;
    setTransform(s, T, cam);
    compactify(s);  // setLastRigidTransformAndCompactify
    BFRayCastParams p = *rpIn;
    std::memcpy(p.viewMatrixInverse.m, s.T.e, 64);
    std::memcpy(p.viewMatrix.m, s.Tinv.e, 64);
    const m4 V = s.Tinv, Vinv = s.T;
    const uint32_t W = p.width, H = p.height;
    // rayIntervalSplatKernel, both passes
    std::vector<Quad> qmin, qmax;
    const float vs = s.hp.virtualVoxelSize;
    for (uint32_t i = 0; i < s.numOccupied; i++) {
        const BFHashEntry& e = s.compact[i];
        if (e.ptr == BF_FREE_ENTRY || !blockInFrustum(s, {e.x, e.y, e.z})) continue;
        const f3 wv = SDFBlockToWorld(s, {e.x, e.y, e.z});
        const f3 MINV = {wv.x - vs / 2.0f, wv.y - vs / 2.0f, wv.z - vs / 2.0f};
        const float ext = (float)BF_SDF_BLOCK_SIZE * vs;
        const f3 maxv = {MINV.x + ext, MINV.y + ext, MINV.z + ext};
        const f3 p000 = rcProj(p, xform(V, mk(MINV.x, MINV.y, MINV.z)));
        const f3 p100 = rcProj(p, xform(V, mk(maxv.x, MINV.y, MINV.z)));
        const f3 p010 = rcProj(p, xform(V, mk(MINV.x, maxv.y, MINV.z)));
        const f3 p001 = rcProj(p, xform(V, mk(MINV.x, MINV.y, maxv.z)));
        const f3 p110 = rcProj(p, xform(V, mk(maxv.x, maxv.y, MINV.z)));
        const f3 p011 = rcProj(p, xform(V, mk(MINV.x, maxv.y, maxv.z)));
        const f3 p101 = rcProj(p, xform(V, mk(maxv.x, MINV.y, maxv.z)));
        const f3 p111 = rcProj(p, xform(V, mk(maxv.x, maxv.y, maxv.z)));
        const f3 mn = fmin3(fmin3(fmin3(p000, p100), fmin3(p010, p001)), fmin3(fmin3(p110, p011), fmin3(p101, p111)));
        const f3 mx = fmax3(fmax3(fmax3(p000, p100), fmax3(p010, p001)), fmax3(fmax3(p110, p011), fmax3(p101, p111)));
        qmin.push_back({mn.x, mx.x, mn.y, mx.y, mn.z, mn.z * (p.maxDepth - p.minDepth) + p.minDepth});
        qmax.push_back({mn.x, mx.x, mn.y, mx.y, mx.z, mx.z * (p.maxDepth - p.minDepth) + p.minDepth});
    }
    std::vector<float> tmin, tmax;
    rasterPass(qmin, p, true, tmin);
    rasterPass(qmax, p, false, tmax);
    if (rayMin) std::memcpy(rayMin, tmin.data(), 4 * tmin.size());
    if (rayMax) std::memcpy(rayMax, tmax.data(), 4 * tmax.size());
    // renderKernel + traverseCoarseGridSimpleSampleAll
    std::vector<float> d4((size_t)W * H * 4, MINF);
    for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = 0; x < W; x++) {
            const size_t pix = (size_t)y * W + x;
            depth[pix] = MINF;
            for (int k = 0; k < 4; k++) depth4[4 * pix + k] = normals[4 * pix + k] = colors[4 * pix + k] = MINF;
            const f3 camDir = normalize(rcDepthToCamera(p, x, y, 1.0f));
            const f3 worldCamPos = xform(Vinv, mk(0.0f, 0.0f, 0.0f));
            const f3 worldDir = normalize(xform4(Vinv, camDir, 0.0f));
            float minI = tmin[pix], maxI = tmax[pix];
            if (minI == 0 || minI == MINF) continue;
            if (maxI == 0 || maxI == MINF) continue;
            minI = std::fmax(minI, p.minDepth);
            maxI = std::fmin(maxI, p.maxDepth);
            float lastSdf = 0.0f, lastAlpha = 0.0f;
            int lastWeight = 0;
            const float d2r = 1.0f / camDir.z;
            float rayCurrent = d2r * std::fmax(p.minDepth, minI);
            const float rayEnd = d2r * std::fmin(p.maxDepth, maxI);
            while (rayCurrent < rayEnd) {
                const f3 cur = worldCamPos + rayCurrent * worldDir;
                float dist;
                uint8_t rgb[3];
                if (trilinear(s, cur, dist, rgb)) {
                    if (lastWeight > 0 && lastSdf > 0.0f && dist < 0.0f) {
                        float a = lastAlpha, aDist = lastSdf, b = rayCurrent, bDist = dist, c = 0.0f;
                        uint8_t rgb2[3] = {0, 0, 0};
                        bool ok = true;
                        for (int it = 0; it < 3; it++) {  // findIntersectionBisection
                            c = a + (aDist / (aDist - bDist)) * (b - a);
                            float cDist;
                            if (!trilinear(s, worldCamPos + c * worldDir, cDist, rgb2)) { ok = false; break; }
                            if (aDist * cDist > 0.0) { a = c; aDist = cDist; }
                            else { b = c; bDist = cDist; }
                        }
                        const float alpha = c;
                        if (ok && std::fabs(lastSdf - dist) < p.thresSampleDist && std::fabs(dist) < p.thresDist) {
                            const float dd = alpha / d2r;
                            depth[pix] = dd;
                            const f3 cp = rcDepthToCamera(p, x, y, dd);
                            depth4[4 * pix] = cp.x; depth4[4 * pix + 1] = cp.y; depth4[4 * pix + 2] = cp.z; depth4[4 * pix + 3] = 1.0f;
                            colors[4 * pix] = rgb2[0] / 255.f; colors[4 * pix + 1] = rgb2[1] / 255.f;
                            colors[4 * pix + 2] = rgb2[2] / 255.f; colors[4 * pix + 3] = 1.0f;
                            if (p.useGradients) {
                                const f3 g = gradientForPoint(s, worldCamPos + alpha * worldDir);
                                const f3 n = xform4(V, mk(-g.x, -g.y, -g.z), 0.0f);
                                normals[4 * pix] = n.x; normals[4 * pix + 1] = n.y; normals[4 * pix + 2] = n.z; normals[4 * pix + 3] = 1.0f;
                            }
                            break;
                        }
                    }
                    lastSdf = dist;
                    lastAlpha = rayCurrent;
                    lastWeight = 1;
                    rayCurrent += p.rayIncrement;
                } else {
                    lastWeight = 0;
                    rayCurrent += p.rayIncrement;
                }
            }
        }
    if (!p.useGradients) {  // computeNormalsDevice (CameraUtil.cu:665-692)
        for (uint32_t y = 0; y < H; y++)
            for (uint32_t x = 0; x < W; x++) {
                float* out = normals + 4 * ((size_t)y * W + x);
                out[0] = out[1] = out[2] = out[3] = MINF;
                if (!(x > 0 && x < W - 1 && y > 0 && y < H - 1)) continue;
                auto at = [&](uint32_t xx, uint32_t yy) {
                    const float* q = depth4 + 4 * ((size_t)yy * W + xx);
                    return f3{q[0], q[1], q[2]};
                };
                const f3 CC = at(x, y), PC = at(x, y + 1), CP = at(x + 1, y), MC = at(x, y - 1), CM = at(x - 1, y);
                if (CC.x != MINF && PC.x != MINF && CP.x != MINF && MC.x != MINF && CM.x != MINF) {
                    const f3 n = cross(PC - MC, CP - CM);
                    const float l = length(n);
                    if (l > 0.0f) { out[0] = n.x / -l; out[1] = n.y / -l; out[2] = n.z / -l; out[3] = 1.0f; }
                }
            }
    }
}

// ---- marching cubes: MarchingCubesData::extractIsoSurfaceAtPosition (MarchingCubesSDFUtil.h:119-227),
// literal, voxel by voxel, over the allocated blocks in heap order (the GPU build's output order; the
// reference kernel visits hash entries, CUDAMarchingCubesSDF.cu:15-27, and appends atomically).
namespace {

constexpr bf::McTables kMc = bf::make_mc_tables();

BFMcVertex vertexInterp(float isolevel, f3 p1, f3 p2, float d1, float d2, const uint8_t c1[4], const uint8_t c2[4]) {
    BFMcVertex r1, r2, res;
    r1.p[0] = p1.x; r1.p[1] = p1.y; r1.p[2] = p1.z;
    r1.c[0] = (float)c1[0] / 255.f; r1.c[1] = (float)c1[1] / 255.f; r1.c[2] = (float)c1[2] / 255.f;
    r2.p[0] = p2.x; r2.p[1] = p2.y; r2.p[2] = p2.z;
    r2.c[0] = (float)c2[0] / 255.f; r2.c[1] = (float)c2[1] / 255.f; r2.c[2] = (float)c2[2] / 255.f;
    if (std::fabs(isolevel - d1) < 0.00001f) return r1;
    if (std::fabs(isolevel - d2) < 0.00001f) return r2;
    if (std::fabs(d1 - d2) < 0.00001f) return r1;
    const float mu = (isolevel - d1) / (d2 - d1);
    res.p[0] = p1.x + mu * (p2.x - p1.x);
    res.p[1] = p1.y + mu * (p2.y - p1.y);
    res.p[2] = p1.z + mu * (p2.z - p1.z);
    res.c[0] = (float)(c1[0] + mu * (float)(c2[0] - c1[0])) / 255.f;
    res.c[1] = (float)(c1[1] + mu * (float)(c2[1] - c1[1])) / 255.f;
    res.c[2] = (float)(c1[2] + mu * (float)(c2[2] - c1[2])) / 255.f;
    return res;
}

void extractIsoSurfaceAtPosition(const Scene& s, const BFMarchingCubesParams& prm, f3 worldPos, std::vector<BFMcTriangle>& out) {
    if (prm.boxEnabled == 1) {  // isInBoxAA
        if (worldPos.x < prm.minCorner[0] || worldPos.x > prm.maxCorner[0]) return;
        if (worldPos.y < prm.minCorner[1] || worldPos.y > prm.maxCorner[1]) return;
        if (worldPos.z < prm.minCorner[2] || worldPos.z > prm.maxCorner[2]) return;
    }
    const float isolevel = 0.0f;
    const float P = s.hp.virtualVoxelSize / 2.0f;
    const float M = -P;
    uint8_t c[3];
    const f3 p000 = worldPos + mk(M, M, M); float dist000; const bool valid000 = trilinear(s, p000, dist000, c);
    const f3 p100 = worldPos + mk(P, M, M); float dist100; const bool valid100 = trilinear(s, p100, dist100, c);
    const f3 p010 = worldPos + mk(M, P, M); float dist010; const bool valid010 = trilinear(s, p010, dist010, c);
    const f3 p001 = worldPos + mk(M, M, P); float dist001; const bool valid001 = trilinear(s, p001, dist001, c);
    const f3 p110 = worldPos + mk(P, P, M); float dist110; const bool valid110 = trilinear(s, p110, dist110, c);
    const f3 p011 = worldPos + mk(M, P, P); float dist011; const bool valid011 = trilinear(s, p011, dist011, c);
    const f3 p101 = worldPos + mk(P, M, P); float dist101; const bool valid101 = trilinear(s, p101, dist101, c);
    const f3 p111 = worldPos + mk(P, P, P); float dist111; const bool valid111 = trilinear(s, p111, dist111, c);
    if (!valid000 || !valid100 || !valid010 || !valid001 || !valid110 || !valid011 || !valid101 || !valid111) return;
    uint32_t cubeindex = 0;
    if (dist010 < isolevel) cubeindex += 1;
    if (dist110 < isolevel) cubeindex += 2;
    if (dist100 < isolevel) cubeindex += 4;
    if (dist000 < isolevel) cubeindex += 8;
    if (dist011 < isolevel) cubeindex += 16;
    if (dist111 < isolevel) cubeindex += 32;
    if (dist101 < isolevel) cubeindex += 64;
    if (dist001 < isolevel) cubeindex += 128;
    const float thres = prm.threshMarchingCubes;
    const float distArray[] = {dist000, dist100, dist010, dist001, dist110, dist011, dist101, dist111};
    for (int k = 0; k < 8; k++)
        for (int l = 0; l < 8; l++) {
            if (distArray[k] * distArray[l] < 0.0f) {
                if (std::fabs(distArray[k]) + std::fabs(distArray[l]) > thres) return;
            } else {
                if (std::fabs(distArray[k] - distArray[l]) > thres) return;
            }
        }
    for (int k = 0; k < 8; k++)
        if (std::fabs(distArray[k]) > prm.threshMarchingCubes2) return;
    const uint32_t et = kMc.edges[cubeindex];
    if (et == 0 || et == 255) return;
    const BFVoxel v = getVoxelWorld(s, worldPos);
    BFMcVertex vertlist[12];
    if (et & 1) vertlist[0] = vertexInterp(isolevel, p010, p110, dist010, dist110, v.color, v.color);
    if (et & 2) vertlist[1] = vertexInterp(isolevel, p110, p100, dist110, dist100, v.color, v.color);
    if (et & 4) vertlist[2] = vertexInterp(isolevel, p100, p000, dist100, dist000, v.color, v.color);
    if (et & 8) vertlist[3] = vertexInterp(isolevel, p000, p010, dist000, dist010, v.color, v.color);
    if (et & 16) vertlist[4] = vertexInterp(isolevel, p011, p111, dist011, dist111, v.color, v.color);
    if (et & 32) vertlist[5] = vertexInterp(isolevel, p111, p101, dist111, dist101, v.color, v.color);
    if (et & 64) vertlist[6] = vertexInterp(isolevel, p101, p001, dist101, dist001, v.color, v.color);
    if (et & 128) vertlist[7] = vertexInterp(isolevel, p001, p011, dist001, dist011, v.color, v.color);
    if (et & 256) vertlist[8] = vertexInterp(isolevel, p010, p011, dist010, dist011, v.color, v.color);
    if (et & 512) vertlist[9] = vertexInterp(isolevel, p110, p111, dist110, dist111, v.color, v.color);
    if (et & 1024) vertlist[10] = vertexInterp(isolevel, p100, p101, dist100, dist101, v.color, v.color);
    if (et & 2048) vertlist[11] = vertexInterp(isolevel, p000, p001, dist000, dist001, v.color, v.color);
    for (int i = 0; i < 3 * kMc.ntri[cubeindex]; i += 3) {
        BFMcTriangle t;
        t.v[0] = vertlist[kMc.tri[cubeindex][i + 0]];
        t.v[1] = vertlist[kMc.tri[cubeindex][i + 1]];
        t.v[2] = vertlist[kMc.tri[cubeindex][i + 2]];
        out.push_back(t);
    }
}

}  // namespace

extern "C" void or_extract_mesh(const ORScene* o, const BFMarchingCubesParams* prm, BFMcTriangle* out, uint32_t cap,
                                uint32_t* n, uint32_t* total) {
    const Scene& s = o->s;
    std::vector<std::pair<int, i3>> blocks;  // allocated hash entries, by heap pointer
    for (const BFHashEntry& e : s.hash)
        if (e.ptr != BF_FREE_ENTRY) blocks.push_back({e.ptr, i3{e.x, e.y, e.z}});
    std::sort(blocks.begin(), blocks.end(), [](const std::pair<int, i3>& a, const std::pair<int, i3>& b) { return a.first < b.first; });
    std::vector<BFMcTriangle> tris;
    for (const auto& b : blocks)
        for (int z = 0; z < BF_SDF_BLOCK_SIZE; z++)
            for (int y = 0; y < BF_SDF_BLOCK_SIZE; y++)
                for (int x = 0; x < BF_SDF_BLOCK_SIZE; x++) {
                    // SDFBlockToVirtualVoxelPos(entry.pos) + threadIdx, virtualVoxelPosToWorld
                    const i3 pi = {b.second.x * BF_SDF_BLOCK_SIZE + x, b.second.y * BF_SDF_BLOCK_SIZE + y, b.second.z * BF_SDF_BLOCK_SIZE + z};
                    const f3 worldPos = mk((float)pi.x, (float)pi.y, (float)pi.z) * s.hp.virtualVoxelSize;
                    extractIsoSurfaceAtPosition(s, *prm, worldPos, tris);
                }
    const uint32_t cnt = (uint32_t)std::min<size_t>(tris.size(), cap);
    if (out && cnt) std::memcpy(out, tris.data(), sizeof(BFMcTriangle) * cnt);
    if (n) *n = cnt;
    if (total) *total = (uint32_t)tris.size();
}

extern "C" void or_mc_tables(uint16_t* edges, uint8_t* ntri, uint8_t* tri) {  // the compiled case tables
    for (int c = 0; c < 256; c++) {
        edges[c] = kMc.edges[c];
        ntri[c] = kMc.ntri[c];
        for (int k = 0; k < 15; k++) tri[c * 15 + k] = kMc.tri[c][k];
    }
}
