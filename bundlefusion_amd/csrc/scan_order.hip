// scan_order.hip — the order in which the batch scan (k_compactify_ops) visits the heap blocks: the allocated
// blocks of [0, n) sorted by the Morton code of their block coordinates, every other slot after them, positions
// >= n unchanged (identity). The scan reads blockPos[order[j]] for j in [0, highWater); any permutation of
// [0, highWater) visits every allocated block exactly once, so the lists it builds (visible list, work list) hold
// the same blocks in another order, and the voxel results do not change. What the order buys: a wave's 64
// blocks lie together in space, so the wave's box pre-cull against each op's frustum rejects most ops at once,
// and consecutive work-list entries (the voxel pass hands runs of them to one XCD) gather from the same
// depth / colour lines. Heap order (allocation order, reused slots after GC) scatters a wave over the room.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "bf_runtime.h"
#include "scan_order.h"

namespace bf {

namespace {

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit of 30
    v &= 0x3FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

// key of heap slot i: Morton code of the block (coordinates offset by 512, 10 bits each: a 32 m cube at 4 mm
// voxels; beyond it the codes wrap, which costs locality, not correctness), 0xFFFFFFFF for a free slot
__global__ __launch_bounds__(256) void k_scan_keys(const int4* __restrict__ blockPos, uint32_t n, uint32_t* keys) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int4 b = blockPos[i];
        keys[i] = b.w ? (spread10((uint32_t)(b.x + 512)) | (spread10((uint32_t)(b.y + 512)) << 1) |
                         (spread10((uint32_t)(b.z + 512)) << 2))
                      : 0xFFFFFFFFu;
    }
}

__global__ __launch_bounds__(256) void k_iota(uint32_t* v, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) v[i] = i;
}

}  // namespace

void ScanOrder::init(uint32_t numBlocks, hipStream_t s) {
    B_ = numBlocks;
    order_.alloc(numBlocks);
    iota_.alloc(numBlocks);
    keys_.alloc(numBlocks);
    keysOut_.alloc(numBlocks);
    size_t bytes = 0;
    BF_HIP(rocprim::radix_sort_pairs(nullptr, bytes, keys_.p, keysOut_.p, iota_.p, order_.p, numBlocks, 0, 32, s));
    temp_.alloc(std::max<size_t>(bytes, 16));
    k_iota<<<1024, 256, 0, s>>>(iota_.p, numBlocks);
    BF_LAUNCH_CHECK();
    reset(s);
}

void ScanOrder::reset(hipStream_t s) {
    BF_HIP(hipMemcpyAsync(order_.p, iota_.p, sizeof(uint32_t) * B_, hipMemcpyDeviceToDevice, s));
}

void ScanOrder::sort(const int4* blockPos, uint32_t n, hipStream_t s) {
    n = std::min(n, B_);
    if (n < 2) return;
    k_scan_keys<<<std::min(1024u, (n + 255) / 256), 256, 0, s>>>(blockPos, n, keys_.p);
    BF_LAUNCH_CHECK();
    size_t bytes = temp_.n;
    // stable: the free slots (key 0xFFFFFFFF) keep ascending slot order after the allocated ones
    BF_HIP(rocprim::radix_sort_pairs(temp_.p, bytes, keys_.p, keysOut_.p, iota_.p, order_.p, n, 0, 32, s));
}

}  // namespace bf
