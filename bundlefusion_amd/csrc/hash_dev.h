// hash_dev.h — device-side hash lookup shared by the TSDF kernels and the raycaster.
#pragma once
#include "bf_math.h"

namespace bf {

__device__ __forceinline__ void hash_load_entry(const BFHashEntry* h, uint32_t i, int4& a, int4& b) {
    const int4* p = reinterpret_cast<const int4*>(h + i);
    a = p[0];
    b = p[1];
}

// getHashEntryForSDFBlockPos (VoxelUtilHashSDF.h:440-485): the 4 bucket slots, then the linked
// list that starts at the bucket's last slot (offset relative to it, wrap mod E, <= maxList hops).
// Returns the entry's ptr or BF_FREE_ENTRY.
__device__ inline int hash_lookup(const BFHashEntry* hash, uint32_t numBuckets, uint32_t numEntries, uint32_t maxList,
                                  int x, int y, int z) {
    const uint32_t h = hash_bucket(x, y, z, numBuckets);
    const uint32_t hp = h * BF_HASH_BUCKET_SIZE;
#pragma unroll
    for (int j = 0; j < BF_HASH_BUCKET_SIZE; j++) {
        int4 a, b;
        hash_load_entry(hash, hp + j, a, b);
        if (a.x == x && a.y == y && a.z == z && a.w != BF_FREE_ENTRY) return a.w;
    }
    const uint32_t last = hp + BF_HASH_BUCKET_SIZE - 1;
    uint32_t i = last;
    for (uint32_t it = 0; it < maxList; it++) {
        int4 a, b;
        hash_load_entry(hash, i, a, b);
        if (a.x == x && a.y == y && a.z == z && a.w != BF_FREE_ENTRY) return a.w;
        if (b.x == 0) break;
        i = (last + (uint32_t)b.x) % numEntries;
    }
    return BF_FREE_ENTRY;
}

}  // namespace bf
