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
// Returns the entry's ptr or BF_FREE_ENTRY. The bucket's four {pos, ptr} words and the last slot's offset
// are loaded together (one memory round trip; the slot-by-slot form waited for each slot's two halves in
// turn, up to eight dependent loads per lookup); the list, rare, is walked entry by entry.
#ifndef BF_HASH_SERIAL
#define BF_HASH_SERIAL 0  // 1: the slot-by-slot form (A/B builds)
#endif
__device__ inline int hash_lookup(const BFHashEntry* hash, uint32_t numBuckets, uint32_t numEntries, uint32_t maxList,
                                  int x, int y, int z) {
    const uint32_t h = hash_bucket(x, y, z, numBuckets);
    const uint32_t hp = h * BF_HASH_BUCKET_SIZE;
#if BF_HASH_SERIAL
    for (int j = 0; j < BF_HASH_BUCKET_SIZE; j++) {
        int4 a, b;
        hash_load_entry(hash, hp + j, a, b);
        if (a.x == x && a.y == y && a.z == z && a.w != BF_FREE_ENTRY) return a.w;
    }
    uint32_t i = hp + BF_HASH_BUCKET_SIZE - 1;
    for (uint32_t it = 0; it < maxList; it++) {
        int4 a, b;
        hash_load_entry(hash, i, a, b);
        if (a.x == x && a.y == y && a.z == z && a.w != BF_FREE_ENTRY) return a.w;
        if (b.x == 0) break;
        i = (hp + BF_HASH_BUCKET_SIZE - 1 + (uint32_t)b.x) % numEntries;
    }
    return BF_FREE_ENTRY;
#endif
    const int4* p = reinterpret_cast<const int4*>(hash + hp);
    int4 e[BF_HASH_BUCKET_SIZE];
#pragma unroll
    for (int j = 0; j < BF_HASH_BUCKET_SIZE; j++) e[j] = p[2 * j];
    uint32_t off = (uint32_t)reinterpret_cast<const int*>(p + 2 * (BF_HASH_BUCKET_SIZE - 1) + 1)[0];
#pragma unroll
    for (int j = 0; j < BF_HASH_BUCKET_SIZE; j++)
        if (e[j].x == x && e[j].y == y && e[j].z == z && e[j].w != BF_FREE_ENTRY) return e[j].w;
    const uint32_t last = hp + BF_HASH_BUCKET_SIZE - 1;
    for (uint32_t it = 1; it < maxList; it++) {
        if (off == 0) break;
        const uint32_t i = (last + off) % numEntries;
        int4 a, b;
        hash_load_entry(hash, i, a, b);
        if (a.x == x && a.y == y && a.z == z && a.w != BF_FREE_ENTRY) return a.w;
        off = (uint32_t)b.x;
    }
    return BF_FREE_ENTRY;
}

}  // namespace bf
