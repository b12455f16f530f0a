// scan_order.h — the batch scan's visiting order of the heap blocks (scan_order.hip): a permutation of the heap
// slots, the allocated ones of [0, n) sorted by the Morton code of their block coordinates.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bf_runtime.h"

namespace bf {

class ScanOrder {
public:
    void init(uint32_t numBlocks, hipStream_t s);  // identity order
    void reset(hipStream_t s);                     // identity order (scene reset)
    // re-sort the slots [0, n) (n <= every later highWater: the order stays a permutation of [0, highWater))
    void sort(const int4* blockPos, uint32_t n, hipStream_t s);
    const uint32_t* order() const { return order_.p; }
    size_t deviceBytes() const { return order_.bytes() + iota_.bytes() + keys_.bytes() + keysOut_.bytes() + temp_.bytes(); }

private:
    uint32_t B_ = 0;
    DevBuf<uint32_t> order_, iota_, keys_, keysOut_;
    DevBuf<uint8_t> temp_;
};

}  // namespace bf
