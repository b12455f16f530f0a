// corr.h — the EntryJ producer (corr.hip) with caller-owned scratch and stream: the FriedLiver app runs it
// at every submap boundary on its input stream, without device allocations (whose frees synchronize the
// whole device) and without the null stream.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/bf/bf.h"
#include "bf_runtime.h"

namespace bf {

struct CorrScratch {
    DevBuf<BFEntryJ> slots;   // [pairs][maxPerPair]
    DevBuf<uint32_t> counts;  // [pairs]
    DevBuf<uint32_t> total;   // [1]
    DevBuf<uint2> pairs;      // (i, cur) per pair
    uint32_t* hostTotal = nullptr;  // pinned
    ~CorrScratch() {
        if (hostTotal) (void)hipHostFree(hostTotal);
    }
    void reserve(uint32_t npairs, uint32_t maxPerPair);
};

// EntryJ of the image pairs list[0..npairs) ((i, cur) each; host array), packed in list order (per pair the
// first maxPerPair matches in candidate order, a pair with fewer than o.minPerPair contributes none): what
// AddCurrToResidualsCU appends for each pair in turn. Queued on stream; waits for it (the count goes to the
// host). Returns the records written (<= cap); *total = all records found.
uint32_t corr_from_pairs(const float* const* depth, const float* T, const float* Tinv, const uint2* list, uint32_t npairs,
                         const BFCorrOptions& o, BFEntryJ* out, uint32_t cap, uint32_t* total, hipStream_t stream,
                         CorrScratch& scratch);

}  // namespace bf
