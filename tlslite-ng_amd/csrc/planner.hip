// planner.hip -- processing order for batches of mixed record lengths.
//
// The batch kernels give each record one lane, so a wave takes as long as
// its longest record.  With mixed lengths (BASELINE config 4: Zipf 64 B -
// 16 KiB) almost every wave of 64 random records holds a 16 KiB one and the
// lanes of the short ones idle.  Launching the records longest first, in the
// order of a descending radix sort of their lengths (rocPRIM, on the stream
// of the launch), gives every wave records of nearly equal length; the
// kernels read record order[t] for thread t.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "common.h"

// scratch == nullptr: *bytes = what a batch of n needs.  Layout: sorted keys
// (n u32) | rocPRIM temporary storage.
int tg_length_order(const uint32_t* len, uint64_t n, uint32_t* order, void* scratch, size_t* bytes,
                    hipStream_t s) {
    size_t tmp = 0;
    rocprim::counting_iterator<uint32_t> iota(0);
    if (rocprim::radix_sort_pairs_desc(nullptr, tmp, len, (uint32_t*)nullptr, iota, (uint32_t*)nullptr,
                                       (size_t)n, 0, 32, s) != hipSuccess)
        return TG_EHIP;
    const size_t keys = (n * sizeof(uint32_t) + 255) & ~(size_t)255;
    if (!scratch) {
        *bytes = keys + tmp;
        return TG_OK;
    }
    if (*bytes < keys + tmp) return TG_EINVAL;
    uint32_t* keys_out = static_cast<uint32_t*>(scratch);
    void* t = static_cast<uint8_t*>(scratch) + keys;
    if (rocprim::radix_sort_pairs_desc(t, tmp, len, keys_out, iota, order, (size_t)n, 0, 32, s) !=
        hipSuccess)
        return TG_EHIP;
    return TG_OK;
}
