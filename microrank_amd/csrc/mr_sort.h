#pragma once
#include "mr_internal.h"

struct SortScratch {
    DBuf<uint64_t> k2;
    DBuf<uint32_t> v2;
    DBuf<int64_t> hist, tmp;
};

// Stable sort of keys[0..n) on their low `bits` bits; vals (nullable) move with the keys.
int mr_radix_sort(mr_ctx* ctx, uint64_t* keys, uint32_t* vals, int64_t n, int bits, SortScratch& ws);
int bits_for(uint64_t maxval);
