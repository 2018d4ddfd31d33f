// One filtered caller's allow list as a slot bitmap (the micro-batcher,
// batcher.hip -> k_pqa_from_rows): bit i of word i >> 5 = slot i = doc id
// id_base + i.  host: the caller's page-locked row; dev: the same memory
// mapped for kernels (read in place); n: the list's length (its select depth).
#pragma once
#include <cstdint>

struct wv_batch_row {
    const uint32_t* dev;
    const uint32_t* host;
    int64_t words;
    int64_t n;
};
