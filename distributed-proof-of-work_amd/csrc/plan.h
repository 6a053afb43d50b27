// plan.h -- host planning of search windows into kernel launches.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/dpow.h"
#include "dpow_common.h"

namespace dpow {

struct PlannedLaunch {
    dpow_plan_launch info;
    Launch L;  // ctrl / cancel / done_target / iters filled at launch time
};

uint32_t chunk_len_of(uint64_t k);
uint64_t segment_end(uint64_t k);
uint32_t remainder_bits(uint32_t worker_bits);
uint32_t base_thread_byte(uint32_t worker_byte, uint32_t worker_bits);

// Returns the number of launches, or a negative DPOW_E* code.
int plan_window(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                uint32_t worker_bits, uint64_t k_begin, uint64_t k_end, std::vector<PlannedLaunch> &out);

void candidate_words(const PlannedLaunch &pl, uint64_t local_idx, uint32_t words[32]);

}  // namespace dpow
