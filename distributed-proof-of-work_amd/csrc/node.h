// node.h -- internal entry points of the node search shared by dpow_api.cpp and board.cpp
// (not part of the C ABI).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "../../include/dpow.h"

namespace dpow {

// dpow_node_vote; a non-NULL abort_flag that is raised ends the wait with DPOW_CANCELLED.
int node_vote(dpow_node_vote_entry *votes, uint32_t rank, uint32_t world, uint64_t epoch, const int64_t in[3],
              int64_t out[3], int64_t timeout_ns, const uint32_t *abort_flag);

// dpow_node_mine; abandon_on_cancel: a rank whose cancel flag is raised leaves without voting.
// role 0: search this rank's partition (dpow_node_mine); 1: search every partition of the node's
// window (worker_bits 0: the node's ranks share this rank's GPU); 2: search nothing, only vote (a
// role-1 rank of the same node covers this rank's partition).
int node_mine(dpow_ctx *c, dpow_node_slot *slot, dpow_node_vote_entry *votes, uint32_t rank, uint32_t world,
              uint64_t *epoch, int64_t vote_timeout_ns, const uint8_t *nonce, size_t nonce_len, uint32_t ntz,
              uint64_t k_begin, uint64_t k_limit, uint64_t first_k, uint64_t batch_k, uint64_t *best_global_idx,
              uint8_t *secret_out, size_t *secret_len, uint32_t *batches, bool abandon_on_cancel, int role);

// The GPU of ctx across the processes of a host (a hash of its PCI bus id, never 0).
uint64_t device_key(const dpow_ctx *c);

// The context searches every partition of a node whose ranks share its GPU (dpow_board_search):
// the young-search rule (plan.h kYoungNs) does not share the device with the idle ranks.
void set_solo(dpow_ctx *c, bool solo);

// Sets dpow_last_error for the calling thread and returns code.
int fail(int code, const char *msg);

}  // namespace dpow
