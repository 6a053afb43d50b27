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
    Launch L;  // ctrl / cancel / claim / chunk / done_target filled at launch time
    // k = 0 (the chunk of zero bytes, msg = nonce || threadByte): hashed by the search's
    // k = 0 kernel (search_ctrl.hip), not by an md5 launch; L.iv / L.T hold its message.
    bool k0 = false;
};

uint32_t chunk_len_of(uint64_t k);
uint64_t segment_end(uint64_t k);
// k-period of word W0 + 2's chunk bytes for byte shift SH (0: launch-uniform
// or a kernel segment word); the planner ends launches on its multiples.
uint64_t word2_period(uint32_t sh);
// The planner may merge chunk lengths 1..3 (k in [1, 2^24)) into one launch: SH = 0
// layouts, R >= 2, equal block counts (WindowPlanner::next).
constexpr uint64_t kLspanMaxExpect = 1ull << 28;
uint64_t lspan_end(size_t nonce_len, uint32_t rbits, uint32_t ntz);
uint32_t remainder_bits(uint32_t worker_bits);
uint32_t base_thread_byte(uint32_t worker_byte, uint32_t worker_bits);

// Incremental planner: one launch at a time, so a window of any size costs
// O(1) host memory.  init() returns 0 or a negative DPOW_E* code.
class WindowPlanner {
   public:
    int init(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte, uint32_t worker_bits,
             uint64_t k_begin, uint64_t k_end);
    bool next(PlannedLaunch &out);  // false when the window is covered
    // Re-plan from k (the start of the launch next() last returned) with that launch at
    // most max_k k long (no chunk-length merging past it): dpow_search's launches while
    // the device is shared.
    void restart(uint64_t k, uint64_t max_k) {
        k_ = k;
        cap_k_ = max_k;
    }

   private:
    uint32_t nblk_of(uint32_t chunk_len) const;
    bool lseg_template(uint64_t k) const;  // the launch's template is chunk length 0's (SH = 0, k < lspan_end_)
    void build_template(uint64_t k, uint32_t chunk_len, uint32_t nblk, uint32_t T[32]) const;
    const uint8_t *nonce_ = nullptr;
    size_t nonce_len_ = 0, blk_v_ = 0;
    uint32_t p_ = 0, ntz_ = 0, rbits_ = 0, base_tb_ = 0;
    uint64_t k_ = 0, k_end_ = 0;
    uint64_t cap_k_ = 0;  // one-shot length cap of the next launch (restart), 0: none
    uint64_t lspan_end_ = 0;  // launches below this k use the chunk-length-0 template and may span
    uint32_t iv_[4] = {0, 0, 0, 0};
};

// Returns the number of launches, or a negative DPOW_E* code.
int plan_window(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                uint32_t worker_bits, uint64_t k_begin, uint64_t k_end, std::vector<PlannedLaunch> &out);

void candidate_words(const PlannedLaunch &pl, uint64_t local_idx, uint32_t words[32]);

// Claim geometry of a launch (dpow_search; CPU-testable through
// dpow_diag_launch_geometry): chunk sizes, the guided tail, the claim count and
// the worker workgroups (at most max_blocks, at least one per claim counter that
// holds a claim); a launch spanning 2^24-k segments gets its wave-blocks counted
// from a multiple of a power-of-two chunk, so no claim straddles a segment.
// Fills pl.L.{wb_begin, n_wblocks, chunk, chunk_tail, n_big, n_chunks, n_head};
// returns 0, or DPOW_EINVAL if a claim counter would be left without waves.
constexpr uint64_t kClaimsPerWave = 16;   // big claims per wave (chunk sizing)
constexpr uint64_t kMinChunk = 4;         // wave-blocks per claim: at least ...
#ifndef DPOW_MAX_CHUNK
#define DPOW_MAX_CHUNK 32
#endif
constexpr uint64_t kMaxChunk = DPOW_MAX_CHUNK;  // ... and at most
#ifndef DPOW_TAIL_CLAIMS
#define DPOW_TAIL_CLAIMS 2  // small claims per wave at the end of a launch (0: none; A/B switch)
#endif
constexpr uint64_t kTailClaimsPerWave = DPOW_TAIL_CLAIMS;
#ifndef DPOW_TAIL_CHUNK
#define DPOW_TAIL_CHUNK 4  // wave-blocks per tail claim (at most the launch's chunk; A/B switch)
#endif
constexpr uint64_t kTailChunk = DPOW_TAIL_CHUNK;
static_assert((kMinChunk & (kMinChunk - 1)) == 0 && (kMaxChunk & (kMaxChunk - 1)) == 0 &&
                  (kTailChunk & (kTailChunk - 1)) == 0 && kTailChunk <= kMinChunk,
              "chunk bounds are powers of two (segment alignment)");
// expect: candidates of the launch expected before its first hit (expected_first_hit;
// ~0 = none): chunks are sized so that >= kClaimsPerWave claims per wave come before it.
// min_chunk: a power of two (diagnostic override of kMinChunk, dpow_api.cpp); claims_per_wave:
// diagnostic override of kClaimsPerWave.
int size_launch(PlannedLaunch &pl, uint64_t max_blocks, uint64_t expect, uint64_t *worker_blocks,
                uint64_t min_chunk = kMinChunk, uint64_t claims_per_wave = kClaimsPerWave);
// Mean number of a partition's candidates before its first hit at N trailing zeros.
uint64_t expected_first_hit(uint32_t ntz, uint32_t rbits);

// Wave-blocks per poll group (Launch::poll_wb).  A wave reads Ctrl::best / Ctrl::stop
// once per group, issued before the group and consumed after it, so a hit elsewhere,
// an injected bound (the node board) or a cancel reaches it within two groups.  Long
// groups cost less issue (DPOW_POLL_WB = 16 for searches expected to run for more than
// kFastPollCands candidates -- the sweep, N >= 9), short ones (kFastPollWb) shorten the
// drain after a hit when the whole search is expected to be short.
#ifndef DPOW_POLL_WB
#define DPOW_POLL_WB 16  // (also md5_search_kernel.h)
#endif
// Round 4 (the early Found fan-out, the claim-ahead in a chunk's last group): searches
// expected beyond kMidExpect poll every 8 wave-blocks (round 3: 4), those up to it every 4.
// An 8-GPU node, emulated (tools/node_probe.py, profiles/r04_node_ab.log r04ab6): [2,2,2,2]/8
// 0.354 -> 0.323 ms, [1,2,3,4]/8 2.67 -> 2.63 ms with every launch at 8.
#ifndef DPOW_FAST_POLL_WB
#define DPOW_FAST_POLL_WB 8
#endif
#ifndef DPOW_MID_POLL_WB
#define DPOW_MID_POLL_WB 4
#endif
// Hits expected within kNearExpect (2^24: one GPU's N = 6, a 2- or 4-GPU rank's N = 6) often lie among the chunks every wave claims first, and the waves above
// the hit hash a whole group before they see it: groups of 2 (round 4,
// profiles/r04_small_probe/: one GPU's [1,2,3,4]/6 0.064-0.073 -> 0.052-0.053 ms at 4 per
// CU; over 24 fresh nonces at N = 6 0.137-0.138 -> 0.141-0.143 ms).
#ifndef DPOW_NEAR_POLL_WB
#define DPOW_NEAR_POLL_WB 2
#endif
constexpr uint64_t kNearExpect = 1ull << 24;
constexpr uint32_t kFastPollWb = DPOW_FAST_POLL_WB;
constexpr uint32_t kMidPollWb = DPOW_MID_POLL_WB;
constexpr uint32_t kNearPollWb = DPOW_NEAR_POLL_WB;
constexpr uint64_t kFastPollCands = 1ull << 30;
uint32_t launch_poll_wb(uint32_t ntz, uint32_t rbits);
// Tiny searches -- a first hit expected within kTinyExpect candidates of the partition (N <= 5
// on one GPU, N = 6 on a rank of a 2-, 4- or 8-GPU node): 2 workgroups per CU, claims of >= 2
// wave-blocks, a poll of Ctrl::best after every wave-block.  There the launch's fixed cost
// -- the waves' first chunks, the drain behind the hit -- outweighs its hashing: each wave
// of a lightly loaded SIMD finishes a wave-block sooner.  Measured over the BASELINE cases
// and 24 fresh nonces each (tools/small_search_probe.py, profiles/r03_small_probe.json):
// [5,6,7,8]/5 0.040 -> 0.025 ms, fresh N = 5 0.044 -> 0.035 ms, an 8-GPU rank's
// [1,2,3,4]/6 0.043 -> 0.026 ms.  (Round 4 tried ending the tier at 2^20, moving an 8-GPU
// rank's N = 6 to 3 workgroups per CU and claims of 4: the emulated node's [1,2,3,4]/6 went
// 0.046 -> 0.056 ms, profiles/r04_small_probe/; not kept.)
// Round 5: the tier reaches 2^23 expected (a 2-GPU rank's N = 6, a 4-GPU rank's 2^22); the
// emulated node's G2 [1,2,3,4]/6 0.045 -> 0.038 ms (one GPU's 0.043: 0.93 -> 1.13x), G4 0.038
// -> 0.034, nothing else moved (profiles/r05_ab.json[r05z_tiny/]).  A launch is tiny by its
// size only up to kTinyLaunch (2^21, round 4's bound), so short windows of a search expected
// late keep their grids.
#ifndef DPOW_TINY_EXPECT_LOG2
#define DPOW_TINY_EXPECT_LOG2 23
#endif
constexpr uint64_t kTinyExpect = 1ull << DPOW_TINY_EXPECT_LOG2;
constexpr uint64_t kTinyLaunch = 1ull << 21;
// Up to kMidExpect (N = 6 on one GPU, N = 7 on a rank of a 4- or 8-GPU node): 4 workgroups
// per CU.  The rate is ~6 % below the full grid's, but a rank that another rank's hit
// stops drains in half the time: stop latency at N = 7 on an 8-GPU rank's window 103 ->
// 52 us (tools/small_search_probe.py --stop, profiles/r03_stop_probe.json), while the owner's
// own search is no slower (0.225 -> 0.212 ms).
constexpr uint64_t kMidExpect = 1ull << 26;
// Up to kFiveExpect (N = 8 on a rank of an 8-GPU node, N = 7 on one GPU): 5 workgroups per CU.
// The SIMD's arbiter issues the oldest wave first, and with 6 waves per SIMD the youngest
// barely progress: the chunks they claimed at the start hold up a first hit below them and the
// drain behind it (tools/wave_trace_node.py: the owner of [2,2,2,2]/8 on an 8-GPU node hashed
// 170 wave-blocks in its oldest waves and 20 in its youngest, whose first chunk took 250 us and
// ended 70 us after the hit).  5 per CU costs the rate ~0.8 %.
#ifndef DPOW_FIVE_EXPECT_LOG2
#define DPOW_FIVE_EXPECT_LOG2 31  // 0: off (A/B switch)
#endif
constexpr uint64_t kFiveExpect = DPOW_FIVE_EXPECT_LOG2 ? 1ull << DPOW_FIVE_EXPECT_LOG2 : 0;
constexpr uint64_t kTinyChunk = 2;
// Claims of at least kMidChunk wave-blocks for hits expected in (kMidChunkExpect, kMidExpect]
// (round 3: kMinChunk = 4): half the claims, and with the claim-ahead in a chunk's last group
// the chunk's first group polls without waiting for the claim atomic.  Emulated 8-GPU node
// (profiles/r04_node_ab.log r04ab7): [1,2,3,4]/7 0.266-0.270 -> 0.251-0.261 ms, its owner
// 0.217-0.223 -> 0.196-0.204 ms.  Not below: every wave's first two claims at 4 per CU and
// 8 wave-blocks cover 2^23 candidates, and a hit inside them waits for its larger chunk
// (one GPU's [1,2,3,4]/6, 2^24 expected: 0.064-0.075 -> 0.079-0.082 ms with chunks of 8).
#ifndef DPOW_MID_CHUNK
#define DPOW_MID_CHUNK 8
#endif
constexpr uint64_t kMidChunk = DPOW_MID_CHUNK;
constexpr uint64_t kMidChunkExpect = 1ull << 24;
uint64_t launch_min_chunk(uint32_t ntz, uint32_t rbits);
// Claims per wave (chunk sizing) of a search expected to end within kFastPollCands
// candidates: 64 (smaller chunks), else kClaimsPerWave.  A rank that another rank's hit stops
// must finish every chunk below it, so the chunk sets its drain: an 8-GPU rank's stop at
// N = 8 186 -> 139 us, its owner's search 2.510 -> 2.517 ms (profiles/r03_cpw_probe.json).
constexpr uint64_t kShortClaimsPerWave = 64;
uint64_t launch_claims_per_wave(uint32_t ntz, uint32_t rbits);

// Worker workgroups per CU for one launch (before the device share).  The full
// persistent grid (kMaxBlocksPerCu = 6) has the highest rate, but a launch that is
// short -- few candidates, or a first hit expected early (16^N candidates of the
// whole enumeration, 16^N R / 256 of this partition) -- finishes sooner with fewer
// waves: 3 per CU up to 2^22 expected candidates, 4 up to 2^24
// (profiles/r02_ab_blocks.log, r02_ab_grid/: time-to-secret N = 6 0.22 -> 0.15 ms, N = 5 0.104 ->
// 0.086 ms; windows of 2^22 / 2^24 candidates 50 -> 43 / 120 -> 110 us).
#ifndef DPOW_BLOCKS_PER_CU
#define DPOW_BLOCKS_PER_CU 6
#endif
constexpr uint64_t kMaxBlocksPerCu = DPOW_BLOCKS_PER_CU;
// share: searches in flight on the device (dpow_api.cpp g_active).  Such a search runs at
// 1/share of the device, so the tiers judge its launch by device time: candidates and the
// expected first hit times share.  BASELINE config 4 (8 logical workers on one GPU, N = 8,
// 2^29 expected each) keeps the full grid.
uint64_t launch_blocks_per_cu(uint64_t candidates, uint32_t ntz, uint32_t rbits, uint64_t share = 1);

// The whole sizing of one dpow_search launch, shared by dpow_search and the geometry
// diagnostic (dpow_diag_launch_geometry), so the diagnostic checks the grids searches run:
// the device share of cus x launch_blocks_per_cu workgroups (at least one per claim
// counter), size_launch with the ntz-dependent expected first hit, minimum chunk and
// claims per wave, and the poll group (L.poll_wb).  Non-zero knobs override the policy
// (the DPOW_DIAG_* A/B environment of dpow_open).
struct LaunchKnobs {
    uint32_t bpc = 0, min_chunk = 0, cpw = 0, poll_wb = 0;
    uint32_t share_launch_us = 0;  // launch length on a shared device (kShareLaunchNs)
    uint32_t share_max = 0;        // grid share cap (kShareMax)
};
// share: the grid is 1/share of the device's; active (>= share): the searches in flight on the
// device, which set the launch's device time (launch_blocks_per_cu).
int size_search_launch(PlannedLaunch &pl, uint32_t ntz, uint64_t cus, uint64_t share, const LaunchKnobs &knobs,
                       uint64_t *worker_blocks, uint64_t active = 1);

// Searches sharing a device (dpow_api.cpp g_active): the coordinator mirror's logical workers
// on one GPU (BASELINE configs 3-5: 4 or 8 workers per GPU in the 1-GPU bench).
//  - A grid is sized once per launch, so while the device is shared a launch lasts about
//    kShareLaunchNs at 1/active of the device's rate (cap_shared_launch): grids follow searches
//    that start or end beside it.  (One launch per window kept a grid sized for a crowd after
//    the crowd was gone: the last of 4 searches ran 47 ms on 1 workgroup per CU.)  8 ms: 8
//    concurrent searches at 210-212 GH/s with 2 ms launches, 213-214 at 4, 215-216 at 8 and
//    16 (each launch boundary costs its queue a drain); config 4 over fresh nonces the same
//    (profiles/r04_share/r04capab/).
//  - A grid is 1/min(active, kShareMax) of the device (grid_share).  The HIP runtime maps a
//    process's streams onto GPU_MAX_HW_QUEUES (4) hardware queues, and the kernels of streams
//    sharing a queue run one after the other: grids of 1/active left the device part-idle.
//    Each search's grid at 1/2 keeps it full across launch boundaries (8 concurrent searches of
//    2^31 candidates: 163-168 GH/s at 1/8, 197 at 1/4, 210-215 at 1/2; BASELINE config 4 over
//    16 fresh nonces 29.8 -> 20.1 ms mean, profiles/r04_share/).
#ifndef DPOW_SHARE_MAX
#define DPOW_SHARE_MAX 2
#endif
#ifndef DPOW_SHARE_LAUNCH_US
#define DPOW_SHARE_LAUNCH_US 8000
#endif
constexpr uint64_t kShareMax = DPOW_SHARE_MAX;
// A search younger than kYoungNs that is alone on its device while other contexts of its
// process were used there within kRecentNs (opened, or a search started: dpow_api.cpp
// recent_contexts) plans its launches for all of them: searches that start together -- the
// coordinator mirror's workers -- then share the device from their first launch, instead of
// the first to register taking one uncapped full-device launch (round 4).  Contexts idle in a
// pool for longer do not count, nor does the rank that searches a whole node's
// window on a shared GPU (dpow_board_search: its co-located ranks only vote).  A process with
// one context per device (a node rank, the bench) is unaffected.
#ifndef DPOW_YOUNG_US
#define DPOW_YOUNG_US 2000
#endif
constexpr int64_t kYoungNs = (int64_t)DPOW_YOUNG_US * 1000;
constexpr int64_t kRecentNs = 100 * 1000 * 1000;
constexpr int64_t kShareLaunchNs = (int64_t)DPOW_SHARE_LAUNCH_US * 1000;
constexpr double kEstRate = 2.3e11;  // candidates/s of one device (bench: 217-218 on the one-block layouts)
uint64_t grid_share(uint64_t active, const LaunchKnobs &knobs);
// Re-plans pl (the launch planner.next() last returned) to at most kShareLaunchNs of hashing
// when active > 1; returns whether it did.
bool cap_shared_launch(WindowPlanner &planner, PlannedLaunch &pl, uint64_t active, const LaunchKnobs &knobs);

}  // namespace dpow
