// md5_search_kernel.h -- the gfx950 proof-of-work search kernel (instantiated
// per message layout by md5_variant.hip).
//
// Replaces the reference miner's inner loop (worker.go:318-400): for every
// candidate threadByte || chunk_k of the worker partition, MD5(nonce || it) and
// the trailing-'0' test of its hex form.  Pure INT32 VALU work: each lane runs
// an unrolled, register-resident MD5 of the final message block(s) of two
// candidates, software-pipelined in hand-ordered asm groups (see pipe::), the
// message words being wave-uniform (kernel arguments, SGPRs) except the 4 bytes
// threadByte | k_lo << 8, and the bytes of k >> 24 (L >= 4), which change once
// per 2^24-k segment of a launch (the segment words, re-derived per wave).
//
// Work decomposition: local index i = k * R + t (the reference's order, k outer,
// t inner).  A wave-block is 64 * kNC consecutive indices (lane l, slot j ->
// i0 + 64 j + l).  Worker waves of a persistent grid claim chunks of
// consecutive wave-blocks from 8 per-XCD counters, each in increasing order;
// the first hit of a wave-block (lowest slot, then lowest lane) goes to
// atomicMin on the global index g = k * 256 + threadByte, which is monotone in
// i, so the minimum is the reference's first hit.  A wave stops at the first
// chunk, or group of DPOW_POLL_WB wave-blocks within one, whose first index is
// >= the current minimum, so every candidate below the answer is evaluated and
// the result is deterministic.
//
// Workgroup 0 of the grid is a watcher: one lane polls the pinned host cancel
// flag (Found/Cancel, worker.go:194,209) and raises Ctrl::stop, which every
// worker wave reads every DPOW_POLL_WB wave-blocks together with Ctrl::best.  The workgroup that
// retires last writes the launch's completion record (Snap) to pinned host
// memory, which the host polls.
#pragma once
#include <hip/hip_runtime.h>

#include "dpow_common.h"

// DPOW_VLS = 1 (md5_variant.hip's "_ls" translation units): the SH = 0 kernels of launches
// below k = 2^24, whose template is chunk length 0's and which may span chunk lengths 1..3
// (Launch::seg0 == kLsegBase): the pad word W0 + 1 and the bit-length word are segment
// words.  0: every other launch.  Separate kernels, in their own namespace: holding the
// bit-length word's K + M in VGPRs cost the sweep kernel 2 % through register assignment
// alone, with an identical instruction count (217.3 -> 214.0 GH/s in an A/B early in round 3;
// that log did not survive the session).
#ifndef DPOW_VLS
#define DPOW_VLS 0
#endif
#if DPOW_VLS
#define DPOW_KNS lsk
#else
#define DPOW_KNS k
#endif

namespace dpow {
namespace DPOW_KNS {

#define DPOW_DEV __device__ __forceinline__
#define DPOW_DEV_CONST __host__ __device__ constexpr

// SGPR budget: <= 80 allocated SGPRs admit 8 four-wave workgroups per CU
// (8 waves per SIMD, MI355X_MICROARCH.md "Residency").  Literal K constants are
// rematerialised by SALU moves, which co-issue beside other waves' VALU.  The budgets are
// tuning values (tools/isa_loop.py builds with others); DESIGN.md records the A/B
// measurements of the alternatives that were removed from this file in round 6.
#ifndef DPOW_NUM_SGPR
#define DPOW_NUM_SGPR 72
#endif
#ifndef DPOW_NUM_SGPR_LONG
#define DPOW_NUM_SGPR_LONG 96  // long-nonce and two-block layouts (kNumSgpr below)
#endif
#ifndef DPOW_NUM_SGPR_W15
#define DPOW_NUM_SGPR_W15 100  // two-block layouts at W0 = 15 (kW15Sgpr below)
#endif
constexpr int kSgprLongW0 = 8;
// The watcher's poll interval, s_sleep units of 64 cycles (round 4: 32).
constexpr int kWatchSleep = 16;
// A wave polls Ctrl::best / Ctrl::stop once per group of Launch::poll_wb wave-blocks
// of a chunk (the host's choice: plan.h launch_poll_wb; DPOW_POLL_WB = 16 for long
// searches).  profiles/r01_ab_poll.log: once per chunk / 12 / 16 / 32 wave-blocks
// -> 216.3 / 217.8 / 218.3 / 218.6 GH/s, time-to-secret N=7 1.57 / 1.47 / 1.49 / 1.56 ms.
#ifndef DPOW_POLL_WB
#define DPOW_POLL_WB 16
#endif
// Retirement counted per claim counter, then on Ctrl::done: in the chunk-length-spanning
// units only -- the launches of short searches, below k = 2^24 -- so that the other units'
// kernels (the sweep's among them) keep their code.
constexpr bool kXcdRetire = DPOW_VLS != 0;
// Static first claims (the "_ls" kernels: the short launches below k = 2^24 that the
// time-to-secret path runs): worker wave w's first claim is chunk w, so a wave starts
// hashing without waiting for a contended counter -- at 4 workgroups per CU the start-up
// burst of 8k claim atomics on 8 counters held the median wave 5 us and the slowest 10 us
// before its first wave-block (tools/wave_trace_tts.py).  Its claim-ahead atomic then
// hides behind that first chunk.  The counters hand out chunks from Launch::n_static on.
// (plan.cpp sets Launch::n_static for exactly those launches.)
constexpr bool kStaticFirst = DPOW_VLS != 0;
// Diagnostic builds only (tools/wave_trace.py, tools/wave_trace_node.py): every worker wave
// records kTraceFields words -- {start, first claim, exit} in s_memrealtime ticks (100 MHz),
// its hashed wave-blocks, the start of its last chunk and that chunk's claim index, why it
// left the claim loop (1 counters drained, 2 a chunk at or above the best, 3 stop) and when
// it found a hit of its own (0: none) -- read back with dpow_diag_wave_trace.
#ifndef DPOW_WAVE_TRACE
#define DPOW_WAVE_TRACE 0
#endif
#if DPOW_WAVE_TRACE
constexpr uint32_t kTraceWaves = 8192;
constexpr uint32_t kTraceFields = 8;
static __device__ unsigned long long g_wave_trace[kTraceWaves * kTraceFields];
#endif

template <int I>
DPOW_DEV uint32_t md5_fn(uint32_t x, uint32_t y, uint32_t z) {
    constexpr int r = I / 16;
    constexpr uint32_t tt = r == 0 ? kBop3F : r == 1 ? kBop3G : r == 2 ? kBop3H : kBop3I;
    return __builtin_amdgcn_bitop3_b32(x, y, z, tt);
}

// Launch-uniform K + M constants kept in VGPRs (every lane the same value).
// Layouts with long nonces need up to ~50 distinct K + M constants in the
// pipelined steps (every nonce word, four times per block).  Under the 80-SGPR
// budget of 8 waves/SIMD the compiler spills them to VGPR lanes and reloads
// each with a v_readlane -- a VALU instruction -- on every use (28-54 per
// wave-block in the two-block kernels).  Copied once per wave into VGPRs with
// an opaque v_mov (so they are not folded back to SGPRs), they cost nothing in
// the loop: v_add3_u32 reads a VGPR operand at the same rate.  Capped so the
// kernel stays within 64 VGPRs (8 waves/SIMD).

struct KConst {
    uint32_t v[128];  // [64 * BLK + I]; only the entries VgprK selects are set
};

// Segment words: the message word(s) holding the chunk bytes above k's low 24
// bits (byte p + 4 on; k >> 24 is one byte for L = 4, two for L = 5).  They
// are launch-uniform within a 2^24-k segment, and a launch spans segments
// (plan.cpp), so their K + M constants are re-derived per wave when it enters
// another segment: word W0 + 1 always, W0 + 2 when SH = 3 (the two-byte field
// of L = 5 crosses into it).
static_assert(DPOW_POLL_WB > 0, "the chunk loop polls per group of wave-blocks");
// For SH != 0 word W0 + 1 also holds the top bytes of V; its K + M is then
// wave-uniform per wave-block anyway (VarWords::hi_s, which carries the
// segment addition too), so only SH = 0's W0 + 1 and SH = 3's W0 + 2 are
// VGPR-held segment words.
// SH = 0 kernels also serve launches spanning chunk-length segments (Launch::lspan):
// there the bit-length word (16 NBLK - 2) and W0 + 1 (the pad of L = 3) change per segment.
template <int NBLK, int W0, int SH>
DPOW_DEV_CONST bool seg_word(int m) {
    return (SH == 0 && m == W0 + 1) || (SH == 3 && m == W0 + 2 && m != 16 * NBLK - 2) ||
           (DPOW_VLS && SH == 0 && (m == W0 + 1 || m == 16 * NBLK - 2));
}

// First hand-ordered step of block 0: W0 + pipe_lead<NBLK, W0, SH>.  4 is the first
// step whose four state words are all per-lane; before it the compiler schedules
// the steps (some state words are wave-uniform there, and it exploits that).
// Which start issues best depends on the layout; the table is the argmax of a
// per-layout sweep of builds with one start for every layout
// (one start for every layout, 1..6: tools/lead_sweep.py, profiles/r02_lead_sweep.json),
// where a start beats 4 by >= 0.8 %.  The headline <1,1,0> keeps 4.
// The build choices of the narrow SH = 3 kernels (hash_wave_block KSPAN = false, the kernels of
// launches with R >= 64): pipe start (0: the general kernel's), VGPR-constant cap (0: the
// general's), kLaunchPoll (-1: the general's) and SGPR budget class (-1: the general's; 1 = 96,
// 2 = 100).  Each row is the per-layout argmax of round 6's same-box sweeps of builds with one
// choice for every narrow kernel (tools/lead_sweep.py; profiles/r06_narrow_sweep.json).  on =
// false: no narrow build beat the layout's general kernel (<1,0,3>), or the layout was not swept
// (<1,12..13,3>: chunks below 2^24 only), so it runs the general kernel for every R.
struct NarrowKnobs {
    bool on;
    int lead, cap, poll, sgpr;
};
constexpr NarrowKnobs narrow_knobs(int nblk, int w0) {
    if (nblk == 1) {
        switch (w0) {
            case 1: case 2: case 3: case 5: case 6: case 11:
                    return {true, 2, 0, 0, 1};
            case 4: return {true, 1, 0, -1, -1};
            case 7: return {true, 2, 0, -1, 1};
            case 8: return {true, 3, 0, 0, -1};
            case 9: return {true, 4, 0, -1, -1};
            case 10: return {true, 2, 0, 0, -1};
            default: return {false, 0, 0, -1, -1};
        }
    }
    switch (w0) {
        case 12: return {true, 3, 0, 0, -1};
        case 13: return {true, 3, 0, -1, -1};
        case 14: return {true, 2, 24, -1, -1};
        case 15: return {true, 2, 0, 0, -1};
        default: return {false, 0, 0, -1, -1};
    }
}
// A/B builds only: one choice for every narrow kernel, over the table (tools/lead_sweep.py)
#ifndef DPOW_NLEAD
#define DPOW_NLEAD 0   // pipe start
#endif
#ifndef DPOW_NCAP
#define DPOW_NCAP 0    // VGPR-constant cap
#endif
#ifndef DPOW_NPOLL
#define DPOW_NPOLL -1  // kLaunchPoll 0 / 1
#endif
#ifndef DPOW_NSGPR
#define DPOW_NSGPR 0   // SGPR budget class 1 / 2
#endif

constexpr int pipe_lead(int nblk, int w0, int sh, bool narrow = false) {
    if (narrow) {
        const int lead = DPOW_NLEAD > 0 ? DPOW_NLEAD : narrow_knobs(nblk, w0).lead;
        if (lead > 0) return lead;
    }
    // (round 4: the same sweep over the round-4 kernels, profiles/r04_lead_sweep.json, moved the
    // entries marked r4 -- a start that beats the table's by >= 1 % -- and dropped <1,10,1..2>'s
    // 3, now 7.4 % below 4)
    if (nblk == 1) {
        switch (w0 * 4 + sh) {
            case 0 * 4 + 0: return 2;  // +1.3 %
            case 0 * 4 + 3: return 2;  // r4 +1.1 %
            case 2 * 4 + 0: return 3;  // +2.0 %
            case 2 * 4 + 1: return 1;  // r4 +1.2 % (round 2: 2)
            case 2 * 4 + 2: return 1;  // r4 +1.2 % (round 2: 2)
            case 3 * 4 + 0: return 3;  // +2.2 %
            case 3 * 4 + 1: return 3;  // r4 +1.2 %
            case 3 * 4 + 2: return 3;  // r4 +1.1 %
            case 3 * 4 + 3: return 1;  // +2.0 %
            case 4 * 4 + 0: return 2;  // r4 +1.5 %
            case 4 * 4 + 3: return 2;  // +1.0 %
            case 6 * 4 + 3: return 2;  // r4 +1.4 %
            case 8 * 4 + 3: return 3;  // +2.2 %
            case 9 * 4 + 0: return 2;  // +3.7 %
            case 9 * 4 + 1: return 3;  // r4 +2.3 %
            case 9 * 4 + 2: return 3;  // r4 +2.3 %
            case 9 * 4 + 3: return 3;  // +1.6 %
            case 10 * 4 + 3: return 5; // +1.8 %
            default: return 4;
        }
    }
    switch (w0 * 4 + sh) {
        case 12 * 4 + 3: return 1;  // +4.3 %
        case 14 * 4 + 1: return 2;  // +5.0 %
        case 14 * 4 + 2: return 2;  // +5.1 %
        case 14 * 4 + 3: return 1;  // +4.3 %
        case 15 * 4 + 0: return 2;  // +4.5 %
        case 15 * 4 + 1: return 2;  // r4 +2.2 %
        case 15 * 4 + 2: return 2;  // r4 +2.3 %
        case 15 * 4 + 3: return 1;  // +5.7 %
        default: return 4;
    }
}

// KS: the KSPAN argument of the kernel (hash_wave_block); kNarrow = SH = 3's narrow kernel.
template <int NBLK, int W0, int SH, bool KS = true>
struct VgprK {
    static constexpr bool kNarrow = SH == 3 && !KS;
    // First step of block 0 in the hand-ordered pipeline (md5_tail's kI0 for
    // the hash loop's ONLY_D call with kNC candidates).
    static constexpr int kEnd0 = NBLK == 1 ? 62 : 64;
    static constexpr int kLead = pipe_lead(NBLK, W0, SH, kNarrow);
    static constexpr int kI0 = W0 + kLead < kEnd0 ? W0 + kLead : kEnd0;
    // Steps the hash loop runs (ONLY_D: the last block stops after step 61).
    static constexpr bool run(int blk, int i) { return !(blk == NBLK - 1 && i >= 62); }
    // Steps reading a segment word: always held in VGPRs (updated at segment changes).
    static constexpr bool seg(int blk, int i) { return seg_word<NBLK, W0, SH>(16 * blk + md5_word(i)) && run(blk, i); }
    static constexpr bool eligible(int blk, int i) {
        const int m = 16 * blk + md5_word(i);
        const bool zero = m > W0 + 2 && m != 16 * NBLK - 2;
        const bool lane = m == W0 || (SH != 0 && m == W0 + 1);
        const bool piped = blk > 0 || i >= kI0;
        return !zero && !lane && piped && run(blk, i) && !seg(blk, i);
    }
    static constexpr int rank(int blk, int i) {
        int r = 0;
        for (int b = 0; b < NBLK; ++b)
            for (int j = 0; j < 64; ++j) {
                if (b == blk && j == i) return r;
                if (eligible(b, j)) ++r;
            }
        return r;
    }
    static constexpr int count() { return rank(NBLK, 0); }
    static constexpr int count_seg() {
        int r = 0;
        for (int b = 0; b < NBLK; ++b)
            for (int j = 0; j < 64; ++j) r += seg(b, j) ? 1 : 0;
        return r;
    }
    // VGPRs the layout uses without VGPR constants (-Rpass-analysis=kernel-resource-usage):
    // one block 34-39 (SH = 0) / 43-49 (SH != 0), two blocks 41-43 / 49-53; each
    // constant costs about one more.  The grid runs 6 waves per SIMD, so up to 80
    // VGPRs cost no occupancy that is used; the caps keep every kernel within 72
    // (7 waves: a queued launch's workgroups still start beside a draining one).
    // The segment-word constants count against them first.  Round 1's caps for
    // <= 64 VGPRs (14 one-block / 10 two-block for SH != 0) left the two-block
    // layouts with 4-11 SGPR spill reloads per wave-block.
    // (round 4, profiles/r04_lead_sweep.json: a cap of 24 for <1,7,1..2> +1.9-2.0 %,
    // <1,4,3> +1.5 %, <1,5,3> +1.0 %; elsewhere it is no better, or costs up to 3 %)
    static constexpr bool kCap24 = NBLK == 1 && ((W0 == 7 && (SH == 1 || SH == 2)) || (SH == 3 && (W0 == 4 || W0 == 5)));
    static constexpr int kNarrowCap = DPOW_NCAP > 0 ? DPOW_NCAP : narrow_knobs(NBLK, W0).cap;
    static constexpr int kCap = kNarrow && kNarrowCap > 0 ? kNarrowCap
                                : kCap24 ? 24
                                : NBLK == 1 ? (SH == 0 ? 24 : SH == 3 ? 14 : 18)
                                            : (SH == 3 ? 20 : 26);
    static constexpr bool use(int blk, int i) {
        return seg(blk, i) || (eligible(blk, i) && rank(blk, i) < kCap - count_seg());
    }
};

template <int NBLK, int W0, int SH, int BLK, int I, bool KS>
DPOW_DEV void kconst_init(KConst &kc, const Launch &L) {
    if constexpr (BLK < NBLK) {
        if constexpr (VgprK<NBLK, W0, SH, KS>::use(BLK, I))
            asm("v_mov_b32 %0, %1" : "=v"(kc.v[64 * BLK + I]) : "s"(L.KT[64 * BLK + I]));
        if constexpr (I + 1 < 64) kconst_init<NBLK, W0, SH, BLK, I + 1, KS>(kc, L);
        else kconst_init<NBLK, W0, SH, BLK + 1, 0, KS>(kc, L);
    }
}

// Additions to the segment words (W0 + 1, W0 + 2) for 2^24-k segment `seg`
// (dpow_common.h seg_word_deltas).
template <int W0, int SH>
DPOW_DEV void seg_deltas(const Launch &L, uint32_t seg, uint32_t &d1, uint32_t &d2) {
    seg_word_deltas(L.T[W0 + 1], L.T[W0 + 2], seg, L.seg_first, SH, d1, d2);
}

// Addition to segment word m: d[0] to W0 + 1, d[1] to W0 + 2, d[2] to the bit-length word
// (where W0 + 1 is the bit-length word, plan.cpp puts the whole difference in d[2]).
template <int NBLK, int W0>
DPOW_DEV uint32_t seg_add(int m, const uint32_t (&d)[3]) {
    return m == 16 * NBLK - 2 ? d[2] : m == W0 + 1 ? d[0] : d[1];
}

// The segment-word additions of segment sg (seg_id): for SH = 0 below k = 2^24 the
// chunk-length deltas against the template's chunk length 0 (lseg_deltas: no Launch field is
// read -- plain kernarg reads here were hoisted out of the claim loop into SGPRs and pushed
// its wave-uniform index arithmetic onto the VALU, +10 VALU per wave-block in <1,1,0>,
// tools/isa_loop.py), else the 2^24-k field (seg_word_deltas); d0 = the addition to W0.
template <int NBLK, int W0, int SH>
DPOW_DEV void seg_all_deltas(const Launch &L, uint32_t sg, uint32_t &d0, uint32_t (&d)[3]) {
    d0 = d[0] = d[1] = d[2] = 0u;
    if (sg >= kLsegBase) {
        if constexpr (SH == 0 && DPOW_VLS) {
            lseg_deltas((sg - kLsegBase) & 3u, d0, d[0], d[2]);
            if constexpr (W0 + 1 == 16 * NBLK - 2) {  // W0 + 1 is the bit-length word
                d[2] += d[0];
                d[0] = 0u;
            }
        }
    } else {
        seg_deltas<W0, SH>(L, sg, d[0], d[1]);
    }
}

// Re-derive the VGPR-held K + M constants of the segment words (wave-uniform,
// once per segment change: a rare branch).
template <int NBLK, int W0, int SH, int BLK, int I, bool KS>
DPOW_DEV void kconst_seg(KConst &kc, const Launch &L, const uint32_t (&d)[3]) {
    if constexpr (BLK < NBLK) {
        if constexpr (VgprK<NBLK, W0, SH, KS>::seg(BLK, I)) {
            constexpr int m = 16 * BLK + md5_word(I);
            const uint32_t k = L.KT[64 * BLK + I] + seg_add<NBLK, W0>(m, d);
            asm volatile("v_mov_b32 %0, %1" : "=v"(kc.v[64 * BLK + I]) : "s"(k));
        }
        if constexpr (I + 1 < 64) kconst_seg<NBLK, W0, SH, BLK, I + 1, KS>(kc, L, d);
        else kconst_seg<NBLK, W0, SH, BLK + 1, 0, KS>(kc, L, d);
    }
}

// Per-candidate variable message parts.  KSPAN: the lanes may span several k (R < 64), so
// SH = 3's word W0 + 1 differs per lane (lane_k); without it that word's K + M is wave-uniform.
template <bool KSPAN>
struct VarWords {
    static constexpr bool kSpan = KSPAN;
    uint32_t lo_s[kNC];  // wave-uniform part of V << 8*SH (word W0)
    uint32_t lo_v;       // per-lane part of V << 8*SH (the same for every slot)
    uint32_t hi_s[kNC];  // SH != 0: the wave-uniform part of word W0+1's addition -- V >> (32 - 8 SH)
                         //  (uniform: a lane's k offset never carries into those bits) plus the
                         //  segment addition d1
    uint32_t lane_k;     // SH = 3: the per-lane part of V >> 8 (the lane's k offset; 0 when R >= 64,
                         //  and not read without KSPAN)
    const KConst *kc;    // launch-uniform K + M constants held in VGPRs (segment words: current segment)
    uint32_t seg_d[3];   // segment-word additions (seg_add) for the steps that read them from L.KT
                         //  (full_check's steps 62-63 of the last block only; the hash loop holds them
                         //  all in kc)
};

// K + M of step I of block BLK for candidate j (the message word M includes the
// candidate's variable bytes when the step reads word W0, or W0 + 1 for SH != 0).
template <int NBLK, int W0, int SH, int BLK, int I, bool KS>
struct StepWord {
    static constexpr int m = 16 * BLK + md5_word(I);
    // Words past the variable bytes, the chunk tail and the 0x80 pad -- every
    // word after W0 + 2 except the bit-length word -- are zero for every launch
    // of this layout (plan.cpp), so K + M folds to the literal K: no SGPR.
    static constexpr bool zero_word = m > W0 + 2 && m != 16 * NBLK - 2;
    static constexpr bool per_lane = m == W0 || (SH == 3 && KS && m == W0 + 1);  // K + M differs per lane
    static constexpr bool vgpr_k = VgprK<NBLK, W0, SH, KS>::use(BLK, I);
    static constexpr bool seg = seg_word<NBLK, W0, SH>(m);
    static DPOW_DEV uint32_t km(const Launch &L, const VarWords<KS> &v, int j) {
        uint32_t k = zero_word ? kMd5K[I] : vgpr_k ? v.kc->v[64 * BLK + I] : L.KT[64 * BLK + I];
        if constexpr (seg && !vgpr_k) k += seg_add<NBLK, W0>(m, v.seg_d);
        if constexpr (m == W0) k = (k + v.lo_s[j]) + v.lo_v;
        if constexpr (SH != 0 && m == W0 + 1) {
            k += v.hi_s[j];                        // SALU: K + M stays uniform
            if constexpr (SH == 3 && KS) k += v.lane_k;  // the one VALU add of the step
        }
        return k;
    }
};

// Steps [I, IE) of block BLK for NCAND candidates, left to the compiler.
template <int NBLK, int W0, int SH, int BLK, int I, int IE, int NCAND, class V>
DPOW_DEV void md5_steps(uint32_t (&x)[4][kNC], const Launch &L, const V &v) {
    if constexpr (I < IE) {
        constexpr int ai = (64 - I) % 4, bi = (ai + 1) % 4, ci = (ai + 2) % 4, di = (ai + 3) % 4;
        constexpr int s = md5_shift(I);
#pragma unroll
        for (int j = 0; j < NCAND; ++j) {
            const uint32_t km = StepWord<NBLK, W0, SH, BLK, I, V::kSpan>::km(L, v, j);
            const uint32_t f = md5_fn<I>(x[bi][j], x[ci][j], x[di][j]);
            x[ai][j] = x[bi][j] + __builtin_rotateleft32(x[ai][j] + f + km, s);
        }
        md5_steps<NBLK, W0, SH, BLK, I + 1, IE, NCAND>(x, L, v);
    }
}

// ---------------------------------------------------------------------------
// Two candidates, issue order fixed by hand.  Each MD5 step is four VALU
// instructions, two full rate (v_bitop3_b32, v_add_u32) and two half rate
// (v_add3_u32, v_alignbit_b32), strictly dependent within a candidate.
// Candidate q runs half a step behind candidate p and the two chains alternate
// instruction by instruction (DPOW_PIPE_BODY below), with s_nop padding after
// the half-rate instructions.  One asm statement per step pair: the compiler
// keeps the order, allocates the registers and places the SALU moves of the K
// constants, and adds no padding of its own inside the group (these plain VALU
// ops are interlocked in hardware; one asm statement per instruction got a
// conservative s_nop after every VOP3).  Against the compiler-scheduled loop:
// 170 -> 214.7 GH/s.  The probes that led here are dpow_diag_valu_rate kinds
// 20-27 (profiles/r01_valu_probe_order.log).
namespace pipe {

template <int I>
constexpr uint32_t tt() {
    return I / 16 == 0 ? kBop3F : I / 16 == 1 ? kBop3G : I / 16 == 2 ? kBop3H : kBop3I;
}

template <int I> struct Roles {
    static constexpr int a = (64 - I) % 4, b = (a + 1) % 4, c = (a + 2) % 4, d = (a + 3) % 4;
};

// Wait states after each instruction kind of a group (-1: none).  A VALU
// instruction issued right behind the one it depends on holds the SIMD's issue
// for the whole dependency latency -- every wave on the SIMD waits -- while an
// s_nop holds only its own wave and lets the other waves issue; the padding
// after the half-rate instructions pays even where nothing depends on them.
// Measured on the sweep (order 1, profiles/r01_ab_nop.log): no padding 170 GH/s;
// s_nop 0 after each rotate 192.5; plus s_nop 0 / 1 / 2 / 3 after each add3
// 200.7 / 203.6 / 209.1 / 205.4; s_nop 1 after the rotate instead 191; any
// padding after the full-rate ops 168-185; no rotate padding 179-180.  Order 2
// (profiles/r01_ab_order.log): the same s_nop 0 / s_nop 2 is best, 214.7; no
// padding 170.7; add3 padding 1 or 3: 210.
#define DPOW_PAD_R "s_nop 0\n\t"  // after v_alignbit_b32 (the rotate; the next add reads it)
#define DPOW_PAD_A "s_nop 2\n\t"  // after v_add3_u32

// Order of a step pair (B bop3, A add3, R rotate, D add; p at step I, q finishing
// step I-1 then starting step I): p.B q.R p.A q.D p.R q.B p.D q.A -- the two chains
// strictly alternate, so every dependency is two instructions apart (F H H F H F F H);
// 214.7 GH/s.  (p.B q.R q.D p.A q.B p.R p.D q.A -- F and H strictly alternate, but each
// rotate sits right before its add -- 209.1 GH/s; two pairs interleaved at NC = 4 with
// both properties, every dependency >= 3 apart: 191 GH/s at best.
// profiles/r01_ab_order.log.)
#define DPOW_PIPE_BODY                                        \
    "v_bitop3_b32 %[fp], %[pb], %[pc], %[pd] bitop3:%[tt]\n\t" \
    "v_alignbit_b32 %[rq], %[tq], %[tq], %[sq]\n\t" DPOW_PAD_R \
    "v_add3_u32 %[tp], %[pa], %[fp], %[kp]\n\t" DPOW_PAD_A     \
    "v_add_u32_e32 %[qb], %[qc], %[rq]\n\t"                   \
    "v_alignbit_b32 %[tp], %[tp], %[tp], %[sp]\n\t" DPOW_PAD_R \
    "v_bitop3_b32 %[fq], %[qb], %[qc], %[qd] bitop3:%[tt]\n\t" \
    "v_add_u32_e32 %[pa], %[pb], %[tp]\n\t"                   \
    "v_add3_u32 %[tq], %[qa], %[fq], %[kq]\n\t" DPOW_PAD_A

#define DPOW_PIPE_PRO                                         \
    "v_bitop3_b32 %[fp], %[pb], %[pc], %[pd] bitop3:%[tt]\n\t" \
    "v_add3_u32 %[tp], %[pa], %[fp], %[kp]\n\t" DPOW_PAD_A     \
    "v_bitop3_b32 %[fq], %[qb], %[qc], %[qd] bitop3:%[tt]\n\t" \
    "v_alignbit_b32 %[tp], %[tp], %[tp], %[sp]\n\t" DPOW_PAD_R \
    "v_add_u32_e32 %[pa], %[pb], %[tp]\n\t"                   \
    "v_add3_u32 %[tq], %[qa], %[fq], %[kq]\n\t" DPOW_PAD_A

// One step pair of candidates p = J, q = J + 1 at step I (q finishes step I-1,
// whose add3 is in tq, and starts step I).  p's state word a is written in the
// middle of the group (`+&v`, early-clobber): where the pipeline starts before
// W0 + 4, p's and q's state words can still be the same wave-uniform value, and a
// plain `+v` lets the register allocator hand q's input that same register, which
// the group then overwrites before q reads it (a wrong hash in <1,0,0> at start
// W0 + 2, caught by test_nonce_lengths_golden / tools/layout_check.py).
template <int NBLK, int W0, int SH, int BLK, int I, int J, class V>
DPOW_DEV void body(uint32_t (&x)[4][kNC], uint32_t &tq, const Launch &L, const V &v) {
    using R = Roles<I>;  // q's step I-1 writes x[R::b][q] from x[R::c][q]
    using W = StepWord<NBLK, W0, SH, BLK, I, V::kSpan>;
    const uint32_t kp = W::km(L, v, J), kq = W::km(L, v, J + 1);
    uint32_t fp, fq, rq, tp;
    if constexpr (W::per_lane || W::vgpr_k)
        asm volatile(DPOW_PIPE_BODY
                     : [pa] "+&v"(x[R::a][J]), [qb] "=&v"(x[R::b][J + 1]), [tq] "+v"(tq), [fp] "=&v"(fp),
                       [fq] "=&v"(fq), [rq] "=&v"(rq), [tp] "=&v"(tp)
                     : [pb] "v"(x[R::b][J]), [pc] "v"(x[R::c][J]), [pd] "v"(x[R::d][J]), [qc] "v"(x[R::c][J + 1]),
                       [qd] "v"(x[R::d][J + 1]), [qa] "v"(x[R::a][J + 1]), [kp] "v"(kp), [kq] "v"(kq),
                       [tt] "i"(tt<I>()), [sp] "i"(32 - md5_shift(I)), [sq] "i"(32 - md5_shift(I - 1)));
    else
        asm volatile(DPOW_PIPE_BODY
                     : [pa] "+&v"(x[R::a][J]), [qb] "=&v"(x[R::b][J + 1]), [tq] "+v"(tq), [fp] "=&v"(fp),
                       [fq] "=&v"(fq), [rq] "=&v"(rq), [tp] "=&v"(tp)
                     : [pb] "v"(x[R::b][J]), [pc] "v"(x[R::c][J]), [pd] "v"(x[R::d][J]), [qc] "v"(x[R::c][J + 1]),
                       [qd] "v"(x[R::d][J + 1]), [qa] "v"(x[R::a][J + 1]), [kp] "s"(kp), [kq] "s"(kq),
                       [tt] "i"(tt<I>()), [sp] "i"(32 - md5_shift(I)), [sq] "i"(32 - md5_shift(I - 1)));
}

// Prologue of a pair at its first pipelined step I0: q's step I0 is left half done.
template <int NBLK, int W0, int SH, int BLK, int I0, int J, class V>
DPOW_DEV void prologue(uint32_t (&x)[4][kNC], uint32_t &tq, const Launch &L, const V &v) {
    using R = Roles<I0>;
    using W = StepWord<NBLK, W0, SH, BLK, I0, V::kSpan>;
    const uint32_t kp = W::km(L, v, J), kq = W::km(L, v, J + 1);
    uint32_t fp, fq, tp;
    if constexpr (W::per_lane || W::vgpr_k)
        asm volatile(DPOW_PIPE_PRO
                     : [pa] "+&v"(x[R::a][J]), [tq] "=&v"(tq), [fp] "=&v"(fp), [fq] "=&v"(fq), [tp] "=&v"(tp)
                     : [pb] "v"(x[R::b][J]), [pc] "v"(x[R::c][J]), [pd] "v"(x[R::d][J]), [qb] "v"(x[R::b][J + 1]),
                       [qc] "v"(x[R::c][J + 1]), [qd] "v"(x[R::d][J + 1]), [qa] "v"(x[R::a][J + 1]), [kp] "v"(kp),
                       [kq] "v"(kq), [tt] "i"(tt<I0>()), [sp] "i"(32 - md5_shift(I0)));
    else
        asm volatile(DPOW_PIPE_PRO
                     : [pa] "+&v"(x[R::a][J]), [tq] "=&v"(tq), [fp] "=&v"(fp), [fq] "=&v"(fq), [tp] "=&v"(tp)
                     : [pb] "v"(x[R::b][J]), [pc] "v"(x[R::c][J]), [pd] "v"(x[R::d][J]), [qb] "v"(x[R::b][J + 1]),
                       [qc] "v"(x[R::c][J + 1]), [qd] "v"(x[R::d][J + 1]), [qa] "v"(x[R::a][J + 1]), [kp] "s"(kp),
                       [kq] "s"(kq), [tt] "i"(tt<I0>()), [sp] "i"(32 - md5_shift(I0)));
}

constexpr int kPairs = kNC / 2;

// Step pairs I .. IE-1 of every candidate pair, the pairs' groups interleaved.
template <int NBLK, int W0, int SH, int BLK, int I, int IE, class V>
DPOW_DEV void run(uint32_t (&x)[4][kNC], uint32_t (&tq)[kPairs], const Launch &L, const V &v) {
    if constexpr (I < IE) {
        body<NBLK, W0, SH, BLK, I, 0>(x, tq[0], L, v);
        if constexpr (kPairs > 1) body<NBLK, W0, SH, BLK, I, 2>(x, tq[1], L, v);
        run<NBLK, W0, SH, BLK, I + 1, IE>(x, tq, L, v);
    }
}

// Steps [I0, IE) of block BLK for all candidates in the alternating order.
template <int NBLK, int W0, int SH, int BLK, int I0, int IE, class V>
DPOW_DEV void steps(uint32_t (&x)[4][kNC], const Launch &L, const V &v) {
    static_assert(kNC == 2 || kNC == 4, "the pipelined path runs one or two candidate pairs");
    if constexpr (I0 < IE) {
        uint32_t tq[kPairs];
        prologue<NBLK, W0, SH, BLK, I0, 0>(x, tq[0], L, v);
        if constexpr (kPairs > 1) prologue<NBLK, W0, SH, BLK, I0, 2>(x, tq[1], L, v);
        run<NBLK, W0, SH, BLK, I0 + 1, IE>(x, tq, L, v);
        // epilogue: each q finishes step IE-1
        using E = Roles<IE - 1>;
#pragma unroll
        for (int p = 0; p < kPairs; ++p)
            x[E::a][2 * p + 1] = x[E::b][2 * p + 1] + __builtin_rotateleft32(tq[p], md5_shift(IE - 1));
    }
}

#undef DPOW_PIPE_BODY
#undef DPOW_PIPE_PRO
#undef DPOW_PAD_R
#undef DPOW_PAD_A

}  // namespace pipe

// Final-block compression(s) of NCAND candidates; returns the digest words.
// With ONLY_D the last block stops after step 61, which writes D (steps 62-63
// only feed A..C): out[3] is exact, out[0..2] are not computed.  With RAW_D
// (one final block) out[3] is the state word without the chaining value:
// D = iv[3] + out[3], which the D-equality test compares against -iv[3].
template <int NBLK, int W0, int SH, int NCAND, bool ONLY_D = false, bool RAW_D = false, class V>
DPOW_DEV void md5_tail(uint32_t (&out)[4][kNC], const Launch &L, const V &v) {
    static_assert(!RAW_D || (ONLY_D && NBLK == 1), "RAW_D: D word of one final block");
    uint32_t x[4][kNC];
#pragma unroll
    for (int j = 0; j < NCAND; ++j) {
        x[0][j] = L.iv[0]; x[1][j] = L.iv[1]; x[2][j] = L.iv[2]; x[3][j] = L.iv[3];
    }
    // The hand-ordered pipeline starts at step W0 + pipe_lead of the first block
    // (all four state words are per-lane from W0 + 4 on; earlier steps are
    // wave-uniform or partly so, and the compiler folds them).
    constexpr bool kPipe = NCAND == kNC && (kNC == 2 || kNC == 4);
    constexpr int kEnd0 = (ONLY_D && NBLK == 1) ? 62 : 64;
    constexpr int kLead = VgprK<NBLK, W0, SH, V::kSpan>::kLead;
    constexpr int kI0 = kPipe ? (W0 + kLead < kEnd0 ? W0 + kLead : kEnd0) : kEnd0;
    md5_steps<NBLK, W0, SH, 0, 0, kI0, NCAND>(x, L, v);
    if constexpr (kPipe) pipe::steps<NBLK, W0, SH, 0, kI0, kEnd0>(x, L, v);
#pragma unroll
    for (int j = 0; j < NCAND; ++j)
#pragma unroll
        for (int w = 0; w < 4; ++w) out[w][j] = (RAW_D && w == 3) ? x[w][j] : L.iv[w] + x[w][j];
    if constexpr (NBLK == 2) {
        constexpr int kEnd1 = ONLY_D ? 62 : 64;
#pragma unroll
        for (int j = 0; j < NCAND; ++j)
#pragma unroll
            for (int w = 0; w < 4; ++w) x[w][j] = out[w][j];
        if constexpr (kPipe)
            pipe::steps<NBLK, W0, SH, 1, 0, kEnd1>(x, L, v);
        else
            md5_steps<NBLK, W0, SH, 1, 0, kEnd1, NCAND>(x, L, v);
#pragma unroll
        for (int j = 0; j < NCAND; ++j)
#pragma unroll
            for (int w = 0; w < 4; ++w) out[w][j] += x[w][j];
    }
}

// V = vs + loff (wave-uniform + per-lane) of slot j.  The lane offset holds the
// thread-byte bits below R and the k bits below 64 / R; vs is zero in both
// (i0 is a multiple of 64), so the sum never carries and V's bits above the
// lane's k offset are wave-uniform: V >> 24 and V >> 16 are uniform, and
// V >> 8 = (vs >> 8) + (loff >> 8).  d1 = the segment addition to word W0 + 1.
template <int SH, class V>
DPOW_DEV void var_words(V &v, int j, uint32_t vs, uint32_t loff, uint32_t d1) {
    v.lo_s[j] = vs << (8 * SH);
    v.lo_v = loff << (8 * SH);
    if constexpr (SH != 0) {
        v.hi_s[j] = (vs >> (32 - 8 * SH)) + d1;
        v.lane_k = SH == 3 && V::kSpan ? loff >> 8 : 0u;
    } else {
        v.hi_s[j] = 0u;
        v.lane_k = 0u;
    }
}

// Full digest test of one lane's candidate (rare path: only when the D-word
// test passed and ntz > 8, i.e. probability 2^-32 per candidate).
// loff: the lane offset, plus (SH = 0) the segment's addition to word W0 (search_body lov);
// sd: the segment's word additions (seg_all_deltas), computed by the caller outside the
// per-lane branch (a dynamic kernarg index inside it moved the hash loop's wave-uniform
// index arithmetic onto the VALU: +10 VALU per wave-block in <1,1,0>, tools/isa_loop.py).
// KS: the kernel's KSPAN (kc holds the constants VgprK<.., KS> selects).
template <int NBLK, int W0, int SH, bool KS>
DPOW_DEV bool full_check(const Launch &L, const KConst &kc, uint32_t vs, uint32_t loff, const uint32_t (&sd)[3]) {
    VarWords<KS> v;
    v.kc = &kc;
    v.seg_d[0] = sd[0];
    v.seg_d[1] = sd[1];
    v.seg_d[2] = sd[2];
    var_words<SH>(v, 0, vs, loff, v.seg_d[0]);
    uint32_t out[4][kNC];
    md5_tail<NBLK, W0, SH, 1>(out, L, v);
    return trailing_zero_nibbles(out[0][0], out[1][0], out[2][0], out[3][0]) >= L.ntz;
}

// The launch's completion record, written by the workgroup that retires last:
// the control block after every hit of this launch (and of earlier ones) was
// performed, then `seq` with release, which the host polls.  Out of line, and
// not in the watcher: either inlined form makes the register allocator spill
// SGPRs inside the hash loop (tools/isa_loop.py: 7-11 v_readlane per
// wave-block, -3.5 % throughput).
//
// It also resets the next search's control block (ctrl_next): every launch of this search
// runs before any of the next one's (stream order), so the next search needs no reset
// kernel in front of its first launch.
// (Some two-block kernels pass ctrl_next = null and publish() derives it from ctrl -- the
// ring is kCtrlRing * 128 bytes, aligned to its size -- where that keeps SGPR spill reloads
// out of their hash loop (kLaunchPoll).  The one-block kernels pass it: deriving it there
// moved the sweep kernel's register assignment and cost it 0.6 % (218.1 -> 216.8 GH/s,
// profiles/r03_ab_publish.log).)
__device__ __attribute__((noinline)) void publish(Ctrl *ctrl, Snap *snap, uint32_t seq, unsigned long long *claim,
                                                  Ctrl *ctrl_next) {
    if (ctrl_next == nullptr) {
        constexpr uintptr_t kRingBytes = kCtrlRing * kCtrlStride * sizeof(Ctrl);
        const uintptr_t a = reinterpret_cast<uintptr_t>(ctrl);
        ctrl_next =
            reinterpret_cast<Ctrl *>((a & ~(kRingBytes - 1)) | ((a + kCtrlStride * sizeof(Ctrl)) & (kRingBytes - 1)));
    }
    // Every workgroup has left its claim loop: recycle the counter slot (claim[1]: the
    // launch's start time, written by the watcher).
    const unsigned long long t_start = __hip_atomic_load(&claim[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t x = 0; x < kClaimCounters; ++x) claim[x * kClaimStride] = 0ull;
    claim[1] = 0ull;
    ctrl_next->best = kNoHit;
    ctrl_next->stop = 0u;
    ctrl_next->done = 0u;
    const unsigned long long best = __hip_atomic_load(&ctrl->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t stop = __hip_atomic_load(&ctrl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&snap->best, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&snap->stop, stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&snap->t_start, t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&snap->t_end, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&snap->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#if DPOW_WAVE_TRACE
    g_wave_trace[kTraceFields * (kTraceWaves - 2) + 3] = __builtin_amdgcn_s_memrealtime();  // the record released
#endif
}

// Workgroup 0, one lane: relays the host cancel flag to Ctrl::stop while the
// launch runs; exits once every worker workgroup has retired.  A launch that
// was still queued when its search returned CANCELLED stops too, even after
// the caller cleared the flag for its next task: the host marks every launch
// up to the last one it queued as stale (int32 sequence distance).
//
// With a node slot attached (Launch::node_best / node_stop: the node's shared host
// memory, mapped), it relays the node's Found fan-out the same way: a lower best of
// another rank goes to Ctrl::best (atomicMin) -- the waves stop at it at their next
// group -- and a raised node stop stops the launch.  The host injecting the same best
// through a kernel on a second stream (round 2's dpow_search_bound) took 50-160 us to start that kernel beside the
// running grid (measured early in round 3 with a stop-latency probe whose log did not survive;
// tools/small_search_probe.py --stop measures the stop as it is now).
//
// The bound injected by dpow_search_bound (a pinned host word) is relayed the same way.
//
// With a node slot attached it also relays Ctrl::best the other way, to the pinned early-hit
// word (Launch::early): a hit of this launch reaches the host ~1 us after the wave's
// atomicMin, which verifies it and posts it to the node slot at once -- the other ranks stop
// at it while this launch is still draining the chunks below it (round 3: the post waited
// for the completion record, the drain plus ~5 us).
//
// It also stamps the launch's start (s_memrealtime into the claim slot's spare word): the
// watcher workgroup is dispatched first, and the kernel time in the completion record
// replaces per-launch HIP timing events, whose profiling packets cost the host ~4.5 us per
// launch on the time-to-secret path (tools/small_search_probe.py, DPOW_DIAG_NO_EVENTS).
// The code-placement pad of the sweep kernels (search_body): 63 s_nop.
constexpr int kPad4B = 63;
DPOW_DEV void watcher(const Launch &L) {
    if (threadIdx.x != 0) return;
    __hip_atomic_store(&L.claim[1], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long node_seen = ~0ull, bound_seen = L.bound0, early_seen = kNoHit;
#if DPOW_WAVE_TRACE
    // the watcher's own record, in the last trace slot: start, the first node best relayed,
    // the first early-hit relay, exit
    unsigned long long *wt = g_wave_trace + kTraceFields * (kTraceWaves - 1);
    wt[0] = __builtin_amdgcn_s_memrealtime();
    wt[1] = wt[2] = 0;
#endif
    // Every word of a poll is loaded at once and waited for together: one round trip to the
    // host's pinned pages per poll.  Round 4's loop consumed each load before issuing the next -- the completion count, the best, then the flags, the bound
    // and the node's words: four round trips, ~8 us per poll under load
    // (tools/search_timeline.py, profiles/r05_ab.json[r05s/]), which every relay waited for:
    // an owner's hit to its early-hit word, another rank's posted hit into Ctrl::best, the
    // watcher's own exit behind the last workgroup (the next launch's start).  The node slot's
    // words are read through pointers selected inside the loop (without a slot: the launch's
    // own bound and cancel words), so the selection stays out of the kernel's entry block.
    for (;;) {
        const unsigned long long *const nbp = L.node_best ? L.node_best : L.ext_bound;
        const uint32_t *const nsp = L.node_stop ? L.node_stop : L.cancel;
        const uint32_t done = __hip_atomic_load(&L.ctrl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long b = __hip_atomic_load(&L.ctrl->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t stale = __hip_atomic_load(L.stale, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t cancel = __hip_atomic_load(L.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long eb = __hip_atomic_load(L.ext_bound, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long nb = __hip_atomic_load(nbp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t nstop = __hip_atomic_load(nsp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (done >= L.done_target) {
#if DPOW_WAVE_TRACE
            wt[3] = __builtin_amdgcn_s_memrealtime();
#endif
            return;
        }
        if (L.early && b < early_seen) {
#if DPOW_WAVE_TRACE
            if (wt[2] == 0) wt[2] = __builtin_amdgcn_s_memrealtime();
#endif
            early_seen = b;
            __hip_atomic_store(L.early, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        bool stop = cancel != 0u || (int32_t)(stale - L.seq) >= 0;
        if (eb < bound_seen) {
            bound_seen = eb;
            __hip_atomic_fetch_min(&L.ctrl->best, eb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (L.node_best) {
            if (nb < node_seen) {
#if DPOW_WAVE_TRACE
                if (wt[1] == 0 && nb < kNoHit) wt[1] = __builtin_amdgcn_s_memrealtime();
#endif
                node_seen = nb;
                __hip_atomic_fetch_min(&L.ctrl->best, nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            stop = stop || nstop != 0u;
        }
        if (stop) {
            __hip_atomic_store(&L.ctrl->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        __builtin_amdgcn_s_sleep(kWatchSleep);
    }
}

// One returning atomic per claim, by lane 0 (claim_issue); its result stays in
// lane 0's VGPR until claim_take broadcasts it to the wave -- the wave waits for
// the atomic only there.  The counter's n-th claim is chunk n * kClaimCounters + x.
// The AMDGPU atomic optimizer rewrites an atomic on a uniform address into a wave-wide
// reduction that reads the returned value at once, which would put the atomic's latency
// back in front of the chunk it was issued ahead of.  A lane-varying (opaque) zero offset
// keeps the address divergent to the compiler, so the claim stays a plain one-lane
// returning atomic, waited for only where claim_take reads it.
template <bool kOpaque>
DPOW_DEV unsigned long long claim_issue(unsigned long long *ctr, uint32_t lane) {
    unsigned long long v = 0;
    if constexpr (kOpaque) {
        uint32_t z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        ctr += z;
    }
    if (lane == 0) v = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
}

// base: the first counter-handed claim (Launch::n_static with static first claims, else 0).
DPOW_DEV uint64_t claim_take(unsigned long long v, uint32_t x, uint64_t base) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (((uint64_t)hi << 32) | lo) * kClaimCounters + x + base;
}

DPOW_DEV uint64_t claim_next(unsigned long long *ctr, uint32_t x, uint32_t lane, uint64_t base) {
    return claim_take(claim_issue<false>(ctr, lane), x, base);
}

DPOW_DEV uint64_t lane_range_mask(int64_t lo, int64_t hi) {
    lo = lo < 0 ? 0 : (lo > 64 ? 64 : lo);
    hi = hi < 0 ? 0 : (hi > 64 ? 64 : hi);
    if (hi <= lo) return 0;
    const uint64_t upto_hi = hi == 64 ? ~0ull : ((1ull << hi) - 1ull);
    const uint64_t below_lo = lo == 64 ? ~0ull : ((1ull << lo) - 1ull);
    return upto_hi & ~below_lo;
}

// Hash one wave-block (64 * kNC consecutive local indices from i0) and publish
// its first hit, if any, to Ctrl::best.  Returns the hit's global index, or
// kNoHitG.
//
// The per-candidate test is one compare: with EQ (one final block, ntz >= 8)
// the raw state word against -iv[3] (D == 0, no add, no mask); otherwise
// D <= dle, the even-nibble prefilter of the mask, which the rare path (a hit
// in the wave, 16^-(ntz & ~1) per candidate) re-tests against the exact mask.
constexpr uint64_t kNoHitG = ~0ull;

// KSPAN (SH = 3 only): the launch's lanes may span several k (R < 64), so word W0 + 1's
// K + M carries each lane's k offset (VarWords::lane_k, one VALU add per candidate in each
// of that word's four steps).  The SH = 3 kernels of launches with R >= 64 (workerBits <= 2:
// the offset is 0) are instantiated without it: the word's K + M stays a wave-uniform SGPR.
template <int NBLK, int W0, int SH, bool EQ, bool KSPAN>
DPOW_DEV uint64_t hash_wave_block(const Launch &L, const KConst &kc, uint64_t i0, uint32_t lane, uint32_t loff) {
    static_assert(!EQ || NBLK == 1, "the D-equality test needs one final block");
    static_assert(KSPAN || SH == 3, "only the SH = 3 kernels have a narrow (R >= 64) instantiation");
    uint32_t vs[kNC];
    VarWords<KSPAN> v;
    v.kc = &kc;
    v.seg_d[0] = v.seg_d[1] = v.seg_d[2] = 0u;  // unused: the hash loop's segment-word steps all read kc
    uint32_t d1 = 0u;               // SH != 0: the segment addition to word W0 + 1 (both slots share
    if constexpr (SH != 0) {        //  the segment: wave-blocks never straddle one)
        uint32_t d2;
        seg_deltas<W0, SH>(L, (uint32_t)((i0 >> L.rbits) >> 24), d1, d2);
    }
#pragma unroll
    for (int j = 0; j < kNC; ++j) {
        vs[j] = wave_uniform_v(i0 + 64u * j, L.rbits, L.base_tb);
        var_words<SH>(v, j, vs[j], loff, d1);
    }
    uint32_t dig[4][kNC];
    md5_tail<NBLK, W0, SH, kNC, true, EQ>(dig, L, v);  // only D is tested here

    uint64_t bal[kNC];
    uint64_t any = 0;
#pragma unroll
    for (int j = 0; j < kNC; ++j) {
        bal[j] = EQ ? __ballot(dig[3][j] == L.deq) : __ballot(dig[3][j] <= L.dle);
        any |= bal[j];
    }
    if (any != 0) {  // rare: lowest valid slot, then lowest lane
#pragma unroll
        for (int j = 0; j < kNC; ++j) {
            const uint64_t ij = i0 + 64u * j;
            uint64_t m = bal[j] & lane_range_mask((int64_t)(L.i_begin - ij), (int64_t)(L.i_end - ij));
            if (!EQ && m != 0) m &= __ballot((dig[3][j] & L.dmask) == 0u);
            if (m != 0 && L.ntz > 8u) {
                uint32_t d0, sd[3];
                seg_all_deltas<NBLK, W0, SH>(L, seg_id((ij < L.i_begin ? L.i_begin : ij) >> L.rbits), d0, sd);
                const bool ok = ((m >> lane) & 1ull) && full_check<NBLK, W0, SH, KSPAN>(L, kc, vs[j], loff, sd);
                m = __ballot(ok);
            }
            if (m != 0) {
                const uint64_t g = global_of_local(ij + (uint64_t)__builtin_ctzll(m), L.rbits, L.base_tb);
                if (lane == 0) {
                    // A returning atomic whose result is consumed: the wave waits (vmcnt)
                    // until the min is performed, before its retirement barrier and the
                    // Ctrl::done increment that lets publish() read Ctrl::best.
                    const unsigned long long prev = __hip_atomic_fetch_min(
                        &L.ctrl->best, (unsigned long long)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("; dpow: atomicMin performed (%0)" ::"v"(prev));
                }
                return g;
            }
        }
    }
    return kNoHitG;
}

// SGPR budget per layout.  The grid is 6 four-wave workgroups per CU (6 waves per
// SIMD, dpow_api.cpp), so a budget that still admits 7 waves costs no occupancy.
// The short-nonce layouts keep the round-1 budget (72: no spill in the hash
// loop; 8 waves admitted, so the next queued launch's workgroups start beside a
// draining one), except those kShort96 lists (round 6).  Layouts with many launch-uniform K + M constants -- long nonces
// and two final blocks -- get 96: at 72 the compiler spills them to VGPR lanes
// and reloads each with a v_readlane in every wave-block (tools/isa_loop.py:
// 4-41 per wave-block; 0 at 96).
// The two-block W0 = 15 layouts get 100 (DPOW_NUM_SGPR_W15): at 96 three of them kept 3
// spill reloads per wave-block in every launch-field choice (kLaunchPoll), at 100 they keep
// 0-1.  Round 4's per-layout sweep of a 100 budget for every long layout (tools/lead_sweep.py,
// profiles/r04_lead_sweep.json) added <2,13,3> (+1.5 %), <2,14,3> (+0.7 %) and <1,11,3>
// (+2.6 %); elsewhere 100 is within +-0.3 % of 96.  7 waves still fit.
// (The attribute takes no template-dependent value: three kernel templates share
// one body, and md5_variant.hip instantiates the one kLongSgpr / kW15Sgpr select.)
template <int NBLK, int W0>
constexpr bool kLongSgpr = NBLK == 2 || W0 >= kSgprLongW0;
template <int NBLK, int W0, int SH>
constexpr bool kW15Sgpr = (NBLK == 2 && W0 == 15) || (NBLK == 2 && SH == 3 && (W0 == 13 || W0 == 14)) ||
                          (NBLK == 1 && W0 == 11 && SH == 3);

// Whether a kernel reads the poll group (Launch::poll_wb) and the next search's control block
// (Launch::ctrl_next) from the launch, or uses the compile-time group and derives the block in
// publish().  The two-block kernels sit at their SGPR budget, and which choice leaves their hash
// loop free of SGPR spill reloads depends on the layout's register assignment, not on the count
// of live values (tools/isa_loop.py over all four combinations; the two flags chosen alike
// leave every two-block layout at 0-1 reloads per wave-block except <2,12,0> (4 in every
// combination) and <2,15,0> / <2,15,3> (3); one reload-heavy choice for all of them cost 3-4 %
// at <2,14,1>, <2,14,3>, <2,15,1> against round 2's build in a same-box A/B).
template <int NBLK, int W0, int SH>
constexpr bool kLaunchPoll = NBLK == 1 || SH == 1 || SH == 2 || (SH == 0 && W0 == 15) || (SH == 3 && W0 >= 14);

// The choices of a kernel (KS: its KSPAN; the narrow SH = 3 kernels' from narrow_knobs):
// kLaunchPoll and the SGPR budget class (0: DPOW_NUM_SGPR, 1: _LONG, 2: _W15).
template <int NBLK, int W0>
constexpr int kNarrowPoll = DPOW_NPOLL >= 0 ? DPOW_NPOLL : narrow_knobs(NBLK, W0).poll;
template <int NBLK, int W0>
constexpr int kNarrowSgpr = DPOW_NSGPR > 0 ? DPOW_NSGPR : narrow_knobs(NBLK, W0).sgpr;
template <int NBLK, int W0, int SH, bool KS>
constexpr bool kPollOf = SH == 3 && !KS && kNarrowPoll<NBLK, W0> >= 0 ? kNarrowPoll<NBLK, W0> != 0
                                                                     : kLaunchPoll<NBLK, W0, SH>;
// Short-nonce one-block layouts (W0 <= 7, below kSgprLongW0) that take the 96 budget instead of
// 72: every one-block kernel at 96 against the build before, per layout (round 6,
// profiles/r06_narrow_sweep.json ab6 at workerBits 0: SH = 1-2 +0.5 to +1.5 %, SH = 0 at W0 3 and
// 5-7 +0.8 to +1.2 %; ab5, SH = 3's general kernels at workerBits 3: W0 2-5 +0.5 to +0.9 %, W0 7
// +6.6 %, where 72 left 7 spill reloads per wave-block).  The rest were within noise or slower
// (<1,0,3> -3 %, <1,6,3> -3 %); the sweep kernel <1,1,0> keeps its code.  Not the "_ls" units.
template <int NBLK, int W0, int SH, bool KS>
constexpr bool kShort96 = NBLK == 1 && !DPOW_VLS && KS && W0 < kSgprLongW0 &&
                          (SH == 1 || SH == 2 || (SH == 0 && (W0 == 3 || W0 >= 5)) ||
                           (SH == 3 && ((W0 >= 2 && W0 <= 5) || W0 == 7)));
template <int NBLK, int W0, int SH, bool KS>
constexpr int kSgprOf = SH == 3 && !KS && kNarrowSgpr<NBLK, W0> > 0 ? kNarrowSgpr<NBLK, W0>
                        : kW15Sgpr<NBLK, W0, SH> ? 2 : kLongSgpr<NBLK, W0> || kShort96<NBLK, W0, SH, KS> ? 1 : 0;

template <int NBLK, int W0, int SH, bool EQ, bool KSPAN>
DPOW_DEV void search_body(const Launch &L) {
    if (blockIdx.x == 0) {  // dispatched first: the watcher
        watcher(L);
        return;
    }
#if DPOW_WAVE_TRACE
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_first = 0, n_wb = 0, t_last = 0, c_last = 0, reason = 0, t_hit = 0;
#endif
    // The 4-byte-nonce D-equality kernel (<1,1,0,eq>, the sweep's and N >= 8's), not the
    // chunk-length-spanning unit: kPad4B s_nop in front of the worker path put its hash
    // block at round 4's offset modulo 256 (tests/test_isa.py checks it).  Any change to the
    // watcher re-runs the whole kernel's register allocation (it is inlined: a noinline
    // watcher costs the hash block 24 VALU per wave-block), and the one-round-trip poll moved
    // the hash block by 4 bytes; a move of that kind alone cost the sweep 0.5 % in round 5
    // (profiles/r05_ab.json[r05q/ab.log]).  Padded: 218.8 vs 218.7 GH/s ([r05s/ab.log]).
    if constexpr (EQ && NBLK == 1 && W0 == 1 && SH == 0 && !DPOW_VLS)
        asm volatile(".rept %0\n s_nop 0\n .endr" ::"i"(kPad4B));
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t loff = lane_offset(L.rbits, lane);
    KConst kc;
    kconst_init<NBLK, W0, SH, 0, 0, KSPAN>(kc, L);
    // The 2^24-k segment kc's segment-word constants belong to; kept in a VGPR
    // (wave-uniform, read once per group): an SGPR live across the hash loop
    // costs spill reloads inside it under the 80-SGPR budget.
    uint32_t cur_seg_v;
    asm("v_mov_b32 %0, %1" : "=v"(cur_seg_v) : "s"(L.seg0));
    // SH = 0: the lane offset plus the current segment's addition to word W0 (the 0x80 pad
    // of chunk lengths <= 2 in launches spanning chunk lengths; 0 in the template's own
    // segment), the per-lane part of W0's K + M.
    uint32_t lov = loff;

    unsigned long long best = __hip_atomic_load(&L.ctrl->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    best = best < L.bound0 ? best : L.bound0;
    uint32_t stop = __hip_atomic_load(&L.ctrl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // Waves claim chunks of L.chunk consecutive wave-blocks from their XCD's
    // counter, which hands its chunks out in increasing index order (the early
    // exit stays exact); neither the grid size nor the residency creates a
    // tail.  The next claim is requested while the current chunk is hashed.  A
    // launch that starts at or above the best index (queued behind a hit) or
    // after a cancel claims nothing: a contended counter serves < 90 claims/us.
    // Worker block b (>= 1) serves counter (b - 1) % 8; the host launches at
    // least min(n_chunks, 8) worker blocks, so every counter holding a chunk
    // has waves.  Workgroups go round-robin to XCDs, so each counter's waves
    // share one XCD.
    // Tail priority: older waves win the SIMD's issue arbitration, so the youngest waves of
    // a CU barely progress until the launch drains, and then finish chunks they claimed
    // early.  Every worker wave runs at priority 1 and drops to 0 once it holds a tail
    // claim: the waves still on earlier chunks issue first.  profiles/r01_ab_tail_prio.log:
    // sweep windows at workerBits 3 (2^29-candidate launches) 209.5 -> 212.8 GH/s,
    // workerBits 0 217.4 -> 218.3.
    __builtin_amdgcn_s_setprio(1);
    // A wave requests its next claim while it hashes the current chunk (profiles/
    // r02_ab_ahead.log: 217.6 against 215.5 GH/s for one claim in flight per wave).  With
    // kDeferClaims (one-block kernels) the claim's atomic is issued in the chunk's last poll
    // group and its result read after the chunk: a slow wave does not sit on an early chunk
    // for the whole of its current one, and the polls of the chunk's earlier groups do not
    // wait for the claim atomic (vmcnt counts in issue order; round 4, profiles/
    // r04_node_ab.log: +0.03 to +0.24 %).  The deferred read holds the claim's value in two
    // more VGPRs across the hash loop; the two-block kernels sit at 71-79 VGPRs, where that
    // costs a wave per SIMD or shifts their register assignment (-5 to -10 %,
    // profiles/r02_ab_layouts/), so they read the claim in front of the chunk.
    constexpr bool kDeferClaims = NBLK == 1;
    uint32_t x = (blockIdx.x - 1u) % kClaimCounters;
    const bool skip = stop != 0u || global_of_local(L.i_begin, L.rbits, L.base_tb) >= best;
    const uint64_t cbase = kStaticFirst ? L.n_static : 0;
    uint64_t claim;
    if constexpr (kStaticFirst) {
        const uint32_t wave_id =
            __builtin_amdgcn_readfirstlane((blockIdx.x - 1u) * (kBlockThreads / 64) + threadIdx.x / 64u);
        claim = skip ? L.n_chunks
                     : (wave_id < cbase ? (uint64_t)wave_id : claim_next(L.claim + x * kClaimStride, x, lane, cbase));
    } else {
        claim = skip ? L.n_chunks : claim_next(L.claim + x * kClaimStride, x, lane, cbase);
    }
#if DPOW_WAVE_TRACE
    t_first = __builtin_amdgcn_s_memrealtime() + (claim & 0);
#endif
    uint32_t hops = 0;
    for (;;) {
        // This counter is drained: move on to the next one (its waves may sit
        // on a slower XCD).  A counter only ever drains, so after a full round
        // of drained counters every chunk has been handed out.
        if (claim >= L.n_chunks) {
#if DPOW_WAVE_TRACE
            reason = 1;
#endif
            if (skip || ++hops >= kClaimCounters) break;
            x = (x + 1u) % kClaimCounters;
            const unsigned long long seen =
                __hip_atomic_load(L.claim + x * kClaimStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            claim = seen * kClaimCounters + x + cbase < L.n_chunks
                        ? claim_next(L.claim + x * kClaimStride, x, lane, cbase)
                        : L.n_chunks;
            continue;
        }
        // kDeferClaims: the next claim's atomic is issued in the chunk's last group and its
        // result read after the chunk (claim_take); else the next claim is taken now.
        unsigned long long next_v = 0;
        uint64_t next = 0;
        bool issued = false;  // kDeferClaims: the next claim's atomic was issued (in the chunk's last group)
        if constexpr (kDeferClaims) (void)issued;
        else next = claim_next(L.claim + x * kClaimStride, x, lane, cbase);
        // Claims [0, n_big) are `chunk` wave-blocks, the rest `chunk_tail`: the
        // launch ends on small claims, so its waves run dry within a few
        // wave-blocks of each other (the tail of a 2.5 ms launch was ~3 %).
        const bool big = claim < L.n_big;
        if (!big) __builtin_amdgcn_s_setprio(0);
        const uint64_t b_begin = big ? claim * L.chunk : L.n_big * L.chunk + (claim - L.n_big) * L.chunk_tail;
        const uint32_t csz = big ? L.chunk : L.chunk_tail;
        const uint32_t nb = (uint32_t)(b_begin + csz < L.n_wblocks ? csz : L.n_wblocks - b_begin);
        const uint64_t i_first = L.wb_begin + b_begin * (uint64_t)kWaveBlock;
        // Early exit at a claim: stop on a cancel, or once this chunk starts at
        // or above the best index found so far.
        // Everything below the best has been or is being hashed by earlier claims.
        if (stop != 0u ||
            global_of_local(i_first < L.i_begin ? L.i_begin : i_first, L.rbits, L.base_tb) >= best) {
#if DPOW_WAVE_TRACE
            reason = stop != 0u ? 3 : 2;
#endif
            break;
        }
#if DPOW_WAVE_TRACE
        t_last = __builtin_amdgcn_s_memrealtime();
        c_last = claim;
#endif
        // The chunk runs in groups of L.poll_wb wave-blocks.  Each group's loads of
        // Ctrl::best / Ctrl::stop are issued before it and consumed after it (the
        // latency hides behind the hashing), so a hit elsewhere or a cancel ends
        // this wave within one group, not at the chunk's end.  A hit of this wave
        // ends the chunk at once: its later wave-blocks hold larger indices.
        // Down-counters keep the loop's live SGPRs at a plain loop's count.
        uint64_t i0 = i_first;
        uint32_t left = nb;
        // (some two-block layouts: the compile-time group, kLaunchPoll)
        const uint32_t poll_wb = kPollOf<NBLK, W0, SH, KSPAN> ? L.poll_wb : (uint32_t)DPOW_POLL_WB;
        for (;;) {
            uint32_t q = left < poll_wb ? left : poll_wb;
            // A chunk never straddles a 2^24-k segment boundary (the host aligns a
            // spanning launch's chunks to them, dpow_api.cpp), so neither does a
            // group; entering another segment re-derives the segment words' K + M
            // constants.  (Splitting groups at boundaries in the kernel instead
            // costs 4 SGPR spill reloads per wave-block: tools/isa_loop.py.)
            {
                // (from the launch's first index: a wave-block below it may hold k = 0, whose
                // lanes are masked off and whose chunk length differs from its neighbours')
                const uint32_t sg = seg_id((i0 < L.i_begin ? L.i_begin : i0) >> L.rbits);
                if (sg != __builtin_amdgcn_readfirstlane(cur_seg_v)) {
                    asm volatile("v_mov_b32 %0, %1" : "=v"(cur_seg_v) : "s"(sg));
                    uint32_t d0, d[3];
                    seg_all_deltas<NBLK, W0, SH>(L, sg, d0, d);
                    kconst_seg<NBLK, W0, SH, 0, 0, KSPAN>(kc, L, d);
                    if constexpr (SH == 0) lov = lane_offset(L.rbits, lane) + d0;
                }
            }
            left -= q;
            if constexpr (kDeferClaims) {
                if (left == 0) {  // the chunk's last group: reserve the next chunk now
                    next_v = claim_issue<true>(L.claim + x * kClaimStride, lane);
                    issued = true;
                }
            }
            const unsigned long long best_seen =
                __hip_atomic_load(&L.ctrl->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t stop_seen = __hip_atomic_load(&L.ctrl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool hit = false;
            for (; q != 0; --q, i0 += (uint64_t)kWaveBlock) {
#if DPOW_WAVE_TRACE
                ++n_wb;
#endif
                const uint64_t g = hash_wave_block<NBLK, W0, SH, EQ, KSPAN>(L, kc, i0, lane, SH == 0 ? lov : loff);
                if (g != kNoHitG) {
                    best = g < best ? g : best;
                    hit = true;
#if DPOW_WAVE_TRACE
                    if (t_hit == 0) t_hit = __builtin_amdgcn_s_memrealtime();
#endif
                    break;
                }
            }
            best = best_seen < best ? best_seen : best;
            stop = stop_seen;
            if (hit || left == 0 || stop != 0u || global_of_local(i0, L.rbits, L.base_tb) >= best) break;
        }
        if constexpr (kDeferClaims) {
            // left the chunk before its last group (a hit, a bound, a stop): every later chunk
            // is at or above the best, or the launch is stopping -- nothing more to claim
            if (!issued) {
#if DPOW_WAVE_TRACE
                reason = 4;
#endif
                break;
            }
            claim = claim_take(next_v, x, cbase);
        } else {
            claim = next;
        }
    }
    // Retirement is counted per workgroup (a quarter of the atomics on the
    // shared counter).  Each wave's atomicMin has been performed already (the
    // hit path consumes the returning atomic's result, which waits on vmcnt);
    // the barrier then covers all four waves, so the Ctrl::done increment --
    // and publish(), which reads Ctrl::best -- come after every hit of the
    // workgroup.  The workgroup whose count completes the launch publishes its
    // completion record.
#if DPOW_WAVE_TRACE
    const uint32_t wave = (blockIdx.x - 1u) * (kBlockThreads / 64) + threadIdx.x / 64u;
    if (lane == 0 && wave < kTraceWaves) {
        unsigned long long *w = g_wave_trace + kTraceFields * wave;
        w[0] = t_start;
        w[1] = t_first;
        w[2] = __builtin_amdgcn_s_memrealtime();
        w[3] = n_wb;
        w[4] = t_last;
        w[5] = c_last;
        w[6] = reason;
        w[7] = t_hit;
    }
#endif
    if constexpr (kDeferClaims) {
        // A wave that left the loop right after issuing its next claim (a hit below the
        // chunk, a bound, a cancel) still has that atomic in flight; the last retiring
        // workgroup re-zeroes the launch's claim counters in publish(), and a claim
        // landing after that would leave the slot's next user one chunk short.  Every
        // claim of the workgroup is performed before its retirement count.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#if DPOW_WAVE_TRACE
    const unsigned long long t_claims = __builtin_amdgcn_s_memrealtime();
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (threadIdx.x == 0) {
#if DPOW_WAVE_TRACE
        const unsigned long long t_bar = __builtin_amdgcn_s_memrealtime();
#endif
        if constexpr (kXcdRetire) {
            // Retirement is counted per claim counter first (worker block b serves counter
            // (b - 1) % 8, its XCD's) on a word of that counter's line, and the counter's last
            // workgroup adds the counter's count to Ctrl::done: a launch's few hundred to ~1500
            // retirements no longer queue on one line (~100 atomics per us) at its end.
            const uint32_t n_wg = gridDim.x - 1u;
            const uint32_t xr = (blockIdx.x - 1u) % kClaimCounters;
            const uint32_t nx = n_wg / kClaimCounters + (xr < n_wg % kClaimCounters ? 1u : 0u);
            unsigned long long *const xc = L.claim + xr * kClaimStride + 2;
            const unsigned long long px = __hip_atomic_fetch_add(xc, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (px + 1ull == (unsigned long long)nx) {
                // every retirement of this counter is in: zero it for the slot's next launch
                __hip_atomic_store(xc, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t prev = __hip_atomic_fetch_add(&L.ctrl->done, nx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if DPOW_WAVE_TRACE
                if (prev + nx == L.done_target) {  // the publisher's retirement: slot kTraceWaves - 2
                    unsigned long long *r = g_wave_trace + kTraceFields * (kTraceWaves - 2);
                    r[0] = t_claims;
                    r[1] = t_bar;
                    r[2] = __builtin_amdgcn_s_memrealtime() + (prev & 0);
                }
#endif
                if (prev + nx == L.done_target)
                    publish(L.ctrl, L.snap, L.seq, L.claim, kPollOf<NBLK, W0, SH, KSPAN> ? L.ctrl_next : nullptr);
            }
        } else {
            const uint32_t prev = __hip_atomic_fetch_add(&L.ctrl->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if DPOW_WAVE_TRACE
            if (prev + 1u == L.done_target) {  // the publisher's retirement: slot kTraceWaves - 2
                unsigned long long *r = g_wave_trace + kTraceFields * (kTraceWaves - 2);
                r[0] = t_claims;
                r[1] = t_bar;
                r[2] = __builtin_amdgcn_s_memrealtime() + (prev & 0);
            }
#endif
            if (prev + 1u == L.done_target) publish(L.ctrl, L.snap, L.seq, L.claim, kPollOf<NBLK, W0, SH, KSPAN> ? L.ctrl_next : nullptr);
        }
    }
}

template <int NBLK, int W0, int SH, bool EQ, bool KSPAN>
__global__ void __launch_bounds__(kBlockThreads) __attribute__((amdgpu_num_sgpr(DPOW_NUM_SGPR)))
md5_search_kernel(const Launch L) {
    search_body<NBLK, W0, SH, EQ, KSPAN>(L);
}

template <int NBLK, int W0, int SH, bool EQ, bool KSPAN>
__global__ void __launch_bounds__(kBlockThreads) __attribute__((amdgpu_num_sgpr(DPOW_NUM_SGPR_LONG)))
md5_search_kernel_lsgpr(const Launch L) {
    search_body<NBLK, W0, SH, EQ, KSPAN>(L);
}

template <int NBLK, int W0, int SH, bool EQ, bool KSPAN>
__global__ void __launch_bounds__(kBlockThreads) __attribute__((amdgpu_num_sgpr(DPOW_NUM_SGPR_W15)))
md5_search_kernel_w15sgpr(const Launch L) {
    search_body<NBLK, W0, SH, EQ, KSPAN>(L);
}

}  // namespace DPOW_KNS
}  // namespace dpow
