// dpow_common.h -- definitions shared by the gfx950 kernels and the host planner.
//
// MD5 constants (RFC 1321 section 3.4) and the launch descriptor that carries
// one launch window of the search (see DESIGN.md "Data layout").
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define DPOW_HD __host__ __device__ __forceinline__
#else
#define DPOW_HD inline
#endif

namespace dpow {

// T[i] = floor(|sin(i+1)| * 2^32)
constexpr uint32_t kMd5K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

constexpr uint32_t kMd5IV[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};

// Rotation of step i.
constexpr int md5_shift(int i) {
    return (i < 16)   ? (i % 4 == 0 ? 7 : i % 4 == 1 ? 12 : i % 4 == 2 ? 17 : 22)
           : (i < 32) ? (i % 4 == 0 ? 5 : i % 4 == 1 ? 9 : i % 4 == 2 ? 14 : 20)
           : (i < 48) ? (i % 4 == 0 ? 4 : i % 4 == 1 ? 11 : i % 4 == 2 ? 16 : 23)
                      : (i % 4 == 0 ? 6 : i % 4 == 1 ? 10 : i % 4 == 2 ? 15 : 21);
}

// Message word read by step i.
constexpr int md5_word(int i) {
    return (i < 16) ? i : (i < 32) ? (1 + 5 * i) % 16 : (i < 48) ? (5 + 3 * i) % 16 : (7 * i) % 16;
}

// bitop3 truth tables, index = (x << 2) | (y << 1) | z.
constexpr uint32_t kBop3F = 0xCA;  // F = x ? y : z
constexpr uint32_t kBop3G = 0xE4;  // G = z ? x : y
constexpr uint32_t kBop3H = 0x96;  // H = x ^ y ^ z
constexpr uint32_t kBop3I = 0x39;  // I = y ^ (x | ~z)

// Launches span 2^24-k segments (plan.cpp; the kernel re-derives the constants of the
// words holding k >> 24); round 1 split a window at every multiple of 2^24 k instead.

// Launches span chunk lengths 1..3 for SH = 0 layouts (plan.cpp lspan_end; the kernel
// re-derives the pad and bit-length words per chunk length); round 2 ran one launch per
// chunk length.

// Candidates per lane per wave-block (interleaved for ILP).
#ifndef DPOW_NC
#define DPOW_NC 2
#endif
constexpr int kNC = DPOW_NC;
constexpr int kWaveBlock = 64 * kNC;  // local indices per wave-block
constexpr int kBlockThreads = 256;    // 4 waves per workgroup
// Claim counters per launch: one per XCD (workgroup b runs on XCD b % 8), each
// on its own 128-byte line.  Counter x hands out chunks x, x + 8, x + 16, ...
// in increasing order, so the early exit stays exact per counter, and eight
// counters serve eight times the claim rate of one.
constexpr uint32_t kClaimCounters = 8;
constexpr uint32_t kClaimStride = 16;  // unsigned long long units (128 B)
constexpr uint32_t kClaimSlot = kClaimCounters * kClaimStride;  // one launch's counters

// Device control block of one search (a context keeps a ring of kCtrlRing in HBM, each
// on its own 128-byte line).  A search's launches find theirs clean -- reset by the
// previous search's launches (Launch::ctrl_next), or at dpow_open -- so a search needs
// no reset kernel in front of its first launch.
constexpr unsigned long long kNoHit = 0x7FFFFFFFFFFFFFFFull;  // = DPOW_NO_HIT (include/dpow.h)
struct Ctrl {
    unsigned long long best;  // min global index found (kNoHit = none), atomicMin target
    uint32_t stop;            // set by the watcher when the host cancel flag is raised
    // Ctrl::done on a 128-byte line of its own: every wave loads best and stop once per poll
    // group, and the retirement count's atomics (one per workgroup, at the end of a launch)
    // queued behind those loads on a shared line.
    uint32_t pad0_;
    unsigned long long pad1_[14];
    uint32_t done;            // worker workgroups retired (cumulative within one search)
    uint32_t pad2_[31];
};
constexpr uint32_t kCtrlLine = 256;  // bytes per ring entry
constexpr uint32_t kCtrlRing = 4;
constexpr uint32_t kCtrlStride = kCtrlLine / sizeof(Ctrl);  // Ctrl units between ring entries
static_assert((kCtrlRing & (kCtrlRing - 1)) == 0 && kCtrlLine % sizeof(Ctrl) == 0, "the ring is aligned to its size");
static_assert(sizeof(Ctrl) == 256 && __builtin_offsetof(Ctrl, done) == 128, "done on its own line");

// Host-visible completion record of one launch (pinned, host-coherent, mapped).
// The launch's last retiring workgroup writes it: the
// control block as of the end of the launch, then `seq` (release), which the
// host polls instead of waiting on a stream event.
struct Snap {
    unsigned long long best;
    uint32_t stop;
    uint32_t seq;  // launch sequence number + 1 (0 = never written)
    unsigned long long t_start, t_end;  // s_memrealtime (100 MHz) at the launch's start and at the record
};
constexpr double kRealtimeNs = 10.0;  // ns per s_memrealtime tick (100 MHz)

// One launch window.  Passed by value as the kernel argument (kernarg segment,
// read with scalar loads).
struct Launch {
    uint32_t iv[4];        // chaining value entering the first final block (midstate)
    uint32_t T[32];        // final block(s) template words, variable bytes zeroed
    uint32_t KT[128];      // K[s] + T[16 b + word(s)] for every step s of block b
    uint64_t i_begin;      // local index range [i_begin, i_end)
    uint64_t i_end;
    uint64_t wb_begin;     // i_begin rounded down to a wave-block (64 * kNC: a wave-block never
                           //  straddles a 2^24-k boundary)
    uint64_t n_wblocks;    // wave-blocks covering [wb_begin, i_end)
    uint32_t rbits;        // R = 1 << rbits threadBytes per k
    uint32_t base_tb;      // uint8(worker_byte << rbits)
    uint32_t dmask;        // mask on the final D word for min(ntz, 8) trailing nibbles
    uint32_t dle;          // prefilter D <= dle: the even-nibble part of dmask (dmask == ~dle for even ntz)
    uint32_t deq;          // D-equality kernels (one final block, ntz >= 8): D == 0 <=> state word == deq = -iv[3]
    uint32_t ntz;          // requested trailing zeros (full digest check when > 8)
    uint32_t seg_first;    // k_begin >> 24: the chunk bytes above the low 24 bits that T / KT hold
                           //  (a launch spans 2^24-k segments; the kernel re-derives the K + M
                           //  constants of the words holding them when a wave enters another one)
    uint32_t done_target;  // Ctrl::done once this launch's worker workgroups have retired
    uint32_t chunk;        // wave-blocks per claim of the first n_big claims
    uint32_t chunk_tail;   // wave-blocks per claim after them (the launch's tail: small claims)
    uint64_t n_big;        // claims of `chunk` wave-blocks
    uint64_t n_chunks;     // claims covering n_wblocks (n_big + tail claims)
    uint64_t n_head;       // the claims every wave takes at its start (2 per wave; host diagnostics)
    uint64_t n_static;     // claims [0, n_static) are handed out by wave index, not by a counter: worker
                           //  wave w's first claim is w (the "_ls" kernels only; 0 for every other launch)
    uint32_t poll_wb;      // wave-blocks per group: a wave reads Ctrl::best / Ctrl::stop once per group
    uint32_t reserved0;    // (round 4's fair-priority tick count; kept so the kernel argument layout,
                           //  and with it the kernels' code, stays as measured)
    unsigned long long *claim;  // this launch's kClaimCounters counters (zero at launch start;
                                //  the launch's last workgroup re-zeroes them for the slot's next user)
    Ctrl *ctrl;              // this search's control block (clean at its first launch)
    Ctrl *ctrl_next;         // the next search's: reset by this launch's last workgroup (which derives it
                             //  from ctrl: the ring is aligned to its size; kept here for the host's checks)
    const uint32_t *cancel;  // device-visible alias of the pinned host cancel flag
    const uint32_t *stale;   // pinned: launches with seq <= *stale (mod 2^32) belong to a cancelled search
    const unsigned long long *ext_bound;  // pinned: the bound dpow_search_bound injected (the watcher relays it)
    Snap *snap;              // device alias of this launch's pinned completion record
    uint32_t seq;            // value the last workgroup writes to snap->seq
    uint32_t pad1;
    unsigned long long bound0;  // the search's bound at its start (the caller's, the node slot's):
                                //  a wave starts from min(Ctrl::best, bound0)
    // Node slot (dpow_node_attach; null when none): device aliases of the slot's best and
    // stop in the node's shared host memory, polled by the watcher -- another rank's hit
    // lowers Ctrl::best, a raised stop stops the launch.
    const unsigned long long *node_best;
    const uint32_t *node_stop;
    // Early hit word (attached node only; null otherwise): pinned, host-coherent.  The watcher
    // relays Ctrl::best here as soon as it drops, so the host can verify and post a hit to the
    // node slot while the launch still drains (the Found fan-out no longer waits for the
    // launch's completion record).  One word per control block of the ring (a stale launch of
    // the previous search writes its own block's word).
    unsigned long long *early;
    // SH = 0 layouts below k = 2^24: T / KT hold the message of chunk length 0 (the pad at
    // byte 1 of word W0, bit length 8 (nonce_len + 1)) with the launch's block count, and a
    // candidate of chunk length l adds lseg_deltas(l) to words W0, W0 + 1 and the bit-length
    // word.  The kernel treats the chunk lengths as segments (seg_id): a wave re-derives those
    // words' K + M when it enters another one, so one launch may span chunk lengths 1..3
    // (lspan: host-side planning information only).
    uint32_t lspan;
    uint32_t seg0;         // segment id of the template (the kernel's first segment)
};

// Chunk length of k < 2^24 (nextChunk^k, worker.go:234-244): 0 for k = 0, else 1 + floor(log256 k).
DPOW_HD uint32_t chunk_len_lt24(uint32_t k) { return (k != 0u) + (k > 0xFFu) + (k > 0xFFFFu); }

// Additions of chunk length l (0..3) to words W0, W0 + 1 and the bit-length word of an
// SH = 0 layout against chunk length 0 (Launch: the template of an SH = 0 launch below
// k = 2^24): the 0x80 pad moves from byte 1 of W0 to byte 1 + l of the (W0, W0 + 1) pair,
// and the bit length grows by 8 l.  Shared by the kernel and the planner.
DPOW_HD void lseg_deltas(uint32_t l, uint32_t &d0, uint32_t &d1, uint32_t &dlen) {
    const uint64_t pad = 0x80ull << (8 * (1 + l));
    d0 = (uint32_t)pad - 0x8000u;
    d1 = (uint32_t)(pad >> 32);
    dlen = 8u * l;
}

// Segment id of chunk k: a launch is uniform within a segment except for the variable
// bytes.  k >> 24 for k >= 2^24 (2^24-k segments, spanned by launches at L >= 4); kLsegBase + L
// below (chunk lengths 0..3, spanned by Launch::lspan launches).
// (The id needs no Launch field: reading Launch::lspan in the kernel's group loop moved its
// wave-uniform index arithmetic onto the VALU, +10 VALU per wave-block, tools/isa_loop.py.)
constexpr uint32_t kLsegBase = 0xFFFFFFF0u;  // ids of chunk lengths 0..3 (k >> 24 < 2^31 below DPOW_K_LIMIT)
DPOW_HD uint32_t seg_id(uint64_t k) {
    return k >> 24 ? (uint32_t)(k >> 24) : kLsegBase + chunk_len_lt24((uint32_t)k);
}

// Nibble positions (bit offsets) of a digest word in hex-string order from the
// end: the last hex character is the low nibble of the word's top byte.
DPOW_HD uint32_t tail_nibble_mask(uint32_t n) {
    const uint32_t pos[8] = {24, 28, 16, 20, 8, 12, 0, 4};
    uint32_t m = 0;
    for (uint32_t j = 0; j < n && j < 8; ++j) m |= 0xFu << pos[j];
    return m;
}

// The one-compare prefilter of the D-word test: (D & tail_nibble_mask(n)) == 0
// implies D <= tail_prefilter_le(n).  For even n the two are equivalent (the
// mask is the top 4n bits); for odd n the prefilter covers the top 4(n-1) bits
// and the rare path re-tests the mask.
DPOW_HD uint32_t tail_prefilter_le(uint32_t n) {
    const uint32_t e = (n < 8 ? n : 8) & ~1u;  // even part
    return e == 0 ? 0xFFFFFFFFu : e >= 8 ? 0u : (0xFFFFFFFFu >> (4 * e));
}

// Kernels with the D-equality test: one final block (D = iv[3] + state word)
// and a test on the whole D word.
DPOW_HD bool use_d_equality(uint32_t nblk, uint32_t ntz) { return nblk == 1 && ntz >= 8; }

DPOW_HD uint32_t bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// Trailing '0' hex characters of the digest (A,B,C,D little-endian words):
// the hex string is the 128-bit big-endian number bswap(A)|bswap(B)|bswap(C)|bswap(D).
DPOW_HD uint32_t trailing_zero_nibbles(uint32_t A, uint32_t B, uint32_t C, uint32_t D) {
    const uint32_t w[4] = {bswap32(D), bswap32(C), bswap32(B), bswap32(A)};
    uint32_t n = 0;
    for (int j = 0; j < 4; ++j) {
        if (w[j] == 0) { n += 8; continue; }
        uint32_t x = w[j];
        while ((x & 0xF) == 0) { x >>= 4; ++n; }
        break;
    }
    return n;
}

// Lane arithmetic shared by the kernel and the host emulation
// (dpow_plan_candidate): the variable 4 bytes V = threadByte | (k mod 2^24) << 8
// of local index i = i0 + lane, i0 a multiple of 64, split into a wave-uniform
// part and a per-lane constant.
DPOW_HD uint32_t lane_offset(uint32_t rbits, uint32_t lane) {
    return rbits >= 6 ? lane : ((lane & ((1u << rbits) - 1u)) | ((lane >> rbits) << 8));
}
DPOW_HD uint32_t wave_uniform_v(uint64_t i0, uint32_t rbits, uint32_t base_tb) {
    const uint64_t R = 1ull << rbits;
    return base_tb | (uint32_t)(i0 & (R - 1)) | ((uint32_t)((i0 >> rbits) & 0xFFFFFFu) << 8);
}
// Segment-word additions (launches spanning 2^24-k segments): a launch's template holds k >> 24 =
// seg_first at byte p + 4 (words W0 + 1 and, for SH = 3, W0 + 2); a candidate
// in 2^24-k segment `seg` adds (seg - seg_first) << 8 SH to that 64-bit word
// pair.  The field never overflows its bytes within one chunk length, but the
// sum may carry from word W0 + 1 into W0 + 2.  Shared by the kernel and the
// host emulation (dpow_plan_candidate).
DPOW_HD void seg_word_deltas(uint32_t t1, uint32_t t2, uint32_t seg, uint32_t seg_first, uint32_t sh,
                             uint32_t &d1, uint32_t &d2) {
    const uint64_t t = ((uint64_t)t2 << 32) | t1;
    const uint64_t x = t + ((uint64_t)(seg - seg_first) << (8 * sh));
    d1 = (uint32_t)x - t1;
    d2 = (uint32_t)(x >> 32) - t2;
}

// Global index g = k * 256 + threadByte of a local index.
DPOW_HD uint64_t global_of_local(uint64_t i, uint32_t rbits, uint32_t base_tb) {
    const uint64_t R = 1ull << rbits;
    return ((i >> rbits) << 8) | (uint64_t)(base_tb | (uint32_t)(i & (R - 1)));
}

}  // namespace dpow
