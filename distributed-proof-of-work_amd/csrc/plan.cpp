// plan.cpp -- host planning of a search window into kernel launches.
//
// The reference enumerates, per worker partition (worker.go:301-316),
//   for k = 0, 1, ... (chunk_k = nextChunk^k([]), worker.go:234-244, 399)
//     for t in 0..R-1: msg = nonce || threadByte[t] || chunk_k   (worker.go:319-353)
// A launch covers a k-range in which the chunk length L is constant (segment
// boundaries k = 1, 2^8, 2^16, ..., 2^48), so the message layout is uniform.
// The per-candidate bytes are V = threadByte | (k mod 2^24) << 8, at byte
// offset p = nonce_len mod 64 of the first final block, and for L >= 4 the
// bytes of k >> 24 at p + 4, which change once every 2^24 k: the template
// holds the launch's first value (Launch::seg_first) and the kernel re-derives
// the K + M constants of the word(s) holding them when a wave moves into
// another 2^24-k segment.  For SH = 1-2 and L >= 6 the top chunk bytes reach
// word W0 + 2, which the kernel holds launch-uniform (word2_period).  Whole
// nonce-only blocks before p are hashed here once (midstate).
#include "plan.h"

#include <algorithm>

#include <string.h>

#include "md5_host.h"

namespace dpow {

uint32_t chunk_len_of(uint64_t k) {
    uint32_t n = 0;
    while (k) { ++n; k >>= 8; }
    return n;
}

uint64_t segment_end(uint64_t k) {
    const uint32_t L = chunk_len_of(k);
    if (L == 0) return 1;
    return 1ull << (8 * L);
}

uint64_t word2_period(uint32_t sh) {
    // k >> 24 sits at byte SH of the 64-bit pair (W0 + 1, W0 + 2): its bits from
    // 32 - 8 SH on land in W0 + 2.  SH = 3's W0 + 2 is a kernel segment word; for
    // SH = 0 nothing reaches W0 + 2 below DPOW_K_LIMIT.
    return (sh == 1 || sh == 2) ? 1ull << (56 - 8 * sh) : 0;
}

uint32_t remainder_bits(uint32_t worker_bits) { return 8u - (worker_bits % 9u); }

uint32_t base_thread_byte(uint32_t worker_byte, uint32_t worker_bits) {
    // uint8((int(WorkerByte) << remainderBits) | i) with i = 0 (worker.go:315)
    return (uint32_t)((worker_byte << remainder_bits(worker_bits)) & 0xFFu);
}

int WindowPlanner::init(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                        uint32_t worker_bits, uint64_t k_begin, uint64_t k_end) {
    if (nonce_len && !nonce) return -1;
    if (worker_byte > 255u) return -1;
    if (k_end > DPOW_K_LIMIT) return DPOW_ERANGE;
    nonce_ = nonce;
    nonce_len_ = nonce_len;
    ntz_ = ntz;
    rbits_ = remainder_bits(worker_bits);
    base_tb_ = base_thread_byte(worker_byte, worker_bits);
    blk_v_ = nonce_len / 64;  // first block holding variable bytes
    p_ = (uint32_t)(nonce_len % 64);
    k_ = k_begin;
    k_end_ = k_end;
    lspan_end_ = lspan_end(nonce_len, rbits_, ntz);
    // Midstate over nonce-only blocks.
    for (int w = 0; w < 4; ++w) iv_[w] = kMd5IV[w];
    for (size_t b = 0; b < blk_v_; ++b) {
        uint32_t M[16];
        for (int w = 0; w < 16; ++w) M[w] = load_le32(nonce + 64 * b + 4 * w);
        md5_compress(iv_, M);
    }
    return 0;
}

uint32_t WindowPlanner::nblk_of(uint32_t chunk_len) const {
    const size_t msg_len = nonce_len_ + 1 + chunk_len;
    return (uint32_t)((msg_len + 8) / 64 + 1 - blk_v_);
}

// Final-block words of the message nonce || threadByte || chunk_k with the variable bytes
// (threadByte and chunk bytes 0..2) zeroed: nonce tail, chunk bytes 3.. of k, the 0x80 pad
// and the bit length (RFC 1321 3.1-3.2).
void WindowPlanner::build_template(uint64_t k, uint32_t L, uint32_t nblk, uint32_t T[32]) const {
    uint8_t buf[128];
    memset(buf, 0, sizeof buf);
    const uint32_t p = p_;
    if (p) memcpy(buf, nonce_ + 64 * blk_v_, p);
    // buf[p] = threadByte and buf[p+1 .. p+min(L,3)] = low chunk bytes: variable (left 0).
    for (uint32_t j = 3; j < L; ++j) buf[p + 1 + j] = (uint8_t)(k >> (8 * j));
    buf[p + 1 + L] = 0x80;
    const uint64_t bits = (uint64_t)(nonce_len_ + 1 + L) * 8u;
    for (int j = 0; j < 8; ++j) buf[64 * nblk - 8 + j] = (uint8_t)(bits >> (8 * j));
    for (uint32_t w = 0; w < 32; ++w) T[w] = w < 16 * nblk ? load_le32(buf + 4 * w) : 0u;
}

uint64_t lspan_end(size_t nonce_len, uint32_t rbits, uint32_t ntz) {
    // SH = 0: the pads of chunk lengths 0..3 fall in words W0 / W0 + 1, whose K + M the
    // kernel re-derives per segment.  R >= 2: a power-of-two chunk of <= 2R wave-blocks puts
    // the boundaries k = 256 and 65536 (256 R and 65536 R indices) on claim boundaries.
    // A first hit expected within kLspanMaxExpect candidates: the spanning (_ls) kernels
    // hash 1.5-2 % slower than the per-length ones (register assignment), which outweighs
    // the two launches they save (~40 us) once the search is expected to run > ~1.5 ms
    // ([1,2,3,4]/8: 19.18 -> 19.45 ms merged).  Past that only chunk lengths 1 and 2 share
    // a launch (k < 2^16, 2^16 R candidates): their two launches cost 17 + 122 us against
    // 77 us of hashing (profiles/r03_tts_timeline_c.json, [1,2,3,4]/8).
    // Returns the k below which launches use the chunk-length-0 template (0: none).
    if (!(nonce_len % 4 == 0 && rbits >= 1)) return 0;
    return expected_first_hit(ntz, rbits) <= kLspanMaxExpect ? 1ull << 24 : 1ull << 16;
}

bool WindowPlanner::lseg_template(uint64_t k) const {
    return k < lspan_end_;
}

bool WindowPlanner::next(PlannedLaunch &pl) {
    if (k_ >= k_end_) return false;
    const uint64_t k = k_;
    memset(&pl, 0, sizeof pl);
    Launch &Lh = pl.L;
    const uint32_t p = p_;
    const uint64_t R = 1ull << rbits_;
    uint64_t ke = segment_end(k) < k_end_ ? segment_end(k) : k_end_;
    if (const uint64_t w2 = word2_period(p_ % 4)) {  // word W0 + 2 changes: end the launch
        const uint64_t we = (k / w2 + 1) * w2;
        if (we < ke) ke = we;
    }
    const uint64_t cap_end = cap_k_ && k_end_ - k > cap_k_ ? k + cap_k_ : k_end_;
    cap_k_ = 0;
    if (cap_end < ke) ke = cap_end;
    const uint32_t L = chunk_len_of(k);
    const uint32_t nblk = nblk_of(L);
    pl.k0 = k == 0;
    // (the k = 0 kernel hashes k = 0 from the real chunk-length-0 template: no deltas)
    uint32_t L_last = L;
    if (!pl.k0 && k >= 1 && lseg_template(k)) {
        // Merge the following chunk lengths (up to 3) with the same block count.
        uint64_t e = ke;
        while (e < k_end_ && e < lspan_end_ && nblk_of(chunk_len_of(e)) == nblk &&
               (segment_end(e) < k_end_ ? segment_end(e) : k_end_) <= cap_end) {  // whole segments only
            e = segment_end(e) < k_end_ ? segment_end(e) : k_end_;
            L_last = chunk_len_of(e - 1);
        }
        if (e > ke) {
            ke = e;
            Lh.lspan = 1;
        }
    }
    build_template(k, L, nblk, Lh.T);
    for (int w = 0; w < 4; ++w) Lh.iv[w] = iv_[w];
    if (lseg_template(k)) {
        // SH = 0 below k = 2^24: the template of chunk length 0 with this block count (the
        // kernel adds lseg_deltas(l) for a candidate of chunk length l, every segment).
        uint32_t d0, d1, dlen;
        lseg_deltas(L, d0, d1, dlen);
        const uint32_t w0 = p / 4, lenw = 16 * nblk - 2;
        if (w0 + 1 == lenw) {
            dlen += d1;
            d1 = 0;
        }
        Lh.T[w0] -= d0;
        Lh.T[w0 + 1] -= d1;
        Lh.T[lenw] -= dlen;
    }
    for (uint32_t b = 0; b < nblk; ++b)
        for (int s = 0; s < 64; ++s) Lh.KT[64 * b + s] = kMd5K[s] + Lh.T[16 * b + md5_word(s)];
    Lh.i_begin = k << rbits_;
    Lh.i_end = pl.k0 ? R : ke << rbits_;
    Lh.wb_begin = Lh.i_begin & ~(uint64_t)(kWaveBlock - 1);
    Lh.n_wblocks = (Lh.i_end - Lh.wb_begin + (uint64_t)kWaveBlock - 1) / (uint64_t)kWaveBlock;
    Lh.rbits = rbits_;
    Lh.base_tb = base_tb_;
    Lh.dmask = tail_nibble_mask(ntz_ < 8 ? ntz_ : 8);
    Lh.dle = tail_prefilter_le(ntz_);
    Lh.deq = 0u - iv_[3];
    Lh.ntz = ntz_;
    Lh.seg_first = (uint32_t)(k >> 24);
    Lh.seg0 = lseg_template(k) ? kLsegBase : seg_id(k);  // the template's own segment
    if (pl.k0) ke = 1;
    pl.info.k_begin = k;
    pl.info.k_end = ke;
    pl.info.i_begin = Lh.i_begin;
    pl.info.i_end = Lh.i_end;
    pl.info.nblk = nblk;
    pl.info.w0 = p / 4;
    pl.info.sh = p % 4;
    pl.info.chunk_len = L;
    pl.info.chunk_len_last = L_last;
    pl.info.start_kernel = pl.k0 ? 1u : 0u;
    k_ = ke;
    return true;
}

int plan_window(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                uint32_t worker_bits, uint64_t k_begin, uint64_t k_end, std::vector<PlannedLaunch> &out) {
    out.clear();
    WindowPlanner wp;
    int rc = wp.init(nonce, nonce_len, ntz, worker_byte, worker_bits, k_begin, k_end);
    if (rc < 0) return rc;
    PlannedLaunch pl;
    while (wp.next(pl)) out.push_back(pl);
    return (int)out.size();
}

// Words of one candidate, assembled as the kernel does (wave-uniform V + lane offset).
void candidate_words(const PlannedLaunch &pl, uint64_t local_idx, uint32_t words[32]) {
    const Launch &Lh = pl.L;
    for (uint32_t w = 0; w < 16 * pl.info.nblk; ++w) words[w] = Lh.T[w];
    const uint64_t i0 = local_idx & ~63ull;
    const uint32_t lane = (uint32_t)(local_idx & 63u);
    const uint32_t V = wave_uniform_v(i0, Lh.rbits, Lh.base_tb) + lane_offset(Lh.rbits, lane);
    const uint32_t sh = pl.info.sh, w0 = pl.info.w0;
    words[w0] += V << (8 * sh);
    if (sh) words[w0 + 1] += V >> (32 - 8 * sh);
    if (Lh.seg0 == kLsegBase && !pl.k0) {  // SH = 0 below 2^24: md5_search_kernel.h seg_all_deltas
        uint32_t d0, d1, dlen;
        // (the kernel takes a group's chunk length from its first index at or above i_begin)
        lseg_deltas(chunk_len_of(local_idx >> Lh.rbits), d0, d1, dlen);
        const uint32_t lenw = 16 * pl.info.nblk - 2;
        if (w0 + 1 == lenw) {
            dlen += d1;
            d1 = 0;
        }
        words[w0] += d0;
        words[w0 + 1] += d1;
        words[lenw] += dlen;
    }
    {  // the segment words, as the kernel re-derives them (md5_search_kernel.h seg_word)
        uint32_t d1, d2;
        const uint32_t seg = (uint32_t)((local_idx >> Lh.rbits) >> 24);
        seg_word_deltas(Lh.T[w0 + 1], Lh.T[w0 + 2], seg, Lh.seg_first, sh, d1, d2);
        words[w0 + 1] += d1;
        if (sh == 3 && w0 + 2 != 16 * pl.info.nblk - 2) words[w0 + 2] += d2;
    }
}

uint64_t expected_first_hit(uint32_t ntz, uint32_t rbits) {
    // A candidate passes with p = 16^-N (MD5's nibbles are uniform): the first hit of a
    // partition is geometric with mean 16^N R / 256 of its candidates, from any start.
    if (ntz >= 14) return ~0ull;
    return ((1ull << (4 * ntz)) << rbits) >> 8;
}

int size_launch(PlannedLaunch &pl, uint64_t max_blocks, uint64_t expect, uint64_t *worker_blocks_out,
                uint64_t min_chunk, uint64_t claims_per_wave) {
    Launch &L = pl.L;
    constexpr uint64_t wpb = kBlockThreads / 64;
    // Chunk: >= kClaimsPerWave claims per wave of the largest grid the launch gets, over
    // the launch -- or over the candidates before its expected first hit, when that is
    // sooner.  A wave hashes its claims in order, and the chunks claimed first (a wave's
    // current one and the one it claimed ahead) are held by every wave from the start,
    // the youngest waves of a SIMD progressing slowest until the launch drains: a hit
    // inside them waits for that.  A 537M-candidate launch (L = 3 at workerBits 3) with
    // its N = 7 hit 29M in took 1.44 ms at chunk 32, against 0.31 ms for the same hit
    // in a 36M-candidate launch at chunk 4 (profiles/r03_node_probe.json).
    uint64_t worker_blocks = (L.n_wblocks + wpb - 1) / wpb;
    if (worker_blocks > max_blocks) worker_blocks = max_blocks;
    uint64_t span_wb = L.n_wblocks;
    if (expect / (uint64_t)kWaveBlock < span_wb) span_wb = expect / (uint64_t)kWaveBlock;
    uint64_t chunk = span_wb / (worker_blocks * wpb * claims_per_wave);
    if (chunk < min_chunk) chunk = min_chunk;
    if (chunk > kMaxChunk) chunk = kMaxChunk;
    if ((pl.info.k_begin >> 24) != ((pl.info.k_end - 1) >> 24) || L.lspan) {
        // The launch spans 2^24-k segments: a power-of-two chunk and wave-blocks
        // counted from a multiple of chunk wave-blocks put every segment boundary
        // (a multiple of 2^24 * R indices) on a claim boundary, big or tail, so no
        // claim straddles one (the kernel switches constants per chunk group).
        // Chunk-length segments (lspan) end at k = 256 and 65536, i.e. 2R and 512R
        // wave-blocks: chunks of at most 2R wave-blocks.
        while (chunk & (chunk - 1)) chunk &= chunk - 1;
        if (L.lspan && chunk > (2ull << L.rbits)) chunk = 2ull << L.rbits;
        L.wb_begin = L.i_begin & ~(chunk * (uint64_t)kWaveBlock - 1);
        L.n_wblocks = (L.i_end - L.wb_begin + (uint64_t)kWaveBlock - 1) / (uint64_t)kWaveBlock;
        // The realignment adds up to chunk - 1 wave-blocks: size the grid on the new count.
        worker_blocks = (L.n_wblocks + wpb - 1) / wpb;
        if (worker_blocks > max_blocks) worker_blocks = max_blocks;
    }
    // Guided tail: the last ~kTailClaimsPerWave claims per wave are kMinChunk
    // wave-blocks, so the waves of a launch run dry together.
    const uint64_t chunk_tail = kTailChunk < chunk ? kTailChunk : chunk;
    const uint64_t tail_wb = worker_blocks * wpb * kTailClaimsPerWave * chunk_tail;
    const uint64_t n_big = L.n_wblocks > tail_wb ? (L.n_wblocks - tail_wb) / chunk : 0;
    const uint64_t rest = L.n_wblocks - n_big * chunk;
    const uint64_t n_chunks = n_big + (rest + chunk_tail - 1) / chunk_tail;
    // No more waves than claims, but a worker block for every counter that holds
    // a claim (block b serves counter (b - 1) % kClaimCounters).
    uint64_t need_blocks = (n_chunks + wpb - 1) / wpb;
    if (need_blocks < n_chunks && need_blocks < kClaimCounters)
        need_blocks = n_chunks < kClaimCounters ? n_chunks : kClaimCounters;
    if (worker_blocks > need_blocks) worker_blocks = need_blocks;
    // Tail claims smaller than a workgroup's share (kTailChunk < kMinChunk) can give a
    // few-wave-block launch more claims than its wave-block count asked workgroups for.
    const uint64_t min_blocks = n_chunks < kClaimCounters ? n_chunks : kClaimCounters;
    if (worker_blocks < min_blocks && min_blocks <= max_blocks) worker_blocks = min_blocks;
    if (worker_blocks < kClaimCounters && worker_blocks < n_chunks) return DPOW_EINVAL;
    L.chunk = (uint32_t)chunk;
    L.chunk_tail = (uint32_t)chunk_tail;
    L.n_big = n_big;
    L.n_chunks = n_chunks;
    L.n_head = 2 * worker_blocks * wpb;
    // Static first claims (md5_search_kernel.h kStaticFirst): the "_ls" kernels (the
    // chunk-length-0 template, L.seg0 == kLsegBase) hand claim w to worker wave w.  Every
    // counter that holds a claim beyond them still has a workgroup (checked above on
    // n_chunks, which bounds the counters' share too).
    L.n_static = L.seg0 == kLsegBase && !pl.k0
                     ? (n_chunks < worker_blocks * wpb ? n_chunks : worker_blocks * wpb)
                     : 0;
    *worker_blocks_out = worker_blocks;
    return 0;
}

uint32_t launch_poll_wb(uint32_t ntz, uint32_t rbits) {
    const uint32_t slow = DPOW_POLL_WB > 0 ? DPOW_POLL_WB : 16;
    const uint64_t expect = expected_first_hit(ntz, rbits);
    if (expect <= kTinyExpect) return 1;
    if (expect <= kNearExpect) return kNearPollWb;
    if (expect <= kMidExpect) return kMidPollWb;
    return expect <= kFastPollCands ? kFastPollWb : slow;
}

uint64_t launch_claims_per_wave(uint32_t ntz, uint32_t rbits) {
    return expected_first_hit(ntz, rbits) <= kFastPollCands ? kShortClaimsPerWave : kClaimsPerWave;
}

uint64_t launch_min_chunk(uint32_t ntz, uint32_t rbits) {
    const uint64_t expect = expected_first_hit(ntz, rbits);
    if (expect <= kTinyExpect) return kTinyChunk;
    return expect > kMidChunkExpect && expect <= kMidExpect ? kMidChunk : kMinChunk;
}

int size_search_launch(PlannedLaunch &pl, uint32_t ntz, uint64_t cus, uint64_t share, const LaunchKnobs &knobs,
                       uint64_t *worker_blocks, uint64_t active) {
    Launch &L = pl.L;
    share = std::max<uint64_t>(share, 1);
    active = std::max<uint64_t>(active, share);
    const uint64_t bpc = knobs.bpc ? knobs.bpc : launch_blocks_per_cu(L.i_end - L.i_begin, ntz, L.rbits, active);
    const uint64_t max_blocks = std::max<uint64_t>(cus * bpc / share, kClaimCounters);
    const int rc = size_launch(pl, max_blocks, expected_first_hit(ntz, L.rbits), worker_blocks,
                               knobs.min_chunk ? knobs.min_chunk : launch_min_chunk(ntz, L.rbits),
                               knobs.cpw ? knobs.cpw : launch_claims_per_wave(ntz, L.rbits));
    if (rc < 0) return rc;
    L.poll_wb = knobs.poll_wb ? knobs.poll_wb : launch_poll_wb(ntz, L.rbits);
    return 0;
}

uint64_t grid_share(uint64_t active, const LaunchKnobs &knobs) {
    const uint64_t cap = knobs.share_max ? knobs.share_max : kShareMax;
    return std::max<uint64_t>(1, std::min(active, cap));
}

bool cap_shared_launch(WindowPlanner &planner, PlannedLaunch &pl, uint64_t active, const LaunchKnobs &knobs) {
    if (active <= 1 || pl.k0) return false;
    const double ns = knobs.share_launch_us ? knobs.share_launch_us * 1e3 : (double)kShareLaunchNs;
    const uint64_t cap_k = std::max<uint64_t>(1, (uint64_t)(kEstRate / (double)active * ns * 1e-9) >> pl.L.rbits);
    if (pl.info.k_end - pl.info.k_begin <= cap_k) return false;
    planner.restart(pl.info.k_begin, cap_k);
    planner.next(pl);
    return true;
}

uint64_t launch_blocks_per_cu(uint64_t candidates, uint32_t ntz, uint32_t rbits, uint64_t share) {
    // Small grids for short launches: candidates of this partition expected before its first hit: 16^N R / 256, and the
    // launch's, in device time (times the searches sharing the device; saturating).
    const auto dev = [share](uint64_t v) { return share > 1 && v > ~0ull / share ? ~0ull : v * (share ? share : 1); };
    const uint64_t expect = dev(expected_first_hit(ntz, rbits));
    const uint64_t eff = dev(candidates) < expect ? dev(candidates) : expect;
    if (expect <= kTinyExpect || dev(candidates) <= kTinyLaunch) return kMaxBlocksPerCu < 2 ? kMaxBlocksPerCu : 2;
    if (eff <= (1ull << 22)) return kMaxBlocksPerCu < 3 ? kMaxBlocksPerCu : 3;
    if (eff <= kMidExpect) return kMaxBlocksPerCu < 4 ? kMaxBlocksPerCu : 4;
    if (kFiveExpect && expect <= kFiveExpect) return kMaxBlocksPerCu < 5 ? kMaxBlocksPerCu : 5;
    return kMaxBlocksPerCu;
}

}  // namespace dpow
