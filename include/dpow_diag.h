/*
 * dpow_diag.h -- diagnostics of libdpow.so (not part of the reference's
 * interface): measures what bounds the search kernel on this device.
 */
#ifndef DPOW_DIAG_H
#define DPOW_DIAG_H

#ifdef __cplusplus
extern "C" {
#endif

/* Sustained VALU issue rate on `device` for one instruction kind, all CUs busy
 * (8 waves per SIMD, 8 independent chains per lane):
 *   kind 0 v_add_u32, 1 v_add3_u32, 2 v_alignbit_b32, 3 v_bitop3_b32,
 *        4 v_fma_f32, 5 the MD5 step mix (bitop3, add3, alignbit, add),
 *        6 v_lshl_add_u32, 7 v_lshl_or_b32, 8 v_xad_u32, 9 v_perm_b32, 10 v_lshlrev_b32,
 *        11 v_or3_b32, 12 v_add_u32 with a literal, 13 v_alignbyte_b32, 14 v_bfi_b32,
 *        15 v_add_lshl_u32, 16 v_xor_b32, 17 v_add3_u32 with an SGPR operand, 18 v_pk_add_u16,
 *        19 the MD5 step mix interleaved across all 8 chains per instruction, 20 the same
 *        interleaved across pairs of chains, 21 as 20 with two v_add_u32 instead of v_add3_u32,
 *        22 two chains software-pipelined so full- and half-rate instructions alternate,
 *        23 the step mix with the v_add3_u32 constant in an SGPR (as the kernel issues it),
 *        24 two candidates with MD5's real dependencies (4 state words each), compiler order,
 *        25 the same in the search kernel's hand-ordered alternating groups,
 *        26/27 kind 22's pattern on fixed registers whose operands sit in distinct / the
 *        same VGPR bank (register index mod 4), 28 v_mad_u32_u24, 29 v_dot2_u32_u16,
 *        30 v_bitop3_b16, 31 v_lshlrev_b64, 32 v_lshl_add_u64, 33 v_pk_mov_b32 (31-33 count
 *        one instruction per register pair), 34 v_add_u32_sdwa (src1 WORD_1), 35 v_add_u16_sdwa
 *        (dst WORD_1, low half preserved), 36 the kernel's order-2 step pair with a 16-bit
 *        rotate, 37 the same with each rotate + add as two SDWA adds.
 * *lane_ops_per_s = wave64 instructions x 64 / s; *clock_ghz = mean in-kernel
 * shader clock (s_memtime / s_memrealtime).  Returns 0, or < 0 on error. */
int dpow_diag_valu_rate(int device, int kind, double *lane_ops_per_s, double *clock_ghz);

/* Host round trip of a one-workgroup launch on `device`, median over `reps`:
 *   mode 0: launch + hipStreamSynchronize;
 *   mode 1: launch + spin on a pinned host word the kernel writes (system scope);
 *   mode 2: a 16-byte device->host hipMemcpyAsync + hipStreamSynchronize.
 * The floor under time-to-secret at small N.  Returns 0, or < 0 on error. */
int dpow_diag_launch_latency(int device, int mode, int reps, double *median_us);

/* The hash loop's per-candidate D-word test (md5_search_kernel.h hash_wave_block), on
 * the host, with the launch fields the planner derives for (nonce, ntz) at chunk index
 * k: the one-compare prefilter (state word == -iv[3] for the D-equality kernels, else
 * D <= dle) and the rare path's exact nibble mask.  `state_d` is the last block's raw D
 * state word, D = iv_d + state_d, where iv_d is the chaining value entering that block
 * (for two final blocks the first block's output, per candidate, so the caller passes
 * it).  Returns 1 if the candidate reaches the hit path (for ntz > 8 still subject to
 * the full-digest check), 0 if not, < 0 on error. */
int dpow_diag_dword_test(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint64_t k,
                         uint32_t iv_d, uint32_t state_d);

/* Claim geometry dpow_search gives each launch of a window (host logic, no GPU), sized by
 * the same functions dpow_search uses (plan.cpp size_search_launch, grid_share,
 * cap_shared_launch): the device share (cus x the ntz- and size-dependent workgroups per CU
 * / min(share, 2), at least one per claim counter), the expected first hit at ntz, the
 * minimum chunk, the claims per wave and the poll group.  `share` is the number of searches
 * in flight on the device (1 alone); above 1 the window is cut into ~8 ms launches.  One
 * entry per launch; returns the number of launches (only the first max_launches are
 * written), or < 0 when a launch would leave a claim counter without waves.
 * (ABI 3: ntz, cus and share replace round 3's max_blocks, which sized every launch as an
 * ntz-less full grid and so never covered the short searches' grids.) */
typedef struct dpow_diag_launch {
    uint64_t k_begin, k_end;      /* chunk range */
    uint64_t i_begin, i_end;      /* local index range */
    uint64_t wb_begin;            /* first wave-block's local index */
    uint64_t n_wblocks;           /* wave-blocks from wb_begin covering i_end */
    uint64_t n_big, n_chunks;     /* claims of `chunk` wave-blocks, all claims */
    uint64_t worker_blocks;       /* worker workgroups launched (plus the watcher) */
    uint32_t chunk, chunk_tail;   /* wave-blocks per big / tail claim */
    uint32_t rbits;               /* R = 2^rbits thread bytes per k */
    uint32_t wave_block;          /* local indices per wave-block */
    uint64_t n_static;            /* claims handed out by wave index (the "_ls" kernels' static first claims) */
    uint32_t poll_wb;             /* wave-blocks per poll group */
    uint32_t pad;
} dpow_diag_launch;
int dpow_diag_launch_geometry(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                              uint32_t worker_bits, uint64_t k_begin, uint64_t k_end, uint32_t cus,
                              uint32_t share, dpow_diag_launch *out, size_t max_launches);

/* Worker workgroups per CU dpow_search gives a launch of `candidates` local indices
 * at (ntz, worker_bits) on a device it has alone (plan.cpp launch_blocks_per_cu): 6 (the
 * full persistent grid) unless the launch is short or a first hit is expected early
 * (16^ntz R / 256 candidates): 2 for a hit expected within 2^23 (round 5; 2^21 before) or
 * a launch of at most 2^21, else by the smaller of the two: 3 up to 2^22, 4 up to 2^26,
 * and 5 while the hit is expected within 2^31. */
uint64_t dpow_diag_blocks_per_cu(uint64_t candidates, uint32_t ntz, uint32_t worker_bits);

/* Host timeline of the context's last dpow_search call, ns from its start (-1: did not
 * happen): [0] the k = 0 kernel queued, [1] the first md5 launch queued, [2] the first
 * completion record seen, [3] the search done (before the host MD5 re-verification),
 * [4] the first launch planned, [5] the k = 0 kernel's record slot retired, [6] the
 * first md5 launch's record slot retired, [7] the search's own hit posted to its node slot
 * by the early Found fan-out.
 * Environment overrides read at dpow_open (A/B runs only): DPOW_DIAG_POLL_WB (wave-blocks
 * per poll group), DPOW_DIAG_BPC (worker workgroups per CU), DPOW_DIAG_MIN_CHUNK (minimum
 * wave-blocks per claim, a power of two), DPOW_DIAG_CPW (big claims per wave: the chunk
 * sizing), DPOW_DIAG_SHARE_LAUNCH_US (launch length while the device is shared),
 * DPOW_DIAG_SHARE_MAX (grid share cap).  Returns 0, or < 0 on error. */
int dpow_diag_search_times(struct dpow_ctx *ctx, int64_t out[8]);

/* The launches of the context's last dpow_search call, in launch order (round 5): the
 * host's CLOCK_MONOTONIC ns when each was queued and when its completion record was
 * consumed (-1: not consumed, e.g. left in flight behind a hit or a covered bound), and
 * the record's device s_memrealtime stamps (100 MHz; the k = 0 kernel's own, an md5
 * launch's start as its watcher stamps it and its end as the last workgroup publishes it;
 * 0 while the record is not written).  *t0_ns: the search's start (CLOCK_MONOTONIC ns).
 * Returns the number of launches (at most 32 are kept; only max_launches are written),
 * or < 0 on error.  dpow_diag_clock_sync maps the device stamps to host time. */
typedef struct dpow_diag_launch_time {
    uint64_t seq;                 /* launch sequence number of the context */
    int32_t kind;                 /* 0 the k = 0 kernel, 1 an md5 launch */
    int32_t recorded;             /* its completion record is written */
    int64_t queued_ns, seen_ns;   /* host: queued, record consumed (-1: not) */
    uint64_t t_start_tick, t_end_tick;  /* device s_memrealtime stamps of the record */
    uint64_t candidates, g_end;   /* local indices; global indices below g_end */
    uint64_t best;                /* the record's best (DPOW_NO_HIT: none) */
} dpow_diag_launch_time;
int dpow_diag_search_launches(struct dpow_ctx *ctx, int64_t *t0_ns, dpow_diag_launch_time *out,
                              size_t max_launches);

/* Pairs the device's s_memrealtime clock with the host's CLOCK_MONOTONIC: `reps` one-thread
 * kernels on the context's stream stamp s_memrealtime into pinned host memory while the
 * host spins on it.  *offset_ns = min over reps of (host ns when the stamp was seen -
 * stamp x 10 ns), so host ns ~= tick x 10 + *offset_ns, late by the stamp's write latency
 * to host memory (~1 us).  Waits for the stream first.  Returns 0, or < 0 on error. */
int dpow_diag_clock_sync(struct dpow_ctx *ctx, int reps, int64_t *offset_ns);

/* The node vote's cost to a node's time-to-secret (dpow_node_vote, round 5), on this host:
 * `world` threads on CPUs spread over the caller's affinity set; ranks 1..world-1 vote first
 * and wait in the vote, rank 0 (the calling thread) votes last.  *last_us: rank 0's vote call;
 * *all_us: from rank 0's call until every rank holds the result.  Medians over `reps`.
 * tools/node_probe.py adds *all_us to the slowest rank's time.  Returns 0, or < 0 on error. */
int dpow_diag_vote_latency(uint32_t world, int reps, double *last_us, double *all_us);

/* Node emulation on one GPU (tools/node_probe.py): post global_idx to a node slot
 * (dpow_node_post) from a detached native thread at CLOCK_MONOTONIC time t_ns, as another
 * rank's process would -- off the caller's thread and its Python interpreter lock.
 * Returns 0, or < 0 on error. */
int dpow_diag_node_post_at(struct dpow_node_slot *slot, uint64_t global_idx, int64_t t_ns);

/* The device alias of the slot attached to ctx, as its watcher reads it (*cached: from the page
 * registry), and as hipHostGetDevicePointer gives it now under ctx's device (*lookup).  They
 * must agree for every context of a process, whatever device registered the page first
 * (round 6: the registry keeps one alias per device).  DPOW_EINVAL when no slot is attached. */
int dpow_diag_node_alias(struct dpow_ctx *ctx, void **cached, void **lookup);

/* Environment knob (no entry point): DPOW_DIAG_BOARD_SPLIT=1 makes dpow_board_search run every
 * rank on its own partition even when all ranks share one GPU -- the multi-GPU role, for tests
 * on a one-GPU box (tests/test_coordinator.py). */

#ifdef __cplusplus
}
#endif
#endif /* DPOW_DIAG_H */
