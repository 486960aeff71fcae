// fw_merge_hopb.h -- k_merge_hopb: the flush + fire kernel of SQL HOP windows with block state.
//
// The slice-per-entry state of k_merge_fire keeps one (key, slice) entry per live slice, and a HOP
// fire follows the key's timer chain of windows, each probing the LDS index for its n slices
// (SliceSharedSyncStateWindowAggProcessor.fireWindow :65-86 with merge :89-118 over
// HoppingSlicesIterable).  Here one entry holds a BLOCK of HB_R consecutive slices of one key
// (block start aligned to HB_R slice intervals from the window offset): (key, block start, data
// mask, acc[HB_R][NWP]).  A partial folds into its slice's slot; a window is the register fold of
// at most two neighbouring blocks, newest slice first (the reference's merge order); and the
// timers become arithmetic: the reference fires exactly the non-empty windows whose end the
// watermark passes (a flushed slice registers its own window end, and nextTriggerWindow chains on
// while the window is not empty, HoppingSliceAssigner.nextTriggerWindow; a late record registers
// the first unfired window holding it, AbstractSliceSyncStateWindowAggProcessor.processElement
// :111-117), so an advance from W0 to W fires every window ending in (W0, W] that holds data --
// each found by the block holding its end slice, or by the block before it when that block does
// not exist.  clearWindow's expiry becomes: a slice is dropped once its last window has fired.
//
// Used for SQL HOP (ONE and GLOBAL phase) with n_slices <= HB_R, NWP <= 2 accumulator words and no
// SQL MIN/MAX(DOUBLE) word groups; every other HOP configuration runs k_merge_fire.
#pragma once
#include "fw_merge_impl.h"

namespace fw {


// Finds (k, bs) or inserts it with an identity ring; *inserted tells the caller it was new.
template <int NWP, int E, uint32_t OPS>
__device__ int hb_find_or_insert(StateLds<HB_R * NWP, E>& S, int64_t k, int64_t bs, const WordDesc& wd) {
    constexpr int NA = HB_R * NWP;
    constexpr uint32_t MASK = StateLds<NA, E>::NI - 1;
    uint32_t h = index_hash(k, bs) & MASK;
    for (int probes = 0; probes < StateLds<NA, E>::NI;) {
        const uint32_t st = __hip_atomic_load(&S.idx[h], __ATOMIC_RELAXED, LDS_SCOPE);
        if (st == 1) continue;
        if (st == 0) {
            uint32_t expect = 0;
            if (__hip_atomic_compare_exchange_strong(&S.idx[h], &expect, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     LDS_SCOPE)) {
                const int e = atomicAdd(&S.n, 1);
                if (e >= E) {
                    S.overflow = 1;
                    __hip_atomic_store(&S.idx[h], IDX_DEAD, __ATOMIC_RELAXED, LDS_SCOPE);
                    return -1;
                }
                S.key[e] = k;
                S.slice[e] = bs;
                S.flag[e] = 0;
#pragma unroll
                for (int i = 0; i < NA; i++) {
                    const int w = i % NWP;
                    S.acc[i][e] = word_on<OPS>(wd, w) ? word_identity(word_op<OPS>(wd, w)) : 0;
                }
                compiler_fence();
                __hip_atomic_store(&S.idx[h], 2u + (uint32_t)e, __ATOMIC_RELAXED, LDS_SCOPE);
                return e;
            }
            continue;
        }
        const uint32_t e = st - 2;
        if (e < (uint32_t)E && S.key[e] == k && S.slice[e] == bs) return (int)e;
        h = (h + 1) & MASK;
        probes++;
    }
    S.overflow = 1;
    return -1;
}

// a narrow entry (hb_narrow_words, level L) <-> the LDS entry
template <int NWP, int E, uint32_t OPS, int L>
__device__ __forceinline__ void hb_load_narrow(const MergeArgs& a, const uint64_t* src, StateLds<HB_R * NWP, E>& S, int e,
                                               int64_t* k, int64_t* bs) {
    constexpr int NA = HB_R * NWP, PN = hb_narrow_words(NWP, L), SB = hb_slot_bytes(L);
    uint64_t p[PN];
    load_words<PN>(src, p);
    *k = (int64_t)p[0];
    *bs = wadd((int64_t)(uint32_t)p[1] * a.win.hb_span, a.win.offset);  // the block index
    const uint32_t fl = (uint32_t)(p[1] >> 32) & 0xFFFFu;
    S.flag[e] = fl;
    const uint32_t mask = fl >> HB_MASK_SHIFT;
#pragma unroll
    for (int i = 0; i < NA; i++) {
        const int b = HB_HDR_BYTES + SB * i;  // the slot's byte offset in the entry
        const uint64_t raw = p[b >> 3] >> (8 * (b & 7));
        const int64_t v = SB == 4 ? (int64_t)(int32_t)(uint32_t)raw : (int64_t)(int16_t)(uint16_t)raw;
        const int w = i % NWP;
        S.acc[i][e] = ((mask >> (i / NWP)) & 1u) ? (uint64_t)v
                      : word_on<OPS>(a.wd, w) ? word_identity(word_op<OPS>(a.wd, w)) : 0;
    }
}
template <int NWP, int E, int L>
__device__ __forceinline__ void hb_store_narrow(const WinDesc& w, uint64_t* dst, const StateLds<HB_R * NWP, E>& S, int e, uint32_t fl) {
    constexpr int NA = HB_R * NWP, PN = hb_narrow_words(NWP, L), SB = hb_slot_bytes(L);
    const uint32_t mask = fl >> HB_MASK_SHIFT;
    uint64_t p[PN];
#pragma unroll
    for (int i = 0; i < PN; i++) p[i] = 0;
    p[0] = (uint64_t)S.key[e];
    // the block index (the write-back checked that it fits 31 bits) and the 16 flag bits
    p[1] = udiv((uint64_t)wsub(S.slice[e], w.offset), w.hb_span_div) | ((uint64_t)(fl & 0xFFFFu) << 32);
#pragma unroll
    for (int i = 0; i < NA; i++) {
        const int b = HB_HDR_BYTES + SB * i;
        const uint64_t v = ((mask >> (i / NWP)) & 1u) ? (S.acc[i][e] & (SB == 4 ? 0xFFFFFFFFull : 0xFFFFull)) : 0ull;
        p[b >> 3] |= v << (8 * (b & 7));
    }
    store_words<PN>(dst, p);
}

// block start of a slice end and the slice's slot in it
__device__ __forceinline__ int64_t hb_block_of(const WinDesc& w, int64_t se) {
    return window_start(wsub(se, 1), w.offset, w.hb_span_div);
}
__device__ __forceinline__ int hb_slot_of(const WinDesc& w, int64_t se, int64_t bs) {
    return (int)udiv((uint64_t)wsub(se, bs), w.slice_div) - 1;
}

// the fold of one slot into acc (merge in the reference's order: acc is the newer side)
template <int NWP, int E, uint32_t OPS>
__device__ __forceinline__ void hb_merge_slot(const MergeArgs& a, const StateLds<HB_R * NWP, E>& S, int e, int slot,
                                              uint64_t* acc) {
    uint64_t o[NWP];
#pragma unroll
    for (int w = 0; w < NWP; w++) o[w] = S.acc[slot * NWP + w][e];
    merge_slice<NWP, false, OPS>(a.wd, a.ad, acc, o);
}

// Fires the windows entry e is responsible for: those ending in its block, and -- when the key has
// no entry for the next block -- those ending in the next block that still hold slices of this one.
// A window fires iff it ends in (W0, W] and holds data.  Returns the windows fired.
template <int NWP, int E, uint32_t OPS>
__device__ __forceinline__ uint32_t hb_fire_entry(const MergeArgs& a, int64_t W, StateLds<HB_R * NWP, E>& S, int e, int64_t w_old, int sb,
                                  int32_t* s_emit) {
    const WinDesc& w = a.win;
    const int n = w.n_slices;
    const int64_t k = S.key[e], bs = S.slice[e];
    const uint32_t mask = S.flag[e] >> HB_MASK_SHIFT;
    if (!mask) return 0;
    // candidate window ends: slot j's slice end, j in [0, HB_R + n - 1)
    int prev = -2, next = -2;  // neighbouring blocks' entries, looked up on first need
    if (FW_ABL(a) & AB_M_NO_HASH) prev = next = -1;  // (diagnostic: fire without neighbour lookups)
    uint32_t nf = 0;
    // UTC: the due window ends lie in (w_old + 1, W + 1], so only the candidates j in
    // [floor((w_old - bs) / slide), floor((W - bs + 1) / slide)] -- a superset by at most one on
    // each side; the exact test below still decides -- need a look (about 2 + advance / slide of
    // the 12, the rest of the loop's iterations cost as much as the windows it fires)
    int j0 = 0, j1 = HB_R + n - 2;
    if (w.tz.n == 0) {
        if (W < bs) return 0;  // every candidate window end is >= bs + slide > W + 1
        j1 = (int)min((uint64_t)j1, udiv((uint64_t)W - (uint64_t)bs + 1u, w.slice_div));
        if (w_old >= bs) j0 = (int)min((uint64_t)(HB_R + n - 1), udiv((uint64_t)w_old - (uint64_t)bs, w.slice_div));
    }
    for (int j = j0; j <= j1; j++) {
        const int64_t we = wadd(bs, (int64_t)(j + 1) * w.interval);
        if (!win_fired(w, we, W) || win_fired(w, we, w_old)) continue;  // not due in this advance
        // the window's slots: j, j-1, ..., j-n+1 (newest first); < 0: previous block, >= HB_R: next
        const int lo = j - n + 1;
        if (j >= HB_R) {  // the next block fires it if it exists
            if (next == -2) next = find_entry(S, k, wadd(bs, w.hb_span));
            if (next >= 0) continue;
        }
        // data in this block's part of the window?  (the next block's part is empty: no entry)
        const int a0 = max(lo, 0), a1 = min(j, HB_R - 1);
        uint32_t here = a1 >= a0 ? (mask >> a0) & ((2u << (a1 - a0)) - 1u) : 0u;
        uint32_t before = 0;
        if (lo < 0) {
            if (prev == -2) prev = find_entry(S, k, wsub(bs, w.hb_span));
            if (prev >= 0) {
                const uint32_t pm = S.flag[prev] >> HB_MASK_SHIFT;
                before = pm >> (HB_R + lo);  // slots HB_R+lo .. HB_R-1 of the previous block
            }
        }
        if (!here && !before) continue;  // empty window: no output (its timer would fire silently)
        uint64_t acc[NWP];
        acc_identity<NWP, OPS>(a.wd, acc);
        for (int t = min(j, HB_R - 1); t >= max(lo, 0); t--)
            if ((mask >> t) & 1u) hb_merge_slot<NWP, E, OPS>(a, S, e, t, acc);
        if (before)
            for (int t = HB_R - 1; t >= HB_R + lo; t--)
                if ((before >> (t - (HB_R + lo))) & 1u) hb_merge_slot<NWP, E, OPS>(a, S, prev, t, acc);
        nf++;
        if (a.ad.count_star_word < 0 || acc[a.ad.count_star_word] != 0) emit_row<NWP, false>(a, sb, s_emit, k, we, acc);
    }
    return nf;
}

template <int NWP, int E, uint32_t OPS, int GF>
__global__ __launch_bounds__(MG_BLOCK, 4) void k_merge_hopb(MergeArgs a) {
    constexpr bool PS = (GF & GF_PASS) != 0;
    constexpr int NA = HB_R * NWP;  // ring words per entry
    constexpr int PW = 2 + NWP;     // partial row words
    constexpr int PWE = 3 + NA;     // state entry words
    constexpr int PW1 = hb_narrow_words(NWP, 1), PW2 = hb_narrow_words(NWP, 2);  // ... in the narrow layouts
    const int64_t CH = a.chunk_rows;
    constexpr int GU = mg_rows_in_flight(NWP);
    __shared__ StateLds<NA, E> S;
    __shared__ int32_t s_work;
    __shared__ int32_t s_nlive;
    __shared__ int64_t s_newmin;
    __shared__ uint32_t s_fired;
    __shared__ int32_t s_emit;
    __shared__ int32_t s_tk;

    const int tid = threadIdx.x;
    kt_start(a.kt);
    Ctrl* c = a.ctrl;
    const WinDesc& win = a.win;
    const int64_t W = merge_watermark(a);
    const int64_t cur = __hip_atomic_load(&c->cur, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t pend = __hip_atomic_load(&c->pending_pushes, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t ntp = __hip_atomic_load(&c->ntp, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t minp = __hip_atomic_load(&c->min_pending, __ATOMIC_RELAXED, DEV_SCOPE);
    const bool adv = !a.force_flush && W > cur;
    const bool do_flush = pend > 0 && (a.force_flush || (adv && (W >= ntp && win_fired(win, minp, W))));
    const bool do_fire = adv;
    const int64_t w_old = cur;
    const int64_t w_new = adv ? W : cur;  // the watermark after this launch (slice expiry)
    // late-record timer requests (n_treq) need no work here: their windows fire by holding data

    const bool xq = a.n_sb % 8 == 0 && gridDim.x % 8 == 0;
    const int nq = xq ? a.n_sb / 8 : a.n_sb;
    uint32_t* const wq = &a.tickets->work[xq ? blockIdx.x % 8 : 0][0];
    const int qbase = xq ? (int)(blockIdx.x % 8) * nq : 0;
    if (tid == 0) s_tk = (int32_t)__hip_atomic_fetch_add(wq, 1u, __ATOMIC_RELAXED, DEV_SCOPE);
    if (!do_flush) {  // nothing to gather: work only where a window is due
        bool due = false;
        for (int i = tid; i < nq; i += MG_BLOCK) due |= do_fire && win_fired(win, a.sb_min_timer[qbase + i], W);
        if (!__syncthreads_or(due)) {
            if (a.reset_out)
                for (int i = tid; i < nq; i += MG_BLOCK) a.sb_out[qbase + i] = 0;
            s_tk = nq;
        }
    }
    __syncthreads();
    for (int tk = s_tk; tk < nq; tk = s_tk) {
        const int sb = qbase + tk;
        const int32_t n0 = a.state_count[sb];
        __syncthreads();
        if (tid == 0) {
            s_tk = (int32_t)__hip_atomic_fetch_add(wq, 1u, __ATOMIC_RELAXED, DEV_SCOPE);
            s_work = do_flush || (do_fire && win_fired(win, a.sb_min_timer[sb], W));
            s_fired = 0;
            s_emit = a.reset_out ? 0 : a.sb_out[sb];
            if (!s_work && a.reset_out) a.sb_out[sb] = 0;
        }
        __syncthreads();
        if (!s_work) continue;
        auto cell_at = [&](int64_t pi, int f) -> uint32_t {  // cells of this superbucket's ingest superbucket
            if (cell_chunk(f) >= a.slot_nch[pi]) return 0u;
            const int pl = PS ? a.ks.pass_log2 : 0;
            const int nis = a.n_sb >> pl;
            const uint32_t* cl = a.cells + (size_t)pi * nis * a.max_nch;
            return cl[((size_t)(f >> 4) * nis + (sb >> pl)) * CELL_LANES + (f & 15)];
        };
        const int lane = tid & 63, wv = tid >> 6;
        auto gather_group = [](int ncell) { return min(64, ncell / (MG_BLOCK / 64)); };
        // this lane's cell word of its wave's first group in push 0 (the next push's is loaded at the top
        // of each push's loop)
        uint32_t v_first = 0;
        if (do_flush && !a.runs && lane < gather_group((int)cell_pad(a.slot_nch[0])))
            v_first = cell_at(0, wv * gather_group((int)cell_pad(a.slot_nch[0])) + lane);
        // ---- load the superbucket's block entries into LDS
        for (int i = tid; i < StateLds<NA, E>::NI; i += MG_BLOCK) S.idx[i] = 0;
        if (tid == 0) {
            S.n = n0;
            S.overflow = 0;
        }
        __syncthreads();
        const uint64_t* st = a.state + (size_t)sb * a.cap_e * PWE;
        const int lv_in = a.sb_nar[sb];  // (uniform) the layout the last write-back chose
        if ((FW_ABL(a) & AB_M_NO_LOAD) && tid == 0) S.n = 0;  // (diagnostic ablations: timing only)
        if (!(FW_ABL(a) & AB_M_NO_LOAD)) for (int e = tid; e < n0; e += MG_BLOCK) {
            int64_t k, bs;
            if (lv_in == 2) {
                hb_load_narrow<NWP, E, OPS, 2>(a, st + (size_t)e * PW2, S, e, &k, &bs);
            } else if (lv_in == 1) {
                hb_load_narrow<NWP, E, OPS, 1>(a, st + (size_t)e * PW1, S, e, &k, &bs);
            } else {
                uint64_t p[PWE];
                load_words<PWE>(st + (size_t)e * PWE, p);
                k = (int64_t)p[0];
                bs = (int64_t)p[1];
                S.flag[e] = (uint32_t)p[2];
#pragma unroll
                for (int i = 0; i < NA; i++) S.acc[i][e] = p[3 + i];
            }
            S.key[e] = k;
            S.slice[e] = bs;
            uint32_t h = index_hash(k, bs) & (StateLds<NA, E>::NI - 1);
            for (;;) {
                uint32_t expect = 0;
                if (__hip_atomic_compare_exchange_strong(&S.idx[h], &expect, 2u + (uint32_t)e, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, LDS_SCOPE))
                    break;
                h = (h + 1) & (StateLds<NA, E>::NI - 1);
            }
        }
        __syncthreads();
        // ---- flush: every pending partial (key, sliceEnd, acc) folds into its block's slot (the
        // software-pipelined gather of k_merge_fire was measured out here: round 3)
        const bool gather = do_flush && !(FW_ABL(a) & AB_M_NO_GATHER);
        if (gather && a.runs) {  // runs (IngestArgs::runs), then the rows chunks kept in their regions
            auto fold_rows = [&](auto& row, uint32_t live) __attribute__((always_inline)) {
                constexpr int GX = std::extent<std::remove_reference_t<decltype(row)>>::value;
                int ge[GX], slot[GX];
                {
                    int64_t gk[GX], gb[GX];
#pragma unroll
                    for (int u = 0; u < GX; u++) {
                        gk[u] = (int64_t)row[u][0];
                        gb[u] = hb_block_of(win, (int64_t)row[u][1]);
                        slot[u] = hb_slot_of(win, (int64_t)row[u][1], gb[u]);
                        row[u][1] = (uint64_t)gb[u];
                    }
                    probe_batch<NA, E, GX>(S, gk, gb, ge);
                }
                static_for<GX>([&](auto UU) {
                    constexpr int u = decltype(UU)::value;
                    if (!((live >> u) & 1u)) return;
                    int e = ge[u];
                    if (e < 0) e = hb_find_or_insert<NWP, E, OPS>(S, (int64_t)row[u][0], (int64_t)row[u][1], a.wd);
                    if (e < 0) return;  // state overflow (flagged)
                    const int sl = slot[u];
#pragma unroll
                    for (int w = 0; w < NWP; w++)
                        if (word_on<OPS>(a.wd, w)) lds_fold(word_op<OPS>(a.wd, w), &S.acc[sl * NWP + w][e], row[u][2 + w]);
                    atomicOr(&S.flag[e], F_ACC | (1u << (HB_MASK_SHIFT + sl)));
                });
            };
            gather_runs<NWP, GU, GF, 1>(a, sb, pend, fold_rows);
            uint32_t ovf = run_overflow(a, sb, pend);
            while (ovf) {
                const int pi = __ffs(ovf) - 1;
                ovf &= ovf - 1;
                gather_cells_push<NWP, GU, GF>(a, sb, pi, fold_rows);
            }
        } else if (gather) {
            for (int64_t pi = 0; pi < pend; pi++) {
                const int ncell = (int)cell_pad(a.slot_nch[pi]);
                const int G = gather_group(ncell);
                const int ngroups = ncell / G;
                for (int g = wv; g < ngroups; g += MG_BLOCK / 64) {
                    const int f = g * G + lane;
                    const uint32_t v = lane >= G ? 0u : g == wv ? v_first : cell_at(pi, f);
                    if (g == wv) {  // the next push's first cell word, in flight during this push
                        v_first = 0;
                        if (pi + 1 < pend) {
                            const int G1 = gather_group((int)cell_pad(a.slot_nch[pi + 1]));
                            if (lane < G1) v_first = cell_at(pi + 1, wv * G1 + lane);
                        }
                    }
                    const CellGroup cg = cell_group(v, f, CH);
                    const uint32_t tot = cg.tot;
                    for (uint32_t r0 = 0; r0 < tot; r0 += 64 * GU) {
                        uint64_t row[GU][PW];
                        const uint32_t live = load_group_rows<NWP, GU, GF>(a, pi, cg, r0, sb, row);
                        int ge[GU], slot[GU];
                        {
                            int64_t gk[GU], gb[GU];
#pragma unroll
                            for (int u = 0; u < GU; u++) {
                                gk[u] = (int64_t)row[u][0];
                                gb[u] = hb_block_of(win, (int64_t)row[u][1]);
                                slot[u] = hb_slot_of(win, (int64_t)row[u][1], gb[u]);
                                row[u][1] = (uint64_t)gb[u];
                            }
                            probe_batch<NA, E, GU>(S, gk, gb, ge);
                        }
                        static_for<GU>([&](auto UU) {
                            constexpr int u = decltype(UU)::value;
                            if (!((live >> u) & 1u)) return;
                            int e = ge[u];
                            if (e < 0) e = hb_find_or_insert<NWP, E, OPS>(S, (int64_t)row[u][0], (int64_t)row[u][1], a.wd);
                            if (e < 0) return;  // state overflow (flagged)
                            const int sl = slot[u];
#pragma unroll
                            for (int w = 0; w < NWP; w++)
                                if (word_on<OPS>(a.wd, w)) lds_fold(word_op<OPS>(a.wd, w), &S.acc[sl * NWP + w][e], row[u][2 + w]);
                            atomicOr(&S.flag[e], F_ACC | (1u << (HB_MASK_SHIFT + sl)));
                        });
                    }
                }
            }
        }
        __syncthreads();
        if (do_flush && a.runs) run_release(a, sb, pend);
        // ---- fire: every due window that holds data, each by exactly one block entry
        if (do_fire && !(FW_ABL(a) & AB_M_NO_FIRE)) {
            const int n = min(S.n, E);
            uint32_t nf = 0;
            for (int b0 = 0; b0 < n; b0 += MG_BLOCK) {
                const int e = fire_deal(b0, n, tid);
                if (e < n) nf += hb_fire_entry<NWP, E, OPS>(a, W, S, e, w_old, sb, &s_emit);
            }
            nf = wave_sum_u32(nf);
            if ((tid & 63) == 0 && nf) atomicAdd(&s_fired, nf);
        }
        // ---- write back: a slice is dropped once its last window has fired (clearWindow); an
        // entry without live slices is dropped.  Pass 1 expires the slices (the entry's flags in LDS)
        // and votes on the narrow layout; pass 2 writes the live entries in the layout chosen.
        if (tid == 0) {
            s_nlive = 0;
            s_newmin = INT64_MAX;
        }
        __syncthreads();  // (the fire reads neighbouring entries' flags, which pass 1 rewrites)
        const int n = min(S.n, E);
        uint64_t* so = a.state + (size_t)sb * a.cap_e * PWE;
        int64_t lnm = INT64_MAX;
        // the first window end that is not fired at w_new (UTC: the slice grid point above w_new + 1)
        const int64_t e_min = win.tz.n == 0 ? slice_end_of(win, wadd(w_new, 1)) : INT64_MIN;
        bool fits = a.hb_narrow >= 1, fits16 = a.hb_narrow >= 2;  // every live slot word fits int32 / int16
        for (int e = tid; e < n; e += MG_BLOCK) {
            const int64_t bs = S.slice[e];
            uint32_t mask = S.flag[e] >> HB_MASK_SHIFT;
            // the narrow header keeps the block index in 31 bits (bs >= offset)
            if (mask && udiv((uint64_t)wsub(bs, win.offset), win.hb_span_div) >= (1ull << 31)) fits = fits16 = false;
            int64_t first = INT64_MAX;
#pragma unroll
            for (int i = 0; i < HB_R; i++) {
                if (!((mask >> i) & 1u)) continue;
                const int64_t se = wadd(bs, (int64_t)(i + 1) * win.interval);
                if (win_fired(win, wadd(se, wsub(win.size, win.interval)), w_new)) {
                    mask &= ~(1u << i);  // its last window fired: expired (its words: identity, below)
                } else {
                    if (first == INT64_MAX) first = se;
#pragma unroll
                    for (int w = 0; w < NWP; w++) {
                        const int64_t v = (int64_t)S.acc[i * NWP + w][e];
                        fits &= v == (int64_t)(int32_t)v;
                        fits16 &= v == (int64_t)(int16_t)v;
                    }
                }
            }
            S.flag[e] = F_ACC | (mask << HB_MASK_SHIFT);
            if (mask) lnm = min(lnm, max(first, e_min));  // no window of this entry is due before it
        }
        const bool f32 = __syncthreads_and(fits) != 0;
        const int lv_out = __syncthreads_and(fits16) ? 2 : f32 ? 1 : 0;
        for (int e = tid; e < n; e += MG_BLOCK) {
            const uint32_t fl = S.flag[e];
            const uint32_t mask = fl >> HB_MASK_SHIFT;
            if (!mask) continue;
            const int pos = wave_claim(&s_nlive);
            if (FW_ABL(a) & AB_M_NO_WB) continue;
            if (lv_out == 2) {
                hb_store_narrow<NWP, E, 2>(win, so + (size_t)pos * PW2, S, e, fl);
            } else if (lv_out == 1) {
                hb_store_narrow<NWP, E, 1>(win, so + (size_t)pos * PW1, S, e, fl);
            } else {
                uint64_t p[PWE];
                p[0] = (uint64_t)S.key[e];
                p[1] = (uint64_t)S.slice[e];
                p[2] = (uint64_t)fl;
#pragma unroll
                for (int i = 0; i < NA; i++) {
                    const int w = i % NWP;
                    p[3 + i] = ((mask >> (i / NWP)) & 1u) ? S.acc[i][e]
                               : word_on<OPS>(a.wd, w) ? word_identity(word_op<OPS>(a.wd, w)) : 0;
                }
                store_words<PWE>(so + (size_t)pos * PWE, p);
            }
        }
        lnm = wave_min_i64(lnm);
        if ((tid & 63) == 0 && lnm != INT64_MAX) __hip_atomic_fetch_min(&s_newmin, lnm, __ATOMIC_RELAXED, LDS_SCOPE);
        __syncthreads();
        if (tid == 0) {
            a.state_count[sb] = s_nlive;
            a.sb_nar[sb] = (uint8_t)lv_out;
            a.sb_min_timer[sb] = s_newmin;
            a.sb_out[sb] = min(s_emit, a.slab_cap);
            if (s_fired) a.sb_fired[sb] += s_fired;
            if (S.overflow) __hip_atomic_fetch_or(&c->error, ERR_STATE, __ATOMIC_RELAXED, DEV_SCOPE);
            __hip_atomic_fetch_add(&c->state_moved, (uint64_t)(n0 + s_nlive), __ATOMIC_RELAXED, DEV_SCOPE);
            __hip_atomic_fetch_max(&c->peak_entries, (uint64_t)max(S.n, 0), __ATOMIC_RELAXED, DEV_SCOPE);
        }
        __syncthreads();
    }
    merge_ticket(a, W);
}

template <int NWP, int GF>
static void merge_hopb_launch(const MergeArgs& a, hipStream_t s) {
    constexpr int E = mg_entries(NWP, KIND_HOPB);
    // COUNT(*) alone / COUNT(*) + SUM(BIGINT) with the word ops as constants; the rest at run time
    constexpr uint32_t L = NWP == 1 ? ops_pack({W_SUM_I}) : ops_pack({W_SUM_I, W_SUM_I});
    if constexpr (GF == GF_COMPACT) {  // COUNT(*) alone with compact rows (the planner's only narrow layout)
        hipLaunchKernelGGL((k_merge_hopb<NWP, E, L, GF_COMPACT>), dim3(merge_grid(a.n_sb)), dim3(MG_BLOCK), 0, s, a);
    } else {
        if (GF == 0 && ops_layout(a.wd) == L)
            hipLaunchKernelGGL((k_merge_hopb<NWP, E, L, 0>), dim3(merge_grid(a.n_sb)), dim3(MG_BLOCK), 0, s, a);
        else
            hipLaunchKernelGGL((k_merge_hopb<NWP, E, OPS_ANY, GF>), dim3(merge_grid(a.n_sb)), dim3(MG_BLOCK), 0, s, a);
    }
}

}  // namespace fw
