// fw_ingest_impl.h -- k_ingest (K1+K2+K3) and its launchers, instantiated per loaded value
// column count in k_ingest_nv*.hip.
#pragma once
#include "fw_kernel_common.h"

namespace fw {
// ======================================================================================
// K1+K2+K3: single-pass ingest = slice/key-group assignment + LDS segmented reduce + a
// chunk-local counting sort of the partials by superbucket.
//
// One workgroup of ig_block(nw, nv) threads (512 for <= 2 accumulator words, two per CU; 1024 for
// wider accumulators, one per CU) owns a chunk of CH = block*RPT rows (4096 either way) and keeps
// all of them in registers (row j*block + tid, coalesced column loads, every load of the chunk in
// flight at once).  The chunk is folded sub-tile by sub-tile (SRPT rows per thread): rows with
// equal (key, slice) meet in one LDS slot table for the chunk whose owner is the lowest row index
// hashing to the slot (so a hot key, which occurs early, keeps its slot); the owner ends up holding
// the folded partial in its registers.  The surviving partials are then ranked per superbucket with LDS atomics, the
// per-superbucket counts are scanned, and every partial is stored at
//     parts[slot][c*CH + start(sb) + rank]
// so each (superbucket, chunk) cell is contiguous.  The cell table (cell_index: XCD-tiled
// [slot][chunk/16][sb][16], start | count << 16) tells the merge kernel where its rows are: no count pass, no global
// scan, one launch per push (+ a one-block stats reduce).
// Restates AbstractSliceSyncStateWindowAggProcessor.processElement (:96-126: slice assignment,
// late drop / late merge + timer), RecordsWindowBuffer.addElement (:81, grouping by
// (key, sliceEnd)) and the per-group fold of AggCombiner.combine (:76-99).
// ======================================================================================

// inclusive scan of one value per thread over an NT-thread block (wave shuffles + LDS)
template <int NT>
__device__ __forceinline__ uint32_t block_incl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int NWV = NT / 64;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    if (tid < 64) {
        uint32_t x = tid < NWV ? wsum[tid] : 0u;
#pragma unroll
        for (int d = 1; d < NWV; d <<= 1) {
            const uint32_t t = __shfl_up(x, d, 64);
            if (lane >= d) x += t;
        }
        if (tid < NWV) wsum[tid] = x;
    }
    __syncthreads();
    if (w > 0) v += wsum[w - 1];
    *total = wsum[NWV - 1];
    return v;
}

// X: the configuration has nullable columns or words that read arrival ordinals (gates, ordinals)
template <int NV, int NW, int RPT, bool X, int IG_BLOCK>
// (launch bounds: 4 waves per SIMD, 128 VGPRs)
__global__ __launch_bounds__(IG_BLOCK, 4) void k_ingest(IngestArgs a) {
    constexpr int CH = IG_BLOCK * RPT;
    // fold sub-tile: IG_SRPT rows per thread where the registers are tight (512 threads, 8 rows), the
    // whole chunk at once for the 1024-thread variants (3 barriers per chunk instead of 7)
    constexpr int SRPT = IG_BLOCK >= 1024 ? RPT : IG_SRPT;
    constexpr int NSUB = RPT / SRPT;
    constexpr int NVR = NV > 0 ? NV : 1;
    constexpr int PW = 2 + NW;
    constexpr int SL = ig_slots(NW);
    constexpr bool CAN_COMPACT = NW == 1;  // compact partial rows (PF_NARROW / PF_UNIT)
    static_assert(RPT % SRPT == 0, "fold sub-tiles must tile the chunk");
    // dynamic LDS only (16-B aligned base, G17): [header 16 words][hist: n_sb u16, padded to
    // 16 B][area: fold table, later the store stage]
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    int64_t* s_min = (int64_t*)&lds[0];
    unsigned long long* s_drop = (unsigned long long*)&lds[1];
    unsigned long long* s_rows = (unsigned long long*)&lds[2];
    uint32_t* s_folded = (uint32_t*)&lds[3] + 1;  // a row of the chunk was folded into another
    uint32_t* wsum = (uint32_t*)&lds[4];  // IG_BLOCK / 64 words
    int64_t* s_pk = (int64_t*)&lds[12];   // PF_PACK ranges of the chunk: key min / max, accumulator min / max
    const int PL = a.ks.pass_log2;
    const int n_sb = a.ks.n_sb >> PL;  // ingest superbuckets: the histogram and the cells
    const int n_units = a.ks.n_sb;     // state superbuckets (route_key's result)
    // partials per superbucket -> cell start: 16-bit (a chunk holds < 2^16 rows), so the histogram of
    // IG_MAX_SB superbuckets takes 32 KiB; counted with 32-bit LDS adds on the counter's half
    static_assert(IG_BLOCK * RPT < (1 << 16), "16-bit superbucket counters");
    uint16_t* hist = (uint16_t*)(lds + IG_HDR_WORDS);
    uint32_t* hist2 = (uint32_t*)hist;
    uint64_t* area = lds + IG_HDR_WORDS + ig_hist_words(n_sb);
    const int area_words = (a.lds_bytes >> 3) - IG_HDR_WORDS - ig_hist_words(n_sb);
    uint32_t* claim = (uint32_t*)area;                   // [SL]
    int64_t* ckey = (int64_t*)(area + (SL >> 1));       // [SL]
    int64_t* cslice = ckey + SL;                         // [SL]
    uint64_t* cacc = (uint64_t*)(cslice + SL);           // [NW][SL]

    const int tid = threadIdx.x;
    Ctrl* ctrl = a.ctrl;
    const int64_t c = blockIdx.x;
    kt_start(a.kt);
    // the push's slot in the partial buffer (the last workgroup of the launch advances
    // pending_pushes); checked after the column loads are issued, so they need not wait for it
    const int64_t slot = __hip_atomic_load(&ctrl->pending_pushes, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t cur_wm = __hip_atomic_load(&ctrl->cur, __ATOMIC_RELAXED, DEV_SCOPE);
    // adaptive fold: when the LDS fold of the previous push merged < 2 % of its rows (uniform keys
    // spread over many more groups than a chunk holds), skip it -- the merge kernel folds those
    // rows anyway; every 8th push folds again to notice a skewed stream
    const bool fold = !a.no_fold && (a.fold_always || !(__hip_atomic_load(&ctrl->fold_skip, __ATOMIC_RELAXED, DEV_SCOPE) &&
                                     (__hip_atomic_load(&ctrl->push_count, __ATOMIC_RELAXED, DEV_SCOPE) & 7u) != 0));
    if (tid == 0) {
        *s_min = INT64_MAX;
        *s_drop = 0;
        *s_rows = 0;
        *s_folded = 0;
        s_pk[0] = s_pk[2] = INT64_MAX;
        s_pk[1] = s_pk[3] = INT64_MIN;
    }
    for (int s = tid; s < (n_sb + 1) >> 1; s += IG_BLOCK) hist2[s] = 0;

    // ---- coalesced column loads of the whole chunk (all in flight before the first use)
    const int64_t base = c * CH;
    const int64_t st = a.stride;  // words per row of a column (1 unless packed rows)
    const int64_t ts0 = a.ts[base * st];  // chunk base for the 32-bit slice arithmetic
    int64_t rk[RPT], rs[RPT];
    uint64_t rv[RPT][NVR];
    int32_t pre[RPT];
    uint32_t rnul[RPT];  // bit q: value slot q is NULL in this row
    uint32_t valid = 0;
    // Loads are unconditional (a partial last chunk clamps its row index to the last row), so
    // every column load of the chunk is in flight at once; liveness is a bit mask computed beside
    // them.  Optional inputs (precomputed hashes, NULL flags, padded-segment counts) are switched
    // per launch, outside the per-row code.
    // Column pointers are rebased to the chunk (scalar) and rows addressed by a 32-bit offset, so
    // all columns of a row share one offset register (saddr + voffset loads).
    const uint32_t last = (uint32_t)min((int64_t)CH - 1, a.n - 1 - base);  // last row of the chunk
    const int64_t* kp = a.key + base * st;
    const int64_t* tp = a.ts + base * st;
    static_for<RPT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t o = (uint32_t)(j * IG_BLOCK + tid);
        const size_t oc = (size_t)min(o, last) * (size_t)st;
        rk[j] = kp[oc];
        rs[j] = tp[oc];
#pragma unroll
        for (int q = 0; q < NVR; q++) rv[j][q] = (q < NV && !(NV > 2 && q >= a.nv)) ? (a.vals[q] + base * st)[oc] : 0;
        pre[j] = 0;
        rnul[j] = 0;
        valid |= (uint32_t)(o <= last) << j;
    });
    if (a.khash)
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            pre[j] = (a.khash + base)[min((uint32_t)(j * IG_BLOCK + tid), last)];
        });
    if (X)
#pragma unroll
        for (int q = 0; q < NV; q++) {
            if (NV > 2 && q >= a.nv) break;
            if (!a.nulls[q]) continue;
            static_for<RPT>([&](auto J) {
                constexpr int j = decltype(J)::value;
                rnul[j] |= ((a.nulls[q] + base)[min((uint32_t)(j * IG_BLOCK + tid), last)] ? 1u : 0u) << q;
            });
        }
    if (a.seg_counts)  // padded all-to-all buffer: each segment's padding rows are not live
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const uint64_t g = (uint64_t)(base + (int64_t)j * IG_BLOCK + tid + a.row0);
            const uint64_t sg = udiv(g, a.seg_div);
            const int64_t cnt = a.seg_counts[sg];
            valid &= ~((uint32_t)((int64_t)(g - sg * a.seg_div.d) >= cnt) << j);
        });
    if (slot >= FW_MAX_PENDING) {  // (uniform) the partial buffer is full: the host sizes pushes so it never is
        if (tid == 0) __hip_atomic_fetch_or(&ctrl->error, ERR_CHUNKS, __ATOMIC_RELAXED, DEV_SCOPE);
        return;
    }
    // arrival ordinal base of this chunk within the flush (W_Q* words; >= 1, see record_word)
    const uint32_t ord0 = (uint32_t)(slot * a.cap_rows + base) + 1u;
    // TIMESTAMP_LTZ: slices live on the shift zone's wall clock (AbstractSliceAssigner
    // .assignSliceEnd -> toUtcTimestampMills, SliceAssigners.java:655-670)
    int64_t tsl0 = ts0;
    if (a.win.tz.n && !a.global) {
        tsl0 = tz_to_utc_ts(a.win.tz, ts0);
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            if (valid & (1u << j)) rs[j] = tz_to_utc_ts(a.win.tz, rs[j]);
        });
    }
    // slice-aligned base 2^30 ms below the chunk's first row: rows within 2^31 ms of it take
    // the 32-bit path (one mul_hi instead of a 64-bit magic division)
    const bool fast = a.win.fast32 && tsl0 > -(1ll << 61) && tsl0 < (1ll << 61);
    const int64_t tbase = fast ? window_start(tsl0, a.win.offset, a.win.slice_div) -
                                     (int64_t)((1u << 30) / (uint32_t)a.win.interval) * a.win.interval
                               : 0;
    // ---- K1/K2: key group -> superbucket, slice end, late classification, record words
    int32_t rsb[RPT];
    uint32_t rm[RPT];
    uint64_t racc[RPT][NW];
    int64_t lmin = INT64_MAX;
    uint32_t ldrop = 0, lrows = 0;
    // Common path, branch free: a UTC SQL slice assignment of a row within 2^31 ms of the chunk
    // base whose window is not fired and whose key group this subtask owns.  Every other row
    // (DataStream, LTZ, GLOBAL phase, late, far-off timestamps, foreign key groups) is marked
    // `slow` and takes the general path below, entered only by waves that have such a row: the
    // per-row divergent branches of the general path cost as many scalar instructions as the
    // vector work itself.
    // (simple_l: the launch's part of it -- the push formats below depend on the launch only, so every
    // chunk agrees on them; a chunk too far off for the 32-bit path sends every row down the general
    // path, which keeps the slice end in the row: PF_WIDE)
    const bool simple_l = a.win.fast32 && !a.win.ds && !a.global && a.win.tz.n == 0;
    const bool simple = fast && simple_l;
    // compact partial rows (PF_NARROW / PF_UNIT) count slices from the push's rank base: the first
    // slice end that is not fired at the current watermark (every row that is not late ends at or
    // after it); the merge kernel reads it from slot_base
    // (planned for COUNT(*)-only layouts, fw_api.hip: the variants with wider accumulators carry
    // none of this code, which would cost them registers)
    const bool nar = CAN_COMPACT && a.narrow && simple_l && cur_wm != INT64_MIN;
    uint32_t slow = simple ? 0u : valid;
    // record words: the word op is uniform, so it is resolved once per launch into a mode and
    // the rows only select (no per-row switch over the op)
    int32_t wmode[NW];  // 0: the value, 1: a count of 1, 2: dkey(value), 3: general (X only)
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const int32_t op = w < a.wd.nw ? a.wd.op[w] : W_SUM_I;
        wmode[w] = X ? 3 : op == W_CNT ? 1 : (op == W_MIN_D || op == W_MAX_D) ? 2 : 0;
    }
    static_for<RPT>([&](auto J) {
        constexpr int j = decltype(J)::value;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            if (w >= a.wd.nw) {
                racc[j][w] = 0;
                continue;
            }
            const uint64_t v = pick_col(rv[j], a.wd.col[w]);
            if (X) {
                const uint64_t gord = ((uint64_t)(uint32_t)a.push_seq << 32) |
                                      (uint64_t)(base + (int64_t)j * IG_BLOCK + tid + a.row0);
                racc[j][w] = gated_word(a.wd, w, v, rnul[j], ord0 + (uint32_t)(j * IG_BLOCK + tid), gord);
            } else {
                const uint64_t dk = (uint64_t)dkey(v);
                racc[j][w] = wmode[w] == 1 ? 1ull : wmode[w] == 2 ? dk : v;
            }
        }
    });
    // key routing with the key-hash kind resolved per launch
    auto route_rows = [&](auto HK) {
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            rsb[j] = route_key(a.ks, rk[j], pre[j], &rm[j], decltype(HK)::value);
        });
    };
    switch (a.ks.hash_kind) {
        case KH_LONG: route_rows(std::integral_constant<int, KH_LONG>{}); break;
        case KH_INT: route_rows(std::integral_constant<int, KH_INT>{}); break;
        case KH_BINROW_BIGINT: route_rows(std::integral_constant<int, KH_BINROW_BIGINT>{}); break;
        case KH_BINROW_INT: route_rows(std::integral_constant<int, KH_BINROW_INT>{}); break;
        default: route_rows(std::integral_constant<int, KH_PRE>{}); break;
    }
    if (simple) static_for<RPT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const int32_t sb = rsb[j];
        const uint64_t d = (uint64_t)rs[j] - (uint64_t)tbase;
        const uint32_t d32 = (uint32_t)d;
        const uint32_t r = d32 - udiv32(d32, a.win.slice_div32) * (uint32_t)a.win.interval;
        const int64_t se = rs[j] - (int64_t)r + a.win.interval;
        const bool live = (valid >> j) & 1u;
        const bool ok = live && d < (1ull << 31) && (uint32_t)sb < (uint32_t)n_units && (a.local || cur_wm < se - 1);
        slow |= (uint32_t)(live && !ok) << j;
        rs[j] = ok ? se : rs[j];
        lmin = ok ? min(lmin, se) : lmin;
        lrows += ok ? 1u : 0u;
    });
    if (__ballot(slow != 0)) static_for<RPT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if (!((slow >> j) & 1u)) return;
        if ((uint32_t)rsb[j] >= (uint32_t)n_units) {  // key group not owned by this subtask
            __hip_atomic_fetch_or(&ctrl->error, ERR_KEYGROUP, __ATOMIC_RELAXED, DEV_SCOPE);
            valid &= ~(1u << j);
            return;
        }
        int64_t se;
        const uint64_t d = (uint64_t)rs[j] - (uint64_t)tbase;
        if (a.global) {
            se = rs[j];  // SlicedSharedSliceAssigner.assignSliceEnd: the row's slice-end field
        } else if (fast && d < (1ull << 31)) {
            const uint32_t d32 = (uint32_t)d;
            const uint32_t r = d32 - udiv32(d32, a.win.slice_div32) * (uint32_t)a.win.interval;
            se = rs[j] - (int64_t)r + a.win.interval;
        } else {
            se = slice_end_of(a.win, rs[j]);
        }
        int64_t target = se;
        if (a.win.ds) {
            // DataStream WindowOperator.processElement (:405-446): the pane's windows, newest
            // first, end at e0, e0 - slide, ...; a window is late once its cleanup time has passed
            // (isWindowLate :609-612), fired once its maxTimestamp has (EventTimeTrigger)
            const int64_t e0 = ds_first_window_end(a.win, se);
            if (ds_cleanup_time(a.win, e0) <= cur_wm) {  // late for every window: skipped
                valid &= ~(1u << j);
                if (wadd(rs[j], a.win.lateness) <= cur_wm) {  // isElementLate (:640-644)
                    if (!a.side_output) {
                        ldrop++;
                    } else {  // sideOutput(element)
                        const int64_t r = __hip_atomic_fetch_add(&ctrl->n_side, (int64_t)1, __ATOMIC_RELAXED, DEV_SCOPE);
                        if (r < a.side_cap) {
                            int64_t* p = a.side + (size_t)r * SOW;
                            const int64_t i = base + (int64_t)j * IG_BLOCK + tid;
                            p[0] = rk[j];
                            p[1] = rs[j];
                            p[2] = ((int64_t)a.push_seq << 32) | (int64_t)(i + a.row0);
#pragma unroll
                            for (int q = 0; q < NV; q++)  // reloaded: rv is dead after the record words
                                p[3 + q] = (NV > 2 && q >= a.nv) ? 0 : (int64_t)a.vals[q][i * st];
                        } else {
                            __hip_atomic_fetch_or(&ctrl->error, ERR_LATE, __ATOMIC_RELAXED, DEV_SCOPE);
                        }
                    }
                }
                return;
            }
            // the newest fired window; if it is not cleaned yet the element fires it again at
            // once (EventTimeTrigger.onElement returns FIRE): a late-fire row, handled in order of
            // arrival by the merge kernel
            bool late_fire = false;
            if (cur_wm >= wsub(e0, 1)) {
                late_fire = true;  // e0 fired, and not cleaned (checked above)
            } else if (a.win.n_win > 1) {
                const uint64_t d = (uint64_t)wsub(wsub(e0, 1), cur_wm);
                uint64_t kf = udiv(d, a.win.slide_div);
                kf += (kf * (uint64_t)a.win.slide != d);
                if (kf < (uint64_t)a.win.n_win && ds_window_holds_pane(a.win, wsub(e0, (int64_t)kf * a.win.slide), se))
                    late_fire = ds_cleanup_time(a.win, wsub(e0, (int64_t)kf * a.win.slide)) > cur_wm;
            }
            if (late_fire) {
                valid &= ~(1u << j);
                const int64_t r = __hip_atomic_fetch_add(&ctrl->n_lfire, (int64_t)1, __ATOMIC_RELAXED, DEV_SCOPE);
                if (r < a.lfire_cap) {
                    uint64_t* p = a.lfire + (size_t)r * LFW;
                    p[0] = (uint64_t)rk[j];
                    p[1] = (uint64_t)se;
                    p[2] = (uint64_t)(uint32_t)rsb[j] | ((uint64_t)(ord0 + (uint32_t)(j * IG_BLOCK + tid)) << 32);
#pragma unroll
                    for (int w = 0; w < NW; w++) p[3 + w] = racc[j][w];
                } else {
                    __hip_atomic_fetch_or(&ctrl->error, ERR_LATE, __ATOMIC_RELAXED, DEV_SCOPE);
                }
                return;
            }
        } else if (!a.local && win_fired(a.win, se, cur_wm)) {
            if (win_fired(a.win, last_window_end_of(a.win, se), cur_wm)) {  // late for every window: drop
                valid &= ~(1u << j);
                ldrop++;
                return;
            }
            target = merge_target_of(a.win, se);
            // timer for the first unfired window (processElement :111-117)
            int64_t unfired;
            if (a.win.tz.n == 0) {
                const int64_t steps = (int64_t)((uint64_t)wsub(wadd(cur_wm, 1), se) / (uint64_t)a.win.interval) + 1;
                unfired = wadd(se, steps * a.win.interval);
            } else {  // window ends are not equally spaced in epoch time across a DST change
                unfired = se;
                while (win_fired(a.win, unfired, cur_wm)) unfired = wadd(unfired, a.win.interval);
            }
            const int64_t r = __hip_atomic_fetch_add(&ctrl->n_treq, (int64_t)1, __ATOMIC_RELAXED, DEV_SCOPE);
            if (r < a.treq_cap) {
                a.treq[3 * r] = rk[j];
                a.treq[3 * r + 1] = unfired;
                a.treq[3 * r + 2] = rsb[j];
            } else {
                __hip_atomic_fetch_or(&ctrl->error, ERR_TREQ, __ATOMIC_RELAXED, DEV_SCOPE);
            }
        }
        rs[j] = target;
        lmin = min(lmin, target);
        lrows++;
    });
    // a row left valid by the general path keeps its slice end in its partial row (PF_WIDE chunk)
    const bool wide_row = (slow & valid) != 0;
    const uint32_t valid_unfolded = valid;
    const bool do_fold = fold && !(FW_ABL(a) & AB_NO_FOLD);
    if (!do_fold) __syncthreads();  // the header and histogram are initialised (the fold's first barrier does it)
    // ---- K3: fold equal (key, slice) rows over the whole chunk, SRPT rows per thread at a time.
    // The slot table lives for the chunk: a slot's owner is the lowest row index hashing to it (the
    // first occurrence -- a hot key keeps its slot), so a later sub-tile's rows fold into owners of
    // earlier sub-tiles too; owners take their folded partials back once, after the last sub-tile.
    if (do_fold) {
        for (int h = tid; h < SL; h += IG_BLOCK) claim[h] = 0xFFFFFFFFu;
        static_for<NSUB>([&](auto S) {
            constexpr int s = decltype(S)::value;
            uint32_t rh[SRPT];
            __syncthreads();  // the table is reset / the previous sub-tile's folds are done
            static_for<SRPT>([&](auto Q) {
                constexpr int q = decltype(Q)::value;
                constexpr int j = s * SRPT + q;
                rh[q] = fold_slot(rm[j], rs[j], SL);
                if (valid & (1u << j)) atomicMin(&claim[rh[q]], (uint32_t)(j * IG_BLOCK + tid));
            });
            __syncthreads();
            static_for<SRPT>([&](auto Q) {  // this sub-tile's new owners publish their (key, slice) and partial
                constexpr int q = decltype(Q)::value;
                constexpr int j = s * SRPT + q;
                if (!(valid & (1u << j)) || claim[rh[q]] != (uint32_t)(j * IG_BLOCK + tid)) return;
                ckey[rh[q]] = rk[j];
                cslice[rh[q]] = rs[j];
#pragma unroll
                for (int w = 0; w < NW; w++) cacc[w * SL + rh[q]] = racc[j][w];
            });
            __syncthreads();
            static_for<SRPT>([&](auto Q) {  // everyone else folds into a matching owner
                constexpr int q = decltype(Q)::value;
                constexpr int j = s * SRPT + q;
                const uint32_t h = rh[q];
                if (!(valid & (1u << j)) || claim[h] == (uint32_t)(j * IG_BLOCK + tid)) return;
                if (ckey[h] == rk[j] && cslice[h] == rs[j]) {
#pragma unroll
                    for (int w = 0; w < NW; w++)
                        if (w < a.wd.nw) lds_fold(a.wd.op[w], &cacc[w * SL + h], racc[j][w]);
                    valid &= ~(1u << j);
                }
            });
        });
        __syncthreads();
        static_for<RPT>([&](auto J) {  // owners take the folded partial back (slot recomputed: no registers held)
            constexpr int j = decltype(J)::value;
            const uint32_t h = fold_slot(rm[j], rs[j], SL);
            if (!(valid & (1u << j)) || claim[h] != (uint32_t)(j * IG_BLOCK + tid)) return;
#pragma unroll
            for (int w = 0; w < NW; w++) racc[j][w] = cacc[w * SL + h];
        });
    }
    // PF_UNIT needs a chunk in which no row folded into another: one LDS flag store per wave that folded
    if (a.narrow == 2 && do_fold && __ballot(valid != valid_unfolded) && (tid & 63) == 0) *s_folded = 1u;
    // ---- PF_PACK (runs, one integer word, no NULLs / ordinals): every push measures the key and
    // accumulator ranges of its partials for the next flush epoch; the epoch's first push (slot 0)
    // takes the parameters the previous push measured, the others the epoch's
    const bool pk_stats = CAN_COMPACT && !X && a.pack != 0;
    int64_t pk_k = 0, pk_v = 0;
    uint32_t pk_bits = 0;
    if (pk_stats) {
        pk_k = __hip_atomic_load(slot == 0 ? &ctrl->pk_next_k : &ctrl->pk_cur_k, __ATOMIC_RELAXED, DEV_SCOPE);
        pk_v = __hip_atomic_load(slot == 0 ? &ctrl->pk_next_v : &ctrl->pk_cur_v, __ATOMIC_RELAXED, DEV_SCOPE);
        pk_bits = __hip_atomic_load(slot == 0 ? &ctrl->pk_next_bits : &ctrl->pk_cur_bits, __ATOMIC_RELAXED, DEV_SCOPE);
        int64_t kmn = INT64_MAX, kmx = INT64_MIN, vmn = INT64_MAX, vmx = INT64_MIN;
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const bool v = (valid >> j) & 1u;
            kmn = v ? min(kmn, rk[j]) : kmn;
            kmx = v ? max(kmx, rk[j]) : kmx;
            vmn = v ? min(vmn, (int64_t)racc[j][0]) : vmn;
            vmx = v ? max(vmx, (int64_t)racc[j][0]) : vmx;
        });
        kmn = wred_min_i64(kmn);
        kmx = wred_max_i64(kmx);
        vmn = wred_min_i64(vmn);
        vmx = wred_max_i64(vmx);
        if ((tid & 63) == 0 && kmn <= kmx) {
            __hip_atomic_fetch_min(&s_pk[0], kmn, __ATOMIC_RELAXED, LDS_SCOPE);
            __hip_atomic_fetch_max(&s_pk[1], kmx, __ATOMIC_RELAXED, LDS_SCOPE);
            __hip_atomic_fetch_min(&s_pk[2], vmn, __ATOMIC_RELAXED, LDS_SCOPE);
            __hip_atomic_fetch_max(&s_pk[3], vmx, __ATOMIC_RELAXED, LDS_SCOPE);
        }
    }
    // ---- rank the partials per superbucket, scan, publish the cells
    uint32_t rdst[RPT];
    const bool sort = !(FW_ABL(a) & AB_NO_SORT);
    static_for<RPT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t i = (uint32_t)(rsb[j] >> PL), sh = (i & 1u) << 4;
        rdst[j] = (sort && (valid & (1u << j))) ? (atomicAdd(&hist2[i >> 1], 1u << sh) >> sh) & 0xFFFFu
                                                : (uint32_t)(j * IG_BLOCK + tid);
    });
    __syncthreads();
    // ---- the chunk's partial-row format (PF_*): compact unless a row kept its own slice end or
    // the chunk's slice ends spread over more than rank_lim slices
    bool wide = wide_row || !nar;
    const bool runs = a.runs != nullptr && sort;
    // PF_PACK push: runs, the epoch's parameters valid, every row on the common path's slice grid
    const bool pk = pk_stats && runs && (pk_bits & PK_OK) && simple_l && cur_wm != INT64_MIN;
    const uint32_t pk_kb = pk_bits & 255u, pk_rb = (pk_bits >> 8) & 255u, pk_vb = (pk_bits >> 16) & 255u;
    // (re-read here rather than kept live through the fold: the watermark does not change during a push);
    // a PF_PACK push counts ranks from the epoch's rank base (slot 0's, every later row's slice end is >= it)
    const int64_t nbase = (pk && slot > 0) ? a.slot_base[0]
                          : (nar || pk) ? slice_end_of(a.win, wadd(__hip_atomic_load(&ctrl->cur, __ATOMIC_RELAXED, DEV_SCOPE), 1))
                                        : 0;
    if (pk) {  // uniform: does every row of the chunk fit the epoch's bit fields?
        const uint64_t rlim = min((uint64_t)a.rank_lim, (uint64_t)a.win.interval << pk_rb);
        bool fit = !wide_row;
        if (fit)
            static_for<RPT>([&](auto J) {
                constexpr int j = decltype(J)::value;
                if ((valid & (1u << j)) && ((uint64_t)(rs[j] - nbase) >= rlim || ((uint64_t)(rk[j] - pk_k) >> pk_kb) != 0 ||
                                            ((uint64_t)((int64_t)racc[j][0] - pk_v) >> pk_vb) != 0))
                    fit = false;
            });
        wide = !__syncthreads_and(fit);
    } else if (nar) {  // uniform: the block-wide vote only when compact rows are possible
        if (!wide)
            static_for<RPT>([&](auto J) {
                constexpr int j = decltype(J)::value;
                if ((valid & (1u << j)) && (uint64_t)(rs[j] - nbase) >= (uint64_t)a.rank_lim) wide = true;
            });
        wide = __syncthreads_or(wide);
    }
    uint32_t* cells = a.cells + (size_t)slot * n_sb * a.max_nch;
    // runs (IngestArgs::runs): a push's run rows share one format -- PF_PACK, else compact when the
    // push is (COUNT(*) alone: PF_UNIT when no chunk folds, else PF_NARROW); a chunk that must write
    // PF_WIDE rows in a compact push keeps them all in its own region
    const uint32_t push_fmt = pk ? PF_PACK
                              : (runs && CAN_COMPACT && nar) ? ((!X && a.narrow == 2 && !do_fold) ? PF_UNIT : PF_NARROW)
                                                             : PF_WIDE;
    // COUNT(*) alone and nothing folded in this chunk: every row counts 1
    const uint32_t fmt = runs ? (wide ? PF_WIDE : push_fmt)
                         : (!CAN_COMPACT || wide || !sort) ? PF_WIDE
                         : (!X && a.narrow == 2 && !*s_folded) ? PF_UNIT
                                                                 : PF_NARROW;
    const bool to_runs = runs && fmt == push_fmt;
    // (runs) claim this chunk's stretch of every superbucket's sub-run now -- the counts are final --
    // so the claims' round trip overlaps the scan and the staging of the first store window.
    // Superbuckets strided over the threads (the host enables runs for n_sb <= RUN_KMAX * IG_BLOCK):
    // a wave's claims hit 64 neighbouring counters.  (These reads of hist precede the scan's barriers,
    // after which it is overwritten.)
    const uint32_t xr = (uint32_t)c & (RUN_X - 1);
    uint32_t pos[RUN_KMAX], cnt[RUN_KMAX];
#pragma unroll
    for (int k = 0; k < RUN_KMAX; k++) {
        const int i = tid + k * IG_BLOCK;
        cnt[k] = (runs && i < n_sb) ? hist[i] : 0u;
        pos[k] = (to_runs && cnt[k]) ? atomicAdd(a.run_fill + ((size_t)slot * RUN_X + xr) * n_sb + i, cnt[k]) : 0u;
    }
    const int per = (n_sb + IG_BLOCK - 1) / IG_BLOCK;
    const int sb0 = min(tid * per, n_sb), sb1 = min(sb0 + per, n_sb);
    uint32_t seg = 0;
    for (int i = sb0; i < sb1; i++) seg += hist[i];
    uint32_t total;
    const uint32_t incl = block_incl_scan<IG_BLOCK>(seg, wsum, &total);
    uint32_t run = incl - seg;
    if (sort)
        for (int i = sb0; i < sb1; i++) {
            const uint32_t v = hist[i];
            hist[i] = run;
            if (!runs) cells[cell_index(c, n_sb, i)] = run | (v << 16) | (fmt << 30);
            run += v;
        }
    if (fmt != PF_WIDE)  // compact rows keep their rank instead of their slice end
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            rs[j] = (int64_t)udiv32((uint32_t)(rs[j] - nbase), a.win.slice_div32);
        });
    __syncthreads();
    if (sort)
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            if (valid & (1u << j)) rdst[j] += hist[rsb[j] >> PL];
        });
    else
        total = CH;
    // ---- store the partials through an LDS stage so every global store is a full line (runs:
    // word by word to each row's destination, neighbouring lanes on neighbouring words of a
    // superbucket's stretch).  The chunk's region keeps its PF_WIDE size; a compact format fills its
    // front, and its rank bytes are staged behind the rows and stored to the side array.
    // (runs) per superbucket: chunk positions below rbound go to the run at position + roff, every
    // row's destination in sdst (RUN_LOCAL | position for the rows that stay in the chunk's region).
    // They live where the fold table was; the store stage follows them.
    const int n_sb_pad = (n_sb + 3) & ~3;
    uint32_t* rbound = (uint32_t*)area;
    uint32_t* roff = rbound + n_sb_pad;
    uint32_t* sdst = roff + n_sb_pad;
    const int PWX = pf_stride(fmt, NW);
    const int aoff = fmt == PF_WIDE ? 2 : 1;  // first accumulator word of a row
    uint64_t* out = a.parts + ((size_t)slot * a.cap_rows + (size_t)base) * PW;
    uint64_t* stage = runs ? area + (((size_t)2 * n_sb_pad + CH + 3) / 4) * 2 : area;  // 16-B aligned
    const int64_t stage_words = area_words - (int64_t)(stage - area);
    const uint32_t wrows = fmt == PF_WIDE ? (uint32_t)(stage_words / PW) & ~15u
                                          : (uint32_t)(stage_words * 8 / (8 * PWX + 1)) & ~15u;
    uint8_t* rstage = (uint8_t*)(stage + (size_t)wrows * PWX);
    uint64_t* rslot = runs ? a.runs + (size_t)slot * a.run_rows * PW : nullptr;
    auto stage_rows = [&](uint32_t w0) {
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const uint32_t d = rdst[j] - w0;
            if (!(valid & (1u << j)) || d >= wrows) return;
            uint64_t* p = stage + (size_t)d * PWX;
            if (CAN_COMPACT && fmt == PF_PACK) {  // rs is the rank here
                p[0] = ((uint64_t)(rk[j] - pk_k) << (64 - pk_kb)) | ((uint64_t)rs[j] << pk_vb) |
                       (uint64_t)((int64_t)racc[j][0] - pk_v);
                return;
            }
            p[0] = (uint64_t)rk[j];
            if (fmt == PF_WIDE) p[1] = (uint64_t)rs[j];
            else rstage[d] = (uint8_t)rs[j];  // the rank (set below the format decision)
            if (fmt != PF_UNIT)
#pragma unroll
                for (int w = 0; w < NW; w++) p[aoff + w] = racc[j][w];
        });
    };
    const bool store = !(FW_ABL(a) & AB_NO_STORE);
    if (runs) {
        if (store) stage_rows(0);  // the first window, while the claims are in flight
        const uint32_t scap = (uint32_t)a.sub_cap;
#pragma unroll
        for (int k = 0; k < RUN_KMAX; k++) {
            const int i = tid + k * IG_BLOCK;
            if (i >= n_sb) break;
            const uint32_t st0 = hist[i], v = cnt[k];
            const uint32_t n_in = to_runs ? (pos[k] >= scap ? 0u : min(v, scap - pos[k])) : 0u;
            rbound[i] = st0 + n_in;
            roff[i] = (uint32_t)(((size_t)i * RUN_X + xr) * scap + pos[k]) - st0;
            cells[cell_index(c, n_sb, i)] = (st0 + n_in) | ((v - n_in) << 16) | (fmt << 30);
            if (n_in < v) a.run_ovf[(size_t)slot * n_sb + i] = 1u;
        }
        __syncthreads();
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            if (!(valid & (1u << j))) return;
            const uint32_t d = rdst[j];
            const int i = rsb[j] >> PL;
            sdst[d] = d < rbound[i] ? d + roff[i] : (RUN_LOCAL | d);
        });
    }
    if (store)
        for (uint32_t w0 = 0; w0 < total; w0 += wrows) {
            __syncthreads();  // fold table / previous window no longer read
            if (!(runs && w0 == 0)) stage_rows(w0);
            __syncthreads();
            const uint32_t nr = min(wrows, total - w0);
            const uint32_t nwords = nr * PWX;
            if (runs) {
                // row by row (the stride as a constant): one destination lookup per row, 16-B stores
                // where the row's words pair up on 16-B boundaries (neighbouring lanes hold neighbouring
                // rows of a superbucket's stretch)
                auto copy_out = [&](auto PC) {
                    constexpr uint32_t P = decltype(PC)::value;
                    for (uint32_t r = tid; r < nr; r += IG_BLOCK) {
                        const uint32_t dd = (FW_ABL(a) & AB_IG_LINEAR) ? (RUN_LOCAL | (w0 + r)) : sdst[w0 + r];
                        const uint64_t* src = stage + (size_t)r * P;
                        uint64_t* dst = (dd & RUN_LOCAL) ? out + (size_t)(dd & ~RUN_LOCAL) * P : rslot + (size_t)dd * P;
                        if (FW_ABL(a) & AB_IG_NO_GSTORE) {
                            asm volatile("" ::"v"(src[0]), "v"(dst));
                            continue;
                        }
                        if constexpr (P % 2 == 0) {
#pragma unroll
                            for (uint32_t k = 0; k < P / 2; k++) {
                                const ulonglong2 x = *(const ulonglong2*)(src + 2 * k);
                                st16(dst + 2 * k, x.x, x.y);
                            }
                        } else {
                            uint64_t v[P];
#pragma unroll
                            for (uint32_t k = 0; k < P; k++) v[k] = src[k];
                            if constexpr (P == 1) {
                                st8(dst, v[0]);
                            } else {  // the lone 8-B word first or last, so the pairs are 16-B aligned
                                const bool odd = ((uintptr_t)dst & 8) != 0;
                                st8(odd ? dst : dst + (P - 1), odd ? v[0] : v[P - 1]);
                                uint64_t* q = dst + (odd ? 1 : 0);
#pragma unroll
                                for (uint32_t k = 0; k < (P - 1) / 2; k++)
                                    st16(q + 2 * k, odd ? v[2 * k + 1] : v[2 * k], odd ? v[2 * k + 2] : v[2 * k + 1]);
                            }
                        }
                    }
                };
                if (fmt == PF_WIDE) copy_out(std::integral_constant<uint32_t, (uint32_t)PW>{});
                else if (fmt == PF_NARROW) copy_out(std::integral_constant<uint32_t, (uint32_t)(1 + NW)>{});
                else copy_out(std::integral_constant<uint32_t, 1u>{});
                if (pf_rank_bytes(fmt))
                    for (uint32_t r = tid; r < nr; r += IG_BLOCK) {
                        const uint32_t dd = sdst[w0 + r];
                        uint8_t* rd = (dd & RUN_LOCAL) ? a.ranks + (size_t)slot * a.cap_rows + (size_t)base + (dd & ~RUN_LOCAL)
                                                       : a.run_ranks + (size_t)slot * a.run_rows + dd;
                        *rd = rstage[r];
                    }
                continue;
            }
            uint64_t* dst = out + (size_t)w0 * PWX;  // 16-B aligned: slot, chunk and window bases are 16-row multiples
            for (uint32_t q = 2 * tid; q < nwords; q += 2 * IG_BLOCK) {
                if (q + 1 < nwords) {
                    const ulonglong2 x = *(const ulonglong2*)(stage + q);
                    st16(dst + q, x.x, x.y);
                } else {
                    st8(dst + q, stage[q]);
                }
            }
            if (pf_rank_bytes(fmt)) {
                uint8_t* rd = a.ranks + (size_t)slot * a.cap_rows + (size_t)base + w0;  // 16-B aligned
                for (uint32_t q = 16 * tid; q < nr; q += 16 * IG_BLOCK) {
                    if (q + 16 <= nr) {
                        *(uint4*)(rd + q) = *(const uint4*)(rstage + q);
                    } else {
                        for (uint32_t b = q; b < nr; b++) rd[b] = rstage[b];
                    }
                }
            }
        }
    // ---- control counters.  Each chunk publishes its stats with agent-scope stores (they bypass
    // the XCD's L2, so any XCD reads them), then takes a ticket; the last workgroup of the launch
    // reduces every chunk's stats into the control block and commits the push's slot
    // (RecordsWindowBuffer's minSliceEnd and the late-drop counter).  No extra launch.
    // wave reductions first: one LDS atomic per wave, not 3 x 512 on the same three words (they
    // serialise: ~10 us of a CFG2 launch)
    {
        const int64_t wm = wred_min_i64(lmin);
        const uint32_t wd = wred_sum_u32(ldrop), wr = wred_sum_u32(lrows);
        if ((tid & 63) == 0) {
            if (wm != INT64_MAX) __hip_atomic_fetch_min(s_min, wm, __ATOMIC_RELAXED, LDS_SCOPE);
            if (wd) atomicAdd(s_drop, (unsigned long long)wd);
            if (wr) atomicAdd(s_rows, (unsigned long long)wr);
        }
    }
    __syncthreads();
    int32_t* s_last = (int32_t*)&lds[3];
    if (tid == 0) {
        __hip_atomic_store(&a.chunk_stats[CS_WORDS * c], *s_min, __ATOMIC_RELAXED, DEV_SCOPE);
        __hip_atomic_store(&a.chunk_stats[CS_WORDS * c + 1], (int64_t)*s_drop, __ATOMIC_RELAXED, DEV_SCOPE);
        __hip_atomic_store(&a.chunk_stats[CS_WORDS * c + 2], (int64_t)*s_rows, __ATOMIC_RELAXED, DEV_SCOPE);
        __hip_atomic_store(&a.chunk_stats[CS_WORDS * c + 3], (int64_t)total, __ATOMIC_RELAXED, DEV_SCOPE);
        // bytes of partial rows (+ rank bytes) this chunk wrote, and whether they are compact
        __hip_atomic_store(&a.chunk_stats[CS_WORDS * c + 4],
                           (int64_t)total * (8 * PWX + (pf_rank_bytes(fmt) ? 1 : 0)) | ((int64_t)(fmt != PF_WIDE) << 40),
                           __ATOMIC_RELAXED, DEV_SCOPE);
        if (pk_stats)
#pragma unroll
            for (int q = 0; q < 4; q++) __hip_atomic_store(&a.chunk_stats[CS_WORDS * c + 8 + q], s_pk[q], __ATOMIC_RELAXED, DEV_SCOPE);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *s_last = grid_last_wg(a.tickets->c[0]);
    }
    __syncthreads();
    if (!*s_last) return;
    int64_t m = INT64_MAX, d = 0, r = 0, q = 0, y = 0;
    for (int64_t i = tid; i < (int64_t)gridDim.x; i += IG_BLOCK) {
        m = min(m, __hip_atomic_load(&a.chunk_stats[CS_WORDS * i], __ATOMIC_RELAXED, DEV_SCOPE));
        d += __hip_atomic_load(&a.chunk_stats[CS_WORDS * i + 1], __ATOMIC_RELAXED, DEV_SCOPE);
        r += __hip_atomic_load(&a.chunk_stats[CS_WORDS * i + 2], __ATOMIC_RELAXED, DEV_SCOPE);
        q += __hip_atomic_load(&a.chunk_stats[CS_WORDS * i + 3], __ATOMIC_RELAXED, DEV_SCOPE);
        y += __hip_atomic_load(&a.chunk_stats[CS_WORDS * i + 4], __ATOMIC_RELAXED, DEV_SCOPE);  // no carry: < 2^40 per chunk
    }
    m = wred_min_i64(m);
    d = wred_sum_i64(d);
    r = wred_sum_i64(r);
    q = wred_sum_i64(q);
    y = wred_sum_i64(y);
    int64_t* red = (int64_t*)area;  // [5][IG_BLOCK / 64]
    constexpr int NWV = IG_BLOCK / 64;
    if ((tid & 63) == 0) {
        red[tid >> 6] = m;
        red[NWV + (tid >> 6)] = d;
        red[2 * NWV + (tid >> 6)] = r;
        red[3 * NWV + (tid >> 6)] = q;
        red[4 * NWV + (tid >> 6)] = y;
    }
    __syncthreads();
    if (tid == 0) {
#pragma unroll 1
        for (int v = 1; v < NWV; v++) {
            m = min(m, red[v]);
            d += red[NWV + v];
            r += red[2 * NWV + v];
            q += red[3 * NWV + v];
            y += red[4 * NWV + v];
        }
        a.slot_nch[slot] = (int32_t)gridDim.x;
        a.slot_base[slot] = slice_end_of(a.win, wadd(cur_wm, 1));  // used by compact chunks only
        if (a.runs) a.slot_fmt[slot] = (int32_t)push_fmt;
        ctrl->pending_pushes = slot + 1;
        ctrl->min_pending = min(ctrl->min_pending, m);
        ctrl->pending_rows += (uint64_t)r;
        ctrl->partials += (uint64_t)q;
        ctrl->part_bytes += (uint64_t)(y & ((1ll << 40) - 1));
        ctrl->compact_chunks += (uint64_t)(y >> 40);
        if (fold) ctrl->fold_skip = q * 50 > r * 49;  // folded away fewer than 2 % of the rows
        ctrl->push_count += 1;
        ctrl->late_dropped += (uint64_t)d;
    }
    if (pk_stats) {  // (uniform) the push's key and accumulator ranges -> the next epoch's PF_PACK fields
        int64_t kmn = INT64_MAX, kmx = INT64_MIN, vmn = INT64_MAX, vmx = INT64_MIN;
        for (int64_t i = tid; i < (int64_t)gridDim.x; i += IG_BLOCK) {
            const int64_t* cs = a.chunk_stats + CS_WORDS * i + 8;
            kmn = min(kmn, __hip_atomic_load(&cs[0], __ATOMIC_RELAXED, DEV_SCOPE));
            kmx = max(kmx, __hip_atomic_load(&cs[1], __ATOMIC_RELAXED, DEV_SCOPE));
            vmn = min(vmn, __hip_atomic_load(&cs[2], __ATOMIC_RELAXED, DEV_SCOPE));
            vmx = max(vmx, __hip_atomic_load(&cs[3], __ATOMIC_RELAXED, DEV_SCOPE));
        }
        kmn = wred_min_i64(kmn);
        kmx = wred_max_i64(kmx);
        vmn = wred_min_i64(vmn);
        vmx = wred_max_i64(vmx);
        __syncthreads();  // tid 0 is done with red
        if ((tid & 63) == 0) {
            red[tid >> 6] = kmn;
            red[NWV + (tid >> 6)] = kmx;
            red[2 * NWV + (tid >> 6)] = vmn;
            red[3 * NWV + (tid >> 6)] = vmx;
        }
        __syncthreads();
        if (tid == 0) {
#pragma unroll 1
            for (int v = 1; v < NWV; v++) {
                kmn = min(kmn, red[v]);
                kmx = max(kmx, red[NWV + v]);
                vmn = min(vmn, red[2 * NWV + v]);
                vmx = max(vmx, red[3 * NWV + v]);
            }
            if (slot == 0) {  // this push opened the flush epoch with the parameters it read
                ctrl->pk_cur_k = pk_k;
                ctrl->pk_cur_v = pk_v;
                ctrl->pk_cur_bits = pk_bits;
            }
            ctrl->pk_next_bits = pack_fields(kmn, kmx, vmn, vmx, &ctrl->pk_next_k, &ctrl->pk_next_v, ctrl->pk_next_bits);
        }
    }
    if (tid == 0) kt_end(a.kt);
}

template <int NV, int NW, bool X>
static hipError_t ingest_x(const IngestArgs& a, hipStream_t s, KTimer* t) {
    constexpr int RPT = ig_rpt(NW, NV);
    constexpr int BLK = ig_block(NW, NV);
    const int64_t nch = a.n_chunks;
    if (nch == 0) return hipSuccess;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)k_ingest<NV, NW, RPT, X, BLK>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, ig_lds(BLK));
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    // the fold table and the histogram must fit the dynamic LDS
    if ((int64_t)(IG_HDR_WORDS + ig_hist_words(a.ks.n_sb >> a.ks.pass_log2)) * 8 + ig_fold_bytes(NW) > a.lds_bytes)
        return hipErrorInvalidValue;
    if (a.lds_bytes != ig_lds(BLK)) return hipErrorInvalidValue;
    if (a.runs && !ig_runs_fit(a.ks.n_sb >> a.ks.pass_log2, BLK, RPT, NW)) return hipErrorInvalidValue;
    kt_mark(t, FW_KT_REDUCE, false, s);
    hipLaunchKernelGGL((k_ingest<NV, NW, RPT, X, BLK>), dim3((unsigned)nch), dim3(BLK), a.lds_bytes, s, a);
    kt_mark(t, FW_KT_REDUCE, true, s);
    return hipGetLastError();
}

template <int NV, int NW>
static hipError_t ingest_nw(const IngestArgs& a, hipStream_t s, KTimer* t) {
    bool x = a.wd.has_ord != 0;
    for (int q = 0; q < MAX_KCOLS; q++) x = x || a.nulls[q] != nullptr;
    return x ? ingest_x<NV, NW, true>(a, s, t) : ingest_x<NV, NW, false>(a, s, t);
}

template <int NV>
hipError_t ingest_nv(const IngestArgs& a, hipStream_t s, KTimer* t) {
    const int nw = a.wd.nw;
    if (nw <= 1) return ingest_nw<NV, 1>(a, s, t);
    if (nw <= 2) return ingest_nw<NV, 2>(a, s, t);
    if (nw <= 4) return ingest_nw<NV, 4>(a, s, t);
    return ingest_nw<NV, 8>(a, s, t);
}

}  // namespace fw
