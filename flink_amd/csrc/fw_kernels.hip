// fw_kernels.hip -- gfx950 kernels of libflinkwin (MI355X, CDNA4, wave64).
//
// Data path per watermark interval (SURVEY.md 2.2 kernel list):
//   k_ingest      (K1+K2+K3)  key-group + slice assignment + late classification, then a
//                 coalesced-load, LDS-staged segmented reduce: a direct-mapped LDS cache folds
//                 repeated (key, slice) pairs (hot keys), the rest pass through; the chunk's
//                 partials are counting-sorted by superbucket in LDS and written contiguously.
//                 Restates AbstractSliceSyncStateWindowAggProcessor.processElement (:96-126),
//                 RecordsWindowBuffer.addElement (:81) and the per-group fold of AggCombiner (:76-99).
//   k_merge_fire  (K4+K5)  one workgroup per superbucket: loads its slice-state entries from HBM
//                 into an LDS hash table, merges the pending partials (flush), registers timers,
//                 then fires every due (key, window) timer in timestamp rounds (fireWindow / merge /
//                 clearWindow / nextTriggerWindow) and writes the live entries back.
//                 Restates RecordsWindowBuffer.flush (:115), AggCombiner.combine (:76-115),
//                 InternalTimerServiceImpl.tryAdvanceWatermark (:328-348), WindowAggOperator.onTimer
//                 (:258), Slice{Unshared,Shared}SyncStateWindowAggProcessor.fireWindow and
//                 AbstractSliceSyncStateWindowAggProcessor.clearWindow (:161-167).
// All control decisions (flush? fire? next trigger progress) are made on the device from the
// Ctrl block, so a watermark cycle is two launches and no host synchronisation.
#include <hip/hip_runtime.h>

#include <utility>

#include "fw_internal.h"

namespace fw {

// compile-time loop: f(std::integral_constant<int, J>) for J in [0, N).  Keeps per-record
// register arrays indexed by constants regardless of the unroller's size heuristics.
template <typename F, int... Js>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Js...>) {
    (f(std::integral_constant<int, Js>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

#define LDS_SCOPE __HIP_MEMORY_SCOPE_WORKGROUP
#define DEV_SCOPE __HIP_MEMORY_SCOPE_AGENT

__device__ __forceinline__ double as_f64(uint64_t b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ uint64_t f64_bits(double d) { return (uint64_t)__double_as_longlong(d); }

// select value column `col` from a per-record register array without dynamic indexing
template <int N>
__device__ __forceinline__ uint64_t pick_col(const uint64_t (&v)[N], int32_t col) {
    uint64_t r = v[0];
#pragma unroll
    for (int c = 1; c < N; c++)
        if (col == c) r = v[c];
    return r;
}

__device__ __forceinline__ bool f64_isnan(uint64_t b) { return (b & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull; }
__device__ __forceinline__ bool f64_iszero(uint64_t b) { return (b & 0x7FFFFFFFFFFFFFFFull) == 0; }

// value of one accumulator word for a single non-NULL record (accumulate on the identity);
// `ord` >= 1 is the record's arrival ordinal within the flush (W_Q* words only)
__device__ __forceinline__ uint64_t record_word(int32_t op, uint64_t v, uint32_t ord) {
    switch (op) {
        case W_CNT: return 1;
        case W_MIN_D:
        case W_MAX_D: return (uint64_t)dkey(v);
        case W_QMIN:
        case W_QMAX: return f64_isnan(v) ? word_identity(op) : f64_iszero(v) ? 0ull : (uint64_t)dkey(v);
        case W_QFIRST: return ((uint64_t)ord << 32) | (f64_isnan(v) ? (v >> 32) : 0ull);
        case W_QNANLO: return f64_isnan(v) ? (((uint64_t)ord << 32) | (v & 0xFFFFFFFFull)) : Q_EMPTY;
        case W_QZERO: return f64_iszero(v) ? (((uint64_t)ord << 1) | (v >> 63)) : Q_EMPTY;
        default: return v;  // SUM_I, SUM_F (bits), MIN_I, MAX_I, CNTV
    }
}
// a record's word, honouring the word's NULL gate (null_slots: bit s = value slot s is NULL)
__device__ __forceinline__ uint64_t gated_word(const WordDesc& wd, int w, uint64_t v, uint32_t null_slots, uint32_t ord) {
    const int32_t g = wd.gate[w];
    if (g >= 0 && ((null_slots >> g) & 1u)) return word_identity(wd.op[w]);
    return record_word(wd.op[w], v, ord);
}

// atomically fold `v` into an LDS accumulator word (element-level combine: commutative)
__device__ __forceinline__ void lds_fold(int32_t op, uint64_t* slot, uint64_t v) {
    switch (op) {
        case W_CNT:
        case W_CNTV:
        case W_SUM_I: __hip_atomic_fetch_add(slot, v, __ATOMIC_RELAXED, LDS_SCOPE); break;
        case W_SUM_F: __hip_atomic_fetch_add((double*)slot, as_f64(v), __ATOMIC_RELAXED, LDS_SCOPE); break;
        case W_MIN_I:
        case W_MIN_D:
        case W_QMIN: __hip_atomic_fetch_min((int64_t*)slot, (int64_t)v, __ATOMIC_RELAXED, LDS_SCOPE); break;
        case W_QFIRST:
        case W_QNANLO:
        case W_QZERO: __hip_atomic_fetch_min(slot, v, __ATOMIC_RELAXED, LDS_SCOPE); break;
        default: __hip_atomic_fetch_max((int64_t*)slot, (int64_t)v, __ATOMIC_RELAXED, LDS_SCOPE); break;
    }
}

// element-level fold in registers
__device__ __forceinline__ uint64_t reg_fold(int32_t op, uint64_t a, uint64_t b) {
    switch (op) {
        case W_CNT:
        case W_CNTV:
        case W_SUM_I: return a + b;
        case W_SUM_F: return f64_bits(as_f64(a) + as_f64(b));
        case W_MIN_I:
        case W_MIN_D:
        case W_QMIN: return (int64_t)a < (int64_t)b ? a : b;
        case W_QFIRST:
        case W_QNANLO:
        case W_QZERO: return a < b ? a : b;
        default: return (int64_t)a > (int64_t)b ? a : b;
    }
}

// ---- SQL MIN/MAX(DOUBLE) word groups ------------------------------------------------------
// result of aggregate g from its words: the NaN that arrived first, else the extremum of the
// non-NaN values (a zero takes the sign of the earliest zero); *isnull when no non-NULL value
__device__ __forceinline__ uint64_t q_result(const AggDesc& ad, int g, const uint64_t* acc, bool* isnull) {
    const uint64_t f = acc[ad.qf[g]];
    *isnull = f == Q_EMPTY;
    if (*isnull) return 0;
    if ((uint32_t)f) return (f << 32) | (acc[ad.qn[g]] & 0xFFFFFFFFull);
    const int64_t k = (int64_t)acc[ad.w0[g]];
    if (k != 0) return dkey_inv(k);
    const uint64_t z = acc[ad.qz[g]];
    return z != Q_EMPTY ? ((z & 1ull) << 63) : 0ull;
}

// words of a group after the write-back of a flush: every recorded ordinal becomes 0 ("earlier
// than anything a later flush adds"), and a non-NaN-first group forgets its NaNs
__device__ __forceinline__ uint64_t q_normalise(const WordDesc& wd, int w, const uint64_t* acc) {
    const uint64_t v = acc[w];
    switch (wd.op[w]) {
        case W_QFIRST: return v != Q_EMPTY ? (v & 0xFFFFFFFFull) : v;
        case W_QZERO: return v != Q_EMPTY ? (v & 1ull) : v;
        case W_QNANLO: {
            const uint64_t f = acc[wd.qfirst[w]];
            return (f != Q_EMPTY && (uint32_t)f) ? (v & 0xFFFFFFFFull) : Q_EMPTY;
        }
        default: return v;
    }
}

// slice merge at fire time, in the reference's order: acc = merge(acc, other) with the aggregates'
// mergeExpressions (acc earlier).  Counts and sums add; integer and DataStream min/max are order
// free; SQL MIN/MAX(DOUBLE) compare result values with a strict `<` / `>` (MaxAggFunction.java:82-95)
// and the merged value is re-encoded as one element with ordinal 0.
// the SQL-double part, out of line: it only runs in the Q kernel variants and keeps its
// scratch arrays out of the hot path's register budget
__device__ __noinline__ void merge_q_groups(const WordDesc& wd, const AggDesc& ad, uint64_t* acc, const uint64_t* other) {
    uint64_t res[FW_MAX_AGGS];
    bool nul[FW_MAX_AGGS];
    {
        for (int g = 0; g < ad.n; g++) {
            if (ad.qf[g] < 0) continue;
            bool na, no;
            const uint64_t ra = q_result(ad, g, acc, &na);
            const uint64_t ro = q_result(ad, g, other, &no);
            const bool take = !no && (na || (ad.kind[g] == FW_AGG_MAX ? as_f64(ro) > as_f64(ra) : as_f64(ro) < as_f64(ra)));
            res[g] = take ? ro : ra;
            nul[g] = na && no;
        }
    }
    {
        for (int g = 0; g < ad.n; g++)
            if (ad.qf[g] >= 0) {
                acc[ad.qf[g]] = Q_EMPTY;
                acc[ad.qn[g]] = Q_EMPTY;
                acc[ad.qz[g]] = Q_EMPTY;
            }
        for (int g = 0; g < ad.n; g++) {
            if (ad.qf[g] < 0) continue;
            const int op = wd.op[ad.w0[g]];
            if (nul[g]) {
                acc[ad.w0[g]] = word_identity(op);
                continue;
            }
            const uint64_t b = res[g];
            const bool nan = f64_isnan(b);
            acc[ad.qf[g]] = nan ? (b >> 32) : 0ull;
            if (nan) acc[ad.qn[g]] = b & 0xFFFFFFFFull;
            if (f64_iszero(b)) acc[ad.qz[g]] = b >> 63;
            acc[ad.w0[g]] = nan ? word_identity(op) : f64_iszero(b) ? 0ull : (uint64_t)dkey(b);
        }
    }
}

template <int NW, bool Q>
__device__ __forceinline__ void merge_slice(const WordDesc& wd, const AggDesc& ad, uint64_t* acc, const uint64_t* other) {
    if constexpr (Q) {
        // acc/other travel through memory for the out-of-line group merge
        uint64_t a2[MAX_WORDS], o2[MAX_WORDS];
#pragma unroll
        for (int w = 0; w < MAX_WORDS; w++) {
            a2[w] = w < NW ? acc[w] : 0;
            o2[w] = w < NW ? other[w] : 0;
        }
        merge_q_groups(wd, ad, a2, o2);
#pragma unroll
        for (int w = 0; w < NW; w++)
            acc[w] = (w < wd.nw && !is_qword(wd.op[w])) ? reg_fold(wd.op[w], acc[w], other[w]) : a2[w];
    } else {
#pragma unroll
        for (int w = 0; w < NW; w++)
            if (w < wd.nw) acc[w] = reg_fold(wd.op[w], acc[w], other[w]);
    }
}

// fold slot of a (key, slice): from the key's murmur (already computed for routing) and the slice
__device__ __forceinline__ uint32_t fold_slot(uint32_t m, int64_t s, int slots) {
    const uint32_t h = (m ^ ((uint32_t)s * 0x9E3779B1u) ^ (uint32_t)((uint64_t)s >> 32)) * 0x85EBCA6Bu;
    return (h ^ (h >> 15)) & (uint32_t)(slots - 1);
}
// LDS state-table index hash of a (key, slice): 32-bit multiply-xorshift (build-internal)
__device__ __forceinline__ uint32_t index_hash(int64_t k, int64_t s) {
    uint32_t h = (uint32_t)k * 0x9E3779B1u ^ (uint32_t)((uint64_t)k >> 32) * 0x85EBCA77u;
    h ^= ((uint32_t)s * 0xC2B2AE3Du) ^ (uint32_t)((uint64_t)s >> 32);
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    return h ^ (h >> 13);
}

// wave-level reductions: one LDS atomic per wave instead of one per lane (same-address LDS
// atomics serialise lane by lane)
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = min(v, (int64_t)__shfl_xor((long long)v, d, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d, 64);
    return v;
}
// slot claim for the active lanes of a wave: one atomicAdd on *ctr, each lane gets base + rank
__device__ __forceinline__ int32_t wave_claim(int32_t* ctr) {
    const uint64_t act = __ballot(1);
    const int lane = __lane_id();
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int rank = __popcll(act & ((1ull << lane) - 1ull));
    int32_t base = 0;
    if (lane == leader) base = atomicAdd(ctr, (int32_t)__popcll(act));
    return __shfl(base, leader, 64) + rank;
}

// Last-workgroup election, called by one thread per workgroup once the workgroup's published
// stores have completed (s_waitcnt vmcnt(0)).  True for exactly one workgroup of the grid, the
// last to arrive; it may then read what every other workgroup published (agent-scope loads).
// Workgroup b counts on group counter b % TK_GROUPS and the last of each group on the top
// counter: same-address device-scope atomics serialise at the memory side, so 1024 workgroups
// on one counter cost tens of microseconds.  Counters are left at 0 for the next launch.
__device__ bool grid_last_wg(uint32_t (*t)[32]) {
    const uint32_t G = gridDim.x, g = blockIdx.x % TK_GROUPS;
    const uint32_t in_g = (G - g + TK_GROUPS - 1) / TK_GROUPS;
    const uint32_t ng = min(G, (uint32_t)TK_GROUPS);
    if (__hip_atomic_fetch_add(&t[g][0], 1u, __ATOMIC_RELAXED, DEV_SCOPE) != in_g - 1) return false;
    __hip_atomic_store(&t[g][0], 0u, __ATOMIC_RELAXED, DEV_SCOPE);
    if (__hip_atomic_fetch_add(&t[TK_GROUPS][0], 1u, __ATOMIC_RELAXED, DEV_SCOPE) != ng - 1) return false;
    __hip_atomic_store(&t[TK_GROUPS][0], 0u, __ATOMIC_RELAXED, DEV_SCOPE);
    return true;
}

// ======================================================================================
// K1+K2+K3: single-pass ingest = slice/key-group assignment + LDS segmented reduce + a
// chunk-local counting sort of the partials by superbucket.
//
// One 1024-thread workgroup owns a chunk of CH = 1024*RPT rows and keeps all of them in
// registers (row j*1024 + tid, coalesced column loads, every load of the chunk in flight at
// once).  The chunk is folded in fold sub-tiles of 2048 rows: rows with equal (key, slice) meet
// in an LDS slot table whose owner is the lowest row index hashing to the slot (so a hot key,
// which occurs early, keeps its slot); the owner ends up holding the folded partial in its
// registers.  The surviving partials are then ranked per superbucket with LDS atomics, the
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

// X: the configuration has nullable columns or SQL MIN/MAX(DOUBLE) words (gates, ordinals)
template <int NV, int NW, int RPT, bool X>
__global__ __launch_bounds__(IG_BLOCK, 4) void k_ingest(IngestArgs a) {
    constexpr int CH = IG_BLOCK * RPT;
    constexpr int NSUB = RPT / IG_SRPT;
    constexpr int NVR = NV > 0 ? NV : 1;
    constexpr int PW = 2 + NW;
    constexpr int SL = ig_slots(NW);
    static_assert(RPT % IG_SRPT == 0, "fold sub-tiles must tile the chunk");
    // dynamic LDS only (16-B aligned base, G17): [header 16 words][hist: n_sb u32, padded to
    // 16 B][area: fold table, later the store stage]
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    int64_t* s_min = (int64_t*)&lds[0];
    unsigned long long* s_drop = (unsigned long long*)&lds[1];
    unsigned long long* s_rows = (unsigned long long*)&lds[2];
    uint32_t* wsum = (uint32_t*)&lds[4];  // IG_BLOCK / 64 words
    const int n_sb = a.ks.n_sb;
    uint32_t* hist = (uint32_t*)(lds + IG_HDR_WORDS);  // partials per superbucket -> cell start
    uint64_t* area = lds + IG_HDR_WORDS + ig_hist_words(n_sb);
    const int area_words = (a.lds_bytes >> 3) - IG_HDR_WORDS - ig_hist_words(n_sb);
    uint32_t* claim = (uint32_t*)area;                   // [SL]
    int64_t* ckey = (int64_t*)(area + (SL >> 1));       // [SL]
    int64_t* cslice = ckey + SL;                         // [SL]
    uint64_t* cacc = (uint64_t*)(cslice + SL);           // [NW][SL]

    const int tid = threadIdx.x;
    Ctrl* ctrl = a.ctrl;
    const int64_t c = blockIdx.x;
    // the push's slot in the partial buffer; k_push_stats (next launch) advances pending_pushes
    const int64_t slot = __hip_atomic_load(&ctrl->pending_pushes, __ATOMIC_RELAXED, DEV_SCOPE);
    if (slot >= FW_MAX_PENDING) {
        if (tid == 0) __hip_atomic_fetch_or(&ctrl->error, ERR_CHUNKS, __ATOMIC_RELAXED, DEV_SCOPE);
        return;
    }
    const int64_t cur_wm = __hip_atomic_load(&ctrl->cur, __ATOMIC_RELAXED, DEV_SCOPE);
    if (tid == 0) {
        *s_min = INT64_MAX;
        *s_drop = 0;
        *s_rows = 0;
    }
    for (int s = tid; s < n_sb; s += IG_BLOCK) hist[s] = 0;

    // ---- coalesced column loads of the whole chunk (all in flight before the first use)
    const int64_t base = c * CH;
    const int64_t ts0 = a.ts[base];  // chunk base for the 32-bit slice arithmetic
    int64_t rk[RPT], rs[RPT];
    uint64_t rv[RPT][NVR];
    int32_t pre[RPT];
    uint32_t rnul[RPT];  // bit q: value slot q is NULL in this row
    uint32_t valid = 0;
    static_for<RPT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const int64_t i = base + (int64_t)j * IG_BLOCK + tid;
        rk[j] = 0;
        rs[j] = 0;
        pre[j] = 0;
        rnul[j] = 0;
#pragma unroll
        for (int q = 0; q < NVR; q++) rv[j][q] = 0;
        if (i < a.n) {
            rk[j] = a.key[i];
            rs[j] = a.ts[i];
            if (a.khash) pre[j] = a.khash[i];
#pragma unroll
            for (int q = 0; q < NV; q++) {
                if (NV > 2 && q >= a.nv) break;  // the NV = 4 / 8 variants also serve 3 / 5-7 columns
                rv[j][q] = a.vals[q][i];
                if (X && a.nulls[q] && a.nulls[q][i]) rnul[j] |= 1u << q;
            }
            valid |= 1u << j;
        }
    });
    // arrival ordinal base of this chunk within the flush (W_Q* words; >= 1, see record_word)
    const uint32_t ord0 = (uint32_t)(slot * a.cap_rows + base) + 1u;
    // slice-aligned base 2^30 ms below the chunk's first row: rows within 2^31 ms of it take
    // the 32-bit path (one mul_hi instead of a 64-bit magic division)
    const bool fast = a.win.fast32 && ts0 > -(1ll << 61) && ts0 < (1ll << 61);
    const int64_t tbase = fast ? window_start(ts0, a.win.offset, a.win.slice_div) -
                                     (int64_t)((1u << 30) / (uint32_t)a.win.interval) * a.win.interval
                               : 0;
    // ---- K1/K2: key group -> superbucket, slice end, late classification, record words
    int32_t rsb[RPT];
    uint32_t rm[RPT];
    uint64_t racc[RPT][NW];
    int64_t lmin = INT64_MAX;
    uint32_t ldrop = 0, lrows = 0;
    static_for<RPT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        rsb[j] = 0;
        rm[j] = 0;
#pragma unroll
        for (int w = 0; w < NW; w++)
            racc[j][w] = w >= a.wd.nw ? 0
                         : X ? gated_word(a.wd, w, pick_col(rv[j], a.wd.col[w]), rnul[j],
                                          ord0 + (uint32_t)(j * IG_BLOCK + tid))
                             : record_word(a.wd.op[w], pick_col(rv[j], a.wd.col[w]), 0);
        if (!(valid & (1u << j))) return;
        rsb[j] = route_key(a.ks, rk[j], pre[j], &rm[j]);
        if ((uint32_t)rsb[j] >= (uint32_t)n_sb) {  // key group not owned by this subtask
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
        if (!a.local && is_fired(se, cur_wm)) {
            if (is_fired(last_window_end_of(a.win, se), cur_wm)) {  // late for every window: drop
                valid &= ~(1u << j);
                ldrop++;
                return;
            }
            target = merge_target_of(a.win, se);
            // timer for the first unfired window (processElement :111-117)
            const int64_t steps = (int64_t)((uint64_t)wsub(wadd(cur_wm, 1), se) / (uint64_t)a.win.interval) + 1;
            const int64_t unfired = wadd(se, steps * a.win.interval);
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
    // ---- K3: fold equal (key, slice) rows, one 1024-row sub-tile at a time
    if (!(a.ablate & AB_NO_FOLD)) static_for<NSUB>([&](auto S) {
        constexpr int s = decltype(S)::value;
        uint32_t rh[IG_SRPT];
        __syncthreads();  // previous sub-tile's owners are done with claim/cacc
        for (int h = tid; h < SL; h += IG_BLOCK) claim[h] = 0xFFFFFFFFu;
        __syncthreads();
        static_for<IG_SRPT>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            constexpr int j = s * IG_SRPT + q;
            rh[q] = fold_slot(rm[j], rs[j], SL);
            if (valid & (1u << j)) atomicMin(&claim[rh[q]], (uint32_t)(j * IG_BLOCK + tid));
        });
        __syncthreads();
        static_for<IG_SRPT>([&](auto Q) {  // slot owners publish their (key, slice) and partial
            constexpr int q = decltype(Q)::value;
            constexpr int j = s * IG_SRPT + q;
            if (!(valid & (1u << j)) || claim[rh[q]] != (uint32_t)(j * IG_BLOCK + tid)) return;
            ckey[rh[q]] = rk[j];
            cslice[rh[q]] = rs[j];
#pragma unroll
            for (int w = 0; w < NW; w++) cacc[w * SL + rh[q]] = racc[j][w];
        });
        __syncthreads();
        static_for<IG_SRPT>([&](auto Q) {  // everyone else folds into a matching owner
            constexpr int q = decltype(Q)::value;
            constexpr int j = s * IG_SRPT + q;
            const uint32_t h = rh[q];
            if (!(valid & (1u << j)) || claim[h] == (uint32_t)(j * IG_BLOCK + tid)) return;
            if (ckey[h] == rk[j] && cslice[h] == rs[j]) {
#pragma unroll
                for (int w = 0; w < NW; w++)
                    if (w < a.wd.nw) lds_fold(a.wd.op[w], &cacc[w * SL + h], racc[j][w]);
                valid &= ~(1u << j);
            }
        });
        __syncthreads();
        static_for<IG_SRPT>([&](auto Q) {  // owners take the folded partial back
            constexpr int q = decltype(Q)::value;
            constexpr int j = s * IG_SRPT + q;
            if (!(valid & (1u << j)) || claim[rh[q]] != (uint32_t)(j * IG_BLOCK + tid)) return;
#pragma unroll
            for (int w = 0; w < NW; w++) racc[j][w] = cacc[w * SL + rh[q]];
        });
    });
    // ---- rank the partials per superbucket, scan, publish the cells
    uint32_t rdst[RPT];
    const bool sort = !(a.ablate & AB_NO_SORT);
    static_for<RPT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        rdst[j] = (sort && (valid & (1u << j))) ? atomicAdd(&hist[rsb[j]], 1u) : (uint32_t)(j * IG_BLOCK + tid);
    });
    __syncthreads();
    uint32_t* cells = a.cells + (size_t)slot * n_sb * a.max_nch;
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
            cells[cell_index(c, n_sb, i)] = run | (v << 16);
            run += v;
        }
    __syncthreads();
    if (sort)
        static_for<RPT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            if (valid & (1u << j)) rdst[j] += hist[rsb[j]];
        });
    else
        total = CH;
    // ---- store the partials through an LDS stage so every global store is a full line
    uint64_t* out = a.parts + ((size_t)slot * a.cap_rows + (size_t)base) * PW;
    const uint32_t wrows = (uint32_t)(area_words / PW) & ~1u;
    if (!(a.ablate & AB_NO_STORE))
        for (uint32_t w0 = 0; w0 < total; w0 += wrows) {
            __syncthreads();  // fold table / previous window no longer read
            static_for<RPT>([&](auto J) {
                constexpr int j = decltype(J)::value;
                const uint32_t d = rdst[j] - w0;
                if (!(valid & (1u << j)) || d >= wrows) return;
                uint64_t* p = area + (size_t)d * PW;
                p[0] = (uint64_t)rk[j];
                p[1] = (uint64_t)rs[j];
#pragma unroll
                for (int w = 0; w < NW; w++) p[2 + w] = racc[j][w];
            });
            __syncthreads();
            const uint32_t nwords = min(wrows, total - w0) * PW;
            uint64_t* dst = out + (size_t)w0 * PW;  // 16-B aligned: slot, chunk and window bases are even rows
            for (uint32_t q = 2 * tid; q < nwords; q += 2 * IG_BLOCK) {
                if (q + 1 < nwords) {
                    *(ulonglong2*)(dst + q) = *(const ulonglong2*)(area + q);
                } else {
                    dst[q] = area[q];
                }
            }
        }
    // ---- control counters.  Each chunk publishes its stats with agent-scope stores (they bypass
    // the XCD's L2, so any XCD reads them), then takes a ticket; the last workgroup of the launch
    // reduces every chunk's stats into the control block and commits the push's slot
    // (RecordsWindowBuffer's minSliceEnd and the late-drop counter).  No extra launch.
    if (lmin != INT64_MAX) __hip_atomic_fetch_min(s_min, lmin, __ATOMIC_RELAXED, LDS_SCOPE);
    if (ldrop) atomicAdd(s_drop, (unsigned long long)ldrop);
    if (lrows) atomicAdd(s_rows, (unsigned long long)lrows);
    __syncthreads();
    int32_t* s_last = (int32_t*)&lds[3];
    if (tid == 0) {
        __hip_atomic_store(&a.chunk_stats[4 * c], *s_min, __ATOMIC_RELAXED, DEV_SCOPE);
        __hip_atomic_store(&a.chunk_stats[4 * c + 1], (int64_t)*s_drop, __ATOMIC_RELAXED, DEV_SCOPE);
        __hip_atomic_store(&a.chunk_stats[4 * c + 2], (int64_t)*s_rows, __ATOMIC_RELAXED, DEV_SCOPE);
        __hip_atomic_store(&a.chunk_stats[4 * c + 3], (int64_t)total, __ATOMIC_RELAXED, DEV_SCOPE);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *s_last = grid_last_wg(a.tickets->c[0]);
    }
    __syncthreads();
    if (!*s_last) return;
    int64_t m = INT64_MAX, d = 0, r = 0, q = 0;
    for (int64_t i = tid; i < (int64_t)gridDim.x; i += IG_BLOCK) {
        m = min(m, __hip_atomic_load(&a.chunk_stats[4 * i], __ATOMIC_RELAXED, DEV_SCOPE));
        d += __hip_atomic_load(&a.chunk_stats[4 * i + 1], __ATOMIC_RELAXED, DEV_SCOPE);
        r += __hip_atomic_load(&a.chunk_stats[4 * i + 2], __ATOMIC_RELAXED, DEV_SCOPE);
        q += __hip_atomic_load(&a.chunk_stats[4 * i + 3], __ATOMIC_RELAXED, DEV_SCOPE);
    }
    m = wave_min_i64(m);
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) {
        d += (int64_t)__shfl_xor((long long)d, k, 64);
        r += (int64_t)__shfl_xor((long long)r, k, 64);
        q += (int64_t)__shfl_xor((long long)q, k, 64);
    }
    int64_t* red = (int64_t*)area;  // [4][IG_BLOCK / 64]
    constexpr int NWV = IG_BLOCK / 64;
    if ((tid & 63) == 0) {
        red[tid >> 6] = m;
        red[NWV + (tid >> 6)] = d;
        red[2 * NWV + (tid >> 6)] = r;
        red[3 * NWV + (tid >> 6)] = q;
    }
    __syncthreads();
    if (tid == 0) {
        for (int v = 1; v < NWV; v++) {
            m = min(m, red[v]);
            d += red[NWV + v];
            r += red[2 * NWV + v];
            q += red[3 * NWV + v];
        }
        a.slot_nch[slot] = (int32_t)gridDim.x;
        ctrl->pending_pushes = slot + 1;
        ctrl->min_pending = min(ctrl->min_pending, m);
        ctrl->pending_rows += (uint64_t)r;
        ctrl->partials += (uint64_t)q;
        ctrl->late_dropped += (uint64_t)d;
    }
}

// ---- result compaction: slabs (+ overflow) -> one contiguous result set ----------------------
__global__ __launch_bounds__(BLOCK) void k_compact_scan(const int32_t* sb_out, int32_t n_sb, int64_t* off, Ctrl* ctrl,
                                                        int64_t out_cap) {
    __shared__ int64_t tmp[BLOCK];
    __shared__ int64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < n_sb; base += BLOCK) {
        const int i = base + threadIdx.x;
        const int64_t v = i < n_sb ? sb_out[i] : 0;
        tmp[threadIdx.x] = v;
        __syncthreads();
        for (int d = 1; d < BLOCK; d <<= 1) {
            const int64_t x = threadIdx.x >= d ? tmp[threadIdx.x - d] : 0;
            __syncthreads();
            tmp[threadIdx.x] += x;
            __syncthreads();
        }
        if (i < n_sb) off[i] = carry + tmp[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == BLOCK - 1) carry += tmp[BLOCK - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int64_t ovf = (int64_t)min(ctrl->out_count[ctrl->ovf_sel & 1], (uint64_t)out_cap);
        off[n_sb] = carry;          // slab rows
        off[n_sb + 1] = carry + ovf;  // total rows
    }
}

__global__ __launch_bounds__(BLOCK) void k_compact_copy(CompactArgs a) {
    const int sb = blockIdx.x;
    int64_t src0, dst0, n;
    if (sb < a.n_sb) {
        src0 = (int64_t)sb * a.slab_cap;
        dst0 = a.off[sb];
        n = a.sb_out[sb];
    } else {  // overflow region
        src0 = (int64_t)a.n_sb * a.slab_cap;
        dst0 = a.off[a.n_sb];
        n = a.off[a.n_sb + 1] - a.off[a.n_sb];
    }
    for (int64_t i = threadIdx.x; i < n; i += BLOCK) {
        const int64_t d = dst0 + i, sidx = src0 + i;
        if (d >= a.res_cap) break;
        a.res_key[d] = a.out_key[sidx];
        a.res_ws[d] = a.out_ws[sidx];
        a.res_we[d] = a.out_we[sidx];
        a.res_null[d] = a.out_null[sidx];
        for (int g = 0; g < a.n_aggs; g++) a.res_val[g][d] = a.out_val[g][sidx];
    }
}

// ======================================================================================
// K4+K5: merge pending partials into the HBM slice-state table, fire due timers
// ======================================================================================
template <int NW, int E>
struct StateLds {
    uint32_t idx[2 * E];   // open-addressing index: 0 empty, 1 claiming, 2+e entry e
    int64_t key[E];
    int64_t slice[E];
    uint32_t flag[E];
    uint64_t acc[NW][E];
    uint16_t due[E];       // entries whose timer is due at this watermark (each fires once)
    int32_t ndue;
    int32_t n;             // entries in use
    uint32_t overflow;
};

constexpr uint32_t IDX_DEAD = 0xFFFFFFFFu;

template <int NW, int E>
__device__ __forceinline__ void init_entry_acc(StateLds<NW, E>& S, int e, const WordDesc& wd) {
#pragma unroll
    for (int w = 0; w < NW; w++) S.acc[w][e] = w < wd.nw ? word_identity(wd.op[w]) : 0;
}

// LDS publication protocol of the index: the inserting lane writes the entry's fields, then
// (after a compiler barrier) the index word with a relaxed store.  LDS executes one wave's
// requests in issue order and a reader's field loads depend on the index value it read, so a
// reader that sees 2+e sees the fields.  Acquire/release orderings are not used: at workgroup
// scope they also order global memory, making every publish wait for earlier result stores.
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

template <int NW, int E>
__device__ int find_entry(StateLds<NW, E>& S, int64_t k, int64_t s) {
    constexpr uint32_t MASK = 2 * E - 1;
    uint32_t h = index_hash(k, s) & MASK;
    for (int probes = 0; probes < 2 * E;) {
        const uint32_t st = __hip_atomic_load(&S.idx[h], __ATOMIC_RELAXED, LDS_SCOPE);
        if (st == 0) return -1;
        if (st == 1) continue;  // being inserted by another lane: re-read
        const uint32_t e = st - 2;
        if (e < (uint32_t)E && S.key[e] == k && S.slice[e] == s) return (int)e;
        h = (h + 1) & MASK;
        probes++;
    }
    return -1;
}

// Finds (k, s) or inserts it.  A new entry starts from `v` folded into the identity (or the
// identity when v is null) with flags `flag0`; *inserted tells the caller it must not fold v again.
template <int NW, int E>
__device__ int find_or_insert(StateLds<NW, E>& S, int64_t k, int64_t s, const WordDesc& wd,
                              const uint64_t* v = nullptr, uint32_t flag0 = 0, bool* inserted = nullptr) {
    constexpr uint32_t MASK = 2 * E - 1;
    uint32_t h = index_hash(k, s) & MASK;
    for (int probes = 0; probes < 2 * E;) {
        const uint32_t st = __hip_atomic_load(&S.idx[h], __ATOMIC_RELAXED, LDS_SCOPE);
        if (st == 1) continue;
        if (st == 0) {
            uint32_t expect = 0;
            if (__hip_atomic_compare_exchange_strong(&S.idx[h], &expect, 1u, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, LDS_SCOPE)) {
                const int e = atomicAdd(&S.n, 1);
                if (e >= E) {
                    S.overflow = 1;
                    __hip_atomic_store(&S.idx[h], IDX_DEAD, __ATOMIC_RELAXED, LDS_SCOPE);
                    return -1;
                }
                S.key[e] = k;
                S.slice[e] = s;
                S.flag[e] = flag0;
#pragma unroll
                for (int w = 0; w < NW; w++)
                    S.acc[w][e] = w < wd.nw ? (v ? reg_fold(wd.op[w], word_identity(wd.op[w]), v[w])
                                                 : word_identity(wd.op[w]))
                                            : 0;
                compiler_fence();
                __hip_atomic_store(&S.idx[h], 2u + (uint32_t)e, __ATOMIC_RELAXED, LDS_SCOPE);
                if (inserted) *inserted = true;
                return e;
            }
            continue;  // lost the race: re-read this slot
        }
        const uint32_t e = st - 2;
        if (e < (uint32_t)E && S.key[e] == k && S.slice[e] == s) return (int)e;
        h = (h + 1) & MASK;
        probes++;
    }
    S.overflow = 1;
    return -1;
}

// First-probe lookups of M (key, slice) pairs with their LDS loads issued together (the lookups
// of one lane are independent; issuing them back to back overlaps their latencies).  e[j] is the
// entry, -1 when the home slot is empty, -2 when the first probe does not decide (collision or
// an insertion in flight): the caller then takes the probing path.
template <int NW, int E, int M>
__device__ __forceinline__ void probe_batch(StateLds<NW, E>& S, const int64_t* k, const int64_t* s, int* e,
                                            int m = M) {
    // only the first m (<= M, uniform) lookups are needed; the others issue no LDS reads
    constexpr uint32_t MASK = 2 * E - 1;
    uint32_t st[M];
#pragma unroll
    for (int j = 0; j < M; j++)
        st[j] = j < m ? __hip_atomic_load(&S.idx[index_hash(k[j], s[j]) & MASK], __ATOMIC_RELAXED, LDS_SCOPE) : 0u;
    int64_t kk[M], ss[M];
#pragma unroll
    for (int j = 0; j < M; j++) {
        kk[j] = 0;
        ss[j] = 0;
        if (j >= m) continue;
        const uint32_t ei = min(st[j] - 2u, (uint32_t)(E - 1));
        kk[j] = S.key[ei];
        ss[j] = S.slice[ei];
    }
#pragma unroll
    for (int j = 0; j < M; j++)
        e[j] = st[j] == 0 ? -1
               : (st[j] >= 2 && st[j] - 2 < (uint32_t)E && kk[j] == k[j] && ss[j] == s[j]) ? (int)(st[j] - 2)
                                                                                          : -2;
}

// register an event-time timer on entry e; a timer that is already due at this watermark joins
// the due list (an entry's timer fires at most once per advance: its timestamp is its slice end)
template <int NW, int E>
__device__ __forceinline__ void set_timer(StateLds<NW, E>& S, int e, int64_t W) {
    const uint32_t old = atomicOr(&S.flag[e], F_TIMER);
    if (!(old & F_TIMER) && is_fired(S.slice[e], W)) {
        const int q = atomicAdd(&S.ndue, 1);
        if (q < E) S.due[q] = (uint16_t)e;
    }
}

// Emission is atomic-free at device scope: each superbucket appends to its own output slab
// (LDS cursor); only slab overflow falls back to a shared overflow region.  fw_results compacts
// slabs + overflow into one contiguous result set on demand (k_compact_*).
// output row position: the superbucket's slab, or the shared overflow region; -1 when full
__device__ __forceinline__ int64_t claim_out_row(const MergeArgs& a, int sb, int32_t* s_emit) {
    Ctrl* c = a.ctrl;
    const int32_t pos = wave_claim(s_emit);
    if (pos < a.slab_cap) return (int64_t)sb * a.slab_cap + pos;
    // a launch that resets the results counts on the spare counter (kept 0), see Ctrl::out_count
    const int sel = (__hip_atomic_load(&c->ovf_sel, __ATOMIC_RELAXED, DEV_SCOPE) ^ a.reset_out) & 1;
    const uint64_t o = atomicAdd((unsigned long long*)&c->out_count[sel], 1ull);
    if ((int64_t)o >= a.out_cap) {
        __hip_atomic_fetch_or(&c->error, ERR_OUTPUT, __ATOMIC_RELAXED, DEV_SCOPE);
        return -1;
    }
    return (int64_t)a.n_sb * a.slab_cap + (int64_t)o;
}

template <int NW, bool Q>
__device__ void emit_row(const MergeArgs& a, int sb, int32_t* s_emit, int64_t key, int64_t we, const uint64_t* acc) {
    if (a.ablate & AB_M_NO_EMIT) return;
    const int64_t i = claim_out_row(a, sb, s_emit);
    if (i < 0) return;
    a.out_key[i] = key;
    a.out_ws[i] = window_start_of(a.win, we);
    a.out_we[i] = we;
    uint32_t nm = 0;
    for (int g = 0; g < a.ad.n; g++) {
        const int32_t kind = a.ad.kind[g], type = a.ad.type[g];
        const uint64_t w0 = acc[a.ad.w0[g]];
        // SUM / MIN / MAX are NULL without a non-NULL input (SumAggFunction.java:66-69)
        const bool no_rows = a.ad.nn[g] >= 0 && acc[a.ad.nn[g]] == 0;
        uint64_t v = 0;
        switch (kind) {
            case FW_AGG_COUNT_STAR:
            case FW_AGG_COUNT: v = w0; break;
            case FW_AGG_SUM:
                v = type == FW_T_I32 ? (uint64_t)(int64_t)(int32_t)(uint32_t)w0 : w0;
                if (no_rows) nm |= 1u << g;
                break;
            case FW_AGG_MIN:
            case FW_AGG_MAX:
                if (Q && a.ad.qf[g] >= 0) {
                    bool isnull;
                    v = q_result(a.ad, g, acc, &isnull);
                    if (isnull) nm |= 1u << g;
                    break;
                }
                v = type == FW_T_F64 ? dkey_inv((int64_t)w0) : w0;
                if (no_rows) nm |= 1u << g;
                break;
            case FW_AGG_AVG: {
                const uint64_t cnt = acc[a.ad.w1[g]];
                if (cnt == 0) { nm |= 1u << g; break; }
                if (type == FW_T_F64) v = f64_bits(as_f64(w0) / (double)(int64_t)cnt);
                else {
                    int64_t q = (int64_t)w0 / (int64_t)cnt;
                    if (type == FW_T_I32) q = (int32_t)q;
                    v = (uint64_t)q;
                }
                break;
            }
        }
        a.out_val[g][i] = ((nm >> g) & 1u) ? 0ull : v;  // a NULL's value word is 0
    }
    a.out_null[i] = nm;
}

// LOCAL phase output (LocalAggCombiner.combine :69-97 -> output(key, window, acc)): one row per
// (key, sliceEnd) of the flush holding the local accumulator fields of every aggregate in order
// (COUNT(*) / COUNT: count; SUM, MIN, MAX: value, NULL-able; AVG: sum, count), window_end =
// window_start = sliceEnd.  The GLOBAL phase ingests exactly these columns.
template <int NW, bool Q>
__device__ void emit_partial(const MergeArgs& a, int sb, int32_t* s_emit, int64_t key, int64_t se, const uint64_t* acc) {
    const int64_t i = claim_out_row(a, sb, s_emit);
    if (i < 0) return;
    a.out_key[i] = key;
    a.out_ws[i] = se;
    a.out_we[i] = se;
    uint32_t nm = 0;
    int j = 0;
    for (int g = 0; g < a.ad.n; g++) {
        const int32_t kind = a.ad.kind[g], type = a.ad.type[g];
        const uint64_t w0 = acc[a.ad.w0[g]];
        const bool no_rows = a.ad.nn[g] >= 0 && acc[a.ad.nn[g]] == 0;
        uint64_t v = w0;
        bool isnull = false;
        switch (kind) {
            case FW_AGG_SUM:
                v = type == FW_T_I32 ? (uint64_t)(int64_t)(int32_t)(uint32_t)w0 : w0;
                isnull = no_rows;
                break;
            case FW_AGG_MIN:
            case FW_AGG_MAX:
                if (Q && a.ad.qf[g] >= 0) {
                    v = q_result(a.ad, g, acc, &isnull);
                    break;
                }
                v = type == FW_T_F64 ? dkey_inv((int64_t)w0) : w0;
                isnull = no_rows;
                break;
            case FW_AGG_AVG:  // (sum, count); the sum of AVG(INT) is a BIGINT (IntAvgAggFunction)
                a.out_val[j][i] = w0;
                j++;
                v = acc[a.ad.w1[g]];
                break;
            default: break;  // counts
        }
        if (isnull) nm |= 1u << j;
        a.out_val[j][i] = isnull ? 0ull : v;
        j++;
    }
    a.out_null[i] = nm;
}

// flags that live only inside one k_merge_fire launch (dropped at write-back)
constexpr uint32_t F_FIRED = 4u;    // HOP: window (key, this slice end) fired in this advance (chain claim)
constexpr uint32_t F_NOTHEAD = 8u;  // CUMULATE: an earlier due step of the same window chains to this one
constexpr uint32_t F_EXPIRE = 16u;  // HOP: slice expired by a window fired in this advance (cleared at write-back)

template <int NW>
__device__ __forceinline__ void acc_identity(const WordDesc& wd, uint64_t* acc) {
#pragma unroll
    for (int i = 0; i < NW; i++) acc[i] = i < wd.nw ? word_identity(wd.op[i]) : 0;
}

// acc = merge(acc, state of entry e) when the entry holds an accumulator (windowState.value != null)
template <int NW, int E, bool Q>
__device__ __forceinline__ void merge_entry(const MergeArgs& a, StateLds<NW, E>& S, int e, uint64_t* acc) {
    if (e < 0 || !(S.flag[e] & F_ACC)) return;
    uint64_t o[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) o[i] = S.acc[i][e];
    merge_slice<NW, Q>(a.wd, a.ad, acc, o);
}

// TUMBLE: SliceUnsharedSyncStateWindowAggProcessor.fireWindow (:54-66) + clearWindow
// (expiredSlices(we) = [we]); DataStream tumbling: WindowOperator.onEventTime + clearAllState.
// Windows of different keys and of one key are independent: every due entry fires once.
template <int NW, int E, bool Q>
__device__ __forceinline__ uint32_t fire_tumble(const MergeArgs& a, StateLds<NW, E>& S, int e, int sb, int32_t* s_emit) {
    uint64_t acc[NW];
    const uint32_t f = atomicAnd(&S.flag[e], ~(F_TIMER | F_ACC));
    if (f & F_ACC) {
#pragma unroll
        for (int i = 0; i < NW; i++) acc[i] = S.acc[i][e];
    } else {
        acc_identity<NW>(a.wd, acc);
    }
    if (a.ad.count_star_word < 0 || acc[a.ad.count_star_word] != 0) emit_row<NW, Q>(a, sb, s_emit, S.key[e], S.slice[e], acc);
    return 1;
}

// HOP: the timer chain of one key starting at due entry e, fired without timestamp rounds.
// SliceSharedSyncStateWindowAggProcessor.fireWindow (:65-86): merge the n slices ending at we
// newest first into a fresh accumulator, emit unless empty (hidden COUNT(*)), and while the window
// is non-empty register we + slice (nextTriggerWindow); a registered timer that is already due
// fires in this same advance (InternalTimerServiceImpl.tryAdvanceWatermark :328-348), so the
// chain continues.  clearWindow expires windowStart + slice: that slice also belongs to the
// earlier windows of the key that are due in this advance, so the expiry is deferred to the
// write-back (F_EXPIRE), after every window of the advance has read its slices.  With that, the
// chains of one key may run concurrently in any order; the F_FIRED claim makes every window fire
// exactly once.
template <int NW, int E, bool Q>
__device__ uint32_t fire_hop_chain(const MergeArgs& a, StateLds<NW, E>& S, int e, int sb, int32_t* s_emit) {
    const WinDesc& w = a.win;
    const WordDesc& wd = a.wd;
    constexpr int HB = NW <= 2 ? 8 : NW <= 4 ? 4 : 2;
    const int64_t k = S.key[e];
    int64_t we = S.slice[e];
    int ew = e;
    uint32_t nf = 0;
    for (;;) {
        const uint32_t old = atomicOr(&S.flag[ew], F_FIRED);
        if (old & F_FIRED) break;  // fired by another chain of this key
        atomicAnd(&S.flag[ew], ~F_TIMER);
        nf++;
        uint64_t acc[NW];
        acc_identity<NW>(wd, acc);
        const int n = w.n_slices;
        const int64_t s_exp = wadd(wsub(we, w.size), w.interval);  // clearWindow's expired slice
        int e_exp = -3;
        int64_t s = we;
        for (int j0 = 0; j0 < n; j0 += HB) {
            int64_t kk[HB], ss[HB];
            int eb[HB];
#pragma unroll
            for (int j = 0; j < HB; j++) {
                kk[j] = k;
                ss[j] = s;
                s = wsub(s, w.interval);  // wrapping, like the reference's long arithmetic
            }
            probe_batch<NW, E, HB>(S, kk, ss, eb, min(HB, n - j0));
#pragma unroll
            for (int j = 0; j < HB; j++) {
                if (j0 + j >= n) break;
                int e2 = eb[j];
                if (e2 == -2) e2 = find_entry(S, k, ss[j]);
                merge_entry<NW, E, Q>(a, S, e2, acc);
                if (ss[j] == s_exp) e_exp = e2;
            }
        }
        const bool nonempty = a.ad.count_star_word < 0 || acc[a.ad.count_star_word] != 0;
        if (nonempty) emit_row<NW, Q>(a, sb, s_emit, k, we, acc);
        const int e2 = e_exp != -3 ? e_exp : find_entry(S, k, s_exp);
        if (e2 >= 0) atomicOr(&S.flag[e2], F_EXPIRE);
        if (!nonempty) break;
        const int64_t nx = wadd(we, w.interval);
        const int en = find_or_insert(S, k, nx, wd);
        if (en < 0) break;  // state overflow (flagged)
        if (!is_fired(nx, a.wm)) {
            atomicOr(&S.flag[en], F_TIMER);
            break;
        }
        we = nx;
        ew = en;
    }
    return nf;
}

// CUMULATE: the steps of one cumulative window of one key, from its earliest due step, in order:
// mergeSlices merges step we's slice into the first-slice state (CumulativeSliceAssigner
// .mergeSlices, SliceSharedSyncStateWindowAggProcessor.merge :89-118), the window is emitted
// unless empty, the next step is registered up to the window's last step (nextTriggerWindow), and
// clearWindow expires we (and the first slice at the last step).  The merged accumulator stays in
// registers across the chain and is written back to the first slice once.
template <int NW, int E, bool Q>
__device__ uint32_t fire_cumulate_chain(const MergeArgs& a, StateLds<NW, E>& S, int e, int sb, int32_t* s_emit) {
    const WinDesc& w = a.win;
    const WordDesc& wd = a.wd;
    const int64_t k = S.key[e];
    int64_t we = S.slice[e];
    const int64_t ws = window_start_of(w, we);
    const int64_t first = wadd(ws, w.interval);
    const int64_t last = wadd(ws, w.size);
    const int ef = find_or_insert(S, k, first, wd);
    uint64_t acc[NW];
    if (ef >= 0 && (S.flag[ef] & F_ACC)) {
#pragma unroll
        for (int i = 0; i < NW; i++) acc[i] = S.acc[i][ef];
    } else {
        acc_identity<NW>(wd, acc);
    }
    uint32_t nf = 0;
    bool done = false;
    int ewe = e;
    for (;;) {
        if (ewe >= 0) atomicAnd(&S.flag[ewe], ~F_TIMER);
        if (we != first) merge_entry<NW, E, Q>(a, S, ewe, acc);
        nf++;
        if (a.ad.count_star_word < 0 || acc[a.ad.count_star_word] != 0) emit_row<NW, Q>(a, sb, s_emit, k, we, acc);
        if (we != first && ewe >= 0) atomicAnd(&S.flag[ewe], ~F_ACC);
        if (we == last) {  // expiredSlices(last) = [last, first]
            if (ef >= 0) atomicAnd(&S.flag[ef], ~F_ACC);
            done = true;
            break;
        }
        const int64_t nx = wadd(we, w.interval);
        if (!is_fired(nx, a.wm)) {
            const int en = find_or_insert(S, k, nx, wd);
            if (en >= 0) atomicOr(&S.flag[en], F_TIMER);
            break;
        }
        we = nx;
        ewe = we == first ? ef : find_entry(S, k, we);
    }
    if (!done && ef >= 0) {  // windowState.update(firstSlice, acc)
#pragma unroll
        for (int i = 0; i < NW; i++) S.acc[i][ef] = acc[i];
        atomicOr(&S.flag[ef], F_ACC);
    }
    return nf;
}

// CUMULATE pre-pass: a due step whose window has an earlier due step is reached by that step's
// chain (CUMULATE chains never stop before the window's last step), so it starts no chain of its
// own.  Each due step marks the next due step of its window.
template <int NW, int E>
__device__ __forceinline__ void mark_cumulate_successor(const MergeArgs& a, StateLds<NW, E>& S, int e) {
    const WinDesc& w = a.win;
    const int64_t k = S.key[e];
    const int64_t we = S.slice[e];
    const int64_t last = wadd(window_start_of(w, we), w.size);
    for (int64_t s = we; s != last;) {
        s = wadd(s, w.interval);
        if (!is_fired(s, a.wm)) break;
        const int e2 = find_entry(S, k, s);
        if (e2 >= 0 && (S.flag[e2] & F_TIMER)) {
            atomicOr(&S.flag[e2], F_NOTHEAD);
            break;
        }
    }
}

// diagnostic phase stamps (FW_ABLATE & AB_STAMPS): lane 0 sums cycles per phase
struct Stamps {
    bool on;
    uint64_t t;
    uint64_t acc[N_STAMPS];
    __device__ void init(bool enable) {
        on = enable;
        for (int i = 0; i < N_STAMPS; i++) acc[i] = 0;
        if (on) t = __builtin_amdgcn_s_memtime();
    }
    __device__ void mark(int phase) {  // call right after a __syncthreads()
        if (!on) return;
        const uint64_t n = __builtin_amdgcn_s_memtime();
        acc[phase] += n - t;
        t = n;
    }
    __device__ void flush(unsigned long long* dst) {
        if (!on || threadIdx.x != 0 || !dst) return;
        for (int i = 0; i < N_STAMPS; i++)
            if (acc[i]) atomicAdd(&dst[i], (unsigned long long)acc[i]);
    }
};

// XCD-aware superbucket order: blocks b, b+8, b+16, ... are dealt to one XCD (round robin,
// speed only), so they get consecutive superbuckets, whose cells sit next to each other in
// every chunk region -> the boundary lines two cells share are read from the same L2.
__device__ __forceinline__ int sb_of_block(int b, int n_sb) {
    if (n_sb % 8 != 0) return b;
    return (b % 8) * (n_sb / 8) + b / 8;
}

// the last workgroup of a k_merge_fire launch applies the launch's control decisions (every
// workgroup read the old values at its start): advanceProgress bookkeeping of the processor
// (AbstractSliceSyncStateWindowAggProcessor.java:139-153), the buffer reset after a flush, the
// consumed timer requests, and the overflow-counter switch of a result reset.
__device__ void merge_finalize(const MergeArgs& a) {
    Ctrl* c = a.ctrl;
    const int64_t W = a.wm;
    const int64_t cur = c->cur, pend = c->pending_pushes, ntp = c->ntp;
    const bool adv = !a.force_flush && W > cur;
    const bool do_flush = pend > 0 && (a.force_flush || (adv && (a.always_flush || (W >= ntp && is_fired(c->min_pending, W)))));
    if (adv) {
        c->cur = W;
        if (W >= ntp) c->ntp = next_trigger_watermark(W, a.win.slice_div);
    }
    if (do_flush) {
        c->pending_pushes = 0;
        c->min_pending = INT64_MAX;
        c->pending_rows = 0;
    }
    c->n_treq = 0;
    const int sel = (c->ovf_sel ^ a.reset_out) & 1;
    c->ovf_sel = sel;
    __hip_atomic_store(&c->out_count[sel ^ 1], 0ull, __ATOMIC_RELAXED, DEV_SCOPE);
}

__device__ __forceinline__ void merge_ticket(const MergeArgs& a) {
    if (threadIdx.x != 0) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (grid_last_wg(a.tickets->c[1])) merge_finalize(a);
}

// rows of one cell loaded together in the gather (VGPR budget of the 1024-thread workgroup)
constexpr int mg_rows_in_flight(int nw) { return nw <= 1 ? 4 : nw <= 2 ? 3 : nw <= 4 ? 2 : 1; }

template <int NW, int E, bool Q, int KIND>
__global__ __launch_bounds__(MG_BLOCK) void k_merge_fire(MergeArgs a) {
    constexpr int PW = 2 + NW;
    constexpr int PWE = 3 + NW;
    const int64_t CH = a.chunk_rows;  // chunk rows of the ingest kernel that wrote the cells
    constexpr int GU = mg_rows_in_flight(NW);
    __shared__ StateLds<NW, E> S;
    __shared__ int32_t s_work;
    __shared__ int32_t s_nlive;
    __shared__ int64_t s_newmin;
    __shared__ uint32_t s_fired;
    __shared__ int32_t s_emit;

    const int tid = threadIdx.x;
    const int sb = sb_of_block(blockIdx.x, a.n_sb);
    Ctrl* c = a.ctrl;
    const int64_t W = a.wm;
    // control decisions; the launch's last workgroup applies them to the control block (merge_finalize)
    const int64_t cur = __hip_atomic_load(&c->cur, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t pend = __hip_atomic_load(&c->pending_pushes, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t ntreq = min(__hip_atomic_load(&c->n_treq, __ATOMIC_RELAXED, DEV_SCOPE), (int64_t)0x7fffffff);
    const int64_t ntp = __hip_atomic_load(&c->ntp, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t minp = __hip_atomic_load(&c->min_pending, __ATOMIC_RELAXED, DEV_SCOPE);
    const bool adv = !a.force_flush && W > cur;
    const bool do_flush = pend > 0 &&
                          (a.force_flush || (adv && (a.always_flush || (W >= ntp && is_fired(minp, W)))));
    const bool do_fire = adv;
    const int64_t w_old = cur;
    const int32_t n0 = a.state_count[sb];

    Stamps stm;
    stm.init((a.ablate & AB_STAMPS) != 0);
    if (tid == 0) {
        s_work = (ntreq > 0) || do_flush || (do_fire && is_fired(a.sb_min_timer[sb], W));
        s_fired = 0;
        s_emit = a.reset_out ? 0 : a.sb_out[sb];
        if (!s_work && a.reset_out) a.sb_out[sb] = 0;
    }
    __syncthreads();
    if (!s_work) {
        merge_ticket(a);
        return;
    }
    const bool gather = do_flush && !(a.ablate & AB_M_NO_GATHER);
    // this thread's first cell word, loaded while the state loads (the gather below walks the
    // cells of every pending push, one cell per thread per pass, in flat tile order f:
    // cell_chunk(f) is the chunk, positions past the push's last chunk are padding)
    auto cell_at = [&](int64_t pi, int f) -> uint32_t {
        if (cell_chunk(f) >= a.slot_nch[pi]) return 0u;
        const uint32_t* cl = a.cells + (size_t)pi * a.n_sb * a.max_nch;
        return cl[((size_t)(f >> 4) * a.n_sb + sb) * CELL_LANES + (f & 15)];
    };
    // the gather splits a push's cells into groups of gather_group(ncell) <= 64 consecutive
    // cells, one group per wave per pass (16 groups when a push has <= 1024 cells)
    const int lane = tid & 63, wv = tid >> 6;
    auto gather_group = [](int ncell) { return min(64, ncell / (MG_BLOCK / 64)); };
    uint32_t v_first = 0;
    if (gather && lane < gather_group((int)cell_pad(a.slot_nch[0])))
        v_first = cell_at(0, wv * gather_group((int)cell_pad(a.slot_nch[0])) + lane);
    // ---- load this superbucket's entries into LDS
    for (int i = tid; i < 2 * E; i += MG_BLOCK) S.idx[i] = 0;
    if (tid == 0) {
        S.n = (a.ablate & AB_M_NO_LOAD) ? 0 : n0;
        S.overflow = 0;
        S.ndue = 0;
    }
    __syncthreads();
    const uint64_t* st = a.state + (size_t)sb * a.cap_e * PWE;
    if (!(a.ablate & AB_M_NO_LOAD)) for (int e = tid; e < n0; e += MG_BLOCK) {
        const uint64_t* p = st + (size_t)e * PWE;
        const int64_t k = (int64_t)p[0], s = (int64_t)p[1];
        S.key[e] = k;
        S.slice[e] = s;
        S.flag[e] = (uint32_t)p[2];
#pragma unroll
        for (int w = 0; w < NW; w++) S.acc[w][e] = p[3 + w];
        uint32_t h = index_hash(k, s) & (2 * E - 1);
        for (;;) {
            uint32_t expect = 0;
            if (__hip_atomic_compare_exchange_strong(&S.idx[h], &expect, 2u + (uint32_t)e, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, LDS_SCOPE))
                break;
            h = (h + 1) & (2 * E - 1);
        }
    }
    __syncthreads();
    stm.mark(0);
    // ---- timers registered by late records in processElement
    for (int64_t r = tid; r < ntreq; r += MG_BLOCK) {
        if (a.treq[3 * r + 2] != sb) continue;
        const int e = find_or_insert(S, a.treq[3 * r], a.treq[3 * r + 1], a.wd);
        if (e >= 0) atomicOr(&S.flag[e], F_TIMER);
    }
    // ---- flush: AggCombiner.combine for every pending (key, slice) partial of this bucket.
    // A wave takes a group of cells (the rows ingest chunks wrote for this superbucket), scans
    // their row counts and deals the rows of the whole group over its 64 lanes, GU rows per lane
    // per pass: every lane is busy whatever the cells' sizes, and neighbouring lanes load
    // neighbouring rows.  Rows are looked up in the LDS table (first probes batched), hits
    // folded; the misses of a lane are then inserted one at a time.
    // diagnostic (AB_GSTAMPS): thread 0's cycles in row loads / first probes / fold + insert
    const bool gst = (a.ablate & AB_GSTAMPS) && stm.on && tid == 0;
    if (gather) {
        for (int64_t pi = 0; pi < pend; pi++) {
            const int ncell = (int)cell_pad(a.slot_nch[pi]);
            const int G = gather_group(ncell);
            const int ngroups = ncell / G;
            const uint64_t* seg = a.parts + (size_t)pi * a.cap_rows * PW;
            for (int g = wv; g < ngroups; g += MG_BLOCK / 64) {
                const int f = g * G + lane;
                const uint32_t v = lane >= G ? 0u : (pi == 0 && g == wv) ? v_first : cell_at(pi, f);
                const uint32_t cnt = v >> 16;
                uint32_t inc = cnt;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t t = (uint32_t)__shfl_up((int)inc, d, 64);
                    if (lane >= d) inc += t;
                }
                const uint32_t tot = (uint32_t)__shfl((int)inc, 63, 64);
                const uint32_t excl = inc - cnt;
                // segment row of this cell's first row, less the rows of the group before it
                const uint32_t adj = (uint32_t)(cell_chunk(f) * CH + (v & 0xFFFFu)) - excl;
                for (uint32_t r0 = 0; r0 < tot; r0 += 64 * GU) {
                    uint64_t row[GU][PW];
                    uint64_t g0 = gst ? __builtin_amdgcn_s_memtime() : 0;
#pragma unroll
                    for (int u = 0; u < GU; u++) {
                        // the group's row x lives in the last cell whose first row is <= x
                        const uint32_t x = min(r0 + (uint32_t)(u * 64 + lane), tot - 1);
                        int lo = 0;
#pragma unroll
                        for (int step = 32; step > 0; step >>= 1)
                            if ((uint32_t)__shfl((int)excl, lo + step, 64) <= x) lo += step;
                        const uint64_t* p = seg + (size_t)((uint32_t)__shfl((int)adj, lo, 64) + x) * PW;
#pragma unroll
                        for (int w = 0; w < PW; w++) row[u][w] = p[w];
                    }
                    if (gst) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        const uint64_t g1 = __builtin_amdgcn_s_memtime();
                        stm.acc[2] += g1 - g0;
                        g0 = g1;
                    }
                    if (a.ablate & AB_M_NO_HASH) {  // diagnostic: loads only
                        uint64_t x = 0;
#pragma unroll
                        for (int u = 0; u < GU; u++) x ^= row[u][0] ^ row[u][1] ^ row[u][PW - 1];
                        asm volatile("" ::"v"(x));  // keeps the loads
                        continue;
                    }
                    int ge[GU];
                    {
                        int64_t gk[GU], gs[GU];
#pragma unroll
                        for (int u = 0; u < GU; u++) {
                            gk[u] = (int64_t)row[u][0];
                            gs[u] = (int64_t)row[u][1];
                        }
                        probe_batch<NW, E, GU>(S, gk, gs, ge);
                    }
                    if (gst) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        const uint64_t g1 = __builtin_amdgcn_s_memtime();
                        stm.acc[4] += g1 - g0;
                        g0 = g1;
                    }
                    // register the window timer unless already fired (AggCombiner.java:103-110);
                    // the LOCAL phase keeps no timers (LocalAggCombiner.java:69-97)
                    auto flags_of = [&](int64_t sl) -> uint32_t {
                        return (a.local || is_fired(sl, w_old)) ? F_ACC : (F_ACC | F_TIMER);
                    };
                    uint32_t miss = 0;
                    static_for<GU>([&](auto UU) {
                        constexpr int u = decltype(UU)::value;
                        if (r0 + (uint32_t)(u * 64 + lane) >= tot) return;
                        const int e = ge[u];  // -1 / -2: not found by the batched first probe
                        if (e < 0) {
                            miss |= 1u << u;
                            return;
                        }
                        if (a.ablate & AB_M_NO_FOLDOP) return;
#pragma unroll
                        for (int w = 0; w < NW; w++)
                            if (w < a.wd.nw) lds_fold(a.wd.op[w], &S.acc[w][e], row[u][2 + w]);
                        atomicOr(&S.flag[e], flags_of((int64_t)row[u][1]));
                    });
                    while (miss) {  // the wave loops max(popcount) times, not GU times
                        const int um = __ffs(miss) - 1;
                        miss &= miss - 1;
                        uint64_t r[PW];
                        static_for<GU>([&](auto UU) {
                            constexpr int u = decltype(UU)::value;
                            if (u == um) {
#pragma unroll
                                for (int w = 0; w < PW; w++) r[w] = row[u][w];
                            }
                        });
                        const int64_t k = (int64_t)r[0], sl = (int64_t)r[1];
                        const uint32_t fl = flags_of(sl);
                        bool ins = false;
                        const int e = find_or_insert(S, k, sl, a.wd, &r[2], fl, &ins);
                        if (e < 0 || ins || (a.ablate & AB_M_NO_FOLDOP)) continue;
#pragma unroll
                        for (int w = 0; w < NW; w++)
                            if (w < a.wd.nw) lds_fold(a.wd.op[w], &S.acc[w][e], r[2 + w]);
                        atomicOr(&S.flag[e], fl);
                    }
                    if (gst) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        stm.acc[7] += __builtin_amdgcn_s_memtime() - g0;
                    }
                }
            }
        }
    }
    __syncthreads();
    stm.mark(1);
    // ---- fire: InternalTimerServiceImpl.tryAdvanceWatermark (:328-348) -> WindowAggOperator
    // .onTimer -> fireWindow + clearWindow.  One pass over the entries whose timer is due; HOP and
    // CUMULATE follow their timer chains per key (no timestamp rounds, see fire_*_chain).
    if (do_fire && !(a.ablate & AB_M_NO_FIRE)) {
        const int n = min(S.n, E);
        for (int e = tid; e < n; e += MG_BLOCK)
            if ((S.flag[e] & F_TIMER) && is_fired(S.slice[e], W)) {
                const int q = wave_claim(&S.ndue);
                if (q < E) S.due[q] = (uint16_t)e;
            }
        __syncthreads();
        const int nd = min(S.ndue, E);
        if (KIND == FW_WIN_CUMULATE) {
            for (int q = tid; q < nd; q += MG_BLOCK) mark_cumulate_successor<NW, E>(a, S, S.due[q]);
            __syncthreads();
        }
        stm.mark(6);
        uint32_t nf = 0;
        for (int q = tid; q < nd; q += MG_BLOCK) {
            const int e = S.due[q];
            if (KIND == FW_WIN_TUMBLE) {
                nf += fire_tumble<NW, E, Q>(a, S, e, sb, &s_emit);
            } else if (KIND == FW_WIN_HOP) {
                nf += fire_hop_chain<NW, E, Q>(a, S, e, sb, &s_emit);
            } else {
                if (!(S.flag[e] & F_NOTHEAD)) nf += fire_cumulate_chain<NW, E, Q>(a, S, e, sb, &s_emit);
            }
        }
        nf = wave_sum_u32(nf);
        if ((tid & 63) == 0 && nf) atomicAdd(&s_fired, nf);
        if (S.ndue > E && tid == 0) S.overflow = 1;
    }
    // ---- write back live entries (LOCAL phase: emit every partial instead, keep no state)
    if (tid == 0) {
        s_nlive = 0;
        s_newmin = INT64_MAX;
    }
    __syncthreads();
    stm.mark(5);
    const int n = min(S.n, E);
    uint64_t* so = a.state + (size_t)sb * a.cap_e * PWE;
    int64_t lnm = INT64_MAX;
    if (a.local) {
        if (gather)
            for (int e = tid; e < n; e += MG_BLOCK) {
                uint64_t v[NW];
#pragma unroll
                for (int w = 0; w < NW; w++) v[w] = S.acc[w][e];
                emit_partial<NW, Q>(a, sb, &s_emit, S.key[e], S.slice[e], v);
            }
    } else if (!(a.ablate & AB_M_NO_WB)) {
        for (int e = tid; e < n; e += MG_BLOCK) {
            const uint32_t f0 = S.flag[e];
            const uint32_t f = f0 & ((f0 & F_EXPIRE) ? F_TIMER : (F_ACC | F_TIMER));
            if (!f) continue;
            const int pos = wave_claim(&s_nlive);
            uint64_t* p = so + (size_t)pos * PWE;
            p[0] = (uint64_t)S.key[e];
            p[1] = (uint64_t)S.slice[e];
            p[2] = f;
            if (Q) {
                uint64_t v[NW];
#pragma unroll
                for (int w = 0; w < NW; w++) v[w] = S.acc[w][e];
#pragma unroll
                for (int w = 0; w < NW; w++) p[3 + w] = w < a.wd.nw ? q_normalise(a.wd, w, v) : v[w];
            } else {
#pragma unroll
                for (int w = 0; w < NW; w++) p[3 + w] = S.acc[w][e];
            }
            if (f & F_TIMER) lnm = min(lnm, S.slice[e]);
        }
    }
    lnm = wave_min_i64(lnm);
    if ((tid & 63) == 0 && lnm != INT64_MAX) __hip_atomic_fetch_min(&s_newmin, lnm, __ATOMIC_RELAXED, LDS_SCOPE);
    __syncthreads();
    if (tid == 0) {
        a.state_count[sb] = a.local ? 0 : s_nlive;
        a.sb_min_timer[sb] = s_newmin;
        a.sb_out[sb] = min(s_emit, a.slab_cap);
        if (s_fired) a.sb_fired[sb] += s_fired;
        if (S.overflow) __hip_atomic_fetch_or(&c->error, ERR_STATE, __ATOMIC_RELAXED, DEV_SCOPE);
    }
    __syncthreads();
    stm.mark(3);
    stm.flush(a.stamps);
    merge_ticket(a);
}

__global__ void k_init_ctrl(Ctrl* c) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        c->cur = INT64_MIN;
        c->ntp = INT64_MIN;
        c->min_pending = INT64_MAX;
        c->pending_pushes = 0;
        c->push_slot = 0;
        c->n_treq = 0;
        c->out_count[0] = 0;
        c->out_count[1] = 0;
        c->ovf_sel = 0;
        c->late_dropped = 0;
        c->fired = 0;
        c->pending_rows = 0;
        c->live_entries = 0;
        c->error = 0;
        c->partials = 0;
    }
}

hipError_t launch_compact(const CompactArgs& a, hipStream_t s, KTimer* t) {
    kt_mark(t, FW_KT_OTHER, false, s);
    hipLaunchKernelGGL(k_compact_scan, dim3(1), dim3(BLOCK), 0, s, a.sb_out, a.n_sb, a.off, a.ctrl, a.res_cap);
    hipLaunchKernelGGL(k_compact_copy, dim3(a.n_sb + 1), dim3(BLOCK), 0, s, a);
    kt_mark(t, FW_KT_OTHER, true, s);
    return hipGetLastError();
}

hipError_t launch_init_ctrl(Ctrl* c, hipStream_t s) {
    hipLaunchKernelGGL(k_init_ctrl, dim3(1), dim3(64), 0, s, c);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// template dispatch
// ---------------------------------------------------------------------------------------
template <int NV, int NW, bool X>
static hipError_t ingest_x(const IngestArgs& a, hipStream_t s, KTimer* t) {
    constexpr int RPT = ig_rpt(NW, NV);
    const int64_t nch = a.n_chunks;
    if (nch == 0) return hipSuccess;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)k_ingest<NV, NW, RPT, X>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, IG_LDS);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    // the fold table and the histogram must fit the dynamic LDS
    if ((int64_t)(IG_HDR_WORDS + ig_hist_words(a.ks.n_sb)) * 8 + ig_fold_bytes(NW) > a.lds_bytes) return hipErrorInvalidValue;
    kt_mark(t, FW_KT_REDUCE, false, s);
    hipLaunchKernelGGL((k_ingest<NV, NW, RPT, X>), dim3((unsigned)nch), dim3(IG_BLOCK), a.lds_bytes, s, a);
    kt_mark(t, FW_KT_REDUCE, true, s);
    return hipGetLastError();
}

template <int NV, int NW>
static hipError_t ingest_nw(const IngestArgs& a, hipStream_t s, KTimer* t) {
    bool x = a.wd.has_q != 0;
    for (int q = 0; q < MAX_KCOLS; q++) x = x || a.nulls[q] != nullptr;
    return x ? ingest_x<NV, NW, true>(a, s, t) : ingest_x<NV, NW, false>(a, s, t);
}

template <int NV>
static hipError_t ingest_nv(const IngestArgs& a, hipStream_t s, KTimer* t) {
    const int nw = a.wd.nw;
    if (nw <= 1) return ingest_nw<NV, 1>(a, s, t);
    if (nw <= 2) return ingest_nw<NV, 2>(a, s, t);
    if (nw <= 4) return ingest_nw<NV, 4>(a, s, t);
    return ingest_nw<NV, 8>(a, s, t);
}

hipError_t launch_ingest(const IngestArgs& a, hipStream_t s, KTimer* t) {
    switch (ig_nv(a.nv)) {
        case 0: return ingest_nv<0>(a, s, t);
        case 1: return ingest_nv<1>(a, s, t);
        case 2: return ingest_nv<2>(a, s, t);
        case 4: return ingest_nv<4>(a, s, t);
        default: return ingest_nv<8>(a, s, t);
    }
}

template <int NW, bool Q>
static hipError_t merge_q(const MergeArgs& a, hipStream_t s) {
    constexpr int E = mg_entries(NW);
    switch (a.win.kind) {
        case FW_WIN_TUMBLE: hipLaunchKernelGGL((k_merge_fire<NW, E, Q, FW_WIN_TUMBLE>), dim3(a.n_sb), dim3(MG_BLOCK), 0, s, a); break;
        case FW_WIN_HOP: hipLaunchKernelGGL((k_merge_fire<NW, E, Q, FW_WIN_HOP>), dim3(a.n_sb), dim3(MG_BLOCK), 0, s, a); break;
        default: hipLaunchKernelGGL((k_merge_fire<NW, E, Q, FW_WIN_CUMULATE>), dim3(a.n_sb), dim3(MG_BLOCK), 0, s, a); break;
    }
    return hipGetLastError();
}

template <int NW>
static hipError_t merge_nw(const MergeArgs& a, hipStream_t s) {
    return a.wd.has_q ? merge_q<NW, true>(a, s) : merge_q<NW, false>(a, s);
}

static hipError_t merge_any(const MergeArgs& a, hipStream_t s) {
    const int nw = a.wd.nw;
    if (nw <= 1) return merge_nw<1>(a, s);
    if (nw <= 2) return merge_nw<2>(a, s);
    if (nw <= 4) return merge_nw<4>(a, s);
    return merge_nw<8>(a, s);
}

hipError_t launch_merge_fire(const MergeArgs& a, hipStream_t s, KTimer* t) {
    kt_mark(t, FW_KT_MERGE, false, s);
    hipError_t e = merge_any(a, s);
    kt_mark(t, FW_KT_MERGE, true, s);
    return e;
}

// ======================================================================================
// stand-alone kernels: key groups, exchange partitioning, synthetic generator
// ======================================================================================
__global__ void k_key_groups(const int64_t* key, const int32_t* kh, int64_t n, int32_t kind, int32_t max_p,
                             int32_t p, int32_t* kg, int32_t* dest) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t g = key_group_for_hash(java_key_hash(kind, key[i], kh ? kh[i] : 0), max_p);
    if (kg) kg[i] = g;
    if (dest) dest[i] = operator_for_key_group(max_p, p, g);
}

constexpr int PART_TILE = 4096;
constexpr int PART_MAXP = 64;

__global__ __launch_bounds__(BLOCK) void k_part_hist(const int64_t* key, const int32_t* kh, int64_t n, int32_t kind,
                                                     int32_t max_p, int32_t p, uint32_t* counts) {
    __shared__ uint32_t h[PART_MAXP];
    const int tid = threadIdx.x;
    if (tid < PART_MAXP) h[tid] = 0;
    __syncthreads();
    const int64_t b = (int64_t)blockIdx.x * PART_TILE;
    for (int j = tid; j < PART_TILE; j += BLOCK) {
        const int64_t i = b + j;
        if (i >= n) break;
        const int32_t g = key_group_for_hash(java_key_hash(kind, key[i], kh ? kh[i] : 0), max_p);
        atomicAdd(&h[operator_for_key_group(max_p, p, g)], 1u);
    }
    __syncthreads();
    if (tid < p) counts[(size_t)blockIdx.x * p + tid] = h[tid];
}

// one block: offsets[blk][d] = sum_{d'<d} total(d') + sum_{b'<blk} counts[b'][d]
__global__ __launch_bounds__(BLOCK) void k_part_scan(uint32_t* counts, int64_t nblk, int32_t p, int64_t* totals) {
    __shared__ uint64_t tot[PART_MAXP];
    const int tid = threadIdx.x;
    if (tid < p) {
        uint64_t s = 0;
        for (int64_t b = 0; b < nblk; b++) s += counts[b * p + tid];
        tot[tid] = s;
    }
    __syncthreads();
    if (tid < p) {
        uint64_t base = 0;
        for (int d = 0; d < tid; d++) base += tot[d];
        uint64_t run = base;
        for (int64_t b = 0; b < nblk; b++) {
            const uint32_t v = counts[b * p + tid];
            counts[b * p + tid] = (uint32_t)run;  // fits: n < 2^32 per call
            run += v;
        }
        totals[tid] = (int64_t)tot[tid];
    }
}

__global__ __launch_bounds__(BLOCK) void k_part_scatter(const int64_t* key, const int32_t* kh, const int64_t* ts,
                                                        const uint64_t* const* vals,
                                                        int32_t ncols, int64_t n, int32_t kind, int32_t max_p,
                                                        int32_t p, const uint32_t* offsets, int64_t* okey, int64_t* ots,
                                                        uint64_t* const* ovals) {
    // Stable: rows keep their input order within a destination (the order a Netty channel
    // delivers them in, ChannelSelectorRecordWriter.emit :54), so a DOUBLE SUM downstream adds in
    // the same order on every run.  Each wave ranks its 64 rows per destination with ballots;
    // the waves of one pass are ordered through a per-wave count table.
    constexpr int NWV = BLOCK / 64;
    __shared__ uint32_t h[PART_MAXP];         // next output position per destination
    __shared__ uint32_t wc[NWV][PART_MAXP];   // rows per (wave, destination) of the current pass
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid < p) h[tid] = offsets[(size_t)blockIdx.x * p + tid];
    const uint64_t lt = (1ull << lane) - 1ull;
    const int64_t b = (int64_t)blockIdx.x * PART_TILE;
    for (int j0 = 0; j0 < PART_TILE; j0 += BLOCK) {
        const int64_t i = b + j0 + tid;
        int32_t d = -1;
        int64_t k = 0;
        if (i < n) {
            k = key[i];
            d = operator_for_key_group(max_p, p, key_group_for_hash(java_key_hash(kind, k, kh ? kh[i] : 0), max_p));
        }
        uint32_t rank = 0;
        for (int dd = 0; dd < p; dd++) {
            const uint64_t m = __ballot(d == dd);
            if (d == dd) rank = (uint32_t)__popcll(m & lt);
            if (lane == 0) wc[w][dd] = (uint32_t)__popcll(m);
        }
        __syncthreads();  // wc of every wave and h of the previous pass are visible
        uint32_t pos = 0;
        if (d >= 0) {
            pos = h[d] + rank;
            for (int v = 0; v < w; v++) pos += wc[v][d];
        }
        __syncthreads();  // every lane has read h
        if (tid < p) {
            uint32_t t = 0;
            for (int v = 0; v < NWV; v++) t += wc[v][tid];
            h[tid] += t;
        }
        if (d >= 0) {
            okey[pos] = k;
            ots[pos] = ts[i];
            for (int c = 0; c < ncols; c++) ovals[c][pos] = vals[c][i];
        }
        __syncthreads();  // h updated before the next pass reads it; wc free to overwrite
    }
}

__global__ void k_key_row_hash(KeyRowDesc d, int64_t n, int32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = key_row_hash(d, i);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) { return mix64(x + 0x9E3779B97F4A7C15ull); }

__global__ void k_generate(fw_gen_params gp, int64_t i0, int64_t n, int64_t* key, int64_t* ts, int64_t* val) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t i = (uint64_t)(i0 + j);
    const uint64_t u = splitmix64(gp.seed ^ (i * 0x9E3779B97F4A7C15ull));
    const int64_t t = gp.t0_ms + (int64_t)i * 1000 / gp.rate_per_s - (int64_t)(u % (uint64_t)gp.ooo_ms);
    int64_t k;
    if (gp.key_dist == 0) {
        k = gp.key_base + (int64_t)((u >> 20) % (uint64_t)gp.key_count);
    } else {
        const double x = (double)(u >> 11) * (1.0 / 9007199254740992.0);
        int64_t lo = 0, hi = gp.key_count - 1;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (gp.zipf_cdf[mid] > x) hi = mid; else lo = mid + 1;
        }
        k = gp.key_base + lo;
    }
    uint64_t v;
    if (gp.value_kind == 0) v = 1 + u % 1000000000ull;
    else if (gp.value_kind == 1) v = f64_bits(1000.0 * (double)(u >> 11) * (1.0 / 9007199254740992.0));
    else v = u % 1000000ull;
    if (key) key[j] = k;
    if (ts) ts[j] = t;
    if (val) val[j] = (int64_t)v;
}

}  // namespace fw

// ======================================================================================
// C-ABI wrappers for the stand-alone kernels
// ======================================================================================
using namespace fw;

extern "C" int fw_assign_key_groups(const int64_t* d_key, const int32_t* d_key_hash, int64_t n, int32_t key_hash_kind,
                                    int32_t max_parallelism, int32_t parallelism, int32_t* d_kg, int32_t* d_dest,
                                    void* stream) {
    if (n <= 0) return FW_OK;
    if (!d_key || max_parallelism <= 0 || parallelism <= 0) return FW_E_INVALID;
    hipLaunchKernelGGL(k_key_groups, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_key,
                       d_key_hash, n, key_hash_kind, max_parallelism, parallelism, d_kg, d_dest);
    return hipGetLastError() == hipSuccess ? FW_OK : FW_E_DEVICE;
}

// fw_key_field[] -> KeyRowDesc (FW_E_INVALID on a bad description)
static int key_row_desc(const fw_key_field* fields, int32_t n_fields, KeyRowDesc* d) {
    if (!fields || n_fields <= 0 || n_fields > FW_MAX_KEY_FIELDS || n_fields > KR_MAX_FIELDS) return FW_E_INVALID;
    *d = KeyRowDesc{};
    d->n = n_fields;
    for (int f = 0; f < n_fields; f++) {
        const fw_key_field& k = fields[f];
        if (k.kind != FW_KF_STRING && k.kind != FW_KF_FIXED1 && k.kind != FW_KF_FIXED2 && k.kind != FW_KF_FIXED4 &&
            k.kind != FW_KF_FIXED8)
            return FW_E_INVALID;
        d->width[f] = k.kind;
        if (k.kind == FW_KF_STRING) {
            if (!k.offsets || !k.bytes || ((uintptr_t)k.bytes & 3)) return FW_E_INVALID;
        } else if (!k.fixed) {
            return FW_E_INVALID;
        }
        d->fixed[f] = k.fixed;
        d->offs[f] = k.offsets;
        d->bytes[f] = k.bytes;
        d->nulls[f] = k.nulls;
    }
    return FW_OK;
}

extern "C" int fw_key_row_hash(const fw_key_field* fields, int32_t n_fields, int64_t n, int32_t* d_hash, void* stream) {
    KeyRowDesc d;
    if (const int rc = key_row_desc(fields, n_fields, &d)) return rc;
    if (n <= 0) return FW_OK;
    if (!d_hash) return FW_E_INVALID;
    hipLaunchKernelGGL(k_key_row_hash, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d, n,
                       d_hash);
    return hipGetLastError() == hipSuccess ? FW_OK : FW_E_DEVICE;
}

extern "C" int fw_host_key_row_hash(const fw_key_field* fields, int32_t n_fields, int64_t n, int32_t* hash) {
    KeyRowDesc d;
    if (const int rc = key_row_desc(fields, n_fields, &d)) return rc;
    if (n > 0 && !hash) return FW_E_INVALID;
    for (int64_t i = 0; i < n; i++) hash[i] = key_row_hash(d, i);
    return FW_OK;
}

extern "C" int64_t fw_partition_workspace_bytes(int64_t n, int32_t parallelism) {
    const int64_t nblk = (n + PART_TILE - 1) / PART_TILE;
    return (nblk * parallelism * 4 + 2 * FW_MAX_COLS * 8 + 255) & ~255ll;
}

extern "C" int fw_partition_by_dest(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                                    const void* const* d_values, int32_t n_cols, int64_t n, int32_t key_hash_kind,
                                    int32_t max_parallelism, int32_t parallelism, int64_t* d_out_key,
                                    int64_t* d_out_ts, void* const* d_out_values, int64_t* d_counts,
                                    void* d_workspace, int64_t workspace_bytes, void* stream) {
    if (parallelism <= 0 || parallelism > PART_MAXP || n_cols < 0 || n_cols > FW_MAX_COLS) return FW_E_INVALID;
    if (key_hash_kind == FW_KEYHASH_PRECOMPUTED && n > 0 && !d_key_hash) return FW_E_INVALID;
    if (key_hash_kind != FW_KEYHASH_PRECOMPUTED) d_key_hash = nullptr;
    if (workspace_bytes < fw_partition_workspace_bytes(n, parallelism)) return FW_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    if (n <= 0) {
        return hipMemsetAsync(d_counts, 0, sizeof(int64_t) * parallelism, s) == hipSuccess ? FW_OK : FW_E_DEVICE;
    }
    const int64_t nblk = (n + PART_TILE - 1) / PART_TILE;
    uint32_t* counts = (uint32_t*)d_workspace;
    // value-column pointer arrays live in the workspace tail (device-visible)
    const uint64_t** dv = (const uint64_t**)((char*)d_workspace + nblk * parallelism * 4);
    dv = (const uint64_t**)(((uintptr_t)dv + 15) & ~(uintptr_t)15);
    uint64_t** dov = (uint64_t**)(dv + FW_MAX_COLS);
    const void* hv[2 * FW_MAX_COLS] = {nullptr};
    for (int c = 0; c < n_cols; c++) {
        hv[c] = d_values[c];
        hv[FW_MAX_COLS + c] = d_out_values[c];
    }
    if (hipMemcpyAsync(dv, hv, sizeof(hv), hipMemcpyHostToDevice, s) != hipSuccess) return FW_E_DEVICE;
    hipLaunchKernelGGL(k_part_hist, dim3((unsigned)nblk), dim3(BLOCK), 0, s, d_key, d_key_hash, n, key_hash_kind,
                       max_parallelism, parallelism, counts);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(BLOCK), 0, s, counts, nblk, parallelism, d_counts);
    hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)nblk), dim3(BLOCK), 0, s, d_key, d_key_hash, d_ts,
                       (const uint64_t* const*)dv, n_cols, n, key_hash_kind, max_parallelism, parallelism, counts,
                       d_out_key, d_out_ts, (uint64_t* const*)dov);
    return hipGetLastError() == hipSuccess ? FW_OK : FW_E_DEVICE;
}

extern "C" int fw_generate(const fw_gen_params* gp, int64_t i0, int64_t n, int64_t* d_key, int64_t* d_ts,
                           int64_t* d_value, void* stream) {
    if (!gp || gp->rate_per_s <= 0 || gp->ooo_ms <= 0 || gp->key_count <= 0) return FW_E_INVALID;
    if (gp->key_dist == 1 && !gp->zipf_cdf) return FW_E_INVALID;
    if (n <= 0) return FW_OK;
    hipLaunchKernelGGL(k_generate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *gp, i0, n,
                       d_key, d_ts, d_value);
    return hipGetLastError() == hipSuccess ? FW_OK : FW_E_DEVICE;
}
