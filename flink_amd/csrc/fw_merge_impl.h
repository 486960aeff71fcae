// fw_merge_impl.h -- k_merge_fire (K4+K5) and its launchers, instantiated per accumulator word
// count in k_merge_nw*.hip.
#pragma once
#include <type_traits>

#include "fw_kernel_common.h"

namespace fw {
// ======================================================================================
// K4+K5: merge pending partials into the HBM slice-state table, fire due timers
// ======================================================================================
template <int NW, int E>
struct StateLds {
    static constexpr int NI = mg_idx_slots(NW, E);  // 4E slots where they fit (mg_idx_slots)
    uint32_t idx[NI];      // open-addressing index: 0 empty, 1 claiming, 2+e entry e
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

// W consecutive 8-byte words at p with 16-byte accesses: a partial row or state entry is one
// lane's scattered record, so every load instruction touches up to 64 cache lines -- halving the
// instruction count halves that traffic through the texture path.  Even W: p is 16-B aligned (an
// even word offset from an aligned base).  Odd W: the lane's parity picks where the lone 8-byte
// word sits; every lane runs the same instructions.
template <int W>
__device__ __forceinline__ void load_words(const uint64_t* p, uint64_t (&o)[W]) {
    if constexpr (W % 2 == 0) {
#pragma unroll
        for (int k = 0; k < W / 2; k++) {
            const ulonglong2 v = *(const ulonglong2*)(p + 2 * k);
            o[2 * k] = v.x;
            o[2 * k + 1] = v.y;
        }
    } else {
        const bool odd = ((uintptr_t)p & 8) != 0;
        const uint64_t one = *(odd ? p : p + (W - 1));
        const uint64_t* q = p + (odd ? 1 : 0);
        uint64_t pr[W - 1 > 0 ? W - 1 : 1];
#pragma unroll
        for (int k = 0; k < (W - 1) / 2; k++) {
            const ulonglong2 v = *(const ulonglong2*)(q + 2 * k);
            pr[2 * k] = v.x;
            pr[2 * k + 1] = v.y;
        }
        if constexpr (W == 1) {
            o[0] = one;
        } else {
            o[0] = odd ? one : pr[0];
#pragma unroll
            for (int w = 1; w < W - 1; w++) o[w] = odd ? pr[w - 1] : pr[w];
            o[W - 1] = odd ? pr[W - 2] : one;
        }
    }
}
template <int W>
__device__ __forceinline__ void store_words(uint64_t* p, const uint64_t (&v)[W]) {
    if constexpr (W % 2 == 0) {
#pragma unroll
        for (int k = 0; k < W / 2; k++) st16(p + 2 * k, v[2 * k], v[2 * k + 1]);
    } else {
        const bool odd = ((uintptr_t)p & 8) != 0;
        st8(odd ? p : p + (W - 1), odd ? v[0] : v[W - 1]);
        uint64_t* q = p + (odd ? 1 : 0);
#pragma unroll
        for (int k = 0; k < (W - 1) / 2; k++) st16(q + 2 * k, odd ? v[2 * k + 1] : v[2 * k], odd ? v[2 * k + 2] : v[2 * k + 1]);
    }
}

// LDS publication protocol of the index: the inserting lane writes the entry's fields, then
// (after a compiler barrier) the index word with a relaxed store.  LDS executes one wave's
// requests in issue order and a reader's field loads depend on the index value it read, so a
// reader that sees 2+e sees the fields.  Acquire/release orderings are not used: at workgroup
// scope they also order global memory, making every publish wait for earlier result stores.
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

template <int NW, int E>
__device__ int find_entry(StateLds<NW, E>& S, int64_t k, int64_t s) {
    constexpr uint32_t MASK = StateLds<NW, E>::NI - 1;
    uint32_t h = index_hash(k, s) & MASK;
    for (int probes = 0; probes < StateLds<NW, E>::NI;) {
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
template <int NW, int E, uint32_t OPS = OPS_ANY>
__device__ __forceinline__ int find_or_insert(StateLds<NW, E>& S, int64_t k, int64_t s, const WordDesc& wd,
                              const uint64_t* v = nullptr, uint32_t flag0 = 0, bool* inserted = nullptr) {
    constexpr uint32_t MASK = StateLds<NW, E>::NI - 1;
    uint32_t h = index_hash(k, s) & MASK;
    for (int probes = 0; probes < StateLds<NW, E>::NI;) {
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
                    S.acc[w][e] = word_on<OPS>(wd, w) ? (v ? reg_fold(word_op<OPS>(wd, w), word_identity(word_op<OPS>(wd, w)), v[w])
                                                           : word_identity(word_op<OPS>(wd, w)))
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
                                            int m = M, uint32_t want = ~0u) {
    // only the first m (<= M, uniform) lookups, and of those the ones set in `want`, are needed;
    // the others issue no LDS reads (and come back -1)
    constexpr uint32_t MASK = StateLds<NW, E>::NI - 1;
    uint32_t st[M];
#pragma unroll
    for (int j = 0; j < M; j++)
        st[j] = j < m && ((want >> j) & 1u) ? __hip_atomic_load(&S.idx[index_hash(k[j], s[j]) & MASK], __ATOMIC_RELAXED, LDS_SCOPE) : 0u;
    int64_t kk[M], ss[M];
#pragma unroll
    for (int j = 0; j < M; j++) {
        kk[j] = 0;
        ss[j] = 0;
        if (j >= m || !((want >> j) & 1u)) continue;
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

// Inserts of the rows whose home slot was empty at the first probe (ge[u] == -1, bit u of
// `miss`), batched over the wave: each lane claims its rows' home slots (empty -> 1, in insertion)
// with back-to-back compare-and-swaps, one LDS add reserves the wave's entries for the claims it
// won, and each lane writes its entries and publishes them (1 -> 2 + e) -- three LDS round trips
// for the whole batch instead of a probe / claim / allocate / publish chain per row.  Lost claims
// (another lane took the slot, possibly for the same (key, slice)) take the probing path, which
// waits out slots in insertion; every slot this wave claimed is published before it returns.
template <int NW, int E, int GX, uint32_t OPS, typename Row, typename FlagsOf>
__device__ __forceinline__ uint32_t insert_fresh(StateLds<NW, E>& S, const WordDesc& wd, const Row& row, uint32_t miss,
                                                 const int* ge, const FlagsOf& flags_of) {
    constexpr uint32_t MASK = StateLds<NW, E>::NI - 1;
    uint32_t hs[GX];
    uint32_t won = 0;
#pragma unroll
    for (int u = 0; u < GX; u++) {
        hs[u] = index_hash((int64_t)row[u][0], (int64_t)row[u][1]) & MASK;
        if (!(((miss >> u) & 1u) && ge[u] == -1)) continue;
        uint32_t expect = 0;
        if (__hip_atomic_compare_exchange_strong(&S.idx[hs[u]], &expect, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED, LDS_SCOPE))
            won |= 1u << u;
    }
    uint64_t bal[GX];
    int total = 0;
#pragma unroll
    for (int u = 0; u < GX; u++) {
        bal[u] = __ballot((won >> u) & 1u);
        total += __popcll(bal[u]);
    }
    if (total == 0) return miss;
    const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
    int base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(&S.n, total);
    base = __shfl(base, leader, 64);
    int en[GX];
    int pre = 0;
#pragma unroll
    for (int u = 0; u < GX; u++) {
        const uint64_t b = bal[u];
        en[u] = base + pre + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        pre += __popcll(b);
    }
#pragma unroll
    for (int u = 0; u < GX; u++) {
        if (!((won >> u) & 1u)) continue;
        const int e = en[u];
        if (e >= E) continue;
        S.key[e] = (int64_t)row[u][0];
        S.slice[e] = (int64_t)row[u][1];
        S.flag[e] = flags_of((int64_t)row[u][1]);
#pragma unroll
        for (int w = 0; w < NW; w++)
            S.acc[w][e] = word_on<OPS>(wd, w) ? reg_fold(word_op<OPS>(wd, w), word_identity(word_op<OPS>(wd, w)), row[u][2 + w]) : 0;
    }
    compiler_fence();
#pragma unroll
    for (int u = 0; u < GX; u++) {
        if (!((won >> u) & 1u)) continue;
        if (en[u] >= E) S.overflow = 1;
        __hip_atomic_store(&S.idx[hs[u]], en[u] < E ? 2u + (uint32_t)en[u] : IDX_DEAD, __ATOMIC_RELAXED, LDS_SCOPE);
    }
    return miss & ~won;
}

// register an event-time timer on entry e; a timer that is already due at this watermark joins
// the due list (an entry's timer fires at most once per advance: its timestamp is its slice end)
template <int NW, int E>
__device__ __forceinline__ void set_timer(StateLds<NW, E>& S, int e, int64_t W, const WinDesc& w) {
    const uint32_t old = atomicOr(&S.flag[e], F_TIMER);
    if (!(old & F_TIMER) && win_fired(w, S.slice[e], W)) {
        const int q = atomicAdd(&S.ndue, 1);
        if (q < E) S.due[q] = (uint16_t)e;
    }
}

// The fire passes deal n items (due entries, HOP block entries) to the 1024 threads in passes of
// 1024, in thread order: the lanes of a wave take consecutive items, and consecutive entries sit in
// consecutive LDS words, so the fire's entry reads are bank-conflict free.  Round 4's lane-major
// dealing (l * 16 + w: every wave busy when fewer items than threads) put a wave's lanes
// 16 entries apart, 32-way conflicts on every 8-byte entry read; measured round 5: thread order
// CFG3 merge 267 -> 248 us, CFG5 317 -> 300, CFG4 196 -> 187, CFG2 131 -> 127 us per flush; blocks
// of consecutive items for every wave landed in between.
__device__ __forceinline__ int fire_deal(int b0, int n, int tid) {
    return b0 + tid;
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
__device__ __forceinline__ void emit_row(const MergeArgs& a, int sb, int32_t* s_emit, int64_t key, int64_t we, const uint64_t* acc) {
    if (FW_ABL(a) & AB_M_NO_EMIT) return;
    const int64_t i = claim_out_row(a, sb, s_emit);
    if (i < 0) return;
    st8(&a.out_key[i], (uint64_t)key);
    // (no window_start column: it is window_start_of(window_end), derived where rows are read)
    st8(&a.out_we[i], (uint64_t)we);
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
            case FW_AGG_MINBY:  // the arg's field: its key decoded (a NaN as the canonical NaN)
            case FW_AGG_MAXBY:
                if (Q && a.ad.qf[g] >= 0) {
                    bool isnull;
                    v = q_result(a.ad, g, acc, &isnull);
                    if (isnull) nm |= 1u << g;
                    break;
                }
                v = type == FW_T_F64 ? dkey_inv((int64_t)w0) : w0;
                // DataStream: a NaN result is the NaN that arrived last, with its own bits
                if (a.ad.dn_hi[g] >= 0 && f64_isnan(v))
                    v = (acc[a.ad.dn_hi[g]] << 32) | (acc[a.ad.dn_lo[g]] & 0xFFFFFFFFull);
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
        st8(&a.out_val[g][i], ((nm >> g) & 1u) ? 0ull : v);  // a NULL's value word is 0
    }
    if (a.ad.first_word >= 0) st8(&a.out_val[a.ad.n][i], acc[a.ad.first_word]);  // value1's arrival ordinal
    a.out_null[i] = nm;
}

// LOCAL phase output (LocalAggCombiner.combine :69-97 -> output(key, window, acc)): one row per
// (key, sliceEnd) of the flush holding the local accumulator fields of every aggregate in order
// (COUNT(*) / COUNT: count; SUM, MIN, MAX: value, NULL-able; AVG: sum, count), window_end =
// sliceEnd (window_start = sliceEnd too, derived by the readers).  The GLOBAL phase ingests exactly these columns.
template <int NW, bool Q>
__device__ __forceinline__ void emit_partial(const MergeArgs& a, int sb, int32_t* s_emit, int64_t key, int64_t se, const uint64_t* acc) {
    const int64_t i = claim_out_row(a, sb, s_emit);
    if (i < 0) return;
    a.out_key[i] = key;
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
constexpr uint32_t F_NOTHEAD = 8u;  // CUMULATE / HOP: an earlier due window's chain reaches this one
constexpr uint32_t F_EXPIRE = 16u;  // HOP: slice expired by a window fired in this advance (cleared at write-back)
constexpr uint32_t F_NEW = 64u;     // DataStream: window state created in this launch (first element retained)

// DataStream first-element events (MergeArgs::ordev), called by the lanes that have one
__device__ __forceinline__ void push_ordev(const MergeArgs& a, int64_t ev) {
    const int64_t r = wave_claim_dev(&a.ctrl->n_ordev);
    if (r < a.ordev_cap) a.ordev[r] = ev;
    else __hip_atomic_fetch_or(&a.ctrl->error, ERR_ORDEV, __ATOMIC_RELAXED, DEV_SCOPE);
}

template <int NW, uint32_t OPS = OPS_ANY>
__device__ __forceinline__ void acc_identity(const WordDesc& wd, uint64_t* acc) {
#pragma unroll
    for (int i = 0; i < NW; i++) acc[i] = word_on<OPS>(wd, i) ? word_identity(word_op<OPS>(wd, i)) : 0;
}

// acc = merge(acc, state of entry e) when the entry holds an accumulator (windowState.value != null)
template <int NW, int E, bool Q, uint32_t OPS>
__device__ __forceinline__ void merge_entry(const MergeArgs& a, StateLds<NW, E>& S, int e, uint64_t* acc) {
    if (e < 0 || !(S.flag[e] & F_ACC)) return;
    uint64_t o[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) o[i] = S.acc[i][e];
    merge_slice<NW, Q, OPS>(a.wd, a.ad, acc, o);
}

// TUMBLE: SliceUnsharedSyncStateWindowAggProcessor.fireWindow (:54-66) + clearWindow
// (expiredSlices(we) = [we]); DataStream tumbling: WindowOperator.onEventTime + clearAllState.
// Windows of different keys and of one key are independent: every due entry fires once.
template <int NW, int E, bool Q, uint32_t OPS>
__device__ __forceinline__ uint32_t fire_tumble(const MergeArgs& a, StateLds<NW, E>& S, int e, int sb, int32_t* s_emit) {
    uint64_t acc[NW];
    const uint32_t f = atomicAnd(&S.flag[e], ~(F_TIMER | F_ACC));
    if (f & F_ACC) {
#pragma unroll
        for (int i = 0; i < NW; i++) acc[i] = S.acc[i][e];
    } else {
        acc_identity<NW, OPS>(a.wd, acc);
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
// exactly once.  A chain step reuses the entries of the window it just fired: the next window's
// slices are the new slice (the entry nextTriggerWindow found or inserted) plus all but the oldest
// of the previous window's, so with n <= HB slices per window only the chain's first window probes.
// (An entry absent when cached may since have been inserted by another chain of the key, but only
// empty -- without F_ACC -- which merges like an absent one.)
template <int NW, int E, bool Q, uint32_t OPS>
__device__ __forceinline__ uint32_t fire_hop_chain(const MergeArgs& a, int64_t W, StateLds<NW, E>& S, int e, int sb, int32_t* s_emit,
                                   uint64_t* fst = nullptr) {
    const WinDesc& w = a.win;
    const WordDesc& wd = a.wd;
    constexpr int HB = NW <= 2 ? 8 : NW <= 4 ? 4 : 2;
    const int64_t k = S.key[e];
    int64_t we = S.slice[e];
    int ew = e;
    uint32_t nf = 0;
    const int n = w.n_slices;
    int ring[HB];  // entries of window we's slices, newest first (n <= HB), -1 absent
    bool have_ring = false;
    uint64_t t0 = fst ? __builtin_amdgcn_s_memtime() : 0;
    auto lap = [&](int i) {  // diagnostic (AB_FSTAMPS): per-lane cycles of the chain's parts
        if (!fst) return;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        fst[i] += t1 - t0;
        t0 = t1;
    };
    for (;;) {
        const uint32_t old = atomicOr(&S.flag[ew], F_FIRED);
        if (old & F_FIRED) break;  // fired by another chain of this key
        atomicAnd(&S.flag[ew], ~F_TIMER);
        nf++;
        lap(3);
        uint64_t acc[NW];
        acc_identity<NW, OPS>(wd, acc);
        const int64_t s_exp = wadd(wsub(we, w.size), w.interval);  // clearWindow's expired slice
        int e_exp = -3;
        int64_t s = we;
        if (have_ring) {
#pragma unroll
            for (int j = 0; j < HB; j++) {
                if (j >= n) break;
                merge_entry<NW, E, Q, OPS>(a, S, ring[j], acc);
                if (j == n - 1) e_exp = ring[j];  // the oldest slice is clearWindow's
            }
        } else for (int j0 = 0; j0 < n; j0 += HB) {
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
                merge_entry<NW, E, Q, OPS>(a, S, e2, acc);
                if (ss[j] == s_exp) e_exp = e2;
                ring[j] = e2;  // j0 == 0 whenever the ring is used (n <= HB)
            }
        }
        lap(0);
        const bool nonempty = a.ad.count_star_word < 0 || acc[a.ad.count_star_word] != 0;
        if (nonempty) emit_row<NW, Q>(a, sb, s_emit, k, we, acc);
        lap(1);
        const int e2 = e_exp != -3 ? e_exp : find_entry(S, k, s_exp);
        if (e2 >= 0) atomicOr(&S.flag[e2], F_EXPIRE);
        if (!nonempty) break;
        const int64_t nx = wadd(we, w.interval);
        const int en = find_or_insert<NW, E, OPS>(S, k, nx, wd);
        lap(2);
        if (en < 0) break;  // state overflow (flagged)
        if (!win_fired(w, nx, W)) {
            atomicOr(&S.flag[en], F_TIMER);
            break;
        }
        if (n <= HB) {  // window nx: slice nx, then window we's slices but its oldest
#pragma unroll
            for (int j = HB - 1; j > 0; j--) ring[j] = ring[j - 1];
            ring[0] = en;
            have_ring = true;
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
template <int NW, int E, bool Q, uint32_t OPS>
__device__ __forceinline__ uint32_t fire_cumulate_chain(const MergeArgs& a, int64_t W, StateLds<NW, E>& S, int e, int sb, int32_t* s_emit) {
    const WinDesc& w = a.win;
    const WordDesc& wd = a.wd;
    const int64_t k = S.key[e];
    int64_t we = S.slice[e];
    const int64_t ws = window_start_of(w, we);
    const int64_t first = wadd(ws, w.interval);
    const int64_t last = wadd(ws, w.size);
    const int ef = find_or_insert<NW, E, OPS>(S, k, first, wd);
    uint64_t acc[NW];
    if (ef >= 0 && (S.flag[ef] & F_ACC)) {
#pragma unroll
        for (int i = 0; i < NW; i++) acc[i] = S.acc[i][ef];
    } else {
        acc_identity<NW, OPS>(wd, acc);
    }
    uint32_t nf = 0;
    bool done = false;
    int ewe = e;
    for (;;) {
        if (ewe >= 0) atomicAnd(&S.flag[ewe], ~F_TIMER);
        if (we != first) merge_entry<NW, E, Q, OPS>(a, S, ewe, acc);
        nf++;
        if (a.ad.count_star_word < 0 || acc[a.ad.count_star_word] != 0) emit_row<NW, Q>(a, sb, s_emit, k, we, acc);
        if (we != first && ewe >= 0) atomicAnd(&S.flag[ewe], ~F_ACC);
        if (we == last) {  // expiredSlices(last) = [last, first]
            if (ef >= 0) atomicAnd(&S.flag[ef], ~F_ACC);
            done = true;
            break;
        }
        const int64_t nx = wadd(we, w.interval);
        if (!win_fired(w, nx, W)) {
            const int en = find_or_insert<NW, E, OPS>(S, k, nx, wd);
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
__device__ __forceinline__ void mark_cumulate_successor(const MergeArgs& a, int64_t W, StateLds<NW, E>& S, int e) {
    const WinDesc& w = a.win;
    const int64_t k = S.key[e];
    const int64_t we = S.slice[e];
    const int64_t last = wadd(window_start_of(w, we), w.size);
    for (int64_t s = we; s != last;) {
        s = wadd(s, w.interval);
        if (!win_fired(w, s, W)) break;
        const int e2 = find_entry(S, k, s);
        if (e2 >= 0 && (S.flag[e2] & F_TIMER)) {
            atomicOr(&S.flag[e2], F_NOTHEAD);
            break;
        }
    }
}

// HOP pre-pass: a due window whose predecessor window (we - slide) is due and non-empty is
// reached by the chain that fires the predecessor (which continues while its windows are
// non-empty), so it starts no chain of its own.  Conservative: the predecessor's own slice holding
// an accumulator (with its COUNT(*) > 0) proves the predecessor window non-empty; a window whose
// predecessor cannot be proven so starts a chain, and the F_FIRED claim settles any overlap.
template <int NW, int E>
__device__ __forceinline__ void mark_hop_successor(const MergeArgs& a, int64_t W, StateLds<NW, E>& S, int e) {
    const int64_t k = S.key[e];
    const int64_t pe = wsub(S.slice[e], a.win.interval);
    const int p = find_entry(S, k, pe);
    if (p >= 0 && (S.flag[p] & (F_TIMER | F_ACC)) == (F_TIMER | F_ACC) && win_fired(a.win, pe, W) &&
        (a.ad.count_star_word < 0 || S.acc[a.ad.count_star_word][p] != 0))
        atomicOr(&S.flag[e], F_NOTHEAD);
}

// ---- DataStream windows (KIND_DSWIN): one entry per (key, window end), as WindowOperator keeps
// one state per (key, window).  A pane partial (key, pane end) is added to every window of the
// pane that is not late (HeapReducingState.add per window, WindowOperator.java:405-433); a window
// gets its maxTimestamp timer (EventTimeTrigger.onElement) and its cleanup timer
// (registerCleanupTimer).  Windows the watermark already fired are not reached here: their rows
// took the late-fire path.
// minBy / maxBy: folds the element (v = field key, o = arrival ordinal) into entry e's pair.  The
// two words change together, so lanes take the entry's lock bit in turn.  The retry loop is
// wave-uniform (it runs until no active lane is left): a lane that wins the bit runs its critical
// section and releases it in the same pass, so neither a lane of the same wave spinning on the bit
// nor the compiler moving the section out of the loop can stall the holder.
constexpr uint32_t F_BYLOCK = 1u << 30;
template <int NW, int E>
__device__ __forceinline__ void by_fold(const MergeArgs& a, StateLds<NW, E>& S, int e, uint64_t v, uint64_t o) {
    const int wv = a.ad.w0[0], wo = a.ad.first_word;
    const int32_t vop = a.wd.op[wv], oop = a.wd.op[wo];
    bool done = false;
    do {
        if (!done && !(atomicOr(&S.flag[e], F_BYLOCK) & F_BYLOCK)) {
            compiler_fence();
            if (by_better(vop, oop, v, o, S.acc[wv][e], S.acc[wo][e])) {
                S.acc[wv][e] = v;
                S.acc[wo][e] = o;
            }
            compiler_fence();
            atomicAnd(&S.flag[e], ~F_BYLOCK);
            done = true;
        }
    } while (__ballot(!done) != 0);
}

template <int NW, int E>
__device__ __forceinline__ void ds_add_to_windows(const MergeArgs& a, StateLds<NW, E>& S, int64_t k, int64_t pe, const uint64_t* v,
                                  int64_t w_old, bool late_rows) {
    const WinDesc& w = a.win;
    const int64_t e0 = ds_first_window_end(w, pe);
    for (int i = 0; i < w.n_win; i++) {
        const int64_t e = wsub(e0, (int64_t)i * w.slide);
        if (!ds_window_holds_pane(w, e, pe)) break;
        const int64_t ct = ds_cleanup_time(w, e);
        if (ct <= w_old) continue;  // isWindowLate
        const bool fired_already = is_fired(e, w_old);
        if (fired_already && !late_rows) continue;
        const uint32_t fl = F_ACC | (ct != INT64_MAX ? F_CLEAN : 0u) | (fired_already ? 0u : F_TIMER);
        bool ins = false;
        const int en = find_or_insert(S, k, e, a.wd, v, fl | F_NEW, &ins);
        if (en < 0 || ins) continue;
#pragma unroll
        for (int q = 0; q < NW; q++)
            if (q < a.wd.nw) lds_fold(a.wd.op[q], &S.acc[q][en], v[q]);  // (pair words: no-op)
        if (a.ad.by_prev >= 0) by_fold<NW, E>(a, S, en, v[a.ad.w0[0]], v[a.ad.first_word]);
        atomicOr(&S.flag[en], fl);
    }
}

// is window `e` one of pane `pe`'s windows
__device__ __forceinline__ bool ds_pane_in_window(const WinDesc& w, int64_t pe, int64_t e) {
    const int64_t e0 = ds_first_window_end(w, pe);
    const uint64_t d = (uint64_t)wsub(e0, e);
    if ((int64_t)d < 0) return false;
    const uint64_t q = udiv(d, w.slide_div);
    return q * (uint64_t)w.slide == d && q < (uint64_t)w.n_win && ds_window_holds_pane(w, e, pe);
}

// DataStream timers of one entry at watermark W (WindowOperator.onEventTime :450-494): the
// maxTimestamp timer FIREs (emitWindowContents), the cleanup timer clears the window state; with
// allowedLateness 0 they are the same timer (fire, then clear)
template <int NW, int E>
__device__ __forceinline__ uint32_t fire_ds(const MergeArgs& a, int64_t W, StateLds<NW, E>& S, int e, int sb, int32_t* s_emit) {
    const int64_t we = S.slice[e];
    const uint32_t f = S.flag[e];
    const bool fire = (f & F_TIMER) && is_fired(we, W);
    const bool clean = (f & F_CLEAN) && ds_cleanup_time(a.win, we) <= W;
    if (fire && (f & F_ACC)) {
        uint64_t acc[NW];
#pragma unroll
        for (int i = 0; i < NW; i++) acc[i] = S.acc[i][e];
        emit_row<NW, false>(a, sb, s_emit, S.key[e], we, acc);
    }
    S.flag[e] = f & ~((fire ? F_TIMER : 0u) | (clean ? (F_ACC | F_TIMER | F_CLEAN) : 0u));
    // clearAllState: a window state retained by an earlier launch releases its first element
    // (minBy / maxBy: the arg retained at the last write-back, if any)
    if (clean && (f & F_ACC) && a.ad.by_prev >= 0) {
        const uint64_t pv = S.acc[a.ad.by_prev][e];
        if (pv != ~0ull) push_ordev(a, ORDEV_RELEASE | (int64_t)pv);
    } else if (clean && (f & F_ACC) && !(f & F_NEW) && a.ad.first_word >= 0) {
        push_ordev(a, ORDEV_RELEASE | (int64_t)S.acc[a.ad.first_word][e]);
    }
    return fire ? 1u : 0u;
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
    __device__ __forceinline__ void mark(int phase) {  // call right after a __syncthreads()
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

// the watermark of this advance: the launch argument, or (fw_advance_device) the value a device-side
// watermark valve left in device memory (StatusWatermarkValve min over input channels, computed on the
// device without a host round trip)
__device__ __forceinline__ int64_t merge_watermark(const MergeArgs& a) {
    return a.wm_dev ? __hip_atomic_load(a.wm_dev, __ATOMIC_RELAXED, DEV_SCOPE) : a.wm;
}

// the last workgroup of a k_merge_fire launch applies the launch's control decisions (every
// workgroup read the old values at its start): advanceProgress bookkeeping of the processor
// (AbstractSliceSyncStateWindowAggProcessor.java:139-153), the buffer reset after a flush, the
// consumed timer requests, and the overflow-counter switch of a result reset.
__device__ void merge_finalize(const MergeArgs& a, int64_t W) {
    Ctrl* c = a.ctrl;
    const int64_t cur = c->cur, pend = c->pending_pushes, ntp = c->ntp;
    const bool adv = !a.force_flush && W > cur;
    const bool do_flush = pend > 0 && (a.force_flush || (adv && (a.always_flush || (W >= ntp && win_fired(a.win, c->min_pending, W)))));
    if (adv) {
        c->cur = W;
        if (W >= ntp) c->ntp = tz_next_trigger_watermark(a.win.tz, W, a.win.slice_div);
    }
    if (do_flush) {
        c->pending_pushes = 0;
        c->min_pending = INT64_MAX;
        c->pending_rows = 0;
        c->n_lfire = 0;
        c->flush_launches += 1;
        c->parts_merged = c->partials;  // a flush reads every partial written so far
        c->part_bytes_merged = c->part_bytes;
    }
    c->n_treq = 0;
    for (int q = 0; q < 8; q++) __hip_atomic_store(&a.tickets->work[q][0], 0u, __ATOMIC_RELAXED, DEV_SCOPE);
    const int sel = (c->ovf_sel ^ a.reset_out) & 1;
    c->ovf_sel = sel;
    __hip_atomic_store(&c->out_count[sel ^ 1], 0ull, __ATOMIC_RELAXED, DEV_SCOPE);
    // the overflow region's rows, beside the slab counts (fw_results_device_segments)
    a.sb_out[a.n_sb] = (int32_t)min((int64_t)__hip_atomic_load(&c->out_count[sel], __ATOMIC_RELAXED, DEV_SCOPE), a.out_cap);
    if (a.host_mirror)  // vector store to host-mapped memory (system scope)
        __hip_atomic_store(a.host_mirror, (unsigned long long)((a.merge_seq << 8) | (uint64_t)(do_flush ? 0 : pend)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void merge_ticket(const MergeArgs& a, int64_t W) {
    if (threadIdx.x != 0) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (grid_last_wg(a.tickets->c[1])) {
        merge_finalize(a, W);
        kt_end(a.kt);
    }
}

// rows of one cell loaded together in the gather (VGPR budget of the 1024-thread workgroup)
// rows per lane per gather pass by accumulator words (measured against the round-3 sizes: one word
// 3 rows per lane instead of 4 -- CFG2 flush 176 -> 167 us, CFG3 274 -> 266 us; two words 2 instead
// of 3 -- CFG4 203 -> 191 us; four words stay at 2)
constexpr int mg_rows_in_flight(int nw) {
    return nw <= 1 ? 3 : nw <= 2 ? 2 : nw <= 4 ? 2 : 1;
}


// ---- the gather's view of the pending partials.  A wave takes a group of up to 64 consecutive
// cells of one push slot (lane l holds cell word v of flat cell position f), scans their row
// counts and deals the group's rows over its lanes.
struct CellGroup {
    uint32_t tot;       // rows in the group
    uint32_t excl;      // this lane's cell: rows of the group's cells before it
    uint32_t adj;       // this lane's cell: slot row index of its first row, less excl (mod 2^32)
    uint32_t fmt;       // this lane's cell: its chunk's partial-row format (PF_*)
};
__device__ __forceinline__ CellGroup cell_group(uint32_t v, int f, int64_t CH) {
    const int lane = threadIdx.x & 63;
    const uint32_t cnt = cell_count(v);
    uint32_t inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)inc, d, 64);
        if (lane >= d) inc += t;
    }
    CellGroup g;
    g.tot = (uint32_t)__shfl((int)inc, 63, 64);
    g.excl = inc - cnt;
    g.adj = (uint32_t)(cell_chunk(f) * CH + cell_start(v)) - g.excl;
    g.fmt = cell_fmt(v);
    return g;
}
// Row r0 + u * 64 + lane of the group (clamped to the last row), in the PF_WIDE layout (key,
// sliceEnd, acc[NW]) whatever its chunk's format: the compact formats' slice end is the push's rank
// base + rank * interval, PF_UNIT's count is 1.  Returns the rows to fold (bit u): those inside the
// group and -- when several superbuckets share the ingest superbucket (ks.pass_log2 > 0) -- routed
// to superbucket `sb`.
// gather variants of the merge kernels (template GF): the superbuckets outnumber the ingest
// superbuckets (rows are routed again), and / or the chunks may hold compact rows.  Reading compact
// rows costs the wide-row gather of the other layouts ~10 % even when no chunk is compact, so only
// the COUNT(*)-only layouts, whose compact rows are the key alone, are built with it.
constexpr int GF_PASS = 1;
constexpr int GF_COMPACT = 2;

// PF_PACK rows (fw_internal.h): the flush epoch's fields and bases, and one row decoded into the
// PF_WIDE layout (key, sliceEnd, acc)
struct PackDec {
    int64_t kbase, vbase, rbase;
    uint32_t ksh, rb, vb;
};
__device__ __forceinline__ PackDec pack_dec(const MergeArgs& a) {
    PackDec d;
    const uint32_t bits = __hip_atomic_load(&a.ctrl->pk_cur_bits, __ATOMIC_RELAXED, DEV_SCOPE);
    d.kbase = __hip_atomic_load(&a.ctrl->pk_cur_k, __ATOMIC_RELAXED, DEV_SCOPE);
    d.vbase = __hip_atomic_load(&a.ctrl->pk_cur_v, __ATOMIC_RELAXED, DEV_SCOPE);
    d.rbase = a.slot_base[0];
    d.ksh = 64u - (bits & 255u);
    d.rb = (bits >> 8) & 255u;
    d.vb = (bits >> 16) & 255u;
    return d;
}
template <int PW>
__device__ __forceinline__ void unpack_row(const PackDec& d, uint64_t w, int64_t interval, uint64_t (&row)[PW]) {
    static_assert(PW == 3, "PF_PACK rows carry one accumulator word");
    row[0] = (uint64_t)d.kbase + (w >> d.ksh);
    const uint32_t rank = (uint32_t)(w >> d.vb) & ((1u << d.rb) - 1u);
    // rank * interval < 2^31 (IngestArgs::rank_lim)
    row[1] = (uint64_t)(d.rbase + (int64_t)(rank * (uint32_t)interval));
    row[2] = (uint64_t)d.vbase + (w & ((1ull << d.vb) - 1ull));
}

template <int NW, int GU, int GF>
__device__ __forceinline__ uint32_t load_group_rows(const MergeArgs& a, int64_t pi, const CellGroup& g, uint32_t r0,
                                                    int sb, uint64_t (&row)[GU][2 + NW]) {
    constexpr int PW = 2 + NW;
    constexpr bool PS = (GF & GF_PASS) != 0, CR = (GF & GF_COMPACT) != 0;
    const int lane = threadIdx.x & 63;
    const uint64_t* seg = a.parts + (size_t)pi * a.cap_rows * PW;
#pragma unroll
    for (int u = 0; u < GU; u++) {
        // the group's row x lives in the last cell whose first row is <= x
        const uint32_t x = min(r0 + (uint32_t)(u * 64 + lane), g.tot - 1);
        int lo = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
            if ((uint32_t)__shfl((int)g.excl, lo + step, 64) <= x) lo += step;
        const uint32_t rg = (uint32_t)__shfl((int)g.adj, lo, 64) + x;  // row index in the slot
        const uint32_t fmt = (uint32_t)__shfl((int)g.fmt, lo, 64);
        if (!CR || fmt == PF_WIDE) {
            load_words<PW>(seg + (size_t)rg * PW, row[u]);
        } else if (NW == 1 && fmt == PF_PACK) {
            const uint32_t within = rg & ((1u << a.ch_log2) - 1u);
            if constexpr (NW == 1) unpack_row(pack_dec(a), seg[(size_t)(rg - within) * PW + within], a.win.interval, row[u]);
        } else {
            // a compact chunk fills the front of its PF_WIDE-sized region
            const uint32_t within = rg & ((1u << a.ch_log2) - 1u);
            const uint64_t* p = seg + (size_t)(rg - within) * PW;
            const uint32_t rank = a.ranks[(size_t)pi * a.cap_rows + rg];
            // slot_base + rank * interval: 32-bit product (rank * interval < 2^31, IngestArgs::rank_lim)
            row[u][1] = (uint64_t)(a.slot_base[pi] + (int64_t)(rank * (uint32_t)a.win.interval));
            if (fmt == PF_NARROW) {
                uint64_t t[1 + NW];
                load_words<1 + NW>(p + (size_t)within * (1 + NW), t);
                row[u][0] = t[0];
#pragma unroll
                for (int w = 0; w < NW; w++) row[u][2 + w] = t[1 + w];
            } else {  // PF_UNIT: COUNT(*) alone, nothing folded
                row[u][0] = p[within];
#pragma unroll
                for (int w = 0; w < NW; w++) row[u][2 + w] = w == 0 ? 1ull : 0ull;
            }
        }
    }
    uint32_t live = 0;
#pragma unroll
    for (int u = 0; u < GU; u++) live |= (uint32_t)(r0 + (uint32_t)(u * 64 + lane) < g.tot) << u;
    if constexpr (PS)
#pragma unroll
        for (int u = 0; u < GU; u++) {
            uint32_t m;
            if ((live >> u) & 1u) live &= ~((uint32_t)(route_key(a.ks, (int64_t)row[u][0], 0, &m) != sb) << u);
        }
    return live;
}

// TimeWindowUtil.isWindowFired in a shift zone, kept out of the gather's hot loop
// (the zone table by value: a reference into the kernel arguments would copy them to scratch)
static __device__ __noinline__ bool tz_fired_out_of_line(TzTable z, int64_t we, int64_t progress) {
    return tz_is_fired(z, we, progress);
}

// ---- the gather over runs (IngestArgs::runs).  The pending pushes' rows of one ingest superbucket
// lie in RUN_X contiguous sub-runs per push; lane l of every wave holds segment l = (push l / RUN_X,
// sub-run l % RUN_X), so the 64 lanes cover FW_MAX_PENDING pushes.  A wave deals a block of 64 * G
// consecutive rows of the concatenated segments over its lanes: neighbouring lanes load neighbouring
// rows, and no load depends on another (no cell words).
static_assert(FW_MAX_PENDING * RUN_X <= 64, "one lane per (push, sub-run)");
struct RunSegs {
    uint32_t tot;   // rows in all segments
    uint32_t excl;  // this lane's segment: rows of the segments before it
    uint32_t adj;   // this lane's segment: run row index of its first row, less excl (mod 2^32)
    uint32_t pf;    // this lane's segment: push | run format << 4
};
__device__ __forceinline__ RunSegs run_segs(const MergeArgs& a, int isb, int64_t pend) {
    const int lane = threadIdx.x & 63;
    const int p = lane / RUN_X, x = lane % RUN_X;
    uint32_t n = 0, fm = 0;
    if (p < pend) {
        n = min(a.run_fill[((size_t)p * RUN_X + x) * a.n_sb + isb], (uint32_t)a.sub_cap);
        fm = (uint32_t)a.slot_fmt[p];
    }
    uint32_t inc = n;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)inc, d, 64);
        if (lane >= d) inc += t;
    }
    RunSegs g;
    g.tot = (uint32_t)__shfl((int)inc, 63, 64);
    g.excl = inc - n;
    g.adj = (uint32_t)(((size_t)isb * RUN_X + x) * (size_t)a.sub_cap) - g.excl;
    g.pf = (uint32_t)p | (fm << 4);
    return g;
}
// rows r0 + u * 64 + lane of the segments (clamped to the last), in the PF_WIDE layout whatever their
// push's format (as load_group_rows); returns the rows inside the segments (bit u).  r0 is
// wave-uniform, so the segments a block touches are found with scalar reads of the lanes' segment
// words (v_readlane): the block's first row by a scalar binary search, then the (few) segment
// boundaries inside the block -- no per-row cross-lane shuffles.
template <int NW, int GU, int GF>
__device__ __forceinline__ uint32_t load_run_rows(const MergeArgs& a, const RunSegs& g, uint32_t r0_,
                                                  uint64_t (&row)[GU][2 + NW]) {
    constexpr int PW = 2 + NW;
    constexpr bool CR = (GF & GF_COMPACT) != 0;
    const int lane = threadIdx.x & 63;
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)r0_);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readfirstlane((int)g.tot);
    const uint32_t last = min(r0 + (uint32_t)(64 * GU), tot) - 1u;  // the block's last row (tot > 0)
    PackDec pk{};
    if constexpr (CR && NW == 1) pk = pack_dec(a);
    const uint32_t first = min(r0, tot - 1u);  // a block past the end re-reads the last row
    int cur = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1)
        if ((uint32_t)__builtin_amdgcn_readlane((int)g.excl, cur + step) <= first) cur += step;
    uint32_t x[GU], adj[GU], pf[GU];
    {
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)g.adj, cur);
        const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)g.pf, cur);
#pragma unroll
        for (int u = 0; u < GU; u++) {
            x[u] = min(r0 + (uint32_t)(u * 64 + lane), tot - 1u);
            adj[u] = a0;
            pf[u] = p0;
        }
    }
    while (cur < 63) {  // (uniform) the boundaries inside the block, empty segments included
        const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)g.excl, cur + 1);
        if (b > last) break;
        cur++;
        const uint32_t an = (uint32_t)__builtin_amdgcn_readlane((int)g.adj, cur);
        const uint32_t pn = (uint32_t)__builtin_amdgcn_readlane((int)g.pf, cur);
#pragma unroll
        for (int u = 0; u < GU; u++) {
            adj[u] = x[u] >= b ? an : adj[u];
            pf[u] = x[u] >= b ? pn : pf[u];
        }
    }
#pragma unroll
    for (int u = 0; u < GU; u++) {
        const uint32_t ri = adj[u] + x[u];  // row index in its push's run region
        const uint32_t p = pf[u] & 15u, fmt = (pf[u] >> 4) & 3u;
        const uint64_t* base = a.runs + (size_t)p * a.run_rows * PW;
        if (!CR || fmt == PF_WIDE) {
            // plain 8-B loads straight into the row's registers: no lane-parity selects, so the
            // wait for a block's rows is a counted s_waitcnt at its first use
            const uint64_t* q = base + (size_t)ri * PW;
#pragma unroll
            for (int w = 0; w < PW; w++) row[u][w] = q[w];
        } else if (NW == 1 && fmt == PF_PACK) {
            if constexpr (NW == 1) unpack_row(pk, base[ri], a.win.interval, row[u]);
        } else {
            const uint32_t rank = a.run_ranks[(size_t)p * a.run_rows + ri];
            row[u][1] = (uint64_t)(a.slot_base[p] + (int64_t)(rank * (uint32_t)a.win.interval));
            if (fmt == PF_NARROW) {
                uint64_t t[1 + NW];
                load_words<1 + NW>(base + (size_t)ri * (1 + NW), t);
                row[u][0] = t[0];
#pragma unroll
                for (int w = 0; w < NW; w++) row[u][2 + w] = t[1 + w];
            } else {  // PF_UNIT: COUNT(*) alone, nothing folded
                row[u][0] = base[ri];
#pragma unroll
                for (int w = 0; w < NW; w++) row[u][2 + w] = w == 0 ? 1ull : 0ull;
            }
        }
    }
    uint32_t live = 0;
#pragma unroll
    for (int u = 0; u < GU; u++) live |= (uint32_t)(r0 + (uint32_t)(u * 64 + lane) < tot) << u;
    return live;
}
// every run row of superbucket sb's pending pushes through process(rows, live): waves take blocks of
// 64 * G rows in turn.  D > 1: a ring of D blocks -- the loads of the next D - 1 blocks are in flight
// while the current one is processed.  They are issued unconditionally (past the end a block re-reads
// the last row, live bits 0), so each wait is a counted s_waitcnt that leaves the younger blocks'
// loads in flight.
template <int NW, int G, int GF, int D, typename F>
__device__ __forceinline__ void gather_runs(const MergeArgs& a, int sb, int64_t pend, F&& process) {
    constexpr int PW = 2 + NW;
    constexpr uint32_t STEP = (uint32_t)MG_BLOCK * G;  // (MG_BLOCK / 64) waves x 64 lanes x G rows
    const RunSegs g = run_segs(a, sb, pend);
    uint32_t r0 = (uint32_t)(threadIdx.x >> 6) * 64u * G;
    if (r0 >= g.tot) return;  // (wave-uniform)
    if constexpr (D > 1) {
        uint64_t buf[D][G][PW];
        uint32_t live[D];
        static_for<D - 1>([&](auto K) {
            constexpr int k = decltype(K)::value;
            live[k] = load_run_rows<NW, G, GF>(a, g, r0 + (uint32_t)k * STEP, buf[k]);
        });
        bool done = false;
        while (!done) {  // unrolled by D: the ring's slots rotate without copies
            static_for<D>([&](auto K) {
                constexpr int k = decltype(K)::value;
                constexpr int kn = (k + D - 1) % D;
                if (done) return;
                live[kn] = load_run_rows<NW, G, GF>(a, g, r0 + (uint32_t)(D - 1) * STEP, buf[kn]);
                process(buf[k], live[k]);
                r0 += STEP;
                done = r0 >= g.tot;
            });
        }
    } else {
        for (; r0 < g.tot; r0 += STEP) {
            uint64_t row[G][PW];
            const uint32_t live = load_run_rows<NW, G, GF>(a, g, r0, row);
            process(row, live);
        }
    }
}
// the pushes (bit p) in which some chunk left rows of superbucket sb in its own region (wave-uniform)
__device__ __forceinline__ uint32_t run_overflow(const MergeArgs& a, int sb, int64_t pend) {
    const int lane = threadIdx.x & 63;
    const bool o = lane < pend && a.run_ovf[(size_t)lane * a.n_sb + sb] != 0;
    return (uint32_t)__ballot(o);
}
// after the flush has read them: superbucket sb's fill counters and overflow flags start the next
// pushes at 0 (one reader per superbucket: runs are planned without pass_log2)
__device__ __forceinline__ void run_release(const MergeArgs& a, int sb, int64_t pend) {
    const int t = threadIdx.x;
    if (t >= 64) return;
    const int p = t / RUN_X, x = t % RUN_X;
    if (p >= pend) return;
    a.run_fill[((size_t)p * RUN_X + x) * a.n_sb + sb] = 0u;
    if (x == 0) a.run_ovf[(size_t)p * a.n_sb + sb] = 0u;
}
// the rows push pi's chunks kept in their own regions (their cell words) through process(rows, live)
template <int NW, int GU, int GF, typename F>
__device__ __forceinline__ void gather_cells_push(const MergeArgs& a, int sb, int64_t pi, F&& process) {
    constexpr int PW = 2 + NW;
    constexpr bool PS = (GF & GF_PASS) != 0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ncell = (int)cell_pad(a.slot_nch[pi]);
    const int G = min(64, ncell / (MG_BLOCK / 64));
    const int ngroups = ncell / G;
    const int pl = PS ? a.ks.pass_log2 : 0;
    const int nis = a.n_sb >> pl;
    const uint32_t* cl = a.cells + (size_t)pi * nis * a.max_nch;
    for (int gi = wv; gi < ngroups; gi += MG_BLOCK / 64) {
        const int f = gi * G + lane;
        const uint32_t v = (lane >= G || cell_chunk(f) >= a.slot_nch[pi]) ? 0u : cl[((size_t)(f >> 4) * nis + (sb >> pl)) * CELL_LANES + (f & 15)];
        const CellGroup cg = cell_group(v, f, a.chunk_rows);
        for (uint32_t r0 = 0; r0 < cg.tot; r0 += 64 * GU) {
            uint64_t row[GU][PW];
            const uint32_t live = load_group_rows<NW, GU, GF>(a, pi, cg, r0, sb, row);
            process(row, live);
        }
    }
}

// GF: gather variant (GF_PASS: KeySpace.pass_log2 > 0, GF_COMPACT: compact partial rows)
template <int NW, int E, bool Q, int KIND, uint32_t OPS, int GF>
__global__ __launch_bounds__(MG_BLOCK, 4) void k_merge_fire(MergeArgs a) {
    constexpr bool PS = (GF & GF_PASS) != 0;
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
    kt_start(a.kt);
    Ctrl* c = a.ctrl;
    const int64_t W = merge_watermark(a);
    // control decisions; the launch's last workgroup applies them to the control block (merge_finalize)
    const int64_t cur = __hip_atomic_load(&c->cur, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t pend = __hip_atomic_load(&c->pending_pushes, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t ntreq = min(__hip_atomic_load(&c->n_treq, __ATOMIC_RELAXED, DEV_SCOPE), (int64_t)0x7fffffff);
    const int64_t nlf = KIND == KIND_DSWIN ? min(__hip_atomic_load(&c->n_lfire, __ATOMIC_RELAXED, DEV_SCOPE), a.lfire_cap) : 0;
    const int64_t ntp = __hip_atomic_load(&c->ntp, __ATOMIC_RELAXED, DEV_SCOPE);
    const int64_t minp = __hip_atomic_load(&c->min_pending, __ATOMIC_RELAXED, DEV_SCOPE);
    const bool adv = !a.force_flush && W > cur;
    const bool do_flush = pend > 0 &&
                          (a.force_flush || (adv && (a.always_flush || (W >= ntp && win_fired(a.win, minp, W)))));
    const bool do_fire = adv;
    const int64_t w_old = cur;

    Stamps stm;
    stm.init((FW_ABL(a) & AB_STAMPS) != 0);
    // Persistent workgroups (one per CU: the LDS table fills it) pull superbuckets from a work
    // counter per XCD (the dispatcher deals blocks to XCDs round robin, block b to XCD b % 8), each
    // XCD owning a contiguous eighth of the superbuckets so their cells share its L2.  A launch
    // pays one round of workgroup start-up instead of n_sb / CUs rounds, a watermark with nothing
    // to flush or fire costs one short pass, and skewed superbuckets balance within an XCD.  The
    // next ticket is fetched while the current superbucket is processed.
    const bool xq = a.n_sb % 8 == 0 && gridDim.x % 8 == 0;
    const int nq = xq ? a.n_sb / 8 : a.n_sb;
    uint32_t* const wq = &a.tickets->work[xq ? blockIdx.x % 8 : 0][0];
    const int qbase = xq ? (int)(blockIdx.x % 8) * nq : 0;
    __shared__ int32_t s_tk;
    if (tid == 0) s_tk = (int32_t)__hip_atomic_fetch_add(wq, 1u, __ATOMIC_RELAXED, DEV_SCOPE);
    // Without a flush or timer requests, a superbucket has work only if one of its timers is due:
    // every workgroup checks its XCD's whole share in one parallel pass, and when nothing is due
    // (a watermark that crosses no window end) the launch ends here -- results reset aside.
    if (!do_flush && ntreq == 0) {
        bool due = false;
        for (int i = tid; i < nq; i += MG_BLOCK) due |= do_fire && win_fired(a.win, a.sb_min_timer[qbase + i], W);
        if (!__syncthreads_or(due)) {
            if (a.reset_out)
                for (int i = tid; i < nq; i += MG_BLOCK) a.sb_out[qbase + i] = 0;
            s_tk = nq;  // written by every thread: no superbucket for this workgroup
        }
    }
    __syncthreads();
    for (int tk = s_tk; tk < nq; tk = s_tk) {
    const int sb = qbase + tk;
    const int32_t n0 = a.state_count[sb];
    __syncthreads();  // every thread has read s_tk; the previous superbucket is done with the LDS
    if (tid == 0) {
        s_tk = (int32_t)__hip_atomic_fetch_add(wq, 1u, __ATOMIC_RELAXED, DEV_SCOPE);  // the next one
        s_work = (ntreq > 0) || do_flush || (do_fire && win_fired(a.win, a.sb_min_timer[sb], W));
        s_fired = 0;
        s_emit = a.reset_out ? 0 : a.sb_out[sb];
        if (!s_work && a.reset_out) a.sb_out[sb] = 0;
    }
    __syncthreads();
    if (!s_work) continue;
    const bool gather = do_flush && !(FW_ABL(a) & AB_M_NO_GATHER);
    // this thread's first cell word, loaded while the state loads (the gather below walks the
    // cells of every pending push, one cell per thread per pass, in flat tile order f:
    // cell_chunk(f) is the chunk, positions past the push's last chunk are padding)
    auto cell_at = [&](int64_t pi, int f) -> uint32_t {  // cells of this superbucket's ingest superbucket
        if (cell_chunk(f) >= a.slot_nch[pi]) return 0u;
        const int pl = PS ? a.ks.pass_log2 : 0;
        const int nis = a.n_sb >> pl;
        const uint32_t* cl = a.cells + (size_t)pi * nis * a.max_nch;
        return cl[((size_t)(f >> 4) * nis + (sb >> pl)) * CELL_LANES + (f & 15)];
    };
    // the gather splits a push's cells into groups of gather_group(ncell) <= 64 consecutive
    // cells, one group per wave per pass (16 groups when a push has <= 1024 cells)
    const int lane = tid & 63, wv = tid >> 6;
    auto gather_group = [](int ncell) { return min(64, ncell / (MG_BLOCK / 64)); };
    // this lane's cell word of its wave's first group in push 0, loaded beside the state; each
    // push's loop then loads the next push's first cell word before it gathers, so that
    // round trip overlaps the current push's rows
    uint32_t v_first = 0;
    if (gather && !a.runs && lane < gather_group((int)cell_pad(a.slot_nch[0])))
        v_first = cell_at(0, wv * gather_group((int)cell_pad(a.slot_nch[0])) + lane);
    // ---- load this superbucket's entries into LDS
    for (int i = tid; i < StateLds<NW, E>::NI; i += MG_BLOCK) S.idx[i] = 0;
    if (tid == 0) {
        S.n = (FW_ABL(a) & AB_M_NO_LOAD) ? 0 : n0;
        S.overflow = 0;
        S.ndue = 0;
    }
    __syncthreads();
    const uint64_t* st = a.state + (size_t)sb * a.cap_e * PWE;
    if (!(FW_ABL(a) & AB_M_NO_LOAD)) for (int e = tid; e < n0; e += MG_BLOCK) {
        uint64_t p[PWE];
        load_words<PWE>(st + (size_t)e * PWE, p);
        const int64_t k = (int64_t)p[0], s = (int64_t)p[1];
        S.key[e] = k;
        S.slice[e] = s;
        S.flag[e] = (uint32_t)p[2];
#pragma unroll
        for (int w = 0; w < NW; w++) S.acc[w][e] = p[3 + w];
        uint32_t h = index_hash(k, s) & (StateLds<NW, E>::NI - 1);
        for (;;) {
            uint32_t expect = 0;
            if (__hip_atomic_compare_exchange_strong(&S.idx[h], &expect, 2u + (uint32_t)e, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, LDS_SCOPE))
                break;
            h = (h + 1) & (StateLds<NW, E>::NI - 1);
        }
    }
    __syncthreads();
    stm.mark(0);
    // ---- timers registered by late records in processElement
    for (int64_t r = tid; r < ntreq; r += MG_BLOCK) {
        if (a.treq[3 * r + 2] != sb) continue;
        const int e = find_or_insert<NW, E, OPS>(S, a.treq[3 * r], a.treq[3 * r + 1], a.wd);
        if (e >= 0) atomicOr(&S.flag[e], F_TIMER);
    }
    // ---- flush: AggCombiner.combine for every pending (key, slice) partial of this bucket.
    // A wave takes a group of cells (the rows ingest chunks wrote for this superbucket), scans
    // their row counts and deals the rows of the whole group over its 64 lanes, GU rows per lane
    // per pass: every lane is busy whatever the cells' sizes, and neighbouring lanes load
    // neighbouring rows.  Rows are looked up in the LDS table (first probes batched), hits
    // folded; the misses of a lane are then inserted one at a time.
    // diagnostic (AB_GSTAMPS): thread 0's cycles in row loads / first probes / fold + insert
    const bool gst = (FW_ABL(a) & AB_GSTAMPS) && stm.on && tid == 0;
    // TUMBLE and CUMULATE with up to 4 accumulator words (HOP runs k_merge_hopb or, with wider or
    // SQL-double layouts, the plain loop: its chain code leaves no registers): the gather is
    // software-pipelined over the wave's blocks of rows -- the next block's rows (and the next
    // group's cell word) are in flight while the current block is probed and folded.  Two blocks of
    // GU / 2 rows per lane take the registers of one block of GU rows.
    // (one-word layouts lost with half-size blocks: round 3, CFG2 merge 69.7 -> 74.1 us per step)
    constexpr bool PIPE = NW >= 2 && NW <= 4 && (KIND == FW_WIN_TUMBLE || KIND == FW_WIN_CUMULATE);
    if (gather && a.runs) {
        // runs (IngestArgs::runs): the superbucket's rows of every pending push as RUN_X contiguous
        // stretches per push, then the rows chunks kept in their own regions (overflow)
        // register the window timer unless already fired (AggCombiner.java:103-110); the LOCAL phase
        // keeps no timers (LocalAggCombiner.java:69-97).  UTC: fired <=> sliceEnd - 1 <= w_old, i.e.
        // sliceEnd <= fired_lim (one compare per row); shift zones take the out-of-line zone rule
        const bool utc = a.win.tz.n == 0;
        auto flags_of = [&](int64_t sl) -> uint32_t {
            const bool fired = a.local || (utc ? is_fired(sl, w_old) : tz_fired_out_of_line(a.win.tz, sl, w_old));
            return fired ? F_ACC : (F_ACC | F_TIMER);
        };
        auto fold_rows = [&](auto& row, uint32_t live) __attribute__((always_inline)) {
            constexpr int GX = std::extent<std::remove_reference_t<decltype(row)>>::value;
            if (FW_ABL(a) & AB_M_NO_HASH) {  // diagnostic: loads only
                uint64_t x = 0;
#pragma unroll
                for (int u = 0; u < GX; u++) x ^= row[u][0] ^ row[u][1] ^ row[u][PW - 1];
                asm volatile("" ::"v"(x));
                return;
            }
            if constexpr (KIND == KIND_DSWIN) {
                static_for<GX>([&](auto UU) {
                    constexpr int u = decltype(UU)::value;
                    if ((live >> u) & 1u)
                        ds_add_to_windows<NW, E>(a, S, (int64_t)row[u][0], (int64_t)row[u][1], &row[u][2], w_old, false);
                });
            } else {
                // diagnostic (AB_GSTAMPS, thread 0): [2] rows ready + hash + first probes, [4] hit folds,
                // [7] misses, [13] the whole gather loop (stamped in gather_runs' caller)
                uint64_t g0 = gst ? __builtin_amdgcn_s_memtime() : 0;
                auto gstamp = [&](int i) {
                    if (!gst) return;
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    const uint64_t g1 = __builtin_amdgcn_s_memtime();
                    stm.acc[i] += g1 - g0;
                    g0 = g1;
                };
                // batched first probes of the rows in `want`: folds the hits, returns the rest
                int ge[GX];
                auto probe_fold = [&](uint32_t want) __attribute__((always_inline)) -> uint32_t {
                    {
                        int64_t gk[GX], gs[GX];
#pragma unroll
                        for (int u = 0; u < GX; u++) {
                            gk[u] = (int64_t)row[u][0];
                            gs[u] = (int64_t)row[u][1];
                        }
                        probe_batch<NW, E, GX>(S, gk, gs, ge, GX, want);
                    }
                    uint32_t rest = 0;
                    static_for<GX>([&](auto UU) {
                        constexpr int u = decltype(UU)::value;
                        if (!((want >> u) & 1u)) return;
                        const int e = ge[u];  // -1 / -2: not decided by the batched first probe
                        if (e < 0) {
                            rest |= 1u << u;
                            return;
                        }
                        if (FW_ABL(a) & AB_M_NO_FOLDOP) return;
#pragma unroll
                        for (int w = 0; w < NW; w++)
                            if (word_on<OPS>(a.wd, w)) lds_fold(word_op<OPS>(a.wd, w), &S.acc[w][e], row[u][2 + w]);
                        atomicOr(&S.flag[e], flags_of((int64_t)row[u][1]));
                    });
                    return rest;
                };
                uint32_t miss = probe_fold(live);
                gstamp(4);
                const bool gcount = (FW_ABL(a) & AB_GSTAMPS) && stm.on && (tid >> 6) == 0;  // wave 0's row census
                if (gcount) {
                    uint32_t lv = 0, fr = 0, ud = 0;
#pragma unroll
                    for (int u = 0; u < GX; u++)
                        if ((live >> u) & 1u) {
                            lv++;
                            fr += ge[u] == -1;
                            ud += ge[u] == -2;
                        }
                    lv = wave_sum_u32(lv);
                    fr = wave_sum_u32(fr);
                    ud = wave_sum_u32(ud);
                    if (tid == 0) {
                        stm.acc[8] += lv;
                        stm.acc[9] += fr;
                        stm.acc[10] += ud;
                    }
                }
                miss = insert_fresh<NW, E, GX, OPS>(S, a.wd, row, miss, ge, flags_of);
                if (gcount) {
                    const uint32_t sl = wave_sum_u32((uint32_t)__popc(miss));
                    if (tid == 0) stm.acc[11] += sl;
                }
                gstamp(14);
                while (miss) {  // the wave loops max(popcount) times, not GX times
                    const int um = __ffs(miss) - 1;
                    miss &= miss - 1;
                    if (gst) stm.acc[12]++;
                    uint64_t r[PW];
                    static_for<GX>([&](auto UU) {
                        constexpr int u = decltype(UU)::value;
                        if (u == um) {
#pragma unroll
                            for (int w = 0; w < PW; w++) r[w] = row[u][w];
                        }
                    });
                    const uint32_t fl = flags_of((int64_t)r[1]);
                    bool ins = false;
                    const int e = find_or_insert<NW, E, OPS>(S, (int64_t)r[0], (int64_t)r[1], a.wd, &r[2], fl, &ins);
                    if (e < 0 || ins || (FW_ABL(a) & AB_M_NO_FOLDOP)) continue;
#pragma unroll
                    for (int w = 0; w < NW; w++)
                        if (word_on<OPS>(a.wd, w)) lds_fold(word_op<OPS>(a.wd, w), &S.acc[w][e], r[2 + w]);
                    atomicOr(&S.flag[e], fl);
                }
                gstamp(7);
            }
        };
        // TUMBLE / CUMULATE up to 4 words: software-pipelined (two blocks in flight); the others
        // (HOP chains, DataStream windows) leave no registers for a second block
        constexpr bool RP = NW <= 4 && (KIND == FW_WIN_TUMBLE || KIND == FW_WIN_CUMULATE);
        // one-word TUMBLE: one block of 4 rows per lane (measured round 5, CFG2 runs flush 144.5 ->
        // 128.7 us; 3 rows: 131.8, 2 rows: 133.3, 5 rows: 130.1, 6 rows: 141.7; the freed registers go to the probe loop); CFG4 (two
        // words, 197 -> 201 us) and CFG5 (CUMULATE, 322 -> 370 us) keep two blocks of half of
        // mg_rows_in_flight
        constexpr bool ONE_BLOCK = NW == 1 && KIND == FW_WIN_TUMBLE;
        constexpr int GR = !RP ? GU : ONE_BLOCK ? 4 : GU / 2 > 0 ? GU / 2 : 1;
        constexpr int GD = !RP ? 1 : ONE_BLOCK ? 1 : 2;
        const uint64_t gl0 = gst ? __builtin_amdgcn_s_memtime() : 0;
        gather_runs<NW, GR, GF, GD>(a, sb, pend, fold_rows);
        if (gst) stm.acc[13] += __builtin_amdgcn_s_memtime() - gl0;
        uint32_t ovf = run_overflow(a, sb, pend);
        while (ovf) {
            const int pi = __ffs(ovf) - 1;
            ovf &= ovf - 1;
            gather_cells_push<NW, GU, GF>(a, sb, pi, fold_rows);
        }
    } else if (PIPE && gather) {
        constexpr int GP = NW == 1 ? GU : GU / 2 > 0 ? GU / 2 : 1;  // one word: two full blocks fit
        // register the window timer unless already fired (AggCombiner.java:103-110); the LOCAL phase
        // keeps no timers; shift zones take the out-of-line zone rule
        const bool utc = a.win.tz.n == 0;
        auto flags_of = [&](int64_t sl) -> uint32_t {
            const bool fired = a.local || (utc ? is_fired(sl, w_old) : tz_fired_out_of_line(a.win.tz, sl, w_old));
            return fired ? F_ACC : (F_ACC | F_TIMER);
        };
        auto ngroups_of = [&](int64_t p) {
            const int nc = (int)cell_pad(a.slot_nch[p]);
            return nc / gather_group(nc);
        };
        auto norm = [&](int64_t& p, int& q) {  // the first group (p, q) of this wave that exists
            while (p < pend && q >= ngroups_of(p)) {
                p++;
                q = wv;
            }
        };
        auto fpos = [&](int64_t p, int q) { return q * gather_group((int)cell_pad(a.slot_nch[p])) + lane; };
        auto cword = [&](int64_t p, int q) -> uint32_t {
            return lane < gather_group((int)cell_pad(a.slot_nch[p])) ? cell_at(p, fpos(p, q)) : 0u;
        };
        // current block: group (cp) with scan cg, rows r0 + [0, 64 * GP); next group (np, nq) with
        // its cell word vn loaded one group ahead
        CellGroup cg;
        cg.tot = cg.excl = cg.adj = cg.fmt = 0;
        int64_t cp = 0;
        uint32_t r0 = 0;
        int64_t np = 0;
        int nq = wv;
        norm(np, nq);
        uint32_t vn = np < pend ? ((np == 0 && nq == wv) ? v_first : cword(np, nq)) : 0u;
        auto next_block = [&]() -> bool {
            r0 += 64 * GP;
            while (r0 >= cg.tot) {
                if (np >= pend) return false;
                const uint32_t vc = vn;
                const int f = fpos(np, nq);
                cp = np;
                nq += MG_BLOCK / 64;
                norm(np, nq);
                vn = np < pend ? cword(np, nq) : 0u;
                cg = cell_group(vc, f, CH);
                r0 = 0;
            }
            return true;
        };
        auto process = [&](auto& row, uint32_t live) {
            constexpr int GX = std::extent<std::remove_reference_t<decltype(row)>>::value;
            if (FW_ABL(a) & AB_M_NO_HASH) {  // diagnostic: loads only
                uint64_t x = 0;
#pragma unroll
                for (int u = 0; u < GX; u++) x ^= row[u][0] ^ row[u][1] ^ row[u][PW - 1];
                asm volatile("" ::"v"(x));
                return;
            }
            int ge[GX];
            {
                int64_t gk[GX], gs[GX];
#pragma unroll
                for (int u = 0; u < GX; u++) {
                    gk[u] = (int64_t)row[u][0];
                    gs[u] = (int64_t)row[u][1];
                }
                probe_batch<NW, E, GX>(S, gk, gs, ge);
            }
            uint32_t miss = 0;
            static_for<GX>([&](auto UU) {
                constexpr int u = decltype(UU)::value;
                if (!((live >> u) & 1u)) return;
                const int e = ge[u];
                if (e < 0) {
                    miss |= 1u << u;
                    return;
                }
                if (FW_ABL(a) & AB_M_NO_FOLDOP) return;
#pragma unroll
                for (int w = 0; w < NW; w++)
                    if (word_on<OPS>(a.wd, w)) lds_fold(word_op<OPS>(a.wd, w), &S.acc[w][e], row[u][2 + w]);
                atomicOr(&S.flag[e], flags_of((int64_t)row[u][1]));
            });
            while (miss) {
                const int um = __ffs(miss) - 1;
                miss &= miss - 1;
                uint64_t r[PW];
                static_for<GX>([&](auto UU) {
                    constexpr int u = decltype(UU)::value;
                    if (u == um) {
#pragma unroll
                        for (int w = 0; w < PW; w++) r[w] = row[u][w];
                    }
                });
                const uint32_t fl = flags_of((int64_t)r[1]);
                bool ins = false;
                const int e = find_or_insert<NW, E, OPS>(S, (int64_t)r[0], (int64_t)r[1], a.wd, &r[2], fl, &ins);
                if (e < 0 || ins || (FW_ABL(a) & AB_M_NO_FOLDOP)) continue;
#pragma unroll
                for (int w = 0; w < NW; w++)
                    if (word_on<OPS>(a.wd, w)) lds_fold(word_op<OPS>(a.wd, w), &S.acc[w][e], r[2 + w]);
                atomicOr(&S.flag[e], fl);
            }
        };
        uint64_t ra[GP][PW], rb[GP][PW];
        uint32_t la = 0, lb = 0;
        bool ha = next_block();
        if (ha) la = load_group_rows<NW, GP, GF>(a, cp, cg, r0, sb, ra);
        while (ha) {  // unrolled by two: the buffers alternate, no copies (a copy would wait for the loads)
            const bool hb = next_block();
            if (hb) lb = load_group_rows<NW, GP, GF>(a, cp, cg, r0, sb, rb);
            process(ra, la);
            if (!hb) break;
            ha = next_block();
            if (ha) la = load_group_rows<NW, GP, GF>(a, cp, cg, r0, sb, ra);
            process(rb, lb);
        }
    } else if (gather) {
        for (int64_t pi = 0; pi < pend; pi++) {
            const int ncell = (int)cell_pad(a.slot_nch[pi]);
            const int G = gather_group(ncell);
            const int ngroups = ncell / G;
            for (int g = wv; g < ngroups; g += MG_BLOCK / 64) {
                const int f = g * G + lane;
                uint64_t gc0 = gst ? __builtin_amdgcn_s_memtime() : 0;
                const uint32_t v = lane >= G ? 0u : g == wv ? v_first : cell_at(pi, f);
                    if (g == wv) {  // the next push's first cell word, in flight during this push
                        v_first = 0;
                        if (pi + 1 < pend) {
                            const int G1 = gather_group((int)cell_pad(a.slot_nch[pi + 1]));
                            if (lane < G1) v_first = cell_at(pi + 1, wv * G1 + lane);
                        }
                    }
                if (gst) {  // diagnostic: cell word wait
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    const uint64_t g1 = __builtin_amdgcn_s_memtime();
                    stm.acc[13] += g1 - gc0;
                    gc0 = g1;
                }
                const CellGroup cg = cell_group(v, f, CH);
                const uint32_t tot = cg.tot;
                if (gst) stm.acc[14] += __builtin_amdgcn_s_memtime() - gc0;  // diagnostic: scan
                for (uint32_t r0 = 0; r0 < tot; r0 += 64 * GU) {
                    uint64_t row[GU][PW];
                    uint64_t g0 = gst ? __builtin_amdgcn_s_memtime() : 0;
                    const uint32_t live = load_group_rows<NW, GU, GF>(a, pi, cg, r0, sb, row);
                    if (gst) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        const uint64_t g1 = __builtin_amdgcn_s_memtime();
                        stm.acc[2] += g1 - g0;
                        g0 = g1;
                    }
                    if (FW_ABL(a) & AB_M_NO_HASH) {  // diagnostic: loads only
                        uint64_t x = 0;
#pragma unroll
                        for (int u = 0; u < GU; u++) x ^= row[u][0] ^ row[u][1] ^ row[u][PW - 1];
                        asm volatile("" ::"v"(x));  // keeps the loads
                        continue;
                    }
                    if constexpr (KIND == KIND_DSWIN) {
                        static_for<GU>([&](auto UU) {
                            constexpr int u = decltype(UU)::value;
                            if ((live >> u) & 1u)
                                ds_add_to_windows<NW, E>(a, S, (int64_t)row[u][0], (int64_t)row[u][1], &row[u][2], w_old, false);
                        });
                        continue;
                    }
                    // register the window timer unless already fired (AggCombiner.java:103-110);
                    // the LOCAL phase keeps no timers (LocalAggCombiner.java:69-97); shift zones take
                    // the out-of-line zone rule
                    const bool utc = a.win.tz.n == 0;
                    auto flags_of = [&](int64_t sl) -> uint32_t {
                        const bool fired = a.local || (utc ? is_fired(sl, w_old) : tz_fired_out_of_line(a.win.tz, sl, w_old));
                        return fired ? F_ACC : (F_ACC | F_TIMER);
                    };
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
                    uint32_t miss = 0;
                    static_for<GU>([&](auto UU) {
                        constexpr int u = decltype(UU)::value;
                        if (!((live >> u) & 1u)) return;
                        const int e = ge[u];  // -1 / -2: not found by the batched first probe
                        if (e < 0) {
                            miss |= 1u << u;
                            return;
                        }
                        if (FW_ABL(a) & AB_M_NO_FOLDOP) return;
#pragma unroll
                        for (int w = 0; w < NW; w++)
                            if (word_on<OPS>(a.wd, w)) lds_fold(word_op<OPS>(a.wd, w), &S.acc[w][e], row[u][2 + w]);
                        atomicOr(&S.flag[e], flags_of((int64_t)row[u][1]));
                    });
                    const uint64_t gm0 = gst ? __builtin_amdgcn_s_memtime() : 0;
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
                        const int e = find_or_insert<NW, E, OPS>(S, k, sl, a.wd, &r[2], fl, &ins);
                        if (e < 0 || ins || (FW_ABL(a) & AB_M_NO_FOLDOP)) continue;
#pragma unroll
                        for (int w = 0; w < NW; w++)
                            if (word_on<OPS>(a.wd, w)) lds_fold(word_op<OPS>(a.wd, w), &S.acc[w][e], r[2 + w]);
                        atomicOr(&S.flag[e], fl);
                    }
                    if (gst) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        const uint64_t g1 = __builtin_amdgcn_s_memtime();
                        stm.acc[7] += g1 - g0;
                        stm.acc[15] += g1 - gm0;
                    }
                }
            }
        }
    }
    __syncthreads();
    stm.mark(1);
    if (gather && a.runs) run_release(a, sb, pend);
    // ---- DataStream late-fire rows: an element for a fired window that is not cleaned yet fires
    // that window at once with the element added (EventTimeTrigger.onElement -> FIRE,
    // WindowOperator.java:418-426).  Every such element emits the window's contents as of its own
    // arrival: the state before this flush plus the late elements of the same (key, window) up to
    // it (arrival ordinals).  Pass 1 emits from the unchanged state, pass 2 adds the elements to
    // all their live windows.  The superbucket's rows are listed in LDS first (one scan of the
    // launch's rows), so both passes cost O(rows of this superbucket^2 x windows per row); beyond
    // LF_LDS rows the passes scan the launch's rows instead.
    if (KIND == KIND_DSWIN && gather && nlf > 0) {
        constexpr int LF_LDS = 1024;
        __shared__ int32_t s_lf[LF_LDS];
        __shared__ int s_nlf;
        if (tid == 0) s_nlf = 0;
        __syncthreads();
        for (int64_t r = tid; r < nlf; r += MG_BLOCK)
            if ((uint32_t)a.lfire[(size_t)r * LFW + 2] == (uint32_t)sb) {
                const int q = atomicAdd(&s_nlf, 1);
                if (q < LF_LDS) s_lf[q] = (int32_t)r;
            }
        __syncthreads();
        const bool listed = s_nlf <= LF_LDS;
        const int64_t nscan = listed ? (int64_t)s_nlf : nlf;
        auto lf_row = [&](int64_t i) { return a.lfire + (size_t)(listed ? (int64_t)s_lf[i] : i) * LFW; };
        const WinDesc& w = a.win;
        for (int64_t r = tid; r < nscan; r += MG_BLOCK) {
            const uint64_t* p = lf_row(r);
            if ((uint32_t)p[2] != (uint32_t)sb) continue;
            const int64_t k = (int64_t)p[0], pe = (int64_t)p[1];
            const uint32_t ord = (uint32_t)(p[2] >> 32);
            const int64_t e0 = ds_first_window_end(w, pe);
            for (int i = 0; i < w.n_win; i++) {
                const int64_t e = wsub(e0, (int64_t)i * w.slide);
                if (!ds_window_holds_pane(w, e, pe)) break;
                if (ds_cleanup_time(w, e) <= w_old || !is_fired(e, w_old)) continue;
                uint64_t acc[NW];
                const int es = find_entry(S, k, e);
                if (es >= 0 && (S.flag[es] & F_ACC)) {
#pragma unroll
                    for (int q = 0; q < NW; q++) acc[q] = S.acc[q][es];
                } else {
                    acc_identity<NW>(a.wd, acc);
                }
                for (int64_t q2 = 0; q2 < nscan; q2++) {
                    const uint64_t* o = lf_row(q2);
                    if ((uint32_t)o[2] != (uint32_t)sb || (int64_t)o[0] != k || (uint32_t)(o[2] >> 32) > ord) continue;
                    if (!ds_pane_in_window(w, (int64_t)o[1], e)) continue;
#pragma unroll
                    for (int q = 0; q < NW; q++)
                        if (q < a.wd.nw && !is_byword(a.wd.op[q])) acc[q] = reg_fold(a.wd.op[q], acc[q], o[3 + q]);
                    if (a.ad.by_prev >= 0) {  // minBy / maxBy pair (by_fold in registers)
                        const int wv = a.ad.w0[0], wo = a.ad.first_word;
                        uint64_t cv = 0, co = 0;
#pragma unroll
                        for (int q = 0; q < NW; q++) {
                            if (q == wv) cv = acc[q];
                            if (q == wo) co = acc[q];
                        }
                        if (by_better(a.wd.op[wv], a.wd.op[wo], o[3 + wv], o[3 + wo], cv, co)) {
#pragma unroll
                            for (int q = 0; q < NW; q++)
                                if (q == wv || q == wo) acc[q] = o[3 + q];
                        }
                    }
                }
                emit_row<NW, false>(a, sb, &s_emit, k, e, acc);
            }
        }
        __syncthreads();
        for (int64_t r = tid; r < nscan; r += MG_BLOCK) {
            const uint64_t* p = lf_row(r);
            if ((uint32_t)p[2] != (uint32_t)sb) continue;
            uint64_t v[NW];
#pragma unroll
            for (int q = 0; q < NW; q++) v[q] = p[3 + q];
            ds_add_to_windows<NW, E>(a, S, (int64_t)p[0], (int64_t)p[1], v, w_old, true);
        }
        __syncthreads();
    }
    // ---- fire: InternalTimerServiceImpl.tryAdvanceWatermark (:328-348) -> WindowAggOperator
    // .onTimer -> fireWindow + clearWindow.  One pass over the entries whose timer is due; HOP and
    // CUMULATE follow their timer chains per key (no timestamp rounds, see fire_*_chain).
    if (do_fire && !(FW_ABL(a) & AB_M_NO_FIRE)) {
        const int n = min(S.n, E);
        for (int e = tid; e < n; e += MG_BLOCK)
            if (KIND == KIND_DSWIN ? (((S.flag[e] & F_TIMER) && is_fired(S.slice[e], W)) ||
                                      ((S.flag[e] & F_CLEAN) && ds_cleanup_time(a.win, S.slice[e]) <= W))
                                   : ((S.flag[e] & F_TIMER) && win_fired(a.win, S.slice[e], W))) {
                const int q = wave_claim(&S.ndue);
                if (q < E) S.due[q] = (uint16_t)e;
            }
        __syncthreads();
        const int nd = min(S.ndue, E);
        // due entries are dealt to every wave (fire_deal)
        if (KIND == FW_WIN_CUMULATE || KIND == FW_WIN_HOP) {
            for (int b0 = 0; b0 < nd; b0 += MG_BLOCK) {
                const int q = fire_deal(b0, nd, tid);
                if (q >= nd) continue;
                if (KIND == FW_WIN_CUMULATE) mark_cumulate_successor<NW, E>(a, W, S, S.due[q]);
                else mark_hop_successor<NW, E>(a, W, S, S.due[q]);
            }
            __syncthreads();
        }
        stm.mark(6);
        uint32_t nf = 0;
        uint64_t fst[4] = {0, 0, 0, 0};
        const bool fs = (FW_ABL(a) & AB_FSTAMPS) != 0;
        for (int b0 = 0; b0 < nd; b0 += MG_BLOCK) {
            const int q = fire_deal(b0, nd, tid);
            if (q >= nd) continue;
            const int e = S.due[q];
            if (KIND == KIND_DSWIN) {
                nf += fire_ds<NW, E>(a, W, S, e, sb, &s_emit);
            } else if (KIND == FW_WIN_TUMBLE) {
                nf += fire_tumble<NW, E, Q, OPS>(a, S, e, sb, &s_emit);
            } else if (KIND == FW_WIN_HOP) {
                if (!(S.flag[e] & F_NOTHEAD)) nf += fire_hop_chain<NW, E, Q, OPS>(a, W, S, e, sb, &s_emit, fs ? fst : nullptr);
            } else {
                if (!(S.flag[e] & F_NOTHEAD)) nf += fire_cumulate_chain<NW, E, Q, OPS>(a, W, S, e, sb, &s_emit);
            }
        }
        if (fs && a.stamps) {
            const uint32_t nfw = wave_sum_u32(nf);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                uint64_t x = fst[i];
                for (int d = 32; d > 0; d >>= 1) x += (uint64_t)__shfl_xor((long long)x, d, 64);
                if ((tid & 63) == 0) atomicAdd(&a.stamps[8 + i], (unsigned long long)x);
            }
            if ((tid & 63) == 0) atomicAdd(&a.stamps[12], (unsigned long long)nfw);
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
    } else if (!(FW_ABL(a) & AB_M_NO_WB)) {
        for (int e = tid; e < n; e += MG_BLOCK) {
            const uint32_t f0 = S.flag[e];
            const uint32_t f = f0 & ((f0 & F_EXPIRE) ? F_TIMER : (F_ACC | F_TIMER | F_CLEAN));
            if (!f) continue;
            const int pos = wave_claim(&s_nlive);
            uint64_t p[PWE];
            p[0] = (uint64_t)S.key[e];
            p[1] = (uint64_t)S.slice[e];
            p[2] = f;
            if (Q || (KIND == KIND_DSWIN && a.wd.has_ord)) {
                uint64_t v[NW];
#pragma unroll
                for (int w = 0; w < NW; w++) v[w] = S.acc[w][e];
#pragma unroll
                for (int w = 0; w < NW; w++) p[3 + w] = w < a.wd.nw ? q_normalise(a.wd, w, v) : v[w];
                // a new DataStream window state: its first element is retained by the host shim;
                // minBy / maxBy: a changed arg is retained, the one it replaced released
                if (KIND == KIND_DSWIN && (f & F_ACC) && a.ad.by_prev >= 0) {
                    const uint64_t o = v[a.ad.first_word], pv = v[a.ad.by_prev];
                    if (o != pv) {
                        push_ordev(a, (int64_t)o);
                        if (pv != ~0ull) push_ordev(a, ORDEV_RELEASE | (int64_t)pv);
                        p[3 + a.ad.by_prev] = o;
                    }
                } else if (KIND == KIND_DSWIN && (f0 & F_NEW) && (f & F_ACC) && a.ad.first_word >= 0) {
                    push_ordev(a, (int64_t)v[a.ad.first_word]);
                }
            } else {
#pragma unroll
                for (int w = 0; w < NW; w++) p[3 + w] = S.acc[w][e];
            }
            store_words<PWE>(so + (size_t)pos * PWE, p);
            if (f & F_TIMER) lnm = min(lnm, S.slice[e]);
            if (KIND == KIND_DSWIN && (f & F_CLEAN)) lnm = min(lnm, wadd(ds_cleanup_time(a.win, S.slice[e]), 1));
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
        // state traffic of this superbucket: entries loaded + entries written back
        __hip_atomic_fetch_add(&c->state_moved, (uint64_t)(n0 + (a.local ? 0 : s_nlive)), __ATOMIC_RELAXED, DEV_SCOPE);
        __hip_atomic_fetch_max(&c->peak_entries, (uint64_t)max(S.n, 0), __ATOMIC_RELAXED, DEV_SCOPE);
        if (S.overflow) __hip_atomic_fetch_or(&c->error, ERR_STATE, __ATOMIC_RELAXED, DEV_SCOPE);
    }
    __syncthreads();
    stm.mark(3);
    }  // superbuckets of this workgroup (s_tk was published before the last barrier)
    stm.flush(a.stamps);
    merge_ticket(a, W);
}

// persistent grid of the merge kernel: one workgroup per CU, at most one per superbucket
static unsigned merge_grid(int n_sb) {
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
    }
    return (unsigned)(n_sb < n_cu ? n_sb : n_cu);
}

// the accumulator layouts with a compiled variant per accumulator width (the others, and every SQL
// MIN/MAX(DOUBLE) query, run the OPS_ANY variant): the built-in aggregates' common combinations
template <int NW> struct MergeLayouts;
template <> struct MergeLayouts<1> {  // COUNT(*) / SUM, MAX, MIN, SUM(DOUBLE)
    static constexpr uint32_t L[] = {ops_pack({W_SUM_I}), ops_pack({W_MAX_I}), ops_pack({W_MIN_I}), ops_pack({W_SUM_F})};
};
template <> struct MergeLayouts<2> {  // AVG / SUM+AVG (DOUBLE, BIGINT), COUNT(*) + SUM / MAX / MIN
    static constexpr uint32_t L[] = {ops_pack({W_SUM_F, W_SUM_I}), ops_pack({W_SUM_I, W_SUM_I}),
                                     ops_pack({W_SUM_I, W_MAX_I}), ops_pack({W_SUM_I, W_MIN_I})};
};
template <> struct MergeLayouts<4> {  // COUNT(*), SUM, MIN, MAX
    static constexpr uint32_t L[] = {ops_pack({W_SUM_I, W_SUM_I, W_MIN_I, W_MAX_I})};
};
template <> struct MergeLayouts<8> {
    static constexpr uint32_t L[] = {OPS_ANY};
};

template <int NW, bool Q, uint32_t OPS, int GF = 0>
static void merge_launch(const MergeArgs& a, hipStream_t s) {
    constexpr int ET = mg_entries(NW, FW_WIN_TUMBLE), EH = mg_entries(NW, FW_WIN_HOP), EC = mg_entries(NW, FW_WIN_CUMULATE);
    switch (a.win.kind) {
        case FW_WIN_TUMBLE: hipLaunchKernelGGL((k_merge_fire<NW, ET, Q, FW_WIN_TUMBLE, OPS, GF>), dim3(merge_grid(a.n_sb)), dim3(MG_BLOCK), 0, s, a); break;
        case FW_WIN_HOP: hipLaunchKernelGGL((k_merge_fire<NW, EH, Q, FW_WIN_HOP, OPS, GF>), dim3(merge_grid(a.n_sb)), dim3(MG_BLOCK), 0, s, a); break;
        default: hipLaunchKernelGGL((k_merge_fire<NW, EC, Q, FW_WIN_CUMULATE, OPS, GF>), dim3(merge_grid(a.n_sb)), dim3(MG_BLOCK), 0, s, a); break;
    }
}

template <int NW, int I>
static bool merge_layout_launch(const MergeArgs& a, uint32_t lay, hipStream_t s) {
    constexpr int N = (int)(sizeof(MergeLayouts<NW>::L) / sizeof(uint32_t));
    if constexpr (I >= N) {
        return false;
    } else {
        constexpr uint32_t L = MergeLayouts<NW>::L[I];
        if (L != OPS_ANY && lay == L) {
            // compact rows come with the one-word layouts (fw_api.hip plans narrow for them alone)
            if constexpr (NW == 1) {
                if (a.compact) {
                    merge_launch<NW, false, L, GF_COMPACT>(a, s);
                    return true;
                }
            }
            merge_launch<NW, false, L>(a, s);
            return true;
        }
        return merge_layout_launch<NW, I + 1>(a, lay, s);
    }
}

template <int NWP, int GF>
static void merge_hopb_launch(const MergeArgs& a, hipStream_t s);  // fw_merge_hopb.h

template <int NW>
hipError_t merge_nw(const MergeArgs& a, hipStream_t s) {
    // more superbuckets than the ingest partitions into (KeySpace.pass_log2): the run-time layout
    // variants, which route every partial row again (PS)
    const bool ps = a.ks.pass_log2 > 0;
    if (a.win.hopb) {  // SQL HOP with block state
        if constexpr (NW <= 2) {
            if (a.cap_e != mg_entries(NW, KIND_HOPB)) return hipErrorInvalidValue;
            if (ps) merge_hopb_launch<NW, GF_PASS>(a, s);
            else if (NW == 1 && a.compact) merge_hopb_launch<NW, GF_COMPACT>(a, s);
            else merge_hopb_launch<NW, 0>(a, s);
            return hipGetLastError();
        } else {
            return hipErrorInvalidValue;
        }
    }
    if (a.win.ds) {  // DataStream: per-window state, no SQL MIN/MAX(DOUBLE) word groups
        if (a.wd.has_q) return hipErrorInvalidValue;
        constexpr int E = mg_entries(NW, KIND_DSWIN);
        if (ps) hipLaunchKernelGGL((k_merge_fire<NW, E, false, KIND_DSWIN, OPS_ANY, GF_PASS>), dim3(merge_grid(a.n_sb)), dim3(MG_BLOCK), 0, s, a);
        else hipLaunchKernelGGL((k_merge_fire<NW, E, false, KIND_DSWIN, OPS_ANY, 0>), dim3(merge_grid(a.n_sb)), dim3(MG_BLOCK), 0, s, a);
        return hipGetLastError();
    }
    // the planner sized the superbuckets for mg_entries(nw, kind) entries (fw_api.hip)
    if (a.cap_e != mg_entries(NW, a.win.kind)) return hipErrorInvalidValue;
    if (ps) {
        if (a.wd.has_q) merge_launch<NW, true, OPS_ANY, GF_PASS>(a, s);
        else merge_launch<NW, false, OPS_ANY, GF_PASS>(a, s);
    } else if (a.wd.has_q) {
        merge_launch<NW, true, OPS_ANY>(a, s);
    } else if (!merge_layout_launch<NW, 0>(a, ops_layout(a.wd), s)) {
        merge_launch<NW, false, OPS_ANY>(a, s);
    }
    return hipGetLastError();
}

}  // namespace fw
