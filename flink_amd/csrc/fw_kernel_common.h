// fw_kernel_common.h -- device helpers shared by the kernel translation units of libflinkwin
// (fw_kernels.hip, k_ingest_nv*.hip, k_merge_nw*.hip).  Split so the template instantiations of
// the ingest and merge kernels compile in parallel.
#pragma once


#include <utility>


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


// value of one accumulator word for a single non-NULL record (accumulate on the identity);
// `ord` >= 1 is the record's arrival ordinal within the flush (W_Q*, W_DN* words), `gord` its
// global arrival ordinal push_seq << 32 | row (W_FIRST)
__device__ __forceinline__ uint64_t record_word(int32_t op, uint64_t v, uint32_t ord, uint64_t gord = 0) {
    switch (op) {
        case W_CNT: return 1;
        case W_MIN_D:
        case W_MAX_D: return (uint64_t)dkey(v);
        case W_QMIN:
        case W_QMAX: return f64_isnan(v) ? word_identity(op) : f64_iszero(v) ? 0ull : (uint64_t)dkey(v);
        case W_QFIRST: return ((uint64_t)ord << 32) | (f64_isnan(v) ? (v >> 32) : 0ull);
        case W_QNANLO: return f64_isnan(v) ? (((uint64_t)ord << 32) | (v & 0xFFFFFFFFull)) : Q_EMPTY;
        case W_QZERO: return f64_iszero(v) ? (((uint64_t)ord << 1) | (v >> 63)) : Q_EMPTY;
        case W_FIRST: return gord;
        case W_DNHI: return f64_isnan(v) ? (((uint64_t)ord << 32) | (v >> 32)) : 0ull;
        case W_DNLO: return f64_isnan(v) ? (((uint64_t)ord << 32) | (v & 0xFFFFFFFFull)) : 0ull;
        case W_BYMAX_D:
        case W_BYMIN_D: return (uint64_t)dkey(f64_isnan(v) ? 0x7FF8000000000000ull : v);
        case W_BYO_FIRST:
        case W_BYO_LAST: return gord;
        case W_BYPREV: return ~0ull;
        default: return v;  // SUM_I, SUM_F (bits), MIN_I, MAX_I, CNTV, BYMAX_I, BYMIN_I
    }
}
// a record's word, honouring the word's NULL gate (null_slots: bit s = value slot s is NULL)
__device__ __forceinline__ uint64_t gated_word(const WordDesc& wd, int w, uint64_t v, uint32_t null_slots, uint32_t ord,
                                               uint64_t gord = 0) {
    const int32_t g = wd.gate[w];
    if (g >= 0 && ((null_slots >> g) & 1u)) return word_identity(wd.op[w]);
    return record_word(wd.op[w], v, ord, gord);
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
        case W_QZERO:
        case W_FIRST: __hip_atomic_fetch_min(slot, v, __ATOMIC_RELAXED, LDS_SCOPE); break;
        case W_DNHI:
        case W_DNLO: __hip_atomic_fetch_max(slot, v, __ATOMIC_RELAXED, LDS_SCOPE); break;
        case W_BYMAX_I:
        case W_BYMIN_I:
        case W_BYMAX_D:
        case W_BYMIN_D:
        case W_BYO_FIRST:
        case W_BYO_LAST:
        case W_BYPREV: break;  // pair words: by_fold (fw_merge_impl.h)
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
        case W_QZERO:
        case W_FIRST: return a < b ? a : b;
        case W_DNHI:
        case W_DNLO: return a > b ? a : b;
        // pair words (by_fold): folded only onto their identity, when an entry is created
        case W_BYMIN_I:
        case W_BYMIN_D: return (int64_t)a < (int64_t)b ? a : b;
        case W_BYO_FIRST:
        case W_BYO_LAST: return b;
        case W_BYPREV: return a;
        default: return (int64_t)a > (int64_t)b ? a : b;  // also W_BYMAX_*
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
        case W_DNHI:
        case W_DNLO: return v & 0xFFFFFFFFull;  // ordinal 0: earlier than any later flush's NaN
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
static __device__ __noinline__ void merge_q_groups(const WordDesc& wd, const AggDesc& ad, uint64_t* acc, const uint64_t* other) {
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

// word w of a merge-kernel variant with layout OPS: present?  its op (class representative)?
template <uint32_t OPS>
__device__ __forceinline__ bool word_on(const WordDesc& wd, int w) {
    if constexpr (OPS == OPS_ANY) return w < wd.nw;
    else return ((OPS >> (4 * w)) & 15u) != OPS_NONE;
}
template <uint32_t OPS>
__device__ __forceinline__ int32_t word_op(const WordDesc& wd, int w) {
    if constexpr (OPS == OPS_ANY) return wd.op[w];
    else return (int32_t)((OPS >> (4 * w)) & 15u);
}

template <int NW, bool Q, uint32_t OPS = OPS_ANY>
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
            if (word_on<OPS>(wd, w)) acc[w] = reg_fold(word_op<OPS>(wd, w), acc[w], other[w]);
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

// 16-B and 8-B stores of the bulk outputs (partial rows, state write-back, result slabs).  Plain
// stores: write-through (sc1) versions, to spare the kernel boundary the dirty L2 lines, were measured
// out in round 5 (CFG2 runs ingest 67 -> 116 us, CFG4 78 -> 152 us; the step gaps did not shrink).
__device__ __forceinline__ void st16(void* p, uint64_t lo, uint64_t hi) { *(ulonglong2*)p = make_ulonglong2(lo, hi); }
__device__ __forceinline__ void st8(void* p, uint64_t v) { *(uint64_t*)p = v; }

// wave-level reductions: one LDS atomic per wave instead of one per lane (same-address LDS
// atomics serialise lane by lane)
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = min(v, (int64_t)__shfl_xor((long long)v, d, 64));
    return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = max(v, (int64_t)__shfl_xor((long long)v, d, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d, 64);
    return v;
}
// Whole-wave reductions on DPP (no LDS): butterfly inside each 16-lane row (quad perms, half-row and
// row mirrors), then row_bcast:15 / row_bcast:31 carry the rows into lane 63, read back as a scalar.
// Every lane of the wave must be active.  (The __shfl_xor butterflies above go through
// ds_bpermute: six dependent LDS round trips per 32-bit step.)
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t old, uint64_t v) {
    const uint32_t lo = dpp_u32<CTRL, RM>((uint32_t)old, (uint32_t)v);
    const uint32_t hi = dpp_u32<CTRL, RM>((uint32_t)(old >> 32), (uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
template <typename T, typename Op>
__device__ __forceinline__ T wred(T v, T ident, Op op) {
    if constexpr (sizeof(T) == 8) {
        v = op(v, (T)dpp_u64<0xB1, 0xf>((uint64_t)ident, (uint64_t)v));   // quad_perm [1,0,3,2]
        v = op(v, (T)dpp_u64<0x4E, 0xf>((uint64_t)ident, (uint64_t)v));   // quad_perm [2,3,0,1]
        v = op(v, (T)dpp_u64<0x141, 0xf>((uint64_t)ident, (uint64_t)v));  // row_half_mirror
        v = op(v, (T)dpp_u64<0x140, 0xf>((uint64_t)ident, (uint64_t)v));  // row_mirror
        v = op(v, (T)dpp_u64<0x142, 0xa>((uint64_t)ident, (uint64_t)v));  // row_bcast:15 -> rows 1, 3
        v = op(v, (T)dpp_u64<0x143, 0xc>((uint64_t)ident, (uint64_t)v));  // row_bcast:31 -> rows 2, 3
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, 63);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), 63);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        v = op(v, (T)dpp_u32<0xB1, 0xf>((uint32_t)ident, (uint32_t)v));
        v = op(v, (T)dpp_u32<0x4E, 0xf>((uint32_t)ident, (uint32_t)v));
        v = op(v, (T)dpp_u32<0x141, 0xf>((uint32_t)ident, (uint32_t)v));
        v = op(v, (T)dpp_u32<0x140, 0xf>((uint32_t)ident, (uint32_t)v));
        v = op(v, (T)dpp_u32<0x142, 0xa>((uint32_t)ident, (uint32_t)v));
        v = op(v, (T)dpp_u32<0x143, 0xc>((uint32_t)ident, (uint32_t)v));
        return (T)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    }
}
__device__ __forceinline__ int64_t wred_min_i64(int64_t v) {
    return wred<int64_t>(v, INT64_MAX, [](int64_t a, int64_t b) { return a < b ? a : b; });
}
__device__ __forceinline__ int64_t wred_max_i64(int64_t v) {
    return wred<int64_t>(v, INT64_MIN, [](int64_t a, int64_t b) { return a > b ? a : b; });
}
__device__ __forceinline__ uint32_t wred_sum_u32(uint32_t v) {
    return wred<uint32_t>(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ int64_t wred_sum_i64(int64_t v) {
    return wred<int64_t>(v, 0, [](int64_t a, int64_t b) { return a + b; });
}

// PF_PACK fields for the next flush epoch from a push's key and accumulator ranges (fw_internal.h):
// each field twice the measured span (kb + rb + vb = 64, 2 <= rb <= 8, the spare bits widen the
// accumulator field: sums drift), the bases centred on the ranges.  Returns the fields word (0: the
// spans do not fit one word); no rows seen (kmn > kmx): the previous word stands.
__device__ __forceinline__ uint32_t pack_fields(int64_t kmn, int64_t kmx, int64_t vmn, int64_t vmx, int64_t* kbase,
                                                int64_t* vbase, uint32_t prev) {
    if (kmn > kmx) return prev;
    const uint64_t ks = (uint64_t)kmx - (uint64_t)kmn, vs = (uint64_t)vmx - (uint64_t)vmn;
    const uint32_t kb = (ks ? 64u - (uint32_t)__clzll((long long)ks) : 1u) + 1u;
    uint32_t vb = (vs ? 64u - (uint32_t)__clzll((long long)vs) : 1u) + 1u;
    if (kb + vb + 2u > 64u) return 0u;
    const uint32_t rb = min(64u - kb - vb, 8u);
    vb = 64u - kb - rb;
    *kbase = (int64_t)((uint64_t)kmn - ((((1ull << kb) - 1ull) - ks) >> 1));
    *vbase = (int64_t)((uint64_t)vmn - ((((1ull << vb) - 1ull) - vs) >> 1));
    return kb | (rb << 8) | (vb << 16) | PK_OK;
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

// slot claim on a device-scope counter for the active lanes of a wave (one atomic per wave)
__device__ __forceinline__ int64_t wave_claim_dev(int64_t* ctr) {
    const uint64_t act = __ballot(1);
    const int lane = __lane_id();
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int rank = __popcll(act & ((1ull << lane) - 1ull));
    long long base = 0;
    if (lane == leader)
        base = (long long)__hip_atomic_fetch_add(ctr, (int64_t)__popcll(act), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (int64_t)__shfl(base, leader, 64) + rank;
}

// Last-workgroup election, called by one thread per workgroup once the workgroup's published
// stores have completed (s_waitcnt vmcnt(0)).  True for exactly one workgroup of the grid, the
// last to arrive; it may then read what every other workgroup published (agent-scope loads).
// Workgroup b counts on group counter b % TK_GROUPS and the last of each group on the top
// counter: same-address device-scope atomics serialise at the memory side, so 1024 workgroups
// on one counter cost tens of microseconds.  Counters are left at 0 for the next launch.
static __device__ bool grid_last_wg(uint32_t (*t)[32]) {
    const uint32_t G = gridDim.x, g = blockIdx.x % TK_GROUPS;
    const uint32_t in_g = (G - g + TK_GROUPS - 1) / TK_GROUPS;
    const uint32_t ng = min(G, (uint32_t)TK_GROUPS);
    if (__hip_atomic_fetch_add(&t[g][0], 1u, __ATOMIC_RELAXED, DEV_SCOPE) != in_g - 1) return false;
    __hip_atomic_store(&t[g][0], 0u, __ATOMIC_RELAXED, DEV_SCOPE);
    if (__hip_atomic_fetch_add(&t[TK_GROUPS][0], 1u, __ATOMIC_RELAXED, DEV_SCOPE) != ng - 1) return false;
    __hip_atomic_store(&t[TK_GROUPS][0], 0u, __ATOMIC_RELAXED, DEV_SCOPE);
    return true;
}

// launch timing (KT_WORDS): block 0 stamps the start, the grid's last workgroup the duration
__device__ __forceinline__ void kt_start(unsigned long long* kt) {
    if (kt && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&kt[0], (unsigned long long)wall_clock64(), __ATOMIC_RELAXED, DEV_SCOPE);
}
__device__ __forceinline__ void kt_end(unsigned long long* kt) {  // one thread of the last workgroup
    if (!kt) return;
    const unsigned long long t0 = __hip_atomic_load(&kt[0], __ATOMIC_RELAXED, DEV_SCOPE);
    __hip_atomic_fetch_add(&kt[1], (unsigned long long)wall_clock64() - t0, __ATOMIC_RELAXED, DEV_SCOPE);
    __hip_atomic_fetch_add(&kt[2], 1ull, __ATOMIC_RELAXED, DEV_SCOPE);
}

}  // namespace fw
