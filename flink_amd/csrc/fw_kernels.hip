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

#include "fw_kernel_common.h"

namespace fw {

template <int NV>
hipError_t ingest_nv(const IngestArgs& a, hipStream_t s, KTimer* t);  // k_ingest_nv*.hip
template <int NW>
hipError_t merge_nw(const MergeArgs& a, hipStream_t s);  // k_merge_nw*.hip
extern template hipError_t ingest_nv<0>(const IngestArgs&, hipStream_t, KTimer*);
extern template hipError_t ingest_nv<1>(const IngestArgs&, hipStream_t, KTimer*);
extern template hipError_t ingest_nv<2>(const IngestArgs&, hipStream_t, KTimer*);
extern template hipError_t ingest_nv<4>(const IngestArgs&, hipStream_t, KTimer*);
extern template hipError_t ingest_nv<8>(const IngestArgs&, hipStream_t, KTimer*);
extern template hipError_t merge_nw<1>(const MergeArgs&, hipStream_t);
extern template hipError_t merge_nw<2>(const MergeArgs&, hipStream_t);
extern template hipError_t merge_nw<4>(const MergeArgs&, hipStream_t);
extern template hipError_t merge_nw<8>(const MergeArgs&, hipStream_t);

// ---- result compaction: slabs (+ overflow) -> one contiguous result set ----------------------
// One launch: block b copies the slabs of superbuckets [b·R, (b+1)·R) in order; its first output row
// is the sum of the slab counts before its range (a block-wide reduction over sb_out, read from L2:
// at most 512 blocks, so <= n_sb / 2 reads each on average).  The last block also copies the shared
// overflow region and publishes the totals (off[n_sb] = slab rows, off[n_sb + 1] = all rows).
__device__ __forceinline__ int64_t block_sum_i64(int64_t v, int64_t* tmp) {
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    if ((threadIdx.x & 63) == 0) tmp[threadIdx.x >> 6] = v;
    __syncthreads();
    int64_t t = 0;
    for (int w = 0; w < BLOCK / 64; w++) t += tmp[w];
    __syncthreads();
    return t;
}

__global__ __launch_bounds__(BLOCK) void k_compact(CompactArgs a, int32_t R) {
    __shared__ int64_t tmp[BLOCK / 64];
    const int s0 = blockIdx.x * R, s1 = min(s0 + R, a.n_sb);
    int64_t part = 0;
    for (int i = threadIdx.x; i < s0; i += BLOCK) part += a.sb_out[i];
    int64_t base = block_sum_i64(part, tmp);
    auto copy = [&](int64_t src0, int64_t dst0, int64_t n) {
        for (int64_t i = threadIdx.x; i < n; i += BLOCK) {
            const int64_t d = dst0 + i, sidx = src0 + i;
            if (d >= a.res_cap) break;
            a.res_key[d] = a.out_key[sidx];
            const int64_t we = a.out_we[sidx];
            a.res_ws[d] = a.local_out ? we : window_start_of(a.win, we);  // SliceAssigner.getWindowStart
            a.res_we[d] = we;
            a.res_null[d] = a.out_null[sidx];
            for (int g = 0; g < a.n_aggs; g++) a.res_val[g][d] = a.out_val[g][sidx];
        }
    };
    for (int sb = s0; sb < s1; sb++) {
        const int64_t n = a.sb_out[sb];
        if (threadIdx.x == 0) a.off[sb] = base;
        copy((int64_t)sb * a.slab_cap, base, n);
        base += n;
    }
    if (blockIdx.x != gridDim.x - 1) return;
    const int64_t ovf = (int64_t)min(a.ctrl->out_count[a.ctrl->ovf_sel & 1], (uint64_t)a.res_cap);
    copy((int64_t)a.n_sb * a.slab_cap, base, ovf);
    if (threadIdx.x == 0) {
        a.off[a.n_sb] = base;          // slab rows
        a.off[a.n_sb + 1] = base + ovf;  // total rows
        if (a.host_n)  // fw_results_async: the count, next to the rows in mapped host memory (vector store)
            __hip_atomic_store(a.host_n, base + ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
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
        c->fold_skip = 0;
        c->push_count = 0;
        c->n_lfire = 0;
        c->n_side = 0;
        c->n_ordev = 0;
        c->flush_launches = 0;
        c->parts_merged = 0;
        c->part_bytes = 0;
        c->part_bytes_merged = 0;
        c->compact_chunks = 0;
        c->state_moved = 0;
        c->peak_entries = 0;
        c->kr_next_id = 0;
        c->kr_free_count = 0;
        c->kr_free_cursor = 0;
        c->kr_epoch = 0;
        c->kr_gc = 0;
        c->kr_collections = 0;
        c->pk_next_k = c->pk_next_v = c->pk_cur_k = c->pk_cur_v = 0;
        c->pk_next_bits = c->pk_cur_bits = 0;  // no PF_PACK until a push has measured its ranges
    }
}

hipError_t launch_compact(const CompactArgs& a, hipStream_t s, KTimer* t) {
    kt_mark(t, FW_KT_OTHER, false, s);
    const int R = (a.n_sb + 511) / 512;  // superbuckets per block: at most 512 blocks
    const int nb = (a.n_sb + R - 1) / R;
    hipLaunchKernelGGL(k_compact, dim3((unsigned)nb), dim3(BLOCK), 0, s, a, (int32_t)R);
    kt_mark(t, FW_KT_OTHER, true, s);
    return hipGetLastError();
}

__global__ __launch_bounds__(BLOCK) void k_copy_out(CopyOutArgs a) {
    const int64_t n = min(*a.d_n, a.cap);
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        a.dst_key[i] = a.src_key[i];
        a.dst_ws[i] = a.src_ws[i];
        a.dst_we[i] = a.src_we[i];
        a.dst_null[i] = a.src_null[i];
        for (int g = 0; g < a.n_aggs; g++) a.dst_val[g][i] = a.src_val[g][i];
    }
}

hipError_t launch_copy_out(const CopyOutArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_copy_out, dim3(512), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}

// one column per grid row: 16-B loads of four deltas, two 16-B stores of their words
__global__ __launch_bounds__(BLOCK) void k_widen(WidenArgs a) {
    const int c = blockIdx.y;
    const uint32_t* s = a.src[c];
    uint64_t* d = a.dst[c];
    const uint64_t b = a.base[c];
    const int64_t n4 = a.n >> 2;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n4; i += (int64_t)gridDim.x * BLOCK) {
        const uint4 v = ((const uint4*)s)[i];
        ulonglong2* q = (ulonglong2*)(d + 4 * i);
        q[0] = make_ulonglong2(b + v.x, b + v.y);
        q[1] = make_ulonglong2(b + v.z, b + v.w);
    }
    if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {
        const int64_t i = 4 * n4 + threadIdx.x;
        d[i] = b + s[i];
    }
}

hipError_t launch_widen(const WidenArgs& a, int n_cols, hipStream_t s) {
    if (n_cols <= 0 || a.n <= 0) return hipSuccess;
    const int64_t n4 = (a.n + 3) >> 2;
    const unsigned gx = (unsigned)std::min<int64_t>(1024, (n4 + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_widen, dim3(gx, (unsigned)n_cols), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_init_ctrl(Ctrl* c, hipStream_t s) {
    hipLaunchKernelGGL(k_init_ctrl, dim3(1), dim3(64), 0, s, c);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// template dispatch
// ---------------------------------------------------------------------------------------
hipError_t launch_ingest(const IngestArgs& a, hipStream_t s, KTimer* t) {
    switch (ig_nv(a.nv)) {
        case 0: return ingest_nv<0>(a, s, t);
        case 1: return ingest_nv<1>(a, s, t);
        case 2: return ingest_nv<2>(a, s, t);
        case 4: return ingest_nv<4>(a, s, t);
        default: return ingest_nv<8>(a, s, t);
    }
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
// value-column pointers of the partition kernels, passed by value (no per-call pointer-array copy)
struct PartCols {
    const uint64_t* in[FW_MAX_COLS];
    uint64_t* out[FW_MAX_COLS];
};

__global__ __launch_bounds__(BLOCK) void k_part_hist(const int64_t* key, const int32_t* kh, int64_t n, int32_t kind,
                                                     int32_t max_p, int32_t p, uint32_t* counts,
                                                     const int64_t* n_dev = nullptr) {
    __shared__ uint32_t h[PART_MAXP];
    const int tid = threadIdx.x, lane = tid & 63;
    if (n_dev) n = min(n, *n_dev);  // a row count known only on the device (<= the launch's n)
    if (tid < PART_MAXP) h[tid] = 0;
    __syncthreads();
    // counted per wave with ballots (lane d keeps destination d's count): one LDS add per wave and
    // destination instead of a same-address LDS atomic per row
    uint32_t mine = 0;
    const int64_t b = (int64_t)blockIdx.x * PART_TILE;
    for (int j = tid - lane; j < PART_TILE; j += BLOCK) {
        const int64_t i = b + j + lane;
        int32_t d = -1;
        if (j + lane < PART_TILE && i < n)
            d = operator_for_key_group(max_p, p, key_group_for_hash(java_key_hash(kind, key[i], kh ? kh[i] : 0), max_p));
        for (int dd = 0; dd < p; dd++) {
            const uint32_t c = (uint32_t)__popcll(__ballot(d == dd));
            if (lane == dd) mine += c;
        }
    }
    if (lane < p && mine) atomicAdd(&h[lane], mine);
    __syncthreads();
    if (tid < p) counts[(size_t)blockIdx.x * p + tid] = h[tid];
}

// one block: offsets[blk][d] = sum_{d'<d} total(d') + sum_{b'<blk} counts[b'][d].  Thread (seg, d)
// sums destination d's counts over a contiguous range of tiles, the per-destination segment sums are
// scanned in LDS, and each thread rewrites its range from its running offset (a serial loop over
// every tile per destination took 155 us for 1024 tiles)
constexpr int PSCAN_T = 1024;
__global__ __launch_bounds__(PSCAN_T) void k_part_scan(uint32_t* counts, int64_t nblk, int32_t p, int64_t* totals) {
    __shared__ uint64_t part[PSCAN_T];  // [seg][d] sums, then their exclusive prefix per destination
    __shared__ uint64_t base[PART_MAXP];
    const int tid = threadIdx.x;
    const int S = PSCAN_T / p;  // segments per destination
    const int d = tid % p, seg = tid / p;
    const int64_t per = (nblk + S - 1) / S;
    const int64_t b0 = min(nblk, (int64_t)seg * per), b1 = min(nblk, b0 + per);
    uint64_t sum = 0;
    if (seg < S)
        for (int64_t b = b0; b < b1; b++) sum += counts[b * p + d];
    part[tid] = sum;
    __syncthreads();
    // inclusive scan of each destination's segment sums (stride p: part[seg * p + d]), log2(S) rounds
    for (int off = p; off < S * p; off <<= 1) {
        const uint64_t v = (tid < S * p && tid >= off) ? part[tid - off] : 0;
        __syncthreads();
        if (tid < S * p) part[tid] += v;
        __syncthreads();
    }
    if (tid < p) {  // destination tid's total: its last segment's inclusive sum
        const uint64_t tot = part[(S - 1) * p + tid];
        totals[tid] = (int64_t)tot;
        base[tid] = tot;
    }
    if (seg < S) sum = part[tid] - sum;  // this segment's exclusive offset within its destination
    __syncthreads();
    if (tid == 0) {  // destinations' bases: the totals of the destinations before them
        uint64_t r = 0;
        for (int x = 0; x < p; x++) {
            const uint64_t t = base[x];
            base[x] = r;
            r += t;
        }
    }
    __syncthreads();
    if (seg < S) {
        uint64_t run = base[d] + sum;
        for (int64_t b = b0; b < b1; b++) {
            const uint32_t v = counts[b * p + d];
            counts[b * p + d] = (uint32_t)run;  // fits: n < 2^32 per call
            run += v;
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_part_scatter(const int64_t* key, const int32_t* kh, const int64_t* ts,
                                                        PartCols cols,
                                                        int32_t ncols, int64_t n, int32_t kind, int32_t max_p,
                                                        int32_t p, const uint32_t* offsets, int64_t* okey, int64_t* ots,
                                                        int64_t* orows = nullptr,
                                                        int64_t seg_len = 0, const int64_t* totals = nullptr,
                                                        int64_t* spill = nullptr, const int64_t* n_dev = nullptr) {
    if (n_dev) n = min(n, *n_dev);
    // Stable: rows keep their input order within a destination (the order a Netty channel
    // delivers them in, ChannelSelectorRecordWriter.emit :54), so a DOUBLE SUM downstream adds in
    // the same order on every run.  Each wave ranks its 64 rows per destination with ballots;
    // the waves of one pass are ordered through a per-wave count table.
    constexpr int NWV = BLOCK / 64;
    __shared__ uint32_t h[PART_MAXP];         // next output position per destination
    __shared__ uint32_t wc[NWV][PART_MAXP];   // rows per (wave, destination) of the current pass
    __shared__ int64_t dbase[PART_MAXP];     // packed mode: first output position of each destination
    __shared__ int64_t sbase[PART_MAXP];     // packed mode: first spill row of each destination
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid < p) h[tid] = offsets[(size_t)blockIdx.x * p + tid];
    if (orows && tid < p) {
        int64_t b0 = 0, s0 = 0;
        for (int d = 0; d < tid; d++) {
            b0 += totals[d];
            s0 += max(totals[d] - seg_len, (int64_t)0);
        }
        dbase[tid] = b0;
        sbase[tid] = s0;
    }
    const uint64_t lt = (1ull << lane) - 1ull;
    const int64_t b = (int64_t)blockIdx.x * PART_TILE;
    // every column of a pass is loaded one pass ahead (the next pass's loads are in flight while this
    // pass ranks, waits at its barriers and stores): one exposed load round trip per block, not two
    // per pass
    int64_t ck = 0, ct = 0, nk = 0, nt = 0;
    int32_t ch = 0, nh = 0;
    uint64_t cv[FW_MAX_COLS], nv[FW_MAX_COLS];
    auto load_pass = [&](int64_t i, int64_t& k_, int64_t& t_, int32_t& h_, uint64_t (&v_)[FW_MAX_COLS]) {
        if (i >= n) return;
        k_ = key[i];
        t_ = ts[i];
        h_ = kh ? kh[i] : 0;
#pragma unroll
        for (int c = 0; c < FW_MAX_COLS; c++)
            if (c < ncols) v_[c] = cols.in[c][i];
    };
    load_pass(b + tid, ck, ct, ch, cv);
    for (int j0 = 0; j0 < PART_TILE; j0 += BLOCK) {
        const int64_t i = b + j0 + tid;
        if (j0 + BLOCK < PART_TILE) load_pass(i + BLOCK, nk, nt, nh, nv);
        int32_t d = -1;
        const int64_t k = ck;
        if (i < n) d = operator_for_key_group(max_p, p, key_group_for_hash(java_key_hash(kind, k, ch), max_p));
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
        if (d >= 0 && orows) {  // packed padded segments: row (rank in d) of segment d
            const int64_t r = (int64_t)pos - dbase[d];
            // rows past the segment go to the spill region (destination-major, in input order):
            // the overflow round of the exchange sends them
            int64_t* o = r < seg_len ? orows + ((size_t)d * seg_len + r) * (2 + ncols)
                         : spill      ? spill + (size_t)(sbase[d] + r - seg_len) * (2 + ncols)
                                      : nullptr;
            if (o) {
                o[0] = k;
                o[1] = ct;
#pragma unroll
                for (int c = 0; c < FW_MAX_COLS; c++)
                    if (c < ncols) o[2 + c] = (int64_t)cv[c];
            }
        } else if (d >= 0) {
            okey[pos] = k;
            ots[pos] = ct;
#pragma unroll
            for (int c = 0; c < FW_MAX_COLS; c++)
                if (c < ncols) cols.out[c][pos] = cv[c];
        }
        __syncthreads();  // h updated before the next pass reads it; wc free to overwrite
        ck = nk;
        ct = nt;
        ch = nh;
#pragma unroll
        for (int c = 0; c < FW_MAX_COLS; c++) cv[c] = nv[c];
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
int fw::key_row_desc(const fw_key_field* fields, int32_t n_fields, KeyRowDesc* d) {
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
    PartCols pc{};
    for (int c = 0; c < n_cols; c++) {
        pc.in[c] = (const uint64_t*)d_values[c];
        pc.out[c] = (uint64_t*)d_out_values[c];
    }
    hipLaunchKernelGGL(k_part_hist, dim3((unsigned)nblk), dim3(BLOCK), 0, s, d_key, d_key_hash, n, key_hash_kind,
                       max_parallelism, parallelism, counts);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(PSCAN_T), 0, s, counts, nblk, parallelism, d_counts);
    hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)nblk), dim3(BLOCK), 0, s, d_key, d_key_hash, d_ts,
                       pc, n_cols, n, key_hash_kind, max_parallelism, parallelism, counts,
                       d_out_key, d_out_ts);
    return hipGetLastError() == hipSuccess ? FW_OK : FW_E_DEVICE;
}

extern "C" int fw_partition_packed(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                                   const void* const* d_values, int32_t n_cols, int64_t n, int32_t key_hash_kind,
                                   int32_t max_parallelism, int32_t parallelism, int64_t seg_len, int64_t* d_out_rows,
                                   int64_t* d_counts, void* d_workspace, int64_t workspace_bytes, void* stream) {
    return fw_partition_packed_spill(d_key, d_key_hash, d_ts, d_values, n_cols, n, key_hash_kind, max_parallelism,
                                     parallelism, seg_len, d_out_rows, nullptr, d_counts, d_workspace, workspace_bytes,
                                     stream);
}

static int partition_packed(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                            const void* const* d_values, int32_t n_cols, int64_t n, const int64_t* d_n,
                            int32_t key_hash_kind, int32_t max_parallelism, int32_t parallelism, int64_t seg_len,
                            int64_t* d_out_rows, int64_t* d_spill_rows, int64_t* d_counts, void* d_workspace,
                            int64_t workspace_bytes, void* stream);

extern "C" int fw_partition_packed_spill(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                                         const void* const* d_values, int32_t n_cols, int64_t n, int32_t key_hash_kind,
                                         int32_t max_parallelism, int32_t parallelism, int64_t seg_len,
                                         int64_t* d_out_rows, int64_t* d_spill_rows, int64_t* d_counts,
                                         void* d_workspace, int64_t workspace_bytes, void* stream) {
    return partition_packed(d_key, d_key_hash, d_ts, d_values, n_cols, n, nullptr, key_hash_kind, max_parallelism,
                            parallelism, seg_len, d_out_rows, d_spill_rows, d_counts, d_workspace, workspace_bytes, stream);
}

extern "C" int fw_partition_packed_spill_dn(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                                            const void* const* d_values, int32_t n_cols, int64_t n_max,
                                            const int64_t* d_n, int32_t key_hash_kind, int32_t max_parallelism,
                                            int32_t parallelism, int64_t seg_len, int64_t* d_out_rows,
                                            int64_t* d_spill_rows, int64_t* d_counts, void* d_workspace,
                                            int64_t workspace_bytes, void* stream) {
    if (!d_n) return FW_E_INVALID;
    return partition_packed(d_key, d_key_hash, d_ts, d_values, n_cols, n_max, d_n, key_hash_kind, max_parallelism,
                            parallelism, seg_len, d_out_rows, d_spill_rows, d_counts, d_workspace, workspace_bytes, stream);
}

static int partition_packed(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                            const void* const* d_values, int32_t n_cols, int64_t n, const int64_t* d_n,
                            int32_t key_hash_kind, int32_t max_parallelism, int32_t parallelism, int64_t seg_len,
                            int64_t* d_out_rows, int64_t* d_spill_rows, int64_t* d_counts, void* d_workspace,
                            int64_t workspace_bytes, void* stream) {
    if (parallelism <= 0 || parallelism > PART_MAXP || n_cols < 0 || n_cols > FW_MAX_COLS || seg_len < 1) return FW_E_INVALID;
    if (key_hash_kind == FW_KEYHASH_PRECOMPUTED && n > 0 && !d_key_hash) return FW_E_INVALID;
    if (key_hash_kind != FW_KEYHASH_PRECOMPUTED) d_key_hash = nullptr;
    if (workspace_bytes < fw_partition_workspace_bytes(n, parallelism)) return FW_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    if (n <= 0) {
        return hipMemsetAsync(d_counts, 0, sizeof(int64_t) * parallelism, s) == hipSuccess ? FW_OK : FW_E_DEVICE;
    }
    const int64_t nblk = (n + PART_TILE - 1) / PART_TILE;
    uint32_t* counts = (uint32_t*)d_workspace;
    PartCols pc{};
    for (int c = 0; c < n_cols; c++) pc.in[c] = (const uint64_t*)d_values[c];
    hipLaunchKernelGGL(k_part_hist, dim3((unsigned)nblk), dim3(BLOCK), 0, s, d_key, d_key_hash, n, key_hash_kind,
                       max_parallelism, parallelism, counts, d_n);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(PSCAN_T), 0, s, counts, nblk, parallelism, d_counts);
    hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)nblk), dim3(BLOCK), 0, s, d_key, d_key_hash, d_ts,
                       pc, n_cols, n, key_hash_kind, max_parallelism, parallelism, counts,
                       (int64_t*)nullptr, (int64_t*)nullptr, d_out_rows, seg_len,
                       (const int64_t*)d_counts, d_spill_rows, d_n);
    return hipGetLastError() == hipSuccess ? FW_OK : FW_E_DEVICE;
}

// Device watermark valve (PackedExchange.finish_device): the subtask's [overflow flag, ~watermark,
// largest per-destination share] in one kernel, and after the all-reduce the valve's watermark in
// another (a dozen small torch kernels before, ~55 us per step)
__global__ void k_valve_local(const int64_t* counts, int32_t p, int64_t cap, int64_t watermark, int64_t* out3) {
    const int tid = threadIdx.x;  // one wave: p <= PART_MAXP = 64
    const int64_t c = tid < p ? counts[tid] : 0;
    int64_t m = c;
    uint64_t over = __ballot(tid < p && c > cap);
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) m = max(m, (int64_t)__shfl_xor(m, d, 64));
    if (tid == 0) {
        out3[0] = over != 0;
        out3[1] = ~watermark;  // bitwise NOT reverses the int64 order (Long.MIN_VALUE travels too)
        out3[2] = m;
    }
}
__global__ void k_valve_select(const int64_t* agreed3, const int64_t* prev, int64_t* wm) {
    if (threadIdx.x == 0) *wm = agreed3[0] > 0 ? (prev ? *prev : INT64_MIN) : ~agreed3[1];
}

extern "C" int fw_valve_local(const int64_t* d_counts, int32_t parallelism, int64_t cap, int64_t watermark,
                              int64_t* d_out3, void* stream) {
    if (parallelism <= 0 || parallelism > PART_MAXP || !d_counts || !d_out3) return FW_E_INVALID;
    hipLaunchKernelGGL(k_valve_local, dim3(1), dim3(64), 0, (hipStream_t)stream, d_counts, parallelism, cap, watermark,
                       d_out3);
    return hipGetLastError() == hipSuccess ? FW_OK : FW_E_DEVICE;
}

extern "C" int fw_valve_select(const int64_t* d_agreed3, const int64_t* d_prev_watermark, int64_t* d_watermark,
                               void* stream) {
    if (!d_agreed3 || !d_watermark) return FW_E_INVALID;
    hipLaunchKernelGGL(k_valve_select, dim3(1), dim3(64), 0, (hipStream_t)stream, d_agreed3, d_prev_watermark,
                       d_watermark);
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
