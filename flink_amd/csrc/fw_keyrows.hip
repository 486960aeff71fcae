// fw_keyrows.hip -- key rows (VARCHAR / composite SQL keys) on the device.
//
// The SQL window operator keys its state on the key projection's BinaryRowData
// (BinaryRowDataKeySelector.getKey, TR/keyselector/BinaryRowDataKeySelector.java:54;
// RecordsWindowBuffer.addElement groups by it, TR/operators/aggregate/window/buffers/
// RecordsWindowBuffer.java:81-104) and two keys are the same iff their bytes are
// (BinaryRowData.equals -> BinarySegmentUtils.equals).  A FW_KEYHASH_KEYROW handle receives those
// bytes (images) and interns them here in an HBM table: every distinct image gets a dense int64 id,
// the key the slice-state table, partials and timers carry; its hashCode (BinaryRowData.hashCode,
// MurmurHashUtils.hashBytesByWords) routes it to its key group exactly as the reference does.
// Results come back with their key rows gathered from the table.  Ids no state entry, pending
// partial, timer request or unread result row refers to any more are collected when the fresh ids
// run low (mark / sweep / index rebuild, k_kr_gc_*), so the table holds the live keys, like the
// heap backend's state map holds only keys with state.
//
// Cross-workgroup visibility inside k_kr_intern (per-XCD L2s are not coherent, MI355X_MICROARCH.md
// "inter-workgroup visibility"): an id's row (meta word + image) is written with agent-scope (sc1)
// stores and drained (s_waitcnt vmcnt(0)) before the index slot is published with an agent-scope
// atomic; readers probe slots only with agent-scope atomics (coherent across XCDs) and read rows with
// sc1 loads.  Each id's row is padded to whole 128-B lines and is read in a launch only after its
// slot was published in that launch (ids are recycled only across launches), so no reader's L2 can
// hold an older copy of it.
#include <hip/hip_runtime.h>

#include "fw_kernel_common.h"

namespace fw {

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t kr_slot_of(int32_t h, int64_t n_slots) {
    uint32_t x = (uint32_t)h * 0x9E3779B1u;
    x ^= x >> 16;
    return x & (uint32_t)(n_slots - 1);
}

// BinaryRowWriter images of columnar key rows at the given offsets
__global__ void k_kr_images(KeyRowDesc d, int64_t n, const int64_t* off, uint8_t* bytes) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (off[i] & 7)) return;
    key_row_image_write(d, i, (uint64_t*)(bytes + off[i]));
}

// a fresh id: the free list (ids a collection found dead) first, then never-used ids
__device__ __forceinline__ int64_t kr_alloc(const KeyRowTable& t, Ctrl* c) {
    const int64_t f = __hip_atomic_fetch_add(&c->kr_free_cursor, (int64_t)1, __ATOMIC_RELAXED, DEV_SCOPE);
    if (f < c->kr_free_count) return t.free_list[f];
    const int64_t id = __hip_atomic_fetch_add(&c->kr_next_id, (int64_t)1, __ATOMIC_RELAXED, DEV_SCOPE);
    return id < t.cap_ids ? id : -1;
}

// Interns row i's image: out_id[i] = its id (inserting it if new), out_hash[i] = its hashCode.
__global__ void k_kr_intern(KeyRowTable t, Ctrl* c, int64_t n, const int64_t* off, const uint8_t* bytes,
                            int64_t* out_id, int32_t* out_hash) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t o = off[i], len = off[i + 1] - o;
    if (len < 8 || (len & 7) || (o & 7) || len > t.max_len) {
        __hip_atomic_fetch_or(&c->error, ERR_KEYROW, __ATOMIC_RELAXED, DEV_SCOPE);
        out_id[i] = -1;
        out_hash[i] = 0;
        return;
    }
    const uint64_t* img = (const uint64_t*)(bytes + o);
    const int32_t h = key_row_image_hash(img, len);
    const uint64_t m = ((uint64_t)(uint32_t)h << 32) | (uint64_t)len;
    const int nw = (int)(len >> 3);
    uint32_t sl = kr_slot_of(h, t.n_slots);
    int64_t id = -1;
    for (int64_t probes = 0; probes < t.n_slots;) {
        uint32_t st = 0;
        if (__hip_atomic_compare_exchange_strong(&t.slots[sl], &st, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED, DEV_SCOPE)) {
            // claimed an empty slot: allocate, write the row write-through, then publish
            id = kr_alloc(t, c);
            if (id < 0) {
                __hip_atomic_fetch_or(&c->error, ERR_KEYROW, __ATOMIC_RELAXED, DEV_SCOPE);
                __hip_atomic_exchange(&t.slots[sl], 0u, __ATOMIC_RELAXED, DEV_SCOPE);
                break;
            }
            uint64_t* row = t.arena + (size_t)id * t.stride_words;
            st_sc1(row, m);
            for (int j = 0; j < nw; j++) st_sc1(row + 1 + j, img[j]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_exchange(&t.slots[sl], 2u + (uint32_t)id, __ATOMIC_RELAXED, DEV_SCOPE);
            break;
        }
        if (st == 1u) continue;  // being inserted by another lane: its publish comes next
        const int64_t e = (int64_t)(st - 2u);
        const uint64_t* row = t.arena + (size_t)e * t.stride_words;
        if (ld_sc1(row) == m) {
            bool eq = true;
            for (int j = 0; j < nw && eq; j++) eq = ld_sc1(row + 1 + j) == img[j];
            if (eq) {
                id = e;
                break;
            }
        }
        sl = (sl + 1u) & (uint32_t)(t.n_slots - 1);
        probes++;
    }
    if (id < 0) __hip_atomic_fetch_or(&c->error, ERR_KEYROW, __ATOMIC_RELAXED, DEV_SCOPE);
    out_id[i] = id;
    out_hash[i] = h;
}

// ---- collection: runs after a merge launch, when the fresh ids are running low --------------
// begin: decide (one thread); every other collection kernel returns at once unless c->kr_gc
__global__ void k_kr_gc_begin(KeyRowTable t, Ctrl* c) {
    if (threadIdx.x || blockIdx.x) return;
    const bool free_left = c->kr_free_cursor < c->kr_free_count;
    const bool run = !free_left && c->kr_next_id >= t.cap_ids / 2;
    c->kr_gc = run ? 1 : 0;
    if (run) {
        c->kr_epoch += 1;
        c->kr_collections += 1;
    }
}

__device__ __forceinline__ void kr_mark(const KeyRowTable& t, const Ctrl* c, int64_t id, uint32_t ep) {
    if (id >= 0 && id < c->kr_next_id) t.mark[id] = ep;  // stale rows may hold anything: bounds
}

struct KrMarkArgs {
    KeyRowTable t;
    Ctrl* c;
    const uint64_t* state;  // [n_sb][cap_e][pwe]
    const int32_t* state_count;
    const uint8_t* sb_nar;  // HOP block state: superbucket b's layout level (hb_narrow_words; key first in every layout)
    int32_t hb_nw;
    int32_t n_sb, cap_e, pwe, pw;
    const uint64_t* parts;  // FW_MAX_PENDING slots of cap_rows rows of pw words
    int64_t cap_rows;
    const int64_t* treq;    // (key, window, sb) triples
    const int64_t* out_key; // result slabs [n_sb][slab_cap] + overflow
    const int32_t* sb_out;
    int64_t slab_cap;
};

// mark every id a live state entry, pending partial row, timer request or unread result holds:
// block b < n_sb marks superbucket b's entries and slab rows; the rest stride over the partials
__global__ void k_kr_gc_mark(KrMarkArgs a) {
    const Ctrl* c = a.c;
    if (!c->kr_gc) return;
    const uint32_t ep = c->kr_epoch;
    const int64_t b = blockIdx.x;
    if (b < a.n_sb) {
        const int32_t n = a.state_count[b];
        const uint64_t* st = a.state + (size_t)b * a.cap_e * a.pwe;
        const int lv = a.sb_nar ? a.sb_nar[b] : 0;
        const int stride = lv ? hb_narrow_words(a.hb_nw, lv) : a.pwe;
        for (int e = threadIdx.x; e < n; e += blockDim.x) kr_mark(a.t, c, (int64_t)st[(size_t)e * stride], ep);
        const int32_t no = min((int64_t)a.sb_out[b], a.slab_cap);
        for (int r = threadIdx.x; r < no; r += blockDim.x) kr_mark(a.t, c, a.out_key[b * a.slab_cap + r], ep);
        return;
    }
    const int64_t nb = gridDim.x - a.n_sb, me = b - a.n_sb;
    const int64_t nrows = c->pending_pushes * a.cap_rows;  // every row of a pending slot (stale rows too)
    for (int64_t r = me * blockDim.x + threadIdx.x; r < nrows; r += nb * blockDim.x)
        kr_mark(a.t, c, (int64_t)a.parts[(size_t)r * a.pw], ep);
    const int64_t nt = c->n_treq;
    for (int64_t r = me * blockDim.x + threadIdx.x; r < nt; r += nb * blockDim.x) kr_mark(a.t, c, a.treq[3 * r], ep);
    const int64_t novf = (int64_t)c->out_count[c->ovf_sel & 1];
    for (int64_t r = me * blockDim.x + threadIdx.x; r < novf; r += nb * blockDim.x)
        kr_mark(a.t, c, a.out_key[(size_t)a.n_sb * a.slab_cap + r], ep);
}

// sweep: every id below kr_next_id not marked goes to the free list; the index is cleared
__global__ void k_kr_gc_sweep(KeyRowTable t, Ctrl* c) {
    if (!c->kr_gc) return;
    const uint32_t ep = c->kr_epoch;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t s = g; s < t.n_slots; s += stride) t.slots[s] = 0u;
    const int64_t n = c->kr_next_id;
    for (int64_t id = g; id < n; id += stride) {
        if (t.mark[id] == ep) continue;
        const int64_t p = __hip_atomic_fetch_add(&c->kr_free_count, (int64_t)1, __ATOMIC_RELAXED, DEV_SCOPE);
        t.free_list[p] = id;
    }
}

// rebuild the index from the live ids (no two live ids hold the same image: no comparisons)
__global__ void k_kr_gc_rebuild(KeyRowTable t, Ctrl* c) {
    if (!c->kr_gc) return;
    const uint32_t ep = c->kr_epoch;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t n = c->kr_next_id;
    for (int64_t id = g; id < n; id += stride) {
        if (t.mark[id] != ep) continue;
        const int32_t h = (int32_t)(t.arena[(size_t)id * t.stride_words] >> 32);
        uint32_t sl = kr_slot_of(h, t.n_slots);
        for (;;) {
            uint32_t st = 0;
            if (__hip_atomic_compare_exchange_strong(&t.slots[sl], &st, 2u + (uint32_t)id, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, DEV_SCOPE))
                break;
            sl = (sl + 1u) & (uint32_t)(t.n_slots - 1);
        }
    }
}

// the kernels before the sweep reset the free list: k_kr_gc_begin cannot (the sweep appends to it)
__global__ void k_kr_gc_reset_free(Ctrl* c) {
    if (threadIdx.x || blockIdx.x || !c->kr_gc) return;
    c->kr_free_count = 0;
    c->kr_free_cursor = 0;
}

// result rows' key rows: image of res_key[i] at img + i * stride, its length in len[i]
__global__ void k_kr_result_rows(KeyRowTable t, const int64_t* res_key, const int64_t* n_ptr, int64_t cap,
                                 int32_t* len, uint64_t* img, int32_t stride_words) {
    const int64_t n = min(*n_ptr, cap);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t id = res_key[i];
    if (id < 0 || id >= t.cap_ids) {
        len[i] = 0;
        return;
    }
    const uint64_t* row = t.arena + (size_t)id * t.stride_words;
    const int32_t l = (int32_t)(uint32_t)row[0];
    len[i] = l;
    for (int j = 0; j < (l >> 3); j++) img[(size_t)i * stride_words + j] = row[1 + j];
}

hipError_t launch_kr_intern(const KeyRowTable& t, Ctrl* c, int64_t n, const int64_t* off, const uint8_t* bytes,
                            int64_t* out_id, int32_t* out_hash, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_kr_intern, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, t, c, n, off, bytes, out_id,
                       out_hash);
    return hipGetLastError();
}

hipError_t launch_kr_collect(const KeyRowTable& t, Ctrl* c, const uint64_t* state, const int32_t* state_count,
                             const uint8_t* sb_nar, int32_t hb_nw,
                             int32_t n_sb, int32_t cap_e, int32_t pwe, int32_t pw, const uint64_t* parts,
                             int64_t cap_rows, const int64_t* treq, const int64_t* out_key, const int32_t* sb_out,
                             int64_t slab_cap, hipStream_t s) {
    hipLaunchKernelGGL(k_kr_gc_begin, dim3(1), dim3(64), 0, s, t, c);
    KrMarkArgs a{t, c, state, state_count, sb_nar, hb_nw, n_sb, cap_e, pwe, pw, parts, cap_rows, treq, out_key, sb_out, slab_cap};
    hipLaunchKernelGGL(k_kr_gc_mark, dim3((unsigned)n_sb + 256), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_kr_gc_reset_free, dim3(1), dim3(64), 0, s, c);
    const unsigned g = (unsigned)std::min<int64_t>(4096, (std::max(t.n_slots, t.cap_ids) + 255) / 256);
    hipLaunchKernelGGL(k_kr_gc_sweep, dim3(g), dim3(256), 0, s, t, c);
    hipLaunchKernelGGL(k_kr_gc_rebuild, dim3(g), dim3(256), 0, s, t, c);
    return hipGetLastError();
}

hipError_t launch_kr_result_rows(const KeyRowTable& t, const int64_t* res_key, const int64_t* n_ptr, int64_t cap,
                                 int32_t* len, uint64_t* img, int32_t stride_words, hipStream_t s) {
    if (cap <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_kr_result_rows, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, s, t, res_key, n_ptr, cap,
                       len, img, stride_words);
    return hipGetLastError();
}

}  // namespace fw

using namespace fw;

extern "C" int fw_key_row_images(const fw_key_field* fields, int32_t n_fields, int64_t n, const int64_t* d_offsets,
                                 uint8_t* d_bytes, void* stream) {
    KeyRowDesc d;
    if (const int rc = key_row_desc(fields, n_fields, &d)) return rc;
    if (n <= 0) return FW_OK;
    if (!d_offsets || !d_bytes || ((uintptr_t)d_bytes & 7)) return FW_E_INVALID;
    hipLaunchKernelGGL(k_kr_images, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d, n, d_offsets,
                       d_bytes);
    return hipGetLastError() == hipSuccess ? FW_OK : FW_E_DEVICE;
}

extern "C" int fw_host_key_row_image_lengths(const fw_key_field* fields, int32_t n_fields, int64_t n, int64_t* lens) {
    KeyRowDesc d;
    if (const int rc = key_row_desc(fields, n_fields, &d)) return rc;
    if (n > 0 && !lens) return FW_E_INVALID;
    for (int64_t i = 0; i < n; i++) lens[i] = key_row_image_len(d, i);
    return FW_OK;
}

extern "C" int fw_host_key_row_images(const fw_key_field* fields, int32_t n_fields, int64_t n, const int64_t* offsets,
                                      uint8_t* bytes) {
    KeyRowDesc d;
    if (const int rc = key_row_desc(fields, n_fields, &d)) return rc;
    if (n > 0 && (!offsets || !bytes || ((uintptr_t)bytes & 7))) return FW_E_INVALID;
    for (int64_t i = 0; i < n; i++) {
        if (offsets[i] & 7) return FW_E_INVALID;
        key_row_image_write(d, i, (uint64_t*)(bytes + offsets[i]));
    }
    return FW_OK;
}

extern "C" int32_t fw_host_key_row_image_hash(const uint8_t* image, int64_t len) {
    if (!image || len < 0 || (len & 7) || ((uintptr_t)image & 7)) return 0;
    return key_row_image_hash((const uint64_t*)image, len);
}
