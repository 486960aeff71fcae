// fw_api.hip -- C-ABI of libflinkwin (include/flinkwin.h): one handle per operator subtask.
//
// The handle owns a HIP stream, the device control block, the partial buffer that stands in
// for RecordsWindowBuffer (TR/operators/aggregate/window/buffers/RecordsWindowBuffer.java), the
// HBM slice-state table that replaces HeapKeyedStateBackend for this operator
// (FR/runtime/state/heap/HeapKeyedStateBackend.java:85) together with its timers
// (InternalTimerServiceImpl), and the result buffer.  Calls are asynchronous on the handle's
// stream except where a host value is needed (results, stats, snapshot).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "fw_internal.h"

using namespace fw;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return fail(FW_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

int64_t next_pow2(int64_t x) {
    int64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

int64_t gcd64(int64_t a, int64_t b) {
    while (b) {
        int64_t t = a % b;
        a = b;
        b = t;
    }
    return a < 0 ? -a : a;
}

int round_nw(int nw) { return nw <= 1 ? 1 : nw <= 2 ? 2 : nw <= 4 ? 4 : 8; }

// hipEvent pairs recorded around launches on the handle stream; resolved by fw_get_kernel_times
struct EvTimer final : KTimer {
    struct Rec {
        int kind;
        hipEvent_t b, e;
    };
    std::vector<hipEvent_t> pool;
    std::vector<Rec> recs;
    hipEvent_t open[FW_KT_N] = {};
    double ms[FW_KT_N] = {};
    int64_t n[FW_KT_N] = {};
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        // timing-only events: no system-scope fence (cache write-back + invalidate) at each
        // record, which would otherwise add ~10 us of idle stream time around every launch
        hipEvent_t e = nullptr;
        (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
        return e;
    }
    bool all = false;  // also the small bookkeeping launches (FW_KT_OTHER)
    void mark(int kind, bool end, hipStream_t s) override {
        if (kind == FW_KT_OTHER && !all) return;  // each event record costs the stream a few us
        hipEvent_t ev = get();
        (void)hipEventRecord(ev, s);
        if (!end) {
            open[kind] = ev;
        } else {
            recs.push_back({kind, open[kind], ev});
            open[kind] = nullptr;
        }
    }
    hipError_t resolve() {
        for (const Rec& r : recs) {
            hipError_t e = hipEventSynchronize(r.e);
            if (e != hipSuccess) return e;
            float t = 0.f;
            e = hipEventElapsedTime(&t, r.b, r.e);
            if (e != hipSuccess) return e;
            ms[r.kind] += t;
            n[r.kind]++;
            pool.push_back(r.b);
            pool.push_back(r.e);
        }
        recs.clear();
        return hipSuccess;
    }
    ~EvTimer() override {
        for (const Rec& r : recs) {
            hipEventDestroy(r.b);
            hipEventDestroy(r.e);
        }
        for (hipEvent_t e : pool) hipEventDestroy(e);
    }
};

}  // namespace

struct fw_handle {
    fw_config cfg;
    hipStream_t stream = nullptr;
    WinDesc win{};
    KeySpace ks{};
    WordDesc wd{};
    AggDesc ad{};
    int nv = 0;
    int slot_col[MAX_KCOLS] = {};
    int nw_t = 1;  // template word count (layout stride)
    int pwe = 4;   // words per state entry: key, slice (HOP block: block start), flags, accumulator words
    int n_out = 1; // result value columns (aggregates; LOCAL phase: accumulator fields)
    int64_t cap_rows = 0;     // rows per partial-buffer slot (= max rows per push piece)
    int64_t chunk_rows = 0;   // rows per ingest chunk (IG_BLOCK * ig_rpt(nw_t))
    int64_t max_nch = 0;      // ingest chunks per push piece
    int cap_e = 1024;
    bool always_flush = false;

    Ctrl* ctrl = nullptr;
    uint64_t* parts = nullptr;
    int32_t narrow = 0;          // compact partial rows (IngestArgs::narrow)
    int32_t pack = 0;            // PF_PACK run rows (IngestArgs::pack)
    int64_t* slot_base = nullptr;  // [FW_MAX_PENDING] rank base of each pending push
    uint8_t* ranks = nullptr;      // [FW_MAX_PENDING][cap_rows] rank bytes of compact rows
    int64_t cell_cols = 0;       // cell_pad(max_nch): cells per superbucket per slot
    uint32_t* cells = nullptr;   // [FW_MAX_PENDING][cell_cols / 16][n_sb][16] (cell_index)
    int32_t* slot_nch = nullptr;  // [FW_MAX_PENDING]
    // runs (IngestArgs::runs): superbucket-contiguous partial rows; run_rows == 0: off
    int64_t run_rows = 0;
    int32_t sub_cap = 0;
    uint64_t* runs = nullptr;
    uint8_t* run_ranks = nullptr;
    uint32_t* run_fill = nullptr;
    uint32_t* run_ovf = nullptr;
    int32_t* slot_fmt = nullptr;
    int64_t* treq = nullptr;
    int64_t treq_cap = 0;
    uint64_t* lfire = nullptr;   // DataStream late-fire rows
    int64_t lfire_cap = 0;
    int64_t* side = nullptr;     // DataStream late side-output rows
    int64_t side_cap = 0;
    int64_t* ordev = nullptr;    // DataStream first-element retain / release events
    int64_t ordev_cap = 0;
    std::vector<int64_t> ev_retain, ev_release;  // fw_first_element_events copies
    int32_t push_seq = 0;        // fw_commit / fw_push_device calls (side-output row ids)
    std::vector<int64_t> tz_utc, tz_off, tz_bound;  // shift-zone table (host copy)
    int64_t* d_tz = nullptr;     // device copy: [utc | off | bound]
    std::vector<int64_t> lr_key, lr_ts, lr_seq, lr_row, lr_val[FW_MAX_COLS];  // fw_late_records copies
    uint64_t* state = nullptr;
    int32_t* state_count = nullptr;
    int64_t* sb_min_timer = nullptr;
    uint8_t* sb_nar = nullptr;  // HOP block state: superbucket written in the narrow layout
    int hb_narrow = 2;           // narrowest HOP block layout level (FW_HB_NARROW=0/1: development A/B)
    int64_t* out_key = nullptr;
    int64_t* out_we = nullptr;
    uint64_t* out_val[FW_MAX_AGGS] = {};
    uint32_t* out_null = nullptr;
    int64_t out_cap = 0;       // result rows between resets (= overflow region rows)
    int64_t slab_cap = 0;      // output slab rows per superbucket
    int32_t* sb_out = nullptr;
    uint32_t* sb_fired = nullptr;
    int64_t* chunk_stats = nullptr;
    Tickets* tickets = nullptr;  // last-workgroup election counters of k_ingest / k_merge_fire
    int64_t* coff = nullptr;   // compaction offsets [n_sb + 2]
    int64_t* res_key = nullptr;
    int64_t* res_ws = nullptr;
    int64_t* res_we = nullptr;
    uint64_t* res_val[FW_MAX_AGGS] = {};
    uint32_t* res_null = nullptr;

    // host-staged ingest (FW_STAGE_BUFS pinned column sets)
    int64_t stage_cap = 0;
    int stage_cur = 0;
    int64_t* h_key[FW_STAGE_BUFS] = {};
    int64_t* h_ts[FW_STAGE_BUFS] = {};
    int32_t* h_kh[FW_STAGE_BUFS] = {};
    int64_t* h_val[FW_STAGE_BUFS][FW_MAX_COLS] = {};
    uint8_t* h_nul[FW_STAGE_BUFS][FW_MAX_COLS] = {};
    hipEvent_t stage_ev[FW_STAGE_BUFS] = {};   // H2D from host buffer b done (copy stream)
    // device staging, one set per host set: batch b+1 crosses PCIe on the copy stream while batch b
    // is ingested on the operator stream
    hipStream_t cstream = nullptr;
    hipEvent_t dstage_free[FW_STAGE_BUFS] = {};  // the ingest that read device buffer b has run (operator stream)
    int64_t* d_key[FW_STAGE_BUFS] = {};
    int64_t* d_ts[FW_STAGE_BUFS] = {};
    int32_t* d_kh[FW_STAGE_BUFS] = {};
    int64_t* d_val[FW_STAGE_BUFS][FW_MAX_COLS] = {};
    uint8_t* d_nul[FW_STAGE_BUFS][FW_MAX_COLS] = {};
    // fw_commit_delta32: the 32-bit delta columns of staging set b, FW_PACK_COLS slices of pack_stride
    uint32_t* d_pack[FW_STAGE_BUFS] = {};
    int64_t pack_stride = 0;
    int64_t reserved = -1;

    // asynchronous result delivery (fw_results_async / fw_results_ready): rows compacted on the
    // device into one of FW_AR_BUFS device buffers (ard_*), then moved into pinned host buffers
    // (ar_*); only the row count goes through mapped memory.  Up to FW_AR_BUFS collections are
    // outstanding; fw_results_ready returns the oldest (ar_q, a FIFO of buffer indices)
    int64_t* ard_key[FW_AR_BUFS] = {};
    int64_t* ard_ws[FW_AR_BUFS] = {};
    int64_t* ard_we[FW_AR_BUFS] = {};
    uint64_t* ard_val[FW_AR_BUFS][FW_MAX_AGGS] = {};
    uint32_t* ard_null[FW_AR_BUFS] = {};
    hipStream_t d2h_stream = nullptr;
    int64_t* ar_key[FW_AR_BUFS] = {};
    int64_t* ar_ws[FW_AR_BUFS] = {};
    int64_t* ar_we[FW_AR_BUFS] = {};
    uint64_t* ar_val[FW_AR_BUFS][FW_MAX_AGGS] = {};
    uint32_t* ar_null[FW_AR_BUFS] = {};
    int64_t* ar_n[FW_AR_BUFS] = {};          // row count (written by the compaction kernel)
    hipEvent_t ar_ev[FW_AR_BUFS] = {};
    hipEvent_t ar_dma_ev[FW_AR_BUFS] = {};   // the DMA of buffer b's rows (started early by ar_kick)
    bool ar_copied[FW_AR_BUFS] = {};         // buffer b's rows are (or are queued to be) in host memory
    bool ar_inflight[FW_AR_BUFS] = {};       // buffer b's DMA is queued (ar_kick), fw_results_ready waits for it
    // async result delivery: CU stores of the compacted rows into mapped pinned host memory (1, the
    // default), or DMA on the D2H stream (FW_AR_KERNEL=0).  Measured round 5 (CFG2 end to end):
    // the DMA queues behind the next batch's H2D on the copy engine, so fw_results_ready waited
    // 2.2 ms per step (1.18 G ev/s); the kernel stores run beside that H2D: 1.1 ms (1.64 G ev/s)
    int ar_kernel = 1;
    int ar_cur = 0;                 // buffer of the next fw_results_async
    int ar_q[FW_AR_BUFS] = {};      // outstanding collections, oldest first
    int ar_qhead = 0, ar_qn = 0;
    bool ar_empty[FW_AR_BUFS] = {}; // that call had nothing to collect

    // FW_KEYHASH_KEYROW: the key-row intern table, per-push intern output, key-row staging
    bool keyrow = false;
    KeyRowTable kr{};
    int64_t kr_scratch_n = 0;
    int64_t* d_kid = nullptr;       // interned ids of the push being ingested
    int32_t* d_khash = nullptr;     // their hashCodes
    int64_t* h_kro[FW_STAGE_BUFS] = {};         // pinned staging: key row offsets / bytes (fw_reserve)
    uint8_t* h_krb[FW_STAGE_BUFS] = {};
    int64_t krb_cap = 0;            // staging bytes per batch
    int64_t* d_kro[FW_STAGE_BUFS] = {};
    uint8_t* d_krb[FW_STAGE_BUFS] = {};
    int32_t* res_kr_len = nullptr;  // result key rows (fw_results)
    uint64_t* res_kr_img = nullptr;
    std::vector<int32_t> r_kr_len;
    std::vector<uint64_t> r_kr_img;

    // host copies of results
    std::vector<int64_t> r_key, r_ws, r_we;
    std::vector<uint64_t> r_val[FW_MAX_AGGS];
    std::vector<uint32_t> r_null;

    int64_t pushes_ub = 0;  // upper bound of device pending_pushes
    // pending-push mirror: host-mapped word written by each merge launch (MergeArgs::host_mirror)
    volatile unsigned long long* mirror = nullptr;
    unsigned long long* d_mirror = nullptr;
    uint64_t merge_seq = 0;         // merge launches so far
    uint64_t pushes_total = 0;      // ingest launches so far
    uint64_t pushes_at_merge[64] = {};  // pushes_total when merge launch (seq % 64) was issued
    bool reset_pending = false;  // fw_results_reset called: the next merge launch empties the results
    int64_t host_cur = INT64_MIN;
    // the device's currentProgress / nextTriggerProgress as the launched merges leave them (mirrored
    // on the host from the watermarks it launched; merge_finalize applies the same rule), so fw_advance
    // can tell a watermark that crosses no slice end -- the merge launch would change nothing -- and
    // skip it (FW_SKIP_IDLE=0: launch every advance)
    int64_t dev_cur = INT64_MIN;
    int64_t dev_ntp = INT64_MIN;
    bool skip_idle = true;
    KTimer* timer = nullptr;  // non-null while fw_set_profiling is on
    int ablate = 0;           // FW_ABLATE (development timing builds only; results are wrong)
    int fold_always = 0;      // FW_FOLD=1 (development A/B): no adaptive fold skip
    int fill_pct = 75;        // superbucket LDS fill target (FW_FILL_PCT: development A/B)
    unsigned long long* stamps = nullptr;  // [N_STAMPS] merge phase cycles (FW_ABLATE & AB_STAMPS)
    unsigned long long* kt_dev = nullptr;  // [FW_KT_N][KT_WORDS] in-kernel launch timing
    int kt_device = 0;                     // fw_set_profiling(FW_PROF_DEVICE) is on
};

namespace {

int validate_and_plan(fw_handle* h) {
    const fw_config& c = h->cfg;
    if (c.abi_version != FW_ABI_VERSION) return fail(FW_E_INVALID, "abi_version %d != %d", c.abi_version, FW_ABI_VERSION);
    if (c.api != FW_API_SQL && c.api != FW_API_DATASTREAM) return fail(FW_E_INVALID, "bad api %d", c.api);
    if (c.n_aggs < 1 || c.n_aggs > FW_MAX_AGGS) return fail(FW_E_INVALID, "n_aggs %d out of range", c.n_aggs);
    if (c.n_value_cols < 0 || c.n_value_cols > FW_MAX_COLS) return fail(FW_E_INVALID, "n_value_cols out of range");
    if (c.max_parallelism < 1 || c.max_parallelism > 32768) return fail(FW_E_INVALID, "max_parallelism out of range");
    if (c.parallelism < 1 || c.parallelism > c.max_parallelism) return fail(FW_E_INVALID, "parallelism out of range");
    if (c.subtask_index < 0 || c.subtask_index >= c.parallelism) return fail(FW_E_INVALID, "subtask_index out of range");
    if (c.key_hash < FW_KEYHASH_LONG || c.key_hash > FW_KEYHASH_KEYROW) return fail(FW_E_INVALID, "bad key_hash");
    h->keyrow = c.key_hash == FW_KEYHASH_KEYROW;
    if (h->keyrow) {
        if (c.api != FW_API_SQL) return fail(FW_E_INVALID, "key rows (FW_KEYHASH_KEYROW) are SQL keys");
        const int32_t mb = c.key_row_max_bytes ? c.key_row_max_bytes : 120;  // 120: one 128-B line per id
        if (mb < 16 || mb > 4096 || (mb & 7)) return fail(FW_E_INVALID, "key_row_max_bytes must be a multiple of 8 in [16, 4096]");
        h->kr.stride_words = (int32_t)(((8 + mb) + 127) / 128 * 16);  // meta word + image, whole 128-B lines
        h->kr.max_len = mb;
    }
    if (c.size_ms <= 0) return fail(FW_E_INVALID, "window size must be > 0");
    // ---- window (SliceAssigners constructors' argument checks)
    WinDesc& w = h->win;
    w.kind = c.window_kind;
    w.size = c.size_ms;
    w.offset = c.offset_ms;
    switch (c.window_kind) {
        case FW_WIN_TUMBLE:
            if (!(c.offset_ms > -c.size_ms && c.offset_ms < c.size_ms))
                return fail(FW_E_INVALID, "Tumbling Window parameters must satisfy abs(offset) < size");
            w.interval = c.size_ms;
            w.n_slices = 1;
            if (c.api == FW_API_DATASTREAM) w.offset = c.offset_ms % c.size_ms;
            break;
        case FW_WIN_HOP:
            if (c.slide_ms <= 0) return fail(FW_E_INVALID, "Hopping Window must satisfy slide > 0 and size > 0");
            // SQL slices need slide | size (SliceAssigners.HoppingSliceAssigner); DataStream sliding
            // windows do not (SlidingEventTimeWindows.java:77-90): panes of gcd(size, slide) ms, each in
            // floor or ceil(size / slide) windows
            if (c.api != FW_API_DATASTREAM && c.size_ms % c.slide_ms != 0)
                return fail(FW_E_INVALID, "Slicing Hopping Window requires size must be an integral multiple of slide");
            if (c.api == FW_API_DATASTREAM && c.size_ms < c.slide_ms)  // gaps: panes in no window (not eligible)
                return fail(FW_E_INVALID, "sliding windows with size < slide run on the reference operator");
            if (c.api == FW_API_DATASTREAM && !(c.offset_ms > -c.slide_ms && c.offset_ms < c.slide_ms))
                return fail(FW_E_INVALID, "SlidingEventTimeWindows parameters must satisfy abs(offset) < slide and size > 0");
            w.interval = gcd64(c.size_ms, c.slide_ms);
            w.n_slices = (int32_t)(c.size_ms / w.interval);
            break;
        case FW_WIN_CUMULATE:
            if (c.api != FW_API_SQL) return fail(FW_E_INVALID, "CUMULATE is a SQL window");
            if (c.slide_ms <= 0 || c.size_ms % c.slide_ms != 0)
                return fail(FW_E_INVALID, "Cumulative Window requires maxSize must be an integral multiple of step");
            w.interval = c.slide_ms;
            w.n_slices = (int32_t)(c.size_ms / c.slide_ms);
            break;
        default: return fail(FW_E_INVALID, "bad window kind %d", c.window_kind);
    }
    w.ds = c.api == FW_API_DATASTREAM;
    w.slide = c.window_kind == FW_WIN_HOP ? c.slide_ms : c.size_ms;
    w.n_win = (w.ds && c.window_kind == FW_WIN_HOP) ? (int32_t)((c.size_ms + c.slide_ms - 1) / c.slide_ms) : 1;
    w.slide_div = make_udiv((uint64_t)w.slide);
    // ---- lateness (DataStream) and shift time zone (SQL TIMESTAMP_LTZ)
    if (c.allowed_lateness_ms < 0) return fail(FW_E_INVALID, "The allowed lateness cannot be negative.");
    if (c.api == FW_API_SQL && (c.allowed_lateness_ms != 0 || c.late_side_output))
        return fail(FW_E_INVALID, "allowed lateness and late side outputs are DataStream WindowOperator features");
    w.lateness = c.allowed_lateness_ms;
    if (c.tz_n < 0) return fail(FW_E_INVALID, "tz_n must be >= 0");
    if (c.tz_n > 0) {
        if (c.api != FW_API_SQL) return fail(FW_E_INVALID, "shift time zones belong to SQL TIMESTAMP_LTZ windows");
        if (!c.tz_utc || !c.tz_offset_ms) return fail(FW_E_INVALID, "tz_utc / tz_offset_ms required when tz_n > 0");
        if (c.tz_utc[0] != INT64_MIN) return fail(FW_E_INVALID, "tz_utc[0] must be Long.MIN_VALUE");
        h->tz_utc.assign(c.tz_utc, c.tz_utc + c.tz_n);
        h->tz_off.assign(c.tz_offset_ms, c.tz_offset_ms + c.tz_n);
        h->tz_bound.assign(c.tz_n, INT64_MIN);
        for (int i = 1; i < c.tz_n; i++) {
            if (h->tz_utc[i] <= h->tz_utc[i - 1]) return fail(FW_E_INVALID, "tz_utc must be strictly ascending");
            if (h->tz_off[i] < -18 * 3600000ll || h->tz_off[i] > 18 * 3600000ll) return fail(FW_E_INVALID, "offset out of range");
            h->tz_bound[i] = h->tz_utc[i] + std::max(h->tz_off[i - 1], h->tz_off[i]);
            if (h->tz_bound[i] <= h->tz_bound[i - 1]) return fail(FW_E_INVALID, "tz transitions too close together");
        }
    }
    w.tz = TzTable{h->tz_utc.data(), h->tz_off.data(), h->tz_bound.data(), c.tz_n, c.tz_use_dst ? 1 : 0};
    w.slice_div = make_udiv((uint64_t)w.interval);
    w.size_div = make_udiv((uint64_t)w.size);
    w.fast32 = w.interval < (1ll << 30) && w.offset < (1ll << 61) && w.offset > -(1ll << 61);
    w.slice_div32 = make_udiv32(w.fast32 ? (uint32_t)w.interval : 1u);
    h->always_flush = c.api == FW_API_DATASTREAM;

    // ---- aggregates -> accumulator words
    if (c.api == FW_API_DATASTREAM && c.nullable_cols)
        return fail(FW_E_INVALID, "DataStream field aggregations have no NULL inputs");
    if (c.agg_phase != FW_PHASE_ONE && c.agg_phase != FW_PHASE_LOCAL && c.agg_phase != FW_PHASE_GLOBAL)
        return fail(FW_E_INVALID, "bad agg_phase %d", c.agg_phase);
    if (c.agg_phase != FW_PHASE_ONE && c.api != FW_API_SQL) return fail(FW_E_INVALID, "two-phase aggregation is SQL only");
    WordDesc& wd = h->wd;
    AggDesc& ad = h->ad;
    wd.nw = 0;
    wd.has_q = 0;
    int nslot = 0;
    auto nullable = [&](int col) { return ((c.nullable_cols >> col) & 1u) != 0; };
    auto slot_of = [&](int col) -> int {
        for (int s = 0; s < nslot; s++)
            if (h->slot_col[s] == col) return s;
        if (nslot >= MAX_KCOLS) return -1;
        h->slot_col[nslot] = col;
        return nslot++;
    };
    // one word per (op, slot, gate); COUNT words are identified by their gate alone
    auto word_of = [&](int op, int slot, int gate) -> int {
        for (int i = 0; i < wd.nw; i++)
            if (wd.op[i] == op && wd.gate[i] == gate && (op == W_CNT || wd.col[i] == slot)) return i;
        if (wd.nw >= MAX_WORDS) return -1;
        wd.op[wd.nw] = op;
        wd.col[wd.nw] = op == W_CNT ? 0 : slot;
        wd.gate[wd.nw] = gate;
        wd.qfirst[wd.nw] = -1;
        return wd.nw++;
    };
    ad.n = c.n_aggs;
    ad.count_star_word = -1;
    ad.first_word = -1;
    ad.by_prev = -1;
    for (int g = 0; g < FW_MAX_AGGS; g++) ad.dn_hi[g] = ad.dn_lo[g] = -1;
    if (c.ds_first_ordinals && c.api != FW_API_DATASTREAM)
        return fail(FW_E_INVALID, "ds_first_ordinals is a DataStream option (SQL output rows carry no input fields)");
    bool nn_star[FW_MAX_AGGS] = {};
    for (int g = 0; g < c.n_aggs; g++) {
        const fw_agg_desc& d = c.aggs[g];
        ad.kind[g] = d.kind;
        ad.type[g] = d.type;
        ad.w1[g] = ad.nn[g] = ad.qf[g] = ad.qn[g] = ad.qz[g] = -1;
        if (d.type < FW_T_I64 || d.type > FW_T_I32) return fail(FW_E_INVALID, "agg %d: bad type", g);
        const bool by = d.kind == FW_AGG_MINBY || d.kind == FW_AGG_MAXBY;
        if (d.flags & ~(by ? FW_AGGF_LAST : 0)) return fail(FW_E_INVALID, "agg %d: bad flags %d", g, d.flags);
        if (by && (c.api != FW_API_DATASTREAM || !c.ds_first_ordinals || c.n_aggs != 1))
            return fail(FW_E_INVALID, "minBy / maxBy are the one aggregation of a record-shaped DataStream operator (ds_first_ordinals)");
        int slot = 0, gate = -1;
        const bool global = c.agg_phase == FW_PHASE_GLOBAL;
        if (global) {
            // GLOBAL phase (GlobalAggCombiner.combine :77-110): the value columns are the local
            // accumulator fields the LOCAL phase emits, and every aggregate folds them with its
            // mergeExpressions: counts add, sums add (NULL-able), MIN/MAX compare, AVG adds its
            // (sum, count) pair.  Local counts and AVG sums are never NULL.
            if (d.input_col < 0 || d.input_col >= c.n_value_cols) return fail(FW_E_INVALID, "agg %d: bad input_col", g);
            const int sc = d.input_col;
            const bool fl = d.type == FW_T_F64;
            int w0 = -1;
            auto slot_chk = [&](int col) { const int sl = slot_of(col); return sl; };
            switch (d.kind) {
                case FW_AGG_COUNT_STAR:
                case FW_AGG_COUNT:
                    if (c.value_col_types[sc] != FW_T_I64 || nullable(sc))
                        return fail(FW_E_INVALID, "agg %d: a local count column is a NOT NULL BIGINT", g);
                    if ((slot = slot_chk(sc)) < 0) return fail(FW_E_INVALID, "more than %d distinct value columns", MAX_KCOLS);
                    w0 = word_of(W_CNTV, slot, -1);
                    break;
                case FW_AGG_AVG: {
                    if (sc + 1 >= c.n_value_cols || c.value_col_types[sc] != (fl ? FW_T_F64 : FW_T_I64) ||
                        c.value_col_types[sc + 1] != FW_T_I64 || nullable(sc) || nullable(sc + 1))
                        return fail(FW_E_INVALID, "agg %d: a local AVG is a NOT NULL (sum, BIGINT count) column pair", g);
                    const int s0 = slot_chk(sc), s1 = slot_chk(sc + 1);
                    if (s0 < 0 || s1 < 0) return fail(FW_E_INVALID, "more than %d distinct value columns", MAX_KCOLS);
                    w0 = word_of(fl ? W_SUM_F : W_SUM_I, s0, -1);
                    ad.w1[g] = word_of(W_CNTV, s1, -1);
                    if (ad.w1[g] < 0) return fail(FW_E_INVALID, "too many accumulator words");
                    break;
                }
                default: w0 = -2; break;  // SUM / MIN / MAX: as in one phase, below
            }
            if (w0 != -2) {
                if (w0 < 0) return fail(FW_E_INVALID, "too many accumulator words");
                ad.w0[g] = w0;
                continue;
            }
        }
        if (d.kind != FW_AGG_COUNT_STAR) {
            if (d.input_col < 0 || d.input_col >= c.n_value_cols) return fail(FW_E_INVALID, "agg %d: bad input_col", g);
            if (c.value_col_types[d.input_col] != d.type)
                return fail(FW_E_INVALID, "agg %d: type does not match value column type", g);
            if (d.kind != FW_AGG_COUNT || nullable(d.input_col)) {
                slot = slot_of(d.input_col);
                if (slot < 0) return fail(FW_E_INVALID, "more than %d distinct value columns", MAX_KCOLS);
                if (nullable(d.input_col)) gate = slot;
            }
        }
        if (c.api == FW_API_DATASTREAM && (d.kind == FW_AGG_AVG || d.kind == FW_AGG_COUNT))
            return fail(FW_E_INVALID, "DataStream built-in aggregations are sum/min/max (and COUNT_STAR)");
        const bool f = d.type == FW_T_F64;
        // non-NULL count of the input: gated COUNT for a nullable column, else COUNT(*)
        const int cnt_op = W_CNT;
        int w0 = -1;
        switch (d.kind) {
            case FW_AGG_COUNT_STAR: w0 = word_of(cnt_op, 0, -1); break;
            case FW_AGG_COUNT: w0 = word_of(cnt_op, slot, gate); break;
            case FW_AGG_SUM:
                w0 = word_of(f ? W_SUM_F : W_SUM_I, slot, gate);
                if (gate >= 0) ad.nn[g] = word_of(cnt_op, slot, gate);
                else nn_star[g] = true;
                break;
            case FW_AGG_MIN:
            case FW_AGG_MAX: {
                const bool mx = d.kind == FW_AGG_MAX;
                if (f && c.api == FW_API_SQL) {  // strict comparison in arrival order: word group
                    w0 = word_of(mx ? W_QMAX : W_QMIN, slot, gate);
                    ad.qf[g] = word_of(W_QFIRST, slot, gate);
                    ad.qn[g] = word_of(W_QNANLO, slot, gate);
                    ad.qz[g] = word_of(W_QZERO, slot, gate);
                    if (w0 < 0 || ad.qf[g] < 0 || ad.qn[g] < 0 || ad.qz[g] < 0) return fail(FW_E_INVALID, "too many accumulator words");
                    wd.qfirst[w0] = wd.qfirst[ad.qn[g]] = ad.qf[g];
                    wd.has_q = 1;
                    break;
                }
                w0 = word_of(f ? (mx ? W_MAX_D : W_MIN_D) : (mx ? W_MAX_I : W_MIN_I), slot, gate);
                if (gate >= 0) ad.nn[g] = word_of(cnt_op, slot, gate);
                else nn_star[g] = true;
                if (f && c.api == FW_API_DATASTREAM) {  // the last NaN's bits (Comparator ties)
                    ad.dn_hi[g] = word_of(W_DNHI, slot, gate);
                    ad.dn_lo[g] = word_of(W_DNLO, slot, gate);
                    if (ad.dn_hi[g] < 0 || ad.dn_lo[g] < 0) return fail(FW_E_INVALID, "too many accumulator words");
                }
                break;
            }
            case FW_AGG_AVG:
                w0 = word_of(f ? W_SUM_F : W_SUM_I, slot, gate);
                ad.w1[g] = word_of(cnt_op, slot, gate);
                break;
            case FW_AGG_MINBY:
            case FW_AGG_MAXBY: {  // the arg's field key, its ordinal, the ordinal the host retains
                const bool mx = d.kind == FW_AGG_MAXBY;
                w0 = word_of(f ? (mx ? W_BYMAX_D : W_BYMIN_D) : (mx ? W_BYMAX_I : W_BYMIN_I), slot, gate);
                ad.first_word = word_of((d.flags & FW_AGGF_LAST) ? W_BYO_LAST : W_BYO_FIRST, 0, -1);
                ad.by_prev = word_of(W_BYPREV, 0, -1);
                if (ad.first_word < 0 || ad.by_prev < 0) return fail(FW_E_INVALID, "too many accumulator words");
                break;
            }
            default: return fail(FW_E_INVALID, "agg %d: unsupported kind %d", g, d.kind);
        }
        if (w0 < 0 || (d.kind == FW_AGG_AVG && ad.w1[g] < 0)) return fail(FW_E_INVALID, "too many accumulator words");
        if ((d.kind == FW_AGG_SUM || d.kind == FW_AGG_MIN || d.kind == FW_AGG_MAX) && gate >= 0 && ad.nn[g] < 0 && ad.qf[g] < 0)
            return fail(FW_E_INVALID, "too many accumulator words");
        ad.w0[g] = w0;
    }
    if (c.count_star_index >= 0) {
        if (c.count_star_index >= c.n_aggs) return fail(FW_E_INVALID, "count_star_index out of range");
        const int k = c.aggs[c.count_star_index].kind;
        if (k != FW_AGG_COUNT_STAR && k != FW_AGG_COUNT) return fail(FW_E_INVALID, "count_star_index is not a COUNT");
        ad.count_star_word = ad.w0[c.count_star_index];
    } else if (c.window_kind == FW_WIN_HOP) {
        if (c.api == FW_API_SQL) return fail(FW_E_INVALID, "Hopping window requires a COUNT(*) in the aggregate functions.");
        // DataStream sliding windows emit a window iff it received an element: hidden COUNT(*)
        ad.count_star_word = word_of(W_CNT, 0, -1);
        if (ad.count_star_word < 0) return fail(FW_E_INVALID, "too many accumulator words");
    }
    if (c.ds_first_ordinals && ad.by_prev < 0) {
        ad.first_word = word_of(W_FIRST, 0, -1);
        if (ad.first_word < 0) return fail(FW_E_INVALID, "too many accumulator words");
    }
    wd.has_ord = wd.has_q;
    for (int i = 0; i < wd.nw; i++) wd.has_ord |= wd.op[i] == W_FIRST || is_dnword(wd.op[i]) || is_byword(wd.op[i]);
    // NOT NULL inputs: SUM / MIN / MAX are NULL only for an entry without rows (COUNT(*) == 0),
    // which needs a COUNT(*) word to be observable; without one such an entry never fires
    int star = -1;
    for (int i = 0; i < wd.nw; i++)
        if (wd.op[i] == W_CNT && wd.gate[i] < 0) star = i;
    for (int g = 0; g < c.n_aggs; g++)
        if (nn_star[g]) ad.nn[g] = star;
    h->nv = nslot;
    h->nw_t = round_nw(wd.nw);
    h->n_out = c.n_aggs + (ad.first_word >= 0 ? 1 : 0);  // + value1's ordinal (fw_result.first_ord)
    if (c.agg_phase == FW_PHASE_LOCAL) {  // output = local accumulator fields (AVG: sum, count)
        h->n_out = 0;
        for (int g = 0; g < c.n_aggs; g++) h->n_out += c.aggs[g].kind == FW_AGG_AVG ? 2 : 1;
        if (h->n_out > FW_MAX_AGGS) return fail(FW_E_INVALID, "LOCAL phase: more than %d accumulator fields", FW_MAX_AGGS);
    }
    for (int i = wd.nw; i < MAX_WORDS; i++) {
        wd.op[i] = W_CNT;
        wd.col[i] = 0;
        wd.gate[i] = -1;
        wd.qfirst[i] = -1;
    }

    // ---- key space: this subtask's key groups, split into superbuckets
    KeySpace& ks = h->ks;
    ks.hash_kind = h->keyrow ? FW_KEYHASH_PRECOMPUTED : c.key_hash;  // key rows route by their interned hash
    ks.max_p = c.max_parallelism;
    ks.maxp_div = make_udiv32((uint32_t)c.max_parallelism);
    ks.kg_start = (c.subtask_index * c.max_parallelism + c.parallelism - 1) / c.parallelism;
    const int kg_end = ((c.subtask_index + 1) * c.max_parallelism - 1) / c.parallelism;
    ks.n_kg = kg_end - ks.kg_start + 1;
    // SQL HOP with few slices per window and plain accumulators keeps block state (k_merge_hopb):
    // one entry per (key, HB_R consecutive slices) instead of one per (key, slice)
    const char* hb_env = getenv("FW_HOPB");
    if (const char* nv = getenv("FW_HB_NARROW")) h->hb_narrow = std::min(std::max(atoi(nv), 0), 2);
    w.hopb = c.api == FW_API_SQL && c.window_kind == FW_WIN_HOP && c.agg_phase != FW_PHASE_LOCAL && !wd.has_q &&
             h->nw_t <= 2 && w.n_slices <= HB_R && !(hb_env && atoi(hb_env) == 0);
    if (w.hopb) {
        w.hb_span = HB_R * w.interval;
        w.hb_span_div = make_udiv((uint64_t)w.hb_span);
    }
    h->pwe = 3 + (w.hopb ? HB_R * h->nw_t : h->nw_t);
    // the hint counts (key, slice) entries; a key's live slices (a window plus the batch's newer
    // ones) fit one or two blocks
    const int64_t cap_target = std::max<int64_t>(
        w.hopb ? c.state_capacity * 3 / (2 * (w.n_slices + 3)) : c.state_capacity, 1024);
    // aim for <= ~75% occupancy of the per-superbucket LDS entry table at the hinted capacity (the
    // index has 2E slots, so its load factor stays <= 38%); fewer, fuller superbuckets amortise the
    // merge kernel's per-workgroup costs (CFG5: 4096 -> 2048 superbuckets, merge -27%)
    h->cap_e = mg_entries(h->nw_t, c.api == FW_API_DATASTREAM ? KIND_DSWIN : w.hopb ? KIND_HOPB : c.window_kind);
    const int64_t fill = h->cap_e * h->fill_pct / 100;
    int64_t per_kg = (cap_target + ks.n_kg - 1) / ks.n_kg;
    int64_t sbk = next_pow2((per_kg + fill - 1) / fill);
    // beyond IG_MAX_SB superbuckets the ingest partitions coarser than the state (KeySpace
    // pass_log2): up to MAX_PASS_LOG2 merge passes share one ingest superbucket's partial rows.  A
    // pass re-routes each row's key, so precomputed-hash keys (no hash in the partial rows) cap
    // the state at IG_MAX_SB superbuckets
    const int max_pl = ks.hash_kind == KH_PRE ? 0 : MAX_PASS_LOG2;
    const int64_t max_sb = (int64_t)IG_MAX_SB << max_pl;
    while ((int64_t)ks.n_kg * sbk > max_sb && sbk > 1) sbk >>= 1;
    if ((int64_t)ks.n_kg * sbk > max_sb) return fail(FW_E_INVALID, "too many key groups per subtask for the ingest histogram");
    ks.sb_per_kg_log2 = 0;
    while ((1ll << ks.sb_per_kg_log2) < sbk) ks.sb_per_kg_log2++;
    ks.n_sb = ks.n_kg << ks.sb_per_kg_log2;
    ks.pass_log2 = 0;
    while ((ks.n_sb >> ks.pass_log2) > IG_MAX_SB) ks.pass_log2++;
    if (ks.pass_log2 > ks.sb_per_kg_log2) return fail(FW_E_INVALID, "superbucket split finer than a key group's passes");
    if (c.max_batch_rows <= 0) return fail(FW_E_INVALID, "max_batch_rows must be > 0");
    if (c.output_capacity <= 0) return fail(FW_E_INVALID, "output_capacity must be > 0");
    h->chunk_rows = (int64_t)ig_block(h->nw_t, ig_nv(h->nv)) * ig_rpt(h->nw_t, ig_nv(h->nv));
    h->cap_rows = ((c.max_batch_rows + h->chunk_rows - 1) / h->chunk_rows) * h->chunk_rows;
    h->max_nch = h->cap_rows / h->chunk_rows;
    if (wd.has_ord && (int64_t)FW_MAX_PENDING * h->cap_rows >= (1ll << 32) - 1)
        return fail(FW_E_INVALID, "max_batch_rows too large for MIN/MAX(DOUBLE) / first-element arrival ordinals");
    h->cell_cols = cell_pad(h->max_nch);
    // compact partial rows: SQL rows on the UTC slice grid (the ingest kernel's common path; it falls
    // back to PF_WIDE per chunk), planned for COUNT(*)-only layouts, whose compact row is the key alone:
    // for the others the merge gather's cost of reading two formats outweighed the bytes saved
    // (DESIGN.md 5).  Key-row handles keep PF_WIDE: their collector reads the partial buffer's keys at
    // a fixed stride; split superbuckets (pass_log2) too.  FW_NARROW=0 switches them off (development).
    {
        const char* ne = getenv("FW_NARROW");
        const char* ne1 = getenv("FW_NARROW1");
        const bool count_only = wd.nw == 1 && wd.op[0] == W_CNT && wd.gate[0] < 0;
        // one accumulator word of a class with a compiled merge variant (MergeLayouts<1>): (key, acc)
        // rows, 17 B instead of 24 B per partial with the rank byte
        const bool one_word = wd.nw == 1 && !wd.has_q && !wd.has_ord && wd.gate[0] < 0 && ops_layout(wd) != OPS_ANY;
        const bool ok = c.api == FW_API_SQL && !h->keyrow && c.agg_phase != FW_PHASE_GLOBAL && h->tz_utc.empty() &&
                        w.fast32 && ks.pass_log2 == 0 && !(ne && atoi(ne) == 0) && (h->chunk_rows & (h->chunk_rows - 1)) == 0;
        // (one-word MAX / MIN / SUM layouts read compact rows slower in the merge than they save in the
        // ingest: measured 163 vs 148 us per CFG2 flush, ingest -1.6 us; FW_NARROW1=1 plans them)
        h->narrow = !ok ? 0 : count_only ? 2 : (one_word && ne1 && atoi(ne1) == 1) ? 1 : 0;
    }
    // runs: every chunk claims its stretch of each superbucket's sub-runs, so the merge streams a
    // superbucket's rows (fw_internal.h RUN_X).  Sub-runs hold 5/4 of a uniform share of a full push
    // (+16 rows); skew beyond that stays in the chunks' regions (overflow flags).  Off for key-row
    // handles (their collector reads the chunk regions) and split superbuckets (pass_log2: several
    // readers per ingest superbucket); FW_RUNS=1 / 0 forces them on / off (development A/B).
    {
        const char* re = getenv("FW_RUNS");
        const int n_isb = ks.n_sb >> ks.pass_log2;
        const int blk = ig_block(h->nw_t, ig_nv(h->nv)), rpt = ig_rpt(h->nw_t, ig_nv(h->nv));
        // measured per step: CFG4 (TUMBLE, two words) +2-4%, CFG2 (TUMBLE, one word) +1.5%
        // with its one-block runs gather (round 5: ingest +11 us, merge -14 us), CFG3 (HOP) -5%, CFG5
        // (CUMULATE) -3% -- the ingest's scattered stretch stores cost more than the merge saves there;
        // planned for SQL TUMBLE, FW_RUNS=1 plans them everywhere
        const bool want = re ? atoi(re) != 0 : (c.window_kind == FW_WIN_TUMBLE && c.api == FW_API_SQL);
        if (!h->keyrow && ks.pass_log2 == 0 && ig_runs_fit(n_isb, blk, rpt, h->nw_t) && want) {
            const int64_t subs = (int64_t)n_isb * RUN_X;
            const int64_t sc = ((h->cap_rows * 5 / 4 + subs - 1) / subs + 16 + 15) / 16 * 16;
            if (sc * subs < (1ll << 31)) {
                h->sub_cap = (int32_t)sc;
                h->run_rows = sc * subs;
            }
        }
    }
    // PF_PACK run rows: one 8-B word per partial (key and accumulator offsets, slice rank) for the
    // one-word integer layouts on the compact rows' conditions (COUNT / SUM / MIN / MAX of BIGINT or
    // INT, no NULLs); 24 -> 8 B per partial on the ingest's stores and the merge's reads.  FW_PACK=0
    // switches them off (A/B).
    {
        const char* pe = getenv("FW_PACK");
        const int32_t op = wd.op[0];
        const bool int_word = wd.nw == 1 && !wd.has_q && !wd.has_ord && wd.gate[0] < 0 &&
                              (op == W_CNT || op == W_SUM_I || op == W_MIN_I || op == W_MAX_I) && ops_layout(wd) != OPS_ANY;
        const bool ok = c.api == FW_API_SQL && !h->keyrow && c.agg_phase != FW_PHASE_GLOBAL && h->tz_utc.empty() &&
                        w.fast32 && ks.pass_log2 == 0 && (h->chunk_rows & (h->chunk_rows - 1)) == 0;
        h->pack = ok && int_word && h->run_rows > 0 && !(pe && atoi(pe) == 0);
    }
    h->treq_cap = std::max<int64_t>(c.max_batch_rows * 2, 1 << 16);
    if (c.api == FW_API_DATASTREAM) {
        if (c.allowed_lateness_ms > 0 && (int64_t)FW_MAX_PENDING * h->cap_rows >= (1ll << 32) - 1)
            return fail(FW_E_INVALID, "max_batch_rows too large for late-element arrival ordinals");
        h->lfire_cap = c.allowed_lateness_ms > 0 ? h->treq_cap : 0;
        h->side_cap = c.late_side_output ? h->treq_cap : 0;
        // retains per flush <= new windows of its rows; releases <= live windows
        h->ordev_cap = ad.first_word >= 0
                           ? ((int64_t)FW_MAX_PENDING * h->cap_rows + std::max<int64_t>(c.state_capacity, 0)) * w.n_win + (1 << 16)
                           : 0;
    }
    h->out_cap = c.output_capacity;
    h->slab_cap = std::max<int64_t>(64, (2 * c.output_capacity + ks.n_sb - 1) / ks.n_sb);
    h->stage_cap = c.max_batch_rows;
    if (h->keyrow) {
        h->kr.cap_ids = std::max<int64_t>(1024, std::max<int64_t>(c.state_capacity, 0) + (int64_t)FW_MAX_PENDING * c.max_batch_rows);
        if (h->kr.cap_ids >= (1ll << 31) - 2) return fail(FW_E_INVALID, "key-row table over 2^31 ids");
        h->kr.n_slots = next_pow2(2 * h->kr.cap_ids);
        h->krb_cap = c.max_batch_rows * (int64_t)h->kr.max_len;
    }
    return FW_OK;
}

// queues the DMA of async result buffer b's n rows into its pinned host buffers on the D2H stream
int ar_enqueue_copy(fw_handle* h, int b, int64_t n) {
    hipStream_t ds = h->d2h_stream;
    HIP_TRY(hipMemcpyAsync(h->ar_key[b], h->ard_key[b], (size_t)n * 8, hipMemcpyDeviceToHost, ds));
    HIP_TRY(hipMemcpyAsync(h->ar_ws[b], h->ard_ws[b], (size_t)n * 8, hipMemcpyDeviceToHost, ds));
    HIP_TRY(hipMemcpyAsync(h->ar_we[b], h->ard_we[b], (size_t)n * 8, hipMemcpyDeviceToHost, ds));
    HIP_TRY(hipMemcpyAsync(h->ar_null[b], h->ard_null[b], (size_t)n * 4, hipMemcpyDeviceToHost, ds));
    for (int g = 0; g < h->n_out; g++)
        HIP_TRY(hipMemcpyAsync(h->ar_val[b][g], h->ard_val[b][g], (size_t)n * 8, hipMemcpyDeviceToHost, ds));
    HIP_TRY(hipEventRecord(h->ar_dma_ev[b], ds));
    return FW_OK;
}

// Starts the DMA of the last fw_results_async's rows as soon as its compaction has finished, from
// the calls a pipelined caller makes between fw_results_async and fw_results_ready (the next batch's
// fw_commit / push, fw_advance): the copy then runs beside that batch's kernels and
// fw_results_ready finds it done.  Never blocks; any failure is left for fw_results_ready.
void ar_kick(fw_handle* h) {
    if (h->ar_kernel || !h->d2h_stream) return;
    for (int i = 0; i < h->ar_qn; i++) {  // outstanding collections, oldest first
        const int b = h->ar_q[(h->ar_qhead + i) % FW_AR_BUFS];
        if (h->ar_empty[b] || h->ar_copied[b] || h->ar_inflight[b]) continue;
        if (hipEventQuery(h->ar_ev[b]) != hipSuccess) {  // compaction still queued: try at the next call
            (void)hipGetLastError();
            return;
        }
        const int64_t n = __atomic_load_n(h->ar_n[b], __ATOMIC_ACQUIRE);
        if (n <= 0 || n > h->out_cap) continue;
        if (ar_enqueue_copy(h, b, n) != FW_OK) {
            (void)hipGetLastError();
            return;
        }
        h->ar_inflight[b] = true;
    }
}

template <typename T>
int dalloc(T** p, size_t count) {
    void* v = nullptr;
    HIP_TRY(hipMalloc(&v, std::max<size_t>(count, 1) * sizeof(T)));
    *p = (T*)v;
    return FW_OK;
}

int allocate(fw_handle* h) {
    const fw_config& c = h->cfg;
    HIP_TRY(hipSetDevice(c.device));
    HIP_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    int rc;
    const int PW = 2 + h->nw_t, PWE = h->pwe;
    if ((rc = dalloc(&h->ctrl, 1))) return rc;
    if ((rc = dalloc(&h->parts, (size_t)FW_MAX_PENDING * h->cap_rows * PW))) return rc;
    if ((rc = dalloc(&h->cells, (size_t)FW_MAX_PENDING * (h->ks.n_sb >> h->ks.pass_log2) * h->cell_cols))) return rc;
    if ((rc = dalloc(&h->slot_nch, FW_MAX_PENDING))) return rc;
    if ((rc = dalloc(&h->slot_base, FW_MAX_PENDING))) return rc;
    if (h->narrow && (rc = dalloc(&h->ranks, (size_t)FW_MAX_PENDING * h->cap_rows))) return rc;
    if (h->run_rows) {
        // the runs layout is a plan, not a requirement: FW_MAX_PENDING * run_rows partial rows (about
        // 1.25x the partial buffer) on top of it.  When the device cannot hold them the handle keeps
        // the cell layout instead of failing fw_create.
        void* r = nullptr;
        void* rr = nullptr;
        if (hipMalloc(&r, (size_t)FW_MAX_PENDING * h->run_rows * PW * sizeof(uint64_t)) != hipSuccess ||
            (h->narrow && hipMalloc(&rr, (size_t)FW_MAX_PENDING * h->run_rows) != hipSuccess)) {
            (void)hipGetLastError();
            if (r) hipFree(r);
            h->run_rows = 0;
            h->sub_cap = 0;
            h->pack = 0;
        } else {
            h->runs = (uint64_t*)r;
            h->run_ranks = (uint8_t*)rr;
        }
    }
    if (h->run_rows) {
        const size_t n_isb = (size_t)(h->ks.n_sb >> h->ks.pass_log2);
        if ((rc = dalloc(&h->run_fill, (size_t)FW_MAX_PENDING * RUN_X * n_isb))) return rc;
        if ((rc = dalloc(&h->run_ovf, (size_t)FW_MAX_PENDING * n_isb))) return rc;
        if ((rc = dalloc(&h->slot_fmt, FW_MAX_PENDING))) return rc;
        HIP_TRY(hipMemsetAsync(h->run_fill, 0, sizeof(uint32_t) * FW_MAX_PENDING * RUN_X * n_isb, h->stream));
        HIP_TRY(hipMemsetAsync(h->run_ovf, 0, sizeof(uint32_t) * FW_MAX_PENDING * n_isb, h->stream));
        HIP_TRY(hipMemsetAsync(h->slot_fmt, 0, sizeof(int32_t) * FW_MAX_PENDING, h->stream));
    }
    if ((rc = dalloc(&h->treq, (size_t)h->treq_cap * 3))) return rc;
    if (h->lfire_cap && (rc = dalloc(&h->lfire, (size_t)h->lfire_cap * LFW))) return rc;
    if (h->side_cap && (rc = dalloc(&h->side, (size_t)h->side_cap * SOW))) return rc;
    if (h->ordev_cap && (rc = dalloc(&h->ordev, (size_t)h->ordev_cap))) return rc;
    if (h->keyrow) {
        KeyRowTable& t = h->kr;
        if ((rc = dalloc(&t.slots, (size_t)t.n_slots))) return rc;
        if ((rc = dalloc(&t.arena, (size_t)t.cap_ids * t.stride_words))) return rc;
        if ((rc = dalloc(&t.mark, (size_t)t.cap_ids))) return rc;
        if ((rc = dalloc(&t.free_list, (size_t)t.cap_ids))) return rc;
        HIP_TRY(hipMemsetAsync(t.slots, 0, sizeof(uint32_t) * t.n_slots, h->stream));
        HIP_TRY(hipMemsetAsync(t.mark, 0, sizeof(uint32_t) * t.cap_ids, h->stream));
        if ((rc = dalloc(&h->res_kr_len, (size_t)h->out_cap))) return rc;
        if ((rc = dalloc(&h->res_kr_img, (size_t)h->out_cap * (t.stride_words - 1)))) return rc;
    }
    if (!h->tz_utc.empty()) {  // shift-zone table on the device; the kernels' WinDesc points at it
        const size_t n = h->tz_utc.size();
        if ((rc = dalloc(&h->d_tz, 3 * n))) return rc;
        HIP_TRY(hipMemcpy(h->d_tz, h->tz_utc.data(), 8 * n, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(h->d_tz + n, h->tz_off.data(), 8 * n, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(h->d_tz + 2 * n, h->tz_bound.data(), 8 * n, hipMemcpyHostToDevice));
    }
    if ((rc = dalloc(&h->state, (size_t)h->ks.n_sb * h->cap_e * PWE))) return rc;
    if ((rc = dalloc(&h->state_count, h->ks.n_sb))) return rc;
    if ((rc = dalloc(&h->sb_min_timer, h->ks.n_sb))) return rc;
    if ((rc = dalloc(&h->sb_nar, h->ks.n_sb))) return rc;
    const size_t orows = (size_t)h->ks.n_sb * h->slab_cap + h->out_cap;
    if ((rc = dalloc(&h->out_key, orows))) return rc;
    if ((rc = dalloc(&h->out_we, orows))) return rc;
    if ((rc = dalloc(&h->out_null, orows))) return rc;
    for (int g = 0; g < h->n_out; g++)
        if ((rc = dalloc(&h->out_val[g], orows))) return rc;
    if ((rc = dalloc(&h->res_key, h->out_cap))) return rc;
    if ((rc = dalloc(&h->res_ws, h->out_cap))) return rc;
    if ((rc = dalloc(&h->res_we, h->out_cap))) return rc;
    if ((rc = dalloc(&h->res_null, h->out_cap))) return rc;
    for (int g = 0; g < h->n_out; g++)
        if ((rc = dalloc(&h->res_val[g], h->out_cap))) return rc;
    if ((rc = dalloc(&h->sb_out, h->ks.n_sb + 1))) return rc;  // + the overflow region's rows
    if ((rc = dalloc(&h->sb_fired, h->ks.n_sb))) return rc;
    if ((rc = dalloc(&h->coff, h->ks.n_sb + 2))) return rc;
    if ((rc = dalloc(&h->chunk_stats, CS_WORDS * (h->max_nch + 1)))) return rc;
    if ((rc = dalloc(&h->stamps, N_STAMPS))) return rc;
    if ((rc = dalloc(&h->kt_dev, FW_KT_N * KT_WORDS))) return rc;
    if ((rc = dalloc(&h->tickets, 1))) return rc;
    HIP_TRY(hipHostMalloc((void**)&h->mirror, sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent));
    *h->mirror = ~0ull;
    HIP_TRY(hipHostGetDevicePointer((void**)&h->d_mirror, (void*)h->mirror, 0));
    HIP_TRY(hipMemsetAsync(h->tickets, 0, sizeof(Tickets), h->stream));
    HIP_TRY(hipMemsetAsync(h->stamps, 0, sizeof(unsigned long long) * N_STAMPS, h->stream));
    HIP_TRY(hipMemsetAsync(h->kt_dev, 0, sizeof(unsigned long long) * FW_KT_N * KT_WORDS, h->stream));
    HIP_TRY(hipMemsetAsync(h->sb_out, 0, sizeof(int32_t) * (h->ks.n_sb + 1), h->stream));
    HIP_TRY(hipMemsetAsync(h->sb_fired, 0, sizeof(uint32_t) * h->ks.n_sb, h->stream));
    HIP_TRY(hipMemsetAsync(h->state_count, 0, sizeof(int32_t) * h->ks.n_sb, h->stream));
    HIP_TRY(hipMemsetAsync(h->sb_nar, 0, h->ks.n_sb, h->stream));
    std::vector<int64_t> inf(h->ks.n_sb, INT64_MAX);
    HIP_TRY(hipMemcpyAsync(h->sb_min_timer, inf.data(), sizeof(int64_t) * h->ks.n_sb, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(launch_init_ctrl(h->ctrl, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return FW_OK;
}

int alloc_staging(fw_handle* h) {
    if (h->d_ts[0]) return FW_OK;
    const fw_config& c = h->cfg;
    const size_t n = (size_t)h->stage_cap;
    HIP_TRY(hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking));
    int rc;
    for (int b = 0; b < FW_STAGE_BUFS; b++) {
        HIP_TRY(hipHostMalloc((void**)&h->h_key[b], n * 8, hipHostMallocDefault));
        HIP_TRY(hipHostMalloc((void**)&h->h_ts[b], n * 8, hipHostMallocDefault));
        HIP_TRY(hipHostMalloc((void**)&h->h_kh[b], n * 4, hipHostMallocDefault));
        for (int v = 0; v < c.n_value_cols; v++) {
            HIP_TRY(hipHostMalloc((void**)&h->h_val[b][v], n * 8, hipHostMallocDefault));
            if ((c.nullable_cols >> v) & 1u) HIP_TRY(hipHostMalloc((void**)&h->h_nul[b][v], n, hipHostMallocDefault));
        }
        HIP_TRY(hipEventCreateWithFlags(&h->stage_ev[b], hipEventDisableTiming));
        HIP_TRY(hipEventRecord(h->stage_ev[b], h->cstream));
        HIP_TRY(hipEventCreateWithFlags(&h->dstage_free[b], hipEventDisableTiming));
        HIP_TRY(hipEventRecord(h->dstage_free[b], h->stream));
        if (h->keyrow) {
            HIP_TRY(hipHostMalloc((void**)&h->h_kro[b], (n + 1) * 8, hipHostMallocDefault));
            HIP_TRY(hipHostMalloc((void**)&h->h_krb[b], (size_t)std::max<int64_t>(h->krb_cap, 8), hipHostMallocDefault));
            if ((rc = dalloc(&h->d_kro[b], n + 1))) return rc;
            if ((rc = dalloc(&h->d_krb[b], (size_t)std::max<int64_t>(h->krb_cap, 8)))) return rc;
        } else {
            if ((rc = dalloc(&h->d_key[b], n))) return rc;
        }
        if ((rc = dalloc(&h->d_ts[b], n))) return rc;
        if (c.key_hash == FW_KEYHASH_PRECOMPUTED && (rc = dalloc(&h->d_kh[b], n))) return rc;
        for (int v = 0; v < c.n_value_cols; v++) {
            if ((rc = dalloc(&h->d_val[b][v], n))) return rc;
            if (((c.nullable_cols >> v) & 1u) && (rc = dalloc(&h->d_nul[b][v], n))) return rc;
        }
    }
    return FW_OK;
}

// pinned, device-mapped result buffers of fw_results_async
int alloc_async_results(fw_handle* h) {
    if (h->ar_n[0]) return FW_OK;
    const size_t n = (size_t)h->out_cap;
    int rc;
    HIP_TRY(hipStreamCreateWithFlags(&h->d2h_stream, hipStreamNonBlocking));
    for (int b = 0; b < FW_AR_BUFS; b++) {
        // pinned host buffers: mapped for the kernel delivery, plain for the DMA
        const unsigned fl = h->ar_kernel ? hipHostMallocMapped : hipHostMallocDefault;
        HIP_TRY(hipHostMalloc((void**)&h->ar_key[b], n * 8, fl));
        HIP_TRY(hipHostMalloc((void**)&h->ar_ws[b], n * 8, fl));
        HIP_TRY(hipHostMalloc((void**)&h->ar_we[b], n * 8, fl));
        HIP_TRY(hipHostMalloc((void**)&h->ar_null[b], n * 4, fl));
        for (int g = 0; g < h->n_out; g++) HIP_TRY(hipHostMalloc((void**)&h->ar_val[b][g], n * 8, fl));
        HIP_TRY(hipHostMalloc((void**)&h->ar_n[b], 8, hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipEventCreateWithFlags(&h->ar_ev[b], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&h->ar_dma_ev[b], hipEventDisableTiming));
        if ((rc = dalloc(&h->ard_key[b], n))) return rc;
        if ((rc = dalloc(&h->ard_ws[b], n))) return rc;
        if ((rc = dalloc(&h->ard_we[b], n))) return rc;
        if ((rc = dalloc(&h->ard_null[b], n))) return rc;
        for (int g = 0; g < h->n_out; g++)
            if ((rc = dalloc(&h->ard_val[b][g], n))) return rc;
    }
    return FW_OK;
}

template <typename T>
T* mapped(T* host) {
    void* d = nullptr;
    return hipHostGetDevicePointer(&d, (void*)host, 0) == hipSuccess ? (T*)d : nullptr;
}

int read_ctrl(fw_handle* h, Ctrl* out) {
    HIP_TRY(hipMemcpyAsync(out, h->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (out->error) {
        return fail(FW_E_CAPACITY, "device error (bits 0x%x:%s%s%s%s%s%s%s)", out->error,
                    out->error & ERR_CHUNKS ? " partial-buffer" : "", out->error & ERR_STATE ? " state-table" : "",
                    out->error & ERR_OUTPUT ? " result-buffer" : "", out->error & ERR_TREQ ? " timer-requests" : "",
                    out->error & ERR_KEYGROUP ? " key-group-not-owned" : "",
                    out->error & ERR_LATE ? " late-rows (call fw_late_records more often)" : "",
                    out->error & ERR_ORDEV ? " first-element-events (call fw_first_element_events after each advance)" : "");
    }
    return FW_OK;
}

// the window description the kernels get: the shift-zone table pointers are the device copy's
WinDesc device_win(const fw_handle* h) {
    WinDesc w = h->win;
    if (h->d_tz) {
        const size_t n = h->tz_utc.size();
        w.tz.utc = h->d_tz;
        w.tz.off = h->d_tz + n;
        w.tz.bound = h->d_tz + 2 * n;
    }
    return w;
}

MergeArgs merge_args(fw_handle* h, int64_t wm, int force) {
    MergeArgs a{};
    a.ks = h->ks;
    a.ctrl = h->ctrl;
    a.tickets = h->tickets;
    a.parts = h->parts;
    a.cells = h->cells;
    a.slot_nch = h->slot_nch;
    a.max_nch = h->cell_cols;
    a.cap_rows = h->cap_rows;
    a.treq = h->treq;
    a.state = h->state;
    a.state_count = h->state_count;
    a.sb_min_timer = h->sb_min_timer;
    a.sb_nar = h->sb_nar;
    a.hb_narrow = h->win.hopb ? h->hb_narrow : 0;
    a.n_sb = h->ks.n_sb;
    a.cap_e = h->cap_e;
    a.win = device_win(h);
    a.lfire = h->lfire;
    a.lfire_cap = h->lfire_cap;
    a.wd = h->wd;
    a.ad = h->ad;
    a.always_flush = h->always_flush;
    a.local = h->cfg.agg_phase == FW_PHASE_LOCAL;
    a.chunk_rows = (int32_t)h->chunk_rows;
    a.out_key = h->out_key;
    a.out_we = h->out_we;
    for (int g = 0; g < FW_MAX_AGGS; g++) a.out_val[g] = h->out_val[g] ? h->out_val[g] : h->out_val[0];
    a.out_null = h->out_null;
    a.out_cap = h->out_cap;
    a.slab_cap = h->slab_cap;
    a.sb_out = h->sb_out;
    a.sb_fired = h->sb_fired;
    a.wm = wm;
    a.force_flush = force;
    a.reset_out = h->reset_pending;
    a.ablate = h->ablate;
    a.stamps = h->stamps;
    a.kt = h->kt_device ? h->kt_dev + FW_KT_MERGE * KT_WORDS : nullptr;
    a.host_mirror = h->d_mirror;  // the launch's last workgroup reports merge_seq << 8 | pending pushes
    a.merge_seq = h->merge_seq;
    a.ordev = h->ordev;
    a.ordev_cap = h->ordev_cap;
    a.slot_base = h->slot_base;
    a.ranks = h->ranks;
    a.compact = h->narrow != 0 || h->pack != 0;
    a.runs = h->runs;
    a.run_ranks = h->run_ranks;
    a.run_fill = h->run_fill;
    a.run_ovf = h->run_ovf;
    a.slot_fmt = h->slot_fmt;
    a.run_rows = h->run_rows;
    a.sub_cap = h->sub_cap;
    a.ch_log2 = 0;
    while ((1ll << a.ch_log2) < h->chunk_rows) a.ch_log2++;
    return a;
}

int launch_merge(fw_handle* h, int64_t wm, int force) {
    HIP_TRY(launch_merge_fire(merge_args(h, wm, force), h->stream, h->timer));
    h->pushes_at_merge[h->merge_seq % 64] = h->pushes_total;
    h->merge_seq++;
    h->reset_pending = false;  // the launch started every output slab (and the overflow) afresh
    if (!force && wm > h->dev_cur) {  // merge_finalize's advanceProgress bookkeeping, mirrored
        h->dev_cur = wm;
        if (wm >= h->dev_ntp) h->dev_ntp = tz_next_trigger_watermark(h->win.tz, wm, h->win.slice_div);
    }
    return FW_OK;
}

int force_flush(fw_handle* h) {
    int rc = launch_merge(h, INT64_MIN, 1);
    if (rc) return rc;
    h->pushes_ub = 0;
    return FW_OK;
}

int push(fw_handle* h, int64_t n, const int64_t* key, const int64_t* ts, const int32_t* kh, const void* const* vals,
         const uint8_t* const* nulls, const int64_t* seg_counts = nullptr, int64_t seg_len = 1, int64_t stride = 1) {
    if (h->ad.first_word >= 0 && (n >= (1ll << 32) || h->push_seq >= (1 << 30)))
        return fail(FW_E_INVALID, "arrival ordinals need < 2^32 rows per call and < 2^30 calls");
    for (int64_t o = 0; o < n; o += h->cap_rows) {
        const int64_t m = std::min(h->cap_rows, n - o);
        if (h->pushes_ub >= FW_MAX_PENDING) {
            // what the last completed merge launch left pending, plus the pushes issued after it.
            // While merge launches issued since are still running, wait for them to report
            // instead of draining the stream: the queue stays busy while the host waits.
            const auto t0 = std::chrono::steady_clock::now();
            for (;;) {
                const unsigned long long v = *h->mirror;
                const uint64_t seq = v >> 8;
                const bool valid = v != ~0ull && seq < h->merge_seq && h->merge_seq - seq <= 64;
                if (valid)
                    h->pushes_ub = std::min<int64_t>(h->pushes_ub,
                                                     (int64_t)(v & 0xff) + (int64_t)(h->pushes_total - h->pushes_at_merge[seq % 64]));
                if (h->pushes_ub < FW_MAX_PENDING || !valid || seq + 1 >= h->merge_seq) break;
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;  // read_ctrl below
                std::this_thread::yield();
            }
        }
        if (h->pushes_ub >= FW_MAX_PENDING) {
            Ctrl c;
            int rc = read_ctrl(h, &c);
            if (rc) return rc;
            h->pushes_ub = c.pending_pushes;
            if (h->pushes_ub >= FW_MAX_PENDING) {
                // buffer full: flush into state (RecordsWindowBuffer.addElement EOFException path)
                if ((rc = force_flush(h))) return rc;
            }
        }
        IngestArgs a{};
        a.stride = stride;
        a.key = key + o * stride;
        a.ts = ts + o * stride;
        a.khash = kh ? kh + o : nullptr;
        for (int s = 0; s < MAX_KCOLS; s++) {
            const bool live = s < h->nv;
            a.vals[s] = live ? (const uint64_t*)vals[h->slot_col[s]] + o * stride : nullptr;
            a.nulls[s] = live && ((h->cfg.nullable_cols >> h->slot_col[s]) & 1u) ? nulls[h->slot_col[s]] + o : nullptr;
        }
        a.n = m;
        a.win = device_win(h);
        a.lfire = h->lfire;
        a.lfire_cap = h->lfire_cap;
        a.side = h->side;
        a.side_cap = h->side_cap;
        a.side_output = h->cfg.late_side_output ? 1 : 0;
        a.push_seq = h->push_seq;
        a.row0 = o;
        a.seg_counts = seg_counts;
        a.fold_always = h->fold_always;
        a.no_fold = h->ad.by_prev >= 0;
        a.seg_div = make_udiv((uint64_t)std::max<int64_t>(seg_len, 1));
        a.ks = h->ks;
        a.wd = h->wd;
        a.nv = h->nv;
        a.ctrl = h->ctrl;
        a.tickets = h->tickets;
        a.parts = h->parts;
        a.cap_rows = h->cap_rows;
        a.cells = h->cells;
        a.slot_nch = h->slot_nch;
        a.max_nch = h->cell_cols;
        a.chunk_stats = h->chunk_stats;
        a.n_chunks = (m + h->chunk_rows - 1) / h->chunk_rows;
        a.treq = h->treq;
        a.treq_cap = h->treq_cap;
        a.lds_bytes = ig_lds(ig_block(h->nw_t, ig_nv(h->nv)));
        a.local = h->cfg.agg_phase == FW_PHASE_LOCAL;
        a.global = h->cfg.agg_phase == FW_PHASE_GLOBAL;
        a.ablate = h->ablate;
        a.kt = h->kt_device ? h->kt_dev + FW_KT_REDUCE * KT_WORDS : nullptr;
        a.narrow = h->narrow;
        a.rank_lim = std::min<int64_t>(PF_MAX_RANK + 1, ((1ll << 31) - 1) / std::max<int64_t>(h->win.interval, 1)) *
                     h->win.interval;
        a.slot_base = h->slot_base;
        a.ranks = h->ranks;
        a.runs = h->runs;
        a.run_ranks = h->run_ranks;
        a.run_fill = h->run_fill;
        a.run_ovf = h->run_ovf;
        a.slot_fmt = h->slot_fmt;
        a.run_rows = h->run_rows;
        a.sub_cap = h->sub_cap;
        a.pack = h->pack;
        HIP_TRY(launch_ingest(a, h->stream, h->timer));
        h->pushes_ub++;
        h->pushes_total++;
    }
    h->push_seq++;
    return FW_OK;
}

// interns n key-row images (device) into the table: d_kid / d_khash hold their ids and hashCodes
int kr_intern(fw_handle* h, int64_t n, const int64_t* d_off, const uint8_t* d_bytes) {
    if (n > h->kr_scratch_n) {
        hipFree(h->d_kid);
        hipFree(h->d_khash);
        h->d_kid = nullptr;
        h->d_khash = nullptr;
        h->kr_scratch_n = 0;
        int rc;
        if ((rc = dalloc(&h->d_kid, (size_t)n))) return rc;
        if ((rc = dalloc(&h->d_khash, (size_t)n))) return rc;
        h->kr_scratch_n = n;
    }
    HIP_TRY(launch_kr_intern(h->kr, h->ctrl, n, d_off, d_bytes, h->d_kid, h->d_khash, h->stream));
    return FW_OK;
}

int push_key_rows(fw_handle* h, int64_t n, const int64_t* d_off, const uint8_t* d_bytes, const int64_t* ts,
                  const void* const* vals, const uint8_t* const* nulls) {
    int rc = kr_intern(h, n, d_off, d_bytes);
    if (rc) return rc;
    return push(h, n, h->d_kid, ts, h->d_khash, vals, nulls);
}

// the first n entries of superbucket sb, in the wide layout (key, slice, flags, words) whatever the
// layout the last write-back chose (HOP block state may be narrow, hb_narrow_words)
int state_rows_to_host(const fw_handle* h, size_t sb, int64_t n, uint64_t* out) {
    const int pwe = h->pwe;
    const uint64_t* src = h->state + sb * h->cap_e * pwe;
    uint8_t nar = 0;
    if (h->win.hopb) HIP_TRY(hipMemcpy(&nar, h->sb_nar + sb, 1, hipMemcpyDeviceToHost));
    if (!nar) {
        HIP_TRY(hipMemcpy(out, src, (size_t)n * pwe * 8, hipMemcpyDeviceToHost));
        return FW_OK;
    }
    const int nw = h->nw_t, pwn = hb_narrow_words(nw, nar), sbytes = hb_slot_bytes(nar);
    std::vector<uint64_t> tmp((size_t)n * pwn);
    HIP_TRY(hipMemcpy(tmp.data(), src, tmp.size() * 8, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; i++) {
        const uint8_t* q = (const uint8_t*)(tmp.data() + (size_t)i * pwn);
        uint64_t* e = out + (size_t)i * pwe;
        uint32_t bi;
        uint16_t fl;
        memcpy(&e[0], q, 8);
        memcpy(&bi, q + 8, 4);  // block index: block start = index * hb_span + offset
        memcpy(&fl, q + 12, 2);
        e[1] = (uint64_t)wadd((int64_t)bi * h->win.hb_span, h->win.offset);
        e[2] = fl;
        const uint32_t mask = (uint32_t)fl >> HB_MASK_SHIFT;
        for (int s = 0; s < HB_R; s++)
            for (int x = 0; x < nw; x++) {
                const uint8_t* f = q + HB_HDR_BYTES + sbytes * (s * nw + x);
                int64_t v;
                if (sbytes == 4) {
                    int32_t t;
                    memcpy(&t, f, 4);
                    v = t;
                } else {
                    int16_t t;
                    memcpy(&t, f, 2);
                    v = t;
                }
                e[3 + s * nw + x] = ((mask >> s) & 1u) ? (uint64_t)v : x < h->wd.nw ? word_identity(h->wd.op[x]) : 0;
            }
    }
    return FW_OK;
}

// earliest watermark-visible time of an entry's timers, as a window end (is_fired(x, W) <=> due):
// the maxTimestamp timer at its window end, a DataStream cleanup timer at cleanupTime + 1
int64_t entry_timer_end(const fw_handle* h, int64_t slice, uint64_t flags) {
    if (h->win.hopb) {  // block entry: no window of it is due before its oldest slice with data
        const uint32_t mask = (uint32_t)flags >> 8;
        for (int i = 0; i < HB_R; i++)
            if ((mask >> i) & 1u) return wadd(slice, (int64_t)(i + 1) * h->win.interval);
        return INT64_MAX;
    }
    int64_t m = (flags & F_TIMER) ? slice : INT64_MAX;
    if (h->win.ds && (flags & F_CLEAN)) m = std::min(m, wadd(ds_cleanup_time(h->win, slice), 1));
    return m;
}

}  // namespace

// ======================================================================================
extern "C" {

const char* fw_last_error(void) { return g_err.c_str(); }
int fw_abi_version(void) { return FW_ABI_VERSION; }

int fw_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int fw_create(const fw_config* cfg, fw_handle** out) {
    if (!cfg || !out) return fail(FW_E_INVALID, "null argument");
    *out = nullptr;
    fw_handle* h = new fw_handle();
    h->cfg = *cfg;
    if (const char* ab = getenv("FW_ABLATE")) h->ablate = atoi(ab);
    if (const char* fo = getenv("FW_FOLD")) h->fold_always = atoi(fo);
    if (const char* ak = getenv("FW_AR_KERNEL")) h->ar_kernel = atoi(ak);
    if (const char* fp = getenv("FW_FILL_PCT")) h->fill_pct = std::min(95, std::max(10, atoi(fp)));
    if (const char* si = getenv("FW_SKIP_IDLE")) h->skip_idle = atoi(si) != 0;
    int rc = validate_and_plan(h);
    h->cfg.tz_utc = nullptr;  // the shift-zone table was copied (h->tz_*); never read the caller's
    h->cfg.tz_offset_ms = nullptr;
    if (!rc) rc = allocate(h);
    if (rc) {
        std::string keep = g_err;
        fw_destroy(h);
        g_err = keep;
        return rc;
    }
    *out = h;
    return FW_OK;
}

int fw_destroy(fw_handle* h) {
    if (!h) return FW_OK;
    if (h->stream) hipStreamSynchronize(h->stream);
    hipFree(h->ctrl);
    hipFree(h->parts);
    hipFree(h->runs);
    hipFree(h->run_ranks);
    hipFree(h->run_fill);
    hipFree(h->run_ovf);
    hipFree(h->slot_fmt);
    hipFree(h->cells);
    hipFree(h->slot_nch);
    hipFree(h->slot_base);
    hipFree(h->ranks);
    hipFree(h->treq);
    if (h->mirror) hipHostFree((void*)h->mirror);
    hipFree(h->lfire);
    hipFree(h->side);
    hipFree(h->ordev);
    hipFree(h->kr.slots);
    hipFree(h->kr.arena);
    hipFree(h->kr.mark);
    hipFree(h->kr.free_list);
    hipFree(h->d_kid);
    hipFree(h->d_khash);
    hipFree(h->res_kr_len);
    hipFree(h->res_kr_img);
    for (int b = 0; b < FW_STAGE_BUFS; b++) {
        hipHostFree(h->h_kro[b]);
        hipHostFree(h->h_krb[b]);
    }
    hipFree(h->d_tz);
    hipFree(h->state);
    hipFree(h->state_count);
    hipFree(h->sb_min_timer);
    hipFree(h->sb_nar);
    hipFree(h->out_key);
    hipFree(h->out_we);
    hipFree(h->out_null);
    for (int g = 0; g < FW_MAX_AGGS; g++) hipFree(h->out_val[g]);
    for (int g = 0; g < FW_MAX_AGGS; g++) hipFree(h->res_val[g]);
    hipFree(h->res_key);
    hipFree(h->res_ws);
    hipFree(h->res_we);
    hipFree(h->res_null);
    hipFree(h->sb_out);
    hipFree(h->sb_fired);
    hipFree(h->coff);
    hipFree(h->chunk_stats);
    hipFree(h->tickets);
    hipFree(h->stamps);
    hipFree(h->kt_dev);
    for (int b = 0; b < FW_STAGE_BUFS; b++) {
        hipHostFree(h->h_key[b]);
        hipHostFree(h->h_ts[b]);
        hipHostFree(h->h_kh[b]);
        for (int v = 0; v < FW_MAX_COLS; v++) {
            hipHostFree(h->h_val[b][v]);
            hipHostFree(h->h_nul[b][v]);
        }
        if (h->stage_ev[b]) hipEventDestroy(h->stage_ev[b]);
        if (h->dstage_free[b]) hipEventDestroy(h->dstage_free[b]);
        hipFree(h->d_kro[b]);
        hipFree(h->d_krb[b]);
        hipFree(h->d_key[b]);
        hipFree(h->d_ts[b]);
        hipFree(h->d_pack[b]);
        hipFree(h->d_kh[b]);
        for (int v = 0; v < FW_MAX_COLS; v++) {
            hipFree(h->d_val[b][v]);
            hipFree(h->d_nul[b][v]);
        }
    }
    if (h->d2h_stream) hipStreamSynchronize(h->d2h_stream);  // an early DMA (ar_kick) may still be reading the buffers
    for (int b = 0; b < FW_AR_BUFS; b++) {
        hipHostFree(h->ar_key[b]);
        hipHostFree(h->ar_ws[b]);
        hipHostFree(h->ar_we[b]);
        hipHostFree(h->ar_null[b]);
        for (int g = 0; g < FW_MAX_AGGS; g++) hipHostFree(h->ar_val[b][g]);
        hipHostFree(h->ar_n[b]);
        if (h->ar_ev[b]) hipEventDestroy(h->ar_ev[b]);
        if (h->ar_dma_ev[b]) hipEventDestroy(h->ar_dma_ev[b]);
        hipFree(h->ard_key[b]);
        hipFree(h->ard_ws[b]);
        hipFree(h->ard_we[b]);
        hipFree(h->ard_null[b]);
        for (int g = 0; g < FW_MAX_AGGS; g++) hipFree(h->ard_val[b][g]);
    }
    if (h->d2h_stream) hipStreamDestroy(h->d2h_stream);
    if (h->cstream) hipStreamDestroy(h->cstream);
    delete h->timer;
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
    return FW_OK;
}

void* fw_get_stream(fw_handle* h) { return h ? (void*)h->stream : nullptr; }

int fw_sync(fw_handle* h) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    Ctrl c;
    return read_ctrl(h, &c);
}

int fw_initialize_watermark(fw_handle* h, int64_t watermark) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    HIP_TRY(hipMemcpyAsync(&h->ctrl->cur, &watermark, sizeof(int64_t), hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->host_cur = watermark;
    h->dev_cur = watermark;
    return FW_OK;
}

int fw_reserve(fw_handle* h, int64_t n, fw_host_cols* out) {
    if (!h || !out) return fail(FW_E_INVALID, "null argument");
    if (n < 0 || n > h->stage_cap) return fail(FW_E_INVALID, "reserve %lld rows > max_batch_rows %lld", (long long)n, (long long)h->stage_cap);
    int rc = alloc_staging(h);
    if (rc) return rc;
    const int b = h->stage_cur;
    HIP_TRY(hipEventSynchronize(h->stage_ev[b]));  // previous H2D from this buffer has finished
    memset(out, 0, sizeof *out);
    out->key = h->h_key[b];
    out->ts = h->h_ts[b];
    out->key_hash = h->h_kh[b];
    for (int v = 0; v < h->cfg.n_value_cols; v++) {
        out->values[v] = h->h_val[b][v];
        out->nulls[v] = h->h_nul[b][v];
    }
    if (h->keyrow) {
        out->key_row_offsets = h->h_kro[b];
        out->key_row_bytes = h->h_krb[b];
        out->key_row_bytes_cap = h->krb_cap;
        h->h_kro[b][0] = 0;
    }
    h->reserved = n;
    return FW_OK;
}

static int commit_impl(fw_handle* h, int64_t n, uint32_t packed, const int64_t* bases);

int fw_commit(fw_handle* h, int64_t n) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    return commit_impl(h, n, 0u, nullptr);
}

// the loop vectorises; the wider x86 units where the host has them (chosen at load time)
__attribute__((target_clones("avx512f", "avx2", "default")))
int fw_delta32_encode(const int64_t* src, int64_t n, int64_t base, uint32_t* dst) {
    if (n <= 0) return 0;
    uint64_t out = 0;  // any high bits: a value outside the column's 2^32 window
    for (int64_t i = 0; i < n; i++) {
        const uint64_t d = (uint64_t)src[i] - (uint64_t)base;
        out |= d >> 32;
        dst[i] = (uint32_t)d;
    }
    return out ? 1 : 0;
}

int fw_commit_delta32(fw_handle* h, int64_t n, uint32_t delta_cols, const int64_t* bases) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    const uint32_t valid = FW_DELTA_KEY | FW_DELTA_TS | (((1u << h->cfg.n_value_cols) - 1u) << 2);
    if (delta_cols & ~valid) return fail(FW_E_INVALID, "delta_cols 0x%x names a column the operator does not have", delta_cols);
    if ((delta_cols & FW_DELTA_KEY) && h->keyrow) return fail(FW_E_INVALID, "key-row operators have no key column to pack");
    if (delta_cols && !bases) return fail(FW_E_INVALID, "packed columns need their bases");
    return commit_impl(h, n, delta_cols, bases);
}

static int commit_impl(fw_handle* h, int64_t n, uint32_t packed, const int64_t* bases) {
    ar_kick(h);
    if (h->reserved < 0 || n > h->reserved || n < 0) return fail(FW_E_STATE, "commit without matching reserve");
    h->reserved = -1;
    const int b = h->stage_cur;
    h->stage_cur = (b + 1) % FW_STAGE_BUFS;
    if (n == 0) return FW_OK;
    int64_t krb_n = 0;
    if (h->keyrow) {
        krb_n = h->h_kro[b][n];
        if (h->h_kro[b][0] != 0 || krb_n < 0 || krb_n > h->krb_cap)
            return fail(FW_E_INVALID, "key row offsets must start at 0 and end within key_row_bytes_cap");
    }
    // H2D on the copy stream into device buffer b, once the ingest that last read it has run; the
    // operator stream waits for the copies.  The previous batch's ingest and merge overlap them.
    hipStream_t cs = h->cstream;
    HIP_TRY(hipStreamWaitEvent(cs, h->dstage_free[b], 0));
    // (a second copy stream for the upper half of every column was measured slower: CFG2 end to end
    // 1.76 -> 1.26 G ev/s, its enqueue blocking the host 0.9 ms per batch)
    auto h2d = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, cs);
    };
    if (packed && !h->d_pack[b]) {  // first packed commit into this set (allocation outside any timed loop of the caller's)
        h->pack_stride = (h->stage_cap + 3) & ~3ll;
        HIP_TRY(hipMalloc((void**)&h->d_pack[b], (size_t)FW_PACK_COLS * h->pack_stride * 4));
    }
    // an 8-byte word column: a packed one crosses PCIe as n 32-bit deltas (the first 4n bytes of its
    // staging column) and is widened on the copy stream, behind its copy
    WidenArgs wa{};
    wa.n = n;
    int nw = 0;
    auto col = [&](int slot, void* dst, const void* src) -> hipError_t {
        if (!((packed >> slot) & 1u)) return h2d(dst, src, (size_t)n * 8);
        uint32_t* p = h->d_pack[b] + (size_t)slot * h->pack_stride;
        wa.src[nw] = p;
        wa.dst[nw] = (uint64_t*)dst;
        wa.base[nw] = (uint64_t)bases[slot];
        nw++;
        return h2d(p, src, (size_t)n * 4);
    };
    if (h->keyrow) {
        HIP_TRY(h2d(h->d_kro[b], h->h_kro[b], (n + 1) * 8));
        HIP_TRY(h2d(h->d_krb[b], h->h_krb[b], (size_t)krb_n));
    } else {
        HIP_TRY(col(0, h->d_key[b], h->h_key[b]));
    }
    HIP_TRY(col(1, h->d_ts[b], h->h_ts[b]));
    if (h->cfg.key_hash == FW_KEYHASH_PRECOMPUTED) HIP_TRY(h2d(h->d_kh[b], h->h_kh[b], n * 4));
    for (int s = 0; s < h->nv; s++) {
        const int v = h->slot_col[s];
        HIP_TRY(col(2 + v, h->d_val[b][v], h->h_val[b][v]));
        if (h->d_nul[b][v]) HIP_TRY(h2d(h->d_nul[b][v], h->h_nul[b][v], n));
    }
    HIP_TRY(launch_widen(wa, nw, cs));
    HIP_TRY(hipEventRecord(h->stage_ev[b], cs));
    HIP_TRY(hipStreamWaitEvent(h->stream, h->stage_ev[b], 0));
    const void* vals[FW_MAX_COLS];
    const uint8_t* nuls[FW_MAX_COLS];
    for (int v = 0; v < FW_MAX_COLS; v++) {
        vals[v] = h->d_val[b][v];
        nuls[v] = h->d_nul[b][v];
    }
    const int rc = h->keyrow ? push_key_rows(h, n, h->d_kro[b], h->d_krb[b], h->d_ts[b], vals, nuls)
                             : push(h, n, h->d_key[b], h->d_ts[b],
                                    h->cfg.key_hash == FW_KEYHASH_PRECOMPUTED ? h->d_kh[b] : nullptr, vals, nuls);
    HIP_TRY(hipEventRecord(h->dstage_free[b], h->stream));
    return rc;
}

int fw_push_device_key_rows(fw_handle* h, int64_t n, const int64_t* d_key_row_offsets, const uint8_t* d_key_row_bytes,
                            const int64_t* d_ts, const void* const* d_values, const uint8_t* const* d_nulls) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    if (!h->keyrow) return fail(FW_E_INVALID, "fw_push_device_key_rows needs a FW_KEYHASH_KEYROW operator");
    if (n < 0) return fail(FW_E_INVALID, "negative n");
    if (n == 0) return FW_OK;
    if (!d_key_row_offsets || !d_key_row_bytes || !d_ts) return fail(FW_E_INVALID, "null key row / ts column");
    if (h->nv > 0 && !d_values) return fail(FW_E_INVALID, "value columns required");
    for (int s = 0; s < h->nv; s++) {
        const int v = h->slot_col[s];
        if (!d_values[v]) return fail(FW_E_INVALID, "value column %d is NULL", v);
        if (((h->cfg.nullable_cols >> v) & 1u) && (!d_nulls || !d_nulls[v]))
            return fail(FW_E_INVALID, "nullable value column %d needs its null-flag column", v);
    }
    return push_key_rows(h, n, d_key_row_offsets, d_key_row_bytes, d_ts, d_values, d_nulls);
}

int fw_push_device(fw_handle* h, int64_t n, const int64_t* d_key, const int64_t* d_ts, const int32_t* d_key_hash,
                   const void* const* d_values, const uint8_t* const* d_nulls) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    if (n < 0) return fail(FW_E_INVALID, "negative n");
    ar_kick(h);
    if (n == 0) return FW_OK;
    if (!d_key || !d_ts) return fail(FW_E_INVALID, "null key/ts column");
    if (h->keyrow) return fail(FW_E_INVALID, "a FW_KEYHASH_KEYROW operator takes key rows (fw_push_device_key_rows)");
    if (h->cfg.key_hash == FW_KEYHASH_PRECOMPUTED && !d_key_hash) return fail(FW_E_INVALID, "key_hash column required");
    if (h->nv > 0 && !d_values) return fail(FW_E_INVALID, "value columns required");
    for (int s = 0; s < h->nv; s++) {
        const int v = h->slot_col[s];
        if (!d_values[v]) return fail(FW_E_INVALID, "value column %d is NULL", v);
        if (((h->cfg.nullable_cols >> v) & 1u) && (!d_nulls || !d_nulls[v]))
            return fail(FW_E_INVALID, "nullable value column %d needs its null-flag column", v);
    }
    return push(h, n, d_key, d_ts, d_key_hash, d_values, d_nulls);
}

int fw_push_device_segments(fw_handle* h, int32_t n_segs, int64_t seg_len, const int64_t* d_seg_counts,
                            const int64_t* d_key, const int64_t* d_ts, const int32_t* d_key_hash,
                            const void* const* d_values, const uint8_t* const* d_nulls) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    if (n_segs < 0 || seg_len < 1 || (n_segs > 0 && !d_seg_counts)) return fail(FW_E_INVALID, "bad segments");
    if (h->keyrow) return fail(FW_E_INVALID, "a FW_KEYHASH_KEYROW operator takes key rows (fw_push_device_key_rows)");
    const int64_t n = (int64_t)n_segs * seg_len;
    if (n == 0) return FW_OK;
    if (!d_key || !d_ts) return fail(FW_E_INVALID, "null key/ts column");
    if (h->cfg.key_hash == FW_KEYHASH_PRECOMPUTED && !d_key_hash) return fail(FW_E_INVALID, "key_hash column required");
    if (h->nv > 0 && !d_values) return fail(FW_E_INVALID, "value columns required");
    for (int s = 0; s < h->nv; s++) {
        const int v = h->slot_col[s];
        if (!d_values[v]) return fail(FW_E_INVALID, "value column %d is NULL", v);
        if (((h->cfg.nullable_cols >> v) & 1u) && (!d_nulls || !d_nulls[v]))
            return fail(FW_E_INVALID, "nullable value column %d needs its null-flag column", v);
    }
    return push(h, n, d_key, d_ts, d_key_hash, d_values, d_nulls, d_seg_counts, seg_len);
}

int fw_push_device_packed_segments(fw_handle* h, int32_t n_segs, int64_t seg_len, const int64_t* d_seg_counts,
                                   const int64_t* d_rows, int32_t row_words) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    if (n_segs < 0 || seg_len < 1 || (n_segs > 0 && !d_seg_counts)) return fail(FW_E_INVALID, "bad segments");
    if (row_words != 2 + h->cfg.n_value_cols) return fail(FW_E_INVALID, "row_words %d != 2 + value columns", row_words);
    if (h->cfg.key_hash == FW_KEYHASH_PRECOMPUTED || h->keyrow || h->cfg.nullable_cols)
        return fail(FW_E_INVALID, "packed rows carry no key-hash, key-row or null-flag columns");
    const int64_t n = (int64_t)n_segs * seg_len;
    if (n == 0) return FW_OK;
    if (!d_rows) return fail(FW_E_INVALID, "null rows");
    const void* vals[FW_MAX_COLS] = {nullptr};
    for (int c = 0; c < h->cfg.n_value_cols; c++) vals[c] = d_rows + 2 + c;
    return push(h, n, d_rows, d_rows + 1, nullptr, vals, nullptr, d_seg_counts, seg_len, row_words);
}

int fw_advance(fw_handle* h, int64_t watermark) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    ar_kick(h);
    // A SQL watermark below the next trigger watermark crosses no slice end: no window fires, no
    // buffer flush is due (AbstractSliceSyncStateWindowAggProcessor.advanceProgress :139-153 only
    // flushes at a trigger) and lateness is unchanged (no window end lies between the old and the
    // new watermark), so the merge launch would only move currentProgress.  It is skipped; the next
    // launch moves currentProgress past it and registers any pending late-record timers before it
    // fires.  DataStream cleanup timers are off the slice grid (cleanupTime), so DataStream and
    // key-row operators (whose collector runs with the merge) always launch.
    // The trigger grid is the slice-end grid only in UTC with an offset on the grid: otherwise a
    // timer or a lateness bound can lie between two trigger watermarks, and only a repeated
    // watermark is skipped.
    const bool on_grid = h->win.tz.n == 0 && h->win.offset % h->win.interval == 0;
    if (h->skip_idle && !h->always_flush && !h->keyrow &&
        (watermark <= h->dev_cur || (on_grid && watermark < h->dev_ntp))) {
        if (watermark > h->host_cur) h->host_cur = watermark;
        return FW_OK;
    }
    int rc = launch_merge(h, watermark, 0);
    if (rc) return rc;
    if (h->keyrow)  // key rows no state / partial / timer request / unread result holds any more
        HIP_TRY(launch_kr_collect(h->kr, h->ctrl, h->state, h->state_count, h->sb_nar, h->nw_t, h->ks.n_sb, h->cap_e, h->pwe,
                                  2 + h->nw_t, h->parts, h->cap_rows, h->treq, h->out_key, h->sb_out, h->slab_cap,
                                  h->stream));
    if (watermark > h->host_cur) h->host_cur = watermark;
    return FW_OK;
}

int fw_advance_device(fw_handle* h, const int64_t* d_watermark) {
    if (!h || !d_watermark) return fail(FW_E_INVALID, "null argument");
    MergeArgs a = merge_args(h, INT64_MIN, 0);
    a.wm_dev = d_watermark;
    HIP_TRY(launch_merge_fire(a, h->stream, h->timer));
    // launch_merge's bookkeeping; the host mirrors of currentProgress stay behind the device (they
    // only ever skip launches, so a stale, lower value skips fewer)
    h->pushes_at_merge[h->merge_seq % 64] = h->pushes_total;
    h->merge_seq++;
    h->reset_pending = false;
    if (h->keyrow)
        HIP_TRY(launch_kr_collect(h->kr, h->ctrl, h->state, h->state_count, h->sb_nar, h->nw_t, h->ks.n_sb, h->cap_e, h->pwe,
                                  2 + h->nw_t, h->parts, h->cap_rows, h->treq, h->out_key, h->sb_out, h->slab_cap,
                                  h->stream));
    return FW_OK;
}

int fw_flush(fw_handle* h) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    return force_flush(h);
}

int fw_results(fw_handle* h, fw_result* out, int copy_to_host) {
    if (!h || !out) return fail(FW_E_INVALID, "null argument");
    if (h->reset_pending) {  // consumed and nothing emitted since
        Ctrl c;
        int rc = read_ctrl(h, &c);
        if (rc) return rc;
        memset(out, 0, sizeof *out);
        return FW_OK;
    }
    CompactArgs ca{};
    ca.ctrl = h->ctrl;
    ca.sb_out = h->sb_out;
    ca.off = h->coff;
    ca.n_sb = h->ks.n_sb;
    ca.n_aggs = h->n_out;
    ca.slab_cap = h->slab_cap;
    ca.out_key = h->out_key;
    ca.win = device_win(h);
    ca.local_out = h->cfg.agg_phase == FW_PHASE_LOCAL;
    ca.out_we = h->out_we;
    ca.out_null = h->out_null;
    for (int g = 0; g < h->n_out; g++) {
        ca.out_val[g] = h->out_val[g];
        ca.res_val[g] = h->res_val[g];
    }
    ca.res_key = h->res_key;
    ca.res_ws = h->res_ws;
    ca.res_we = h->res_we;
    ca.res_null = h->res_null;
    ca.res_cap = h->out_cap;
    HIP_TRY(launch_compact(ca, h->stream, h->timer));
    const int32_t krw = h->kr.stride_words - 1;  // image words per result row
    if (h->keyrow)  // each result row's key row, gathered from the table while its id is held
        HIP_TRY(launch_kr_result_rows(h->kr, h->res_key, h->coff + h->ks.n_sb + 1, h->out_cap, h->res_kr_len,
                                      h->res_kr_img, krw, h->stream));
    Ctrl c;
    int rc = read_ctrl(h, &c);
    if (rc) return rc;
    int64_t total = 0;
    HIP_TRY(hipMemcpy(&total, h->coff + h->ks.n_sb + 1, sizeof total, hipMemcpyDeviceToHost));
    if (total > h->out_cap)
        return fail(FW_E_CAPACITY, "%lld result rows exceed output_capacity %lld (read results more often)",
                    (long long)total, (long long)h->out_cap);
    const int64_t n = total;
    memset(out, 0, sizeof *out);
    out->n = n;
    const int na = h->n_out;
    const int nv = h->ad.first_word >= 0 ? na - 1 : na;  // the last column is value1's ordinal
    if (!copy_to_host) {
        out->key = h->res_key;
        out->window_start = h->res_ws;
        out->window_end = h->res_we;
        for (int g = 0; g < nv; g++) out->values[g] = (int64_t*)h->res_val[g];
        if (nv < na) out->first_ord = (int64_t*)h->res_val[nv];
        out->null_mask = h->res_null;
        if (h->keyrow) {
            out->key_row_len = h->res_kr_len;
            out->key_row_bytes = (uint8_t*)h->res_kr_img;
            out->key_row_stride = 8ll * krw;
        }
        return FW_OK;
    }
    h->r_key.resize(n);
    h->r_ws.resize(n);
    h->r_we.resize(n);
    h->r_null.resize(n);
    if (n) {
        HIP_TRY(hipMemcpyAsync(h->r_key.data(), h->res_key, n * 8, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipMemcpyAsync(h->r_ws.data(), h->res_ws, n * 8, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipMemcpyAsync(h->r_we.data(), h->res_we, n * 8, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipMemcpyAsync(h->r_null.data(), h->res_null, n * 4, hipMemcpyDeviceToHost, h->stream));
    }
    for (int g = 0; g < na; g++) {
        h->r_val[g].resize(n);
        if (n) HIP_TRY(hipMemcpyAsync(h->r_val[g].data(), h->res_val[g], n * 8, hipMemcpyDeviceToHost, h->stream));
    }
    if (h->keyrow) {
        h->r_kr_len.resize(n);
        h->r_kr_img.resize((size_t)n * krw);
        if (n) {
            HIP_TRY(hipMemcpyAsync(h->r_kr_len.data(), h->res_kr_len, n * 4, hipMemcpyDeviceToHost, h->stream));
            HIP_TRY(hipMemcpyAsync(h->r_kr_img.data(), h->res_kr_img, (size_t)n * krw * 8, hipMemcpyDeviceToHost, h->stream));
        }
    }
    HIP_TRY(hipStreamSynchronize(h->stream));
    out->key = h->r_key.data();
    out->window_start = h->r_ws.data();
    out->window_end = h->r_we.data();
    for (int g = 0; g < nv; g++) out->values[g] = (int64_t*)h->r_val[g].data();
    if (nv < na) out->first_ord = (int64_t*)h->r_val[nv].data();
    out->null_mask = h->r_null.data();
    if (h->keyrow) {
        out->key_row_len = h->r_kr_len.data();
        out->key_row_bytes = (uint8_t*)h->r_kr_img.data();
        out->key_row_stride = 8ll * krw;
    }
    return FW_OK;
}

int fw_results_async(fw_handle* h) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    if (h->keyrow) return fail(FW_E_INVALID, "key-row operators return their rows through fw_results");
    int rc = alloc_async_results(h);
    if (rc) return rc;
    if (h->ar_qn == FW_AR_BUFS)
        return fail(FW_E_STATE, "%d result collections outstanding: fw_results_ready first", FW_AR_BUFS);
    const int b = h->ar_cur;
    h->ar_cur = (b + 1) % FW_AR_BUFS;
    h->ar_q[(h->ar_qhead + h->ar_qn) % FW_AR_BUFS] = b;
    h->ar_qn++;
    h->ar_empty[b] = h->reset_pending;  // consumed and nothing emitted since
    h->ar_copied[b] = false;
    if (h->ar_inflight[b]) {  // an early DMA of this buffer's previous rows: the compaction waits for it
        HIP_TRY(hipStreamWaitEvent(h->stream, h->ar_dma_ev[b], 0));
        h->ar_inflight[b] = false;
    }
    if (h->ar_empty[b]) return FW_OK;
    CompactArgs ca{};
    ca.ctrl = h->ctrl;
    ca.sb_out = h->sb_out;
    ca.off = h->coff;
    ca.n_sb = h->ks.n_sb;
    ca.n_aggs = h->n_out;
    ca.slab_cap = h->slab_cap;
    ca.out_key = h->out_key;
    ca.win = device_win(h);
    ca.local_out = h->cfg.agg_phase == FW_PHASE_LOCAL;
    ca.out_we = h->out_we;
    ca.out_null = h->out_null;
    for (int g = 0; g < h->n_out; g++) {
        ca.out_val[g] = h->out_val[g];
        ca.res_val[g] = h->ard_val[b][g];
    }
    ca.res_key = h->ard_key[b];
    ca.res_ws = h->ard_ws[b];
    ca.res_we = h->ard_we[b];
    ca.res_null = h->ard_null[b];
    ca.res_cap = h->out_cap;
    ca.host_n = mapped(h->ar_n[b]);
    if (!ca.host_n) return fail(FW_E_DEVICE, "mapped result count unavailable");
    HIP_TRY(launch_compact(ca, h->stream, h->timer));
    if (h->ar_kernel) {
        CopyOutArgs co{};
        co.d_n = h->coff + h->ks.n_sb + 1;
        co.n_aggs = h->n_out;
        co.cap = h->out_cap;
        co.src_key = h->ard_key[b];
        co.src_ws = h->ard_ws[b];
        co.src_we = h->ard_we[b];
        co.src_null = h->ard_null[b];
        co.dst_key = mapped(h->ar_key[b]);
        co.dst_ws = mapped(h->ar_ws[b]);
        co.dst_we = mapped(h->ar_we[b]);
        co.dst_null = mapped(h->ar_null[b]);
        for (int g = 0; g < h->n_out; g++) {
            co.src_val[g] = h->ard_val[b][g];
            co.dst_val[g] = mapped(h->ar_val[b][g]);
            if (!co.dst_val[g]) return fail(FW_E_DEVICE, "mapped result buffer unavailable");
        }
        if (!co.dst_key || !co.dst_ws || !co.dst_we || !co.dst_null) return fail(FW_E_DEVICE, "mapped result buffer unavailable");
        HIP_TRY(launch_copy_out(co, h->stream));
        h->ar_copied[b] = true;  // the rows are in host memory once ar_ev[b] has fired
    }
    HIP_TRY(hipEventRecord(h->ar_ev[b], h->stream));
    h->reset_pending = true;  // the rows are collected: the next merge launch starts the slabs afresh
    return FW_OK;
}

int fw_results_device_segments(fw_handle* h, fw_result_segments* out) {
    if (!h || !out) return fail(FW_E_INVALID, "null argument");
    if (h->keyrow) return fail(FW_E_INVALID, "key-row operators return their rows through fw_results");
    memset(out, 0, sizeof *out);
    const int na = h->n_out;
    const int nv = h->ad.first_word >= 0 ? na - 1 : na;
    out->seg_cap = h->slab_cap;
    out->counts = h->sb_out;
    out->cols.n = (int64_t)h->ks.n_sb * h->slab_cap + h->out_cap;
    out->cols.key = h->out_key;
    out->cols.window_start = nullptr;  // v10: derived from window_end (flinkwin.h)
    out->cols.window_end = h->out_we;
    for (int g = 0; g < nv; g++) out->cols.values[g] = (int64_t*)h->out_val[g];
    if (nv < na) out->cols.first_ord = (int64_t*)h->out_val[nv];
    out->cols.null_mask = h->out_null;
    // consumed and nothing emitted since: no segments (the counts are those of consumed rows)
    out->n_segments = h->reset_pending ? 0 : (int64_t)h->ks.n_sb + 1;
    h->reset_pending = true;  // consumed: the next merge launch starts the slabs afresh
    return FW_OK;
}

int fw_results_device(fw_handle* h, fw_result* out, int64_t** d_n) {
    if (!h || !out || !d_n) return fail(FW_E_INVALID, "null argument");
    if (h->keyrow) return fail(FW_E_INVALID, "key-row operators return their rows through fw_results");
    memset(out, 0, sizeof *out);
    *d_n = h->coff + h->ks.n_sb + 1;
    if (h->reset_pending) {  // consumed and nothing emitted since: zero rows
        HIP_TRY(hipMemsetAsync(*d_n, 0, sizeof(int64_t), h->stream));
    } else {
        CompactArgs ca{};
        ca.ctrl = h->ctrl;
        ca.sb_out = h->sb_out;
        ca.off = h->coff;
        ca.n_sb = h->ks.n_sb;
        ca.n_aggs = h->n_out;
        ca.slab_cap = h->slab_cap;
        ca.out_key = h->out_key;
        ca.win = device_win(h);
    ca.local_out = h->cfg.agg_phase == FW_PHASE_LOCAL;
        ca.out_we = h->out_we;
        ca.out_null = h->out_null;
        for (int g = 0; g < h->n_out; g++) {
            ca.out_val[g] = h->out_val[g];
            ca.res_val[g] = h->res_val[g];
        }
        ca.res_key = h->res_key;
        ca.res_ws = h->res_ws;
        ca.res_we = h->res_we;
        ca.res_null = h->res_null;
        ca.res_cap = h->out_cap;
        HIP_TRY(launch_compact(ca, h->stream, h->timer));
        h->reset_pending = true;
    }
    const int na = h->n_out;
    const int nv = h->ad.first_word >= 0 ? na - 1 : na;
    out->n = h->out_cap;
    out->key = h->res_key;
    out->window_start = h->res_ws;
    out->window_end = h->res_we;
    for (int g = 0; g < nv; g++) out->values[g] = (int64_t*)h->res_val[g];
    if (nv < na) out->first_ord = (int64_t*)h->res_val[nv];
    out->null_mask = h->res_null;
    return FW_OK;
}

int fw_results_ready(fw_handle* h, fw_result* out) {
    if (!h || !out) return fail(FW_E_INVALID, "null argument");
    memset(out, 0, sizeof *out);
    if (h->ar_qn == 0) return fail(FW_E_STATE, "fw_results_ready without an outstanding fw_results_async");
    const int b = h->ar_q[h->ar_qhead];  // the oldest outstanding collection
    h->ar_qhead = (h->ar_qhead + 1) % FW_AR_BUFS;
    h->ar_qn--;
    if (h->ar_empty[b]) return FW_OK;
    HIP_TRY(hipEventSynchronize(h->ar_ev[b]));  // the compaction (long done: it ran a step ago)
    const int64_t n = __atomic_load_n(h->ar_n[b], __ATOMIC_ACQUIRE);
    if (n > h->out_cap)
        return fail(FW_E_CAPACITY, "%lld result rows exceed output_capacity %lld (read results more often)",
                    (long long)n, (long long)h->out_cap);
    const int na = h->n_out;
    const int nv = h->ad.first_word >= 0 ? na - 1 : na;
    if (n > 0 && !h->ar_copied[b]) {  // the rows by DMA on the D2H stream (no CU time, no operator-stream slot)
        if (!h->ar_inflight[b]) {  // not started early by ar_kick
            int rc = ar_enqueue_copy(h, b, n);
            if (rc) return rc;
            h->ar_inflight[b] = true;
        }
        HIP_TRY(hipEventSynchronize(h->ar_dma_ev[b]));
        h->ar_copied[b] = true;
    }
    out->n = n;
    out->key = h->ar_key[b];
    out->window_start = h->ar_ws[b];
    out->window_end = h->ar_we[b];
    for (int g = 0; g < nv; g++) out->values[g] = (int64_t*)h->ar_val[b][g];
    if (nv < na) out->first_ord = (int64_t*)h->ar_val[b][nv];
    out->null_mask = h->ar_null[b];
    return FW_OK;
}

int fw_first_element_events(fw_handle* h, fw_ordinal_events* out) {
    if (!h || !out) return fail(FW_E_INVALID, "null argument");
    memset(out, 0, sizeof *out);
    if (!h->ordev_cap) return fail(FW_E_STATE, "the operator does not track first elements (ds_first_ordinals = 0)");
    Ctrl c;
    int rc = read_ctrl(h, &c);
    if (rc) return rc;
    const int64_t n = std::min<int64_t>(c.n_ordev, h->ordev_cap);
    std::vector<int64_t> raw((size_t)n);
    if (n) HIP_TRY(hipMemcpy(raw.data(), h->ordev, (size_t)n * 8, hipMemcpyDeviceToHost));
    const int64_t zero = 0;
    HIP_TRY(hipMemcpy(&h->ctrl->n_ordev, &zero, 8, hipMemcpyHostToDevice));
    h->ev_retain.clear();
    h->ev_release.clear();
    for (int64_t e : raw) {
        if (e & ORDEV_RELEASE) h->ev_release.push_back(e & ~ORDEV_RELEASE);
        else h->ev_retain.push_back(e);
    }
    out->n_retain = (int64_t)h->ev_retain.size();
    out->retain = h->ev_retain.data();
    out->n_release = (int64_t)h->ev_release.size();
    out->release = h->ev_release.data();
    return FW_OK;
}

int fw_late_records(fw_handle* h, fw_late_rows* out) {
    if (!h || !out) return fail(FW_E_INVALID, "null argument");
    memset(out, 0, sizeof *out);
    if (!h->side_cap) return fail(FW_E_STATE, "the operator has no late side output (late_side_output = 0)");
    Ctrl c;
    int rc = read_ctrl(h, &c);
    if (rc) return rc;
    const int64_t n = std::min<int64_t>(c.n_side, h->side_cap);
    std::vector<int64_t> raw((size_t)n * SOW);
    if (n) HIP_TRY(hipMemcpy(raw.data(), h->side, raw.size() * 8, hipMemcpyDeviceToHost));
    const int64_t zero = 0;
    HIP_TRY(hipMemcpy(&h->ctrl->n_side, &zero, 8, hipMemcpyHostToDevice));
    h->lr_key.resize(n);
    h->lr_ts.resize(n);
    h->lr_seq.resize(n);
    h->lr_row.resize(n);
    for (int v = 0; v < h->cfg.n_value_cols; v++) h->lr_val[v].assign(n, 0);
    for (int64_t i = 0; i < n; i++) {
        const int64_t* p = raw.data() + (size_t)i * SOW;
        h->lr_key[i] = p[0];
        h->lr_ts[i] = p[1];
        h->lr_seq[i] = (int64_t)((uint64_t)p[2] >> 32);
        h->lr_row[i] = p[2] & 0xffffffffll;
        for (int s = 0; s < h->nv; s++) h->lr_val[h->slot_col[s]][i] = p[3 + s];  // loaded value slots
    }
    out->n = n;
    out->key = h->lr_key.data();
    out->ts = h->lr_ts.data();
    out->push_seq = h->lr_seq.data();
    out->row = h->lr_row.data();
    for (int v = 0; v < h->cfg.n_value_cols; v++) out->values[v] = h->lr_val[v].data();
    return FW_OK;
}

int fw_results_reset(fw_handle* h) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    // no launch: the next merge launch starts every output slab and the overflow region afresh
    h->reset_pending = true;
    return FW_OK;
}

int fw_get_stats(fw_handle* h, fw_stats* out) {
    if (!h || !out) return fail(FW_E_INVALID, "null argument");
    Ctrl c;
    const int nsb = h->ks.n_sb;
    std::vector<int32_t> cnt(nsb), sbo(nsb);
    std::vector<uint32_t> fired(nsb);
    HIP_TRY(hipMemcpyAsync(&c, h->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(cnt.data(), h->state_count, 4ll * nsb, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(sbo.data(), h->sb_out, 4ll * nsb, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(fired.data(), h->sb_fired, 4ll * nsb, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    int64_t live = 0, avail = std::min<int64_t>((int64_t)c.out_count[c.ovf_sel & 1], h->out_cap), nf = (int64_t)c.fired;
    for (int s = 0; s < nsb; s++) {
        live += cnt[s];
        avail += sbo[s];
        nf += fired[s];
    }
    if (h->reset_pending) avail = 0;
    memset(out, 0, sizeof *out);
    out->current_watermark = std::max<int64_t>(c.cur, h->host_cur);  // skipped idle advances included
    out->next_trigger_progress = c.ntp;
    out->num_late_records_dropped = (int64_t)c.late_dropped;
    out->live_state_entries = live;
    out->pending_rows = (int64_t)c.pending_rows;
    out->results_available = avail;
    out->num_fired_windows = nf;
    out->partials_emitted = (int64_t)c.partials;
    out->error_flags = (int32_t)c.error;
    out->num_superbuckets = h->ks.n_sb;
    out->flush_launches = (int64_t)c.flush_launches;
    out->partials_merged = (int64_t)c.parts_merged;
    out->state_entries_moved = (int64_t)c.state_moved;
    out->partial_bytes_written = (int64_t)c.part_bytes;
    out->partial_bytes_merged = (int64_t)c.part_bytes_merged;
    out->compact_chunks = (int64_t)c.compact_chunks;
    out->peak_superbucket_entries = (int64_t)c.peak_entries;
    out->superbucket_capacity = h->cap_e;
    out->key_rows = h->keyrow ? c.kr_next_id - std::max<int64_t>(0, c.kr_free_count - std::min(c.kr_free_cursor, c.kr_free_count)) : 0;
    out->key_row_collections = c.kr_collections;
    return FW_OK;
}

int fw_set_profiling(fw_handle* h, int enable) {
    if (!h) return fail(FW_E_INVALID, "null handle");
    HIP_TRY(hipStreamSynchronize(h->stream));
    delete h->timer;
    h->timer = nullptr;
    h->kt_device = enable == FW_PROF_DEVICE;
    HIP_TRY(hipMemsetAsync(h->kt_dev, 0, sizeof(unsigned long long) * FW_KT_N * KT_WORDS, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (enable == FW_PROF_EVENTS || enable == FW_PROF_EVENTS_ALL) {
        EvTimer* t = new EvTimer();
        t->all = enable == FW_PROF_EVENTS_ALL;
        h->timer = t;
    } else if (enable && enable != FW_PROF_DEVICE) {
        return fail(FW_E_INVALID, "bad profiling mode %d", enable);
    }
    return FW_OK;
}

int fw_get_kernel_times(fw_handle* h, fw_kernel_times* out) {
    if (!h || !out) return fail(FW_E_INVALID, "null argument");
    memset(out, 0, sizeof *out);
    unsigned long long st[N_STAMPS];
    HIP_TRY(hipMemcpyAsync(st, h->stamps, sizeof st, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    for (int k = 0; k < N_STAMPS && k < FW_KT_N; k++) out->merge_phase_cycles[k] = (int64_t)st[k];
    if (h->ablate & AB_GSTAMPS)  // diagnostic builds only: thread 0's gather parts
        fprintf(stderr, "gather_parts cells=%llu scan=%llu loads=%llu probe=%llu fold+insert=%llu seq_miss=%llu\n", st[13],
                st[14], st[2], st[4], st[7], st[15]);
    if (h->ablate & AB_GSTAMPS)  // wave 0's rows: live / home empty / undecided / slow path, slow-path rounds
        fprintf(stderr, "gather_rows live=%llu fresh=%llu undecided=%llu slow=%llu slow_rounds=%llu\n", st[8], st[9], st[10],
                st[11], st[12]);
    if (h->ablate & AB_FSTAMPS)  // diagnostic builds only: per-lane cycles of fire_one's parts
        fprintf(stderr, "fire_parts probe+merge=%llu emit=%llu expire+next=%llu claim=%llu windows=%llu\n", st[8], st[9],
                st[10], st[11], st[12]);
    if (h->kt_device) {
        unsigned long long kt[FW_KT_N * KT_WORDS];
        HIP_TRY(hipMemcpyAsync(kt, h->kt_dev, sizeof kt, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        int khz = 0;  // rate of the constant device clock wall_clock64() counts
        HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->cfg.device));
        for (int k = 0; k < FW_KT_N; k++) {
            out->ms[k] = khz > 0 ? (double)kt[k * KT_WORDS + 1] / (double)khz : 0.0;
            out->launches[k] = (int64_t)kt[k * KT_WORDS + 2];
        }
        return FW_OK;
    }
    if (!h->timer) return FW_OK;
    EvTimer* t = static_cast<EvTimer*>(h->timer);
    HIP_TRY(t->resolve());
    for (int k = 0; k < FW_KT_N; k++) {
        out->ms[k] = t->ms[k];
        out->launches[k] = t->n[k];
    }
    return FW_OK;
}

// Fingerprint of everything that gives the stored words their meaning: API, phase, window kind,
// size, slice interval, offset, key hashing, maxParallelism and the accumulator word layout (op,
// value column, NULL gate per word).  A blob is only restored into an operator with the same one.
static uint64_t semantics_fingerprint(const fw_handle* h) {
    uint64_t x = 0xcbf29ce484222325ull;
    auto mix = [&](int64_t v) {
        for (int b = 0; b < 8; b++) {
            x ^= (uint64_t)((v >> (8 * b)) & 0xff);
            x *= 0x100000001b3ull;
        }
    };
    const fw_config& c = h->cfg;
    mix(c.api);
    mix(c.agg_phase);
    mix(h->win.kind);
    mix(h->win.size);
    mix(h->win.interval);
    mix(h->win.offset);
    mix(h->cfg.key_hash);
    mix(h->ks.max_p);
    mix(c.allowed_lateness_ms);
    mix(c.tz_use_dst);
    for (size_t i = 0; i < h->tz_utc.size(); i++) {
        mix(h->tz_utc[i]);
        mix(h->tz_off[i]);
    }
    mix(h->wd.nw);
    for (int w = 0; w < h->wd.nw; w++) {
        mix(h->wd.op[w]);
        mix(h->slot_col[h->wd.col[w]]);
        mix(h->wd.gate[w]);
    }
    return x;
}

// ---- snapshot: [header][state_count[n_sb]][entries of sb 0][entries of sb 1]...
struct SnapHeader {
    uint64_t magic;
    int32_t version, n_sb, cap_e, pwe;
    int64_t cur, late_dropped, fired, live;
    uint64_t semantics;
    int64_t push_seq;  // arrival ordinals continue after the restore (W_FIRST words stay ordered)
};
static const uint64_t SNAP_MAGIC = 0x464c4b57494e3033ull;  // "FLKWIN03"

// ---- key rows in a blob (FW_KEYHASH_KEYROW): the entries carry table ids, which mean nothing to
// another handle, so a blob also holds the key row of every id its entries use:
//   [n_keys] then per key [id, hash << 32 | length, image words...]  (uint64 words)
// and a restore interns the images into its own table and rewrites the entries' keys.
static int kr_section(fw_handle* h, const uint64_t* entries, int64_t n, int pwe, std::vector<uint64_t>* out) {
    out->clear();
    if (!h->keyrow) return FW_OK;
    Ctrl c;
    int rc = read_ctrl(h, &c);
    if (rc) return rc;
    std::vector<int64_t> ids;
    ids.reserve((size_t)n);
    for (int64_t i = 0; i < n; i++) ids.push_back((int64_t)entries[(size_t)i * pwe]);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    const int64_t sw = h->kr.stride_words;
    std::vector<uint64_t> rows;
    if (!ids.empty()) {
        if (ids.front() < 0 || ids.back() >= c.kr_next_id) return fail(FW_E_STATE, "state entry with an unknown key row id");
        rows.resize((size_t)(ids.back() + 1) * sw);
        HIP_TRY(hipMemcpy(rows.data(), h->kr.arena, rows.size() * 8, hipMemcpyDeviceToHost));
    }
    out->push_back((uint64_t)ids.size());
    for (int64_t id : ids) {
        const uint64_t* r = rows.data() + (size_t)id * sw;
        out->push_back((uint64_t)id);
        out->insert(out->end(), r, r + 1 + ((uint32_t)r[0] >> 3));
    }
    return FW_OK;
}

// interns a blob's key-row section: old id -> this handle's id (and its hash); *used = words read
static int kr_restore_section(fw_handle* h, const uint64_t* sec, int64_t avail_words, std::vector<std::pair<int64_t, int64_t>>* map,
                              std::vector<int32_t>* hashes, int64_t* used) {
    map->clear();
    hashes->clear();
    if (avail_words < 1) return fail(FW_E_INVALID, "key-row section truncated");
    const int64_t nk = (int64_t)sec[0];
    int64_t p = 1;
    std::vector<int64_t> off(1, 0);
    std::vector<uint64_t> bytes;
    std::vector<int64_t> old;
    for (int64_t k = 0; k < nk; k++) {
        if (p + 2 > avail_words) return fail(FW_E_INVALID, "key-row section truncated");
        const int64_t id = (int64_t)sec[p];
        const int64_t len = (int64_t)(uint32_t)sec[p + 1];
        if ((len & 7) || p + 2 + len / 8 > avail_words) return fail(FW_E_INVALID, "key-row section truncated");
        old.push_back(id);
        bytes.insert(bytes.end(), sec + p + 2, sec + p + 2 + len / 8);
        off.push_back(off.back() + len);
        p += 2 + len / 8;
    }
    *used = p;
    if (nk == 0) return FW_OK;
    int64_t* d_off = nullptr;
    uint8_t* d_bytes = nullptr;
    int rc;
    if ((rc = dalloc(&d_off, off.size()))) return rc;
    if ((rc = dalloc(&d_bytes, std::max<size_t>(bytes.size() * 8, 8)))) { hipFree(d_off); return rc; }
    HIP_TRY(hipMemcpy(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_bytes, bytes.data(), bytes.size() * 8, hipMemcpyHostToDevice));
    rc = kr_intern(h, nk, d_off, d_bytes);
    std::vector<int64_t> ids((size_t)nk);
    hashes->resize((size_t)nk);
    if (!rc) {
        HIP_TRY(hipMemcpyAsync(ids.data(), h->d_kid, nk * 8, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipMemcpyAsync(hashes->data(), h->d_khash, nk * 4, hipMemcpyDeviceToHost, h->stream));
        Ctrl c;
        rc = read_ctrl(h, &c);  // syncs; a full table is a device error
    }
    hipFree(d_off);
    hipFree(d_bytes);
    if (rc) return rc;
    for (int64_t k = 0; k < nk; k++) map->emplace_back(old[(size_t)k], ids[(size_t)k]);
    std::sort(map->begin(), map->end());
    return FW_OK;
}

static int64_t kr_lookup(const std::vector<std::pair<int64_t, int64_t>>& map, int64_t old, size_t* pos) {
    auto it = std::lower_bound(map.begin(), map.end(), std::make_pair(old, INT64_MIN));
    if (it == map.end() || it->first != old) return -1;
    *pos = (size_t)(it - map.begin());
    return it->second;
}

int fw_snapshot(fw_handle* h, void* buf, int64_t capacity, int64_t* size) {
    if (!h || !size) return fail(FW_E_INVALID, "null argument");
    int rc = force_flush(h);  // prepareSnapshotPreBarrier -> windowBuffer.flush()
    if (rc) return rc;
    Ctrl c;
    if ((rc = read_ctrl(h, &c))) return rc;
    const int nsb = h->ks.n_sb, pwe = h->pwe;
    std::vector<int32_t> cnt(nsb);
    HIP_TRY(hipMemcpy(cnt.data(), h->state_count, sizeof(int32_t) * nsb, hipMemcpyDeviceToHost));
    int64_t total = 0;
    for (int s = 0; s < nsb; s++) total += cnt[s];
    std::vector<uint64_t> ent((size_t)total * pwe);
    {
        uint64_t* e = ent.data();
        for (int s = 0; s < nsb; s++) {
            if (!cnt[s]) continue;
            if ((rc = state_rows_to_host(h, (size_t)s, cnt[s], e))) return rc;
            e += (size_t)cnt[s] * pwe;
        }
    }
    std::vector<uint64_t> krs;
    if ((rc = kr_section(h, ent.data(), total, pwe, &krs))) return rc;
    const int64_t need = (int64_t)sizeof(SnapHeader) + 4ll * nsb + total * pwe * 8 + (int64_t)krs.size() * 8;
    *size = need;
    if (!buf) return FW_OK;
    if (capacity < need) return fail(FW_E_INVALID, "snapshot buffer too small (%lld < %lld)", (long long)capacity, (long long)need);
    SnapHeader hd{SNAP_MAGIC, 3, nsb, h->cap_e, pwe, std::max(c.cur, h->host_cur), (int64_t)c.late_dropped, 0, total, semantics_fingerprint(h),
                  (int64_t)h->push_seq};
    char* p = (char*)buf;
    memcpy(p, &hd, sizeof hd);
    p += sizeof hd;
    memcpy(p, cnt.data(), 4ll * nsb);
    p += 4ll * nsb;
    memcpy(p, ent.data(), ent.size() * 8);
    p += ent.size() * 8;
    if (!krs.empty()) memcpy(p, krs.data(), krs.size() * 8);
    return FW_OK;
}

int fw_restore(fw_handle* h, const void* buf, int64_t size) {
    if (!h || !buf) return fail(FW_E_INVALID, "null argument");
    SnapHeader hd;
    if (size < (int64_t)sizeof hd) return fail(FW_E_INVALID, "snapshot truncated");
    memcpy(&hd, buf, sizeof hd);
    const int nsb = h->ks.n_sb, pwe = h->pwe;
    if (hd.magic != SNAP_MAGIC || hd.n_sb != nsb || hd.pwe != pwe || hd.cap_e != h->cap_e ||
        hd.semantics != semantics_fingerprint(h))
        return fail(FW_E_INVALID, "snapshot layout does not match this operator configuration");
    const int64_t ent_end = (int64_t)sizeof hd + 4ll * nsb + hd.live * pwe * 8;
    if (size < ent_end) return fail(FW_E_INVALID, "snapshot truncated");
    const char* p = (const char*)buf + sizeof hd;
    std::vector<int32_t> cnt(nsb);
    memcpy(cnt.data(), p, 4ll * nsb);
    p += 4ll * nsb;
    std::vector<uint64_t> ent((size_t)hd.live * pwe);
    memcpy(ent.data(), p, ent.size() * 8);
    int rc;
    if (h->keyrow) {  // this handle's ids for the blob's key rows
        std::vector<std::pair<int64_t, int64_t>> map;
        std::vector<int32_t> hashes;
        int64_t used = 0;
        std::vector<uint64_t> sec((size_t)((size - ent_end) / 8));
        memcpy(sec.data(), (const char*)buf + ent_end, sec.size() * 8);
        if ((rc = kr_restore_section(h, sec.data(), (int64_t)sec.size(), &map, &hashes, &used))) return rc;
        for (int64_t i = 0; i < hd.live; i++) {
            size_t pos;
            const int64_t id = kr_lookup(map, (int64_t)ent[(size_t)i * pwe], &pos);
            if (id < 0) return fail(FW_E_INVALID, "snapshot entry without its key row");
            ent[(size_t)i * pwe] = (uint64_t)id;
        }
    }
    HIP_TRY(hipStreamSynchronize(h->stream));
    std::vector<int64_t> mins(nsb, INT64_MAX);
    const uint64_t* e = ent.data();
    for (int s = 0; s < nsb; s++) {
        if (!cnt[s]) continue;
        for (int i = 0; i < cnt[s]; i++)
            mins[s] = std::min(mins[s], entry_timer_end(h, (int64_t)e[(size_t)i * pwe + 1], e[(size_t)i * pwe + 2]));
        HIP_TRY(hipMemcpy(h->state + (size_t)s * h->cap_e * pwe, e, (size_t)cnt[s] * pwe * 8, hipMemcpyHostToDevice));
        e += (size_t)cnt[s] * pwe;
    }
    HIP_TRY(hipMemcpy(h->state_count, cnt.data(), 4ll * nsb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(h->sb_nar, 0, (size_t)nsb));  // restored entries are in the wide layout
    HIP_TRY(hipMemcpy(h->sb_min_timer, mins.data(), 8ll * nsb, hipMemcpyHostToDevice));
    Ctrl c;
    HIP_TRY(hipMemcpy(&c, h->ctrl, sizeof c, hipMemcpyDeviceToHost));  // the key-row allocator survives
    const Ctrl keep = c;
    HIP_TRY(launch_init_ctrl(h->ctrl, h->stream));
    // the restore drops the pending pushes: with runs, their fill counters, overflow flags and formats
    // go too (as allocate() starts them), or the next push would add onto the dropped push's fills and
    // the next flush would fold its stale rows
    if (h->run_rows) {
        const size_t n_isb = (size_t)(h->ks.n_sb >> h->ks.pass_log2);
        HIP_TRY(hipMemsetAsync(h->run_fill, 0, sizeof(uint32_t) * FW_MAX_PENDING * RUN_X * n_isb, h->stream));
        HIP_TRY(hipMemsetAsync(h->run_ovf, 0, sizeof(uint32_t) * FW_MAX_PENDING * n_isb, h->stream));
        HIP_TRY(hipMemsetAsync(h->slot_fmt, 0, sizeof(int32_t) * FW_MAX_PENDING, h->stream));
    }
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(&c, h->ctrl, sizeof c, hipMemcpyDeviceToHost));
    // SQL: union-list watermark state (WindowAggOperator.initializeState :183-206).  DataStream:
    // the WindowOperator keeps no watermark state, its timer service restarts at Long.MIN_VALUE
    // (InternalTimerServiceImpl.java:72) until the next watermark arrives.
    c.cur = h->cfg.api == FW_API_SQL ? hd.cur : INT64_MIN;
    c.ntp = INT64_MIN;
    c.late_dropped = (uint64_t)hd.late_dropped;
    c.fired = (uint64_t)hd.fired;
    c.live_entries = hd.live;
    c.kr_next_id = keep.kr_next_id;
    c.kr_free_count = keep.kr_free_count;
    c.kr_free_cursor = keep.kr_free_cursor;
    c.kr_epoch = keep.kr_epoch;
    c.kr_collections = keep.kr_collections;
    HIP_TRY(hipMemcpy(h->ctrl, &c, sizeof c, hipMemcpyHostToDevice));
    h->pushes_ub = 0;
    h->host_cur = c.cur;
    h->dev_cur = c.cur;
    h->dev_ntp = INT64_MIN;
    h->push_seq = std::max<int64_t>(h->push_seq, hd.push_seq);
    return FW_OK;
}

// ---- key-group-partitioned checkpoint (rescaling) --------------------------------------
// The heap backend writes keyed state per key group (HeapSnapshotStrategy.java:97 ->
// AbstractStateTableSnapshot.writeStateInKeyGroup :112) and a rescaled job hands every new
// subtask the key groups of its computeKeyGroupRangeForOperatorIndex range.  The blob of one key
// group is therefore independent of this build's superbucket split: entries carry the sub-bucket
// they came from, and a restoring handle re-routes every key with the same route_key the
// ingest kernel runs (only a precomputed-hash key cannot be re-hashed; it keeps its sub-bucket
// bits, which works for any target split not finer than the source's).
struct KgHeader {
    uint64_t magic;
    int32_t version, key_group, pwe, nw, sb_log2, hash_kind;
    int64_t win_size, win_interval, cur, n;
    uint64_t semantics;
    int64_t push_seq;  // arrival ordinals of the restoring handle continue after every restored blob's
};
static const uint64_t KG_MAGIC = 0x464c4b574b473033ull;  // "FLKWKG03"

int fw_snapshot_key_group(fw_handle* h, int32_t key_group, void* buf, int64_t capacity, int64_t* size) {
    if (!h || !size) return fail(FW_E_INVALID, "null argument");
    const KeySpace& ks = h->ks;
    const int li = key_group - ks.kg_start;
    if (li < 0 || li >= ks.n_kg) return fail(FW_E_INVALID, "key group %d is not owned by this subtask", key_group);
    int rc = force_flush(h);  // prepareSnapshotPreBarrier -> windowBuffer.flush()
    if (rc) return rc;
    Ctrl c;
    if ((rc = read_ctrl(h, &c))) return rc;
    const int L = ks.sb_per_kg_log2, nsub = 1 << L, pwe = h->pwe;
    std::vector<int32_t> cnt(nsub);
    HIP_TRY(hipMemcpy(cnt.data(), h->state_count + ((size_t)li << L), sizeof(int32_t) * nsub, hipMemcpyDeviceToHost));
    int64_t total = 0;
    for (int q = 0; q < nsub; q++) total += cnt[q];
    std::vector<uint64_t> ent((size_t)total * pwe);
    uint64_t* e = ent.data();
    for (int q = 0; q < nsub; q++) {
        if (!cnt[q]) continue;
        const size_t sb = ((size_t)li << L) + q;
        if ((rc = state_rows_to_host(h, sb, cnt[q], e))) return rc;
        for (int i = 0; i < cnt[q]; i++) e[(size_t)i * pwe + 2] = (uint32_t)e[(size_t)i * pwe + 2] | ((uint64_t)q << 32);
        e += (size_t)cnt[q] * pwe;
    }
    std::vector<uint64_t> krs;
    if ((rc = kr_section(h, ent.data(), total, pwe, &krs))) return rc;
    const int64_t need = (int64_t)sizeof(KgHeader) + total * pwe * 8 + (int64_t)krs.size() * 8;
    *size = need;
    if (!buf) return FW_OK;
    if (capacity < need) return fail(FW_E_INVALID, "snapshot buffer too small (%lld < %lld)", (long long)capacity, (long long)need);
    KgHeader hd{KG_MAGIC, 3, key_group, pwe, h->wd.nw, L, h->cfg.key_hash, h->win.size, h->win.interval,
                std::max(c.cur, h->host_cur), total,
                semantics_fingerprint(h), (int64_t)h->push_seq};
    memcpy(buf, &hd, sizeof hd);
    memcpy((char*)buf + sizeof hd, ent.data(), ent.size() * 8);
    if (!krs.empty()) memcpy((char*)buf + sizeof hd + ent.size() * 8, krs.data(), krs.size() * 8);
    return FW_OK;
}

int fw_restore_key_group(fw_handle* h, const void* buf, int64_t size) {
    if (!h || !buf) return fail(FW_E_INVALID, "null argument");
    KgHeader hd;
    if (size < (int64_t)sizeof hd) return fail(FW_E_INVALID, "key-group snapshot truncated");
    memcpy(&hd, buf, sizeof hd);
    const KeySpace& ks = h->ks;
    const int pwe = h->pwe, L = ks.sb_per_kg_log2;
    if (hd.magic != KG_MAGIC || hd.version != 3) return fail(FW_E_INVALID, "not a key-group snapshot");
    if (hd.pwe != pwe || hd.nw != h->wd.nw || hd.hash_kind != h->cfg.key_hash || hd.win_size != h->win.size ||
        hd.win_interval != h->win.interval || hd.semantics != semantics_fingerprint(h))
        return fail(FW_E_INVALID, "key-group snapshot of a different operator configuration");
    const int64_t ent_end = (int64_t)sizeof hd + hd.n * pwe * 8;
    if (size < ent_end) return fail(FW_E_INVALID, "key-group snapshot truncated");
    const int li = hd.key_group - ks.kg_start;
    if (li < 0 || li >= ks.n_kg) return fail(FW_E_INVALID, "key group %d is not owned by this subtask", hd.key_group);
    if (ks.hash_kind == KH_PRE && !h->keyrow && L > hd.sb_log2)
        return fail(FW_E_INVALID, "precomputed-hash keys cannot be split finer than the snapshot's sub-buckets");
    const int nsub = 1 << L;
    std::vector<int32_t> cnt(nsub);
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(cnt.data(), h->state_count + ((size_t)li << L), sizeof(int32_t) * nsub, hipMemcpyDeviceToHost));
    for (int q = 0; q < nsub; q++)
        if (cnt[q] != 0)  // restored twice, or restored after records of this key group arrived
            return fail(FW_E_STATE, "key group %d already holds state in this subtask", hd.key_group);
    std::vector<uint64_t> src((size_t)hd.n * pwe);
    memcpy(src.data(), (const char*)buf + sizeof hd, src.size() * 8);
    // key rows: this handle's ids, and the hash that routes each (BinaryRowData.hashCode)
    std::vector<std::pair<int64_t, int64_t>> map;
    std::vector<int32_t> hashes;
    if (h->keyrow) {
        int64_t used = 0;
        std::vector<uint64_t> sec((size_t)((size - ent_end) / 8));
        memcpy(sec.data(), (const char*)buf + ent_end, sec.size() * 8);
        int rc = kr_restore_section(h, sec.data(), (int64_t)sec.size(), &map, &hashes, &used);
        if (rc) return rc;
    }
    // target superbucket of every entry
    std::vector<std::vector<uint64_t>> per(nsub);
    for (int64_t i = 0; i < hd.n; i++) {
        uint64_t* e = src.data() + (size_t)i * pwe;
        int sb;
        if (h->keyrow) {
            size_t pos = 0;
            const int64_t id = kr_lookup(map, (int64_t)e[0], &pos);
            if (id < 0) return fail(FW_E_INVALID, "key-group snapshot entry without its key row");
            e[0] = (uint64_t)id;
            uint32_t m;
            sb = route_key(ks, id, hashes[pos], &m);
            if ((sb >> L) != li) return fail(FW_E_INVALID, "entry key does not belong to key group %d", hd.key_group);
        } else if (ks.hash_kind == KH_PRE) {
            sb = (li << L) + (int)((e[2] >> 32) & (uint64_t)(nsub - 1));
        } else {
            uint32_t m;
            sb = route_key(ks, (int64_t)e[0], 0, &m);
            if ((sb >> L) != li) return fail(FW_E_INVALID, "entry key does not belong to key group %d", hd.key_group);
        }
        auto& v = per[sb - (li << L)];
        v.insert(v.end(), e, e + pwe);
        v[v.size() - pwe + 2] = (uint32_t)e[2];  // flags without the source sub-bucket
    }
    std::vector<int64_t> mins(nsub);
    HIP_TRY(hipMemcpy(mins.data(), h->sb_min_timer + ((size_t)li << L), sizeof(int64_t) * nsub, hipMemcpyDeviceToHost));
    for (int q = 0; q < nsub; q++)
        if (cnt[q] + (int64_t)(per[q].size() / pwe) > h->cap_e)
            return fail(FW_E_CAPACITY, "restored key group %d exceeds the state table (%lld entries per superbucket)",
                        hd.key_group, (long long)h->cap_e);
    int64_t added = 0;
    for (int q = 0; q < nsub; q++) {
        const int64_t n = (int64_t)(per[q].size() / pwe);
        if (!n) continue;
        const size_t sb = ((size_t)li << L) + q;
        HIP_TRY(hipMemcpy(h->state + (sb * h->cap_e + cnt[q]) * pwe, per[q].data(), (size_t)n * pwe * 8,
                          hipMemcpyHostToDevice));
        HIP_TRY(hipMemset(h->sb_nar + sb, 0, 1));  // (the superbucket held no entries: cnt[q] == 0)
        for (int64_t i = 0; i < n; i++)
            mins[q] = std::min(mins[q], entry_timer_end(h, (int64_t)per[q][(size_t)i * pwe + 1], per[q][(size_t)i * pwe + 2]));
        cnt[q] += (int32_t)n;
        added += n;
    }
    HIP_TRY(hipMemcpy(h->state_count + ((size_t)li << L), cnt.data(), sizeof(int32_t) * nsub, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->sb_min_timer + ((size_t)li << L), mins.data(), sizeof(int64_t) * nsub, hipMemcpyHostToDevice));
    Ctrl c;
    int rc = read_ctrl(h, &c);
    if (rc) return rc;
    c.live_entries += added;
    c.ntp = INT64_MIN;  // next trigger recomputed at the next advance
    h->dev_ntp = INT64_MIN;
    HIP_TRY(hipMemcpy(h->ctrl, &c, sizeof c, hipMemcpyHostToDevice));
    h->push_seq = std::max<int64_t>(h->push_seq, hd.push_seq);
    return FW_OK;
}

// ---- heap keyed-state backend key-group format ------------------------------------------
// The bytes the heap backend writes for one key group of a window-aggregate operator
// (HeapSnapshotStrategy.java:161-172): writeInt(keyGroup), then per registered state
// writeShort(stateId) and that state's key-group writer --
//   window-aggs ValueState (CopyOnWriteStateMapSnapshot.writeState :127-149):
//       writeInt(n), then per entry namespace (LongSerializer: 8 B big-endian sliceEnd),
//       key (BinaryRowData: writeInt(len) + bytes), accumulator (RowDataSerializer -> BinaryRowData)
//   event / processing window-timers queues (KeyGroupPartitioner.java:241-254 with
//       TimerSerializer.serialize :147-152): writeInt(n), then per timer
//       writeLong(flipSignBit(ts)), key, namespace
// The accumulator row holds every aggregate's buffer fields in order (COUNT(*) / COUNT: count
// BIGINT; SUM / MIN / MAX: value of the aggregate's type, NULL-able; AVG: sum BIGINT|DOUBLE, count
// BIGINT), the LOCAL phase's output fields.  A timer's timestamp is
// toEpochMillsForTimer(window - 1) (SlicingWindowTimerServiceImpl.java:43-46).
namespace {

constexpr int HEAP_MAX_FIELDS = 2 * FW_MAX_AGGS;

struct HeapWriter {
    std::vector<uint8_t> b;
    void u8(uint8_t v) { b.push_back(v); }
    void be32(uint32_t v) { for (int i = 3; i >= 0; i--) b.push_back((uint8_t)(v >> (8 * i))); }
    void be16(uint16_t v) { b.push_back((uint8_t)(v >> 8)); b.push_back((uint8_t)v); }
    void be64(uint64_t v) { for (int i = 7; i >= 0; i--) b.push_back((uint8_t)(v >> (8 * i))); }
    void bytes(const uint8_t* p, size_t n) { b.insert(b.end(), p, p + n); }
};

struct HeapReader {
    const uint8_t* p;
    size_t n, at = 0;
    bool bad = false;
    bool need(size_t k) { if (at + k > n) bad = true; return !bad; }
    uint32_t be32() { if (!need(4)) return 0; uint32_t v = 0; for (int i = 0; i < 4; i++) v = v << 8 | p[at++]; return v; }
    uint16_t be16() { if (!need(2)) return 0; uint16_t v = (uint16_t)(p[at] << 8 | p[at + 1]); at += 2; return v; }
    uint64_t be64() { if (!need(8)) return 0; uint64_t v = 0; for (int i = 0; i < 8; i++) v = v << 8 | p[at++]; return v; }
    const uint8_t* take(size_t k) { if (!need(k)) return nullptr; const uint8_t* q = p + at; at += k; return q; }
};

// the accumulator row's field types (FW_T_*), in order
int heap_fields(const fw_handle* h, int32_t* type) {
    int j = 0;
    for (int g = 0; g < h->ad.n; g++) {
        const int k = h->ad.kind[g], t = h->ad.type[g];
        if (k == FW_AGG_COUNT_STAR || k == FW_AGG_COUNT) type[j++] = FW_T_I64;
        else if (k == FW_AGG_AVG) { type[j++] = t == FW_T_F64 ? FW_T_F64 : FW_T_I64; type[j++] = FW_T_I64; }
        else type[j++] = t;
    }
    return j;
}

int heap_bitset_bytes(int arity) { return ((arity + 63 + 8) / 64) * 8; }  // BinaryRowData.calculateBitSetWidthInBytes

// accumulator words -> buffer field values + NULL mask (emit_partial, restated on the host)
void heap_words_to_fields(const fw_handle* h, const uint64_t* acc, uint64_t* v, uint32_t* nm) {
    const AggDesc& ad = h->ad;
    *nm = 0;
    int j = 0;
    for (int g = 0; g < ad.n; g++) {
        const int kind = ad.kind[g], type = ad.type[g];
        const uint64_t w0 = acc[ad.w0[g]];
        const bool no_rows = ad.nn[g] >= 0 && acc[ad.nn[g]] == 0;
        uint64_t x = w0;
        bool isnull = false;
        if (kind == FW_AGG_SUM) {
            x = type == FW_T_I32 ? (uint64_t)(int64_t)(int32_t)(uint32_t)w0 : w0;
            isnull = no_rows;
        } else if (kind == FW_AGG_MIN || kind == FW_AGG_MAX) {
            if (ad.qf[g] >= 0) {  // q_result (fw_kernel_common.h)
                const uint64_t f = acc[ad.qf[g]];
                isnull = f == Q_EMPTY;
                if (isnull) x = 0;
                else if ((uint32_t)f) x = (f << 32) | (acc[ad.qn[g]] & 0xFFFFFFFFull);
                else if ((int64_t)w0 != 0) x = dkey_inv((int64_t)w0);
                else x = acc[ad.qz[g]] != Q_EMPTY ? ((acc[ad.qz[g]] & 1ull) << 63) : 0ull;
            } else {
                x = type == FW_T_F64 ? dkey_inv((int64_t)w0) : w0;
                isnull = no_rows;
            }
        } else if (kind == FW_AGG_AVG) {
            v[j++] = w0;
            x = acc[ad.w1[g]];
        }
        if (isnull) *nm |= 1u << j;
        v[j++] = isnull ? 0ull : x;
    }
}

// buffer field values -> accumulator words (the inverse; a hidden non-NULL count word becomes 1,
// its only observable property being != 0, and a MIN/MAX(DOUBLE) group is one element of ordinal 0)
void heap_fields_to_words(const fw_handle* h, const uint64_t* v, uint32_t nm, uint64_t* acc) {
    const AggDesc& ad = h->ad;
    const WordDesc& wd = h->wd;
    for (int w = 0; w < h->nw_t; w++) acc[w] = w < wd.nw ? word_identity(wd.op[w]) : 0;
    bool set[MAX_WORDS] = {};
    int j = 0;
    for (int g = 0; g < ad.n; g++) {
        const int kind = ad.kind[g], type = ad.type[g];
        const int w0 = ad.w0[g];
        if (kind == FW_AGG_COUNT_STAR || kind == FW_AGG_COUNT) {
            acc[w0] = v[j++];
            set[w0] = true;
            continue;
        }
        if (kind == FW_AGG_AVG) {
            acc[w0] = v[j++];
            acc[ad.w1[g]] = v[j++];
            set[w0] = set[ad.w1[g]] = true;
            continue;
        }
        const bool isnull = (nm >> j) & 1u;
        const uint64_t x = v[j++];
        if (isnull) continue;  // identity words
        if (ad.qf[g] >= 0) {  // merge_q_groups' re-encoding
            const bool nan = f64_isnan(x);
            acc[ad.qf[g]] = nan ? (x >> 32) : 0ull;
            if (nan) acc[ad.qn[g]] = x & 0xFFFFFFFFull;
            if (f64_iszero(x)) acc[ad.qz[g]] = x >> 63;
            if (!nan) acc[w0] = f64_iszero(x) ? 0ull : (uint64_t)dkey(x);
            continue;
        }
        if ((kind == FW_AGG_MIN || kind == FW_AGG_MAX) && type == FW_T_F64) acc[w0] = (uint64_t)dkey(x);
        else if (type == FW_T_I32) acc[w0] = (uint64_t)(int64_t)(int32_t)(uint32_t)x;
        else acc[w0] = x;
        set[w0] = true;
    }
    for (int g = 0; g < ad.n; g++) {  // hidden non-NULL counts of SUM / MIN / MAX
        const int nn = ad.nn[g];
        if (nn < 0 || set[nn]) continue;
        int jj = 0;  // field index of aggregate g
        for (int q = 0; q < g; q++) jj += ad.kind[q] == FW_AGG_AVG ? 2 : 1;
        if (!((nm >> jj) & 1u)) acc[nn] = 1;
    }
}

void heap_write_row(HeapWriter& w, const fw_handle* h, const uint64_t* v, uint32_t nm) {
    int32_t type[HEAP_MAX_FIELDS];
    const int n = heap_fields(h, type);
    const int bs = heap_bitset_bytes(n);
    w.be32((uint32_t)(bs + 8 * n));
    std::vector<uint8_t> row((size_t)(bs + 8 * n), 0);  // header byte 0 = RowKind.INSERT
    for (int j = 0; j < n; j++) {
        if ((nm >> j) & 1u) {
            row[(size_t)(j + 8) / 8] |= (uint8_t)(1u << ((j + 8) % 8));
            continue;
        }
        const uint64_t x = type[j] == FW_T_I32 ? (uint32_t)v[j] : v[j];
        memcpy(row.data() + bs + 8 * j, &x, 8);  // little-endian slot; an INT in its low 4 bytes
    }
    w.bytes(row.data(), row.size());
}

bool heap_read_row(HeapReader& r, const fw_handle* h, uint64_t* v, uint32_t* nm) {
    int32_t type[HEAP_MAX_FIELDS];
    const int n = heap_fields(h, type);
    const int bs = heap_bitset_bytes(n);
    const uint32_t len = r.be32();
    if (r.bad || len != (uint32_t)(bs + 8 * n)) return false;
    const uint8_t* p = r.take(len);
    if (!p) return false;
    *nm = 0;
    for (int j = 0; j < n; j++) {
        if ((p[(j + 8) / 8] >> ((j + 8) % 8)) & 1u) { *nm |= 1u << j; v[j] = 0; continue; }
        uint64_t x;
        memcpy(&x, p + bs + 8 * j, 8);
        v[j] = type[j] == FW_T_I32 ? (uint64_t)(int64_t)(int32_t)(uint32_t)x : x;
    }
    return true;
}

// the key's BinaryRowData image: BINROW_BIGINT / BINROW_INT keys are the one-field row the key
// projection writes (8 B header, the value slot); key rows carry their interned image
int heap_key_kind(const fw_handle* h) {
    if (h->keyrow) return FW_KEYHASH_KEYROW;
    const int k = h->cfg.key_hash;
    return k == FW_KEYHASH_BINROW_BIGINT || k == FW_KEYHASH_BINROW_INT ? k : -1;
}

int heap_check(const fw_handle* h, const fw_heap_state_ids* ids) {
    if (!ids) return fail(FW_E_INVALID, "null state ids");
    if (h->cfg.api != FW_API_SQL || h->cfg.agg_phase == FW_PHASE_LOCAL)
        return fail(FW_E_INVALID, "the heap key-group format is the SQL window-aggregate operator's keyed state");
    if (heap_key_kind(h) < 0)
        return fail(FW_E_INVALID, "the heap key-group format needs SQL key rows (BINROW_BIGINT, BINROW_INT or KEYROW keys)");
    if (ids->window_state == ids->event_timers || ids->window_state == ids->processing_timers ||
        ids->event_timers == ids->processing_timers)
        return fail(FW_E_INVALID, "state ids must differ");
    return FW_OK;
}

}  // namespace

int fw_snapshot_key_group_heap(fw_handle* h, int32_t key_group, const fw_heap_state_ids* ids, void* buf,
                               int64_t capacity, int64_t* size) {
    if (!h || !size) return fail(FW_E_INVALID, "null argument");
    int rc = heap_check(h, ids);
    if (rc) return rc;
    // the device state of the key group, in this library's own key-group format
    int64_t n_int = 0;
    if ((rc = fw_snapshot_key_group(h, key_group, nullptr, 0, &n_int))) return rc;
    std::vector<uint64_t> blob((size_t)(n_int + 7) / 8);
    if ((rc = fw_snapshot_key_group(h, key_group, blob.data(), (int64_t)blob.size() * 8, &n_int))) return rc;
    KgHeader hd;
    memcpy(&hd, blob.data(), sizeof hd);
    const int pwe = h->pwe, nw = h->nw_t;
    const uint64_t* ent = blob.data() + sizeof hd / 8;
    // key images
    std::unordered_map<int64_t, std::pair<const uint8_t*, uint32_t>> img;
    if (h->keyrow) {
        const uint64_t* sec = ent + (size_t)hd.n * pwe;
        const int64_t nk = (int64_t)sec[0];
        size_t p = 1;
        for (int64_t k = 0; k < nk; k++) {
            const uint32_t len = (uint32_t)sec[p + 1];
            img[(int64_t)sec[p]] = {(const uint8_t*)(sec + p + 2), len};
            p += 2 + len / 8;
        }
    }
    const int kk = heap_key_kind(h);
    auto write_key = [&](HeapWriter& w, int64_t key) {
        if (kk == FW_KEYHASH_KEYROW) {
            const auto& im = img.at(key);
            w.be32(im.second);
            w.bytes(im.first, im.second);
            return;
        }
        uint8_t row[16] = {};
        const uint64_t x = kk == FW_KEYHASH_BINROW_INT ? (uint32_t)key : (uint64_t)key;
        memcpy(row + 8, &x, 8);
        w.be32(16);
        w.bytes(row, 16);
    };
    struct St { int64_t key, ns; const uint64_t* acc; };
    std::vector<St> states;
    std::vector<std::pair<int64_t, int64_t>> timers;  // (key, window)
    std::vector<uint64_t> slot_acc;
    const WinDesc& win = h->win;
    if (win.hopb) {
        // block entries -> one (key, sliceEnd) state per slot with data.  Timers: the reference holds
        // one per unfired slice end with data (AggCombiner.combine step 5) and one at the first
        // unfired window end whose window holds data (the nextTriggerWindow chain, or a late
        // record's registration).  A chain timer at an EMPTY window (its predecessor's only data
        // was in the slice that window expired) is not derivable from the expired state; it fires
        // without output, and is the one timer the export leaves out.
        std::unordered_map<int64_t, std::vector<int64_t>> ends;  // key -> slice ends with data
        for (int64_t i = 0; i < hd.n; i++) {
            const uint64_t* e = ent + (size_t)i * pwe;
            const uint32_t mask = (uint32_t)e[2] >> HB_MASK_SHIFT;
            for (int s = 0; s < HB_R; s++)
                if ((mask >> s) & 1u) {
                    const int64_t se = wadd((int64_t)e[1], (int64_t)(s + 1) * win.interval);
                    states.push_back({(int64_t)e[0], se, e + 3 + s * nw});
                    ends[(int64_t)e[0]].push_back(se);
                }
        }
        for (auto& kv : ends) {
            auto& v = kv.second;
            std::sort(v.begin(), v.end());
            for (int64_t se : v)
                if (!win_fired(win, se, hd.cur)) timers.push_back({kv.first, se});
            if (win_fired(win, v.front(), hd.cur)) {  // some data slice fired: the chain's next window
                int64_t e1 = v.front();
                while (win_fired(win, e1, hd.cur)) e1 = wadd(e1, win.interval);
                const int64_t lo = wsub(e1, win.size);  // window (e1 - size, e1] holds data?
                const bool data = std::any_of(v.begin(), v.end(), [&](int64_t se) { return se > lo && se <= e1; });
                if (data && !std::binary_search(v.begin(), v.end(), e1)) timers.push_back({kv.first, e1});
            }
        }
    } else {
        for (int64_t i = 0; i < hd.n; i++) {
            const uint64_t* e = ent + (size_t)i * pwe;
            if (e[2] & F_ACC) states.push_back({(int64_t)e[0], (int64_t)e[1], e + 3});
            if (e[2] & F_TIMER) timers.push_back({(int64_t)e[0], (int64_t)e[1]});
        }
    }
    std::sort(timers.begin(), timers.end(), [&](const std::pair<int64_t, int64_t>& a, const std::pair<int64_t, int64_t>& b) {
        return a.second != b.second ? a.second < b.second : a.first < b.first;
    });
    HeapWriter w;
    w.be32((uint32_t)key_group);
    const int16_t order[3] = {ids->window_state, ids->event_timers, ids->processing_timers};
    int16_t sorted[3] = {order[0], order[1], order[2]};
    std::sort(sorted, sorted + 3);
    for (int16_t sid : sorted) {
        w.be16((uint16_t)sid);
        if (sid == ids->window_state) {
            w.be32((uint32_t)states.size());
            uint64_t v[HEAP_MAX_FIELDS];
            uint32_t nm;
            for (const St& s : states) {
                w.be64((uint64_t)s.ns);
                write_key(w, s.key);
                heap_words_to_fields(h, s.acc, v, &nm);
                heap_write_row(w, h, v, nm);
            }
        } else if (sid == ids->event_timers) {
            w.be32((uint32_t)timers.size());
            for (const auto& t : timers) {
                const int64_t ts = tz_epoch_for_timer(win.tz, wsub(t.second, 1));
                w.be64((uint64_t)ts ^ (1ull << 63));  // MathUtils.flipSignBit
                write_key(w, t.first);
                w.be64((uint64_t)t.second);
            }
        } else {
            w.be32(0);  // event-time operator: no processing-time timers
        }
    }
    *size = (int64_t)w.b.size();
    if (!buf) return FW_OK;
    if (capacity < *size) return fail(FW_E_INVALID, "snapshot buffer too small (%lld < %lld)", (long long)capacity, (long long)*size);
    memcpy(buf, w.b.data(), w.b.size());
    return FW_OK;
}

int fw_restore_key_group_heap(fw_handle* h, const void* buf, int64_t size, const fw_heap_state_ids* ids) {
    if (!h || !buf || size < 0) return fail(FW_E_INVALID, "null argument");
    int rc = heap_check(h, ids);
    if (rc) return rc;
    HeapReader r{(const uint8_t*)buf, (size_t)size};
    const int32_t kg = (int32_t)r.be32();
    const int kk = heap_key_kind(h);
    // keys: BIGINT / INT values, or key-row images numbered in order of appearance
    std::vector<std::vector<uint8_t>> images;
    std::map<std::vector<uint8_t>, int64_t> image_id;
    auto read_key = [&](int64_t* key) -> bool {
        const uint32_t len = r.be32();
        if (r.bad || len > (1u << 24)) return false;
        const uint8_t* p = r.take(len);
        if (!p) return false;
        if (kk == FW_KEYHASH_KEYROW) {
            if (len % 8) return false;
            std::vector<uint8_t> im(p, p + len);
            auto it = image_id.find(im);
            if (it == image_id.end()) {
                it = image_id.emplace(im, (int64_t)images.size()).first;
                images.push_back(im);
            }
            *key = it->second;
            return true;
        }
        if (len != 16) return false;
        for (int i = 0; i < 8; i++)
            if (p[i]) return false;  // RowKind INSERT, key field not NULL
        uint64_t x;
        memcpy(&x, p + 8, 8);
        *key = kk == FW_KEYHASH_BINROW_INT ? (int64_t)(int32_t)(uint32_t)x : (int64_t)x;
        return kk == FW_KEYHASH_BINROW_BIGINT || (x >> 32) == 0;
    };
    struct Acc { uint64_t v[HEAP_MAX_FIELDS]; uint32_t nm; };
    std::map<std::pair<int64_t, int64_t>, std::pair<int, int>> ent;  // (key, ns) -> (state index or -1, timer)
    std::vector<Acc> accs;
    bool seen[3] = {};
    while (!r.bad && r.at < r.n) {
        const int16_t sid = (int16_t)r.be16();
        const uint32_t n = r.be32();
        if (r.bad) break;
        if (sid == ids->window_state && !seen[0]) {
            seen[0] = true;
            for (uint32_t i = 0; i < n && !r.bad; i++) {
                const int64_t ns = (int64_t)r.be64();
                int64_t key;
                Acc a;
                if (!read_key(&key) || !heap_read_row(r, h, a.v, &a.nm)) { r.bad = true; break; }
                auto& slot = ent.emplace(std::make_pair(key, ns), std::make_pair(-1, 0)).first->second;
                if (slot.first >= 0) return fail(FW_E_INVALID, "duplicate window state (key, namespace) in key group %d", kg);
                slot.first = (int)accs.size();
                accs.push_back(a);
            }
        } else if (sid == ids->event_timers && !seen[1]) {
            seen[1] = true;
            for (uint32_t i = 0; i < n && !r.bad; i++) {
                const int64_t ts = (int64_t)(r.be64() ^ (1ull << 63));
                int64_t key;
                if (!read_key(&key)) { r.bad = true; break; }
                const int64_t ns = (int64_t)r.be64();
                if (ts != tz_epoch_for_timer(h->win.tz, wsub(ns, 1)))
                    return fail(FW_E_INVALID, "timer %lld of window %lld is not the window's end timer", (long long)ts, (long long)ns);
                ent.emplace(std::make_pair(key, ns), std::make_pair(-1, 0)).first->second.second = 1;
            }
        } else if (sid == ids->processing_timers && !seen[2]) {
            seen[2] = true;
            if (n != 0) return fail(FW_E_INVALID, "processing-time timers in an event-time window operator");
        } else {
            return fail(FW_E_INVALID, "unexpected state id %d in key group %d", (int)sid, kg);
        }
    }
    if (r.bad) return fail(FW_E_INVALID, "heap key-group data truncated or malformed");
    // -> this library's key-group blob, restored by fw_restore_key_group
    const int pwe = h->pwe, nw = h->nw_t;
    const WinDesc& win = h->win;
    std::vector<uint64_t> out;
    int64_t n_out = 0;
    if (win.hopb) {  // (key, sliceEnd) states -> blocks; timers are arithmetic there
        std::map<std::pair<int64_t, int64_t>, size_t> blk;  // (key, block start) -> word offset
        for (const auto& kv : ent) {
            if (kv.second.first < 0) continue;  // a timer without state fires without output
            const int64_t key = kv.first.first, se = kv.first.second;
            const int64_t bs = window_start(wsub(se, 1), win.offset, win.hb_span_div);
            const int slot = (int)((se - bs) / win.interval) - 1;
            if (slot < 0 || slot >= HB_R || wadd(bs, (int64_t)(slot + 1) * win.interval) != se)
                return fail(FW_E_INVALID, "namespace %lld is not a slice end of this window", (long long)se);
            auto it = blk.find({key, bs});
            if (it == blk.end()) {
                it = blk.emplace(std::make_pair(key, bs), out.size()).first;
                out.resize(out.size() + pwe, 0);
                uint64_t* e = out.data() + it->second;
                e[0] = (uint64_t)key;
                e[1] = (uint64_t)bs;
                for (int s = 0; s < HB_R; s++)
                    for (int x = 0; x < nw; x++) e[3 + s * nw + x] = x < h->wd.nw ? word_identity(h->wd.op[x]) : 0;
                n_out++;
            }
            uint64_t* e = out.data() + it->second;
            e[2] |= (uint64_t)(1u << slot) << HB_MASK_SHIFT;
            const Acc& a = accs[(size_t)kv.second.first];
            heap_fields_to_words(h, a.v, a.nm, e + 3 + slot * nw);
        }
    } else {
        for (const auto& kv : ent) {
            out.resize(out.size() + pwe, 0);
            uint64_t* e = out.data() + (size_t)n_out * pwe;
            e[0] = (uint64_t)kv.first.first;
            e[1] = (uint64_t)kv.first.second;
            e[2] = (kv.second.first >= 0 ? F_ACC : 0u) | (kv.second.second ? F_TIMER : 0u);
            if (kv.second.first >= 0) heap_fields_to_words(h, accs[(size_t)kv.second.first].v, accs[(size_t)kv.second.first].nm, e + 3);
            else
                for (int x = 0; x < nw; x++) e[3 + x] = x < h->wd.nw ? word_identity(h->wd.op[x]) : 0;
            n_out++;
        }
    }
    Ctrl c;
    if ((rc = read_ctrl(h, &c))) return rc;
    KgHeader hd{KG_MAGIC, 3, kg, pwe, h->wd.nw, h->ks.sb_per_kg_log2, h->cfg.key_hash, h->win.size, h->win.interval,
                c.cur, n_out, semantics_fingerprint(h), (int64_t)h->push_seq};
    std::vector<uint64_t> blob(sizeof hd / 8);
    memcpy(blob.data(), &hd, sizeof hd);
    blob.insert(blob.end(), out.begin(), out.end());
    if (h->keyrow) {  // key-row section: [n][id, length, image words]
        blob.push_back((uint64_t)images.size());
        for (size_t k = 0; k < images.size(); k++) {
            blob.push_back((uint64_t)k);
            blob.push_back((uint64_t)images[k].size());
            const size_t at = blob.size();
            blob.resize(at + images[k].size() / 8);
            memcpy(blob.data() + at, images[k].data(), images[k].size());
        }
    }
    return fw_restore_key_group(h, blob.data(), (int64_t)blob.size() * 8);
}

// ---- DataStream WindowOperator key-group state ---------------------------------------------
// A heap-backend savepoint of the DataStream WindowOperator holds, per key group, the
// "window-contents" reducing state (WindowOperatorBuilder.java:81: namespace TimeWindow, value the
// reduced record) and the "window-timers" queues (WindowOperator.java:232).  The value is the user's
// record type -- value1 with the aggregated field set, whose bytes only the operator shim can write
// -- so the heap bytes are assembled there (flink_amd/datastream/heap_state.py); this pair moves
// the device side as one fw_ds_window per (key, window) holding state or a timer.
namespace {

int ds_state_check(const fw_handle* h) {
    if (h->cfg.api != FW_API_DATASTREAM)
        return fail(FW_E_INVALID, "DataStream key-group windows are the DataStream WindowOperator's state");
    // LONG / INT keys are re-routed from the key itself; precomputed-hash keys (interned String keys)
    // from the hash the shim passes with each restored window (fw_ds_window.key_hash)
    if (h->cfg.key_hash != FW_KEYHASH_LONG && h->cfg.key_hash != FW_KEYHASH_INT && h->cfg.key_hash != FW_KEYHASH_PRECOMPUTED)
        return fail(FW_E_INVALID, "DataStream key-group windows need LONG, INT or precomputed-hash keys");
    if (h->ad.n != 1) return fail(FW_E_INVALID, "DataStream key-group windows hold one aggregated field");
    return FW_OK;
}

// the field value of a window from its words (emit_row's DataStream branch, restated on the host)
uint64_t ds_value_of(const fw_handle* h, const uint64_t* acc) {
    const AggDesc& ad = h->ad;
    const uint64_t w0 = acc[ad.w0[0]];
    switch (ad.kind[0]) {
        case FW_AGG_SUM: return ad.type[0] == FW_T_I32 ? (uint64_t)(int64_t)(int32_t)(uint32_t)w0 : w0;
        case FW_AGG_MIN:
        case FW_AGG_MAX:
        case FW_AGG_MINBY:
        case FW_AGG_MAXBY: {
            uint64_t v = ad.type[0] == FW_T_F64 ? dkey_inv((int64_t)w0) : w0;
            if (ad.dn_hi[0] >= 0 && f64_isnan(v)) v = (acc[ad.dn_hi[0]] << 32) | (acc[ad.dn_lo[0]] & 0xFFFFFFFFull);
            return v;
        }
        default: return w0;  // counts
    }
}

// the words of a window state holding `value` whose first element has ordinal `first` (the state
// after one element of that value, in its written-back form: NaN bits at ordinal 0)
void ds_words_of(const fw_handle* h, uint64_t value, int64_t first, uint64_t* acc) {
    const AggDesc& ad = h->ad;
    const WordDesc& wd = h->wd;
    for (int w = 0; w < h->nw_t; w++) acc[w] = w < wd.nw ? word_identity(wd.op[w]) : 0;
    const int w0 = ad.w0[0];
    const bool f = ad.type[0] == FW_T_F64;
    switch (ad.kind[0]) {
        case FW_AGG_SUM: acc[w0] = ad.type[0] == FW_T_I32 ? (uint64_t)(int64_t)(int32_t)(uint32_t)value : value; break;
        case FW_AGG_MIN:
        case FW_AGG_MAX:
            acc[w0] = f ? (uint64_t)dkey(value) : ad.type[0] == FW_T_I32 ? (uint64_t)(int64_t)(int32_t)(uint32_t)value : value;
            if (ad.dn_hi[0] >= 0 && f64_isnan(value)) {
                acc[ad.dn_hi[0]] = value >> 32;
                acc[ad.dn_lo[0]] = value & 0xFFFFFFFFull;
            }
            break;
        case FW_AGG_MINBY:
        case FW_AGG_MAXBY:
            acc[w0] = f ? (uint64_t)dkey(f64_isnan(value) ? 0x7FF8000000000000ull : value)
                        : ad.type[0] == FW_T_I32 ? (uint64_t)(int64_t)(int32_t)(uint32_t)value : value;
            acc[ad.by_prev] = (uint64_t)first;  // the restored element is retained
            break;
        default: acc[w0] = value; break;
    }
    // hidden counts (the sliding window's COUNT(*), a non-NULL count): only != 0 is observable
    if (ad.count_star_word >= 0 && ad.count_star_word != w0) acc[ad.count_star_word] = 1;
    if (ad.nn[0] >= 0 && ad.nn[0] != w0) acc[ad.nn[0]] = 1;
    if (ad.first_word >= 0) acc[ad.first_word] = (uint64_t)first;
}

}  // namespace

int fw_ds_snapshot_key_group(fw_handle* h, int32_t key_group, fw_ds_window* out, int64_t capacity, int64_t* n) {
    if (!h || !n) return fail(FW_E_INVALID, "null argument");
    int rc = ds_state_check(h);
    if (rc) return rc;
    int64_t sz = 0;
    if ((rc = fw_snapshot_key_group(h, key_group, nullptr, 0, &sz))) return rc;  // flushes
    std::vector<uint64_t> blob((size_t)(sz + 7) / 8);
    if ((rc = fw_snapshot_key_group(h, key_group, blob.data(), (int64_t)blob.size() * 8, &sz))) return rc;
    KgHeader hd;
    memcpy(&hd, blob.data(), sizeof hd);
    const int pwe = h->pwe;
    const uint64_t* ent = blob.data() + sizeof hd / 8;
    int64_t m = 0;
    for (int64_t i = 0; i < hd.n; i++) {
        const uint64_t* e = ent + (size_t)i * pwe;
        const uint32_t f = (uint32_t)e[2];
        const int32_t fl = ((f & F_ACC) ? FW_DSW_CONTENTS : 0) | ((f & F_TIMER) ? FW_DSW_TRIGGER : 0) |
                           ((f & F_CLEAN) ? FW_DSW_CLEANUP : 0);
        if (!fl) continue;
        if (out && m < capacity) {
            fw_ds_window& w = out[m];
            w.key = (int64_t)e[0];
            w.window_end = (int64_t)e[1];
            w.value = (f & F_ACC) ? (int64_t)ds_value_of(h, e + 3) : 0;
            w.first_ord = (f & F_ACC) && h->ad.first_word >= 0 ? (int64_t)e[3 + h->ad.first_word] : -1;
            w.flags = fl;
            w.key_hash = 0;
        }
        m++;
    }
    *n = m;
    if (out && capacity < m) return fail(FW_E_INVALID, "window buffer too small (%lld < %lld)", (long long)capacity, (long long)m);
    return FW_OK;
}

int fw_ds_restore_key_group(fw_handle* h, int32_t key_group, const fw_ds_window* in, int64_t n, int64_t next_push_seq) {
    if (!h || (n > 0 && !in) || n < 0) return fail(FW_E_INVALID, "null argument");
    int rc = ds_state_check(h);
    if (rc) return rc;
    const WinDesc& win = h->win;
    const int pwe = h->pwe;
    if (key_group < h->ks.kg_start || key_group >= h->ks.kg_start + h->ks.n_kg)
        return fail(FW_E_INVALID, "key group %d is not owned by this subtask", key_group);
    std::vector<uint64_t> ent;
    ent.reserve((size_t)n * pwe);
    for (int64_t i = 0; i < n; i++) {
        const fw_ds_window& w = in[i];
        if (w.flags & ~(FW_DSW_CONTENTS | FW_DSW_TRIGGER | FW_DSW_CLEANUP) || !w.flags)
            return fail(FW_E_INVALID, "window %lld: bad flags %d", (long long)i, w.flags);
        // a window of this assigner: start = end - size on the slide grid (SlidingEventTimeWindows
        // .assignWindows :77-90; tumbling: slide = size)
        const int64_t st = wsub(w.window_end, win.size);
        if (window_start(st, win.offset, win.slide_div) != st)
            return fail(FW_E_INVALID, "window [%lld, %lld) is not a window of this assigner", (long long)st, (long long)w.window_end);
        if ((w.flags & FW_DSW_CLEANUP) && ds_cleanup_time(win, w.window_end) == INT64_MAX)
            return fail(FW_E_INVALID, "window %lld has no cleanup time but a cleanup timer", (long long)w.window_end);
        // precomputed-hash keys (a shim's interned String keys): the window's superbucket comes from
        // the key's hash, routed as the ingest routes the key's records; the sub-bucket rides in the
        // high half of the flags word like a key-group blob's (fw_restore_key_group)
        uint64_t sub = 0;
        if (h->ks.hash_kind == KH_PRE && !h->keyrow) {
            uint32_t m;
            const int sb = route_key(h->ks, w.key, w.key_hash, &m);
            if ((sb >> h->ks.sb_per_kg_log2) != key_group - h->ks.kg_start)
                return fail(FW_E_INVALID, "window %lld: key hash %d is not in key group %d", (long long)i, w.key_hash, key_group);
            sub = (uint64_t)(sb & ((1 << h->ks.sb_per_kg_log2) - 1));
        }
        const size_t at = ent.size();
        ent.resize(at + pwe, 0);
        uint64_t* e = ent.data() + at;
        e[0] = (uint64_t)w.key;
        e[1] = (uint64_t)w.window_end;
        e[2] = ((w.flags & FW_DSW_CONTENTS) ? F_ACC : 0u) | ((w.flags & FW_DSW_TRIGGER) ? F_TIMER : 0u) |
               ((w.flags & FW_DSW_CLEANUP) ? F_CLEAN : 0u) | (sub << 32);
        if (w.flags & FW_DSW_CONTENTS) {
            if (h->ad.first_word >= 0 && (w.first_ord < 0 || (w.first_ord >> 32) >= next_push_seq))
                return fail(FW_E_INVALID, "window %lld: first element ordinal not below push %lld", (long long)i,
                            (long long)next_push_seq);
            ds_words_of(h, (uint64_t)w.value, w.first_ord, e + 3);
        } else {
            for (int x = 0; x < h->nw_t; x++) e[3 + x] = x < h->wd.nw ? word_identity(h->wd.op[x]) : 0;
        }
    }
    Ctrl c;
    if ((rc = read_ctrl(h, &c))) return rc;
    KgHeader hd{KG_MAGIC, 3, key_group, pwe, h->wd.nw, h->ks.sb_per_kg_log2, h->cfg.key_hash, win.size, win.interval,
                c.cur, (int64_t)(ent.size() / pwe), semantics_fingerprint(h), std::max<int64_t>(next_push_seq, 0)};
    std::vector<uint64_t> blob(sizeof hd / 8);
    memcpy(blob.data(), &hd, sizeof hd);
    blob.insert(blob.end(), ent.begin(), ent.end());
    return fw_restore_key_group(h, blob.data(), (int64_t)blob.size() * 8);
}

// ---- host-side restatements (the exact code the kernels run), for host partitioners/tests
int32_t fw_host_key_group(int32_t key_hash_kind, int64_t key, int32_t precomputed_hash, int32_t max_parallelism) {
    return key_group_for_hash(java_key_hash(key_hash_kind, key, precomputed_hash), max_parallelism);
}
int fw_host_assign_key_groups(const int64_t* key, const int32_t* key_hash, int64_t n, int32_t key_hash_kind,
                              int32_t max_parallelism, int32_t parallelism, int32_t* kg, int32_t* dest) {
    if (n < 0 || (n > 0 && !key) || max_parallelism <= 0 || parallelism <= 0 || parallelism > max_parallelism)
        return fail(FW_E_INVALID, "fw_host_assign_key_groups: bad arguments");
    for (int64_t i = 0; i < n; i++) {
        const int32_t g = key_group_for_hash(java_key_hash(key_hash_kind, key[i], key_hash ? key_hash[i] : 0), max_parallelism);
        if (kg) kg[i] = g;
        if (dest) dest[i] = operator_for_key_group(max_parallelism, parallelism, g);
    }
    return FW_OK;
}
int64_t fw_host_window_start(int64_t ts, int64_t offset, int64_t size) {
    return window_start(ts, offset, make_udiv((uint64_t)size));
}
int64_t fw_host_next_trigger_watermark(int64_t wm, int64_t interval) {
    return next_trigger_watermark(wm, make_udiv((uint64_t)interval));
}

int fw_host_time_op(const fw_config* cfg, int32_t what, int64_t x, int64_t* out) {
    if (!cfg || !out) return fail(FW_E_INVALID, "null argument");
    fw_handle h;
    h.cfg = *cfg;
    const int rc = validate_and_plan(&h);  // host-only planning; w.tz points at h's host copy
    if (rc) return rc;
    const WinDesc& w = h.win;
    switch (what) {
        case 0: *out = tz_to_utc_ts(w.tz, x); break;
        case 1: *out = tz_epoch_for_timer(w.tz, x); break;
        case 2: *out = tz_next_trigger_watermark(w.tz, x, w.slice_div); break;
        case 3: *out = slice_end_of(w, tz_to_utc_ts(w.tz, x)); break;
        case 4: *out = window_start_of(w, x); break;
        default: return fail(FW_E_INVALID, "bad time op %d", what);
    }
    return FW_OK;
}

}  // extern "C"
