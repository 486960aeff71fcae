// fw_internal.h -- structures shared by the gfx950 kernels (fw_kernels.hip) and the C-ABI
// implementation (fw_api.hip).  Not part of the public boundary (include/flinkwin.h is).
#pragma once
#include <stdint.h>

#include <initializer_list>

#include "../../include/flinkwin.h"
#include "fw_device.h"

namespace fw {

constexpr int BLOCK = 256;          // threads per workgroup of the small helper kernels
constexpr int MAX_WORDS = 8;        // accumulator words per (key, slice)
constexpr int MAX_KCOLS = 8;        // value columns a kernel loads per record
constexpr int FW_MAX_PENDING = 8;   // pushes buffered between two flushes

// ---- ingest (K1+K2+K3): one workgroup per chunk of ig_block * RPT rows: 512 threads, two
// workgroups per CU (one loads while the other folds / sorts / stores) while 8 rows per thread fit
// the registers (<= 2 accumulator words); 1024 threads, one workgroup per CU, for the wider
// accumulators, so a chunk still holds 4096 rows (half the cells, half the per-chunk histogram
// and scan work of 2048-row chunks)
constexpr int IG_BLOCK = 512;  // the 512-thread variant (and the default LDS budget below)
constexpr int IG_SRPT = 2;                      // rows per thread per fold sub-tile
constexpr int IG_SUB = IG_BLOCK * IG_SRPT;      // rows per fold sub-tile (1024)
constexpr int IG_LDS = 78 * 1024;               // dynamic LDS per workgroup: histogram + fold/stage area
constexpr int IG_MAX_SB = 16384;                // superbuckets the ingest histogram holds (16-bit counters, 32 KiB)
constexpr int MAX_PASS_LOG2 = 3;                // state superbuckets per ingest superbucket, log2 (KeySpace)
constexpr int IG_HDR_WORDS = 16;                // 8-B words of per-chunk counters at the LDS base
constexpr int ig_hist_words(int n_sb) { return ((n_sb + 7) >> 3) << 1; }  // u16 counters, 16-B multiple
// rows per thread by accumulator words and loaded value columns (template NV): the chunk's rows
// and partials stay in registers (<= 128 VGPRs)
constexpr int ig_rpt(int nw, int nv) { return nv > 4 ? 2 : nw <= 2 ? 8 : nw <= 4 ? 4 : 2; }
constexpr int ig_block(int nw, int nv) { return (nv > 4 || nw > 2) ? 1024 : 512; }
constexpr int ig_lds(int block) { return block == 1024 ? 156 * 1024 : 78 * 1024; }  // (two 512-thread workgroups per CU)
// the template NV of a count of loaded value columns
constexpr int ig_nv(int nv) { return nv <= 2 ? nv : nv <= 4 ? 4 : 8; }
// LDS fold slots per chunk (direct mapped; a collision just leaves the row unfolded).  The
// 1024-thread variants (> 2 words) have a CU's LDS to themselves: 2048 / 1024 slots (round 6; 512 /
// 256 before, and per 2048-row sub-tile)
constexpr int ig_slots(int nw) { return nw <= 2 ? 1024 : nw <= 4 ? 2048 : 1024; }
constexpr int ig_fold_bytes(int nw) { return ig_slots(nw) * (4 + 8 + 8 + 8 * nw); }

// ---- merge/fire (K4+K5): persistent 1024-thread workgroups, one per CU (the LDS entry table fills
// it).  Two 512-thread workgroups per CU with half the entries each were measured out (rounds 2-5:
// half the LDS entries per superbucket, twice the superbuckets; CFG2 flush 127 -> 165 us)
constexpr int MG_BLOCK = 1024;
constexpr int MG_CELL_GROUP = 1024;             // cells (chunks) scanned at a time per pending push (one per thread)
// LDS slice-state capacity (entries) per superbucket by accumulator words
// (kind: FW_WIN_* of a SQL operator, KIND_DSWIN (3) for DataStream windows).  One accumulator word
// and TUMBLE: 3072 entries, which leaves room for an index of 4x the entries (short probes); the
// window kinds that keep several slices per key (HOP, CUMULATE, DataStream panes) keep 4096 entries
// of capacity with a 2x index.
constexpr int mg_entries(int nw, int kind) {
    if (kind == 4) return nw <= 1 ? 1536 : 768;  // KIND_HOPB: HB_R slots of nw words per entry
    return nw <= 1 ? (kind == FW_WIN_TUMBLE ? 3072 : 4096) : nw <= 4 ? 2048 : 1024;
}
// LDS index slots of a table of E entries with NW accumulator words: a power of two, 4E when it
// fits beside the entries in a workgroup's LDS, else the largest that does
constexpr int mg_idx_slots(int nw, int e) {
    const int entry_bytes = 8 + 8 + 4 + 8 * nw + 2;  // key, slice, flag, acc, due
    const int room = (158 * 1024 - e * entry_bytes) / 4;
    int n = 1;
    while (n < 4 * e) n <<= 1;  // 4 index slots per entry aimed at
    while (n > room) n >>= 1;
    return n;
}

// ---- cell table tiling.  A cell word (start | count << 16) is written once per (chunk,
// superbucket) by the ingest workgroup of that chunk.  16 cells share one 64-B line, and the 16
// chunks of a line are ones the dispatcher deals to the same XCD at about the same time
// (blocks c, c+8, ..., c+120 of a 128-block group), so their 4-B stores merge in that XCD's L2
// into one full-line write instead of 16 partial-sector writes.  Per slot the table is
// [tile][n_sb][16]; the merge kernel reads a superbucket's cells as whole lines.
constexpr int CELL_LANES = 16;
__host__ __device__ constexpr int64_t cell_pad(int64_t nch) { return (nch + 127) / 128 * 128; }
__host__ __device__ inline size_t cell_index(int64_t c, int64_t n_sb, int64_t sb) {
    const int64_t tile = (c >> 7) * 8 + (c & 7);
    return ((size_t)tile * n_sb + sb) * CELL_LANES + ((c >> 3) & 15);
}
// flat cell position f (= tile * 16 + lane) -> chunk; inverse of cell_index's (tile, lane)
__host__ __device__ inline int64_t cell_chunk(int64_t f) {
    const int64_t tile = f >> 4;
    return (tile >> 3) * 128 + (tile & 7) + 8 * (f & 15);
}

// ---- runs: the partial rows of one push, superbucket-contiguous.  Each ingest chunk claims, per
// ingest superbucket, a stretch of that superbucket's sub-run with one agent-scope atomic add on the
// sub-run's fill counter, and stores its rows there; there are RUN_X sub-runs per (push, superbucket),
// one per XCD (chunk c -> c % RUN_X, the dispatcher's XCD), so the pieces that share a line come from
// one L2.  The merge kernel then reads each superbucket's rows as RUN_X contiguous stretches per push
// (no per-chunk cell words, no dependent cell -> row round trip).  A sub-run holds sub_cap rows;
// rows past it, and every row of a chunk whose format differs from its push's, stay in the chunk's
// own region of the partial buffer with their cell word (count > 0), and the (push, superbucket)
// overflow flag sends the merge there too.
constexpr int RUN_X = 8;
constexpr int RUN_KMAX = 4;             // ingest superbuckets per ingest thread for the run claims
constexpr uint32_t RUN_LOCAL = 1u << 31;  // k_ingest staging: the row stays in the chunk's region

// the ingest kernel's LDS holds the run bookkeeping of n_isb superbuckets and chunks of block * rpt
// rows beside a store stage of at least 256 rows, and its threads claim every superbucket's stretch
constexpr bool ig_runs_fit(int n_isb, int block, int rpt, int nw) {
    const int64_t lds = block == 1024 ? 156 * 1024 : 78 * 1024;
    const int64_t fixed = 8 * (16 + ((n_isb + 3) >> 2) * 2) + 4 * (2 * (int64_t)((n_isb + 3) & ~3) + block * rpt) + 16;
    return n_isb <= RUN_KMAX * block && lds - fixed >= 256 * 8 * (2 + nw);
}

// Partial-row formats, one per (push slot, chunk); a cell word is start | count << 16 | format << 30
// (chunks hold <= 4096 rows).  A chunk whose rows all took the ingest kernel's common path (UTC SQL
// slice ends on the slice grid, within PF_MAX_RANK slices of the push's rank base) leaves the slice
// end out of its rows: it is slot_base + rank * interval, with the rank byte in a side array.  A
// COUNT(*)-only layout whose chunk folded nothing also leaves out the count (every row counts 1).
constexpr uint32_t PF_WIDE = 0;    // (key, sliceEnd, acc[nw])
constexpr uint32_t PF_NARROW = 1;  // (key, acc[nw]) + rank byte
constexpr uint32_t PF_UNIT = 2;    // (key) + rank byte; acc = 1
// (runs, one integer accumulator word) one 8-B word per partial: the key and the accumulator as
// offsets from the flush epoch's bases and the slice as a rank from its rank base,
//   (key - kbase) << (64 - kb) | rank << vb | (acc - vbase)
// with kb / rb / vb bits (Ctrl::pk_cur_*; the rank base is slot_base[0], the epoch's first push's).
// The bases come from the previous push's key and accumulator ranges (2x headroom); a chunk with a
// row outside them writes PF_WIDE rows into its own region instead.
constexpr uint32_t PF_PACK = 3;
constexpr int64_t PF_MAX_RANK = 255;
constexpr uint32_t PK_OK = 1u << 31;  // Ctrl::pk_*_bits: kb | rb << 8 | vb << 16 | PK_OK
__host__ __device__ inline uint32_t cell_count(uint32_t v) { return (v >> 16) & 0x3FFFu; }
__host__ __device__ inline uint32_t cell_start(uint32_t v) { return v & 0xFFFFu; }
__host__ __device__ inline uint32_t cell_fmt(uint32_t v) { return v >> 30; }
// words per row of a format
__host__ __device__ inline int pf_stride(uint32_t fmt, int nw) { return fmt == PF_WIDE ? 2 + nw : fmt == PF_NARROW ? 1 + nw : 1; }
// a compact format with a side array of rank bytes
__host__ __device__ inline bool pf_rank_bytes(uint32_t fmt) { return fmt == PF_NARROW || fmt == PF_UNIT; }

// Accumulator word operations.  Every built-in aggregate maps to 1 or 2 words, except SQL
// MIN/MAX(DOUBLE), whose strict-comparison-in-arrival-order semantics need a small word group.
enum WordOp : int32_t {
    W_CNT = 0,    // += 1                       COUNT(*), COUNT(col), AVG count (gated: non-null rows)
    W_SUM_I = 1,  // += v (64-bit wrap)         SUM(BIGINT/INT), AVG(BIGINT/INT) sum
    W_SUM_F = 2,  // += v (IEEE double)         SUM(DOUBLE), AVG(DOUBLE) sum
    W_MIN_I = 3,  // min (signed)               MIN(BIGINT/INT)
    W_MAX_I = 4,  // max (signed)               MAX(BIGINT/INT)
    W_MIN_D = 5,  // min over dkey(v)           DataStream min(double): Double.compare order
    W_MAX_D = 6,  // max over dkey(v)           DataStream max(double)
    // SQL MIN/MAX(DOUBLE): MinAggFunction/MaxAggFunction keep the first value and replace it only
    // on a strict `<` / `>` (MaxAggFunction.java:63-72), in arrival order.  So the result is NaN
    // iff the first non-null value is NaN (NaN compares false both ways), else the min/max of the
    // non-NaN values with ties (only -0.0 == +0.0 are equal with different bits) going to the
    // earliest arrival.  That decomposes into order-insensitive atomics over an arrival ordinal
    // `ord` (32 bits, unique per record within one flush; state from earlier flushes has ord 0):
    W_QMIN = 7,    // signed min of dkey(v), -0.0 folded into +0.0, over non-NaN values
    W_QMAX = 8,    // signed max of the same key
    W_QFIRST = 9,  // unsigned min of ord << 32 | (isNaN ? bits >> 32 : 0) over non-null values
                   //   (the high half of a NaN is never 0: its exponent bits are all ones)
    W_QNANLO = 10, // unsigned min of ord << 32 | (bits & 0xffffffff) over NaN values
    W_QZERO = 11,  // unsigned min of ord << 1 | sign over +-0.0 values
    W_CNTV = 12,   // += v                      GLOBAL phase: a local COUNT / AVG count column
    // DataStream (ComparableAggregator / SumAggregator return value1, the window's FIRST element,
    // with the aggregated field set: SumAggregator.java:66-76, ComparableAggregator.java:83-104)
    W_FIRST = 13,  // unsigned min of the global arrival ordinal push_seq << 32 | row: the first element
    // DataStream MIN/MAX(DOUBLE): MaxComparator/MinComparator (Comparator.java:48-101) replace the
    // field unless the accumulator is strictly extremal by Double.compareTo, so among equal values
    // the LAST arrival wins; only NaNs (all equal under compareTo) differ in their bits.  The NaN
    // that arrived last, split in halves, each with the 32-bit arrival ordinal within the flush
    // (state from earlier flushes keeps ordinal 0):
    W_DNHI = 14,   // unsigned max of ord << 32 | (isNaN ? bits >> 32 : 0) over NaN values (0: none)
    W_DNLO = 15,   // unsigned max of ord << 32 | (bits & 0xffffffff) over NaN values
    // DataStream minBy / maxBy (ComparableAggregator byAggregate, ComparableAggregator.java:89-96):
    // the element with the extremal field, ties to the first (or last) arrival.  That is the
    // lexicographic extremum of (field under compareTo, arrival ordinal), one commutative fold of
    // a word PAIR: the field key and the arg's global ordinal change together (by_fold, under the
    // entry's lock bit in LDS; ingest partials are not pre-folded).  The third word keeps the
    // ordinal the host retains the element for (write-back retain / release events).
    W_BYMAX_I = 16,   // field key of the arg: the value (Long / Integer.compareTo)
    W_BYMIN_I = 17,
    W_BYMAX_D = 18,   // dkey of the value with NaN canonical (Double.compareTo: -0.0 < 0.0 < NaN)
    W_BYMIN_D = 19,
    W_BYO_FIRST = 20, // global arrival ordinal of the arg; ties to the smaller ordinal
    W_BYO_LAST = 21,  //   ... ties to the larger ordinal
    W_BYPREV = 22     // the arg ordinal as of the last write-back (~0: none), never folded
};

FW_HD uint64_t word_identity(int32_t op) {
    switch (op) {
        case W_MIN_I:
        case W_MIN_D:
        case W_QMIN: return (uint64_t)INT64_MAX;
        case W_MAX_I:
        case W_MAX_D:
        case W_QMAX: return (uint64_t)INT64_MIN;
        case W_QFIRST:
        case W_QNANLO:
        case W_QZERO:
        case W_FIRST: return ~0ull;
        case W_BYMAX_I:
        case W_BYMAX_D: return (uint64_t)INT64_MIN;
        case W_BYMIN_I:
        case W_BYMIN_D: return (uint64_t)INT64_MAX;
        case W_BYO_FIRST:
        case W_BYPREV: return ~0ull;
        default: return 0;  // counts, integer sums, +0.0 for double sums; W_DNHI / W_DNLO: no NaN yet;
                            // W_BYO_LAST: earlier than any element
    }
}
FW_HD bool is_byword(int32_t op) { return op >= W_BYMAX_I && op <= W_BYPREV; }
// does the element (v, o) replace the arg (cv, co) of a minBy / maxBy pair: strictly extremal
// field key, or an equal key and the tie rule's ordinal (MaxByComparator / MinByComparator,
// Comparator.java:58-101, then `first ? value1 : value2` on c == 0)
FW_HD bool by_better(int32_t vop, int32_t oop, uint64_t v, uint64_t o, uint64_t cv, uint64_t co) {
    const bool mx = vop == W_BYMAX_I || vop == W_BYMAX_D;
    if (v != cv) return mx ? (int64_t)v > (int64_t)cv : (int64_t)v < (int64_t)cv;
    return oop == W_BYO_FIRST ? o < co : o > co;
}
FW_HD bool is_qword(int32_t op) { return op >= W_QMIN && op <= W_QZERO; }
FW_HD bool is_dnword(int32_t op) { return op == W_DNHI || op == W_DNLO; }
constexpr uint64_t Q_EMPTY = ~0ull;
FW_HD bool f64_isnan(uint64_t b) { return (b & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull; }
FW_HD bool f64_iszero(uint64_t b) { return (b & 0x7FFFFFFFFFFFFFFFull) == 0; }

// Entry flags of the HBM slice-state table.
constexpr uint32_t F_ACC = 1u;    // windowState(key, slice) != null
constexpr uint32_t F_TIMER = 2u;  // event-time timer registered for (key, window = slice)
// DataStream window entries (KIND_DSWIN): F_TIMER is the window's maxTimestamp timer, F_CLEAN its
// cleanup timer at cleanupTime (WindowOperator.registerCleanupTimer :616-628)
constexpr uint32_t F_CLEAN = 32u;

// Error bits reported through Ctrl::error (= fw_stats.error_flags, FW_ERRF_* in flinkwin.h).
constexpr uint32_t ERR_CHUNKS = 1u;
constexpr uint32_t ERR_STATE = 2u;
constexpr uint32_t ERR_OUTPUT = 4u;
constexpr uint32_t ERR_TREQ = 8u;
constexpr uint32_t ERR_KEYGROUP = 16u;  // a record's key group is outside this subtask's range
constexpr uint32_t ERR_LATE = 32u;      // late-fire rows or late side-output rows over capacity
constexpr uint32_t ERR_ORDEV = 64u;     // first-element retain / release events over capacity
constexpr uint32_t ERR_KEYROW = 128u;   // key-row table full, or a key row over key_row_max_bytes / misaligned
static_assert(ERR_CHUNKS == FW_ERRF_CHUNKS && ERR_STATE == FW_ERRF_STATE && ERR_OUTPUT == FW_ERRF_OUTPUT &&
                  ERR_TREQ == FW_ERRF_TREQ && ERR_KEYGROUP == FW_ERRF_KEYGROUP && ERR_LATE == FW_ERRF_LATE &&
                  ERR_ORDEV == FW_ERRF_ORDEV && ERR_KEYROW == FW_ERRF_KEYROW,
              "error bits and the public FW_ERRF_* values");

// FW_KEYHASH_KEYROW: the key-row intern table in HBM.  The window state keys on a dense int64 id per
// distinct key row; the id's image (the key row's BinaryRowData bytes, what BinaryRowData.equals
// compares) sits at arena[id * stride_words], its hashCode and length in meta[id].  An open-
// addressing index over the images gives each pushed row its id (k_kr_intern); ids whose key row
// no state entry, pending partial, timer request or unread result holds any more are collected
// (k_kr_gc_*) when the fresh ids run low, reused through the free list, and the index is rebuilt
// without them.
struct KeyRowTable {
    uint32_t* slots;        // [n_slots] 0 empty, 1 being inserted, 2 + id
    int64_t n_slots;        // power of two, >= 2 * cap_ids
    int64_t* meta;          // [cap_ids] hash << 32 | image length
    uint64_t* arena;        // [cap_ids * stride_words]
    int32_t stride_words;   // words per id: meta word + image, padded to whole 128-B lines
    int32_t max_len;        // key_row_max_bytes: longest image accepted
    int64_t cap_ids;
    uint32_t* mark;         // [cap_ids] collection epoch that found the id live
    int64_t* free_list;     // [cap_ids]
};

// Device-resident operator control block (one per handle).  Only kernels write it, so a
// watermark cycle needs no host round trip.
// Last-workgroup election counters (grid_last_wg): [ingest | merge][16 groups + top], one
// 128-byte line each, so the grid's device-scope atomics do not queue on one address.
constexpr int TK_GROUPS = 16;
struct Tickets {
    uint32_t c[2][TK_GROUPS + 1][32];
    uint32_t work[8][32];  // k_merge_fire: next superbucket of each XCD's share (reset by the last workgroup)
};

struct Ctrl {
    int64_t cur;             // currentProgress == operator / timer-service watermark
    int64_t ntp;             // nextTriggerProgress
    int64_t min_pending;     // RecordsWindowBuffer.minSliceEnd of the pending partials
    int64_t pending_pushes;  // pushes waiting in the partial buffer (flushed by k_merge_fire)
    int64_t n_treq;          // pending timer requests (late records)
    uint64_t out_count[2];   // rows in the shared overflow region since the last reset; [ovf_sel] is
                             // live, the other is kept 0 so a merge launch that resets the results
                             // can start on it while the previous rows are still counted
    uint64_t late_dropped;   // numLateRecordsDropped
    uint64_t fired;          // fired (key, window) timers
    uint64_t pending_rows;   // rows ingested but not yet flushed
    int64_t live_entries;    // live (key, slice) entries in the state table
    uint32_t error;
    int32_t push_slot;       // partial-buffer slot of the push being ingested
    uint64_t partials;       // partials written by the ingest kernels (cumulative)
    uint32_t fold_skip;      // k_ingest: the last pushes' LDS fold merged (almost) nothing -> skip it
    uint32_t push_count;     // pushes ingested (every 8th one folds regardless, to re-measure)
    int32_t ovf_sel;         // live out_count
    int32_t pad0;
    int64_t n_lfire;         // DataStream late-fire rows pending (EventTimeTrigger.onElement FIRE)
    int64_t n_side;          // DataStream late side-output rows since the last fw_late_records
    int64_t n_ordev;         // DataStream first-element retain / release events since the last read
    uint64_t flush_launches; // merge launches that flushed pending partials (cumulative)
    uint64_t parts_merged;   // partial rows those flushes read (cumulative)
    uint64_t part_bytes;     // bytes of partial rows (and rank bytes) the ingest kernels wrote (cumulative)
    uint64_t part_bytes_merged;  // of those, the bytes flushes read (cumulative)
    uint64_t compact_chunks; // chunks written in a compact partial-row format (cumulative)
    uint64_t state_moved;    // state entries the merge launches loaded + wrote back (cumulative)
    uint64_t peak_entries;   // most entries one superbucket's LDS table held in a merge (since create / restore)
    // FW_KEYHASH_KEYROW: the key-row intern table's allocator (KeyRowTable)
    int64_t kr_next_id;      // ids handed out fresh so far (ids < kr_next_id exist)
    int64_t kr_free_count;   // ids in the free list (rebuilt by each collection)
    int64_t kr_free_cursor;  // free-list ids handed out since that collection
    uint32_t kr_epoch;       // mark epoch of the current collection
    int32_t kr_gc;           // a collection runs in the current advance (set by k_kr_gc_begin)
    int64_t kr_collections;  // collections so far
    // PF_PACK parameters (IngestArgs::pack): pk_next_* measured by the last push (its key and
    // accumulator ranges), taken by the next flush epoch's first push (slot 0) into pk_cur_*, which
    // every push of the epoch and the merge that flushes them decode with
    int64_t pk_next_k, pk_next_v;
    int64_t pk_cur_k, pk_cur_v;
    uint32_t pk_next_bits, pk_cur_bits;  // kb | rb << 8 | vb << 16 | PK_OK
};

// Window / slice description shared by both kernels (SliceAssigners.java).
struct WinDesc {
    int32_t kind;         // FW_WIN_*
    int32_t n_slices;     // HOP slices per window
    int64_t size;         // window size / cumulate max size
    int64_t interval;     // slice size (getSliceEndInterval)
    int64_t offset;
    UDiv slice_div;       // divisor = interval
    UDiv size_div;        // divisor = size (CUMULATE getWindowStart)
    UDiv32 slice_div32;   // divisor = interval, for the 32-bit fast path
    int32_t fast32;       // interval < 2^30 and |offset| < 2^61: rows near a chunk base use 32-bit math
    int32_t ds;           // DataStream WindowOperator: per-window state (KIND_DSWIN)
    TzTable tz;           // SQL shift time zone (device pointers); tz.n == 0: UTC
    // DataStream: windows are [start, start + size) with start on the slide grid; a pane (slice)
    // of `interval` ms belongs to n_win consecutive windows (1 for tumbling)
    int64_t slide;
    int64_t lateness;     // allowedLateness (cleanupTime = maxTimestamp + lateness, saturating)
    UDiv slide_div;
    int32_t n_win;
    // SQL HOP with block state (k_merge_hopb): one entry per (key, block of HB_R slices)
    int32_t hopb;
    int64_t hb_span;      // HB_R * interval
    UDiv hb_span_div;
};

// merge/fire kernel variant of a handle: the SQL window kinds, or DataStream windows
constexpr int KIND_DSWIN = 3;
constexpr int KIND_HOPB = 4;  // SQL HOP, block state (fw_merge_hopb.h)
constexpr int HB_R = 8;       // slices per HOP block entry
// Narrow HOP block entries (k_merge_hopb write-back, per superbucket: every slot word with data fits
// the level's width and every block start is (block index) * hb_span + offset with a block index
// below 2^31): key (8 B), block index (4 B), flags (2 B: F_ACC | slot mask << 8), then the HB_R * nw
// slot words as int32 (level 1) or int16 (level 2), zero-padded to whole 8-byte words.  A slot
// without data -- its mask bit clear -- holds the word's identity, restored on load.  One
// accumulator word: 11 words wide, 6 at level 1, 4 at level 2; two: 19, 10, 6.
constexpr int HB_LEVELS = 3;  // 0: wide (3 + HB_R * nw words), 1: int32 slots, 2: int16 slots
constexpr int HB_HDR_BYTES = 14;  // narrow entry header: key, block index, flags
constexpr int hb_slot_bytes(int level) { return level == 1 ? 4 : 2; }
constexpr int hb_narrow_words(int nw, int level = 1) { return (HB_HDR_BYTES + hb_slot_bytes(level) * HB_R * nw + 7) / 8; }
constexpr uint32_t HB_MASK_SHIFT = 8;  // block entry flag bits 8.. : slot i holds data

// TimeWindowUtil.isWindowFired in the window's shift zone (UTC when tz.n == 0)
FW_HD bool win_fired(const WinDesc& w, int64_t we, int64_t progress) {
    if (w.tz.n == 0) return is_fired(we, progress);
    return tz_is_fired(w.tz, we, progress);
}

// ---- DataStream windows of a pane (WindowOperator over Tumbling/SlidingEventTimeWindows)
// end of the latest window holding pane `pe` (SlidingEventTimeWindows.assignWindows :77-90:
// lastStart = getWindowStartWithOffset(ts, offset, slide), windows down to start > ts - size)
FW_HD int64_t ds_first_window_end(const WinDesc& w, int64_t pe) {
    if (w.n_win == 1) return pe;
    const int64_t ts0 = wsub(pe, w.interval);  // the pane's first millisecond
    return wadd(window_start(ts0, w.offset, w.slide_div), w.size);
}
// does the window ending at e hold pane pe?  SlidingEventTimeWindows.assignWindows' loop condition
// start > timestamp - size for the pane's last millisecond (the windows of a pane are e0, e0 - slide,
// ...: n_win = ceil(size / slide) candidates, the last one outside the pane when slide does not
// divide size)
FW_HD bool ds_window_holds_pane(const WinDesc& w, int64_t e, int64_t pe) {
    return wsub(e, w.size) > wsub(wsub(pe, 1), w.size);
}
// WindowOperator.cleanupTime (:670-677) of the window ending at we: maxTimestamp + lateness,
// Long.MAX_VALUE on overflow (then no cleanup timer is registered, registerCleanupTimer :616-628)
FW_HD int64_t ds_cleanup_time(const WinDesc& w, int64_t we) {
    const int64_t mt = wsub(we, 1);
    const int64_t ct = wadd(mt, w.lateness);
    return ct >= mt ? ct : INT64_MAX;
}

FW_HD int64_t slice_end_of(const WinDesc& w, int64_t ts) {
    return wadd(window_start(ts, w.offset, w.slice_div), w.interval);
}
// SliceAssigner.getWindowStart(windowEnd)
FW_HD int64_t window_start_of(const WinDesc& w, int64_t we) {
    if (w.kind == FW_WIN_CUMULATE) return window_start(wsub(we, 1), w.offset, w.size_div);
    return wsub(we, w.size);
}
// SliceAssigner.getLastWindowEnd(sliceEnd)
FW_HD int64_t last_window_end_of(const WinDesc& w, int64_t se) {
    if (w.kind == FW_WIN_TUMBLE) return se;
    if (w.kind == FW_WIN_HOP) return wadd(wsub(se, w.interval), w.size);
    return wadd(window_start_of(w, se), w.size);
}
// sliceStateMergeTarget (SliceSharedSyncStateWindowAggProcessor.java:120-132)
FW_HD int64_t merge_target_of(const WinDesc& w, int64_t se) {
    if (w.kind == FW_WIN_CUMULATE) return wadd(window_start_of(w, se), w.interval);
    return se;
}

// Superbuckets are the unit of state: each is one merge workgroup's LDS table.  The ingest kernel
// partitions its partials by ingest superbucket = superbucket >> pass_log2 (its LDS histogram holds
// IG_MAX_SB of them), so beyond IG_MAX_SB superbuckets the 2^pass_log2 superbuckets of one ingest
// superbucket share its partial rows and each merge pass keeps the rows that route to its own.
struct KeySpace {
    int32_t hash_kind;
    int32_t max_p;
    int32_t kg_start;      // first key group owned by this subtask
    int32_t n_kg;          // key groups owned
    int32_t sb_per_kg_log2;
    int32_t n_sb;          // superbuckets = n_kg << sb_per_kg_log2
    UDiv32 maxp_div;       // divisor max_p
    int32_t pass_log2;     // superbuckets per ingest superbucket (log2); 0 unless n_sb > IG_MAX_SB
    int32_t pad;
};

// Routing of one key: m = MathUtils.murmurHash(key.hashCode()) (>= 0), key group = m % maxP
// (KeyGroupRangeAssignment.computeKeyGroupForKeyHash), and the build's own sub-bucket inside
// the key group from the quotient bits m / maxP (uniform, since m is a murmur hash).
// `kind` overrides ks.hash_kind with a compile-time constant where the caller resolved it.
FW_HD int32_t route_key(const KeySpace& ks, int64_t key, int32_t pre, uint32_t* m_out, int32_t kind = -1) {
    const uint32_t m = (uint32_t)flink_murmur_hash(java_key_hash(kind >= 0 ? kind : ks.hash_kind, key, pre));
    const uint32_t q = udiv32(m, ks.maxp_div);
    const int32_t kg = (int32_t)(m - q * (uint32_t)ks.max_p);
    const uint32_t sub = q & ((1u << ks.sb_per_kg_log2) - 1u);
    *m_out = m;
    return ((kg - ks.kg_start) << ks.sb_per_kg_log2) + (int32_t)sub;
}
FW_HD int32_t superbucket_of(const KeySpace& ks, int64_t key, int32_t pre) {
    uint32_t m;
    return route_key(ks, key, pre, &m);
}

struct WordDesc {
    int32_t nw;
    int32_t op[MAX_WORDS];
    int32_t col[MAX_WORDS];   // value slot the word reads
    int32_t gate[MAX_WORDS];  // value slot whose NULL rows the word skips, -1: none (COUNT(*))
    int32_t qfirst[MAX_WORDS];  // W_QNANLO / W_QMIN / W_QMAX: the W_QFIRST word of its group
    int32_t has_q;            // any W_Q* word (write-back normalisation, fire-time merges)
    int32_t has_ord;          // any word that reads an arrival ordinal (W_Q*, W_FIRST, W_DN*)
};

// Compile-time accumulator layout of a k_merge_fire variant: 4 bits per word (word 0 lowest),
// the word's merge class -- W_SUM_I (integer add: also COUNT words), W_SUM_F, W_MIN_I (also
// MIN_D), W_MAX_I (also MAX_D) -- or OPS_NONE past the last word.  Inside the merge a word is
// only ever folded, merged and reset to its identity, and those agree within a class, so a
// variant with the layout as a constant folds the per-word op switches away.  OPS_ANY: the
// layout is read from the WordDesc at run time.
constexpr uint32_t OPS_ANY = 0xFFFFFFFFu;
constexpr uint32_t OPS_NONE = 15u;
constexpr uint32_t ops_pack(std::initializer_list<int32_t> ops) {
    uint32_t l = 0xFFFFFFFFu;
    int w = 0;
    for (int32_t o : ops) {
        l &= ~(15u << (4 * w));
        l |= (uint32_t)o << (4 * w);
        w++;
    }
    return l;
}
// the layout of a WordDesc, OPS_ANY when a word is outside the four classes (SQL DOUBLE MIN/MAX)
inline uint32_t ops_layout(const WordDesc& wd) {
    if (wd.has_q || wd.nw > MAX_WORDS) return OPS_ANY;
    uint32_t l = 0;
    for (int w = 0; w < MAX_WORDS; w++) {
        uint32_t c = OPS_NONE;
        if (w < wd.nw) {
            switch (wd.op[w]) {
                case W_CNT: case W_CNTV: case W_SUM_I: c = W_SUM_I; break;
                case W_SUM_F: c = W_SUM_F; break;
                case W_MIN_I: case W_MIN_D: c = W_MIN_I; break;
                case W_MAX_I: case W_MAX_D: c = W_MAX_I; break;
                default: return OPS_ANY;
            }
        }
        l |= c << (4 * w);
    }
    return l;
}

struct AggDesc {
    int32_t n;
    int32_t kind[FW_MAX_AGGS];
    int32_t type[FW_MAX_AGGS];
    int32_t w0[FW_MAX_AGGS];
    int32_t w1[FW_MAX_AGGS];  // AVG count word
    int32_t nn[FW_MAX_AGGS];  // word whose value 0 makes SUM / MIN / MAX NULL, -1: never
    int32_t qf[FW_MAX_AGGS];  // SQL MIN/MAX(DOUBLE): W_QFIRST, W_QNANLO, W_QZERO words (else -1)
    int32_t qn[FW_MAX_AGGS];
    int32_t qz[FW_MAX_AGGS];
    int32_t count_star_word;  // word of the SQL indexOfCountStar aggregate, -1 if none
    int32_t dn_hi[FW_MAX_AGGS];  // DataStream MIN/MAX(DOUBLE): the W_DNHI / W_DNLO words (else -1)
    int32_t dn_lo[FW_MAX_AGGS];
    int32_t first_word;       // DataStream: the W_FIRST word (-1: the first element is not tracked);
                              // minBy / maxBy: the arg's W_BYO_* word
    int32_t by_prev;          // minBy / maxBy: the W_BYPREV word (-1: not a minBy / maxBy layout)
};

constexpr int CS_WORDS = 12;  // IngestArgs::chunk_stats words per chunk
struct IngestArgs {
    const int64_t* key;
    const int64_t* ts;
    const int32_t* khash;
    const uint64_t* vals[MAX_KCOLS];
    const uint8_t* nulls[MAX_KCOLS];  // null flags per value slot (nullptr: NOT NULL column)
    int64_t n;
    WinDesc win;
    KeySpace ks;
    WordDesc wd;
    int32_t nv;            // value columns loaded
    Ctrl* ctrl;
    uint64_t* parts;       // partial buffer: FW_MAX_PENDING slots of cap_rows * (2 + nw) words;
                           // chunk c owns rows [c*CH, (c+1)*CH) of its slot, sorted by superbucket
    int64_t cap_rows;      // rows per slot (>= rows of one push)
    uint32_t* cells;       // [FW_MAX_PENDING][max_nch / 16][n_sb][16] (cell_index): start | count << 16
                           // of each (superbucket, chunk) cell inside the chunk's region
    int32_t* slot_nch;     // [FW_MAX_PENDING] chunks of each pending push
    int64_t max_nch;       // cell_pad(chunks per slot): cells per superbucket per slot
    int64_t* chunk_stats;  // [n_chunks][CS_WORDS]: min target slice, dropped rows, accepted rows, partials,
                           // partial bytes | compact << 40, -, -, -, key min / max, accumulator min / max
    Tickets* tickets;
    int64_t n_chunks;
    int64_t* treq;         // timer requests: (key, window, sb) triples
    int64_t treq_cap;
    int32_t lds_bytes;     // dynamic LDS of the launch (IG_LDS)
    int32_t local;         // LOCAL phase: no late-record handling (LocalSlicingWindowAggOperator)
    int32_t global;        // GLOBAL phase: the ts column holds the slice end (SliceAssigners.sliced)
    int32_t ablate;        // development only (FW_ABLATE env): skip phases to time the others
    // DataStream lateness: rows that fire an already fired window (late-fire rows) and rows sent
    // to the late side output
    uint64_t* lfire;       // [lfire_cap][3 + MAX_WORDS]: key, pane end, sb | ord << 32, words
    int64_t lfire_cap;
    int64_t* side;         // [side_cap][3 + nv]: key, ts, push_seq << 32 | row, value slots
    int64_t side_cap;
    int32_t side_output;   // late side output instead of numLateRecordsDropped
    int32_t push_seq;      // fw_commit / fw_push_device call number (side-output rows)
    int64_t row0;          // row offset of this launch within its call
    int32_t fold_always;   // development (FW_FOLD=1): fold every push (no adaptive skip)
    int32_t no_fold;       // minBy / maxBy: word pairs do not fold per word -- partials stay per element
    const int64_t* seg_counts;  // padded exchange buffer: valid rows per segment (nullptr: all valid)
    UDiv seg_div;          // divisor = segment length
    unsigned long long* kt;  // launch timing (fw_set_profiling FW_PROF_DEVICE): KtSlot of this kernel class
    int64_t stride;        // words between consecutive rows of a key / ts / value column (1: plain
                           // columns; 2 + value columns: the packed rows of fw_push_device_packed_segments)
    // compact partial rows (PF_*): 0 always PF_WIDE, 1 PF_NARROW allowed, 2 PF_UNIT too (COUNT(*) only)
    int32_t narrow;
    int64_t rank_lim;      // span of the ranks in ms: min(PF_MAX_RANK + 1, (2^31 - 1) / interval) * interval
    int64_t* slot_base;    // [FW_MAX_PENDING]: rank base of each push (its last workgroup writes it)
    uint8_t* ranks;        // [FW_MAX_PENDING][cap_rows]: rank byte of each narrow row
    // runs (nullptr: every chunk keeps its rows in its own region, the cells tell where)
    uint64_t* runs;        // [FW_MAX_PENDING][run_rows] rows, at the push format's stride
    uint8_t* run_ranks;    // [FW_MAX_PENDING][run_rows]: rank bytes of compact run rows
    uint32_t* run_fill;    // [FW_MAX_PENDING][RUN_X][n_isb]: rows claimed in each sub-run (may exceed sub_cap)
    uint32_t* run_ovf;     // [FW_MAX_PENDING][n_isb]: a chunk left rows of this superbucket in its region
    int32_t* slot_fmt;     // [FW_MAX_PENDING]: the run rows' format (PF_*) of each push
    int64_t run_rows;      // rows per slot: n_isb * RUN_X * sub_cap
    int32_t sub_cap;       // rows per sub-run
    int32_t pack;          // PF_PACK run rows allowed (runs, one integer word; fw_api.hip plans it)
};
// Development ablations and phase stamps (FW_ABLATE) are compiled into the kernels only in a
// diagnostic build (make DIAG=1): in the production build their checks fold away, so the hot loops
// carry no scalar branches for them.
#ifndef FW_DIAG
#define FW_DIAG 0
#endif
#define FW_ABL(a) (FW_DIAG ? (a).ablate : 0)
constexpr int AB_NO_FOLD = 1;    // skip the LDS fold
constexpr int AB_NO_SORT = 2;    // skip rank/scan/cells; store partials at their row position
constexpr int AB_NO_STORE = 4;   // skip the partial stores
constexpr int AB_M_NO_GATHER = 8;    // merge: skip reading/merging the pending partials
constexpr int AB_M_NO_FIRE = 16;     // merge: skip the fire rounds
constexpr int AB_M_NO_WB = 32;       // merge: skip the state write-back
constexpr int AB_M_NO_LOAD = 64;     // merge: skip loading the state into LDS
constexpr int AB_STAMPS = 128;       // merge: accumulate per-phase s_memtime cycles (diagnostic)
constexpr int AB_M_NO_HASH = 512;    // merge: gather loads the partials but does not insert them
constexpr int AB_M_NO_FOLDOP = 1024; // merge: insert the partials but skip the accumulator/flag atomics
constexpr int AB_GSTAMPS = 256;      // merge: with AB_STAMPS, stamps 2/4/7 = thread 0 gather loads/probe/fold
constexpr int AB_M_NO_EMIT = 4096;  // merge: fire without writing result rows (diagnostic)
constexpr int AB_FSTAMPS = 8192;    // merge: per-lane cycles of fire_one's parts into stamps[8..11]
constexpr int AB_IG_LINEAR = 16384;  // ingest (runs): store every staged row at its chunk position (no scatter)
constexpr int AB_IG_NO_GSTORE = 32768;  // ingest: stage the rows in LDS but issue no global store
constexpr int N_STAMPS = 16;

struct MergeArgs {
    KeySpace ks;             // routing of a partial row's key (ks.pass_log2 > 0: rows of other superbuckets are skipped)
    Ctrl* ctrl;
    Tickets* tickets;
    const uint64_t* parts;
    const uint32_t* cells;   // see IngestArgs
    const int32_t* slot_nch;
    int64_t max_nch;
    int64_t cap_rows;
    const int64_t* treq;
    uint64_t* state;         // [n_sb][cap_e][3 + nw] words: key, slice, flags, acc...
    int32_t* state_count;    // live entries per superbucket
    int64_t* sb_min_timer;   // min windowEnd with a timer per superbucket (INT64_MAX: none)
    uint8_t* sb_nar;         // HOP block state: the superbucket's layout level (0 wide, 1 / 2 narrow: hb_narrow_words)
    int32_t hb_narrow;       // HOP block state: the narrowest layout level a write-back may choose (0..2)
    int32_t n_sb;
    int32_t cap_e;
    WinDesc win;
    WordDesc wd;
    AggDesc ad;
    int32_t always_flush;    // DataStream: state is updated per record, flush every advance
    int32_t local;           // LOCAL phase: emit every gathered (key, slice) partial, keep no state
    int32_t chunk_rows;      // rows per ingest chunk (IG_BLOCK * ig_rpt): the cells' row stride
    int64_t* out_key;        // output slabs: [n_sb][slab_cap] rows, then out_cap overflow rows
    int64_t* out_we;
    uint64_t* out_val[FW_MAX_AGGS];
    uint32_t* out_null;
    int32_t* sb_out;         // rows in each superbucket's slab
    uint32_t* sb_fired;      // fired timers per superbucket (cumulative)
    int64_t slab_cap;
    int64_t out_cap;         // overflow rows
    int64_t wm;              // watermark of this advance
    const int64_t* wm_dev;   // (fw_advance_device) the watermark in device memory instead of wm
    int32_t force_flush;     // prepareCheckpoint: flush, no timers
    int32_t reset_out;       // the results were consumed (fw_results_reset): emit from slab row 0
    int32_t ablate;          // development only (FW_ABLATE)
    unsigned long long* stamps;  // [N_STAMPS] phase cycles summed over workgroups (AB_STAMPS)
    const uint64_t* lfire;   // DataStream late-fire rows (IngestArgs::lfire)
    int64_t lfire_cap;
    // host-mapped word the launch's last workgroup sets to merge_seq << 8 | pending pushes after
    // the launch: the host learns how full the partial buffer is without a stream sync
    unsigned long long* host_mirror;
    uint64_t merge_seq;
    unsigned long long* kt;  // launch timing (fw_set_profiling FW_PROF_DEVICE): KtSlot of this kernel class
    // DataStream first-element tracking (AggDesc::first_word >= 0): retain events (the ordinal of a
    // new window state's first element) and release events (ORDEV_RELEASE | ordinal of a cleaned
    // window's first element), for the host shim that keeps those records (value1 of the reduce)
    int64_t* ordev;
    int64_t ordev_cap;
    const int64_t* slot_base;   // compact partial rows (IngestArgs)
    const uint8_t* ranks;
    int32_t ch_log2;            // log2(chunk_rows)
    int32_t compact;            // chunks may hold compact rows (IngestArgs::narrow != 0)
    // runs (IngestArgs); the merge zeroes a flushed push's fill counters and overflow flags
    const uint64_t* runs;
    const uint8_t* run_ranks;
    uint32_t* run_fill;
    uint32_t* run_ovf;
    const int32_t* slot_fmt;
    int64_t run_rows;
    int32_t sub_cap;
};
constexpr int64_t ORDEV_RELEASE = (int64_t)1 << 62;
constexpr int LFW = 3 + MAX_WORDS;  // words per late-fire row
constexpr int SOW = 3 + MAX_KCOLS;  // words per late side-output row

struct CompactArgs {
    Ctrl* ctrl;
    const int32_t* sb_out;
    int64_t* off;            // [n_sb + 2]
    int32_t n_sb;
    int32_t n_aggs;
    int64_t slab_cap;
    const int64_t* out_key;
    WinDesc win;             // window_start = window_start_of(window_end) (LOCAL phase: = window_end)
    int32_t local_out;
    const int64_t* out_we;
    const uint64_t* out_val[FW_MAX_AGGS];
    const uint32_t* out_null;
    int64_t* res_key;
    int64_t* res_ws;
    int64_t* res_we;
    uint64_t* res_val[FW_MAX_AGGS];
    uint32_t* res_null;
    int64_t res_cap;
    int64_t* host_n;         // fw_results_async: also store the row count here (mapped host memory)
};

// host staging buffers of fw_reserve / fw_commit (pinned host + device): batch b + 1 is filled while
// batch b crosses PCIe.  (3 measured neutral on the end-to-end leg, which is PCIe-bound: CFG2 2.25 ->
// 2.27 ms per step, the wait for the staging buffer moving to the wait for the rows)
constexpr int FW_STAGE_BUFS = 2;

// fw_results_async buffers: up to this many collections outstanding (fw_results_ready reads the
// oldest), so a caller can read watermark b - 2's rows while b - 1's and b's are still in flight
constexpr int FW_AR_BUFS = 3;

// fw_results_async with kernel delivery (FW_AR_KERNEL=1): the compacted rows copied by CU stores into
// mapped pinned host memory (runs beside the H2D of the next batch, which occupies the DMA engine)
struct CopyOutArgs {
    const int64_t* d_n;      // rows (the compaction's total, device)
    int32_t n_aggs;
    int64_t cap;
    const int64_t* src_key;
    const int64_t* src_ws;
    const int64_t* src_we;
    const uint64_t* src_val[FW_MAX_AGGS];
    const uint32_t* src_null;
    int64_t* dst_key;
    int64_t* dst_ws;
    int64_t* dst_we;
    uint64_t* dst_val[FW_MAX_AGGS];
    uint32_t* dst_null;
};
hipError_t launch_copy_out(const CopyOutArgs& a, hipStream_t s);

// fw_commit_delta32: transfer columns of 32-bit deltas widened on the device into the 8-byte words the
// ingest reads (word = base + delta, modulo 2^64).  Column slot c of a launch: src[c] -> dst[c].
constexpr int FW_PACK_COLS = 2 + FW_MAX_COLS;  // key, ts, value columns
struct WidenArgs {
    int64_t n;
    const uint32_t* src[FW_PACK_COLS];
    uint64_t* dst[FW_PACK_COLS];
    uint64_t base[FW_PACK_COLS];
};
hipError_t launch_widen(const WidenArgs& a, int n_cols, hipStream_t s);

// In-kernel launch timing (fw_set_profiling FW_PROF_DEVICE): per kernel class 4 words -- the
// constant-rate device clock (s_memrealtime) when block 0 started the current launch, the summed
// launch durations, the launch count, spare.  Block 0 stamps the start; the last workgroup of the
// grid (the one the launch's ticket election picks, after every other workgroup has finished)
// adds now - start.  Unlike stream events this adds no work between launches.
constexpr int KT_WORDS = 4;

// Optional per-launch timing hook (fw_set_profiling FW_PROF_EVENTS): records hipEvents around launches.
struct KTimer {
    virtual void mark(int kind, bool end, hipStream_t s) = 0;
    virtual ~KTimer() = default;
};
inline void kt_mark(KTimer* t, int kind, bool end, hipStream_t s) {
    if (t) t->mark(kind, end, s);
}

// launchers (fw_kernels.hip)
hipError_t launch_compact(const CompactArgs& a, hipStream_t s, KTimer* t);
hipError_t launch_ingest(const IngestArgs& a, hipStream_t s, KTimer* t);
hipError_t launch_merge_fire(const MergeArgs& a, hipStream_t s, KTimer* t);
hipError_t launch_init_ctrl(Ctrl* c, hipStream_t s);
// key rows (fw_keyrows.hip)
int key_row_desc(const fw_key_field* fields, int32_t n_fields, KeyRowDesc* d);
hipError_t launch_kr_intern(const KeyRowTable& t, Ctrl* c, int64_t n, const int64_t* off, const uint8_t* bytes,
                            int64_t* out_id, int32_t* out_hash, hipStream_t s);
hipError_t launch_kr_collect(const KeyRowTable& t, Ctrl* c, const uint64_t* state, const int32_t* state_count,
                             const uint8_t* sb_nar, int32_t hb_nw,
                             int32_t n_sb, int32_t cap_e, int32_t pwe, int32_t pw, const uint64_t* parts,
                             int64_t cap_rows, const int64_t* treq, const int64_t* out_key, const int32_t* sb_out,
                             int64_t slab_cap, hipStream_t s);
hipError_t launch_kr_result_rows(const KeyRowTable& t, const int64_t* res_key, const int64_t* n_ptr, int64_t cap,
                                 int32_t* len, uint64_t* img, int32_t stride_words, hipStream_t s);

}  // namespace fw
