/*
 * flinkwin.h -- C-ABI of libflinkwin, the MI355X-native windowed keyed-aggregation
 * operator core that sits behind Flink's own window-operator seams.
 *
 * One fw_handle == one operator subtask (one Flink WindowAggOperator / WindowOperator
 * instance).  All calls on a handle must come from one thread (Flink's mailbox thread,
 * flink-runtime/.../tasks/mailbox/MailboxProcessor.java:58-91).  Every entry point
 * returns 0 on success and a negative FW_E_* code on failure; the message is then
 * available from fw_last_error() (thread-local).  No torch / HIP types appear here:
 * device buffers are plain pointers, streams are opaque void*.
 *
 * Reference interfaces each entry point replaces (paths relative to the Flink tree,
 * TR = flink-table/flink-table-runtime/src/main/java/org/apache/flink/table/runtime,
 * FR = flink-runtime/src/main/java/org/apache/flink):
 *
 *   fw_create        SlicingSyncStateWindowProcessor construction in
 *                    WindowAggOperatorBuilder.buildSlicingWindowProcessor
 *                    (TR/operators/aggregate/window/WindowAggOperatorBuilder.java:220-260)
 *                    + WindowProcessor.open (TR/operators/window/tvf/common/WindowProcessor.java:42);
 *                    DataStream: WindowOperatorBuilder.buildWindowOperator
 *                    (FR/streaming/runtime/operators/windowing/WindowOperatorBuilder.java:432-446)
 *   fw_initialize_watermark
 *                    WindowProcessor.initializeWatermark (WindowProcessor.java:48) /
 *                    InternalTimerServiceImpl.initializeWatermark
 *   fw_reserve/fw_commit(_delta32), fw_push_device
 *                    SyncStateWindowProcessor.processElement(key,row) -> dropped
 *                    (TR/operators/window/tvf/common/SyncStateWindowProcessor.java:37),
 *                    i.e. AbstractSliceSyncStateWindowAggProcessor.processElement :96-126
 *                    + RecordsWindowBuffer.addElement :81; DataStream WindowOperator.processElement
 *                    (FR/.../windowing/WindowOperator.java:293-447). Batched: one call per
 *                    columnar batch buffered between watermarks.
 *   fw_advance       WindowAggOperator.processWatermark (TR/.../tvf/common/WindowAggOperator.java:227)
 *                    = advanceProgress (flush, AbstractSliceSyncStateWindowAggProcessor.java:139)
 *                    + InternalTimerServiceImpl.tryAdvanceWatermark (FR/streaming/api/operators/
 *                    InternalTimerServiceImpl.java:328) -> onTimer -> fireWindow/clearWindow.
 *                    Results for W are produced before the call returns (the caller forwards W
 *                    afterwards, AbstractStreamOperator.java:700-702).
 *   fw_flush         prepareCheckpoint (WindowAggOperator.prepareSnapshotPreBarrier :268 ->
 *                    AbstractSliceSyncStateWindowAggProcessor.prepareCheckpoint :156)
 *   fw_snapshot/fw_restore
 *                    keyed-state + timer snapshot of the operator (HeapSnapshotStrategy /
 *                    InternalTimerServiceImpl.snapshotTimersForKeyGroup :360) and the union-list
 *                    watermark state (WindowAggOperator.java:183-206)
 *   fw_get_stats     numLateRecordsDropped (WindowAggOperator.java:101,164; WindowOperator.java:144)
 *   fw_assign_key_groups
 *                    KeyGroupRangeAssignment.assignToKeyGroup / computeOperatorIndexForKeyGroup
 *                    (FR/runtime/state/KeyGroupRangeAssignment.java:63-127) as used by
 *                    KeyGroupStreamPartitioner.selectChannel (FR/streaming/runtime/partitioner/
 *                    KeyGroupStreamPartitioner.java:55-65)
 *   fw_key_row_hash  BinaryRowDataKeySelector.getKey(row).hashCode() for VARCHAR / composite keys
 *                    (TR/keyselector/BinaryRowDataKeySelector.java:54 -> BinaryRowData.hashCode
 *                    :459 -> MurmurHashUtils.hashBytesByWords :70-170), feeding
 *                    FW_KEYHASH_PRECOMPUTED handles and partitioning
 *   fw_partition_by_dest
 *                    the keyBy exchange's record routing (ChannelSelectorRecordWriter.emit,
 *                    FR/runtime/io/network/api/writer/ChannelSelectorRecordWriter.java:54): rows
 *                    bucketed per destination subtask, ready for an RCCL all-to-all.
 */
#ifndef FLINKWIN_H_
#define FLINKWIN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FW_ABI_VERSION 10
#define FW_MAX_AGGS 8
#define FW_MAX_COLS 8

/* ---- error codes ---------------------------------------------------------------- */
#define FW_OK 0
#define FW_E_INVALID (-1)       /* bad argument / unsupported configuration            */
#define FW_E_DEVICE (-2)        /* HIP runtime error                                    */
#define FW_E_CAPACITY (-3)      /* a device table / buffer capacity was exceeded        */
#define FW_E_STATE (-4)         /* call not allowed in the current state               */
#define FW_E_NOMEM (-5)

/* ---- configuration ----------------------------------------------------------------- */
typedef enum {
    FW_API_SQL = 0,         /* Table/SQL slicing WindowAggOperator (window TVF aggregate) */
    FW_API_DATASTREAM = 1   /* DataStream WindowOperator + EventTimeTrigger (+ allowedLateness,
                               late side output)                                        */
} fw_api_kind;

typedef enum {
    FW_WIN_TUMBLE = 0,      /* SQL TUMBLE / DataStream TumblingEventTimeWindows         */
    FW_WIN_HOP = 1,         /* SQL HOP / DataStream SlidingEventTimeWindows (size%slide==0) */
    FW_WIN_CUMULATE = 2     /* SQL CUMULATE                                             */
} fw_window_kind;

typedef enum {
    FW_AGG_COUNT_STAR = 0,  /* COUNT(*)            Count1AggFunction                    */
    FW_AGG_COUNT = 1,       /* COUNT(col)          CountAggFunction (counts non-null)    */
    FW_AGG_SUM = 2,         /* SUM(col)            SumAggFunction / SumAggregator        */
    FW_AGG_MIN = 3,         /* MIN(col)            MinAggFunction / ComparableAggregator */
    FW_AGG_MAX = 4,         /* MAX(col)            MaxAggFunction / ComparableAggregator */
    FW_AGG_AVG = 5,         /* AVG(col)            AvgAggFunction                        */
    /* v7, DataStream only (record-shaped operators, ds_first_ordinals = 1): the ELEMENT with the
       extremal field (WindowedStream.minBy / maxBy :725-790, ComparableAggregator byAggregate
       :89-96, MinByComparator / MaxByComparator: Comparable.compareTo, Double.compareTo for
       DOUBLE); ties go to the first element, or to the last with FW_AGGF_LAST in flags.  The
       result's value column is the field (a NaN as the canonical NaN), fw_result.first_ord the
       element's arrival ordinal. */
    FW_AGG_MINBY = 6,
    FW_AGG_MAXBY = 7
} fw_agg_kind;
enum { FW_AGGF_LAST = 1 };  /* fw_agg_desc.flags: minBy / maxBy(field, first = false) */

/* Aggregation phase (TwoStageOptimizedWindowAggregateRule.java:80-109).  ONE: the slicing
   WindowAggOperator with AggCombiner.  LOCAL: LocalSlicingWindowAggOperator + LocalAggCombiner
   (LocalAggCombiner.java:69-97): no state, no timers; every flush emits one partial accumulator row
   per (key, sliceEnd).  GLOBAL: WindowAggOperator with GlobalAggCombiner (GlobalAggCombiner.java:77-110):
   input rows are local accumulators, folded with the aggregates' merge expressions. */
typedef enum {
    FW_PHASE_ONE = 0,
    FW_PHASE_LOCAL = 1,
    FW_PHASE_GLOBAL = 2
} fw_agg_phase;

typedef enum {
    FW_T_I64 = 0,           /* BIGINT / long                                            */
    FW_T_F64 = 1,           /* DOUBLE / double (values passed as IEEE-754 bits)          */
    FW_T_I32 = 2            /* INT / int, passed sign-extended in an int64 column; SUM
                               wraps at 32 bits, AVG result is INT                      */
} fw_value_type;

typedef enum {
    FW_KEYHASH_LONG = 0,         /* DataStream Long key: Long.hashCode = (int)(v ^ v>>>32)      */
    FW_KEYHASH_INT = 1,          /* DataStream Integer key: Integer.hashCode = v                */
    FW_KEYHASH_BINROW_BIGINT = 2,/* SQL key row (BIGINT): BinaryRowData.hashCode, 16-byte row  */
    FW_KEYHASH_BINROW_INT = 3,   /* SQL key row (INT):    BinaryRowData.hashCode, 16-byte row   */
    FW_KEYHASH_PRECOMPUTED = 4,  /* key column holds an opaque id; the Java hashCode of the real
                                    key is passed in the key_hash column (VARCHAR, composite)   */
    FW_KEYHASH_KEYROW = 5        /* v5, SQL: the key IS a key row (BinaryRowData image, any
                                    VARCHAR / composite key).  Pushes carry the images
                                    (fw_push_device_key_rows, or the key-row staging of
                                    fw_reserve); the handle interns them in an HBM table keyed by
                                    the image bytes (BinaryRowData.equals), routes by
                                    BinaryRowData.hashCode, and returns each result's key row   */
} fw_key_hash_kind;

typedef struct {
    int32_t kind;        /* fw_agg_kind                                   */
    int32_t input_col;   /* value column index (ignored for COUNT_STAR)   */
    int32_t type;        /* fw_value_type of the input column             */
    int32_t flags;       /* v7: FW_AGGF_LAST for MINBY / MAXBY, else 0    */
} fw_agg_desc;

typedef struct {
    int32_t abi_version;      /* must be FW_ABI_VERSION                                    */
    int32_t api;              /* fw_api_kind                                               */
    int32_t window_kind;      /* fw_window_kind                                            */
    int32_t key_hash;         /* fw_key_hash_kind                                          */
    int64_t size_ms;          /* TUMBLE size, HOP size, CUMULATE max size                  */
    int64_t slide_ms;         /* HOP slide, CUMULATE step (0 for TUMBLE)                   */
    int64_t offset_ms;        /* window offset (withOffset)                                */
    int32_t n_aggs;
    int32_t count_star_index; /* SQL indexOfCountStar: agg index whose value is COUNT(*),
                                 -1 if none (required for HOP, as in the reference)        */
    fw_agg_desc aggs[FW_MAX_AGGS];
    int32_t n_value_cols;
    int32_t value_col_types[FW_MAX_COLS];
    uint32_t nullable_cols;   /* bit c: value column c may hold SQL NULLs; every push then
                                 carries a null-flag column for it (SQL only)               */
    int32_t agg_phase;        /* fw_agg_phase (SQL only)                                    */
    int32_t max_parallelism;  /* number of key groups (pipeline.max-parallelism)           */
    int32_t parallelism;      /* operator parallelism p                                    */
    int32_t subtask_index;    /* this subtask: owns computeKeyGroupRangeForOperatorIndex   */
    int32_t device;           /* HIP device ordinal                                        */
    int32_t ds_first_ordinals;/* v5, DataStream: 1 = track each window's first element, the value1
                                 SumAggregator / ComparableAggregator copy into every output record
                                 (SumAggregator.java:66-76, ComparableAggregator.java:83-104): results
                                 carry its arrival ordinal (fw_result.first_ord) and
                                 fw_first_element_events tells the shim which records to keep    */
    int64_t state_capacity;   /* expected max live (key, slice) state entries (sizing hint) */
    int64_t max_batch_rows;   /* max rows per fw_commit / fw_push_device call              */
    int64_t output_capacity;  /* result rows kept between fw_results_reset calls           */
    /* ---- v4: lateness (DataStream) and shift time zones (SQL TIMESTAMP_LTZ) ---------------- */
    int64_t allowed_lateness_ms; /* DataStream WindowOperator allowedLateness (>= 0; SQL: 0).  A
                                    window fires at maxTimestamp and keeps its state until
                                    cleanupTime = maxTimestamp + lateness (WindowOperator.java
                                    :609-682); an element for a fired, not yet cleaned window
                                    fires it again at once (EventTimeTrigger.onElement)           */
    int32_t late_side_output;    /* DataStream: 1 = elements late for every window go to the late
                                    side output (fw_late_records; WindowOperator.sideOutput, the
                                    sideOutputLateData tag) instead of numLateRecordsDropped      */
    int32_t tz_use_dst;          /* TimeZone.getTimeZone(shiftTimeZone).useDaylightTime()          */
    int32_t tz_n;                /* SQL TIMESTAMP_LTZ rowtime: entries of the shift time zone's
                                    offset table (TimeWindowUtil.getShiftTimeZone); 0 = UTC       */
    int32_t key_row_max_bytes;   /* v5, FW_KEYHASH_KEYROW: largest key-row image (bytes, multiple
                                    of 8, <= 4096; 0 = 120).  A longer key row is a device error
                                    (the builder keeps such keys on the reference operator)       */
    const int64_t* tz_utc;       /* tz_n ascending UTC epoch ms, tz_utc[0] = INT64_MIN: offset
                                    tz_offset_ms[i] is in force from tz_utc[i] (ZoneRules
                                    .getOffset(Instant)); host memory, copied by fw_create        */
    const int64_t* tz_offset_ms;
} fw_config;

typedef struct fw_handle fw_handle;

/* Pinned host staging columns returned by fw_reserve (valid until fw_commit).
   Null flags are one byte per row, non-zero = SQL NULL: the layout of Flink's heap columnar
   vectors (AbstractHeapVector.isNull, a boolean[] per column).  A NULL row's value word is
   ignored.  nulls[c] is non-NULL exactly for the columns in fw_config.nullable_cols. */
typedef struct {
    int64_t* key;
    int64_t* ts;                       /* event time, epoch ms (rowtime)               */
    int32_t* key_hash;                 /* only for FW_KEYHASH_PRECOMPUTED              */
    int64_t* values[FW_MAX_COLS];      /* int64 or double bits, per value_col_types     */
    uint8_t* nulls[FW_MAX_COLS];       /* null flags of the nullable columns            */
    /* v5, FW_KEYHASH_KEYROW (key unused): row i's key row image -- the bytes of its
       BinaryRowData (the key projection's output, BinaryRowDataKeySelector.getKey) -- is
       key_row_bytes[key_row_offsets[i] .. key_row_offsets[i + 1]); offsets 8-byte aligned,
       key_row_offsets[0] = 0, at most key_row_bytes_cap bytes */
    int64_t* key_row_offsets;          /* n + 1 entries                                 */
    uint8_t* key_row_bytes;
    int64_t key_row_bytes_cap;
} fw_host_cols;

/* Window results: SQL rows are key ++ aggs ++ (window_start, window_end); DataStream
   records are the window's first element with the aggregated field set to values[0], record
   timestamp window.maxTimestamp() = window_end - 1.
   Arrival ordinal of an element: push_seq << 32 | row, push_seq counting fw_commit /
   fw_push_device* calls from 0 (continued across fw_restore*), row its index in that call. */
typedef struct {
    int64_t n;
    int64_t* key;
    int64_t* window_start;
    int64_t* window_end;
    int64_t* values[FW_MAX_AGGS];      /* per agg: int64, or double bits for DOUBLE results */
    uint32_t* null_mask;               /* bit a set => agg a is SQL NULL                */
    int64_t* first_ord;                /* v5, DataStream with ds_first_ordinals: arrival ordinal of
                                          the window's first element (value1), else NULL */
    /* v5, FW_KEYHASH_KEYROW: row i's key row image is key_row_bytes[i * key_row_stride ..
       + key_row_len[i]) (BinaryRowData.pointTo); key[] holds the handle's internal key ids */
    int32_t* key_row_len;
    uint8_t* key_row_bytes;
    int64_t key_row_stride;
} fw_result;

typedef struct {
    int64_t current_watermark;         /* operator currentWatermark / processor currentProgress */
    int64_t next_trigger_progress;
    int64_t num_late_records_dropped;
    int64_t live_state_entries;
    int64_t pending_rows;              /* rows buffered (not yet flushed into state)    */
    int64_t results_available;
    int64_t num_fired_windows;         /* numFiredTimers analogue                       */
    int64_t partials_emitted;          /* partial (key, slice) aggregates written by ingest */
    int32_t error_flags;               /* FW_ERRF_* bits raised by the device since create / restore */
    int32_t num_superbuckets;
    /* v5: merge traffic counters (cumulative, device-side): measurement of the flush kernel */
    int64_t flush_launches;            /* fw_advance / flush launches that merged pending partials */
    int64_t partials_merged;           /* partial rows those flushes read                */
    int64_t state_entries_moved;       /* state entries loaded + written back by merge launches */
    /* v5, FW_KEYHASH_KEYROW: key rows in the intern table (ids handed out and not collected) */
    int64_t key_rows;
    int64_t key_row_collections;       /* collections of unreferenced key rows so far    */
    /* v6: partial-row traffic (cumulative, device-side) */
    int64_t partial_bytes_written;     /* bytes of partial rows (+ rank bytes) the ingest wrote */
    int64_t partial_bytes_merged;      /* of those, the bytes flushes have read          */
    int64_t compact_chunks;            /* ingest chunks written in a compact row format  */
    /* v9: state sizing -- the most (key, slice) entries one superbucket held in a merge since create /
       restore, against the entries a superbucket's table holds (FW_ERRF_STATE beyond it).  The peak
       over the capacity hint's superbuckets tells how much of the hint a stream really uses. */
    int64_t peak_superbucket_entries;
    int32_t superbucket_capacity;
    int32_t reserved_stats0;
} fw_stats;

/* ---- lifecycle ------------------------------------------------------------------- */
int fw_create(const fw_config* cfg, fw_handle** out);
int fw_destroy(fw_handle* h);
const char* fw_last_error(void);
int fw_abi_version(void);
/* Number of visible HIP devices (hipGetDeviceCount); 0 when the runtime finds none or fails.  The
 * JNI binding's FlinkWin.deviceCount() uses it for available(). */
int fw_device_count(void);
/* hipStream_t of the handle, as void* (so a caller can order its own work with it). */
void* fw_get_stream(fw_handle* h);
int fw_sync(fw_handle* h);

int fw_initialize_watermark(fw_handle* h, int64_t watermark);

/* ---- ingest ------------------------------------------------------------------------ */
int fw_reserve(fw_handle* h, int64_t n, fw_host_cols* out);
int fw_commit(fw_handle* h, int64_t n);
/* v9: fw_commit with narrow transfer columns.  For each column named in delta_cols the caller wrote n
   uint32 deltas into the first 4n bytes of its fw_reserve staging column; the column's 8-byte word of
   row i is bases[slot] + delta_i (modulo 2^64), slot 0 the key, 1 the ts, 2 + c value column c.  The
   deltas cross PCIe (half the bytes) and a device kernel widens them behind the copy, so the ingest
   sees the same words as fw_commit's.  A JNI shim packs a column of a batch whose values span
   < 2^32 (event times of one watermark interval; INT keys; bounded BIGINT ids) with bases[slot] its
   minimum, and writes the others as words.  Returns FW_E_INVALID for a slot the operator does not
   have (key-row operators have no key column). */
#define FW_DELTA_KEY 1u
#define FW_DELTA_TS 2u
#define FW_DELTA_VALUE(c) (4u << (c))
int fw_commit_delta32(fw_handle* h, int64_t n, uint32_t delta_cols, const int64_t* bases);
/* v9, host helper (no device work): dst[i] = src[i] - base as uint32, for a shim that packs a column
   in bulk; returns 1 if some value lies outside [base, base + 2^32) (that column then goes as
   words), else 0.  Slices of one column may be encoded from several threads with the same base. */
int fw_delta32_encode(const int64_t* src, int64_t n, int64_t base, uint32_t* dst);
/* Device-resident columns (caller-owned device memory, ordered on the handle stream).
   d_values[c] points at n 8-byte words of value column c; d_key_hash may be NULL unless
   key_hash == FW_KEYHASH_PRECOMPUTED; d_nulls may be NULL unless nullable_cols != 0, and then
   d_nulls[c] points at n null-flag bytes of each nullable column c.
   Every push is asynchronous until 8 pushes may be buffered and unflushed (the device buffer):
   the call then waits for the merge launches already issued to report (a host-mapped word),
   and only when none is outstanding reads the control block and flushes (the reference's
   RecordsWindowBuffer full path). */
int fw_push_device(fw_handle* h, int64_t n, const int64_t* d_key, const int64_t* d_ts,
                   const int32_t* d_key_hash, const void* const* d_values,
                   const uint8_t* const* d_nulls);

/* FW_KEYHASH_KEYROW: device-resident key row images (Arrow layout: row i's BinaryRowData image is
   d_key_row_bytes[d_key_row_offsets[i] .. d_key_row_offsets[i + 1]), offsets 8-byte aligned).  The
   key's identity in the window state is the image bytes (BinaryRowData.equals); its hashCode
   (MurmurHashUtils.hashBytesByWords, seed 42) routes it.  Otherwise as fw_push_device. */
int fw_push_device_key_rows(fw_handle* h, int64_t n, const int64_t* d_key_row_offsets, const uint8_t* d_key_row_bytes,
                            const int64_t* d_ts, const void* const* d_values, const uint8_t* const* d_nulls);

/* The receive buffer of a padded all-to-all (the keyBy exchange without a host round trip for
   the row counts): n_segs segments of seg_len rows, one per sending subtask; segment s holds
   d_seg_counts[s] valid rows (device int64, e.g. the counts all-to-all's result), the rest is
   padding and is never read.  Otherwise as fw_push_device. */
int fw_push_device_segments(fw_handle* h, int32_t n_segs, int64_t seg_len, const int64_t* d_seg_counts,
                            const int64_t* d_key, const int64_t* d_ts, const int32_t* d_key_hash,
                            const void* const* d_values, const uint8_t* const* d_nulls);

/* The receive buffer of the packed padded all-to-all (fw_partition_packed): n_segs segments of
   seg_len rows of row_words = 2 + n_value_cols int64 words each (key, ts, value columns in
   config order); segment s holds d_seg_counts[s] valid rows.  One buffer, one all-to-all per
   batch instead of one per column.  Not for FW_KEYHASH_PRECOMPUTED or NULL-able configurations
   (their extra columns travel with fw_push_device_segments). */
int fw_push_device_packed_segments(fw_handle* h, int32_t n_segs, int64_t seg_len, const int64_t* d_seg_counts,
                                   const int64_t* d_rows, int32_t row_words);

/* ---- progress / output --------------------------------------------------------------- */
/* Late side output of a DataStream operator with late_side_output (WindowOperator.sideOutput,
   WindowOperator.java:440-446,549): the elements skipped as late for every window since the last
   call, as columns.  push_seq counts fw_commit / fw_push_device calls from 0, row is the element's
   index in that call (so a host shim can forward its original record); values[c] holds the value
   columns the aggregates read (0 for the others).  Host arrays owned by the
   handle, valid until the next call; the rows are consumed. */
typedef struct {
    int64_t n;
    int64_t* key;
    int64_t* ts;
    int64_t* values[FW_MAX_COLS];
    int64_t* push_seq;
    int64_t* row;
} fw_late_rows;
int fw_late_records(fw_handle* h, fw_late_rows* out);

/* DataStream with ds_first_ordinals: which first elements the host shim must keep.  The reference
   keeps value1 inside the window state (HeapReducingState holds the reduced record); here the state
   holds only the aggregate and the first element's arrival ordinal, and the shim keeps the record.
   retain: ordinals of elements that became the first element of a window state that outlives the
   advance that created it (one event per window: an element of n sliding windows may be retained
   n times).  release: ordinals whose window state was cleared (cleanupTime, WindowOperator
   .clearAllState :494).  A window created and cleared within one advance is neither: its records
   are still the caller's pending batch.  Ordering for the shim, per advance: fw_results, then the
   retains (copy the records out of the pushed batches), resolve the results' first_ord, then the
   releases.  After fw_advance moves the watermark forward every pushed row has been flushed, so the
   pushed batches may be dropped once the events are read.  Host arrays owned by the handle, valid
   until the next call; the events are consumed. */
typedef struct {
    int64_t n_retain;
    int64_t* retain;
    int64_t n_release;
    int64_t* release;
} fw_ordinal_events;
int fw_first_element_events(fw_handle* h, fw_ordinal_events* out);

int fw_advance(fw_handle* h, int64_t watermark);
/* fw_advance with the watermark read from DEVICE memory (d_watermark[0]) by the merge launch when it
   runs on the handle's stream: the keyBy exchange's watermark valve (StatusWatermarkValve
   .inputWatermark, StatusWatermarkValve.java:153 -- the minimum over the input channels) is then an
   all-reduce on the device, and a step enqueues ingest and advance without waiting for its own GPU
   work.  The caller orders the handle's stream after the producer of d_watermark.  The host cannot
   skip watermarks that cross no slice end here (it does not know the value): the launch finds out on
   the device. */
int fw_advance_device(fw_handle* h, const int64_t* d_watermark);
int fw_flush(fw_handle* h);
/* copy_to_host != 0: host arrays owned by the handle, valid until the next call;
   otherwise device pointers. */
int fw_results(fw_handle* h, fw_result* out, int copy_to_host);
int fw_results_reset(fw_handle* h);
/* v6, pipelined emission (the shim's collector side of WindowAggOperator.onTimer ->
   output.collect, WindowAggOperator.java:227-238, and WindowOperator.emitWindowContents :568-575):
   fw_results_async queues the collection of every result row emitted since the last collection
   (compacted on the device into one of the handle's FW_AR_BUFS = 3 device buffers; only the row
   count goes to mapped host memory) and returns at once (the rows count as consumed, as after
   fw_results_reset); at most 3 collections may be outstanding (a 4th call fails with FW_E_STATE).
   fw_results_ready returns the OLDEST outstanding collection (v8; with one outstanding, as before,
   the last one): it waits for its rows to reach pinned host memory (a copy kernel queued behind the
   compaction stores them into mapped host memory, beside the next batch's H2D on the copy engine;
   FW_AR_KERNEL=0 moves them by hipMemcpyAsync on a D2H stream instead) and returns them as host
   arrays, valid until the third fw_results_async after their own.  So a caller emits watermark b's
   rows while batch b + 1 is ingested, or -- reading two collections behind -- while batches b + 1
   and b + 2 are ingested, which takes the collection off the caller's critical path.  Not for
   FW_KEYHASH_KEYROW operators (fw_results returns their key rows). */
int fw_results_async(fw_handle* h);
int fw_results_ready(fw_handle* h, fw_result* out);
/* v6, device-side consumers (the two-phase plan's LOCAL -> GLOBAL exchange): queues the collection
   of the rows emitted since the last collection into the handle's device result columns and
   returns their device pointers without waiting; the row count is the device int64 at *d_n and
   out->n is only its bound (output_capacity).  The rows count as consumed; read them on the
   handle's stream (fw_get_stream) or after it, before the next call that collects results. */
int fw_results_device(fw_handle* h, fw_result* out, int64_t** d_n);
/* v7, device-side consumers without a copy: the rows emitted since the last collection where the
   merge wrote them.  Segment s < n_segments - 1 (superbucket s) holds counts[s] rows at rows
   [s * seg_cap, s * seg_cap + counts[s]) of the columns in cols (device pointers; cols.n bounds
   the row index); the last segment, the shared overflow region, holds counts[n_segments - 1] rows
   from row (n_segments - 1) * seg_cap.  counts is a device int32 array written by the merge
   kernels, so read it (and the rows) on the handle's stream (fw_get_stream) or after it, before
   the next call that can run a merge (see FW_ERRF_OUTPUT below).  n_segments = 0 when nothing was emitted since the last
   collection.  The rows count as consumed.  fw_results / fw_results_device compact the same rows
   into one contiguous set (a copy of every row).
   v10: cols.window_start is NULL.  The merge stores no window start (8 B less per row); a row's
   start is SliceAssigner.getWindowStart(window_end): window_end - size for TUMBLE / HOP (and the
   DataStream assigners), getWindowStartWithOffset(window_end - 1, offset, size) for CUMULATE, and
   window_end itself for a LOCAL phase (its rows are slices).  fw_host_time_op(cfg, 4, we) computes
   it on the host; fw_results / fw_results_device fill window_start as before. */
typedef struct {
    int64_t n_segments;
    int64_t seg_cap;
    const int32_t* counts;
    fw_result cols;
} fw_result_segments;
int fw_results_device_segments(fw_handle* h, fw_result_segments* out);
/* fw_stats.error_flags bits.  fw_results / fw_results_device turn FW_ERRF_OUTPUT into FW_E_CAPACITY;
   fw_results_device_segments returns the rows it has (the overflow region's count is clamped to the
   output capacity), so a segments consumer checks error_flags (fw_get_stats) for FW_ERRF_OUTPUT.
   A segments consumer also finishes with the rows before ANY call that can run a merge: fw_advance,
   fw_advance_device, fw_flush, and every push (a push starts a flush by itself once the pending
   pushes fill the handle's FW_MAX_PENDING slots). */
#define FW_ERRF_CHUNKS 1      /* ingest chunk table over capacity                          */
#define FW_ERRF_STATE 2       /* state table full (FW_E_CAPACITY)                          */
#define FW_ERRF_OUTPUT 4      /* emitted rows over output_capacity: rows past it dropped  */
#define FW_ERRF_TREQ 8        /* timer request buffer over capacity                        */
#define FW_ERRF_KEYGROUP 16   /* a record's key group is outside this subtask's range      */
#define FW_ERRF_LATE 32       /* late-fire rows or late side-output rows over capacity     */
#define FW_ERRF_ORDEV 64      /* first-element retain / release events over capacity       */
#define FW_ERRF_KEYROW 128    /* key-row table full, or a key row over key_row_max_bytes   */
int fw_get_stats(fw_handle* h, fw_stats* out);

/* ---- per-kernel device timing (in-kernel clock stamps, or hipEvents around each launch) --- */
/* The reference has no per-kernel profiler for this path (flame graphs and latency
   markers only); this is the MI355X-side equivalent used by bench.py for the roofline figure. */
#define FW_KT_PARTITION 0   /* K1: key group -> superbucket row histogram per chunk            */
#define FW_KT_SCAN 1        /* exclusive scan of the [superbucket][chunk] histogram             */
#define FW_KT_REDUCE 2      /* K2+K3: slice assign + LDS segmented reduce + scatter of partials */
#define FW_KT_MERGE 3       /* K4+K5: merge partials into the HBM slice table + fire windows    */
#define FW_KT_OTHER 4       /* control-block / stats / compaction launches                      */
#define FW_KT_N 8
typedef struct {
    double ms[FW_KT_N];          /* accumulated device time per kernel class                 */
    int64_t launches[FW_KT_N];   /* timed launches per kernel class                          */
    int64_t merge_phase_cycles[FW_KT_N];  /* diagnostic builds only (FW_ABLATE stamps): shader
                                             cycles per merge phase, summed over workgroups     */
} fw_kernel_times;
/* FW_PROF_DEVICE times the ingest (FW_KT_REDUCE) and merge/fire (FW_KT_MERGE) launches inside the
   kernels: block 0 stamps the device's constant-rate clock at its start and the grid's last
   workgroup adds the launch's duration, so nothing is inserted into the stream between launches.
   FW_PROF_EVENTS times the same launches with hipEvents around them (each record costs the stream a
   few microseconds of idle time); FW_PROF_EVENTS_ALL also the small bookkeeping launches
   (FW_KT_OTHER).  0 stops timing.  Enabling resets the accumulators. */
#define FW_PROF_DEVICE 1
#define FW_PROF_EVENTS 2
#define FW_PROF_EVENTS_ALL 3
int fw_set_profiling(fw_handle* h, int enable);
/* synchronises the handle stream, then returns the accumulated times */
int fw_get_kernel_times(fw_handle* h, fw_kernel_times* out);

/* ---- checkpoint -------------------------------------------------------------------- */
/* Flushes, then serialises watermark + state + timers.  *size receives the byte count;
   call with buf == NULL to query it. */
int fw_snapshot(fw_handle* h, void* buf, int64_t capacity, int64_t* size);
int fw_restore(fw_handle* h, const void* buf, int64_t size);

/* Key-group-partitioned checkpoint, for restoring at a different parallelism (rescaling).
   fw_snapshot_key_group flushes, then serialises the live (key, slice) entries and timers of ONE
   owned key group; buf == NULL queries *size.  Replaces the heap backend's per-key-group state
   write (HeapSnapshotStrategy.java:97, AbstractStateTableSnapshot.writeStateInKeyGroup :112,
   InternalTimerServiceImpl.snapshotTimersForKeyGroup :360).  fw_restore_key_group adds such a blob
   to a handle whose key-group range (computeKeyGroupRangeForOperatorIndex, KeyGroupRangeAssignment
   .java:93-106) contains it (InternalTimerServiceImpl.restoreTimersForKeyGroup :406).  The operator
   watermark is union-list state restored as the min over all subtasks (WindowAggOperator.java
   :183-206): the blob carries its handle's watermark, and the caller passes the min to
   fw_initialize_watermark. */
int fw_snapshot_key_group(fw_handle* h, int32_t key_group, void* buf, int64_t capacity, int64_t* size);
int fw_restore_key_group(fw_handle* h, const void* buf, int64_t size);

/* v6: one key group in the HEAP keyed-state backend's own byte format, so a savepoint writer /
   reader on the Java side can move window state between this library and a heap-backend
   WindowAggOperator.  Layout (HeapSnapshotStrategy.java:161-172): writeInt(keyGroup), then per
   state in ascending id order writeShort(id) and
     window_state  ("window-aggs" ValueState, CopyOnWriteStateMapSnapshot.writeState :127-149):
                   writeInt(n), n x [namespace: 8 B big-endian slice end][key: writeInt(len) +
                   BinaryRowData bytes][accumulator: writeInt(len) + BinaryRowData bytes]
     event_timers  ("_timer_state/event_window-timers", KeyGroupPartitioner.java:241-254 +
                   TimerSerializer.serialize :147-152): writeInt(n), n x [writeLong(flipSignBit(
                   toEpochMillsForTimer(window - 1)))][key][namespace]
     processing_timers: writeInt(0).
   The accumulator row holds the aggregates' buffer fields in order (COUNT(*)/COUNT: BIGINT count;
   SUM/MIN/MAX: the aggregate's type, NULL-able; AVG: sum BIGINT|DOUBLE, count BIGINT) -- the
   LOCAL phase's output columns.  SQL ONE / GLOBAL phase with BINROW_BIGINT, BINROW_INT or KEYROW
   keys only.  HOP operators with block state export every slice with data and the
   timers the reference holds, except a chain timer at an EMPTY window (it fires without output);
   on restore they derive their timers from the data.  The restore side accepts the states in any
   order; restoring twice into one key group, or a key of another group, is an error. */
typedef struct {
    int16_t window_state;
    int16_t event_timers;
    int16_t processing_timers;
    int16_t reserved;
} fw_heap_state_ids;
int fw_snapshot_key_group_heap(fw_handle* h, int32_t key_group, const fw_heap_state_ids* ids, void* buf,
                               int64_t capacity, int64_t* size);
int fw_restore_key_group_heap(fw_handle* h, const void* buf, int64_t size, const fw_heap_state_ids* ids);

/* v7: the DataStream WindowOperator's keyed state of ONE key group, for a heap-backend savepoint
   of that operator: the "window-contents" reducing state (WindowOperatorBuilder.java:81; namespace
   TimeWindow.Serializer = start, end) and the "window-timers" event-time queue (WindowOperator.java
   :232, InternalTimerServiceImpl.snapshotTimersForKeyGroup :360 / restoreTimersForKeyGroup :406).
   The state's value is the user's record (value1 with the aggregated field set), so the operator
   shim writes the heap bytes (flink_amd/datastream/heap_state.py) from one fw_ds_window per (key,
   window end) that holds state or a timer: value = the field value (as fw_result reports it),
   first_ord = the arrival ordinal of the window's first element (the retained record), flags:
   CONTENTS (the window holds state), TRIGGER (timer at window.maxTimestamp()), CLEANUP (timer at
   cleanupTime(window); with allowedLateness 0 both timers are the same one).  fw_ds_snapshot_key_group
   flushes first; out == NULL queries *n.  fw_ds_restore_key_group adds a key group's windows to a
   handle owning it; restored first elements carry caller-chosen ordinals below push
   next_push_seq, after which the handle's arrival ordinals continue.  v8: key_hash -- for a
   FW_KEYHASH_PRECOMPUTED handle (keys the shim interns, e.g. String keys: key = the interned id,
   key_hash = String.hashCode) the key's hash, which routes the restored window exactly as the
   ingest routes the key's records; ignored for LONG / INT keys; 0 on snapshot: the state keeps no
   hash per entry (the shim knows its keys' hashes), so a caller that restores a snapshotted array
   into a FW_KEYHASH_PRECOMPUTED handle must fill key_hash back in first -- an unfilled array is
   refused (FW_E_INVALID) for every key whose hash 0 does not route to the key group. */
enum { FW_DSW_CONTENTS = 1, FW_DSW_TRIGGER = 2, FW_DSW_CLEANUP = 4 };
typedef struct {
    int64_t key;
    int64_t window_end;
    int64_t value;
    int64_t first_ord;
    int32_t flags;
    int32_t key_hash;     /* v8 (was reserved): FW_KEYHASH_PRECOMPUTED handles: the key's hash on restore */
} fw_ds_window;
int fw_ds_snapshot_key_group(fw_handle* h, int32_t key_group, fw_ds_window* out, int64_t capacity, int64_t* n);
int fw_ds_restore_key_group(fw_handle* h, int32_t key_group, const fw_ds_window* in, int64_t n, int64_t next_push_seq);

/* ---- key rows: VARCHAR / composite keys ------------------------------------------------ */
/* A key row field, as the key projection writes it into a BinaryRowData (BinaryRowWriter,
   TR/data/writer/BinaryRowWriter.java:39-122 + AbstractBinaryWriter.java:83-106,242-345).
   A FIXEDn field occupies the low n bytes of its 8-byte slot; a STRING field is UTF-8 text
   (VARCHAR / CHAR) or bytes (VARBINARY / BINARY). */
#define FW_MAX_KEY_FIELDS 8
typedef enum {
    FW_KF_STRING = 0,   /* VARCHAR, CHAR, VARBINARY, BINARY           writeString / writeBinary        */
    FW_KF_FIXED1 = 1,   /* BOOLEAN, TINYINT                           writeBoolean / writeByte         */
    FW_KF_FIXED2 = 2,   /* SMALLINT                                   writeShort                       */
    FW_KF_FIXED4 = 4,   /* INT, DATE, TIME(0-3), FLOAT (IEEE bits)    writeInt / writeFloat            */
    FW_KF_FIXED8 = 8    /* BIGINT, DOUBLE (bits), TIMESTAMP(0-3) millis, DECIMAL(p<=18) unscaled long   */
} fw_key_field_kind;
typedef struct {
    int32_t kind;              /* fw_key_field_kind                                          */
    int32_t reserved;
    const int64_t* fixed;      /* FIXEDn: one int64 per row (low n bytes used)               */
    const int32_t* offsets;    /* STRING: n + 1 byte offsets into bytes (Arrow layout)       */
    const uint8_t* bytes;      /* STRING: the bytes; base 4-byte aligned                      */
    const uint8_t* nulls;      /* NULL or 1 byte per row, non-zero = NULL (setNullAt)         */
} fw_key_field;
/* d_hash[i] = hashCode() of row i's key row (BinaryRowData.hashCode, BinaryRowData.java:459):
   the Java hash a FW_KEYHASH_PRECOMPUTED handle / fw_partition_by_dest routes by.  All pointers
   in fields are device pointers; the key's identity in the window state (the int64 key column
   pushed alongside) is the caller's, e.g. a dictionary id. */
int fw_key_row_hash(const fw_key_field* fields, int32_t n_fields, int64_t n, int32_t* d_hash, void* stream);
/* BinaryRowWriter's image of each key row (what BinaryRowDataKeySelector.getKey holds), written at
   d_offsets[i] of d_bytes (device pointers; d_offsets[i + 1] - d_offsets[i] must be the image
   length, fw_host_key_row_image_lengths).  The input of fw_push_device_key_rows. */
int fw_key_row_images(const fw_key_field* fields, int32_t n_fields, int64_t n, const int64_t* d_offsets,
                      uint8_t* d_bytes, void* stream);
/* host forms: image lengths (lens[i], bytes), images (host columns), and an image's hashCode */
int fw_host_key_row_image_lengths(const fw_key_field* fields, int32_t n_fields, int64_t n, int64_t* lens);
int fw_host_key_row_images(const fw_key_field* fields, int32_t n_fields, int64_t n, const int64_t* offsets,
                           uint8_t* bytes);
int32_t fw_host_key_row_image_hash(const uint8_t* image, int64_t len);

/* ---- stand-alone device kernels (partitioner, tests) ---------------------------------- */
/* d_kg[i] = key group, d_dest[i] = computeOperatorIndexForKeyGroup(maxP, p, kg). */
int fw_assign_key_groups(const int64_t* d_key, const int32_t* d_key_hash, int64_t n,
                         int32_t key_hash_kind, int32_t max_parallelism, int32_t parallelism,
                         int32_t* d_kg, int32_t* d_dest, void* stream);
/* Counting-sort rows by destination subtask.  d_counts[p] receives rows per destination;
   output columns are grouped by destination in ascending order, rows in input order within a
   destination. n_cols value columns.  d_key_hash is the Java key hash per row, required for
   FW_KEYHASH_PRECOMPUTED (e.g. from fw_key_row_hash) and ignored otherwise; a caller that needs
   it on the receiving side moves it as one of the value columns. */
int fw_partition_by_dest(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                         const void* const* d_values,
                         int32_t n_cols, int64_t n, int32_t key_hash_kind,
                         int32_t max_parallelism, int32_t parallelism,
                         int64_t* d_out_key, int64_t* d_out_ts, void* const* d_out_values,
                         int64_t* d_counts, void* d_workspace, int64_t workspace_bytes,
                         void* stream);
int64_t fw_partition_workspace_bytes(int64_t n, int32_t parallelism);
/* fw_partition_by_dest into the send buffer of a packed padded all-to-all: destination d's rows
   go to segment d of d_out_rows (seg_len rows of 2 + n_cols int64 words: key, ts, values), in
   input order, at most seg_len of them (d_counts[d] still counts all: the caller checks
   d_counts <= seg_len).  The segment padding is not written. */
int fw_partition_packed(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                        const void* const* d_values, int32_t n_cols, int64_t n, int32_t key_hash_kind,
                        int32_t max_parallelism, int32_t parallelism, int64_t seg_len, int64_t* d_out_rows,
                        int64_t* d_counts, void* d_workspace, int64_t workspace_bytes, void* stream);
/* v5: fw_partition_packed whose rows past a destination's seg_len are not dropped: they go to
   d_spill_rows (up to n rows of 2 + n_cols words), destination-major, each destination's in input
   order -- destination d's max(0, d_counts[d] - seg_len) rows follow those of destinations < d.
   The exchange sends them in an overflow round, so the segment size never has to bound a batch. */
int fw_partition_packed_spill(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                              const void* const* d_values, int32_t n_cols, int64_t n, int32_t key_hash_kind,
                              int32_t max_parallelism, int32_t parallelism, int64_t seg_len, int64_t* d_out_rows,
                              int64_t* d_spill_rows, int64_t* d_counts, void* d_workspace, int64_t workspace_bytes,
                              void* stream);
/* v6: fw_partition_packed_spill of the first *d_n (a device int64, <= n_max) rows: the batch's size
   is known only on the device, e.g. the LOCAL phase's partial rows of fw_results_device, so the
   two-phase exchange (TwoStageOptimizedWindowAggregateRule.java:80-109) needs no host round trip. */
int fw_partition_packed_spill_dn(const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                                 const void* const* d_values, int32_t n_cols, int64_t n_max, const int64_t* d_n,
                                 int32_t key_hash_kind, int32_t max_parallelism, int32_t parallelism, int64_t seg_len,
                                 int64_t* d_out_rows, int64_t* d_spill_rows, int64_t* d_counts, void* d_workspace,
                                 int64_t workspace_bytes, void* stream);
/* The device watermark valve (StatusWatermarkValve.java:153, the min over input channels) around one
   all-reduce (MAX) of three int64 words per subtask.  fw_valve_local writes this subtask's words:
   [d_counts[d] > cap for any destination d, ~watermark (bitwise NOT reverses the int64 order), the
   largest d_counts[d]] (parallelism <= 64).  After the all-reduce, fw_valve_select writes the valve's
   watermark: the previous one (*d_prev_watermark, or Long.MIN_VALUE when NULL) while any subtask's
   segments overflowed -- its overflow round must arrive before the watermark passes it -- else the
   minimum, ~agreed[1].  fw_advance_device reads it from device memory.  Both are stream-ordered and
   never wait on the host. */
int fw_valve_local(const int64_t* d_counts, int32_t parallelism, int64_t cap, int64_t watermark, int64_t* d_out3,
                   void* stream);
int fw_valve_select(const int64_t* d_agreed3, const int64_t* d_prev_watermark, int64_t* d_watermark, void* stream);

/* Synthetic Nexmark-shaped generator: event i in [i0, i0+n). */
typedef struct {
    uint64_t seed;
    int64_t t0_ms;
    int64_t rate_per_s;        /* events per second of event time                 */
    int64_t ooo_ms;            /* out-of-orderness J                              */
    int64_t key_base;
    int64_t key_count;
    int32_t key_dist;          /* 0 uniform: key_base + (u>>20) % key_count; 1 zipf    */
    int32_t value_kind;        /* 0: 1 + u % 1e9 (int64); 1: 1000*(u>>11)*2^-53 (double);
                                  2: u % 1e6 (int64)                                */
    const double* zipf_cdf;    /* device pointer, key_count entries (key_dist == 1) */
} fw_gen_params;
int fw_generate(const fw_gen_params* gp, int64_t i0, int64_t n, int64_t* d_key, int64_t* d_ts,
                int64_t* d_value, void* stream);

/* ---- host-side restatements (no device use): the same code the kernels run -------------- */
/* KeyGroupRangeAssignment.assignToKeyGroup on key.hashCode() as fw_key_hash_kind defines it. */
int32_t fw_host_key_group(int32_t key_hash_kind, int64_t key, int32_t precomputed_hash, int32_t max_parallelism);
/* Vector form for host-resident batches (the Java-side partitioner of host-staged records):
   kg[i] / dest[i] as fw_assign_key_groups computes them on the device. Either output may be NULL. */
int fw_host_assign_key_groups(const int64_t* key, const int32_t* key_hash, int64_t n, int32_t key_hash_kind,
                              int32_t max_parallelism, int32_t parallelism, int32_t* kg, int32_t* dest);
/* fw_key_row_hash over host-resident columns (the Java-side partitioner of host-staged records). */
int fw_host_key_row_hash(const fw_key_field* fields, int32_t n_fields, int64_t n, int32_t* hash);
/* TimeWindow.getWindowStartWithOffset (FR/streaming/api/windowing/windows/TimeWindow.java:264). */
int64_t fw_host_window_start(int64_t ts, int64_t offset, int64_t size);
/* TimeWindowUtil.getNextTriggerWatermark, UTC (TR/util/TimeWindowUtil.java:186). */
int64_t fw_host_next_trigger_watermark(int64_t watermark, int64_t interval);
/* Window / shift-zone arithmetic of an operator configuration (no device use): the plan
   fw_create makes from cfg and the code the kernels run.  what = 0 toUtcTimestampMills(x)
   (TimeWindowUtil.java:52), 1 toEpochMillsForTimer(x) (:69), 2 getNextTriggerWatermark(x, slice
   interval, useDaylightTime) (:186), 3 the slice end assigned to rowtime x
   (AbstractSliceAssigner.assignSliceEnd, SliceAssigners.java:655-670), 4 the window start of
   slice end x (SliceAssigner.getWindowStart).  *out receives the value; returns FW_E_INVALID for a
   configuration fw_create would reject. */
int fw_host_time_op(const fw_config* cfg, int32_t what, int64_t x, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* FLINKWIN_H_ */
