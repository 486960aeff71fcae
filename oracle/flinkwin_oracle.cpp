// ORACLE -- TEST INFRASTRUCTURE ONLY.
//
// A CPU restatement of Apache Flink's windowed keyed-aggregation semantics (reference tree
// mounted at /root/reference, Flink 2.3-SNAPSHOT), used ONLY by tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg as the checker.  The product (libflinkwin, flink_amd/) never
// links, imports or calls anything in this directory.
//
// It restates, record by record and timer by timer, the reference algorithms:
//   TR = flink-table/flink-table-runtime/src/main/java/org/apache/flink/table/runtime
//   FR = flink-runtime/src/main/java/org/apache/flink
//   * hashing             flink-core/.../util/MathUtils.java:137-200 (murmurHash, bitMix)
//                         FR/runtime/state/KeyGroupRangeAssignment.java:63-147
//                         flink-table-common/.../data/binary/MurmurHashUtils.java:70-170
//                         + BinaryRowData.java:69-124,459 (hashByWords, seed 42)
//   * window math         FR/streaming/api/windowing/windows/TimeWindow.java:84,264-272
//                         TR/operators/window/tvf/slicing/SliceAssigners.java:140-757
//                         TR/util/TimeWindowUtil.java:52-211 (shift zones over java.time
//                           ZoneRules semantics: ZonedDateTime.ofLocal gap / overlap rules)
//   * SQL operator        TR/operators/window/tvf/common/WindowAggOperator.java:216-265
//                         TR/operators/aggregate/window/processors/
//                           AbstractSliceSyncStateWindowAggProcessor.java:96-167
//                           SliceUnsharedSyncStateWindowAggProcessor.java:54-71
//                           SliceSharedSyncStateWindowAggProcessor.java:65-132
//                           AbstractSyncStateWindowAggProcessor.java:92-118 (WindowIsEmptySupplier)
//                         TR/operators/aggregate/window/buffers/RecordsWindowBuffer.java:81-126
//                         TR/operators/aggregate/window/combines/AggCombiner.java:76-115
//                         FR/streaming/api/operators/InternalTimerServiceImpl.java:249,328-348
//   * SQL aggregates      flink-table-planner/.../functions/aggfunctions/
//                           {Count1,Count,Sum,Max,Min,Avg}AggFunction.java
//   * DataStream operator FR/streaming/runtime/operators/windowing/WindowOperator.java:293-682
//                           (allowedLateness, cleanup timers, late side output :440-446,549,609-682)
//                         FR/streaming/api/windowing/triggers/EventTimeTrigger.java:37-52
//                         FR/streaming/api/windowing/assigners/{Tumbling,Sliding}EventTimeWindows.java
//                         FR/streaming/api/functions/aggregation/{SumAggregator,ComparableAggregator,
//                           Comparator}.java
// Java `long`/`int` wrap-around is reproduced with unsigned arithmetic; Java `%` truncates.
#include "../include/flinkwin.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace {

// ------------------------------------------------------------------------------------
// Java arithmetic helpers
// ------------------------------------------------------------------------------------
inline int32_t jmul32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
inline int32_t jadd32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
inline int32_t rotl32(int32_t x, int r) { uint32_t u = (uint32_t)x; return (int32_t)((u << r) | (u >> (32 - r))); }
inline int32_t ushr32(int32_t x, int r) { return (int32_t)((uint32_t)x >> r); }
inline int64_t jadd64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
inline int64_t jsub64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

// MathUtils.bitMix (MathUtils.java:194-200)
int32_t bit_mix(int32_t in) {
    in ^= ushr32(in, 16);
    in = jmul32(in, (int32_t)0x85ebca6b);
    in ^= ushr32(in, 13);
    in = jmul32(in, (int32_t)0xc2b2ae35);
    in ^= ushr32(in, 16);
    return in;
}

// MathUtils.murmurHash (MathUtils.java:137-155)
int32_t murmur_hash(int32_t code) {
    code = jmul32(code, (int32_t)0xcc9e2d51);
    code = rotl32(code, 15);
    code = jmul32(code, (int32_t)0x1b873593);
    code = rotl32(code, 13);
    code = jadd32(jmul32(code, 5), (int32_t)0xe6546b64);
    code ^= 4;
    code = bit_mix(code);
    if (code >= 0) return code;
    if (code != INT32_MIN) return -code;
    return 0;
}

// MurmurHashUtils.mixK1 / mixH1 / fmix (MurmurHashUtils.java:143-170)
int32_t mix_k1(int32_t k1) {
    k1 = jmul32(k1, (int32_t)0xcc9e2d51);
    k1 = rotl32(k1, 15);
    return jmul32(k1, (int32_t)0x1b873593);
}
int32_t mix_h1(int32_t h1, int32_t k1) {
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    return jadd32(jmul32(h1, 5), (int32_t)0xe6546b64);
}
int32_t fmix32(int32_t h) {
    h ^= ushr32(h, 16);
    h = jmul32(h, (int32_t)0x85ebca6b);
    h ^= ushr32(h, 13);
    h = jmul32(h, (int32_t)0xc2b2ae35);
    h ^= ushr32(h, 16);
    return h;
}

// BinaryRowData.hashCode of a one-field key row (BinaryRowData.java:459 ->
// BinarySegmentUtils.hashByWords -> MurmurHashUtils.hashBytesByWords, seed 42).
// Row layout (BinaryRowData.java:69-124; BinaryRowWriter.reset zeroes the 8-byte header):
// [header/null-bits 8 B = 0][field slot 8 B little endian]; an INT writes 4 bytes only.
int32_t binrow_hash_words(const int32_t* words, int nwords) {
    int32_t h1 = 42;
    for (int i = 0; i < nwords; i++) h1 = mix_h1(h1, mix_k1(words[i]));
    return fmix32(h1 ^ (nwords * 4));
}

// BinaryRowData.hashCode of a general key row, restated by building the row's bytes exactly as
// BinaryRowWriter does (BinaryRowWriter.java:39-122: reset zeroes the null-bit words, the fixed
// part is nullBitsSizeInBytes + 8 * arity, complete() sets the size to the cursor;
// AbstractBinaryWriter.java:83-106 writeString / writeBytes, :242-246 zeroOutPaddingBytes,
// :295-310 writeBytesToVarLenPart, :323-331 roundNumberOfBytesToNearestWord, :333-348
// writeBytesToFixLenPart; setNullAt :59-62 writes the null bit and a 0 slot) on a
// little-endian machine, then hashing the bytes as 4-byte ints (BinarySegmentUtils.hashByWords).
std::vector<uint8_t> key_row_image(const fw_key_field* f, int nf, int64_t i) {
    const int null_bytes = ((nf + 63 + 8) / 64) * 8;  // calculateBitSetWidthInBytes (:71-73)
    std::vector<uint8_t> row((size_t)null_bytes + 8 * (size_t)nf, 0);
    auto put_long = [&](size_t at, uint64_t v) { for (int b = 0; b < 8; b++) row[at + b] = (uint8_t)(v >> (8 * b)); };
    for (int p = 0; p < nf; p++) {
        const size_t slot = (size_t)null_bytes + 8 * (size_t)p;  // getFieldOffset (:114-116)
        if (f[p].nulls && f[p].nulls[i]) {
            const int bit = p + 8;  // HEADER_SIZE_IN_BITS
            row[(size_t)bit >> 3] |= (uint8_t)(1u << (bit & 7));
            put_long(slot, 0);
            continue;
        }
        if (f[p].kind != FW_KF_STRING) {  // putLong / putInt / putShort / put write `width` bytes
            const uint64_t v = (uint64_t)f[p].fixed[i];
            for (int b = 0; b < f[p].kind; b++) row[slot + b] = (uint8_t)(v >> (8 * b));
            continue;
        }
        const int32_t o = f[p].offsets[i], len = f[p].offsets[i + 1] - o;
        const uint8_t* bytes = f[p].bytes + o;
        if (len <= 7) {
            uint64_t seven = 0;
            for (int b = 0; b < len; b++) seven |= (uint64_t)bytes[b] << (8 * b);
            put_long(slot, ((uint64_t)(len | 0x80) << 56) | seven);
        } else {
            const size_t cursor = row.size();
            const size_t rounded = (size_t)(len + 7) / 8 * 8;
            row.resize(cursor + rounded, 0);
            memcpy(&row[cursor], bytes, (size_t)len);
            put_long(slot, ((uint64_t)cursor << 32) | (uint64_t)len);
        }
    }
    return row;
}
// BinaryRowData.hashCode of the image (BinaryRowData.java:459 -> hashBytesByWords)
int32_t key_row_hash_bytes(const fw_key_field* f, int nf, int64_t i) {
    const std::vector<uint8_t> row = key_row_image(f, nf, i);
    std::vector<int32_t> words(row.size() / 4);
    memcpy(words.data(), row.data(), row.size());
    return binrow_hash_words(words.data(), (int)words.size());
}

int32_t java_key_hash(int kind, int64_t key, int32_t precomputed) {
    switch (kind) {
        case FW_KEYHASH_LONG: return (int32_t)(key ^ (int64_t)((uint64_t)key >> 32));  // Long.hashCode
        case FW_KEYHASH_INT: return (int32_t)key;                                       // Integer.hashCode
        case FW_KEYHASH_BINROW_BIGINT: {
            int32_t w[4] = {0, 0, (int32_t)(uint32_t)(uint64_t)key, (int32_t)(uint32_t)((uint64_t)key >> 32)};
            return binrow_hash_words(w, 4);
        }
        case FW_KEYHASH_BINROW_INT: {
            int32_t w[4] = {0, 0, (int32_t)key, 0};
            return binrow_hash_words(w, 4);
        }
        default: return precomputed;
    }
}

// KeyGroupRangeAssignment.computeKeyGroupForKeyHash (:75) / computeOperatorIndexForKeyGroup (:124)
int32_t key_group_for_hash(int32_t h, int32_t max_p) { return murmur_hash(h) % max_p; }
int32_t operator_index_for_kg(int32_t max_p, int32_t p, int32_t kg) { return kg * p / max_p; }

// ------------------------------------------------------------------------------------
// window math
// ------------------------------------------------------------------------------------
// TimeWindow.getWindowStartWithOffset (TimeWindow.java:264-272), Java long semantics.
int64_t window_start_with_offset(int64_t ts, int64_t offset, int64_t size) {
    const int64_t remainder = jsub64(ts, offset) % size;  // C++ % truncates like Java
    if (remainder < 0) return jsub64(ts, jadd64(remainder, size));
    return jsub64(ts, remainder);
}

// TimeWindowUtil.getNextTriggerWatermark (TimeWindowUtil.java:186-211), no DST.
int64_t next_trigger_watermark(int64_t wm, int64_t interval) {
    if (wm == INT64_MAX) return wm;
    int64_t start = window_start_with_offset(wm, 0, interval);
    int64_t trig = jsub64(jadd64(start, interval), 1);
    return trig > wm ? trig : jadd64(trig, interval);
}

int64_t gcd64(int64_t a, int64_t b) {  // commons-math3 ArithmeticUtils.gcd for positive args
    while (b != 0) { int64_t t = a % b; a = b; b = t; }
    return a < 0 ? -a : a;
}

// ------------------------------------------------------------------------------------
// accumulators: SQL built-in aggregate functions (declarative expressions) and the
// DataStream SumAggregator / ComparableAggregator.
// ------------------------------------------------------------------------------------
struct AggState {
    int64_t i = 0;        // integer sum / min / max / count / avg-sum(int)
    double d = 0.0;       // double sum / min / max / avg-sum(double)
    int64_t cnt = 0;      // AVG count
    bool is_null = true;  // SUM/MIN/MAX null flag (SQL); COUNT never null
};

struct Row {
    AggState a[FW_MAX_AGGS];
    int64_t first = -1;  // DataStream: arrival ordinal (push << 32 | row) of the state's first element,
                         // the value1 every later reduce copies (SumAggregator.java:66-76)
};

struct OutRow {
    int64_t key, ws, we;
    uint64_t v[FW_MAX_AGGS];
    uint32_t null_mask;
    int64_t epoch;  // index of the watermark call that produced it
    int64_t first;  // DataStream: Row::first of the emitted window
};
constexpr int MAX_FIELDS = FW_MAX_AGGS;

inline double bits_to_double(uint64_t b) { double d; std::memcpy(&d, &b, 8); return d; }
inline uint64_t double_to_bits(double d) { uint64_t b; std::memcpy(&b, &d, 8); return b; }

// Double.compare (JDK): total order with -0.0 < 0.0 and NaN greatest.
int java_double_compare(double a, double b) {
    if (a < b) return -1;
    if (a > b) return 1;
    // doubleToLongBits canonicalises NaN
    const int64_t x = std::isnan(a) ? 0x7ff8000000000000LL : (int64_t)double_to_bits(a);
    const int64_t y = std::isnan(b) ? 0x7ff8000000000000LL : (int64_t)double_to_bits(b);
    return x == y ? 0 : (x < y ? -1 : 1);
}

// A shift time zone as java.time ZoneRules sees it: offset off[i] from UTC instant utc[i]
// (utc[0] = Long.MIN_VALUE).  Empty = UTC (no shift).
struct Zone {
    std::vector<int64_t> utc, off;
    bool dst = false;  // TimeZone.getTimeZone(zone).useDaylightTime()
    bool utc_zone() const { return utc.empty(); }
    // ZoneRules.getOffset(Instant)
    int64_t offset_of_instant(int64_t epoch) const {
        size_t i = (size_t)(std::upper_bound(utc.begin(), utc.end(), epoch) - utc.begin());
        return off[i - 1];
    }
    // LocalDateTime.atZone(zone).toInstant().toEpochMilli(): ZonedDateTime.ofLocal(ldt, zone,
    // null) walks the transitions: before a transition's local range the old offset holds; inside
    // a gap (offset grows) the local time moves later by the gap and takes the new offset; inside
    // an overlap (offset shrinks) the earlier (old) offset wins
    int64_t local_to_epoch(int64_t local) const {
        for (size_t i = 1; i < utc.size(); i++) {
            const int64_t before = off[i - 1], after = off[i];
            const int64_t lb = jadd64(utc[i], before), la = jadd64(utc[i], after);
            if (local < std::min(lb, la)) return jsub64(local, before);
            if (local < std::max(lb, la)) {
                if (after > before) return jsub64(jadd64(local, after - before), after);  // gap
                return jsub64(local, before);                                            // overlap
            }
        }
        return jsub64(local, off.back());
    }
};

// TimeWindowUtil.toUtcTimestampMills (:52-60)
int64_t to_utc_timestamp_mills(int64_t epoch, const Zone& z) {
    if (z.utc_zone() || epoch == INT64_MAX) return epoch;
    return jadd64(epoch, z.offset_of_instant(epoch));
}
// TimeWindowUtil.toEpochMillsForTimer (:69-140)
int64_t to_epoch_mills_for_timer(int64_t utc_ts, const Zone& z) {
    if (z.utc_zone() || utc_ts == INT64_MAX) return utc_ts;
    if (z.dst) {
        const int64_t hour = 3600LL * 1000;
        const int64_t t1 = z.local_to_epoch(utc_ts);
        const int64_t t2 = z.local_to_epoch(jadd64(utc_ts, hour));  // plusSeconds(SECONDS_PER_HOUR)
        const bool no_epoch = t1 == t2, two_epochs = jsub64(t2, t1) > hour;
        if (no_epoch) return jsub64(t1, t1 % hour);
        if (two_epochs) return jadd64(t1, hour);
        return t1;
    }
    return z.local_to_epoch(utc_ts);
}
// TimeWindowUtil.isWindowFired (:175-183)
bool is_window_fired_tz(int64_t window_end, int64_t progress, const Zone& z) {
    if (window_end == INT64_MAX) return false;
    return progress >= to_epoch_mills_for_timer(jsub64(window_end, 1), z);
}
// TimeWindowUtil.getNextTriggerWatermark (:186-211)
int64_t next_trigger_watermark_tz(int64_t wm, int64_t interval, const Zone& z) {
    if (wm == INT64_MAX) return wm;
    int64_t trig;
    if (z.dst) {
        const int64_t utc_start = window_start_with_offset(to_utc_timestamp_mills(wm, z), 0, interval);
        trig = to_epoch_mills_for_timer(jadd64(utc_start, interval) - 1, z);
    } else {
        trig = jsub64(jadd64(window_start_with_offset(wm, 0, interval), interval), 1);
    }
    return trig > wm ? trig : jadd64(trig, interval);
}

struct Config {
    fw_config c;
    int64_t interval;  // slice size (SliceAssigner.getSliceEndInterval)
    int n_slices;      // HOP slices per window
    Zone zone;         // SQL shift time zone (TimeWindowUtil.getShiftTimeZone)
    int64_t lateness = 0;  // DataStream allowedLateness
};

struct Oracle {
    Config cfg;
    bool ds;  // DataStream operator
    int phase = FW_PHASE_ONE;  // SQL: ONE / LOCAL / GLOBAL (TwoStageOptimizedWindowAggregateRule)
    // operator / processor progress
    int64_t current_watermark = INT64_MIN;      // WindowAggOperator.currentWatermark
    int64_t current_progress = INT64_MIN;       // WindowAggProcessorBase.currentProgress
    int64_t next_trigger_progress = INT64_MIN;  // AbstractSliceSyncStateWindowAggProcessor
    int64_t timer_watermark = INT64_MIN;        // InternalTimerServiceImpl.currentWatermark
    int64_t late_dropped = 0;
    int64_t fired = 0;
    int64_t epoch = 0;

    // RecordsWindowBuffer: (sliceEnd, key) -> records in insertion order
    struct BufRec { uint64_t vals[FW_MAX_COLS]; uint8_t nul[FW_MAX_COLS]; };
    std::vector<std::pair<std::pair<int64_t, int64_t>, std::vector<BufRec>>> buffer;
    std::map<std::pair<int64_t, int64_t>, size_t> buffer_index;
    int64_t min_slice_end = INT64_MAX;

    // keyed state: (key, namespace) -> accumulator row
    std::map<std::pair<int64_t, int64_t>, Row> state;
    // event-time timers: (timestamp, key, namespace) -- a set, so registration dedups
    std::set<std::tuple<int64_t, int64_t, int64_t>> timers;

    std::vector<OutRow> out;
    // DataStream late side output (WindowOperator.sideOutput): (key, ts, values, push, row)
    struct SideRow { int64_t key, ts; uint64_t v[FW_MAX_COLS]; int64_t push, row; };
    std::vector<SideRow> side;
    int64_t push_seq = 0;

    // -------------------------------------------------------------------------------
    // aggregate function expressions
    // -------------------------------------------------------------------------------
    Row create_accumulators() const { return Row(); }

    // accumulateExpressions; nul[c] != 0: value column c is NULL in this record, and every
    // aggregate of that column keeps its accumulator (ifThenElse(isNull(operand(0)), acc, ...))
    void accumulate(Row& r, const uint64_t* vals, const uint8_t* nul) const {
        for (int a = 0; a < cfg.c.n_aggs; a++) {
            const fw_agg_desc& g = cfg.c.aggs[a];
            AggState& s = r.a[a];
            if (g.kind != FW_AGG_COUNT_STAR && nul[g.input_col]) continue;
            const uint64_t raw = g.kind == FW_AGG_COUNT_STAR ? 0 : vals[g.input_col];
            const bool isf = g.type == FW_T_F64;
            const int64_t iv = (int64_t)raw;
            const double dv = bits_to_double(raw);
            switch (g.kind) {
                case FW_AGG_COUNT_STAR:  // Count1AggFunction: count + 1
                case FW_AGG_COUNT:       // CountAggFunction: count + 1 for a non-NULL operand
                    s.i = jadd64(s.i, 1);
                    s.is_null = false;
                    break;
                case FW_AGG_SUM:  // SumAggFunction: isNull(sum) ? operand : sum + operand
                    if (isf) s.d = s.is_null ? dv : s.d + dv;
                    else if (g.type == FW_T_I32) s.i = s.is_null ? (int32_t)iv : (int32_t)jadd32((int32_t)s.i, (int32_t)iv);
                    else s.i = s.is_null ? iv : jadd64(s.i, iv);
                    s.is_null = false;
                    break;
                case FW_AGG_MAX:
                case FW_AGG_MIN: {
                    const bool mx = g.kind == FW_AGG_MAX;
                    if (s.is_null) {
                        if (isf) s.d = dv; else s.i = iv;
                    } else if (isf) {
                        if (ds) {
                            // ComparableAggregator.reduce (:83-104): c = isExtremal(acc, new);
                            // MaxComparator is 1 iff acc.compareTo(new) > 0 (Comparator.java:73-80),
                            // and c == 0 sets the field to the new value: ties (equal under
                            // Double.compareTo -- only NaNs differ in bits) go to the LATER element
                            const int c = java_double_compare(s.d, dv);
                            if (!(mx ? c > 0 : c < 0)) s.d = dv;
                        } else {   // MaxAggFunction: operand > max ; MinAggFunction: operand < min
                            if (mx ? dv > s.d : dv < s.d) s.d = dv;
                        }
                    } else {
                        if (mx ? iv > s.i : iv < s.i) s.i = iv;
                    }
                    s.is_null = false;
                    break;
                }
                case FW_AGG_AVG:  // AvgAggFunction: sum + operand, count + 1
                    if (isf) s.d = s.d + dv; else s.i = jadd64(s.i, iv);
                    s.cnt = jadd64(s.cnt, 1);
                    s.is_null = false;
                    break;
            }
        }
    }

    // DataStream minBy / maxBy (WindowedStream.java:725-790): the reducing state holds an ELEMENT;
    // ComparableAggregator.reduce (:83-104) with byAggregate keeps value1 (the state) when
    // MaxByComparator / MinByComparator (Comparator.java:58-101) says it is strictly extremal, and
    // on c == 0 keeps value1 iff `first`.  Row::first is the kept element's arrival ordinal and the
    // aggregate its field.
    bool is_by() const {
        return ds && cfg.c.n_aggs == 1 && (cfg.c.aggs[0].kind == FW_AGG_MINBY || cfg.c.aggs[0].kind == FW_AGG_MAXBY);
    }
    void by_reduce(Row& r, const uint64_t* vals, int64_t ord, bool fresh) const {
        const fw_agg_desc& g = cfg.c.aggs[0];
        AggState& s = r.a[0];
        const uint64_t raw = vals[g.input_col];
        const bool isf = g.type == FW_T_F64;
        if (!fresh) {
            // o1 = the state's field, o2 = the new element's: c = sign of o1.compareTo(o2), flipped for minBy
            int c;
            if (isf) c = java_double_compare(s.d, bits_to_double(raw));
            else c = s.i < (int64_t)raw ? -1 : s.i > (int64_t)raw ? 1 : 0;
            if (g.kind == FW_AGG_MINBY) c = -c;
            const bool first = !(g.flags & FW_AGGF_LAST);
            if (c > 0 || (c == 0 && first)) return;  // value1 stays
        }
        if (isf) s.d = bits_to_double(raw); else s.i = (int64_t)raw;
        s.is_null = false;
        r.first = ord;
    }

    // mergeExpressions of the same functions
    void merge(Row& r, const Row& o) const {
        for (int a = 0; a < cfg.c.n_aggs; a++) {
            const fw_agg_desc& g = cfg.c.aggs[a];
            AggState& s = r.a[a];
            const AggState& t = o.a[a];
            const bool isf = g.type == FW_T_F64;
            switch (g.kind) {
                case FW_AGG_COUNT_STAR:
                case FW_AGG_COUNT:
                    s.i = jadd64(s.i, t.i);
                    s.is_null = false;
                    break;
                case FW_AGG_SUM:
                    if (t.is_null) break;
                    if (isf) s.d = s.is_null ? t.d : s.d + t.d;
                    else if (g.type == FW_T_I32) s.i = s.is_null ? t.i : (int32_t)jadd32((int32_t)s.i, (int32_t)t.i);
                    else s.i = s.is_null ? t.i : jadd64(s.i, t.i);
                    s.is_null = false;
                    break;
                case FW_AGG_MAX:
                case FW_AGG_MIN: {
                    if (t.is_null) break;
                    const bool mx = g.kind == FW_AGG_MAX;
                    if (s.is_null) { s.i = t.i; s.d = t.d; }
                    else if (isf) {
                        if (ds) { int c = java_double_compare(t.d, s.d); if (mx ? c > 0 : c < 0) s.d = t.d; }
                        else if (mx ? t.d > s.d : t.d < s.d) s.d = t.d;
                    } else if (mx ? t.i > s.i : t.i < s.i) s.i = t.i;
                    s.is_null = false;
                    break;
                }
                case FW_AGG_AVG:
                    if (isf) s.d = s.d + t.d; else s.i = jadd64(s.i, t.i);
                    s.cnt = jadd64(s.cnt, t.cnt);
                    s.is_null = false;
                    break;
            }
        }
    }

    // LocalAggCombiner.output (LocalAggCombiner.java:100-106): the accumulator fields of every
    // aggregate in order -- COUNT(*) / COUNT: count; SUM / MIN / MAX: value (NULL-able);
    // AVG: sum, count.  Returns the field count.
    int acc_fields(const Row& r, uint64_t* v, uint32_t* nm) const {
        *nm = 0;
        int j = 0;
        for (int a = 0; a < cfg.c.n_aggs; a++) {
            const fw_agg_desc& g = cfg.c.aggs[a];
            const AggState& s = r.a[a];
            const bool isf = g.type == FW_T_F64;
            switch (g.kind) {
                case FW_AGG_COUNT_STAR:
                case FW_AGG_COUNT: v[j++] = (uint64_t)s.i; break;
                case FW_AGG_AVG:
                    v[j++] = isf ? double_to_bits(s.d) : (uint64_t)s.i;
                    v[j++] = (uint64_t)s.cnt;
                    break;
                default:
                    if (s.is_null) { *nm |= 1u << j; v[j++] = 0; break; }
                    v[j++] = isf ? double_to_bits(s.d) : (uint64_t)s.i;
                    break;
            }
        }
        return j;
    }

    // the inverse: a local accumulator row as an accumulator Row (GLOBAL phase input; aggregate a
    // reads its fields from column input_col, AVG's count from the next column)
    Row row_from_fields(const uint64_t* v, const uint8_t* nul) const {
        Row r;
        for (int a = 0; a < cfg.c.n_aggs; a++) {
            const fw_agg_desc& g = cfg.c.aggs[a];
            AggState& s = r.a[a];
            const bool isf = g.type == FW_T_F64;
            int j = g.input_col;
            switch (g.kind) {
                case FW_AGG_COUNT_STAR:
                case FW_AGG_COUNT: s.i = (int64_t)v[j++]; s.is_null = false; break;
                case FW_AGG_AVG:
                    if (isf) s.d = bits_to_double(v[j]); else s.i = (int64_t)v[j];
                    j++;
                    s.cnt = (int64_t)v[j++];
                    s.is_null = false;
                    break;
                default:
                    s.is_null = nul[j] != 0;
                    if (isf) s.d = bits_to_double(v[j]); else s.i = (int64_t)v[j];
                    j++;
                    break;
            }
        }
        return r;
    }

    // getValueExpression; returns value words + null mask
    void get_value(const Row& r, uint64_t* v, uint32_t* nm) const {
        *nm = 0;
        for (int a = 0; a < cfg.c.n_aggs; a++) {
            const fw_agg_desc& g = cfg.c.aggs[a];
            const AggState& s = r.a[a];
            const bool isf = g.type == FW_T_F64;
            v[a] = 0;
            switch (g.kind) {
                case FW_AGG_COUNT_STAR:
                case FW_AGG_COUNT: v[a] = (uint64_t)s.i; break;
                case FW_AGG_SUM:
                case FW_AGG_MAX:
                case FW_AGG_MIN:
                    if (s.is_null) { *nm |= 1u << a; break; }
                    v[a] = isf ? double_to_bits(s.d) : (uint64_t)s.i;
                    break;
                case FW_AGG_MINBY:  // the kept element's field (its element: Row::first)
                case FW_AGG_MAXBY:
                    v[a] = isf ? double_to_bits(s.d) : (uint64_t)s.i;
                    break;
                case FW_AGG_AVG:  // count == 0 ? null : cast(sum / count)
                    if (s.cnt == 0) { *nm |= 1u << a; break; }
                    if (isf) v[a] = double_to_bits(s.d / (double)s.cnt);
                    else {
                        int64_t q = (s.i == INT64_MIN && s.cnt == -1) ? INT64_MIN : s.i / s.cnt;
                        if (g.type == FW_T_I32) q = (int32_t)q;
                        v[a] = (uint64_t)q;
                    }
                    break;
            }
        }
    }

    int64_t count_star(const Row& r) const {
        int idx = cfg.c.count_star_index;
        return r.a[idx].i;
    }

    // -------------------------------------------------------------------------------
    // SliceAssigner (SliceAssigners.java)
    // -------------------------------------------------------------------------------
    // AbstractSliceAssigner.assignSliceEnd(element, clock) (SliceAssigners.java:655-670): the
    // rowtime goes through toUtcTimestampMills first
    int64_t assign_slice_end(int64_t ts) const {
        const fw_config& c = cfg.c;
        const int64_t step = cfg.interval;
        return jadd64(window_start_with_offset(to_utc_timestamp_mills(ts, cfg.zone), c.offset_ms, step), step);
    }
    bool wfired(int64_t window_end, int64_t progress) const { return is_window_fired_tz(window_end, progress, cfg.zone); }
    int64_t get_window_start(int64_t we) const {
        const fw_config& c = cfg.c;
        if (c.window_kind == FW_WIN_CUMULATE)
            return window_start_with_offset(jsub64(we, 1), c.offset_ms, c.size_ms);
        return jsub64(we, c.size_ms);
    }
    int64_t get_last_window_end(int64_t slice_end) const {
        const fw_config& c = cfg.c;
        switch (c.window_kind) {
            case FW_WIN_TUMBLE: return slice_end;
            case FW_WIN_HOP: return jadd64(jsub64(slice_end, cfg.interval), c.size_ms);
            default: return jadd64(get_window_start(slice_end), c.size_ms);
        }
    }
    // sliceStateMergeTarget: unshared -> itself; hop -> itself (null merge target);
    // cumulate -> first slice of the window (mergeSlices callback target).
    int64_t merge_target(int64_t slice_end) const {
        if (cfg.c.window_kind == FW_WIN_CUMULATE) return jadd64(get_window_start(slice_end), cfg.interval);
        return slice_end;
    }

    void register_timer(int64_t key, int64_t window) {
        // SlicingWindowTimerServiceImpl.registerEventTimeWindowTimer (:43-46):
        // ts = toEpochMillsForTimer(window - 1, shiftTimeZone)
        timers.insert(std::make_tuple(to_epoch_mills_for_timer(jsub64(window, 1), cfg.zone), key, window));
    }

    // -------------------------------------------------------------------------------
    // SQL: AbstractSliceSyncStateWindowAggProcessor.processElement (:96-126)
    // -------------------------------------------------------------------------------
    bool sql_process_element(int64_t key, int64_t ts, const uint64_t* vals, const uint8_t* nul) {
        if (phase == FW_PHASE_LOCAL) {  // LocalSlicingWindowAggOperator.processElement (:109-115)
            buffer_add(key, assign_slice_end(ts), vals, nul);
            return false;
        }
        // GLOBAL: SliceAssigners.sliced -> the row's slice-end field (here: the ts column)
        const int64_t slice_end = phase == FW_PHASE_GLOBAL ? ts : assign_slice_end(ts);
        if (wfired(slice_end, current_progress)) {
            const int64_t last = get_last_window_end(slice_end);
            if (wfired(last, current_progress)) return true;  // dropped
            buffer_add(key, merge_target(slice_end), vals, nul);
            int64_t unfired = slice_end;
            while (wfired(unfired, current_progress)) unfired = jadd64(unfired, cfg.interval);
            register_timer(key, unfired);
            return false;
        }
        buffer_add(key, slice_end, vals, nul);
        return false;
    }

    void buffer_add(int64_t key, int64_t slice, const uint64_t* vals, const uint8_t* nul) {
        auto wk = std::make_pair(slice, key);
        auto it = buffer_index.find(wk);
        size_t gi;
        if (it == buffer_index.end()) {
            gi = buffer.size();
            buffer_index.emplace(wk, gi);
            buffer.push_back({wk, {}});
        } else {
            gi = it->second;
        }
        BufRec r;
        std::memcpy(r.vals, vals, sizeof(r.vals));
        std::memcpy(r.nul, nul, sizeof(r.nul));
        buffer[gi].second.push_back(r);
        min_slice_end = std::min(min_slice_end, slice);
    }

    // RecordsWindowBuffer.flush (:115-126) -> AggCombiner.combine (:76-115); LOCAL:
    // LocalAggCombiner.combine (:69-97) emits the accumulator; GLOBAL: GlobalAggCombiner.combine
    // (:77-110) merges the local accumulators into a fresh one, then into the state.
    void flush() {
        for (auto& g : buffer) {
            const int64_t slice = g.first.first, key = g.first.second;
            if (phase == FW_PHASE_LOCAL) {
                Row acc = create_accumulators();
                for (auto& rec : g.second) accumulate(acc, rec.vals, rec.nul);
                OutRow o;
                o.key = key;
                o.ws = o.we = slice;
                acc_fields(acc, o.v, &o.null_mask);
                o.epoch = epoch;
                out.push_back(o);
                continue;
            }
            auto sk = std::make_pair(key, slice);
            auto it = state.find(sk);
            Row acc = it == state.end() ? create_accumulators() : it->second;
            if (phase == FW_PHASE_GLOBAL) {
                Row local = create_accumulators();
                for (auto& rec : g.second) merge(local, row_from_fields(rec.vals, rec.nul));
                merge(acc, local);
            } else {
                for (auto& rec : g.second) accumulate(acc, rec.vals, rec.nul);
            }
            state[sk] = acc;
            if (!wfired(slice, timer_watermark)) register_timer(key, slice);
        }
        buffer.clear();
        buffer_index.clear();
        min_slice_end = INT64_MAX;
    }

    void emit(int64_t key, int64_t we, const Row& acc) {
        OutRow o;
        o.key = key;
        o.we = we;
        o.ws = ds ? jsub64(we, cfg.c.size_ms) : get_window_start(we);
        o.first = acc.first;
        get_value(acc, o.v, &o.null_mask);
        o.epoch = epoch;
        out.push_back(o);
    }

    bool is_empty(const Row& acc) const {  // WindowIsEmptySupplier.get
        if (cfg.c.count_star_index < 0) return false;
        return count_star(acc) == 0;
    }

    void sql_fire_window(int64_t key, int64_t we) {
        const fw_config& c = cfg.c;
        if (c.window_kind == FW_WIN_TUMBLE) {  // SliceUnsharedSyncStateWindowAggProcessor.fireWindow
            auto it = state.find({key, we});
            Row acc = it == state.end() ? create_accumulators() : it->second;
            if (is_empty(acc)) return;
            emit(key, we, acc);
            return;
        }
        // SliceSharedSyncStateWindowAggProcessor.fireWindow -> mergeSlices -> merge
        Row acc;
        if (c.window_kind == FW_WIN_HOP) {
            acc = create_accumulators();  // null merge target: heap accumulator
            int64_t s = we;
            for (int i = 0; i < cfg.n_slices; i++) {  // HoppingSlicesIterable
                auto it = state.find({key, s});
                if (it != state.end()) merge(acc, it->second);
                s = jsub64(s, cfg.interval);
            }
        } else {
            const int64_t first = jadd64(get_window_start(we), cfg.interval);
            auto it = state.find({key, first});
            acc = it == state.end() ? create_accumulators() : it->second;
            if (we != first) {
                auto jt = state.find({key, we});
                if (jt != state.end()) merge(acc, jt->second);
            }
            state[{key, first}] = acc;  // windowState.update(mergeResult, acc)
        }
        const bool empty = is_empty(acc);
        if (!empty) emit(key, we, acc);
        // nextTriggerWindow
        if (c.window_kind == FW_WIN_HOP) {
            if (!empty) register_timer(key, jadd64(we, cfg.interval));
        } else {
            const int64_t next = jadd64(we, cfg.interval);
            const int64_t max_we = jadd64(get_window_start(we), c.size_ms);
            if (!(next > max_we)) register_timer(key, next);
        }
    }

    // AbstractSliceSyncStateWindowAggProcessor.clearWindow -> expiredSlices
    void sql_clear_window(int64_t key, int64_t we) {
        const fw_config& c = cfg.c;
        if (c.window_kind == FW_WIN_TUMBLE) {
            state.erase({key, we});
        } else if (c.window_kind == FW_WIN_HOP) {
            state.erase({key, jadd64(jsub64(we, c.size_ms), cfg.interval)});
        } else {
            const int64_t ws = get_window_start(we);
            const int64_t first = jadd64(ws, cfg.interval);
            const int64_t last = jadd64(ws, c.size_ms);
            if (we == first) {
            } else if (we == last) {
                state.erase({key, we});
                state.erase({key, first});
            } else {
                state.erase({key, we});
            }
        }
    }

    // InternalTimerServiceImpl.tryAdvanceWatermark (:328-348)
    void advance_timers(int64_t wm) {
        timer_watermark = wm;
        while (!timers.empty()) {
            auto t = *timers.begin();
            if (std::get<0>(t) > wm) break;
            timers.erase(timers.begin());
            fired++;
            const int64_t key = std::get<1>(t), ns = std::get<2>(t);
            if (ds) {
                ds_on_event_time(key, ns, std::get<0>(t));
            } else {  // WindowAggOperator.onTimer: fireWindow then clearWindow
                sql_fire_window(key, ns);
                sql_clear_window(key, ns);
            }
        }
    }

    // LocalSlicingWindowAggOperator.processWatermark (:117-130): flush (emit partials) when the
    // watermark may trigger a window; no timers, no state
    void local_process_watermark(int64_t wm) {
        if (wm > current_watermark) {
            current_watermark = wm;
            if (current_watermark >= next_trigger_progress) {
                if (wfired(min_slice_end, current_watermark)) flush();
                next_trigger_progress = next_trigger_watermark_tz(current_watermark, cfg.interval, cfg.zone);
            }
        }
    }

    // WindowAggOperator.processWatermark (:227-238)
    void sql_process_watermark(int64_t wm) {
        if (wm > current_watermark) {
            // AbstractSliceSyncStateWindowAggProcessor.advanceProgress (:139-153)
            if (wm > current_progress) {
                current_progress = wm;
                if (current_progress >= next_trigger_progress) {
                    // RecordsWindowBuffer.advanceProgress (:107-112)
                    if (wfired(min_slice_end, current_progress)) flush();
                    next_trigger_progress = next_trigger_watermark_tz(current_progress, cfg.interval, cfg.zone);
                }
            }
            current_watermark = wm;
            advance_timers(wm);
        }
    }

    // -------------------------------------------------------------------------------
    // DataStream: WindowOperator.processElement (non-merging branch :405-446) with
    // EventTimeTrigger, allowedLateness >= 0 and an optional late side output.
    // -------------------------------------------------------------------------------
    // WindowOperator.cleanupTime (:670-677): maxTimestamp + allowedLateness, Long.MAX_VALUE on overflow
    int64_t cleanup_time(int64_t max_ts) const {
        const int64_t t = jadd64(max_ts, cfg.lateness);
        return t >= max_ts ? t : INT64_MAX;
    }
    bool ds_process_element(int64_t key, int64_t ts, const uint64_t* vals, int64_t row) {
        static const uint8_t no_nulls[FW_MAX_COLS] = {0};
        const fw_config& c = cfg.c;
        std::vector<int64_t> starts;
        if (c.window_kind == FW_WIN_TUMBLE) {
            // TumblingEventTimeWindows.assignWindows (:69-87), stagger offset 0
            starts.push_back(window_start_with_offset(ts, c.offset_ms % c.size_ms, c.size_ms));
        } else {
            // SlidingEventTimeWindows.assignWindows (:77-90)
            const int64_t last_start = window_start_with_offset(ts, c.offset_ms, c.slide_ms);
            for (int64_t s = last_start; s > jsub64(ts, c.size_ms); s = jsub64(s, c.slide_ms)) starts.push_back(s);
        }
        bool skipped = true;
        for (int64_t s : starts) {
            const int64_t end = jadd64(s, c.size_ms);
            const int64_t max_ts = jsub64(end, 1);
            if (cleanup_time(max_ts) <= timer_watermark) continue;  // isWindowLate (:609-612)
            skipped = false;
            auto sk = std::make_pair(key, end);
            auto it = state.find(sk);
            Row acc = it == state.end() ? create_accumulators() : it->second;
            const int64_t ord = (int64_t)(((uint64_t)push_seq << 32) | (uint64_t)row);
            if (it == state.end()) acc.first = ord;
            if (is_by()) by_reduce(acc, vals, ord, it == state.end());
            else accumulate(acc, vals, no_nulls);  // HeapReducingState.add / HeapAggregatingState.add
            state[sk] = acc;
            // EventTimeTrigger.onElement (:37-45): a window whose maxTimestamp the watermark has
            // passed FIRES at once (emitWindowContents), else its timer is registered
            if (max_ts <= timer_watermark) emit(key, end, acc);
            else timers.insert(std::make_tuple(max_ts, key, end));
            // registerCleanupTimer (:616-628): no timer for a cleanup time of Long.MAX_VALUE
            const int64_t ct = cleanup_time(max_ts);
            if (ct != INT64_MAX) timers.insert(std::make_tuple(ct, key, end));
        }
        // isSkippedElement && isElementLate (:438-446, :640-644)
        if (skipped && jadd64(ts, cfg.lateness) <= timer_watermark) {
            if (c.late_side_output) {
                SideRow r{key, ts, {0}, push_seq, row};
                std::memcpy(r.v, vals, sizeof(r.v));
                side.push_back(r);
                return false;
            }
            return true;  // numLateRecordsDropped
        }
        return false;
    }

    // WindowOperator.onEventTime (:450-494)
    void ds_on_event_time(int64_t key, int64_t end, int64_t time) {
        const int64_t max_ts = jsub64(end, 1);
        auto it = state.find({key, end});
        if (time == max_ts) {  // EventTimeTrigger.onEventTime -> FIRE
            if (it != state.end()) emit(key, end, it->second);  // emitWindowContents, ts = maxTimestamp
        }
        if (time == cleanup_time(max_ts)) state.erase({key, end});  // isCleanupTime -> clearAllState
    }

    void ds_process_watermark(int64_t wm) {
        if (wm > timer_watermark) advance_timers(wm);
        current_watermark = std::max(current_watermark, wm);
        current_progress = current_watermark;
    }

    void process_watermark(int64_t wm) {
        if (ds) ds_process_watermark(wm);
        else if (phase == FW_PHASE_LOCAL) local_process_watermark(wm);
        else sql_process_watermark(wm);
        epoch++;
    }

    // SQL: prepareSnapshotPreBarrier -> windowBuffer.flush(); then a restored operator starts with
    // nextTriggerProgress = Long.MIN_VALUE and the watermark from union-list state
    // (WindowAggOperator.java:183-206).  DataStream: the WindowOperator snapshots no watermark, so
    // the restored timer service starts at Long.MIN_VALUE (InternalTimerServiceImpl.java:72) and
    // nothing is late until the next watermark; state and timers are kept.
    void snapshot_restore() {
        if (!ds) flush();
        next_trigger_progress = INT64_MIN;
        if (ds) {
            timer_watermark = INT64_MIN;
            current_watermark = INT64_MIN;
            current_progress = INT64_MIN;
        }
    }
};

thread_local char g_err[256];

}  // namespace

// ======================================================================================
// C ABI (tests only)
// ======================================================================================
extern "C" {

const char* or_last_error(void) { return g_err; }

void* or_create(const fw_config* c) {
    if (!c || c->n_aggs < 0 || c->n_aggs > FW_MAX_AGGS) { snprintf(g_err, sizeof g_err, "bad config"); return nullptr; }
    Oracle* o = new Oracle();
    o->cfg.c = *c;
    o->ds = c->api == FW_API_DATASTREAM;
    o->phase = c->agg_phase;
    if (c->window_kind == FW_WIN_TUMBLE) { o->cfg.interval = c->size_ms; o->cfg.n_slices = 1; }
    else if (c->window_kind == FW_WIN_HOP) {
        o->cfg.interval = gcd64(c->size_ms, c->slide_ms);
        o->cfg.n_slices = (int)(c->size_ms / o->cfg.interval);
    } else { o->cfg.interval = c->slide_ms; o->cfg.n_slices = (int)(c->size_ms / c->slide_ms); }
    o->cfg.lateness = o->ds ? c->allowed_lateness_ms : 0;
    if (c->tz_n > 0 && c->tz_utc && c->tz_offset_ms) {
        o->cfg.zone.utc.assign(c->tz_utc, c->tz_utc + c->tz_n);
        o->cfg.zone.off.assign(c->tz_offset_ms, c->tz_offset_ms + c->tz_n);
        o->cfg.zone.dst = c->tz_use_dst != 0;
    }
    o->cfg.c.tz_utc = nullptr;  // the table lives in cfg.zone
    o->cfg.c.tz_offset_ms = nullptr;
    return o;
}

void or_destroy(void* h) { delete (Oracle*)h; }

void or_initialize_watermark(void* h, int64_t wm) {
    Oracle* o = (Oracle*)h;
    o->current_watermark = wm;
    o->current_progress = wm;
    o->timer_watermark = wm;
}

// Row-major value columns: vals[col * n + i] (8-byte words); nulls[col * n + i] != 0 marks a
// SQL NULL (nulls may be NULL: no NULLs).
int64_t or_process_batch(void* h, int64_t n, const int64_t* key, const int64_t* ts, const uint64_t* vals, int32_t ncols,
                         const uint8_t* nulls) {
    Oracle* o = (Oracle*)h;
    int64_t dropped = 0;
    uint64_t row[FW_MAX_COLS] = {0};
    uint8_t nul[FW_MAX_COLS] = {0};
    for (int64_t i = 0; i < n; i++) {
        for (int c = 0; c < ncols; c++) {
            row[c] = vals[(int64_t)c * n + i];
            nul[c] = nulls ? nulls[(int64_t)c * n + i] : 0;
        }
        bool d = o->ds ? o->ds_process_element(key[i], ts[i], row, i) : o->sql_process_element(key[i], ts[i], row, nul);
        if (d) dropped++;
    }
    o->late_dropped += dropped;
    o->push_seq++;
    return dropped;
}

void or_process_watermark(void* h, int64_t wm) { ((Oracle*)h)->process_watermark(wm); }
void or_flush(void* h) { Oracle* o = (Oracle*)h; if (!o->ds) o->flush(); }
void or_snapshot_restore(void* h) { ((Oracle*)h)->snapshot_restore(); }
int64_t or_late_dropped(void* h) { return ((Oracle*)h)->late_dropped; }
int64_t or_state_size(void* h) { return (int64_t)((Oracle*)h)->state.size(); }
int64_t or_timer_count(void* h) { return (int64_t)((Oracle*)h)->timers.size(); }
int64_t or_current_watermark(void* h) { return ((Oracle*)h)->current_watermark; }

// Keyed state and timers as the heap backend holds them: (key, namespace, accumulator fields) per
// window state entry and (timestamp, key, namespace) per event-time timer, for checking
// fw_snapshot_key_group_heap.  Return the entry counts (rows beyond cap are not written);
// fields[i * FW_MAX_AGGS * 2 + j].
int64_t or_state_dump(void* h, int64_t* key, int64_t* ns, uint64_t* fields, uint32_t* nm, int64_t cap) {
    Oracle* o = (Oracle*)h;
    int64_t i = 0;
    for (const auto& kv : o->state) {
        if (i < cap) {
            key[i] = kv.first.first;
            ns[i] = kv.first.second;
            o->acc_fields(kv.second, fields + i * FW_MAX_AGGS * 2, nm + i);
        }
        i++;
    }
    return i;
}
// DataStream window-contents (WindowOperatorBuilder.java:81): per (key, window end) the value the
// window would emit (the reduced record's aggregated field) and its first element's arrival
// ordinal (the record is value1, SumAggregator.java:66-76)
int64_t or_ds_state_dump(void* h, int64_t* key, int64_t* end, uint64_t* value, int64_t* first, int64_t cap) {
    Oracle* o = (Oracle*)h;
    int64_t i = 0;
    for (const auto& kv : o->state) {
        if (i < cap) {
            uint64_t v[FW_MAX_AGGS];
            uint32_t nm = 0;
            o->get_value(kv.second, v, &nm);
            key[i] = kv.first.first;
            end[i] = kv.first.second;
            value[i] = v[0];
            first[i] = kv.second.first;
        }
        i++;
    }
    return i;
}
int64_t or_timer_dump(void* h, int64_t* ts, int64_t* key, int64_t* ns, int64_t cap) {
    Oracle* o = (Oracle*)h;
    int64_t i = 0;
    for (const auto& t : o->timers) {
        if (i < cap) {
            ts[i] = std::get<0>(t);
            key[i] = std::get<1>(t);
            ns[i] = std::get<2>(t);
        }
        i++;
    }
    return i;
}

int64_t or_num_results(void* h) { return (int64_t)((Oracle*)h)->out.size(); }
// result value columns: the aggregates, or the LOCAL phase's accumulator fields
int32_t or_num_value_columns(void* h) {
    Oracle* o = (Oracle*)h;
    if (o->phase != FW_PHASE_LOCAL) return o->cfg.c.n_aggs;
    int n = 0;
    for (int a = 0; a < o->cfg.c.n_aggs; a++) n += o->cfg.c.aggs[a].kind == FW_AGG_AVG ? 2 : 1;
    return n;
}
// Copies results into SoA arrays (each may be NULL): vals[a * n + i].
void or_get_results(void* h, int64_t* key, int64_t* ws, int64_t* we, uint64_t* vals, uint32_t* nm, int64_t* epoch) {
    Oracle* o = (Oracle*)h;
    const int64_t n = (int64_t)o->out.size();
    for (int64_t i = 0; i < n; i++) {
        const OutRow& r = o->out[i];
        if (key) key[i] = r.key;
        if (ws) ws[i] = r.ws;
        if (we) we[i] = r.we;
        if (nm) nm[i] = r.null_mask;
        if (epoch) epoch[i] = r.epoch;
        if (vals) for (int a = 0; a < or_num_value_columns(h); a++) vals[(int64_t)a * n + i] = r.v[a];
    }
}
void or_clear_results(void* h) { ((Oracle*)h)->out.clear(); }
// DataStream: the first-element arrival ordinal of each result (Row::first), same order as or_get_results
void or_get_first(void* h, int64_t* first) {
    Oracle* o = (Oracle*)h;
    for (size_t i = 0; i < o->out.size(); i++) first[i] = o->out[i].first;
}
// late side output rows since the last call (consumed): SoA, vals[c * n + i]
int64_t or_num_side_rows(void* h) { return (int64_t)((Oracle*)h)->side.size(); }
void or_take_side_rows(void* h, int64_t* key, int64_t* ts, uint64_t* vals, int64_t* push, int64_t* row) {
    Oracle* o = (Oracle*)h;
    const int64_t n = (int64_t)o->side.size();
    for (int64_t i = 0; i < n; i++) {
        const Oracle::SideRow& r = o->side[i];
        key[i] = r.key;
        ts[i] = r.ts;
        push[i] = r.push;
        row[i] = r.row;
        for (int c = 0; c < o->cfg.c.n_value_cols; c++) vals[(int64_t)c * n + i] = r.v[c];
    }
    o->side.clear();
}
// shift-zone arithmetic of an operator (what: 0 toUtcTimestampMills, 1 toEpochMillsForTimer,
// 2 getNextTriggerWatermark, 3 assignSliceEnd, 4 getWindowStart)
int64_t or_time_op(void* h, int32_t what, int64_t x) {
    Oracle* o = (Oracle*)h;
    switch (what) {
        case 0: return to_utc_timestamp_mills(x, o->cfg.zone);
        case 1: return to_epoch_mills_for_timer(x, o->cfg.zone);
        case 2: return next_trigger_watermark_tz(x, o->cfg.interval, o->cfg.zone);
        case 3: return o->assign_slice_end(x);
        default: return o->get_window_start(x);
    }
}

// Hash / key-group restatements.
int32_t or_murmur_hash(int32_t code) { return murmur_hash(code); }
int32_t or_java_key_hash(int32_t kind, int64_t key, int32_t pre) { return java_key_hash(kind, key, pre); }
void or_key_row_hash(const fw_key_field* fields, int32_t n_fields, int64_t n, int32_t* out) {
    for (int64_t i = 0; i < n; i++) out[i] = key_row_hash_bytes(fields, n_fields, i);
}
// row i's BinaryRowWriter image; returns its length (bytes copied only if <= cap)
int64_t or_key_row_image(const fw_key_field* fields, int32_t n_fields, int64_t i, uint8_t* out, int64_t cap) {
    const std::vector<uint8_t> row = key_row_image(fields, n_fields, i);
    if ((int64_t)row.size() <= cap) memcpy(out, row.data(), row.size());
    return (int64_t)row.size();
}
int32_t or_key_group(int32_t kind, int64_t key, int32_t pre, int32_t max_p) {
    return key_group_for_hash(java_key_hash(kind, key, pre), max_p);
}
int32_t or_operator_index(int32_t max_p, int32_t p, int32_t kg) { return operator_index_for_kg(max_p, p, kg); }
// the subtask of each key (assignKeyToParallelOperator, KeyGroupRangeAssignment.java:49-73): the
// bench's multi-threaded CPU baseline partitions its sample like a keyBy at parallelism p
void or_operator_indices(int32_t kind, const int64_t* keys, int64_t n, int32_t pre, int32_t max_p, int32_t p,
                         int32_t* out) {
    for (int64_t i = 0; i < n; i++)
        out[i] = operator_index_for_kg(max_p, p, key_group_for_hash(java_key_hash(kind, keys[i], pre), max_p));
}
void or_key_group_range(int32_t max_p, int32_t p, int32_t idx, int32_t* start, int32_t* end) {
    // computeKeyGroupRangeForOperatorIndex (:93-106)
    *start = (idx * max_p + p - 1) / p;
    *end = ((idx + 1) * max_p - 1) / p;
}
int64_t or_window_start_with_offset(int64_t ts, int64_t off, int64_t size) { return window_start_with_offset(ts, off, size); }
int64_t or_next_trigger_watermark(int64_t wm, int64_t interval) { return next_trigger_watermark(wm, interval); }

// Synthetic generator, same definition as the device generator.
static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
void or_generate(const fw_gen_params* gp, const double* zipf_cdf, int64_t i0, int64_t n,
                 int64_t* key, int64_t* ts, int64_t* val) {
    for (int64_t j = 0; j < n; j++) {
        const uint64_t i = (uint64_t)(i0 + j);
        const uint64_t u = splitmix64(gp->seed ^ (i * 0x9E3779B97F4A7C15ULL));
        const int64_t t = gp->t0_ms + (int64_t)((__int128)i * 1000 / gp->rate_per_s) - (int64_t)(u % (uint64_t)gp->ooo_ms);
        int64_t k;
        if (gp->key_dist == 0) {
            k = gp->key_base + (int64_t)((u >> 20) % (uint64_t)gp->key_count);
        } else {
            const double x = (double)(u >> 11) * (1.0 / 9007199254740992.0);
            int64_t lo = 0, hi = gp->key_count - 1;  // first index with cdf > x
            while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (zipf_cdf[mid] > x) hi = mid; else lo = mid + 1; }
            k = gp->key_base + lo;
        }
        uint64_t v;
        if (gp->value_kind == 0) v = 1 + u % 1000000000ULL;
        else if (gp->value_kind == 1) { double d = 1000.0 * (double)(u >> 11) * (1.0 / 9007199254740992.0); std::memcpy(&v, &d, 8); }
        else v = u % 1000000ULL;
        if (key) key[j] = k;
        if (ts) ts[j] = t;
        if (val) val[j] = (int64_t)v;
    }
}

}  // extern "C"
