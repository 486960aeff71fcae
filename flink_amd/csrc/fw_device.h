// fw_device.h -- arithmetic shared by the gfx950 kernels and the host side of libflinkwin.
//
// Everything here is __host__ __device__ so the exact same code that runs in the kernels can
// be exercised on the CPU (fw_host_* entry points, tests/test_native_host.py).
//
// Java semantics: `long`/`int` arithmetic wraps (two's complement), `%` truncates toward zero.
// The reference functions restated here:
//   MathUtils.murmurHash / bitMix          flink-core/.../util/MathUtils.java:137-155,194-200
//   KeyGroupRangeAssignment                 FR/runtime/state/KeyGroupRangeAssignment.java:63-147
//   BinaryRowData.hashCode                  flink-table-common/.../data/binary/BinaryRowData.java:459
//     -> MurmurHashUtils.hashBytesByWords   .../MurmurHashUtils.java:70,92-96,131-170 (seed 42)
//   TimeWindow.getWindowStartWithOffset     FR/streaming/api/windowing/windows/TimeWindow.java:264-272
//   TimeWindowUtil.isWindowFired / getNextTriggerWatermark
//                                           TR/util/TimeWindowUtil.java:175-211 (UTC)
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#define FW_HD __host__ __device__ __forceinline__

namespace fw {

// ---------------------------------------------------------------------------------------
// 32-bit Java int helpers (done in uint32 to get wrap-around without UB)
// ---------------------------------------------------------------------------------------
FW_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

FW_HD uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

FW_HD uint32_t murmur_k1(uint32_t k) { return rotl32(k * 0xcc9e2d51u, 15) * 0x1b873593u; }
FW_HD uint32_t murmur_h1(uint32_t h, uint32_t k1) { return rotl32(h ^ k1, 13) * 5u + 0xe6546b64u; }

// MathUtils.murmurHash(int): one 4-byte Murmur3 block (seed 0), length 4, then |h| with
// Integer.MIN_VALUE -> 0.
FW_HD int32_t flink_murmur_hash(int32_t code) {
    uint32_t h = murmur_h1(0u, murmur_k1((uint32_t)code));
    h = fmix32(h ^ 4u);
    const int32_t s = (int32_t)h;
    if (s >= 0) return s;
    if (s != INT32_MIN) return -s;
    return 0;
}

enum KeyHashKind : int32_t { KH_LONG = 0, KH_INT = 1, KH_BINROW_BIGINT = 2, KH_BINROW_INT = 3, KH_PRE = 4 };

// key.hashCode() as the reference sees it.
FW_HD int32_t java_key_hash(int32_t kind, int64_t key, int32_t pre) {
    const uint64_t u = (uint64_t)key;
    switch (kind) {
        case KH_LONG: return (int32_t)(uint32_t)(u ^ (u >> 32));
        case KH_INT: return (int32_t)(uint32_t)u;
        case KH_BINROW_BIGINT:
        case KH_BINROW_INT: {
            // 16-byte key row: 8-byte zero header (BinaryRowWriter.reset), then the field slot.
            uint32_t h = 42u;
            h = murmur_h1(h, murmur_k1(0u));
            h = murmur_h1(h, murmur_k1(0u));
            h = murmur_h1(h, murmur_k1((uint32_t)u));
            h = murmur_h1(h, murmur_k1(kind == KH_BINROW_BIGINT ? (uint32_t)(u >> 32) : 0u));
            return (int32_t)fmix32(h ^ 16u);
        }
        default: return pre;
    }
}

// ---------------------------------------------------------------------------------------
// BinaryRowData.hashCode of a general key row (VARCHAR / composite keys), streamed word by
// word from the key's columns without materialising the row.  The row image is the one
// BinaryRowWriter builds (TR/data/writer/BinaryRowWriter.java:39-122, AbstractBinaryWriter.java
// :83-106,242-345; layout BinaryRowData.java:69-124, BinaryFormat.java:30-54):
//   [null bits: ((n + 71) / 64) * 8 B; byte 0 = RowKind (INSERT = 0), bit 8 + i = field i NULL]
//   [n fixed 8-byte slots: NULL -> 0; BOOLEAN/TINYINT/SMALLINT/INT/FLOAT/BIGINT/DOUBLE... -> the
//    value's low `width` bytes (the writer's reset() leaves the rest 0); string of len <= 7 ->
//    bytes little endian | (0x80 | len) << 56; longer -> (offset << 32) | len]
//   [variable part: each longer string's bytes in field order, zero-padded to 8 B]
// and the hash is MurmurHashUtils.hashBytesByWords (seed 42) over all of it (BinaryRowData
// .java:459 -> BinarySegmentUtils.hashByWords).
// ---------------------------------------------------------------------------------------
constexpr int KR_MAX_FIELDS = 8;
struct KeyRowDesc {
    int32_t n;                            // fields
    int32_t width[KR_MAX_FIELDS];         // 1 / 2 / 4 / 8 fixed slot bytes; 0 = string
    const int64_t* fixed[KR_MAX_FIELDS];  // fixed fields: one int64 per row
    const int32_t* offs[KR_MAX_FIELDS];   // strings: n + 1 byte offsets into bytes
    const uint8_t* bytes[KR_MAX_FIELDS];  // strings: 4-byte aligned base
    const uint8_t* nulls[KR_MAX_FIELDS];  // optional NULL flags (non-zero = NULL)
};

// up to 4 bytes of a string at byte p (avail >= 1 of them valid), little endian, zero-padded.
// Device: aligned dword loads (the base is 4-byte aligned; a dword is read only if it holds a
// valid byte); host: byte loads.
FW_HD uint32_t kr_load_word(const uint8_t* base, int64_t p, int64_t avail) {
    uint32_t w;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t* a = (const uint32_t*)(base + (p & ~(int64_t)3));
    const uint32_t sh = (uint32_t)(p & 3) * 8u;
    uint64_t v = a[0] >> sh;
    if (sh && avail > 4 - (int64_t)(p & 3)) v |= (uint64_t)a[1] << (32u - sh);
    w = (uint32_t)v;
#else
    w = 0;
    for (int b = 0; b < 4 && b < avail; b++) w |= (uint32_t)base[p + b] << (8 * b);
#endif
    if (avail < 4) w &= (1u << (8 * avail)) - 1u;
    return w;
}

FW_HD int32_t key_row_hash(const KeyRowDesc& d, int64_t i) {
    const int nb = ((d.n + 71) / 64) * 8;  // BinaryRowData.calculateBitSetWidthInBytes (n <= 56: 8)
    uint64_t hdr = 0;
    for (int f = 0; f < d.n; f++)
        if (d.nulls[f] && d.nulls[f][i]) hdr |= 1ull << (8 + f);
    uint32_t h = 42u;
    h = murmur_h1(h, murmur_k1((uint32_t)hdr));
    h = murmur_h1(h, murmur_k1((uint32_t)(hdr >> 32)));
    uint32_t cursor = (uint32_t)(nb + 8 * d.n);  // the writer's cursor: start of the variable part
    for (int f = 0; f < d.n; f++) {
        uint64_t slot = 0;
        if (!((hdr >> (8 + f)) & 1u)) {
            const int w = d.width[f];
            if (w > 0) {
                const uint64_t v = (uint64_t)d.fixed[f][i];
                slot = w == 8 ? v : v & ((1ull << (8 * w)) - 1ull);
            } else {
                const int64_t o = d.offs[f][i];
                const uint32_t len = (uint32_t)(d.offs[f][i + 1] - o);
                if (len <= 7) {  // writeBytesToFixLenPart
                    slot = (uint64_t)(0x80u | len) << 56;
                    if (len) slot |= kr_load_word(d.bytes[f], o, len);
                    if (len > 4) slot |= (uint64_t)kr_load_word(d.bytes[f], o + 4, len - 4) << 32;
                } else {  // writeBytesToVarLenPart: setOffsetAndSize(pos, cursor, len)
                    slot = ((uint64_t)cursor << 32) | len;
                    cursor += (len + 7u) & ~7u;
                }
            }
        }
        h = murmur_h1(h, murmur_k1((uint32_t)slot));
        h = murmur_h1(h, murmur_k1((uint32_t)(slot >> 32)));
    }
    for (int f = 0; f < d.n; f++) {
        if (d.width[f] > 0 || ((hdr >> (8 + f)) & 1u)) continue;
        const int64_t o = d.offs[f][i];
        const int64_t len = d.offs[f][i + 1] - o;
        if (len <= 7) continue;
        const int64_t padded = (len + 7) & ~(int64_t)7;
        for (int64_t j = 0; j < padded; j += 4)
            h = murmur_h1(h, murmur_k1(j < len ? kr_load_word(d.bytes[f], o + j, len - j) : 0u));
    }
    // the null-bit region beyond the first word (n > 56) is all zero bits here (n <= 8)
    return (int32_t)fmix32(h ^ cursor);
}

// ---- key row images: the bytes BinaryRowWriter writes for a key row (layout above), which the
// SQL operator's state keys on (BinaryRowData.equals compares them byte by byte) ----------------
// length in bytes: fixed part + each long string padded to 8 (always a multiple of 8)
FW_HD int64_t key_row_image_len(const KeyRowDesc& d, int64_t i) {
    int64_t len = ((d.n + 71) / 64) * 8 + 8 * (int64_t)d.n;
    for (int f = 0; f < d.n; f++) {
        if (d.width[f] > 0 || (d.nulls[f] && d.nulls[f][i])) continue;
        const int64_t l = d.offs[f][i + 1] - d.offs[f][i];
        if (l > 7) len += (l + 7) & ~(int64_t)7;
    }
    return len;
}
// row i's image as 8-byte words at out (8-byte aligned)
FW_HD void key_row_image_write(const KeyRowDesc& d, int64_t i, uint64_t* out) {
    uint64_t hdr = 0;
    for (int f = 0; f < d.n; f++)
        if (d.nulls[f] && d.nulls[f][i]) hdr |= 1ull << (8 + f);
    int64_t w = 0;
    out[w++] = hdr;  // n <= 8 < 56: one null-bit word
    uint32_t cursor = (uint32_t)(8 + 8 * d.n);
    for (int f = 0; f < d.n; f++) {
        uint64_t slot = 0;
        if (!((hdr >> (8 + f)) & 1u)) {
            const int wd = d.width[f];
            if (wd > 0) {
                const uint64_t v = (uint64_t)d.fixed[f][i];
                slot = wd == 8 ? v : v & ((1ull << (8 * wd)) - 1ull);
            } else {
                const int64_t o = d.offs[f][i];
                const uint32_t len = (uint32_t)(d.offs[f][i + 1] - o);
                if (len <= 7) {
                    slot = (uint64_t)(0x80u | len) << 56;
                    if (len) slot |= kr_load_word(d.bytes[f], o, len);
                    if (len > 4) slot |= (uint64_t)kr_load_word(d.bytes[f], o + 4, len - 4) << 32;
                } else {
                    slot = ((uint64_t)cursor << 32) | len;
                    cursor += (len + 7u) & ~7u;
                }
            }
        }
        out[w++] = slot;
    }
    for (int f = 0; f < d.n; f++) {
        if (d.width[f] > 0 || ((hdr >> (8 + f)) & 1u)) continue;
        const int64_t o = d.offs[f][i];
        const int64_t len = d.offs[f][i + 1] - o;
        if (len <= 7) continue;
        for (int64_t j = 0; j < len; j += 8) {
            const uint64_t lo = kr_load_word(d.bytes[f], o + j, len - j);
            const uint64_t hi = j + 4 < len ? kr_load_word(d.bytes[f], o + j + 4, len - j - 4) : 0u;
            out[w++] = lo | (hi << 32);
        }
    }
}
// BinaryRowData.hashCode of an image: MurmurHashUtils.hashBytesByWords (seed 42) over its words
FW_HD int32_t key_row_image_hash(const uint64_t* img, int64_t len) {
    uint32_t h = 42u;
    for (int64_t j = 0; j < len / 8; j++) {
        const uint64_t v = img[j];
        h = murmur_h1(h, murmur_k1((uint32_t)v));
        h = murmur_h1(h, murmur_k1((uint32_t)(v >> 32)));
    }
    return (int32_t)fmix32(h ^ (uint32_t)len);
}

// KeyGroupRangeAssignment.computeKeyGroupForKeyHash
FW_HD int32_t key_group_for_hash(int32_t h, int32_t max_p) { return flink_murmur_hash(h) % max_p; }
// KeyGroupRangeAssignment.computeOperatorIndexForKeyGroup
FW_HD int32_t operator_for_key_group(int32_t max_p, int32_t p, int32_t kg) { return kg * p / max_p; }

// 64-bit finaliser used for the build's OWN bucketing (not a Flink-visible hash).
FW_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ---------------------------------------------------------------------------------------
// unsigned 64-bit division by an invariant divisor (round-up magic multiplier)
// ---------------------------------------------------------------------------------------
struct UDiv {
    uint64_t d;
    uint64_t magic;  // 0 => power of two
    uint32_t shift;
    uint32_t add;    // 65-bit variant
};

FW_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

inline UDiv make_udiv(uint64_t d) {  // host only; d > 0
    UDiv r{};
    r.d = d;
    uint32_t l = 63 - (uint32_t)__builtin_clzll(d);
    if ((d & (d - 1)) == 0) {
        r.magic = 0;
        r.shift = l;
        r.add = 0;
        return r;
    }
    const unsigned __int128 num = (unsigned __int128)1 << (64 + l);
    uint64_t m = (uint64_t)(num / d);
    uint64_t rem = (uint64_t)(num - (unsigned __int128)m * d);
    const uint64_t e = d - rem;
    if (e < ((uint64_t)1 << l)) {
        r.shift = l;
        r.add = 0;
    } else {
        m += m;
        const uint64_t twice = rem + rem;
        if (twice >= d || twice < rem) m += 1;
        r.shift = l;
        r.add = 1;
    }
    r.magic = m + 1;
    return r;
}

FW_HD uint64_t udiv(uint64_t x, const UDiv& v) {
    if (v.magic == 0) return x >> v.shift;
    const uint64_t q = mulhi64(v.magic, x);
    if (v.add) return (((x - q) >> 1) + q) >> v.shift;
    return q >> v.shift;
}

// unsigned 32-bit division by an invariant divisor (Granlund-Montgomery round-up multiplier)
struct UDiv32 {
    uint32_t d;
    uint32_t magic;
    uint32_t sh1, sh2;
};

inline UDiv32 make_udiv32(uint32_t d) {  // host only; d > 0
    UDiv32 r{};
    r.d = d;
    uint32_t l = 0;
    while ((1ull << l) < d) l++;  // ceil(log2 d)
    r.magic = (uint32_t)((((uint64_t)1 << 32) * ((1ull << l) - d)) / d + 1);
    r.sh1 = l < 1 ? l : 1;
    r.sh2 = l - r.sh1;
    return r;
}

FW_HD uint32_t udiv32(uint32_t n, const UDiv32& v) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t t = __umulhi(v.magic, n);
#else
    const uint32_t t = (uint32_t)(((uint64_t)v.magic * n) >> 32);
#endif
    return (t + ((n - t) >> v.sh1)) >> v.sh2;
}

// TimeWindow.getWindowStartWithOffset(ts, offset, size) with Java long semantics.
FW_HD int64_t window_start(int64_t ts, int64_t offset, const UDiv& size) {
    const uint64_t x = (uint64_t)ts - (uint64_t)offset;
    const bool neg = (int64_t)x < 0;
    const uint64_t ax = neg ? (0ull - x) : x;
    const uint64_t r = ax - udiv(ax, size) * size.d;  // |x| % size
    if (neg && r != 0) return (int64_t)((uint64_t)ts - (size.d - r));  // ts - (rem + size)
    return (int64_t)((uint64_t)ts - r);
}

FW_HD int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
FW_HD int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

// TimeWindowUtil.isWindowFired, UTC shift zone: progress >= windowEnd - 1 (MAX never fires).
FW_HD bool is_fired(int64_t window_end, int64_t progress) {
    if (window_end == INT64_MAX) return false;
    return progress >= wsub(window_end, 1);
}

// TimeWindowUtil.getNextTriggerWatermark (no daylight saving).
FW_HD int64_t next_trigger_watermark(int64_t wm, const UDiv& interval) {
    if (wm == INT64_MAX) return wm;
    const int64_t start = window_start(wm, 0, interval);
    const int64_t trig = wsub(wadd(start, (int64_t)interval.d), 1);
    return trig > wm ? trig : wadd(trig, (int64_t)interval.d);
}

// ---------------------------------------------------------------------------------------
// Shift time zone of a TIMESTAMP_LTZ window (TR/util/TimeWindowUtil.java:52-211).  The zone is a
// piecewise-constant UTC offset table (the caller expands java.time ZoneRules into it):
//   from UTC instant utc[i] on (utc[0] = Long.MIN_VALUE) the offset is off[i] ms, and
//   bound[i] = utc[i] + max(off[i-1], off[i]) (bound[0] = MIN) is the first local time that
//   LocalDateTime.atZone maps with off[i]: a local time in a gap maps with the offset before the
//   gap (ZonedDateTime.ofLocal moves it later by the gap length and takes the later offset, which
//   is the same instant), a local time in an overlap with the earlier offset.
// n == 0 is the UTC zone (TIMESTAMP rowtime): every conversion is the identity.
// ---------------------------------------------------------------------------------------
struct TzTable {
    const int64_t* utc;
    const int64_t* off;
    const int64_t* bound;
    int32_t n;
    int32_t dst;  // TimeZone.getTimeZone(zone).useDaylightTime()
};

// last i with a[i] <= x (a[0] = INT64_MIN, ascending)
FW_HD int tz_find(const int64_t* a, int n, int64_t x) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// TimeWindowUtil.toUtcTimestampMills (:52-60): the local wall-clock millis of an epoch instant
FW_HD int64_t tz_to_utc_ts(const TzTable& z, int64_t epoch) {
    if (z.n == 0 || epoch == INT64_MAX) return epoch;
    return wadd(epoch, z.off[tz_find(z.utc, z.n, epoch)]);
}
// LocalDateTime.atZone(zone).toInstant().toEpochMilli() of a local wall-clock millis value
FW_HD int64_t tz_local_to_epoch(const TzTable& z, int64_t local) {
    return wsub(local, z.off[tz_find(z.bound, z.n, local)]);
}
// TimeWindowUtil.toEpochMillsForTimer (:69-140): the timer instant of a local timestamp; in a DST
// gap the first skipped instant's hour, in an overlap the later of the two instants
FW_HD int64_t tz_epoch_for_timer(const TzTable& z, int64_t local) {
    if (z.n == 0 || local == INT64_MAX) return local;
    const int64_t t1 = tz_local_to_epoch(z, local);
    if (!z.dst) return t1;
    const int64_t hour = 3600000;
    const int64_t t2 = tz_local_to_epoch(z, wadd(local, hour));
    if (t1 == t2) return wsub(t1, t1 % hour);  // Java % truncates toward zero, as C++
    if (wsub(t2, t1) > hour) return wadd(t1, hour);
    return t1;
}

// TimeWindowUtil.isWindowFired (:175-183) in a shift time zone
FW_HD bool tz_is_fired(const TzTable& z, int64_t window_end, int64_t progress) {
    if (window_end == INT64_MAX) return false;
    return progress >= tz_epoch_for_timer(z, wsub(window_end, 1));
}

// TimeWindowUtil.getNextTriggerWatermark (:186-211) with the shift zone's useDaylightTime(); a
// zone without daylight saving (and UTC) takes the epoch-space branch, as the reference does
FW_HD int64_t tz_next_trigger_watermark(const TzTable& z, int64_t wm, const UDiv& interval) {
    if (wm == INT64_MAX) return wm;
    if (z.n == 0 || !z.dst) return next_trigger_watermark(wm, interval);
    const int64_t start = window_start(tz_to_utc_ts(z, wm), 0, interval);
    const int64_t trig = tz_epoch_for_timer(z, wsub(wadd(start, (int64_t)interval.d), 1));
    return trig > wm ? trig : wadd(trig, (int64_t)interval.d);
}

// Sortable 64-bit key of a double (total order of Double.compare: NaN canonicalised, greatest).
FW_HD int64_t dkey(uint64_t bits) {
    if ((bits & 0x7FF0000000000000ull) == 0x7FF0000000000000ull && (bits & 0x000FFFFFFFFFFFFFull))
        bits = 0x7FF8000000000000ull;
    const int64_t s = (int64_t)bits;
    return s ^ (int64_t)(((uint64_t)(s >> 63)) >> 1);
}
FW_HD uint64_t dkey_inv(int64_t k) { return (uint64_t)(k ^ (int64_t)(((uint64_t)(k >> 63)) >> 1)); }

}  // namespace fw
