// ORACLE -- TEST INFRASTRUCTURE ONLY.  Sanitizer driver: runs the oracle's C ABI over seeded
// random streams for every window kind, API, aggregation phase and value type, with SQL NULLs,
// NaN / +-0.0 doubles, late records, flushes and snapshot/restore cuts.  Built with
// AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle san`) and run by
// tests/test_oracle_sanitize.py; any report aborts the process (-fno-sanitize-recover).
// Prints one line per scenario with its result count, so the run is also a smoke check.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/flinkwin.h"

extern "C" {
void* or_create(const fw_config* c);
void or_destroy(void* h);
void or_initialize_watermark(void* h, int64_t wm);
int64_t or_process_batch(void* h, int64_t n, const int64_t* key, const int64_t* ts, const uint64_t* vals, int32_t ncols,
                         const uint8_t* nulls);
void or_process_watermark(void* h, int64_t wm);
void or_flush(void* h);
void or_snapshot_restore(void* h);
int64_t or_num_results(void* h);
int32_t or_num_value_columns(void* h);
void or_get_results(void* h, int64_t* key, int64_t* ws, int64_t* we, uint64_t* vals, uint32_t* nm, int64_t* epoch);
void or_clear_results(void* h);
int32_t or_key_group(int32_t kind, int64_t key, int32_t pre, int32_t max_p);
}

namespace {

uint64_t g_rng = 0x2545F4914F6CDD1DULL;
uint64_t rnd() {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return g_rng;
}

uint64_t dbits(double d) {
    uint64_t b;
    memcpy(&b, &d, 8);
    return b;
}

struct Scenario {
    const char* name;
    int api, kind, phase;
    int64_t size, slide, offset;
};

fw_config base_config(const Scenario& s) {
    fw_config c;
    memset(&c, 0, sizeof c);
    c.abi_version = FW_ABI_VERSION;
    c.api = s.api;
    c.window_kind = s.kind;
    c.key_hash = s.api == FW_API_SQL ? FW_KEYHASH_BINROW_BIGINT : FW_KEYHASH_LONG;
    c.size_ms = s.size;
    c.slide_ms = s.slide;
    c.offset_ms = s.offset;
    c.count_star_index = -1;
    c.max_parallelism = 128;
    c.parallelism = 1;
    c.agg_phase = s.phase;
    c.state_capacity = 1 << 16;
    c.max_batch_rows = 1 << 12;
    c.output_capacity = 1 << 20;
    if (s.api == FW_API_DATASTREAM) {  // one aggregate over one column
        c.n_aggs = 1;
        c.aggs[0] = {FW_AGG_MAX, 0, FW_T_I64, 0};
        c.n_value_cols = 1;
        c.value_col_types[0] = FW_T_I64;
        return c;
    }
    // SQL: every aggregate kind over BIGINT, INT and DOUBLE columns, DOUBLE / INT nullable
    c.n_value_cols = 3;
    c.value_col_types[0] = FW_T_I64;
    c.value_col_types[1] = FW_T_F64;
    c.value_col_types[2] = FW_T_I32;
    c.nullable_cols = (1u << 1) | (1u << 2);
    const fw_agg_desc aggs[] = {
        {FW_AGG_COUNT_STAR, 0, FW_T_I64, 0}, {FW_AGG_SUM, 0, FW_T_I64, 0}, {FW_AGG_MAX, 1, FW_T_F64, 0},
        {FW_AGG_MIN, 1, FW_T_F64, 0},        {FW_AGG_AVG, 2, FW_T_I32, 0}, {FW_AGG_COUNT, 1, FW_T_F64, 0},
        {FW_AGG_SUM, 1, FW_T_F64, 0},        {FW_AGG_MIN, 2, FW_T_I32, 0},
    };
    c.n_aggs = s.phase == FW_PHASE_LOCAL ? 7 : 8;  // LOCAL: at most FW_MAX_COLS accumulator fields
    for (int a = 0; a < c.n_aggs; a++) c.aggs[a] = aggs[a];
    c.count_star_index = 0;
    return c;
}

// the GLOBAL-phase config of a LOCAL config (flink_amd/abi.py global_config)
fw_config global_of(const fw_config& l) {
    fw_config g = l;
    g.agg_phase = FW_PHASE_GLOBAL;
    g.nullable_cols = 0;
    int j = 0;
    for (int a = 0; a < l.n_aggs; a++) {
        const int kind = l.aggs[a].kind, typ = l.aggs[a].type;
        g.aggs[a].input_col = j;
        if (kind == FW_AGG_COUNT_STAR || kind == FW_AGG_COUNT) {
            g.value_col_types[j] = FW_T_I64;
        } else if (kind == FW_AGG_AVG) {
            g.value_col_types[j] = typ == FW_T_F64 ? FW_T_F64 : FW_T_I64;
            g.value_col_types[j + 1] = FW_T_I64;
        } else {
            g.value_col_types[j] = typ;
            g.nullable_cols |= 1u << j;
        }
        j += kind == FW_AGG_AVG ? 2 : 1;
    }
    g.n_value_cols = j;
    return g;
}

uint64_t random_value(int type) {
    if (type != FW_T_F64) return (uint64_t)(int64_t)((int64_t)(rnd() % 2001) - 1000);
    switch (rnd() % 16) {
        case 0: return dbits(NAN);
        case 1: return dbits(0.0);
        case 2: return dbits(-0.0);
        case 3: return dbits(INFINITY);
        default: return dbits(((double)(rnd() % 100000) - 50000.0) / 7.0);
    }
}

// one batch of n rows, event time around t with out-of-orderness, SoA value / null columns
void make_batch(const fw_config& c, int64_t n, int64_t t, int64_t ooo, std::vector<int64_t>& k,
                std::vector<int64_t>& ts, std::vector<uint64_t>& v, std::vector<uint8_t>& nl) {
    k.resize(n);
    ts.resize(n);
    v.assign((size_t)n * c.n_value_cols, 0);
    nl.assign((size_t)n * c.n_value_cols, 0);
    for (int64_t i = 0; i < n; i++) {
        k[i] = (int64_t)(rnd() % 97) - 40;
        ts[i] = t + (int64_t)(rnd() % (uint64_t)(2 * ooo + 1)) - ooo;
        for (int col = 0; col < c.n_value_cols; col++) {
            v[(size_t)col * n + i] = random_value(c.value_col_types[col]);
            if ((c.nullable_cols >> col) & 1u) nl[(size_t)col * n + i] = rnd() % 5 == 0;
        }
    }
}

struct Results {
    std::vector<int64_t> key, ws, we, epoch;
    std::vector<uint64_t> vals;
    std::vector<uint32_t> nm;
    int ncols = 0;
};

Results take(void* h) {
    Results r;
    const int64_t n = or_num_results(h);
    r.ncols = or_num_value_columns(h);
    r.key.resize(n);
    r.ws.resize(n);
    r.we.resize(n);
    r.epoch.resize(n);
    r.nm.resize(n);
    r.vals.resize((size_t)n * r.ncols);
    or_get_results(h, r.key.data(), r.ws.data(), r.we.data(), r.vals.data(), r.nm.data(), r.epoch.data());
    or_clear_results(h);
    return r;
}

int64_t run(const Scenario& s) {
    fw_config c = base_config(s);
    void* h = or_create(&c);
    if (!h) {
        fprintf(stderr, "%s: or_create failed\n", s.name);
        exit(2);
    }
    void* g = nullptr;
    fw_config gc;
    if (s.phase == FW_PHASE_LOCAL) {
        gc = global_of(c);
        g = or_create(&gc);
    }
    std::vector<int64_t> k, ts;
    std::vector<uint64_t> v;
    std::vector<uint8_t> nl;
    int64_t total = 0, t = 1600000000000LL;
    const int64_t ooo = 2 * s.size;
    for (int b = 0; b < 40; b++) {
        const int64_t n = 1 + (int64_t)(rnd() % 700);
        make_batch(c, n, t, ooo, k, ts, v, nl);
        or_process_batch(h, n, k.data(), ts.data(), v.data(), c.n_value_cols,
                         c.nullable_cols ? nl.data() : nullptr);
        t += 1 + (int64_t)(rnd() % (uint64_t)s.size);
        const int64_t wm = t - ooo;
        if (b % 7 == 3 && s.phase != FW_PHASE_LOCAL) or_snapshot_restore(h);
        if (b % 11 == 5) or_flush(h);
        or_process_watermark(h, wm);
        Results r = take(h);
        total += (int64_t)r.key.size();
        if (g && !r.key.empty()) {  // LOCAL partials feed the GLOBAL phase: ts = slice end
            const int64_t m = (int64_t)r.key.size();
            std::vector<uint8_t> gn((size_t)m * gc.n_value_cols, 0);
            for (int col = 0; col < gc.n_value_cols; col++)
                if ((gc.nullable_cols >> col) & 1u)
                    for (int64_t i = 0; i < m; i++) gn[(size_t)col * m + i] = (r.nm[i] >> col) & 1u;
            or_process_batch(g, m, r.key.data(), r.we.data(), r.vals.data(), gc.n_value_cols, gn.data());
            or_process_watermark(g, wm);
            total += (int64_t)take(g).key.size();
        }
    }
    or_process_watermark(h, INT64_MAX);
    total += (int64_t)take(h).key.size();
    if (g) {
        or_process_watermark(g, INT64_MAX);
        total += (int64_t)take(g).key.size();
        or_destroy(g);
    }
    or_destroy(h);
    return total;
}

}  // namespace

int main() {
    const Scenario sc[] = {
        {"sql_tumble", FW_API_SQL, FW_WIN_TUMBLE, FW_PHASE_ONE, 1000, 0, 0},
        {"sql_tumble_offset", FW_API_SQL, FW_WIN_TUMBLE, FW_PHASE_ONE, 1000, 0, 300},
        {"sql_hop", FW_API_SQL, FW_WIN_HOP, FW_PHASE_ONE, 3000, 1000, 0},
        {"sql_cumulate", FW_API_SQL, FW_WIN_CUMULATE, FW_PHASE_ONE, 3000, 1000, 0},
        {"sql_two_phase_tumble", FW_API_SQL, FW_WIN_TUMBLE, FW_PHASE_LOCAL, 1000, 0, 0},
        {"sql_two_phase_hop", FW_API_SQL, FW_WIN_HOP, FW_PHASE_LOCAL, 3000, 1000, 0},
        {"sql_two_phase_cumulate", FW_API_SQL, FW_WIN_CUMULATE, FW_PHASE_LOCAL, 3000, 1000, 0},
        {"ds_tumble", FW_API_DATASTREAM, FW_WIN_TUMBLE, FW_PHASE_ONE, 1000, 0, 0},
        {"ds_sliding", FW_API_DATASTREAM, FW_WIN_HOP, FW_PHASE_ONE, 3000, 1000, 0},
    };
    for (const Scenario& s : sc) printf("%s %lld\n", s.name, (long long)run(s));
    // key-group restatements over extreme keys (integer overflow paths)
    const int64_t keys[] = {0, -1, 1, INT64_MIN, INT64_MAX, (int64_t)0x80000000LL, -(int64_t)0x80000000LL};
    int64_t acc = 0;
    for (int64_t key : keys)
        for (int kind = FW_KEYHASH_LONG; kind <= FW_KEYHASH_BINROW_INT; kind++) acc += or_key_group(kind, key, 0, 32768);
    printf("key_groups %lld\n", (long long)acc);
    return 0;
}
