"""ctypes mirror of include/flinkwin.h (the C-ABI of libflinkwin).

Only plain data types live here so both the product bindings (flink_amd._native) and the
test-side oracle wrapper can build the same ``fw_config`` structure.
"""
import ctypes as C

FW_ABI_VERSION = 10
FW_MAX_AGGS = 8
FW_MAX_COLS = 8

FW_OK = 0
FW_E_INVALID = -1
FW_E_DEVICE = -2
FW_E_CAPACITY = -3
FW_E_STATE = -4
FW_E_NOMEM = -5

# fw_api_kind
API_SQL = 0
API_DATASTREAM = 1
# fw_window_kind
WIN_TUMBLE = 0
WIN_HOP = 1
WIN_CUMULATE = 2
# fw_agg_kind
AGG_COUNT_STAR = 0
AGG_COUNT = 1
AGG_SUM = 2
AGG_MIN = 3
AGG_MAX = 4
AGG_AVG = 5
AGG_MINBY = 6  # DataStream minBy / maxBy: the extremal element (ComparableAggregator byAggregate)
AGG_MAXBY = 7
AGGF_LAST = 1  # fw_agg_desc.flags: ties go to the last element (minBy / maxBy(field, first=false))
# fw_agg_phase (TwoStageOptimizedWindowAggregateRule: one-phase, or local + global)
PHASE_ONE = 0
PHASE_LOCAL = 1
PHASE_GLOBAL = 2
# fw_value_type
T_I64 = 0
T_F64 = 1
T_I32 = 2
# fw_key_hash_kind
KEYHASH_LONG = 0
KEYHASH_INT = 1
KEYHASH_BINROW_BIGINT = 2
KEYHASH_BINROW_INT = 3
KEYHASH_PRECOMPUTED = 4
KEYHASH_KEYROW = 5

# fw_stats.error_flags bits (FW_ERRF_*)
ERRF = {"CHUNKS": 1, "STATE": 2, "OUTPUT": 4, "TREQ": 8, "KEYGROUP": 16, "LATE": 32, "ORDEV": 64, "KEYROW": 128}

# fw_key_field_kind (key-row fields for fw_key_row_hash)
KF_STRING, KF_FIXED1, KF_FIXED2, KF_FIXED4, KF_FIXED8 = 0, 1, 2, 4, 8
FW_MAX_KEY_FIELDS = 8
# SQL key field type -> fw_key_field_kind (BinaryRowWriter slot width; strings go to the var part)
KEY_FIELD_KINDS = {"BOOLEAN": KF_FIXED1, "TINYINT": KF_FIXED1, "SMALLINT": KF_FIXED2, "INT": KF_FIXED4,
                   "DATE": KF_FIXED4, "FLOAT": KF_FIXED4, "BIGINT": KF_FIXED8, "DOUBLE": KF_FIXED8,
                   "TIMESTAMP": KF_FIXED8, "VARCHAR": KF_STRING, "CHAR": KF_STRING, "STRING": KF_STRING,
                   "VARBINARY": KF_STRING, "BINARY": KF_STRING, "BYTES": KF_STRING}

AGG_NAMES = {"COUNT_STAR": AGG_COUNT_STAR, "COUNT": AGG_COUNT, "SUM": AGG_SUM,
             "MIN": AGG_MIN, "MAX": AGG_MAX, "AVG": AGG_AVG}
TYPE_NAMES = {"BIGINT": T_I64, "DOUBLE": T_F64, "INT": T_I32}
WINDOW_NAMES = {"TUMBLE": WIN_TUMBLE, "HOP": WIN_HOP, "CUMULATE": WIN_CUMULATE}


class fw_agg_desc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("input_col", C.c_int32), ("type", C.c_int32),
                ("flags", C.c_int32)]


class fw_config(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32),
        ("api", C.c_int32),
        ("window_kind", C.c_int32),
        ("key_hash", C.c_int32),
        ("size_ms", C.c_int64),
        ("slide_ms", C.c_int64),
        ("offset_ms", C.c_int64),
        ("n_aggs", C.c_int32),
        ("count_star_index", C.c_int32),
        ("aggs", fw_agg_desc * FW_MAX_AGGS),
        ("n_value_cols", C.c_int32),
        ("value_col_types", C.c_int32 * FW_MAX_COLS),
        ("nullable_cols", C.c_uint32),
        ("agg_phase", C.c_int32),
        ("max_parallelism", C.c_int32),
        ("parallelism", C.c_int32),
        ("subtask_index", C.c_int32),
        ("device", C.c_int32),
        ("ds_first_ordinals", C.c_int32),
        ("state_capacity", C.c_int64),
        ("max_batch_rows", C.c_int64),
        ("output_capacity", C.c_int64),
        ("allowed_lateness_ms", C.c_int64),
        ("late_side_output", C.c_int32),
        ("tz_use_dst", C.c_int32),
        ("tz_n", C.c_int32),
        ("key_row_max_bytes", C.c_int32),
        ("tz_utc", C.POINTER(C.c_int64)),
        ("tz_offset_ms", C.POINTER(C.c_int64)),
    ]


class fw_key_field(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32), ("fixed", C.c_void_p),
                ("offsets", C.c_void_p), ("bytes", C.c_void_p), ("nulls", C.c_void_p)]


class fw_heap_state_ids(C.Structure):
    """state ids of the heap backend's key-group data (HeapSnapshotStrategy.java:171)"""
    _fields_ = [("window_state", C.c_int16), ("event_timers", C.c_int16),
                ("processing_timers", C.c_int16), ("reserved", C.c_int16)]


DSW_CONTENTS, DSW_TRIGGER, DSW_CLEANUP = 1, 2, 4


class fw_ds_window(C.Structure):
    """one (key, window) of a DataStream WindowOperator key group (flinkwin.h fw_ds_snapshot_key_group)"""
    _fields_ = [("key", C.c_int64), ("window_end", C.c_int64), ("value", C.c_int64), ("first_ord", C.c_int64),
                ("flags", C.c_int32), ("key_hash", C.c_int32)]


class fw_host_cols(C.Structure):
    _fields_ = [("key", C.POINTER(C.c_int64)), ("ts", C.POINTER(C.c_int64)),
                ("key_hash", C.POINTER(C.c_int32)),
                ("values", C.POINTER(C.c_int64) * FW_MAX_COLS),
                ("nulls", C.POINTER(C.c_uint8) * FW_MAX_COLS),
                ("key_row_offsets", C.POINTER(C.c_int64)), ("key_row_bytes", C.POINTER(C.c_uint8)),
                ("key_row_bytes_cap", C.c_int64)]


class fw_result(C.Structure):
    _fields_ = [("n", C.c_int64), ("key", C.POINTER(C.c_int64)),
                ("window_start", C.POINTER(C.c_int64)), ("window_end", C.POINTER(C.c_int64)),
                ("values", C.POINTER(C.c_int64) * FW_MAX_AGGS),
                ("null_mask", C.POINTER(C.c_uint32)), ("first_ord", C.POINTER(C.c_int64)),
                ("key_row_len", C.POINTER(C.c_int32)), ("key_row_bytes", C.POINTER(C.c_uint8)),
                ("key_row_stride", C.c_int64)]


class fw_result_segments(C.Structure):
    """flinkwin.h fw_results_device_segments: per-superbucket result slabs, no copy"""
    _fields_ = [("n_segments", C.c_int64), ("seg_cap", C.c_int64), ("counts", C.c_void_p),
                ("cols", fw_result)]


class fw_ordinal_events(C.Structure):
    _fields_ = [("n_retain", C.c_int64), ("retain", C.POINTER(C.c_int64)),
                ("n_release", C.c_int64), ("release", C.POINTER(C.c_int64))]


class fw_late_rows(C.Structure):
    _fields_ = [("n", C.c_int64), ("key", C.POINTER(C.c_int64)), ("ts", C.POINTER(C.c_int64)),
                ("values", C.POINTER(C.c_int64) * FW_MAX_COLS), ("push_seq", C.POINTER(C.c_int64)),
                ("row", C.POINTER(C.c_int64))]


class fw_stats(C.Structure):
    _fields_ = [("current_watermark", C.c_int64), ("next_trigger_progress", C.c_int64),
                ("num_late_records_dropped", C.c_int64), ("live_state_entries", C.c_int64),
                ("pending_rows", C.c_int64), ("results_available", C.c_int64),
                ("num_fired_windows", C.c_int64), ("partials_emitted", C.c_int64),
                ("error_flags", C.c_int32),
                ("num_superbuckets", C.c_int32),
                ("flush_launches", C.c_int64), ("partials_merged", C.c_int64),
                ("state_entries_moved", C.c_int64), ("key_rows", C.c_int64),
                ("key_row_collections", C.c_int64),
                ("partial_bytes_written", C.c_int64), ("partial_bytes_merged", C.c_int64),
                ("compact_chunks", C.c_int64),
                ("peak_superbucket_entries", C.c_int64), ("superbucket_capacity", C.c_int32),
                ("reserved_stats0", C.c_int32)]


KT_PARTITION, KT_SCAN, KT_REDUCE, KT_MERGE, KT_OTHER = 0, 1, 2, 3, 4
FW_KT_N = 8


class fw_kernel_times(C.Structure):
    _fields_ = [("ms", C.c_double * FW_KT_N), ("launches", C.c_int64 * FW_KT_N),
                ("merge_phase_cycles", C.c_int64 * FW_KT_N)]


class fw_gen_params(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("t0_ms", C.c_int64), ("rate_per_s", C.c_int64),
                ("ooo_ms", C.c_int64), ("key_base", C.c_int64), ("key_count", C.c_int64),
                ("key_dist", C.c_int32), ("value_kind", C.c_int32),
                ("zipf_cdf", C.c_void_p)]


def make_config(*, api=API_SQL, window_kind=WIN_TUMBLE, size_ms, slide_ms=0, offset_ms=0,
                aggs=(), count_star_index=-1, value_col_types=(), key_hash=KEYHASH_BINROW_BIGINT,
                max_parallelism=128, parallelism=1, subtask_index=0, device=0,
                state_capacity=1 << 20, max_batch_rows=1 << 22, output_capacity=1 << 22,
                nullable_cols=(), agg_phase=PHASE_ONE, allowed_lateness_ms=0, late_side_output=False,
                shift_zone=None, ds_first_ordinals=False, key_row_max_bytes=0):
    """Build an fw_config.  ``aggs`` is a sequence of (kind, input_col, type); ``nullable_cols``
    the value columns that may hold SQL NULLs; ``shift_zone`` a TIMESTAMP_LTZ window's time zone
    (a zone name, or a ShiftZone from flink_amd.table.time_zone; None / "UTC": no shift)."""
    if len(aggs) > FW_MAX_AGGS or len(value_col_types) > FW_MAX_COLS:
        raise ValueError("too many aggregates or value columns")
    c = fw_config()
    c.abi_version = FW_ABI_VERSION
    c.api = api
    c.window_kind = window_kind
    c.key_hash = key_hash
    c.size_ms = size_ms
    c.slide_ms = slide_ms
    c.offset_ms = offset_ms
    c.n_aggs = len(aggs)
    c.count_star_index = count_star_index
    for i, agg in enumerate(aggs):
        kind, col, typ = agg[:3]
        c.aggs[i].kind = kind
        c.aggs[i].input_col = col
        c.aggs[i].type = typ
        c.aggs[i].flags = agg[3] if len(agg) > 3 else 0
    c.n_value_cols = len(value_col_types)
    for i, t in enumerate(value_col_types):
        c.value_col_types[i] = t
    c.nullable_cols = sum(1 << int(col) for col in nullable_cols)
    c.agg_phase = agg_phase
    c.max_parallelism = max_parallelism
    c.parallelism = parallelism
    c.subtask_index = subtask_index
    c.device = device
    c.state_capacity = state_capacity
    c.max_batch_rows = max_batch_rows
    c.output_capacity = output_capacity
    c.allowed_lateness_ms = allowed_lateness_ms
    c.late_side_output = 1 if late_side_output else 0
    c.ds_first_ordinals = 1 if ds_first_ordinals else 0
    c.key_row_max_bytes = key_row_max_bytes
    set_shift_zone(c, shift_zone)
    return c


def set_shift_zone(c, zone):
    """Attach a shift time zone's offset table to a config (the arrays are kept alive on it)."""
    if zone is None or zone == "UTC":
        c.tz_n, c.tz_use_dst = 0, 0
        c.tz_utc = C.POINTER(C.c_int64)()
        c.tz_offset_ms = C.POINTER(C.c_int64)()
        c._zone = None
        return
    if isinstance(zone, str):
        from .table.time_zone import ShiftZone
        zone = ShiftZone.of(zone)
    n = len(zone.utc)
    utc = (C.c_int64 * n)(*zone.utc)
    off = (C.c_int64 * n)(*zone.offset_ms)
    c._zone = (zone, utc, off)  # keeps the arrays alive while the config is
    c.tz_n = n
    c.tz_use_dst = 1 if zone.use_dst else 0
    c.tz_utc = C.cast(utc, C.POINTER(C.c_int64))
    c.tz_offset_ms = C.cast(off, C.POINTER(C.c_int64))


def result_columns(cfg):
    """Result value columns of an operator: one per aggregate, or (LOCAL phase) the local
    accumulator fields -- COUNT(*) / COUNT / SUM / MIN / MAX: one, AVG: sum and count."""
    if cfg.agg_phase != PHASE_LOCAL:
        return cfg.n_aggs
    return sum(2 if cfg.aggs[i].kind == AGG_AVG else 1 for i in range(cfg.n_aggs))


def global_config(cfg, **overrides):
    """The GLOBAL-phase operator of a two-phase plan (TwoStageOptimizedWindowAggregateRule): same
    window, key and aggregates, fed with the LOCAL phase's accumulator rows -- value column j is
    accumulator field j (see result_columns), SUM / MIN / MAX fields NULL-able; the ts column
    carries the slice end.  With NOT NULL inputs (cfg.nullable_cols == 0) no field is NULL-able:
    the LOCAL phase emits a (key, slice) partial only for a slice that received a record, so its
    SUM / MIN / MAX are never NULL."""
    aggs, types, nullable, j = [], [], [], 0
    for i in range(cfg.n_aggs):
        kind, typ = cfg.aggs[i].kind, cfg.aggs[i].type
        aggs.append((kind, j, typ))
        if kind in (AGG_COUNT_STAR, AGG_COUNT):
            types.append(T_I64)
        elif kind == AGG_AVG:
            types += [T_F64 if typ == T_F64 else T_I64, T_I64]
        else:
            types.append(typ)
            if cfg.nullable_cols:
                nullable.append(j)
        j += 2 if kind == AGG_AVG else 1
    kw = dict(api=cfg.api, window_kind=cfg.window_kind, size_ms=cfg.size_ms, slide_ms=cfg.slide_ms,
              offset_ms=cfg.offset_ms, aggs=aggs, count_star_index=cfg.count_star_index, value_col_types=types,
              key_hash=cfg.key_hash, max_parallelism=cfg.max_parallelism, parallelism=cfg.parallelism,
              subtask_index=cfg.subtask_index, device=cfg.device, state_capacity=cfg.state_capacity,
              max_batch_rows=cfg.max_batch_rows, output_capacity=cfg.output_capacity, nullable_cols=nullable,
              agg_phase=PHASE_GLOBAL, shift_zone=getattr(cfg, "_zone", None) and cfg._zone[0])
    kw.update(overrides)
    return make_config(**kw)


def result_is_double(kind, typ):
    """Whether an aggregate's SQL/DataStream result column is DOUBLE."""
    if kind in (AGG_COUNT_STAR, AGG_COUNT):
        return False
    return typ == T_F64
