"""GPU-backed drop-in for the SQL slicing window aggregate operator.

Mirrors WindowAggOperator (flink-table-runtime/.../window/tvf/common/WindowAggOperator.java:96-265)
driving a SlicingSyncStateWindowProcessor built by WindowAggOperatorBuilder
(.../aggregate/window/WindowAggOperatorBuilder.java:181-260).  Records are processed per
columnar batch (the rows buffered between two watermarks, exactly what RecordsWindowBuffer
holds); processWatermark returns the rows the reference emits for that watermark, before the
watermark is forwarded.  Output rows are key ++ aggs ++ (window_start, window_end)
(WindowAggProcessorBase.collect :116-119 with the window properties of
AggsHandlerCodeGenerator.scala:1092-1125).
"""
import numpy as np

from .. import abi
from ..runtime.handle import WindowAggHandle
from ..runtime.options import gpu_enabled
from .key_rows import KeyRowColumns, decode_key_row
from .slice_assigners import SliceAssigner

GPU_AGGS = {"COUNT_STAR", "COUNT", "SUM", "MIN", "MAX", "AVG"}
GPU_TYPES = {"BIGINT", "INT", "DOUBLE"}
KEY_HASH = {"BIGINT": abi.KEYHASH_BINROW_BIGINT, "INT": abi.KEYHASH_BINROW_INT,
            "HOST_HASHED": abi.KEYHASH_PRECOMPUTED}


def is_gpu_eligible(assigner, aggs, value_types, *, is_event_time=True, shift_time_zone="UTC",
                    has_distinct=False, needs_retraction=False, key_type="BIGINT", conf=None):
    """The builder-seam eligibility rule: rowtime (TIMESTAMP, or TIMESTAMP_LTZ with
    any shift time zone), built-in SUM/COUNT/COUNT(*)/MIN/MAX/AVG on numeric columns, no DISTINCT /
    retraction / UDAF.  ``conf``: the job configuration the builder passes (runtime/options.py):
    ``gpu.window-agg.enabled`` must be true (default false); None = the caller already chose the
    GPU operator.  Returns (ok, reason); callers fall back to the reference processor when not ok."""
    if conf is not None and not gpu_enabled(conf):
        return False, "gpu.window-agg.enabled is false"
    if not isinstance(assigner, SliceAssigner):
        return False, "not a slicing assigner"
    if not is_event_time or not assigner.is_event_time():
        return False, "processing-time windows run on the reference operator"
    if shift_time_zone not in (None, "UTC"):
        try:
            from .time_zone import ShiftZone
            ShiftZone.of(shift_time_zone)
        except Exception:
            return False, f"unknown shift time zone {shift_time_zone}"
    if has_distinct or needs_retraction:
        return False, "DISTINCT / retraction aggregates run on the reference operator"
    if isinstance(key_type, (tuple, list)):  # key row of several / non-integer fields (fw_key_row_hash)
        if not 1 <= len(key_type) <= abi.FW_MAX_KEY_FIELDS:
            return False, f"key rows of {len(key_type)} fields run on the reference operator"
        bad = [t for t in key_type if t not in abi.KEY_FIELD_KINDS]
        if bad:
            return False, f"key field type {bad[0]} runs on the reference operator"
    elif key_type not in KEY_HASH:
        return False, f"key type {key_type} must be host-hashed"
    for kind, col, typ in aggs:
        if kind not in GPU_AGGS:
            return False, f"aggregate {kind} is not a built-in GPU aggregate"
        if kind != "COUNT_STAR" and (typ not in GPU_TYPES or value_types[col] != typ):
            return False, f"aggregate input type {typ} not supported on the GPU"
    return True, ""


class WindowAggOperator:
    def __init__(self, assigner, aggs, value_types, count_star_index=-1, key_type="BIGINT",
                 max_parallelism=128, parallelism=1, subtask_index=0, device=0,
                 state_capacity=1 << 20, max_batch_rows=1 << 22, output_capacity=1 << 22,
                 nullable_cols=(), key_row_max_bytes=0):
        """``assigner``: a SliceAssigner; a TIMESTAMP_LTZ window's assigner carries its shift time
        zone (``assigner.in_zone(zone)``, SliceAssigners.*(rowtimeIndex, shiftTimeZone, ...))."""
        zone = assigner.shift_zone
        ok, why = is_gpu_eligible(assigner, aggs, value_types, key_type=key_type,
                                  shift_time_zone=zone.name if zone is not None else "UTC")
        if not ok:
            raise ValueError(f"not eligible for the GPU window operator: {why}")
        if assigner.kind == abi.WIN_HOP and count_star_index < 0:
            raise ValueError("Hopping window requires a COUNT(*) in the aggregate functions.")
        self.assigner = assigner
        self.aggs = list(aggs)
        # key rows (VARCHAR / composite keys): the BinaryRowData images go to the device, which keys
        # the state on their bytes and routes by their hashCode (FW_KEYHASH_KEYROW)
        self.key_types = list(key_type) if isinstance(key_type, (tuple, list)) else None
        self.cfg = abi.make_config(
            api=abi.API_SQL, window_kind=assigner.kind, size_ms=assigner.size,
            slide_ms=assigner.slide, offset_ms=assigner.offset,
            aggs=[(abi.AGG_NAMES[k], c, abi.TYPE_NAMES[t]) for k, c, t in aggs],
            count_star_index=count_star_index,
            value_col_types=[abi.TYPE_NAMES[t] for t in value_types],
            key_hash=abi.KEYHASH_KEYROW if self.key_types else KEY_HASH[key_type],
            max_parallelism=max_parallelism,
            parallelism=parallelism, subtask_index=subtask_index, device=device,
            state_capacity=state_capacity, max_batch_rows=max_batch_rows,
            output_capacity=output_capacity, nullable_cols=nullable_cols, shift_zone=zone,
            key_row_max_bytes=key_row_max_bytes)
        self.handle = None
        self.current_watermark = -(1 << 63)

    # ---- AbstractStreamOperator lifecycle
    def open(self):
        self.handle = WindowAggHandle(self.cfg)
        if self.current_watermark != -(1 << 63):
            self.handle.initialize_watermark(self.current_watermark)
        return self

    def close(self):
        if self.handle is not None:
            self.handle.close()
            self.handle = None

    # ---- OneInputStreamOperator
    def process_batch(self, keys, rowtimes, values=(), key_hashes=None, nulls=None):
        """processElement for every row of a columnar batch (host arrays; ``nulls``: {column:
        per-row NULL flags} for NULL-able columns).  With key rows (``key_type`` a tuple of SQL
        types) ``keys`` is a sequence of key tuples: the operator writes their BinaryRowData
        images into the handle's pinned staging (fw_reserve, as the JNI shim copies each key row's
        bytes) and the device interns them."""
        if self.key_types is None:
            self.handle.push_host(keys, rowtimes, values, key_hashes, nulls=nulls)
            return
        off, img = KeyRowColumns.from_rows(keys, self.key_types).images_host()
        longest = int(np.diff(off).max()) if len(off) > 1 else 0
        if longest > (self.cfg.key_row_max_bytes or 120):
            raise ValueError(f"a key row of {longest} bytes exceeds key_row_max_bytes "
                             f"({self.cfg.key_row_max_bytes or 120}); such keys stay on the reference operator")
        self.handle.push_host_key_rows(off, img, rowtimes, values, nulls=nulls)

    def process_batch_device(self, keys, rowtimes, values=(), key_hashes=None, nulls=None):
        """processElement for a batch already resident in HBM (torch cuda tensors)."""
        self.handle.push_device(keys, rowtimes, values, key_hashes, nulls=nulls)

    def process_watermark(self, watermark, collect=True):
        """processWatermark (:227-238): flush if triggered, fire timers <= watermark; returns the
        rows emitted for this watermark (before it is forwarded)."""
        self.handle.advance(watermark)
        if watermark > self.current_watermark:
            self.current_watermark = watermark
        if not collect:
            return None
        return self.handle.results(reset=True)

    def prepare_snapshot_pre_barrier(self, checkpoint_id=0):
        self.handle.flush()

    def snapshot_state(self) -> bytes:
        return self.handle.snapshot()

    def initialize_state(self, blob: bytes):
        self.handle.restore(blob)

    @property
    def num_late_records_dropped(self):
        return self.handle.stats()["num_late_records_dropped"]

    def output_rows(self, res):
        """Materialise result columns as reference-shaped rows: key ++ aggs ++ (ws, we)."""
        rows = []
        for i in range(len(res["key"])):
            vals = []
            for a, (kind, _, typ) in enumerate(self.aggs):
                if res["null_mask"][i] >> a & 1:
                    vals.append(None)
                elif abi.result_is_double(abi.AGG_NAMES[kind], abi.TYPE_NAMES[typ]):
                    vals.append(float(np.int64(res["values"][a][i]).view(np.float64)))
                else:
                    vals.append(int(res["values"][a][i]))
            key = decode_key_row(res["key_rows"][i], self.key_types) if self.key_types else (int(res["key"][i]),)
            rows.append((*key, *vals, int(res["window_start"][i]), int(res["window_end"][i])))
        return rows
