"""GPU-backed drop-in for the DataStream WindowOperator on its eligible subset.

WindowOperatorBuilder.buildWindowOperator (flink-runtime/.../windowing/WindowOperatorBuilder.java:432-446)
would return this operator iff: the assigner is TumblingEventTimeWindows or
SlidingEventTimeWindows (size % slide == 0), the trigger is EventTimeTrigger, there is no
evictor, allowedLateness is 0, there is no late-data side output, and the function is a built-in
field aggregation (SumAggregator / ComparableAggregator for min/max, WindowedStream.java:660-880)
on a numeric field.  Anything else stays on the reference WindowOperator.

Semantics (WindowOperator.java:293-494): per element, every non-late window gets the value and a
timer at window.maxTimestamp(); a watermark fires (key, window) timers in timestamp order and emits
(key, aggregate) with record timestamp window.maxTimestamp(), then clears the window.  Elements
whose windows are all late are counted in numLateRecordsDropped.
"""
import numpy as np

from .. import abi
from ..runtime.handle import WindowAggHandle
from .windowing import EventTimeTrigger, SlidingEventTimeWindows, TumblingEventTimeWindows

_AGG = {"sum": abi.AGG_SUM, "min": abi.AGG_MIN, "max": abi.AGG_MAX, "count": abi.AGG_COUNT_STAR}
_KEY = {"LONG": abi.KEYHASH_LONG, "INT": abi.KEYHASH_INT, "HOST_HASHED": abi.KEYHASH_PRECOMPUTED}
_TYPE = {"LONG": abi.T_I64, "INT": abi.T_I32, "DOUBLE": abi.T_F64}


def is_gpu_eligible(assigner, trigger, aggregation, *, evictor=None, allowed_lateness=0,
                    late_data_output_tag=None):
    if not isinstance(assigner, (TumblingEventTimeWindows, SlidingEventTimeWindows)):
        return False, "assigner is not Tumbling/SlidingEventTimeWindows"
    if isinstance(assigner, SlidingEventTimeWindows) and assigner.size % assigner.slide != 0:
        return False, "sliding windows need size % slide == 0 to share slices"
    if not isinstance(trigger, EventTimeTrigger):
        return False, "custom trigger"
    if evictor is not None or allowed_lateness != 0 or late_data_output_tag is not None:
        return False, "evictor / allowed lateness / late side output"
    if aggregation[0] not in _AGG or aggregation[1] not in _TYPE:
        return False, "not a built-in field aggregation"
    return True, ""


class WindowOperator:
    def __init__(self, assigner, trigger, aggregation, key_type="LONG", max_parallelism=128,
                 parallelism=1, subtask_index=0, device=0, state_capacity=1 << 20,
                 max_batch_rows=1 << 22, output_capacity=1 << 22):
        ok, why = is_gpu_eligible(assigner, trigger, aggregation)
        if not ok:
            raise ValueError(f"not eligible for the GPU window operator: {why}")
        fn, ftype = aggregation
        sliding = isinstance(assigner, SlidingEventTimeWindows)
        self.assigner = assigner
        self.aggregation = aggregation
        t = _TYPE[ftype]
        self.cfg = abi.make_config(
            api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP if sliding else abi.WIN_TUMBLE,
            size_ms=assigner.size, slide_ms=assigner.slide if sliding else 0,
            offset_ms=assigner.offset, aggs=[(_AGG[fn], 0, t)], count_star_index=-1,
            value_col_types=[t], key_hash=_KEY[key_type], max_parallelism=max_parallelism,
            parallelism=parallelism, subtask_index=subtask_index, device=device,
            state_capacity=state_capacity, max_batch_rows=max_batch_rows,
            output_capacity=output_capacity)
        self.handle = None

    def open(self):
        self.handle = WindowAggHandle(self.cfg)
        return self

    def close(self):
        if self.handle is not None:
            self.handle.close()
            self.handle = None

    def process_batch(self, keys, timestamps, values, key_hashes=None):
        self.handle.push_host(keys, timestamps, [values], key_hashes)

    def process_batch_device(self, keys, timestamps, values, key_hashes=None):
        self.handle.push_device(keys, timestamps, [values], key_hashes)

    def process_watermark(self, watermark):
        """Fires all (key, window) timers <= watermark; returns {key, value, timestamp}."""
        self.handle.advance(watermark)
        r = self.handle.results(reset=True)
        return {"key": r["key"], "value": r["values"][0], "timestamp": r["window_end"] - 1,
                "window_start": r["window_start"], "window_end": r["window_end"],
                "values": r["values"], "null_mask": r["null_mask"]}

    def snapshot_state(self) -> bytes:
        return self.handle.snapshot()

    def initialize_state(self, blob: bytes):
        self.handle.restore(blob)

    @property
    def num_late_records_dropped(self):
        return self.handle.stats()["num_late_records_dropped"]

    def output_records(self, res):
        fn, ftype = self.aggregation
        vals = res["value"]
        if ftype == "DOUBLE" and fn != "count":
            vals = vals.view(np.float64)
        elif ftype == "INT" and fn != "count":
            vals = vals.astype(np.int32)
        return [(int(k), v.item(), int(t)) for k, v, t in zip(res["key"], vals, res["timestamp"])]
