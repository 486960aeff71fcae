"""GPU-backed drop-in for the DataStream WindowOperator on its eligible subset.

WindowOperatorBuilder.buildWindowOperator (flink-runtime/.../windowing/WindowOperatorBuilder.java:432-446)
would return this operator iff: the assigner is TumblingEventTimeWindows or
SlidingEventTimeWindows (size % slide == 0), the trigger is EventTimeTrigger, there is no
evictor, and the function is a built-in field aggregation (SumAggregator / ComparableAggregator
for min/max, WindowedStream.java:660-880) on a numeric field.  Any allowedLateness and a
late-data side output (sideOutputLateData) are supported.  Anything else stays on the reference
WindowOperator.

Semantics (WindowOperator.java:293-682): per element, every window that is not late (cleanupTime =
maxTimestamp + allowedLateness > watermark) gets the value; a window the watermark has not
reached gets a timer at window.maxTimestamp(), one it has already passed fires again at once with
the element added (EventTimeTrigger.onElement).  A watermark fires (key, window) timers and emits
(key, aggregate) with record timestamp window.maxTimestamp(); the window state is cleared at its
cleanup time.  Elements late for all their windows go to the late side output when one is set,
else they are counted in numLateRecordsDropped.
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
    if evictor is not None:
        return False, "evictor"
    if allowed_lateness < 0:
        return False, "The allowed lateness cannot be negative."
    if aggregation[0] not in _AGG or aggregation[1] not in _TYPE:
        return False, "not a built-in field aggregation"
    return True, ""


class WindowOperator:
    def __init__(self, assigner, trigger, aggregation, key_type="LONG", max_parallelism=128,
                 parallelism=1, subtask_index=0, device=0, state_capacity=1 << 20,
                 max_batch_rows=1 << 22, output_capacity=1 << 22, allowed_lateness=0,
                 late_data_output_tag=None):
        ok, why = is_gpu_eligible(assigner, trigger, aggregation, allowed_lateness=allowed_lateness,
                                  late_data_output_tag=late_data_output_tag)
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
            output_capacity=output_capacity, allowed_lateness_ms=allowed_lateness,
            late_side_output=late_data_output_tag is not None)
        self.late_data_output_tag = late_data_output_tag
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

    def side_output(self):
        """Records routed to the late-data side output since the last call
        (WindowOperator.sideOutput): {key, timestamp, value, push_seq, row}."""
        r = self.handle.late_records()
        return {"key": r["key"], "timestamp": r["ts"], "value": r["values"][0], "push_seq": r["push_seq"],
                "row": r["row"]}

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
