"""Every golden fixture replayed through the reference-shaped operators (not the raw handle):
flink_amd.table.window_agg.WindowAggOperator for the SQL fixtures (open / processElement /
processWatermark / prepareSnapshotPreBarrier + snapshotState + initializeState), the DataStream
flink_amd.datastream.window_operator.WindowOperator for the WindowOperatorTest fixtures, and the
two-phase plan (flink_amd.table.two_phase) for the fixtures the reference runs with both agg-phase
strategies.  Run on an MI355X."""
import numpy as np
import pytest

from fixture_runner import TwoPhaseGpuAdapter, load_fixtures, replay

pytestmark = pytest.mark.gpu

FIXTURES = load_fixtures()
SQL = [f for f in FIXTURES if f["config"]["api"] == "SQL"]
DS = [f for f in FIXTURES if f["config"]["api"] == "DATASTREAM"]
TWO = [f for f in FIXTURES if f.get("two_phase")]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _slice_assigner(c):
    from flink_amd.table.slice_assigners import SliceAssigners
    kind = c["window"]
    if kind == "TUMBLE":
        a = SliceAssigners.tumbling(0, c["size_ms"])
    elif kind == "HOP":
        a = SliceAssigners.hopping(0, c["size_ms"], c["slide_ms"])
    else:
        a = SliceAssigners.cumulative(0, c["size_ms"], c["slide_ms"])
    a = a.with_offset(c.get("offset_ms", 0)) if c.get("offset_ms") else a
    return a.in_zone(c["shift_zone"]) if c.get("shift_zone") else a


class SqlOperatorAdapter:
    def __init__(self, fx):
        from flink_amd.table.window_agg import WindowAggOperator
        c = fx["config"]
        self.kw = dict(assigner=_slice_assigner(c), aggs=[tuple(a) for a in c["aggs"]], value_types=c["value_cols"],
                       count_star_index=c.get("count_star_index", -1), key_type="HOST_HASHED",
                       state_capacity=1 << 14, max_batch_rows=1 << 12, output_capacity=1 << 12,
                       nullable_cols=c.get("nullable_cols", []))
        self.op = WindowAggOperator(**self.kw).open()

    def process_batch(self, k, t, h, vals, nulls=None):
        self.op.process_batch(k, t, vals, key_hashes=h, nulls=nulls)

    def process_watermark(self, w):
        return self.op.process_watermark(w)

    def snapshot_restore(self):
        from flink_amd.table.window_agg import WindowAggOperator
        self.op.prepare_snapshot_pre_barrier()
        blob = self.op.snapshot_state()
        self.op.close()
        self.op = WindowAggOperator(**self.kw).open()
        self.op.initialize_state(blob)

    @property
    def late_dropped(self):
        return self.op.num_late_records_dropped


class DataStreamOperatorAdapter:
    def __init__(self, fx):
        from flink_amd.datastream.window_operator import WindowOperator
        from flink_amd.datastream.windowing import EventTimeTrigger, SlidingEventTimeWindows, TumblingEventTimeWindows
        c = fx["config"]
        assigner = (TumblingEventTimeWindows.of(c["size_ms"], c.get("offset_ms", 0)) if c["window"] == "TUMBLE"
                    else SlidingEventTimeWindows.of(c["size_ms"], c["slide_ms"], c.get("offset_ms", 0)))
        kind, _, typ = c["aggs"][0]
        self.kw = dict(assigner=assigner, trigger=EventTimeTrigger.create(),
                       aggregation=(kind.lower(), {"BIGINT": "LONG", "INT": "INT", "DOUBLE": "DOUBLE"}[typ]),
                       key_type="HOST_HASHED", state_capacity=1 << 14, max_batch_rows=1 << 12, output_capacity=1 << 12,
                       allowed_lateness=c.get("allowed_lateness_ms", 0),
                       late_data_output_tag="late" if c.get("late_side_output") else None)
        self.op = WindowOperator(**self.kw).open()
        self._side = []

    def process_batch(self, k, t, h, vals, nulls=None):
        self.op.process_batch(k, t, vals[0], key_hashes=h)

    def process_watermark(self, w):
        r = self.op.process_watermark(w)
        # output records carry timestamp window.maxTimestamp() (WindowOperator.java:576)
        assert np.array_equal(r["timestamp"], r["window_end"] - 1)
        return r

    def side_output(self):
        parts = self._side + [self.op.side_output()]
        return {"key": np.concatenate([p["key"] for p in parts]), "ts": np.concatenate([p["timestamp"] for p in parts]),
                "values": [np.concatenate([p["value"] for p in parts])]}

    def snapshot_restore(self):
        from flink_amd.datastream.window_operator import WindowOperator
        if self.kw["late_data_output_tag"] is not None:
            self._side.append(self.op.side_output())
        blob = self.op.snapshot_state()
        self.op.close()
        self.op = WindowOperator(**self.kw).open()
        self.op.initialize_state(blob)

    @property
    def late_dropped(self):
        return self.op.num_late_records_dropped


@pytest.mark.parametrize("fx", SQL, ids=[f["name"] for f in SQL])
def test_sql_window_agg_operator_reproduces_reference_golden(fx):
    replay(fx, SqlOperatorAdapter(fx))


@pytest.mark.parametrize("fx", DS, ids=[f["name"] for f in DS])
def test_datastream_window_operator_reproduces_reference_golden(fx):
    replay(fx, DataStreamOperatorAdapter(fx))


@pytest.mark.parametrize("fx", TWO, ids=[f["name"] for f in TWO])
def test_two_phase_plan_reproduces_reference_golden(fx):
    replay(fx, TwoPhaseGpuAdapter(fx), check_late=False)
