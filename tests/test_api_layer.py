"""The reference-shaped host layer: the slice assigners against the reference's own
SliceAssigner known-answer tests, and the builder-seam eligibility rules for every
fallback reason.  CPU only: the assigners run the library's host restatement
(fw_host_window_start, the code the kernels run); no device call is made.  The GPU replay of the
golden fixtures through WindowAggOperator / WindowOperator is in test_gpu_api_layer.py."""
import pytest

from fixture_runner import load_kats
from flink_amd import abi
from flink_amd.datastream import window_operator as dso
from flink_amd.datastream.windowing import EventTimeTrigger, SlidingEventTimeWindows, TumblingEventTimeWindows
from flink_amd.table import window_agg as sqlo
from flink_amd.table.slice_assigners import (CumulativeSliceAssigner, HoppingSliceAssigner, SliceAssigners,
                                             TumblingSliceAssigner)
from oracle import oracle as O

KATS = load_kats()


def _assigner(kind, size, slide, offset):
    if kind == "TUMBLE":
        return TumblingSliceAssigner(0, size, offset)
    if kind == "HOP":
        return HoppingSliceAssigner(0, size, slide, offset)
    return CumulativeSliceAssigner(0, size, slide, offset)


@pytest.mark.parametrize("kat", KATS, ids=[f"{k['op']}:{k['src'].split('/')[-1]}" for k in KATS])
def test_slice_assigner_known_answers(kat):
    a = _assigner(*kat["assigner"])
    if "zone" in kat:
        a = a.in_zone(kat["zone"])
    for arg, want in kat["cases"]:
        if kat["op"] == "dst_slice":  # assertSliceStartEnd(start, end, epoch, assigner)
            se = a.assign_slice_end(arg)
            assert [a.get_window_start(se), se] == want
        elif kat["op"] == "slice_end":
            assert a.assign_slice_end(arg) == want
            iv = a.get_slice_end_interval()  # the oracle's restatement agrees
            assert O.window_start_with_offset(arg, a.offset, iv) + iv == want
        elif kat["op"] == "window_start":
            assert a.get_window_start(arg) == want
        elif kat["op"] == "expired_slices":
            assert a.expired_slices(arg) == want
        elif kat["op"] == "merge":
            target, slices = a.slices_to_merge(arg)
            assert [target, slices] == want
        elif kat["op"] == "next_trigger":
            assert a.next_trigger_window(arg[0], arg[1]) == want
        else:
            raise AssertionError(kat["op"])


def test_slice_assigner_argument_checks():
    # the reference's messages (HoppingSliceAssignerTest.testInvalidParameters and siblings)
    with pytest.raises(ValueError, match="slide > 0 and size > 0"):
        SliceAssigners.hopping(0, -2000, 1000)
    with pytest.raises(ValueError, match="integral multiple of slide"):
        SliceAssigners.hopping(0, 5000, 2000)
    with pytest.raises(ValueError, match="integral multiple of step"):
        SliceAssigners.cumulative(0, 5000, 2000)
    with pytest.raises(ValueError, match=r"abs\(offset\) < size"):
        TumblingSliceAssigner(0, 10000, 10000)
    SliceAssigners.hopping(0, 10000, 5000).with_offset(-1000)  # should pass
    assert not TumblingSliceAssigner(-1, 5000).is_event_time()


# ---- eligibility: every reason the builder seam keeps the reference operator --------------
SQL_OK = dict(assigner=SliceAssigners.tumbling(0, 10000), aggs=[("SUM", 0, "BIGINT"), ("MAX", 1, "DOUBLE")],
              value_types=["BIGINT", "DOUBLE"])


def test_sql_eligible_builtin_aggregates():
    assert sqlo.is_gpu_eligible(**SQL_OK) == (True, "")
    ok, _ = sqlo.is_gpu_eligible(SliceAssigners.hopping(0, 10000, 2000),
                                 [("COUNT_STAR", 0, "BIGINT"), ("AVG", 0, "INT")], ["INT"], key_type="INT")
    assert ok


@pytest.mark.parametrize("change,reason", [
    (dict(has_distinct=True), "DISTINCT"),
    (dict(needs_retraction=True), "retraction"),
    (dict(shift_time_zone="Mars/Olympus_Mons"), "shift time zone"),
    (dict(is_event_time=False), "processing-time"),
    (dict(aggs=[("FIRST_VALUE", 0, "BIGINT")]), "not a built-in GPU aggregate"),
    (dict(aggs=[("MIN", 0, "FLOAT")], value_types=["FLOAT"]), "FLOAT"),
    (dict(aggs=[("SUM", 0, "DECIMAL(10, 2)")], value_types=["DECIMAL(10, 2)"]), "DECIMAL"),
    (dict(key_type="ARRAY<INT>"), "key type"),
])
def test_sql_fallback_reasons(change, reason):
    kw = dict(SQL_OK)
    kw.update(change)
    ok, why = sqlo.is_gpu_eligible(**kw)
    assert not ok and reason in why


def test_sql_timestamp_ltz_windows_are_eligible():
    for zone in ("Asia/Shanghai", "America/Los_Angeles", "UTC"):
        assert sqlo.is_gpu_eligible(**dict(SQL_OK, shift_time_zone=zone)) == (True, "")


def test_sql_processing_time_assigner_is_not_eligible():
    ok, why = sqlo.is_gpu_eligible(TumblingSliceAssigner(-1, 5000), [("SUM", 0, "BIGINT")], ["BIGINT"])
    assert not ok and "processing-time" in why


def test_sql_hop_without_count_star_rejected_like_the_reference():
    with pytest.raises(ValueError, match="Hopping window requires a COUNT"):
        sqlo.WindowAggOperator(SliceAssigners.hopping(0, 6000, 2000), [("SUM", 0, "BIGINT")], ["BIGINT"])


DS_OK = dict(assigner=TumblingEventTimeWindows.of(5000), trigger=EventTimeTrigger.create(), aggregation=("sum", "LONG"))


def test_datastream_eligible():
    assert dso.is_gpu_eligible(**DS_OK) == (True, "")
    # allowedLateness and sideOutputLateData (WindowOperator.java:609-682, :440-446)
    assert dso.is_gpu_eligible(**dict(DS_OK, allowed_lateness=1000, late_data_output_tag="late")) == (True, "")
    assert dso.is_gpu_eligible(SlidingEventTimeWindows.of(6000, 2000), EventTimeTrigger(), ("max", "DOUBLE"))[0]
    # slide need not divide size (SlidingEventTimeWindows.java:77-90): panes of gcd(size, slide)
    assert dso.is_gpu_eligible(SlidingEventTimeWindows.of(5000, 2000), EventTimeTrigger(), ("sum", "LONG"))[0]
    # minBy / maxBy (WindowedStream.java:725-790), first (default) or last element on ties
    assert dso.is_gpu_eligible(**dict(DS_OK, aggregation=("maxBy", "DOUBLE")))[0]
    assert dso.is_gpu_eligible(**dict(DS_OK, aggregation=("minBy", "LONG", False)))[0]


def test_datastream_minby_maxby_planning():
    """minBy / maxBy emit whole elements: a record-shaped operator (field=...) is required, and the
    first/last flag becomes fw_agg_desc.flags (FW_AGGF_LAST)"""
    with pytest.raises(ValueError):
        dso.WindowOperator(TumblingEventTimeWindows.of(5000), EventTimeTrigger(), ("maxBy", "LONG"))
    op = dso.WindowOperator(TumblingEventTimeWindows.of(5000), EventTimeTrigger(), ("minBy", "LONG", False), field=1)
    assert op.cfg.aggs[0].kind == abi.AGG_MINBY and op.cfg.aggs[0].flags == abi.AGGF_LAST
    assert op.cfg.ds_first_ordinals == 1
    op = dso.WindowOperator(TumblingEventTimeWindows.of(5000), EventTimeTrigger(), ("maxBy", "DOUBLE"), field=0)
    assert op.cfg.aggs[0].kind == abi.AGG_MAXBY and op.cfg.aggs[0].flags == 0


class _CountTrigger:  # a custom trigger (CountTrigger, ContinuousEventTimeTrigger, ...)
    pass


class _Sessions:  # a merging assigner (EventTimeSessionWindows)
    pass


@pytest.mark.parametrize("change,reason", [
    (dict(allowed_lateness=-1), "lateness cannot be negative"),
    (dict(evictor=object()), "evictor"),
    (dict(trigger=_CountTrigger()), "custom trigger"),
    (dict(assigner=_Sessions()), "assigner"),
    (dict(assigner=SlidingEventTimeWindows.of(2000, 5000)), "size < slide"),
    (dict(aggregation=("reduce", "LONG")), "built-in field aggregation"),
    (dict(aggregation=("sum", "FLOAT")), "built-in field aggregation"),
    (dict(aggregation=("sum", "LONG", False)), "first/last flag"),
])
def test_datastream_fallback_reasons(change, reason):
    kw = dict(DS_OK)
    kw.update(change)
    ok, why = dso.is_gpu_eligible(**kw)
    assert not ok and reason in why


def test_assigner_mirrors_match_the_reference_window_assignment():
    # TumblingEventTimeWindows.assignWindows / SlidingEventTimeWindows.assignWindows (10 s / 2 s,
    # a record at 7.5 s belongs to [0, 10), [-2, 8), [2, 12), [4, 14), [6, 16))
    assert TumblingEventTimeWindows.of(5000, 1000).assign_windows(7500) == [(6000, 11000)]
    assert sorted(SlidingEventTimeWindows.of(10000, 2000).assign_windows(7500)) == \
        [(-2000, 8000), (0, 10000), (2000, 12000), (4000, 14000), (6000, 16000)]


def test_gpu_window_agg_options_gate_both_seams():
    """gpu.window-agg.enabled (default false) gates both builder seams; gpu.window-agg.device picks
    the handle's device (SURVEY.md 5 Config/flags)."""
    from flink_amd.runtime import options
    assert not sqlo.is_gpu_eligible(**SQL_OK, conf={})[0]
    assert sqlo.is_gpu_eligible(**SQL_OK, conf={"gpu.window-agg.enabled": "false"})[1] == "gpu.window-agg.enabled is false"
    assert sqlo.is_gpu_eligible(**SQL_OK, conf={"gpu.window-agg.enabled": "true"}) == (True, "")
    assert not dso.is_gpu_eligible(**DS_OK, conf={})[0]
    assert dso.is_gpu_eligible(**DS_OK, conf={"gpu.window-agg.enabled": True}) == (True, "")
    with pytest.raises(ValueError):
        options.gpu_enabled({"gpu.window-agg.enabled": "maybe"})
    assert options.gpu_device({}, 5, 8) == 5 and options.gpu_device({}, 13, 8) == 5
    assert options.gpu_device({"gpu.window-agg.device": "2"}, 13, 8) == 2
