"""Transcribes golden event scripts from the reference's own tests into JSON fixtures.

Each fixture is DATA only: the input records, the watermarks, and the expected output rows
the reference test asserts after each watermark (plus the late-drop counter).  Sources
(paths relative to /root/reference):

  SQL  flink-table/flink-table-runtime/src/test/java/org/apache/flink/table/runtime/operators/
       aggregate/window/SlicingWindowAggOperatorTest.java  (UTC parameterisation)
       - testEventTimeHoppingWindows                        :62-162
       - testEventTimeHoppingWindowWithExpiredSliceAndRestore :164-219
       - testEventTimeHoppingWindowWithExpiredSliceAndNoRestore :221-270
       - testEventTimeCumulativeWindows                     :387-495
       - testEventTimeTumblingWindows                       :628-721
       The test aggregate (WindowAggOperatorTestBase.java:240-377) is SUM(f1) -> BIGINT and
       COUNT(f1); output rows are key ++ (sum, count, window_start, window_end).
  DS   flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/
       windowing/WindowOperatorTest.java
       - testSlidingEventTimeWindows (reduce: Tuple2<String,Integer> SumReducer) :116-219
       - testTumblingEventTimeWindows                                            :333-434
       Output records are (key, sum) with timestamp window.maxTimestamp().
  DOCS docs/content/docs/sql/reference/queries/window-agg.md:55-117 (global TUMBLE / HOP /
       CUMULATE SUM(price) over the Bid table; DECIMAL(10,2) prices carried as BIGINT cents).
  TPRG flink-table/flink-table-planner/src/test/java/org/apache/flink/table/planner/plan/nodes/
       exec/stream/WindowAggregateTestPrograms.java:39-60 (data), :86-375 (expected rows),
       :500-511 (SELECT name, window_start, window_end, COUNT(*), SUM(a_int), COUNT(DISTINCT
       comment)): TUMBLE / HOP / CUMULATE with and without offset, ONE_PHASE and TWO_PHASE, a
       savepoint between the "before" and "after" data.  COUNT(DISTINCT) is not a GPU aggregate
       (the eligibility rule sends it to the reference operator), so those fixtures carry
       COUNT(*) and SUM(a_int) only.  The source's watermark is rowtime - 1 s
       (:75), emitted after every record; end of input emits Long.MAX_VALUE.
  ITC  flink-table/flink-table-planner/src/test/scala/org/apache/flink/table/planner/runtime/
       stream/sql/WindowAggregateITCase.scala:218-282 with TestData.windowDataWithTimestamp
       (flink-table-planner/src/test/scala/.../runtime/utils/TestData.scala:749-762): COUNT(*)
       and MAX(double) (a NULL-able DOUBLE column); SUM(DECIMAL) and MIN(FLOAT) are not GPU
       aggregates.
  KATS flink-table/flink-table-runtime/src/test/java/org/apache/flink/table/runtime/operators/
       window/tvf/slicing/{Tumbling,Hopping,Cumulative}SliceAssignerTest.java (UTC): slice end,
       window start, expired slices, slices to merge, next trigger window; testDstSaving (:63-96,
       :66-100, :66-100) under America/Los_Angeles: slice start / end across the 2021 DST changes.
  LTZ  SlicingWindowAggOperatorTest runs every event-time test under UTC *and* Asia/Shanghai
       (:53-59).  With Asia/Shanghai the expected window_start / window_end are
       localMills(epoch) = toUtcTimestampMills(epoch, zone) = epoch + 8 h
       (WindowAggOperatorTestBase.java:79-81) while elements and watermarks stay epoch millis:
       the *_shanghai fixtures.
  LATE WindowOperatorTest.java allowed lateness / late side output (SumReducer, EventTimeTrigger):
       - testCleanupTimeOverflow                              :2139-2245 (lateness 2000 ms,
         cleanup time past Long.MAX_VALUE)
       - testSideOutputDueToLatenessTumbling                  :2249-2344
       - testSideOutputDueToLatenessSliding                   :2348-2462
       - testCleanupTimerWithEmptyReduceStateForTumblingWindows :3248-3321 (lateness 1 ms)
       "side_output" lists the elements the test expects on the late side output.

Keys that are strings in the reference tests are mapped to integer ids; their Java
String.hashCode is recorded so key-group assignment matches the reference.  "snapshot_restore"
marks the tests' prepareSnapshotPreBarrier + snapshot + close + initializeState + open.

Run:  python tests/golden/make_golden.py   (writes tests/golden/*.json)
"""
import datetime as dt
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
INT64_MAX = (1 << 63) - 1


def java_string_hash(s):
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


KEYS = {"key1": {"id": 1, "hash": java_string_hash("key1")},
        "key2": {"id": 2, "hash": java_string_hash("key2")}}

SQL_CFG_BASE = {"api": "SQL", "aggs": [["SUM", 0, "BIGINT"], ["COUNT", 0, "BIGINT"]],
                "value_cols": ["BIGINT"], "key_hash": "PRECOMPUTED", "offset_ms": 0}
DS_CFG_BASE = {"api": "DATASTREAM", "aggs": [["SUM", 0, "INT"]], "value_cols": ["INT"],
               "key_hash": "PRECOMPUTED", "offset_ms": 0, "count_star_index": -1}


def el(key, ts, v=1):
    return {"op": "element", "key": key, "ts": ts, "values": [v]}


def wm(w, *rows):
    return {"op": "watermark", "wm": w, "expect": list(rows)}


def sql_row(key, s, c, ws, we):
    return {"key": key, "values": [s, c], "window_start": ws, "window_end": we}


def ds_row(key, v, ts):  # StreamRecord(Tuple2(key, v), ts) with ts = window.maxTimestamp()
    return {"key": key, "values": [v], "window_end": ts + 1}


SNAP = {"op": "snapshot_restore"}

OOO = [el("key2", 3999), el("key2", 3000), el("key1", 20), el("key1", 0), el("key1", 999),
       el("key2", 1998), el("key2", 1999), el("key2", 1000)]

FIXTURES = []

# ---------------------------------------------------------------- SQL slicing operator
FIXTURES.append({
    "name": "sql_hop_3s_1s",
    "source": "SlicingWindowAggOperatorTest.java:62-162 testEventTimeHoppingWindows",
    "config": dict(SQL_CFG_BASE, window="HOP", size_ms=3000, slide_ms=1000, count_star_index=1),
    "steps": OOO + [
        wm(999, sql_row("key1", 3, 3, -2000, 1000)),
        wm(1999, sql_row("key1", 3, 3, -1000, 2000), sql_row("key2", 3, 3, -1000, 2000)),
        wm(2999, sql_row("key1", 3, 3, 0, 3000), sql_row("key2", 3, 3, 0, 3000)),
        SNAP,
        wm(3999, sql_row("key2", 5, 5, 1000, 4000)),
        el("key2", 3500),
        wm(4999, sql_row("key2", 3, 3, 2000, 5000)),
        el("key1", 2999),
        wm(5999, sql_row("key2", 3, 3, 3000, 6000)),
        wm(6999), wm(7999)],
    "late_dropped": 1,
})

_expired = [el("key1", 1020), el("key1", 1001), el("key1", 1999),
            wm(2001, sql_row("key1", 3, 3, -1000, 2000))]
_expired_tail = [el("key2", 1500), el("key2", 2998), el("key2", 2999), el("key2", 2000),
                 wm(2999, sql_row("key1", 3, 3, 0, 3000), sql_row("key2", 4, 4, 0, 3000))]
FIXTURES.append({
    "name": "sql_hop_expired_slice_restore",
    "source": "SlicingWindowAggOperatorTest.java:164-219 testEventTimeHoppingWindowWithExpiredSliceAndRestore",
    "config": dict(SQL_CFG_BASE, window="HOP", size_ms=3000, slide_ms=1000, count_star_index=1),
    "steps": _expired + [SNAP] + _expired_tail,
    "late_dropped": 0,
})
FIXTURES.append({
    "name": "sql_hop_expired_slice_norestore",
    "source": "SlicingWindowAggOperatorTest.java:221-270 testEventTimeHoppingWindowWithExpiredSliceAndNoRestore",
    "config": dict(SQL_CFG_BASE, window="HOP", size_ms=3000, slide_ms=1000, count_star_index=1),
    "steps": _expired + _expired_tail,
    "late_dropped": 0,
})

FIXTURES.append({
    "name": "sql_cumulate_3s_1s",
    "source": "SlicingWindowAggOperatorTest.java:387-495 testEventTimeCumulativeWindows",
    "config": dict(SQL_CFG_BASE, window="CUMULATE", size_ms=3000, slide_ms=1000, count_star_index=-1),
    "steps": [el("key2", 2999), el("key2", 3000), el("key1", 20), el("key1", 0), el("key1", 999),
              el("key2", 1998), el("key2", 1999), el("key2", 1000),
              wm(999, sql_row("key1", 3, 3, 0, 1000)),
              wm(1999, sql_row("key1", 3, 3, 0, 2000), sql_row("key2", 3, 3, 0, 2000)),
              SNAP,
              el("key2", 1000),
              wm(1999),
              wm(2999, sql_row("key1", 3, 3, 0, 3000), sql_row("key2", 5, 5, 0, 3000)),
              wm(3999, sql_row("key2", 1, 1, 3000, 4000)),
              el("key1", 3500, 2),
              wm(4999, sql_row("key2", 1, 1, 3000, 5000), sql_row("key1", 2, 1, 3000, 5000)),
              el("key1", 2999),
              wm(5999, sql_row("key2", 1, 1, 3000, 6000), sql_row("key1", 2, 1, 3000, 6000)),
              wm(6999), wm(7999)],
    "late_dropped": 1,
})

FIXTURES.append({
    "name": "sql_tumble_3s",
    "source": "SlicingWindowAggOperatorTest.java:628-721 testEventTimeTumblingWindows",
    "config": dict(SQL_CFG_BASE, window="TUMBLE", size_ms=3000, slide_ms=0, count_star_index=-1),
    "steps": OOO + [
        wm(999), wm(1999), SNAP,
        wm(2999, sql_row("key1", 3, 3, 0, 3000), sql_row("key2", 3, 3, 0, 3000)),
        wm(3999),
        el("key1", 2500),
        wm(4999),
        el("key2", 2999),
        wm(5999, sql_row("key2", 2, 2, 3000, 6000)),
        wm(6999), wm(7999)],
    "late_dropped": 2,
})

# ---------------------------------------------------------------- DataStream WindowOperator
FIXTURES.append({
    "name": "ds_sliding_3s_1s_sum",
    "source": "WindowOperatorTest.java:116-219 testSlidingEventTimeWindows (SumReducer)",
    "config": dict(DS_CFG_BASE, window="HOP", size_ms=3000, slide_ms=1000),
    "steps": OOO + [
        wm(999, ds_row("key1", 3, 999)),
        wm(1999, ds_row("key1", 3, 1999), ds_row("key2", 3, 1999)),
        wm(2999, ds_row("key1", 3, 2999), ds_row("key2", 3, 2999)),
        SNAP,
        wm(3999, ds_row("key2", 5, 3999)),
        wm(4999, ds_row("key2", 2, 4999)),
        wm(5999, ds_row("key2", 2, 5999)),
        wm(6999), wm(7999)],
    "late_dropped": 0,
})
FIXTURES.append({
    "name": "ds_tumbling_3s_sum",
    "source": "WindowOperatorTest.java:333-434 testTumblingEventTimeWindows (SumReducer)",
    "config": dict(DS_CFG_BASE, window="TUMBLE", size_ms=3000, slide_ms=0),
    "steps": OOO + [
        wm(999), wm(1999), SNAP,
        wm(2999, ds_row("key1", 3, 2999), ds_row("key2", 3, 2999)),
        wm(3999), wm(4999),
        wm(5999, ds_row("key2", 2, 5999)),
        wm(6999), wm(7999)],
    "late_dropped": 0,
})

# ---------------------------------------------------------------- DataStream lateness
_LMAX = INT64_MAX - 1750                       # testCleanupTimeOverflow's element timestamp
_LWIN_END = _LMAX - (_LMAX % 1000) + 1000      # its 1 s tumbling window [start, end)
FIXTURES.append({
    "name": "ds_lateness_cleanup_overflow",
    "source": "WindowOperatorTest.java:2139-2245 testCleanupTimeOverflow (lateness 2000 ms)",
    "config": dict(DS_CFG_BASE, window="TUMBLE", size_ms=1000, slide_ms=0, allowed_lateness_ms=2000),
    "steps": [el("key2", _LMAX), wm(INT64_MAX - 1500), wm(_LWIN_END - 1, ds_row("key2", 1, _LWIN_END - 1))],
    "late_dropped": 0,
})
FIXTURES.append({
    "name": "ds_side_output_tumbling_2s",
    "source": "WindowOperatorTest.java:2249-2344 testSideOutputDueToLatenessTumbling",
    "config": dict(DS_CFG_BASE, window="TUMBLE", size_ms=2000, slide_ms=0, allowed_lateness_ms=0, late_side_output=True),
    "steps": [el("key2", 1000), wm(1985),
              el("key2", 1980), wm(1999, ds_row("key2", 2, 1999)),
              el("key2", 1998), el("key2", 2001), wm(2999),
              wm(3999, ds_row("key2", 1, 3999))],
    "side_output": [{"key": "key2", "ts": 1998, "values": [1]}],
    "late_dropped": 0,
})
FIXTURES.append({
    "name": "ds_side_output_sliding_3s_1s",
    "source": "WindowOperatorTest.java:2348-2462 testSideOutputDueToLatenessSliding",
    "config": dict(DS_CFG_BASE, window="HOP", size_ms=3000, slide_ms=1000, allowed_lateness_ms=0, late_side_output=True),
    "steps": [el("key2", 1000), wm(1999, ds_row("key2", 1, 1999)),
              el("key2", 2000), wm(3000, ds_row("key2", 2, 2999)),
              el("key1", 3001), el("key2", 2400), el("key2", 2400), el("key1", 3001), el("key2", 3900),
              wm(6000, ds_row("key2", 5, 3999), ds_row("key1", 2, 3999), ds_row("key2", 4, 4999),
                 ds_row("key1", 2, 4999), ds_row("key2", 1, 5999), ds_row("key1", 2, 5999)),
              el("key1", 3001), wm(25000)],
    "side_output": [{"key": "key1", "ts": 3001, "values": [1]}],
    "late_dropped": 0,
})
FIXTURES.append({
    "name": "ds_lateness_cleanup_timer_tumbling_2s",
    "source": "WindowOperatorTest.java:3248-3321 testCleanupTimerWithEmptyReduceStateForTumblingWindows (lateness 1 ms)",
    "config": dict(DS_CFG_BASE, window="TUMBLE", size_ms=2000, slide_ms=0, allowed_lateness_ms=1),
    "steps": [el("key2", 1000), wm(1599), wm(1999, ds_row("key2", 1, 1999)), wm(2000), wm(5000)],
    "late_dropped": 0,
})

# ---------------------------------------------------------------- docs window-agg.md:55-117


def _ms(hhmm):
    h, m = map(int, hhmm.split(":"))
    return int(dt.datetime(2020, 4, 15, h, m, tzinfo=dt.timezone.utc).timestamp() * 1000)


BID = [("08:05", 400), ("08:07", 200), ("08:09", 500), ("08:11", 300), ("08:13", 100), ("08:17", 600)]
_bid_steps = [{"op": "element", "key": "global", "ts": _ms(t), "values": [p]} for t, p in BID]
DOC_KEYS = {"global": {"id": 0, "hash": 0}}
DOC_CFG = {"api": "SQL", "value_cols": ["BIGINT"], "key_hash": "PRECOMPUTED", "offset_ms": 0}


def doc_row(ws, we, cents):
    return {"key": "global", "values": [cents], "window_start": _ms(ws), "window_end": _ms(we)}


FIXTURES.append({
    "name": "docs_tumble_10min",
    "source": "docs/content/docs/sql/reference/queries/window-agg.md:75-84",
    "keys": DOC_KEYS,
    "config": dict(DOC_CFG, window="TUMBLE", size_ms=600000, slide_ms=0, count_star_index=-1,
                   aggs=[["SUM", 0, "BIGINT"]]),
    "steps": _bid_steps + [wm(INT64_MAX, doc_row("08:00", "08:10", 1100), doc_row("08:10", "08:20", 1000))],
    "late_dropped": 0,
})
FIXTURES.append({
    "name": "docs_hop_5min_10min",
    "source": "docs/content/docs/sql/reference/queries/window-agg.md:86-97 (planner adds hidden COUNT(*), AggregateUtil.scala:285)",
    "keys": DOC_KEYS,
    "config": dict(DOC_CFG, window="HOP", size_ms=600000, slide_ms=300000, count_star_index=1,
                   aggs=[["SUM", 0, "BIGINT"], ["COUNT_STAR", 0, "BIGINT"]], compare_aggs=[0]),
    "steps": _bid_steps + [wm(INT64_MAX, doc_row("08:00", "08:10", 1100), doc_row("08:05", "08:15", 1500),
                                doc_row("08:10", "08:20", 1000), doc_row("08:15", "08:25", 600))],
    "late_dropped": 0,
})
FIXTURES.append({
    "name": "docs_cumulate_2min_10min",
    "source": "docs/content/docs/sql/reference/queries/window-agg.md:99-114",
    "keys": DOC_KEYS,
    "config": dict(DOC_CFG, window="CUMULATE", size_ms=600000, slide_ms=120000, count_star_index=-1,
                   aggs=[["SUM", 0, "BIGINT"]]),
    "steps": _bid_steps + [wm(INT64_MAX,
                              doc_row("08:00", "08:06", 400), doc_row("08:00", "08:08", 600),
                              doc_row("08:00", "08:10", 1100), doc_row("08:10", "08:12", 300),
                              doc_row("08:10", "08:14", 400), doc_row("08:10", "08:16", 400),
                              doc_row("08:10", "08:18", 1000), doc_row("08:10", "08:20", 1000))],
    "late_dropped": 0,
})


# ---------------------------------------------------------------- WindowAggregateTestPrograms
T0_TP = int(dt.datetime(2020, 10, 10, tzinfo=dt.timezone.utc).timestamp() * 1000)
# (seconds after 2020-10-10T00:00, a_int, b_double, name) of BEFORE_DATA / AFTER_DATA (:39-60)
TP_BEFORE = [(1, 1, 1.0, "a"), (2, 2, 2.0, "a"), (3, 2, 2.0, "a"), (4, 5, 5.0, "a"), (7, 3, 3.0, "b"),
             (6, 6, 6.0, "b"), (8, 3, None, "a"), (4, 5, 5.0, "a"), (16, 4, 4.0, "b"), (32, 7, 7.0, None),
             (34, 1, 3.0, "b")]
TP_AFTER = [(40, 10, 3.0, "a"), (42, 11, 4.0, "d"), (43, 12, 5.0, "c"), (44, 13, 6.0, "d")]
TP_KEYS = {"a": {"id": 1, "hash": java_string_hash("a")}, "b": {"id": 2, "hash": java_string_hash("b")},
           "c": {"id": 3, "hash": java_string_hash("c")}, "d": {"id": 4, "hash": java_string_hash("d")},
           "null": {"id": 0, "hash": 0}}


def _tp_time(hms):  # "00:00:05" or "23:59:55" of 2020-10-10 / 2020-10-09
    return hms


def _iso_ms(s):
    return int(dt.datetime.fromisoformat(s).replace(tzinfo=dt.timezone.utc).timestamp() * 1000)


def _records(rows, column, wm_state):
    """elements (+ the rowtime - 1 s watermark after every record that raises it)"""
    steps = []
    for sec, a_int, b_double, name in rows:
        ts = T0_TP + sec * 1000
        key = name if name is not None else "null"
        if column == "a_int":
            steps.append({"op": "element", "key": key, "ts": ts, "values": [a_int]})
        else:
            steps.append({"op": "element", "key": key, "ts": ts, "values": [0.0 if b_double is None else b_double],
                          "nulls": [1 if b_double is None else 0]})
        w = ts - 1000
        if w > wm_state[0]:
            wm_state[0] = w
            steps.append({"op": "watermark", "wm": w})
    return steps


def _parse_rows(rows):
    out = []
    for r in rows:
        f = [x.strip() for x in r[3:-1].split(",")]
        out.append({"key": f[0], "window_start": _iso_ms(f[1]), "window_end": _iso_ms(f[2]),
                    "values": [int(f[3]), int(f[4])]})
    return out


def _tp(name, src, window, size_ms, slide_ms, offset_ms, before, after):
    st = [-(1 << 63)]
    steps = _records(TP_BEFORE, "a_int", st)
    steps.append({"op": "check", "expect": _parse_rows(before)})
    steps.append(SNAP)
    steps += _records(TP_AFTER, "a_int", st)
    steps.append({"op": "watermark", "wm": INT64_MAX})
    steps.append({"op": "check", "expect": _parse_rows(after)})
    FIXTURES.append({
        "name": name, "source": src, "keys": TP_KEYS, "two_phase": True,
        "config": {"api": "SQL", "window": window, "size_ms": size_ms, "slide_ms": slide_ms,
                   "offset_ms": offset_ms, "count_star_index": 0, "key_hash": "PRECOMPUTED",
                   "aggs": [["COUNT_STAR", 0, "BIGINT"], ["SUM", 0, "INT"]], "value_cols": ["INT"]},
        "steps": steps, "late_dropped": None})


_TPF = "WindowAggregateTestPrograms.java"
_tp("tp_tumble_5s", _TPF + ":86-117 TUMBLE_WINDOW_EVENT_TIME(_TWO_PHASE)", "TUMBLE", 5000, 0, 0,
    ["+I[a, 2020-10-10T00:00, 2020-10-10T00:00:05, 4, 10, 2]", "+I[a, 2020-10-10T00:00:05, 2020-10-10T00:00:10, 1, 3, 1]",
     "+I[b, 2020-10-10T00:00:05, 2020-10-10T00:00:10, 2, 9, 2]", "+I[b, 2020-10-10T00:00:15, 2020-10-10T00:00:20, 1, 4, 1]"],
    ["+I[b, 2020-10-10T00:00:30, 2020-10-10T00:00:35, 1, 1, 1]", "+I[null, 2020-10-10T00:00:30, 2020-10-10T00:00:35, 1, 7, 0]",
     "+I[a, 2020-10-10T00:00:40, 2020-10-10T00:00:45, 1, 10, 1]", "+I[c, 2020-10-10T00:00:40, 2020-10-10T00:00:45, 1, 12, 1]",
     "+I[d, 2020-10-10T00:00:40, 2020-10-10T00:00:45, 2, 24, 2]"])
_tp("tp_tumble_5s_offset_1s", _TPF + ":129-160 TUMBLE_WINDOW_EVENT_TIME(_TWO_PHASE)_WITH_OFFSET", "TUMBLE", 5000, 0, 1000,
    ["+I[a, 2020-10-10T00:00:01, 2020-10-10T00:00:06, 4, 10, 2]", "+I[b, 2020-10-10T00:00:06, 2020-10-10T00:00:11, 2, 9, 2]",
     "+I[a, 2020-10-10T00:00:06, 2020-10-10T00:00:11, 1, 3, 1]", "+I[b, 2020-10-10T00:00:16, 2020-10-10T00:00:21, 1, 4, 1]"],
    ["+I[b, 2020-10-10T00:00:31, 2020-10-10T00:00:36, 1, 1, 1]", "+I[null, 2020-10-10T00:00:31, 2020-10-10T00:00:36, 1, 7, 0]",
     "+I[a, 2020-10-10T00:00:36, 2020-10-10T00:00:41, 1, 10, 1]", "+I[c, 2020-10-10T00:00:41, 2020-10-10T00:00:46, 1, 12, 1]",
     "+I[d, 2020-10-10T00:00:41, 2020-10-10T00:00:46, 2, 24, 2]"])
_tp("tp_hop_5s_10s", _TPF + ":172-211 HOP_WINDOW_EVENT_TIME(_TWO_PHASE)", "HOP", 10000, 5000, 0,
    ["+I[a, 2020-10-09T23:59:55, 2020-10-10T00:00:05, 4, 10, 2]", "+I[b, 2020-10-10T00:00, 2020-10-10T00:00:10, 2, 9, 2]",
     "+I[a, 2020-10-10T00:00, 2020-10-10T00:00:10, 6, 18, 3]", "+I[b, 2020-10-10T00:00:05, 2020-10-10T00:00:15, 2, 9, 2]",
     "+I[a, 2020-10-10T00:00:05, 2020-10-10T00:00:15, 1, 3, 1]", "+I[b, 2020-10-10T00:00:10, 2020-10-10T00:00:20, 1, 4, 1]",
     "+I[b, 2020-10-10T00:00:15, 2020-10-10T00:00:25, 1, 4, 1]"],
    ["+I[b, 2020-10-10T00:00:25, 2020-10-10T00:00:35, 1, 1, 1]", "+I[null, 2020-10-10T00:00:25, 2020-10-10T00:00:35, 1, 7, 0]",
     "+I[b, 2020-10-10T00:00:30, 2020-10-10T00:00:40, 1, 1, 1]", "+I[null, 2020-10-10T00:00:30, 2020-10-10T00:00:40, 1, 7, 0]",
     "+I[c, 2020-10-10T00:00:35, 2020-10-10T00:00:45, 1, 12, 1]", "+I[d, 2020-10-10T00:00:35, 2020-10-10T00:00:45, 2, 24, 2]",
     "+I[a, 2020-10-10T00:00:35, 2020-10-10T00:00:45, 1, 10, 1]", "+I[d, 2020-10-10T00:00:40, 2020-10-10T00:00:50, 2, 24, 2]",
     "+I[a, 2020-10-10T00:00:40, 2020-10-10T00:00:50, 1, 10, 1]", "+I[c, 2020-10-10T00:00:40, 2020-10-10T00:00:50, 1, 12, 1]"])
_tp("tp_hop_5s_10s_offset_1s", _TPF + ":223-262 HOP_WINDOW_EVENT_TIME(_TWO_PHASE)_WITH_OFFSET", "HOP", 10000, 5000, 1000,
    ["+I[a, 2020-10-09T23:59:56, 2020-10-10T00:00:06, 4, 10, 2]", "+I[b, 2020-10-10T00:00:01, 2020-10-10T00:00:11, 2, 9, 2]",
     "+I[a, 2020-10-10T00:00:01, 2020-10-10T00:00:11, 6, 18, 3]", "+I[b, 2020-10-10T00:00:06, 2020-10-10T00:00:16, 2, 9, 2]",
     "+I[a, 2020-10-10T00:00:06, 2020-10-10T00:00:16, 1, 3, 1]", "+I[b, 2020-10-10T00:00:11, 2020-10-10T00:00:21, 1, 4, 1]",
     "+I[b, 2020-10-10T00:00:16, 2020-10-10T00:00:26, 1, 4, 1]"],
    ["+I[b, 2020-10-10T00:00:26, 2020-10-10T00:00:36, 1, 1, 1]", "+I[null, 2020-10-10T00:00:26, 2020-10-10T00:00:36, 1, 7, 0]",
     "+I[a, 2020-10-10T00:00:31, 2020-10-10T00:00:41, 1, 10, 1]", "+I[b, 2020-10-10T00:00:31, 2020-10-10T00:00:41, 1, 1, 1]",
     "+I[null, 2020-10-10T00:00:31, 2020-10-10T00:00:41, 1, 7, 0]", "+I[c, 2020-10-10T00:00:36, 2020-10-10T00:00:46, 1, 12, 1]",
     "+I[d, 2020-10-10T00:00:36, 2020-10-10T00:00:46, 2, 24, 2]", "+I[a, 2020-10-10T00:00:36, 2020-10-10T00:00:46, 1, 10, 1]",
     "+I[d, 2020-10-10T00:00:41, 2020-10-10T00:00:51, 2, 24, 2]", "+I[c, 2020-10-10T00:00:41, 2020-10-10T00:00:51, 1, 12, 1]"])
_tp("tp_cumulate_5s_15s", _TPF + ":274-313 CUMULATE_WINDOW_EVENT_TIME(_TWO_PHASE)", "CUMULATE", 15000, 5000, 0,
    ["+I[a, 2020-10-10T00:00, 2020-10-10T00:00:05, 4, 10, 2]", "+I[b, 2020-10-10T00:00, 2020-10-10T00:00:10, 2, 9, 2]",
     "+I[a, 2020-10-10T00:00, 2020-10-10T00:00:10, 6, 18, 3]", "+I[b, 2020-10-10T00:00, 2020-10-10T00:00:15, 2, 9, 2]",
     "+I[a, 2020-10-10T00:00, 2020-10-10T00:00:15, 6, 18, 3]", "+I[b, 2020-10-10T00:00:15, 2020-10-10T00:00:20, 1, 4, 1]",
     "+I[b, 2020-10-10T00:00:15, 2020-10-10T00:00:25, 1, 4, 1]", "+I[b, 2020-10-10T00:00:15, 2020-10-10T00:00:30, 1, 4, 1]"],
    ["+I[b, 2020-10-10T00:00:30, 2020-10-10T00:00:35, 1, 1, 1]", "+I[null, 2020-10-10T00:00:30, 2020-10-10T00:00:35, 1, 7, 0]",
     "+I[b, 2020-10-10T00:00:30, 2020-10-10T00:00:40, 1, 1, 1]", "+I[null, 2020-10-10T00:00:30, 2020-10-10T00:00:40, 1, 7, 0]",
     "+I[b, 2020-10-10T00:00:30, 2020-10-10T00:00:45, 1, 1, 1]", "+I[c, 2020-10-10T00:00:30, 2020-10-10T00:00:45, 1, 12, 1]",
     "+I[d, 2020-10-10T00:00:30, 2020-10-10T00:00:45, 2, 24, 2]", "+I[a, 2020-10-10T00:00:30, 2020-10-10T00:00:45, 1, 10, 1]",
     "+I[null, 2020-10-10T00:00:30, 2020-10-10T00:00:45, 1, 7, 0]"])
_tp("tp_cumulate_5s_15s_offset_1s", _TPF + ":325-365 CUMULATE_WINDOW_EVENT_TIME(_TWO_PHASE)_WITH_OFFSET", "CUMULATE", 15000, 5000, 1000,
    ["+I[a, 2020-10-10T00:00:01, 2020-10-10T00:00:06, 4, 10, 2]", "+I[b, 2020-10-10T00:00:01, 2020-10-10T00:00:11, 2, 9, 2]",
     "+I[a, 2020-10-10T00:00:01, 2020-10-10T00:00:11, 6, 18, 3]", "+I[b, 2020-10-10T00:00:01, 2020-10-10T00:00:16, 2, 9, 2]",
     "+I[a, 2020-10-10T00:00:01, 2020-10-10T00:00:16, 6, 18, 3]", "+I[b, 2020-10-10T00:00:16, 2020-10-10T00:00:21, 1, 4, 1]",
     "+I[b, 2020-10-10T00:00:16, 2020-10-10T00:00:26, 1, 4, 1]", "+I[b, 2020-10-10T00:00:16, 2020-10-10T00:00:31, 1, 4, 1]"],
    ["+I[b, 2020-10-10T00:00:31, 2020-10-10T00:00:36, 1, 1, 1]", "+I[null, 2020-10-10T00:00:31, 2020-10-10T00:00:36, 1, 7, 0]",
     "+I[a, 2020-10-10T00:00:31, 2020-10-10T00:00:41, 1, 10, 1]", "+I[b, 2020-10-10T00:00:31, 2020-10-10T00:00:41, 1, 1, 1]",
     "+I[null, 2020-10-10T00:00:31, 2020-10-10T00:00:41, 1, 7, 0]", "+I[b, 2020-10-10T00:00:31, 2020-10-10T00:00:46, 1, 1, 1]",
     "+I[c, 2020-10-10T00:00:31, 2020-10-10T00:00:46, 1, 12, 1]", "+I[d, 2020-10-10T00:00:31, 2020-10-10T00:00:46, 2, 24, 2]",
     "+I[a, 2020-10-10T00:00:31, 2020-10-10T00:00:46, 1, 10, 1]", "+I[null, 2020-10-10T00:00:31, 2020-10-10T00:00:46, 1, 7, 0]"])


# ---------------------------------------------------------------- WindowAggregateITCase MAX(double)
def _itc(name, src, size_ms, offset_ms, rows):
    st = [-(1 << 63)]
    steps = _records(TP_BEFORE, "b_double", st)
    steps.append({"op": "watermark", "wm": INT64_MAX})
    exp = []
    for key, ws, we, cnt, mx in rows:
        exp.append({"key": key, "window_start": _iso_ms(ws), "window_end": _iso_ms(we),
                    "values": [cnt, mx], "nulls": [0, 1 if mx is None else 0]})
    steps.append({"op": "check", "expect": exp})
    FIXTURES.append({
        "name": name, "source": src, "keys": TP_KEYS, "two_phase": True,
        "config": {"api": "SQL", "window": "TUMBLE", "size_ms": size_ms, "slide_ms": 0, "offset_ms": offset_ms,
                   "count_star_index": -1, "key_hash": "PRECOMPUTED", "nullable_cols": [0],
                   "aggs": [["COUNT_STAR", 0, "BIGINT"], ["MAX", 0, "DOUBLE"]], "value_cols": ["DOUBLE"]},
        "steps": steps, "late_dropped": 1 if size_ms == 5000 else 0})


_ITC = "WindowAggregateITCase.scala"
_itc("itc_tumble_5s_max_double", _ITC + ":218-230 testEventTimeTumbleWindow", 5000, 0, [
    ("a", "2020-10-10T00:00", "2020-10-10T00:00:05", 4, 5.0), ("a", "2020-10-10T00:00:05", "2020-10-10T00:00:10", 1, None),
    ("b", "2020-10-10T00:00:05", "2020-10-10T00:00:10", 2, 6.0), ("b", "2020-10-10T00:00:15", "2020-10-10T00:00:20", 1, 4.0),
    ("b", "2020-10-10T00:00:30", "2020-10-10T00:00:35", 1, 3.0), ("null", "2020-10-10T00:00:30", "2020-10-10T00:00:35", 1, 7.0)])
_itc("itc_tumble_1d_offset_8h_max_double", _ITC + ":232-242 testEventTimeTumbleWindowWithOffset", 86400000, 8 * 3600000, [
    ("a", "2020-10-09T08:00", "2020-10-10T08:00", 6, 5.0), ("b", "2020-10-09T08:00", "2020-10-10T08:00", 4, 6.0),
    ("null", "2020-10-09T08:00", "2020-10-10T08:00", 1, 7.0)])
_itc("itc_tumble_1d_offset_neg8h_max_double", _ITC + ":272-282 testEventTimeTumbleWindowWithNegativeOffset", 86400000, -8 * 3600000, [
    ("a", "2020-10-09T16:00", "2020-10-10T16:00", 6, 5.0), ("b", "2020-10-09T16:00", "2020-10-10T16:00", 4, 6.0),
    ("null", "2020-10-09T16:00", "2020-10-10T16:00", 1, 7.0)])


# ---------------------------------------------------------------- SliceAssigner KATs (UTC)
def _u(s):
    return _iso_ms(s)


H = 3600000
_SAT = "flink-table-runtime/src/test/java/org/apache/flink/table/runtime/operators/window/tvf/slicing/"
KATS = [
    # TumblingSliceAssignerTest.java
    {"src": _SAT + "TumblingSliceAssignerTest.java:35-44", "assigner": ["TUMBLE", 5 * H, 0, 0], "op": "slice_end",
     "cases": [[_u("1970-01-01T00:00:00"), _u("1970-01-01T05:00:00")], [_u("1970-01-01T04:59:59.999"), _u("1970-01-01T05:00:00")],
               [_u("1970-01-01T05:00:00"), _u("1970-01-01T10:00:00")]]},
    {"src": _SAT + "TumblingSliceAssignerTest.java:48-58", "assigner": ["TUMBLE", 5 * H, 0, 100], "op": "slice_end",
     "cases": [[_u("1970-01-01T00:00:00.100"), _u("1970-01-01T05:00:00.100")], [_u("1970-01-01T05:00:00.099"), _u("1970-01-01T05:00:00.100")],
               [_u("1970-01-01T05:00:00.100"), _u("1970-01-01T10:00:00.100")]]},
    {"src": _SAT + "TumblingSliceAssignerTest.java:100-108", "assigner": ["TUMBLE", 5 * H, 0, 0], "op": "window_start",
     "cases": [[_u("1970-01-01T00:00:00"), _u("1969-12-31T19:00:00")], [_u("1970-01-01T05:00:00"), _u("1970-01-01T00:00:00")],
               [_u("1970-01-01T10:00:00"), _u("1970-01-01T05:00:00")]]},
    {"src": _SAT + "TumblingSliceAssignerTest.java:113-121", "assigner": ["TUMBLE", 5 * H, 0, 0], "op": "expired_slices",
     "cases": [[_u("1970-01-01T00:00:00"), [_u("1970-01-01T00:00:00")]], [_u("1970-01-01T05:00:00"), [_u("1970-01-01T05:00:00")]],
               [_u("1970-01-01T10:00:00"), [_u("1970-01-01T10:00:00")]]]},
    # HoppingSliceAssignerTest.java
    {"src": _SAT + "HoppingSliceAssignerTest.java:37-47", "assigner": ["HOP", 5 * H, 1 * H, 0], "op": "slice_end",
     "cases": [[_u("1970-01-01T00:00:00"), _u("1970-01-01T01:00:00")], [_u("1970-01-01T04:59:59.999"), _u("1970-01-01T05:00:00")],
               [_u("1970-01-01T05:00:00"), _u("1970-01-01T06:00:00")]]},
    {"src": _SAT + "HoppingSliceAssignerTest.java:51-63", "assigner": ["HOP", 5 * H, 1 * H, 100], "op": "slice_end",
     "cases": [[_u("1970-01-01T00:00:00.100"), _u("1970-01-01T01:00:00.100")], [_u("1970-01-01T05:00:00.099"), _u("1970-01-01T05:00:00.100")],
               [_u("1970-01-01T05:00:00.100"), _u("1970-01-01T06:00:00.100")]]},
    {"src": _SAT + "HoppingSliceAssignerTest.java:109-128", "assigner": ["HOP", 5 * H, 1 * H, 0], "op": "window_start",
     "cases": [[_u("1970-01-01T%02d:00:00" % h), _u("1970-01-01T%02d:00:00" % (h - 5)) if h >= 5 else
                _u("1969-12-31T%02d:00:00" % (h + 19))] for h in (0, 1, 2, 3, 4, 5, 6, 10)]},
    {"src": _SAT + "HoppingSliceAssignerTest.java:132-141", "assigner": ["HOP", 4 * H, 1 * H, 0], "op": "expired_slices",
     "cases": [[_u("1970-01-01T00:00:00"), [_u("1969-12-31T21:00:00")]], [_u("1970-01-01T04:00:00"), [_u("1970-01-01T01:00:00")]],
               [_u("1970-01-01T08:00:00"), [_u("1970-01-01T05:00:00")]]]},
    {"src": _SAT + "HoppingSliceAssignerTest.java:143-173", "assigner": ["HOP", 5 * H, 1 * H, 0], "op": "merge",
     "cases": [[_u("1970-01-01T00:00:00"), [None, [_u("1970-01-01T00:00:00"), _u("1969-12-31T23:00:00"), _u("1969-12-31T22:00:00"),
                                                    _u("1969-12-31T21:00:00"), _u("1969-12-31T20:00:00")]]],
               [_u("1970-01-01T05:00:00"), [None, [_u("1970-01-01T0%d:00:00" % h) for h in (5, 4, 3, 2, 1)]]],
               [_u("1970-01-01T06:00:00"), [None, [_u("1970-01-01T0%d:00:00" % h) for h in (6, 5, 4, 3, 2)]]]]},
    {"src": _SAT + "HoppingSliceAssignerTest.java:177-210 (window not empty / empty)", "assigner": ["HOP", 5 * H, 1 * H, 0],
     "op": "next_trigger", "cases": [[[_u("1970-01-01T0%d:00:00" % h), False], _u("1970-01-01T0%d:00:00" % (h + 1))] for h in range(7)]
     + [[[_u("1970-01-01T0%d:00:00" % h), True], None] for h in range(7)]},
    # CumulativeSliceAssignerTest.java
    {"src": _SAT + "CumulativeSliceAssignerTest.java testSliceAssignment", "assigner": ["CUMULATE", 24 * H, 1 * H, 0], "op": "slice_end",
     "cases": [[_u("1970-01-01T00:00:00"), _u("1970-01-01T01:00:00")], [_u("1970-01-02T22:59:59.999"), _u("1970-01-02T23:00:00")],
               [_u("1970-01-02T23:00:00"), _u("1970-01-03T00:00:00")]]},
    {"src": _SAT + "CumulativeSliceAssignerTest.java testSliceAssignmentWithOffset", "assigner": ["CUMULATE", 5 * H, 1 * H, 100], "op": "slice_end",
     "cases": [[_u("1970-01-01T00:00:00.100"), _u("1970-01-01T01:00:00.100")], [_u("1970-01-01T05:00:00.099"), _u("1970-01-01T05:00:00.100")],
               [_u("1970-01-01T05:00:00.100"), _u("1970-01-01T06:00:00.100")]]},
    {"src": _SAT + "CumulativeSliceAssignerTest.java testGetWindowStart", "assigner": ["CUMULATE", 5 * H, 1 * H, 0], "op": "window_start",
     "cases": [[_u("1970-01-01T00:00:00"), _u("1969-12-31T19:00:00")]] +
              [[_u("1970-01-01T0%d:00:00" % h), _u("1970-01-01T00:00:00")] for h in (1, 2, 3, 4, 5)] +
              [[_u("1970-01-01T06:00:00"), _u("1970-01-01T05:00:00")], [_u("1970-01-01T08:00:00"), _u("1970-01-01T05:00:00")]]},
    {"src": _SAT + "CumulativeSliceAssignerTest.java testExpiredSlices", "assigner": ["CUMULATE", 5 * H, 1 * H, 0], "op": "expired_slices",
     "cases": [[_u("1970-01-01T01:00:00"), []]] + [[_u("1970-01-01T0%d:00:00" % h), [_u("1970-01-01T0%d:00:00" % h)]] for h in (2, 3, 4)] +
              [[_u("1970-01-01T05:00:00"), [_u("1970-01-01T05:00:00"), _u("1970-01-01T01:00:00")]],
               [_u("1970-01-01T06:00:00"), []],
               [_u("1970-01-01T10:00:00"), [_u("1970-01-01T10:00:00"), _u("1970-01-01T06:00:00")]],
               [_u("1970-01-01T00:00:00"), [_u("1970-01-01T00:00:00"), _u("1969-12-31T20:00:00")]]]},
    {"src": _SAT + "CumulativeSliceAssignerTest.java testMerge", "assigner": ["CUMULATE", 5 * H, 1 * H, 0], "op": "merge",
     "cases": [[_u("1970-01-01T01:00:00"), [_u("1970-01-01T01:00:00"), []]]] +
              [[_u("1970-01-01T0%d:00:00" % h), [_u("1970-01-01T01:00:00"), [_u("1970-01-01T0%d:00:00" % h)]]] for h in (2, 3, 4, 5)] +
              [[_u("1970-01-01T06:00:00"), [_u("1970-01-01T06:00:00"), []]],
               [_u("1970-01-01T08:00:00"), [_u("1970-01-01T06:00:00"), [_u("1970-01-01T08:00:00")]]],
               [_u("1970-01-01T10:00:00"), [_u("1970-01-01T06:00:00"), [_u("1970-01-01T10:00:00")]]],
               [_u("1970-01-01T00:00:00"), [_u("1969-12-31T20:00:00"), [_u("1970-01-01T00:00:00")]]]]},
    {"src": _SAT + "CumulativeSliceAssignerTest.java testNextTriggerWindow", "assigner": ["CUMULATE", 5 * H, 1 * H, 0], "op": "next_trigger",
     "cases": [[[_u("1970-01-01T0%d:00:00" % h, ), empty], (None if h in (0, 5) else _u("1970-01-01T0%d:00:00" % (h + 1)))]
               for empty in (False, True) for h in range(7)]},
]


# ---------------------------------------------------------------- TIMESTAMP_LTZ: Asia/Shanghai
_SH = 8 * H


def _shanghai(name):
    import copy
    f = copy.deepcopy(next(x for x in FIXTURES if x["name"] == name))
    f["name"] = name + "_shanghai"
    f["source"] += " [TimeZone = Asia/Shanghai: window props = localMills(epoch)]"
    f["config"]["shift_zone"] = "Asia/Shanghai"
    for st in f["steps"]:
        for r in st.get("expect", []):
            r["window_start"] += _SH
            r["window_end"] += _SH
    return f


FIXTURES += [_shanghai(n) for n in ("sql_hop_3s_1s", "sql_hop_expired_slice_restore", "sql_hop_expired_slice_norestore",
                                    "sql_cumulate_3s_1s", "sql_tumble_3s")]

# ---------------------------------------------------------------- DST KATs (America/Los_Angeles)
_LA_EPOCHS = [1615708800000, 1615712400000, 1615716000000, 1615719600000,
              1636268400000, 1636272000000, 1636275600000, 1636279200000, 1636282800000, 1636286400000]


def _dst(src, kind, size, slide, pairs):
    # assertSliceStartEnd(start, end, epochMills, assigner): the local wall-clock strings of
    # getWindowStart(assignSliceEnd(epoch)) and assignSliceEnd(epoch)
    return {"src": _SAT + src, "assigner": [kind, size, slide, 0], "zone": "America/Los_Angeles", "op": "dst_slice",
            "cases": [[e, [_u(a + ":00"), _u(b + ":00")]] for e, (a, b) in zip(_LA_EPOCHS, pairs)]}


KATS += [
    _dst("TumblingSliceAssignerTest.java:63-96 testDstSaving", "TUMBLE", 4 * H, 0,
         [("2021-03-14T00:00", "2021-03-14T04:00")] * 3 + [("2021-03-14T04:00", "2021-03-14T08:00")] +
         [("2021-11-07T00:00", "2021-11-07T04:00")] * 5 + [("2021-11-07T04:00", "2021-11-07T08:00")]),
    _dst("HoppingSliceAssignerTest.java:66-100 testDstSaving", "HOP", 4 * H, 1 * H,
         [("2021-03-13T21:00", "2021-03-14T01:00"), ("2021-03-13T22:00", "2021-03-14T02:00"),
          ("2021-03-14T00:00", "2021-03-14T04:00"), ("2021-03-14T01:00", "2021-03-14T05:00"),
          ("2021-11-06T21:00", "2021-11-07T01:00"), ("2021-11-06T22:00", "2021-11-07T02:00"),
          ("2021-11-06T22:00", "2021-11-07T02:00"), ("2021-11-06T23:00", "2021-11-07T03:00"),
          ("2021-11-07T00:00", "2021-11-07T04:00"), ("2021-11-07T01:00", "2021-11-07T05:00")]),
    _dst("CumulativeSliceAssignerTest.java:66-100 testDstSaving", "CUMULATE", 4 * H, 1 * H,
         [("2021-03-14T00:00", "2021-03-14T01:00"), ("2021-03-14T00:00", "2021-03-14T02:00"),
          ("2021-03-14T00:00", "2021-03-14T04:00"), ("2021-03-14T04:00", "2021-03-14T05:00"),
          ("2021-11-07T00:00", "2021-11-07T01:00"), ("2021-11-07T00:00", "2021-11-07T02:00"),
          ("2021-11-07T00:00", "2021-11-07T02:00"), ("2021-11-07T00:00", "2021-11-07T03:00"),
          ("2021-11-07T00:00", "2021-11-07T04:00"), ("2021-11-07T04:00", "2021-11-07T05:00")]),
]


def main():
    with open(os.path.join(HERE, "slice_assigner_kats.json"), "w") as fh:
        json.dump(KATS, fh, indent=1)
    for f in FIXTURES:
        f.setdefault("keys", KEYS)
        with open(os.path.join(HERE, f["name"] + ".json"), "w") as fh:
            json.dump(f, fh, indent=1)
    print(f"wrote {len(FIXTURES)} fixtures")


if __name__ == "__main__":
    main()
