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


def main():
    for f in FIXTURES:
        f.setdefault("keys", KEYS)
        with open(os.path.join(HERE, f["name"] + ".json"), "w") as fh:
            json.dump(f, fh, indent=1)
    print(f"wrote {len(FIXTURES)} fixtures")


if __name__ == "__main__":
    main()
