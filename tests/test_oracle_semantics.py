"""Pins the oracle's aggregate semantics that no reference fixture covers, with expected values
derived by hand from the reference's aggregate-function expressions:

* SQL MAX/MIN(DOUBLE): MaxAggFunction.java:63-72 / MinAggFunction.java keep the first non-NULL
  value and replace it only on a strict `>` / `<` (NaN compares false both ways, -0.0 == +0.0),
  and merge slices the same way on their result values (MaxAggFunction.java:82-95).
* DataStream max/min(double): ComparableAggregator + Comparator (Comparator.java:48-101) use
  Double.compareTo, a total order with -0.0 < +0.0 and NaN greatest.  MaxComparator.isExtremal is 1
  only when the accumulator is strictly greater, and ComparableAggregator.reduce (:83-104) sets the
  field to the new value otherwise, so ties -- all NaNs compare equal -- go to the LATER element.
* DataStream output records: value1 (the window's first element) with the field set
  (SumAggregator.java:66-76): the oracle reports that element's arrival ordinal.
* NULL inputs: SumAggFunction.java:66-69 (NULL until a non-NULL operand), CountAggFunction.java:60-87
  (counts non-NULL operands), AvgAggFunction.java:79-105 (sum and count of non-NULL operands; NULL
  result when the count is 0), Max/MinAggFunction (NULL operands skipped).
CPU only: the oracle is the checker the GPU parity tests trust."""
import math
import struct

import numpy as np
import pytest

from flink_amd import abi
from oracle.oracle import OracleOperator

T0 = 1_600_000_000_000
NAN2 = struct.unpack("<d", struct.pack("<Q", 0xFFF8000000000001))[0]  # non-canonical NaN payload


def bits(x):
    return struct.unpack("<q", struct.pack("<d", x))[0]


def run(values, aggs, api=abi.API_SQL, nulls=None, window=(abi.WIN_TUMBLE, 10_000, 0), count_star=-1, wms=None):
    kind, size, slide = window
    cfg = abi.make_config(api=api, window_kind=kind, size_ms=size, slide_ms=slide, aggs=aggs,
                          count_star_index=count_star, value_col_types=[abi.T_F64, abi.T_I64],
                          nullable_cols=[0, 1] if nulls is not None else [], key_hash=abi.KEYHASH_LONG)
    o = OracleOperator(cfg)
    n = len(values)
    dv = np.array(values, dtype=np.float64)
    iv = np.arange(n, dtype=np.int64) - 3
    nl = None if nulls is None else {0: np.array(nulls, np.uint8), 1: np.array(nulls, np.uint8)}
    o.process_batch(np.zeros(n, np.int64), T0 + np.arange(n, dtype=np.int64), [dv.view(np.int64), iv], nl)
    for w in (wms or [T0 + 10**6]):
        o.process_watermark(w)
    r = o.results()
    o.close()
    return r


def test_sql_max_min_double_strict_first_seen():
    cases = [  # (inputs, SQL MAX, SQL MIN)
        ([-0.0, 0.0], -0.0, -0.0),
        ([0.0, -0.0], 0.0, 0.0),
        ([1.0, math.nan], 1.0, 1.0),
        ([math.nan, 1.0], math.nan, math.nan),
        ([NAN2, 5.0, math.nan], NAN2, NAN2),
        ([3.0, -0.0, 1.0, 0.0], 3.0, -0.0),
        ([-3.0, 0.0, -0.0, -1.0], 0.0, -3.0),
        ([2.0, math.nan, 7.0, -1.0], 7.0, -1.0),
    ]
    for vals, mx, mn in cases:
        r = run(vals, [(abi.AGG_MAX, 0, abi.T_F64), (abi.AGG_MIN, 0, abi.T_F64)])
        assert r["values"][0][0] == bits(mx), (vals, "MAX")
        assert r["values"][1][0] == bits(mn), (vals, "MIN")


def test_datastream_max_min_double_total_order():
    for vals, mx, mn in [([-0.0, 0.0], 0.0, -0.0), ([1.0, math.nan], math.nan, 1.0), ([0.0, -0.0], 0.0, -0.0)]:
        rmax = run(vals, [(abi.AGG_MAX, 0, abi.T_F64)], api=abi.API_DATASTREAM)
        rmin = run(vals, [(abi.AGG_MIN, 0, abi.T_F64)], api=abi.API_DATASTREAM)
        got_max = struct.unpack("<d", struct.pack("<q", int(rmax["values"][0][0])))[0]
        assert (math.isnan(got_max) and math.isnan(mx)) or rmax["values"][0][0] == bits(mx)
        assert rmin["values"][0][0] == bits(mn)


def test_sql_nulls_are_skipped():
    aggs = [(abi.AGG_COUNT_STAR, 0, abi.T_I64), (abi.AGG_COUNT, 1, abi.T_I64), (abi.AGG_SUM, 1, abi.T_I64),
            (abi.AGG_MAX, 1, abi.T_I64), (abi.AGG_AVG, 1, abi.T_I64), (abi.AGG_SUM, 0, abi.T_F64),
            (abi.AGG_MIN, 0, abi.T_F64)]
    # ints are -3, -2, -1, 0; the last two rows are NULL in both columns
    r = run([1.5, 2.5, 100.0, -7.0], aggs, nulls=[0, 0, 1, 1])
    assert [int(r["values"][a][0]) for a in range(5)] == [4, 2, -5, -2, -5 // 2 + 1]  # AVG: Java truncation -5/2 = -2
    assert r["values"][5][0] == bits(4.0) and r["values"][6][0] == bits(1.5)
    assert r["null_mask"][0] == 0
    # every value NULL: COUNT(col) = 0, SUM / MAX / AVG / MIN are NULL, COUNT(*) counts rows
    r = run([1.0, 2.0], aggs, nulls=[1, 1])
    assert int(r["values"][0][0]) == 2 and int(r["values"][1][0]) == 0
    assert r["null_mask"][0] == (1 << 2) | (1 << 3) | (1 << 4) | (1 << 5) | (1 << 6)


def test_sql_hop_merge_uses_result_values():
    # HOP 2 s / 1 s: window [0, 2000) merges slice 2000 first (newest-first), then slice 1000.
    # Slice 1000 = [1.0], slice 2000 = [NaN, 5.0]: slice 2000's MAX is NaN (first value), so the
    # merge sees NaN > 1.0 == false ... taken first as the merge target is null, then 1.0 > NaN
    # is false too: the window MAX is NaN.  Element order would give 5.0.
    cfg = abi.make_config(window_kind=abi.WIN_HOP, size_ms=2000, slide_ms=1000, count_star_index=1,
                          aggs=[(abi.AGG_MAX, 0, abi.T_F64), (abi.AGG_COUNT_STAR, 0, abi.T_I64)],
                          value_col_types=[abi.T_F64], key_hash=abi.KEYHASH_LONG)
    o = OracleOperator(cfg)
    ts = np.array([T0 + 100, T0 + 1100, T0 + 1200], np.int64)
    dv = np.array([1.0, math.nan, 5.0])
    o.process_batch(np.zeros(3, np.int64), ts, [dv.view(np.int64)])
    o.process_watermark(T0 + 1999)
    r = o.results()
    we = list(r["window_end"])
    i = we.index(T0 + 2000)
    assert math.isnan(struct.unpack("<d", struct.pack("<q", int(r["values"][0][i])))[0])
    o.close()


NAN3 = struct.unpack("<d", struct.pack("<Q", 0x7FF0000000000001))[0]  # signalling-NaN payload


def test_datastream_ties_go_to_the_later_element():
    # (inputs, DataStream max, DataStream min) -- NaN bit patterns compared exactly
    cases = [
        ([NAN2, math.nan], math.nan, math.nan),      # both NaN: the later one, for max and min
        ([math.nan, NAN2], NAN2, NAN2),
        ([NAN2, 1.0, NAN3, 2.0], NAN3, 1.0),         # max: the last NaN; min: the least non-NaN
        ([NAN3, NAN2, -0.0, 0.0], NAN2, -0.0),
        ([0.0, -0.0, 0.0], 0.0, -0.0),
    ]
    for vals, mx, mn in cases:
        rmax = run(vals, [(abi.AGG_MAX, 0, abi.T_F64)], api=abi.API_DATASTREAM)
        rmin = run(vals, [(abi.AGG_MIN, 0, abi.T_F64)], api=abi.API_DATASTREAM)
        assert rmax["values"][0][0] == bits(mx), (vals, "max", hex(int(rmax["values"][0][0]) & (2**64 - 1)))
        assert rmin["values"][0][0] == bits(mn), (vals, "min", hex(int(rmin["values"][0][0]) & (2**64 - 1)))


def test_datastream_first_element_ordinal():
    # one key, sliding 2 s / 1 s: rows at T0+0.., each window's first element is its earliest
    # arrival (push << 32 | row), whatever its timestamp
    cfg = abi.make_config(api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP, size_ms=2000, slide_ms=1000,
                          aggs=[(abi.AGG_SUM, 0, abi.T_I64)], value_col_types=[abi.T_I64], key_hash=abi.KEYHASH_LONG)
    o = OracleOperator(cfg)
    o.process_batch(np.zeros(3, np.int64), np.array([T0 + 1500, T0 + 200, T0 + 1700], np.int64), [np.arange(3, dtype=np.int64)])
    o.process_batch(np.zeros(2, np.int64), np.array([T0 + 2500, T0 + 100], np.int64), [np.arange(2, dtype=np.int64)])
    o.process_watermark(T0 + 10_000)
    r = o.results()
    got = dict(zip(r["window_end"].tolist(), r["first_ord"].tolist()))
    assert got == {T0 + 1000: 1, T0 + 2000: 0, T0 + 3000: 0, T0 + 4000: (1 << 32) | 0}
    o.close()


def test_datastream_sliding_windows_slide_not_dividing_size():
    """SlidingEventTimeWindows with slide not dividing size (5 s / 2 s, offset 1 s): every element
    belongs to the windows SlidingEventTimeWindows.assignWindows (:77-90) lists for it -- 2 or 3 of
    them here -- and each fired window holds the sum of exactly those elements.  The expected rows
    come from the assigner's own loop (windowing.py mirrors it), not from the oracle."""
    from flink_amd.datastream.windowing import SlidingEventTimeWindows
    size, slide, off = 5000, 2000, 1000
    asg = SlidingEventTimeWindows.of(size, slide, off)
    cfg = abi.make_config(api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP, size_ms=size, slide_ms=slide, offset_ms=off,
                          aggs=[(abi.AGG_SUM, 0, abi.T_I64)], value_col_types=[abi.T_I64], key_hash=abi.KEYHASH_LONG)
    rng = np.random.default_rng(7)
    n = 4000
    keys = rng.integers(0, 17, n).astype(np.int64)
    ts = (T0 + rng.integers(0, 40_000, n)).astype(np.int64)
    vals = rng.integers(-1000, 1000, n).astype(np.int64)
    want = {}
    for k, t, v in zip(keys.tolist(), ts.tolist(), vals.tolist()):
        wins = asg.assign_windows(t)
        assert len(wins) in (2, 3)
        for s, e in wins:
            want[(k, e)] = want.get((k, e), 0) + v
    o = OracleOperator(cfg)
    o.process_batch(keys, ts, [vals])
    o.process_watermark(T0 + 60_000)
    r = o.results()
    got = {(int(k), int(e)): int(v) for k, e, v in zip(r["key"], r["window_end"], r["values"][0])}
    o.close()
    assert got == want


@pytest.mark.parametrize("fn,last,vals,want_row", [
    # maxBy: 7 arrives at rows 1 and 2 -- the first (default) keeps row 1, first=false takes row 2
    ("MAXBY", False, [5, 7, 7, 2], 1),
    ("MAXBY", True, [5, 7, 7, 2], 2),
    ("MINBY", False, [5, 2, 9, 2], 1),
    ("MINBY", True, [5, 2, 9, 2], 3),
    # Double.compareTo: -0.0 < 0.0, NaN above everything and every NaN equal to every other
    ("MINBY_D", False, [0.0, -0.0, 1.0, -0.0], 1),
    ("MAXBY_D", False, [1.0, float("nan"), 5.0, float("nan")], 1),
    ("MAXBY_D", True, [1.0, float("nan"), 5.0, float("nan")], 3),
])
def test_datastream_minby_maxby_tie_rules(fn, last, vals, want_row):
    """ComparableAggregator.reduce with byAggregate (:89-96): value1 (the state) stays when it is
    strictly extremal (MaxByComparator / MinByComparator, Comparator.java:58-101), and on a tie iff
    `first`; the window emits that ELEMENT (its arrival ordinal is the result's first_ord)."""
    dbl = fn.endswith("_D")
    kind = abi.AGG_MAXBY if fn.startswith("MAXBY") else abi.AGG_MINBY
    t = abi.T_F64 if dbl else abi.T_I64
    cfg = abi.make_config(api=abi.API_DATASTREAM, window_kind=abi.WIN_TUMBLE, size_ms=10_000,
                          aggs=[(kind, 0, t, abi.AGGF_LAST if last else 0)], value_col_types=[t],
                          key_hash=abi.KEYHASH_LONG, ds_first_ordinals=1)
    o = OracleOperator(cfg)
    n = len(vals)
    v = np.array(vals, np.float64).view(np.int64) if dbl else np.array(vals, np.int64)
    o.process_batch(np.full(n, 3, np.int64), np.arange(T0, T0 + n, dtype=np.int64), [v])
    o.process_watermark(T0 + 20_000)
    r = o.results()
    o.close()
    assert r["first_ord"].tolist() == [want_row]  # push 0, row want_row
    assert r["values"][0].tolist() == [int(v[want_row])]
