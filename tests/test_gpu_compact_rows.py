"""GPU parity of the compact partial-row formats (fw_internal.h PF_NARROW / PF_UNIT / PF_PACK).

For COUNT(*)-only layouts (and, with FW_NARROW1=1, every one-word layout) an ingest chunk whose rows
all take the common SQL path stores only the key (PF_UNIT; (key, acc) when rows folded or the word
is a SUM / MIN / MAX: PF_NARROW) and the slice end as a rank byte against the push's rank base; any other chunk of the same push stores full (key,
sliceEnd, acc) rows.  These
streams mix both in every push (late rows and far-future rows force single chunks wide), run several
pushes per watermark, and compare every watermark's results with the oracle; the device counters
must show that compact chunks were written -- and none for the wider layouts, which keep full rows
(DESIGN.md 3).  One-word integer TUMBLE layouts (runs) write PF_PACK rows: one 8-B word per partial
with the key and the accumulator as offsets from the flush epoch's bases, sized from the previous
push's ranges; a chunk with a row outside them writes PF_WIDE rows."""
import os
import zlib

import numpy as np
import pytest

from flink_amd import abi
from parity_common import F64, I64, _cfg, _double_cols, _run_both

pytestmark = pytest.mark.gpu

T0 = 1_600_000_000_000
CH = 4096  # ingest chunk rows of these layouts (<= 2 accumulator words: 512 threads x 8 rows)


def _stream(seed, n_wm, per, n_keys, step_ms, ooo, slice_ms, late_every=3, far_every=4, hot=False):
    """Batches whose rows are on time except: every late_every-th batch puts late rows into its
    third chunk (some dropped, some merged into unfired windows), every far_every-th batch puts one
    row > 255 slices ahead of the watermark into its second chunk; hot: power-law keys (the ingest
    fold merges rows, so COUNT(*) chunks are PF_NARROW rather than PF_UNIT)."""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_wm):
        base = T0 + b * step_ms
        ts = base + rng.integers(0, step_ms, per) - rng.integers(0, ooo, per)
        prev_wm = base - ooo - 1
        if late_every and b % late_every == late_every - 1 and per > 3 * CH:
            i = 2 * CH + rng.integers(0, CH, 40)
            ts[i] = prev_wm - rng.integers(0, 3 * slice_ms, 40)
        if far_every and b % far_every == 1 and per > 2 * CH:
            ts[CH + 17] = base + 300 * slice_ms
        if hot:
            keys = (rng.pareto(1.2, per) * 3).astype(np.int64) % n_keys
        else:
            keys = rng.integers(0, n_keys, per).astype(np.int64)
        keys = keys * 104729 + 11
        iv = rng.integers(-10**6, 10**6, per).astype(np.int64)
        dv = rng.random(per) * 1000.0
        out.append((keys, ts.astype(np.int64), iv, dv, base + step_ms - ooo - 1))
    return out


CASES = {
    # TUMBLE: PF_NARROW (key, max) / PF_UNIT (COUNT(*) alone)
    "tumble_max": dict(window_kind=abi.WIN_TUMBLE, size_ms=10000, aggs=[(abi.AGG_MAX, 0, I64)]),
    "tumble_count_star": dict(window_kind=abi.WIN_TUMBLE, size_ms=5000, aggs=[(abi.AGG_COUNT_STAR, 0, I64)]),
    "tumble_sum_avg_double": dict(window_kind=abi.WIN_TUMBLE, size_ms=4000,
                                  aggs=[(abi.AGG_SUM, 1, F64), (abi.AGG_AVG, 1, F64)]),
    # HOP with block state (k_merge_hopb): COUNT(*) alone -> PF_UNIT
    "hop_count_star": dict(window_kind=abi.WIN_HOP, size_ms=10000, slide_ms=2000, count_star_index=0,
                           aggs=[(abi.AGG_COUNT_STAR, 0, I64)]),
    "hop_count_sum": dict(window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=2000, count_star_index=0,
                          aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64)]),
    # HOP with a slice per entry (k_merge_fire): more slices than a block holds
    "hop_many_slices": dict(window_kind=abi.WIN_HOP, size_ms=10000, slide_ms=1000, count_star_index=0,
                            aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_MAX, 0, I64)]),
    "cumulate_4aggs": dict(window_kind=abi.WIN_CUMULATE, size_ms=12000, slide_ms=2000, count_star_index=0,
                           aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MIN, 0, I64),
                                 (abi.AGG_MAX, 0, I64)]),
    "cumulate_count_star": dict(window_kind=abi.WIN_CUMULATE, size_ms=12000, slide_ms=3000, count_star_index=0,
                                aggs=[(abi.AGG_COUNT_STAR, 0, I64)]),
    "tumble_offset_count_star": dict(window_kind=abi.WIN_TUMBLE, size_ms=7000, offset_ms=-2500, count_star_index=0,
                                     aggs=[(abi.AGG_COUNT_STAR, 0, I64)]),
    "tumble_offset_min": dict(window_kind=abi.WIN_TUMBLE, size_ms=7000, offset_ms=-2500,
                              aggs=[(abi.AGG_MIN, 0, I64), (abi.AGG_COUNT_STAR, 0, I64)]),
}


def _slice_ms(kw):
    return kw.get("slide_ms", kw["size_ms"]) if kw["window_kind"] != abi.WIN_TUMBLE else kw["size_ms"]


@pytest.mark.parametrize("hot", [False, True], ids=["uniform", "hot"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_compact_partial_rows_match_oracle(name, hot):
    kw = CASES[name]
    sl = _slice_ms(kw)
    batches = _stream(zlib.crc32(name.encode()) % 1000 + hot, n_wm=14, per=6 * CH + 333, n_keys=30000,
                      step_ms=3000, ooo=4000, slice_ms=sl, hot=hot)
    st = {}
    _run_both(_cfg(kw, state_capacity=1 << 18, max_batch_rows=1 << 15), batches, _double_cols(kw), split=2, stats=st)
    chunks = 14 * 2 * 4  # 14 watermarks x 2 pushes x 4 chunks (per = 6 chunks + 333 rows, split in two)
    # COUNT(*) alone -- or, with FW_NARROW1=1, one NOT NULL SUM / MIN / MAX, and with runs (TUMBLE) one
    # integer SUM / MIN / MAX in PF_PACK rows -- writes compact rows
    one = len(kw["aggs"]) == 1 and kw["aggs"][0][0] in (abi.AGG_MAX, abi.AGG_MIN, abi.AGG_SUM)
    pack = one and kw["aggs"][0][2] == I64 and kw["window_kind"] == abi.WIN_TUMBLE and os.environ.get("FW_PACK") != "0"
    if kw["aggs"] == [(abi.AGG_COUNT_STAR, 0, I64)] or (one and os.environ.get("FW_NARROW1") == "1") or pack:
        assert st["compact_chunks"] > chunks // 2, st   # the common path writes compact rows ...
        assert st["compact_chunks"] < chunks, st        # ... and the late / far rows force some chunks wide
    else:
        assert st["compact_chunks"] == 0, st
    assert st["partial_bytes_written"] > 0 and st["partial_bytes_merged"] <= st["partial_bytes_written"]


def test_compact_rows_local_phase_matches_oracle():
    """The LOCAL phase (two-phase, LocalSlicingWindowAggOperator) keeps no late handling: compact
    chunks there, and every flushed (key, slice) partial is emitted."""
    kw = dict(window_kind=abi.WIN_HOP, size_ms=8000, slide_ms=2000, count_star_index=0, agg_phase=abi.PHASE_LOCAL,
              aggs=[(abi.AGG_COUNT_STAR, 0, I64)])
    batches = _stream(7, n_wm=10, per=5 * CH, n_keys=20000, step_ms=3000, ooo=4000, slice_ms=2000)
    st = {}
    _run_both(_cfg(kw, max_batch_rows=1 << 15), batches, set(), split=1, stats=st)
    assert st["compact_chunks"] > 0


def test_compact_rows_off_matches_compact_rows_on(monkeypatch):
    """FW_NARROW=0 (every chunk PF_WIDE) and the default give the same results and late counts."""
    from flink_amd.runtime.handle import WindowAggHandle
    kw = dict(window_kind=abi.WIN_CUMULATE, size_ms=12000, slide_ms=2000, count_star_index=0,
              aggs=[(abi.AGG_COUNT_STAR, 0, I64)])
    batches = _stream(11, n_wm=8, per=5 * CH, n_keys=5000, step_ms=3000, ooo=4000, slice_ms=2000)
    outs = []
    for env in ("0", "1"):
        monkeypatch.setenv("FW_NARROW", env)
        g = WindowAggHandle(_cfg(kw, max_batch_rows=1 << 15))
        rows = []
        for k, t, iv, dv, wm in batches:
            g.push_host(k, t, [iv, dv.view(np.int64)])
            g.advance(wm)
            r = g.results(reset=True)
            rows += sorted(zip(r["key"].tolist(), r["window_end"].tolist(), *[v.tolist() for v in r["values"]]))
        st = g.stats()
        g.close()
        outs.append((rows, st["num_late_records_dropped"], st["compact_chunks"] > 0))
    assert outs[0][0] == outs[1][0] and outs[0][1] == outs[1][1]
    assert (outs[0][2], outs[1][2]) == (False, True)


PACK_CASES = {
    "max": [(abi.AGG_MAX, 0, I64)],
    "min": [(abi.AGG_MIN, 0, I64)],
    "sum": [(abi.AGG_SUM, 0, I64)],
    "count_star": [(abi.AGG_COUNT_STAR, 0, I64)],
}


@pytest.mark.parametrize("name", sorted(PACK_CASES))
def test_packed_rows_mixed_with_wide_pushes_match_oracle(name):
    """PF_PACK pushes and wide pushes in the same flush epoch: every third batch moves its keys 2^40 up
    (outside the epoch's key field: every chunk of those pushes writes PF_WIDE rows into its region),
    hot keys fold sums past the accumulator field, late and far-future rows force single chunks wide;
    two pushes per watermark, several watermarks per flush.  Results and late counts match the oracle,
    and both formats were written."""
    aggs = PACK_CASES[name]
    kw = dict(window_kind=abi.WIN_TUMBLE, size_ms=6000, aggs=aggs)
    if aggs[0][0] == abi.AGG_COUNT_STAR:
        kw["count_star_index"] = 0
    batches = _stream(zlib.crc32(name.encode()) % 1000, n_wm=12, per=6 * CH + 333, n_keys=20000, step_ms=2000,
                      ooo=3000, slice_ms=6000, hot=name == "sum")
    for b, (k, t, iv, dv, wm) in enumerate(batches):
        if b % 3 == 2:
            k += np.int64(1) << 40
        if name == "sum" and b % 4 == 3:
            iv[:64] = np.int64(1) << 50  # hot-key sums far outside the previous push's accumulator range
    st = {}
    _run_both(_cfg(kw, state_capacity=1 << 18, max_batch_rows=1 << 15), batches, set(), split=2, stats=st)
    chunks = 12 * 2 * 4  # 12 watermarks x 2 pushes x 4 chunks
    assert 0 < st["compact_chunks"] < chunks, st
    assert st["partial_bytes_written"] > 0 and st["partial_bytes_merged"] <= st["partial_bytes_written"]


def test_packed_rows_off_matches_packed_rows_on(monkeypatch):
    """FW_PACK=0 (no PF_PACK rows) and the default give the same results and late counts."""
    from flink_amd.runtime.handle import WindowAggHandle
    kw = dict(window_kind=abi.WIN_TUMBLE, size_ms=5000, aggs=[(abi.AGG_MAX, 0, I64)])
    batches = _stream(13, n_wm=8, per=5 * CH, n_keys=5000, step_ms=3000, ooo=4000, slice_ms=5000)
    outs = []
    for env in ("0", "1"):
        monkeypatch.setenv("FW_PACK", env)
        g = WindowAggHandle(_cfg(kw, max_batch_rows=1 << 15))
        rows = []
        for k, t, iv, dv, wm in batches:
            g.push_host(k, t, [iv, dv.view(np.int64)])
            g.advance(wm)
            r = g.results(reset=True)
            rows += sorted(zip(r["key"].tolist(), r["window_end"].tolist(), *[v.tolist() for v in r["values"]]))
        st = g.stats()
        g.close()
        outs.append((rows, st["num_late_records_dropped"], st["compact_chunks"] > 0))
    assert outs[0][0] == outs[1][0] and outs[0][1] == outs[1][1]
    assert (outs[0][2], outs[1][2]) == (False, True)
