"""Shared helpers of the GPU parity tests: randomized streams, the GPU-vs-oracle runner and the
comparison rules (integer, window and DOUBLE MIN/MAX results bit-exact; DOUBLE SUM/AVG within 1e-9
relative, north_star).  Imported by the test modules; no tests here."""
import numpy as np
import pytest

from flink_amd import abi

REL_TOL = 1e-9


def _torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _rows(res, cfg, double_cols):
    n_aggs = cfg.n_aggs
    rows = []
    for i in range(len(res["key"])):
        rows.append((int(res["key"][i]), int(res["window_start"][i]), int(res["window_end"][i]),
                     tuple(int(res["values"][a][i]) for a in range(n_aggs)), int(res["null_mask"][i])))
    rows.sort()
    return rows


def _compare(got, want, double_cols, ctx):
    assert len(got) == len(want), f"{ctx}: {len(got)} rows vs oracle {len(want)}"
    for g, w in zip(got, want):
        assert g[:3] == w[:3], f"{ctx}: key/window {g[:3]} != {w[:3]}"
        assert g[4] == w[4], f"{ctx}: null mask {g} != {w}"
        for a, (x, y) in enumerate(zip(g[3], w[3])):
            if a in double_cols and not (g[4] >> a & 1):
                xd = float(np.int64(x).view(np.float64))
                yd = float(np.int64(y).view(np.float64))
                if np.isnan(xd) and np.isnan(yd):
                    continue
                assert xd == pytest.approx(yd, rel=REL_TOL, abs=0.0), f"{ctx}: agg {a} {xd} vs {yd}"
            else:
                assert x == y, f"{ctx}: agg {a} {x} != {y} (row {g} vs {w})"


def _stream(seed, n, n_keys, ooo, step_ms, n_wm, dup_wm=False):
    """Events spread over time with out-of-orderness `ooo`; watermarks lag less than `ooo`, so
    a share of the records is late (some dropped, some merged into unfired windows)."""
    rng = np.random.default_rng(seed)
    per = n // n_wm
    batches = []
    t0 = 1_600_000_000_000
    for b in range(n_wm):
        base = t0 + b * step_ms
        ts = base + rng.integers(0, step_ms, per) - rng.integers(0, ooo, per)
        keys = rng.integers(0, n_keys, per).astype(np.int64) * 7919 - 50000
        iv = rng.integers(-1000, 1000, per).astype(np.int64)
        dv = rng.random(per) * 1000.0
        wm = base + step_ms - ooo // 3
        batches.append((keys, ts.astype(np.int64), iv, dv, wm))
        if dup_wm and b % 3 == 0:
            batches.append((keys[:0], ts[:0], iv[:0], dv[:0], wm - 5))  # non-advancing watermark
    return batches


def _run_both(cfg, batches, double_cols, split=1, snapshot_at=None, nulls=None, stats=None, collect="compact"):
    """nulls: per batch {column: flags} (or None); stats: a dict that receives the handle's final fw_stats;
    collect: "compact" (fw_results) or "segments" (fw_results_device_segments, read back per segment)."""
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    o = OracleOperator(cfg)
    g = WindowAggHandle(cfg)
    for bi, (k, t, iv, dv, wm) in enumerate(batches):
        vals = [iv, dv.view(np.int64)]
        nb = nulls[bi] if nulls is not None else None
        o.process_batch(k, t, vals, nb)
        for part in np.array_split(np.arange(len(k)), split):
            g.push_host(k[part], t[part], [v[part] for v in vals],
                        nulls=None if nb is None else {c: f[part] for c, f in nb.items()})
        o.process_watermark(wm)
        g.advance(wm)
        want = _rows(o.results(clear=True), cfg, double_cols)
        got = _rows(g.results(reset=True) if collect == "compact" else g.segments_to_host(g.result_segments()), cfg,
                    double_cols)
        _compare(got, want, double_cols, f"batch {bi} wm {wm}")
        if snapshot_at is not None and bi == snapshot_at:
            o.snapshot_restore()
            blob = g.snapshot()
            g.close()
            g = WindowAggHandle(cfg)
            g.restore(blob)
        if cfg.late_side_output:  # late side output: the same elements, as a multiset
            # (values: the columns the operator reads; the shim forwards the element by push/row)
            sg, so = g.late_records(), o.side_output()
            used = sorted({cfg.aggs[a].input_col for a in range(cfg.n_aggs) if cfg.aggs[a].kind != abi.AGG_COUNT_STAR})
            side_rows = lambda d: sorted(zip(d["key"].tolist(), d["ts"].tolist(), *[d["values"][c].tolist() for c in used]))
            assert side_rows(sg) == side_rows(so), f"batch {bi}: late side output differs"
            assert sorted(zip(sg["push_seq"].tolist(), sg["row"].tolist())) == \
                sorted(zip(so["push_seq"].tolist(), so["row"].tolist())) or split > 1
    assert g.stats()["num_late_records_dropped"] == o.late_dropped
    assert g.stats()["error_flags"] == 0
    if stats is not None:
        stats.update(g.stats())
    return o.late_dropped


I64, F64, I32 = abi.T_I64, abi.T_F64, abi.T_I32
VT = [I64, F64]
CASES = {
    "sql_tumble_int_aggs": dict(window_kind=abi.WIN_TUMBLE, size_ms=10000,
                                aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MIN, 0, I64), (abi.AGG_MAX, 0, I64)]),
    "sql_tumble_offset": dict(window_kind=abi.WIN_TUMBLE, size_ms=7000, offset_ms=-2500,
                              aggs=[(abi.AGG_MAX, 0, I64), (abi.AGG_COUNT_STAR, 0, I64)]),
    "sql_tumble_double": dict(window_kind=abi.WIN_TUMBLE, size_ms=5000,
                              aggs=[(abi.AGG_SUM, 1, F64), (abi.AGG_AVG, 1, F64), (abi.AGG_MIN, 1, F64), (abi.AGG_MAX, 1, F64)]),
    "sql_hop": dict(window_kind=abi.WIN_HOP, size_ms=10000, slide_ms=2000, count_star_index=0,
                    aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MAX, 1, F64)]),
    "sql_hop_offset": dict(window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=3000, offset_ms=1000, count_star_index=1,
                           aggs=[(abi.AGG_SUM, 0, I64), (abi.AGG_COUNT_STAR, 0, I64)]),
    "sql_cumulate_countstar": dict(window_kind=abi.WIN_CUMULATE, size_ms=12000, slide_ms=2000, count_star_index=0,
                                   aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MIN, 0, I64), (abi.AGG_MAX, 0, I64)]),
    "sql_cumulate_nocount": dict(window_kind=abi.WIN_CUMULATE, size_ms=9000, slide_ms=3000,
                                 aggs=[(abi.AGG_SUM, 0, I64), (abi.AGG_AVG, 0, I64)]),
    "ds_tumble_sum": dict(api=abi.API_DATASTREAM, window_kind=abi.WIN_TUMBLE, size_ms=4000,
                          aggs=[(abi.AGG_SUM, 0, I64)]),
    "ds_sliding_max": dict(api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=2000,
                           aggs=[(abi.AGG_MAX, 0, I64)]),
    "ds_sliding_min_double": dict(api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP, size_ms=4000, slide_ms=1000,
                                  aggs=[(abi.AGG_MIN, 1, F64)]),
    # DataStream allowedLateness (WindowOperator.java:609-682): fired windows keep their state until
    # maxTimestamp + lateness and fire again per late element (EventTimeTrigger.onElement)
    "ds_tumble_lateness": dict(api=abi.API_DATASTREAM, window_kind=abi.WIN_TUMBLE, size_ms=4000, allowed_lateness_ms=3000,
                               aggs=[(abi.AGG_SUM, 0, I64)]),
    "ds_tumble_lateness_double_sum": dict(api=abi.API_DATASTREAM, window_kind=abi.WIN_TUMBLE, size_ms=3000,
                                          allowed_lateness_ms=1500, aggs=[(abi.AGG_SUM, 1, F64)]),
    "ds_sliding_lateness_side_output": dict(api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=2000,
                                            allowed_lateness_ms=2500, late_side_output=True, aggs=[(abi.AGG_MAX, 0, I64)]),
    "ds_sliding_side_output": dict(api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP, size_ms=4000, slide_ms=1000,
                                   late_side_output=True, aggs=[(abi.AGG_MIN, 1, F64)]),
    # slide not dividing size (SlidingEventTimeWindows.java:77-90): 1 s panes, each in 2 or 3 windows
    "ds_sliding_nondiv_sum": dict(api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP, size_ms=5000, slide_ms=2000,
                                  aggs=[(abi.AGG_SUM, 0, I64)]),
    "ds_sliding_nondiv_lateness_side_output": dict(api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP, size_ms=7000,
                                                   slide_ms=3000, offset_ms=1000, allowed_lateness_ms=2500,
                                                   late_side_output=True, aggs=[(abi.AGG_MAX, 1, F64)]),
}


def _cfg(kw, **extra):
    kw = dict(kw)
    kw.update(extra)
    kw.setdefault("value_col_types", VT)
    kw.setdefault("key_hash", abi.KEYHASH_LONG)
    kw.setdefault("state_capacity", 1 << 16)
    kw.setdefault("max_batch_rows", 1 << 16)
    kw.setdefault("output_capacity", 1 << 18)
    return abi.make_config(**kw)


def _double_cols(kw):
    """DOUBLE SUM / AVG results (1e-9 relative); every other column compares bit-exactly."""
    return {a for a, (k, c, t) in enumerate(kw["aggs"]) if t == F64 and k in (abi.AGG_SUM, abi.AGG_AVG)}


