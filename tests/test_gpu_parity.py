"""GPU parity: the HIP operator (libflinkwin) against the CPU oracle and the reference's golden
fixtures.  Integer aggregates, DOUBLE MIN/MAX (bit patterns, including NaN payloads and the sign
of zero) and window boundaries must be bit-exact; DOUBLE SUM/AVG within 1e-9 relative
(north_star; the device adds in a different order).  Run on an MI355X via gpurun."""
import zlib

import numpy as np
import pytest

from fixture_runner import GpuAdapter, load_fixtures, replay
from flink_amd import abi
from parity_common import (CASES, F64, I32, I64, REL_TOL, VT, _cfg, _compare, _double_cols, _rows,  # noqa: F401
                           _run_both, _stream, _torch_cuda)

pytestmark = pytest.mark.gpu

FIXTURES = load_fixtures()


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    _torch_cuda()


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_gpu_reproduces_reference_golden(fx):
    replay(fx, GpuAdapter(fx))


# ------------------------------------------------------------------------------------------
# randomized streams with late records, compared watermark by watermark against the oracle
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", sorted(CASES))
def test_random_stream_matches_oracle(name):
    kw = CASES[name]
    late = _run_both(_cfg(kw), _stream(zlib.crc32(name.encode()) % 1000, 60000, 700, ooo=2 * kw["size_ms"] + 1500,
                                       step_ms=1500, n_wm=30), _double_cols(kw))
    assert late > 0 or kw.get("late_side_output")  # the stream exercises the late-record paths


# Every accumulator layout with its own k_merge_fire variant (fw_merge_impl.h MergeLayouts: the
# word ops as compile-time constants), under each SQL window kind, against the oracle.  HOP needs
# a COUNT(*), so it runs the layouts that have one.
LAYOUT_AGGS = {
    "cnt": [(abi.AGG_COUNT_STAR, 0, I64)],
    "max": [(abi.AGG_MAX, 0, I64)],
    "min": [(abi.AGG_MIN, 0, I64)],
    "sum_f": [(abi.AGG_SUM, 1, F64)],
    "avg_f": [(abi.AGG_AVG, 1, F64)],
    "sum_avg_i": [(abi.AGG_SUM, 0, I64), (abi.AGG_AVG, 0, I64)],
    "cnt_max": [(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_MAX, 0, I64)],
    "cnt_min": [(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_MIN, 0, I64)],
    "cnt_sum_min_max": [(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MIN, 0, I64),
                        (abi.AGG_MAX, 0, I64)],
}
LAYOUT_WINDOWS = {
    "tumble": dict(window_kind=abi.WIN_TUMBLE, size_ms=6000),
    "hop": dict(window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=2000),
    "cumulate": dict(window_kind=abi.WIN_CUMULATE, size_ms=8000, slide_ms=2000),
}
LAYOUT_CASES = [(w, a) for w in LAYOUT_WINDOWS for a in LAYOUT_AGGS
                if w != "hop" or LAYOUT_AGGS[a][0][0] == abi.AGG_COUNT_STAR]


# The rows where the merge wrote them (fw_results_device_segments: per-superbucket slabs and the
# shared overflow region, no compaction) are the oracle's rows -- with an output capacity small
# enough that the slabs overflow into the shared region.
@pytest.mark.parametrize("name,out_cap,n,n_keys", [
    ("sql_tumble_int_aggs", 1 << 20, 30000, 2000), ("sql_hop", 1 << 20, 30000, 2000),
    ("sql_cumulate_countstar", 1 << 20, 30000, 2000), ("ds_sliding_max", 1 << 20, 30000, 2000),
    # ~11 700 rows per firing over 128 superbuckets of 64-row slabs: ~3 500 rows in the overflow region
    ("sql_tumble_int_aggs", 1 << 12, 140000, 12000)])
def test_result_segments_match_oracle(name, out_cap, n, n_keys):
    kw = CASES[name]
    _run_both(_cfg(kw, output_capacity=out_cap), _stream(zlib.crc32(name.encode()) % 997, n, n_keys,
                                                         ooo=2 * kw["size_ms"] + 1500, step_ms=1500, n_wm=14),
              _double_cols(kw), collect="segments")


# layout: the planner's choice, or the partial-row layout forced either way (FW_RUNS: superbucket
# runs vs chunk-local cells, fw_api.hip; runs are planned only for TUMBLE with >= 2 words)
@pytest.mark.parametrize("layout", ["planned", "runs", "cells"])
@pytest.mark.parametrize("win,aggs", LAYOUT_CASES, ids=[f"{w}-{a}" for w, a in LAYOUT_CASES])
def test_compiled_accumulator_layouts_match_oracle(win, aggs, layout, monkeypatch):
    if layout != "planned":
        monkeypatch.setenv("FW_RUNS", "1" if layout == "runs" else "0")
    kw = dict(LAYOUT_WINDOWS[win], aggs=LAYOUT_AGGS[aggs])
    if kw["aggs"][0][0] == abi.AGG_COUNT_STAR:
        kw["count_star_index"] = 0
    _run_both(_cfg(kw), _stream(zlib.crc32(f"{win}{aggs}".encode()) % 1000, 20000, 300, ooo=2 * kw["size_ms"],
                                step_ms=4500, n_wm=20), _double_cols(kw))  # 2-3 slides per watermark: HOP chains


# TIMESTAMP_LTZ windows across daylight-saving changes: slices on the zone's wall clock, timers at
# toEpochMillsForTimer (gap -> first skipped hour, overlap -> the later instant), next trigger
# watermarks through the zone (TimeWindowUtil.java:52-211); bit-exact against the oracle.
LTZ_CASES = {
    "tumble_1h": dict(window_kind=abi.WIN_TUMBLE, size_ms=3600000,
                      aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MAX, 0, I64)]),
    "hop_2h_30min": dict(window_kind=abi.WIN_HOP, size_ms=7200000, slide_ms=1800000, count_star_index=0,
                         aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64)]),
    "cumulate_4h_1h": dict(window_kind=abi.WIN_CUMULATE, size_ms=4 * 3600000, slide_ms=3600000, count_star_index=0,
                           aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_MIN, 0, I64), (abi.AGG_MAX, 0, I64)]),
}


def _ltz_stream(seed, t_mid, n_wm=80, per=1500, n_keys=200, step_ms=600000, ooo=3 * 3600000):
    rng = np.random.default_rng(seed)
    t0 = t_mid - n_wm // 2 * step_ms
    out = []
    for b in range(n_wm):
        base = t0 + b * step_ms
        ts = base + rng.integers(0, step_ms, per) - rng.integers(0, ooo, per)
        keys = rng.integers(0, n_keys, per).astype(np.int64) * 31 + 7
        iv = rng.integers(-1000, 1000, per).astype(np.int64)
        out.append((keys, ts.astype(np.int64), iv, rng.random(per) * 100.0, base + step_ms - ooo // 4))
    return out


@pytest.mark.parametrize("zone,t_mid", [("America/Los_Angeles", 1615716000000), ("America/Los_Angeles", 1636275600000),
                                        ("Asia/Shanghai", 1600000000000), ("Australia/Lord_Howe", 1617460200000)])
@pytest.mark.parametrize("case", sorted(LTZ_CASES))
def test_ltz_windows_across_dst_match_oracle(case, zone, t_mid):
    kw = dict(LTZ_CASES[case], shift_zone=zone)
    _run_both(_cfg(kw), _ltz_stream(zlib.crc32((case + zone).encode()) % 1000, t_mid), set(), snapshot_at=37)


@pytest.mark.parametrize("name", ["sql_hop", "sql_cumulate_countstar", "ds_sliding_max", "ds_tumble_lateness",
                                  "ds_sliding_lateness_side_output"])
def test_split_pushes_snapshot_and_stale_watermarks(name):
    kw = CASES[name]
    _run_both(_cfg(kw), _stream(5, 40000, 300, ooo=2500, step_ms=1000, n_wm=24, dup_wm=True),
              _double_cols(kw), split=3, snapshot_at=11)


# ------------------------------------------------------------------------------------------
# SQL NULLs and DOUBLE MIN/MAX edge values (NaN first / later, NaN payloads, -0.0 vs +0.0) in
# arbitrary arrival orders: MaxAggFunction / MinAggFunction keep the first value and replace it
# only on a strict > / <, Sum/Count/AvgAggFunction skip NULLs.  Bit-exact against the oracle.
# ------------------------------------------------------------------------------------------
_SPECIAL = np.array([0x7FF8000000000000, 0xFFF8000000000001, 0x7FF0000000000001, 0x8000000000000000, 0,
                     np.float64(1.0).view(np.int64), np.float64(-1.0).view(np.int64),
                     np.float64(2.0).view(np.int64), np.float64(-2.5).view(np.int64)], dtype=np.uint64).view(np.int64)


def _special_stream(seed, n_wm=24, per=3000, n_keys=300, step_ms=1000, ooo=2500):
    rng = np.random.default_rng(seed)
    batches, nulls = [], []
    for b, (k, t, iv, dv, wm) in enumerate(_stream(seed, n_wm * per, n_keys, ooo=ooo, step_ms=step_ms, n_wm=n_wm)):
        pick = rng.random(len(k))
        bits = dv.view(np.int64).copy()
        sp = pick < 0.35  # a third of the values are NaN / zero / small ties
        bits[sp] = _SPECIAL[rng.integers(0, len(_SPECIAL), int(sp.sum()))]
        batches.append((k, t, iv, bits.view(np.float64), wm))
        nulls.append({0: (rng.random(len(k)) < 0.15).astype(np.uint8), 1: (rng.random(len(k)) < 0.2).astype(np.uint8)})
    return batches, nulls


NULL_CASES = {
    # (8 accumulator words each: a DOUBLE MIN/MAX group takes 4 + 1 per aggregate)
    "tumble": dict(window_kind=abi.WIN_TUMBLE, size_ms=4000,
                   aggs=[(abi.AGG_MAX, 1, F64), (abi.AGG_MIN, 1, F64), (abi.AGG_SUM, 1, F64), (abi.AGG_AVG, 1, F64),
                         (abi.AGG_COUNT, 1, F64), (abi.AGG_COUNT_STAR, 0, I64)]),
    "hop": dict(window_kind=abi.WIN_HOP, size_ms=5000, slide_ms=1000, count_star_index=2,
                aggs=[(abi.AGG_MAX, 1, F64), (abi.AGG_AVG, 0, I64), (abi.AGG_COUNT_STAR, 0, I64),
                      (abi.AGG_MIN, 1, F64)]),
    "cumulate": dict(window_kind=abi.WIN_CUMULATE, size_ms=6000, slide_ms=2000,
                     aggs=[(abi.AGG_MIN, 1, F64), (abi.AGG_SUM, 0, I64), (abi.AGG_COUNT, 0, I64),
                           (abi.AGG_MAX, 1, F64), (abi.AGG_MAX, 0, I64)]),
}


@pytest.mark.parametrize("name", sorted(NULL_CASES))
def test_nulls_nan_and_signed_zero_match_oracle(name):
    kw = NULL_CASES[name]
    batches, nulls = _special_stream(zlib.crc32(name.encode()) % 1000)
    _run_both(_cfg(kw, nullable_cols=[0, 1]), batches, _double_cols(kw), split=2, nulls=nulls)


def test_double_min_max_not_null_edge_values_match_oracle():
    # NOT NULL DOUBLE column (no gate words) with the same edge values, snapshot/restore mid-run
    kw = dict(window_kind=abi.WIN_HOP, size_ms=4000, slide_ms=2000, count_star_index=0,
              aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_MAX, 1, F64), (abi.AGG_MIN, 1, F64)])
    batches, _ = _special_stream(77)
    _run_both(_cfg(kw), batches, set(), snapshot_at=9)


def test_hot_keys_fold_in_lds_cache():
    # Zipf-skewed keys: most records of a chunk fold into a handful of cache slots
    rng = np.random.default_rng(3)
    kw = CASES["sql_cumulate_countstar"]
    batches = []
    for b in range(10):
        n = 50000
        keys = np.minimum(rng.zipf(1.3, n), 5000).astype(np.int64)
        ts = 1_600_000_000_000 + b * 2000 + rng.integers(0, 2000, n)
        batches.append((keys, ts.astype(np.int64), rng.integers(0, 100, n), rng.random(n), 1_600_000_000_000 + b * 2000 + 1000))
    _run_both(_cfg(kw), batches, set())


# The ingest fold keeps one slot table per chunk (round 6): rows of a later sub-tile fold into
# owners an earlier sub-tile published, and the 1024-thread variants (3-8 words) have 2048 / 1024
# slots.  Zipf keys put the same hot (key, slice) groups in every sub-tile of every chunk; the
# layouts cover the 512-thread and both 1024-thread variants, NULL gates and the DOUBLE MIN/MAX word
# groups whose fold keeps arrival order (ordinals).
FOLD_LAYOUTS = {
    "cfg5_4words": dict(window_kind=abi.WIN_CUMULATE, size_ms=8000, slide_ms=2000, count_star_index=0,
                        aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MIN, 0, I64),
                              (abi.AGG_MAX, 0, I64)]),
    "tumble_2words": dict(window_kind=abi.WIN_TUMBLE, size_ms=4000,
                          aggs=[(abi.AGG_SUM, 0, I64), (abi.AGG_MAX, 0, I64)]),
    "null_double_minmax": NULL_CASES["tumble"],
    "hop_null_double": NULL_CASES["hop"],
}


@pytest.mark.parametrize("name", sorted(FOLD_LAYOUTS))
def test_chunk_fold_across_sub_tiles_matches_oracle(name):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    kw = FOLD_LAYOUTS[name]
    batches, nulls = [], []
    for b in range(8):
        n = 40000 + 977 * b  # ragged: a partial last chunk
        keys = np.minimum(rng.zipf(1.2, n), 20000).astype(np.int64)
        ts = 1_600_000_000_000 + b * 1500 + rng.integers(0, 1500, n)
        dv = rng.integers(-3, 4, n).astype(np.float64)  # many ties, signed zeros
        dv[rng.random(n) < 0.05] = -0.0
        batches.append((keys, ts.astype(np.int64), rng.integers(-50, 50, n), dv, 1_600_000_000_000 + b * 1500 + 700))
        nulls.append({0: (rng.random(n) < 0.1).astype(np.uint8), 1: (rng.random(n) < 0.1).astype(np.uint8)})
    has_nulls = name.startswith(("null", "hop_null"))
    _run_both(_cfg(kw, nullable_cols=[0, 1]) if has_nulls else _cfg(kw), batches, _double_cols(kw),
              nulls=nulls if has_nulls else None)


def test_int_sum_wraps_like_java():
    cfg = _cfg(dict(window_kind=abi.WIN_TUMBLE, size_ms=1000, aggs=[(abi.AGG_SUM, 0, I32), (abi.AGG_SUM, 1, I64)]),
               value_col_types=[I32, I64])
    k = np.zeros(8, np.int64)
    t = np.arange(8, dtype=np.int64)
    big = np.full(8, 2**31 - 7, np.int64)
    huge = np.full(8, 2**62, np.int64)
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    g, o = WindowAggHandle(cfg), OracleOperator(cfg)
    g.push_host(k, t, [big, huge])
    o.process_batch(k, t, [big, huge])
    g.advance(5000)
    o.process_watermark(5000)
    rg, ro = g.results(), o.results()
    w32 = (8 * (2**31 - 7)) & 0xFFFFFFFF
    w32 = w32 - 2**32 if w32 >= 2**31 else w32
    assert list(rg["values"][0]) == list(ro["values"][0]) == [w32]
    assert list(rg["values"][1]) == list(ro["values"][1]) == [0]  # 8 * 2^62 wraps to 0


def test_device_generator_matches_host_generator():
    torch = _torch_cuda()
    from flink_amd import _native
    from oracle import oracle as O
    import ctypes as C
    cdf = O.zipf_cdf(1000, 1.1)
    dcdf = torch.tensor(cdf, device="cuda")
    for dist, vk in ((0, 0), (0, 1), (1, 2)):
        gp = abi.fw_gen_params(seed=42, t0_ms=1599998400000, rate_per_s=1000000, ooo_ms=4000, key_base=1000,
                               key_count=1000 if dist else 1000000, key_dist=dist, value_kind=vk,
                               zipf_cdf=dcdf.data_ptr() if dist else None)
        n, i0 = 100000, 123456789
        k = torch.empty(n, dtype=torch.int64, device="cuda")
        t = torch.empty_like(k)
        v = torch.empty_like(k)
        s = torch.cuda.current_stream().cuda_stream
        _native.check(_native.lib().fw_generate(C.byref(gp), i0, n, k.data_ptr(), t.data_ptr(), v.data_ptr(), s))
        hk, ht, hv = O.generate(gp, i0, n, cdf if dist else None)
        assert np.array_equal(k.cpu().numpy(), hk)
        assert np.array_equal(t.cpu().numpy(), ht)
        assert np.array_equal(v.cpu().numpy(), hv)


def test_device_key_groups_match_oracle():
    torch = _torch_cuda()
    from flink_amd.runtime.keygroups import assign_key_groups_device
    from oracle import oracle as O
    rng = np.random.default_rng(11)
    keys = rng.integers(-(1 << 63), (1 << 63) - 1, 5000, dtype=np.int64)
    for kind in (abi.KEYHASH_LONG, abi.KEYHASH_BINROW_BIGINT):
        kg, dest = assign_key_groups_device(torch.tensor(keys, device="cuda"), 128, 8, kind)
        want = np.array([O.key_group(kind, int(x), 128) for x in keys])
        assert np.array_equal(kg.cpu().numpy(), want)
        assert np.array_equal(dest.cpu().numpy(), want * 8 // 128)


# ------------------------------------------------------------------------------------------
# key-group sharding: p subtasks on one device behind the device partitioner
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("p", [2, 4])
def test_sharded_subtasks_match_unsharded_oracle(p):
    """The N > 1 data path minus the collective: fw_partition_by_dest routes every batch to p
    subtask handles (parallelism p, subtask i owns computeKeyGroupRangeForOperatorIndex(128, p, i));
    the union of their window results equals one unsharded oracle operator, and no handle sees a
    foreign key group (ERR_KEYGROUP would be raised)."""
    torch = _torch_cuda()
    from flink_amd.runtime.exchange import KeyByExchange
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    kw = dict(window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=2000, count_star_index=0,
              aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MIN, 1, F64)])
    cfgs = [_cfg(kw, key_hash=abi.KEYHASH_BINROW_BIGINT, parallelism=p, subtask_index=i) for i in range(p)]
    o = OracleOperator(_cfg(kw, key_hash=abi.KEYHASH_BINROW_BIGINT))
    hs = [WindowAggHandle(c) for c in cfgs]
    ex = KeyByExchange(abi.KEYHASH_BINROW_BIGINT, 128)
    ex.world = p  # route for p subtasks; the all-to-all is replaced by slicing on one device
    for bi, (k, t, iv, dv, wm) in enumerate(_stream(21, 60000, 2000, ooo=3000, step_ms=1500, n_wm=20)):
        vals = [iv, dv.view(np.int64)]
        o.process_batch(k, t, vals)
        dk, dt = torch.tensor(k, device="cuda"), torch.tensor(t, device="cuda")
        dvs = [torch.tensor(v, device="cuda") for v in vals]
        pk, pt, pv, counts = ex.partition(dk, dt, dvs)
        off = 0
        for i, c in enumerate(counts.tolist()):
            if c:
                hs[i].push_device(pk[off:off + c], pt[off:off + c], [v[off:off + c] for v in pv])
            off += c
        o.process_watermark(wm)
        got = []
        for h in hs:
            h.advance(wm)
            got += _rows(h.results(reset=True), cfgs[0], {2})
        _compare(sorted(got), _rows(o.results(clear=True), cfgs[0], {2}), {2}, f"p={p} batch {bi}")
    assert sum(h.stats()["num_late_records_dropped"] for h in hs) == o.late_dropped
    assert all(h.stats()["error_flags"] == 0 for h in hs)
    for h in hs:
        h.close()


@pytest.mark.parametrize("p_from,p_to,case", [(2, 3, "sql_hop"), (4, 1, "sql_cumulate_countstar"),
                                               (1, 2, "ds_sliding_max"), (3, 2, "sql_tumble_int_aggs"),
                                               (2, 3, "ds_tumble_sum")])
def test_rescale_restore_by_key_group(p_from, p_to, case):
    """Checkpoint at parallelism p_from, restore at p_to: every subtask writes one blob per owned
    key group (fw_snapshot_key_group, the heap backend's writeStateInKeyGroup unit), the new
    subtasks restore the key groups of their computeKeyGroupRangeForOperatorIndex range (SQL: plus
    the min of the union-list watermarks; DataStream: the watermark restarts at Long.MIN_VALUE),
    and the run continues.  The union of all window results equals one unsharded oracle that
    checkpoints and restarts at the same cut.

    DataStream state is per window (KIND_DSWIN), so records that arrive between the
    restore and the first watermark into windows that fired before the checkpoint are exact for
    the sliding case too (round 1's shared-slice restore deviation is gone)."""
    torch = _torch_cuda()
    from flink_amd.runtime.exchange import KeyByExchange
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    kw = CASES[case]
    dcols = _double_cols(kw)
    kh = abi.KEYHASH_LONG if kw.get("api") == abi.API_DATASTREAM else abi.KEYHASH_BINROW_BIGINT
    o = OracleOperator(_cfg(kw, key_hash=kh))

    def handles(p):
        cfgs = [_cfg(kw, key_hash=kh, parallelism=p, subtask_index=i) for i in range(p)]
        return cfgs, [WindowAggHandle(c) for c in cfgs]

    cfgs, hs = handles(p_from)
    ex = KeyByExchange(kh, 128)
    cut = 9
    for bi, (k, t, iv, dv, wm) in enumerate(_stream(33, 48000, 1500, ooo=2500, step_ms=1200, n_wm=20)):
        if bi == cut:  # checkpoint (flush + per-key-group state), then restart at p_to
            blobs, wms = {}, []
            for h in hs:
                b, w = h.snapshot_key_groups()
                blobs.update(b)
                wms.append(w)
                h.close()
            assert sorted(blobs) == list(range(128))
            cfgs, hs = handles(p_to)
            for h in hs:
                h.restore_key_groups(blobs, wms)
            o.snapshot_restore()
        vals = [iv, dv.view(np.int64)]
        o.process_batch(k, t, vals)
        ex.world = len(hs)  # route for the current parallelism (slicing replaces the all-to-all)
        dk, dt = torch.tensor(k, device="cuda"), torch.tensor(t, device="cuda")
        pk, pt, pv, counts = ex.partition(dk, dt, [torch.tensor(v, device="cuda") for v in vals])
        off = 0
        for i, c in enumerate(counts.tolist()):
            if c:
                hs[i].push_device(pk[off:off + c], pt[off:off + c], [v[off:off + c] for v in pv])
            off += c
        o.process_watermark(wm)
        got = []
        for h in hs:
            h.advance(wm)
            got += _rows(h.results(reset=True), cfgs[0], dcols)
        _compare(sorted(got), _rows(o.results(clear=True), cfgs[0], dcols), dcols,
                 f"{case} p={p_from}->{p_to} batch {bi}")
    assert all(h.stats()["error_flags"] == 0 for h in hs)
    for h in hs:
        h.close()


def test_key_group_restore_rejects_foreign_and_mismatched_blobs():
    _torch_cuda()
    from flink_amd._native import FlinkWinError
    from flink_amd.runtime.handle import WindowAggHandle
    kw = CASES["sql_hop"]
    a = WindowAggHandle(_cfg(kw, key_hash=abi.KEYHASH_BINROW_BIGINT, parallelism=2, subtask_index=0))
    from flink_amd._native import lib
    keys = np.array([k for k in range(1000) if lib().fw_host_key_group(abi.KEYHASH_BINROW_BIGINT, k, 0, 128) < 64],
                    dtype=np.int64)  # subtask 0 of 2 owns key groups 0..63
    n = len(keys)
    a.push_host(keys, np.full(n, 1_600_000_000_000, np.int64), [np.ones(n, np.int64), np.ones(n, np.int64)])
    blobs, _ = a.snapshot_key_groups()
    assert sorted(blobs) == list(range(64))
    b = WindowAggHandle(_cfg(kw, key_hash=abi.KEYHASH_BINROW_BIGINT, parallelism=2, subtask_index=1))
    with pytest.raises(FlinkWinError):  # key group 0 belongs to subtask 0
        b.restore_key_group_blob(blobs[0])
    c = WindowAggHandle(_cfg(CASES["sql_tumble_int_aggs"], key_hash=abi.KEYHASH_BINROW_BIGINT))
    with pytest.raises(FlinkWinError):  # different window / accumulator layout
        c.restore_key_group_blob(blobs[0])
    for h in (a, b, c):
        h.close()


# ------------------------------------------------------------------------------------------
# BASELINE-sized streams: the bench workloads at full batch size (2^22 events per watermark),
# checked on a key subset against the oracle (window results of a key depend only on that
# key's records, so the oracle replays only the subset) plus size-independent properties
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("wl_name", ["cfg2", "cfg3", "cfg4", "cfg5", "cfg4_10m", "cfg4_10m-h2", "cfg2-runs", "cfg3-runs",
                                     "cfg5-runs", "cfg4-cells"])
def test_bench_workload_full_size_key_subset(wl_name, monkeypatch):
    variant = None
    if "-" in wl_name:
        wl_name, variant = wl_name.split("-")
    if variant in ("runs", "cells"):  # the partial-row layout the planner would not pick, forced (FW_RUNS)
        monkeypatch.setenv("FW_RUNS", "1" if variant == "runs" else "0")
    torch = _torch_cuda()
    import ctypes as C
    import bench
    from flink_amd import _native
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    wl = dict(bench.WORKLOADS[wl_name])
    if variant == "h2":  # capacity hint 2: 16384 superbuckets, the ingest histogram's limit
        wl["state_per_key"] = 2
    # CFG5: 27 steps = 4077 s of event time at 27 778 ev/s, past the 1 h CUMULATE window's last step
    # (its final slice fires and the window's first-slice state is cleared, SliceAssigners.java:398-453)
    steps, B, MOD, PICK = (27 if wl_name == "cfg5" else 6), bench.B, 97, 13
    L = _native.lib()
    zipf_t = None
    if wl["dist"] == 1:
        w = 1.0 / np.power(np.arange(1, wl["keys"] + 1, dtype=np.float64), wl["zipf_s"])
        cdf = np.cumsum(w)
        zipf_t = torch.tensor(cdf / cdf[-1], device="cuda")
    gp, keys_total = bench.gen_params(wl, 1, zipf_t.data_ptr() if zipf_t is not None else None)
    cfg = bench.build_config(wl, 1, 0, keys_total, (8 if keys_total <= 2_000_000 else 2) * keys_total + (1 << 20))
    g, o = WindowAggHandle(cfg), OracleOperator(cfg)
    if wl_name == "cfg4_10m":  # bench hint 1.25: 8192 superbuckets; hint 2: 16384 (one merge pass each)
        assert g.stats()["num_superbuckets"] == (16384 if variant == "h2" else 8192)
    k = torch.empty(B, dtype=torch.int64, device="cuda")
    t, v = torch.empty_like(k), torch.empty_like(k)
    s = torch.cuda.current_stream().cuda_stream
    got, want, n_sub = [], [], 0
    total_rows = 0
    count_sum = 0
    cs = wl["count_star"]
    live, wms, ends = [], [], set()
    for b in range(steps + 1):
        wm = bench.watermark(b, wl["rate"])
        if b == steps:  # last: fire every window (CUMULATE: a few more steps; its 1 h windows
            wm = bench.T0 + 10**9 if wl["window"][0] != "CUMULATE" else wm + 120_000  # emit every step)
        if b < steps:
            _native.check(L.fw_generate(C.byref(gp), b * B, B, k.data_ptr(), t.data_ptr(), v.data_ptr(), s))
            g.push_device(k, t, [v] if cfg.n_value_cols else [])
            m = (k % MOD) == PICK
            hk, ht, hv = k[m].cpu().numpy(), t[m].cpu().numpy(), v[m].cpu().numpy()
            n_sub += len(hk)
            o.process_batch(hk, ht, [hv] if cfg.n_value_cols else [])
        g.advance(wm)
        o.process_watermark(wm)
        r = g.results(reset=True)
        live.append(g.stats()["live_state_entries"])
        wms.append(wm)
        ends.update(np.unique(r["window_end"]).tolist())
        total_rows += len(r["key"])
        if cs >= 0:
            count_sum += int(r["values"][cs].sum())
        sel = (r["key"] % MOD) == PICK
        sub = {"key": r["key"][sel], "window_start": r["window_start"][sel], "window_end": r["window_end"][sel],
               "values": [x[sel] for x in r["values"]], "null_mask": r["null_mask"][sel]}
        dcols = {a for a, (kk, c, ty) in enumerate(wl["aggs"]) if ty == "DOUBLE"}
        got_b, want_b = _rows(sub, cfg, dcols), _rows(o.results(clear=True), cfg, dcols)
        _compare(got_b, want_b, dcols, f"{wl_name} step {b}")
        got += got_b
    st = g.stats()
    assert st["error_flags"] == 0 and st["num_late_records_dropped"] == 0 == o.late_dropped
    # the superbucket peak (fw_stats v9): some table held entries, none beyond its capacity
    assert 0 < st["peak_superbucket_entries"] <= st["superbucket_capacity"]
    assert n_sub > 1000 and len(got) > 100 and total_rows > len(got)
    kind = wl["window"][0]
    if kind == "HOP" and cs >= 0:       # every event is counted in size/slide windows
        assert count_sum == steps * B * (wl["window"][1] // wl["window"][2])
    if kind == "CUMULATE":
        # the first 1 h window's last step fired (window_end = its start + 1 h) ...
        first_end = bench.T0 - bench.T0 % wl["window"][1] + wl["window"][1]
        assert first_end in ends and wms[-1] >= first_end
        # ... and its state (first slice + current slice per key) was cleared: the live entries after
        # the watermark crossed the hour are far fewer than just before it
        cross = next(i for i, w in enumerate(wms) if w >= first_end - 1)
        assert live[cross] < 0.8 * live[cross - 1], (live[cross - 1], live[cross])
    g.close()


# ------------------------------------------------------------------------------------------
# edge cases of the reference's tests: empty batches and watermarks with nothing to fire,
# a single record, and a batch larger than max_batch_rows (split into pushes)
# ------------------------------------------------------------------------------------------
def test_empty_and_tiny_batches_and_oversized_push():
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    kw = CASES["sql_cumulate_countstar"]
    cfg = _cfg(kw, max_batch_rows=4096)
    g, o = WindowAggHandle(cfg), OracleOperator(cfg)
    rng = np.random.default_rng(9)
    t0 = 1_600_000_000_000
    plan = [0, 1, 0, 10000, 3, 0, 25000]
    for bi, n in enumerate(plan):
        k = rng.integers(0, 50, n).astype(np.int64)
        t = (t0 + bi * 2000 + rng.integers(-1000, 2000, n)).astype(np.int64)
        vals = [rng.integers(-5, 5, n).astype(np.int64), rng.random(n).view(np.int64)]
        g.push_host(k, t, vals)
        o.process_batch(k, t, vals)
        wm = t0 + bi * 2000 - 1
        g.advance(wm)
        o.process_watermark(wm)
        _compare(_rows(g.results(reset=True), cfg, set()), _rows(o.results(clear=True), cfg, set()), set(), f"batch {bi}")
    g.advance(t0 + 10**7)
    o.process_watermark(t0 + 10**7)
    _compare(_rows(g.results(reset=True), cfg, set()), _rows(o.results(clear=True), cfg, set()), set(), "final")
    assert g.stats()["num_late_records_dropped"] == o.late_dropped
    g.close()


@pytest.mark.parametrize("p", [2, 8, 37])
def test_partition_by_dest_is_stable(p):
    """fw_partition_by_dest keeps each destination's rows in input order (a channel's order), so the
    routed batch is the same on every run: equal to a stable sort by destination subtask."""
    torch = _torch_cuda()
    from flink_amd.runtime.exchange import KeyByExchange
    from oracle import oracle as O
    rng = np.random.default_rng(p)
    n = 50_000 + p
    k = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    t = np.arange(n, dtype=np.int64)
    v = rng.integers(0, 1 << 62, n).astype(np.int64)
    ex = KeyByExchange(abi.KEYHASH_BINROW_BIGINT, 128)
    ex.world = p
    pk, pt, pv, counts = ex.partition(torch.tensor(k, device="cuda"), torch.tensor(t, device="cuda"),
                                      [torch.tensor(v, device="cuda")])
    dest = np.array([O.operator_index(128, p, O.key_group(abi.KEYHASH_BINROW_BIGINT, int(x), 128)) for x in k])
    order = np.argsort(dest, kind="stable")
    assert np.array_equal(counts.cpu().numpy(), np.bincount(dest, minlength=p))
    assert np.array_equal(pk.cpu().numpy(), k[order])
    assert np.array_equal(pt.cpu().numpy(), t[order])
    assert np.array_equal(pv[0].cpu().numpy(), v[order])


# ------------------------------------------------------------------------------------------
# two-phase (local / global) aggregation: TwoStageOptimizedWindowAggregateRule's plan
# ------------------------------------------------------------------------------------------
TWO_PHASE_CASES = {
    "tumble": dict(window_kind=abi.WIN_TUMBLE, size_ms=4000, offset_ms=-700,
                   aggs=[(abi.AGG_SUM, 0, I64), (abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_AVG, 1, F64),
                         (abi.AGG_MAX, 0, I64), (abi.AGG_COUNT, 1, F64)]),
    "hop": dict(window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=2000, count_star_index=1,
                aggs=[(abi.AGG_MIN, 0, I64), (abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 1, F64), (abi.AGG_AVG, 0, I64)]),
    "cumulate": dict(window_kind=abi.WIN_CUMULATE, size_ms=8000, slide_ms=2000, count_star_index=0,
                     aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_MAX, 1, F64), (abi.AGG_MIN, 0, I64)]),
}


def _push_partials_to_oracle(og, key, se, fields, nm):
    n = key.numel()
    if n == 0:
        return
    nmh = nm.cpu().numpy()
    og.process_batch(key.cpu().numpy(), se.cpu().numpy(), [f.cpu().numpy() for f in fields],
                     {j: (nmh >> j) & 1 for j in range(len(fields))})


@pytest.mark.parametrize("name", sorted(TWO_PHASE_CASES))
def test_two_phase_local_global_matches_oracle(name):
    """LOCAL on the GPU against LocalAggCombiner's partials (oracle LOCAL, as a multiset per
    watermark), GLOBAL on the GPU against the oracle GLOBAL fed the same partial rows, and the
    end-to-end two-phase results against one one-phase operator (the plans agree)."""
    torch = _torch_cuda()
    from flink_amd.table.two_phase import TwoPhaseWindowAgg
    from oracle.oracle import OracleOperator
    kw = TWO_PHASE_CASES[name]
    cfg = _cfg(kw, nullable_cols=[1])
    tp = TwoPhaseWindowAgg(cfg)
    ol, og, o1 = OracleOperator(tp.local_cfg), OracleOperator(tp.global_cfg), OracleOperator(cfg)
    rng = np.random.default_rng(len(name))
    for bi, (k, t, iv, dv, wm) in enumerate(_stream(40 + len(name), 40000, 500, ooo=2 * kw["size_ms"], step_ms=1300, n_wm=22)):
        nul = {1: (rng.random(len(k)) < 0.2).astype(np.uint8)}
        vals = [iv, dv.view(np.int64)]
        tp.process_batch(k, t, vals, nulls=nul)
        ol.process_batch(k, t, vals, nul)
        o1.process_batch(k, t, vals, nul)
        key, se, fields, nm = tp.local_partials(wm)
        ol.process_watermark(wm)
        want_l = _rows(ol.results(clear=True), tp.local_cfg, set())
        got_l = sorted((int(a), int(b), int(b), tuple(int(f[i]) for f in fields), int(c))
                       for i, (a, b, c) in enumerate(zip(key.tolist(), se.tolist(), nm.tolist())))
        # LOCAL: DOUBLE sums fold in a different order (1e-9), the rest bit-exact
        dcols_l = {j for j, ty in enumerate(tp.global_cfg.value_col_types[:tp.n_fields]) if ty == F64}
        _compare(got_l, want_l, dcols_l, f"{name} LOCAL batch {bi}")
        # GLOBAL fed the GPU's partials (in the GPU's order) on both sides
        _push_partials_to_oracle(og, key, se, fields, nm)
        tp.global_ingest(key, se, fields, nm)
        tp.glob.advance(wm)
        og.process_watermark(wm)
        o1.process_watermark(wm)
        got = _rows(tp.glob.results(reset=True), cfg, _double_cols(kw))
        _compare(got, _rows(og.results(clear=True), cfg, _double_cols(kw)), _double_cols(kw), f"{name} GLOBAL batch {bi}")
        want1 = _rows(o1.results(clear=True), cfg, _double_cols(kw))
        if not kw.get("offset_ms"):
            # The plans agree on slice-aligned trigger grids.  With an offset they need not: both
            # operators flush their buffers only when the watermark crosses the trigger grid of
            # TimeWindowUtil.getNextTriggerWatermark, which ignores the window offset, so a LOCAL
            # flush can reach the GLOBAL operator after its slice fired (then it drops as late),
            # where the one-phase operator had accepted those records at arrival.
            _compare(got, want1, _double_cols(kw), f"{name} vs one-phase batch {bi}")
    # the GLOBAL operator counts dropped partial rows (one per (key, slice) group), not records
    assert tp.num_late_records_dropped == og.late_dropped
    tp.close()


@pytest.mark.parametrize("p", [2, 4])
def test_two_phase_sharded_subtasks_match_one_phase(p):
    """p source subtasks run LOCAL, their partials are routed by fw_partition_by_dest to p GLOBAL
    subtasks (computeKeyGroupRangeForOperatorIndex), and the union of the GLOBAL results equals one
    unsharded one-phase operator."""
    torch = _torch_cuda()
    from flink_amd.runtime.exchange import KeyByExchange
    from flink_amd.table.two_phase import TwoPhaseWindowAgg
    from oracle.oracle import OracleOperator
    kw = TWO_PHASE_CASES["hop"]
    cfgs = [_cfg(kw, key_hash=abi.KEYHASH_BINROW_BIGINT, parallelism=p, subtask_index=i) for i in range(p)]
    ops = [TwoPhaseWindowAgg(c) for c in cfgs]
    o1 = OracleOperator(_cfg(kw, key_hash=abi.KEYHASH_BINROW_BIGINT))
    ex = KeyByExchange(abi.KEYHASH_BINROW_BIGINT, 128)
    ex.world = p
    for bi, (k, t, iv, dv, wm) in enumerate(_stream(77 + p, 50000, 3000, ooo=4000, step_ms=1500, n_wm=18)):
        vals = [iv, dv.view(np.int64)]
        o1.process_batch(k, t, vals)
        for src, part in enumerate(np.array_split(np.arange(len(k)), p)):  # source subtasks
            ops[src].process_batch(k[part], t[part], [v[part] for v in vals])
        o1.process_watermark(wm)
        # every source's partials, routed to the global subtasks (slicing replaces the all-to-all)
        for src in range(p):
            key, se, fields, nm = ops[src].local_partials(wm)
            pk, pse, pcols, counts = ex.partition(key, se, fields + [nm])
            off = 0
            for d, c in enumerate(counts.tolist()):
                if c:
                    ops[d].global_ingest(pk[off:off + c], pse[off:off + c], [x[off:off + c] for x in pcols[:-1]],
                                         pcols[-1][off:off + c])
                off += c
        got = []
        for op in ops:
            op.glob.advance(wm)
            got += _rows(op.glob.results(reset=True), cfgs[0], _double_cols(kw))
        _compare(sorted(got), _rows(o1.results(clear=True), cfgs[0], _double_cols(kw)), _double_cols(kw),
                 f"two-phase p={p} batch {bi}")
    for op in ops:
        assert op.glob.stats()["error_flags"] == 0
        op.close()


@pytest.mark.parametrize("name", ["sql_hop", "sql_tumble_int_aggs", "ds_tumble_lateness"])
def test_padded_segments_ingest_matches_oracle(name):
    """fw_push_device_segments (the padded all-to-all receive buffer of the bench's exchange):
    segments of a fixed capacity whose tails hold garbage rows (keys of foreign key groups, wild
    timestamps) that must never be read; results equal the oracle fed only the valid rows."""
    torch = _torch_cuda()
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    kw = CASES[name]
    cfg = _cfg(kw, parallelism=2, subtask_index=1, key_hash=abi.KEYHASH_LONG)
    g, o = WindowAggHandle(cfg), OracleOperator(cfg)
    from flink_amd._native import lib
    rng = np.random.default_rng(3)
    for bi, (k, t, iv, dv, wm) in enumerate(_stream(9, 30000, 400, ooo=2500, step_ms=1000, n_wm=12)):
        mine = np.array([lib().fw_host_key_group(abi.KEYHASH_LONG, int(x), 0, 128) >= 64 for x in k])
        k, t, iv, dv = k[mine], t[mine], iv[mine], dv[mine]
        nseg, cap = 3, len(k) + 50
        cuts = np.sort(rng.integers(0, len(k) + 1, nseg - 1))
        parts = np.split(np.arange(len(k)), cuts)
        counts = np.array([len(p) for p in parts], np.int64)
        assert counts.max() <= cap
        cols = {c: np.zeros(nseg * cap, np.int64) for c in ("k", "t", "i", "d")}
        for c in cols:  # garbage everywhere first: foreign keys, timestamps far in the past / future
            cols[c][:] = rng.integers(-(1 << 62), 1 << 62, nseg * cap)
        for s_, p_ in enumerate(parts):
            sl = slice(s_ * cap, s_ * cap + len(p_))
            cols["k"][sl], cols["t"][sl], cols["i"][sl], cols["d"][sl] = k[p_], t[p_], iv[p_], dv[p_].view(np.int64)
        dvc = lambda a: torch.tensor(a, device="cuda")
        g.push_device_segments(dvc(counts), dvc(cols["k"]), dvc(cols["t"]), [dvc(cols["i"]), dvc(cols["d"])])
        o.process_batch(k, t, [iv, dv.view(np.int64)])
        g.advance(wm)
        o.process_watermark(wm)
        _compare(_rows(g.results(reset=True), cfg, _double_cols(kw)), _rows(o.results(clear=True), cfg, _double_cols(kw)),
                 _double_cols(kw), f"{name} batch {bi}")
    assert g.stats()["error_flags"] == 0
    assert g.stats()["num_late_records_dropped"] == o.late_dropped
    g.close()


@pytest.mark.parametrize("name", ["sql_tumble_int_aggs", "sql_tumble_double", "sql_hop", "sql_cumulate_countstar", "ds_sliding_max"])
def test_packed_segments_ingest_matches_oracle(name):
    """fw_push_device_packed_segments (the packed padded all-to-all receive buffer the bench's
    exchange ingests): (key, ts, values) rows side by side, segments of a fixed capacity whose
    tails hold garbage rows; results equal the oracle fed only the valid rows."""
    torch = _torch_cuda()
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    kw = CASES[name]
    cfg = _cfg(kw, parallelism=2, subtask_index=1, key_hash=abi.KEYHASH_LONG)
    g, o = WindowAggHandle(cfg), OracleOperator(cfg)
    from flink_amd._native import lib
    rng = np.random.default_rng(5)
    w = 2 + cfg.n_value_cols
    for bi, (k, t, iv, dv, wm) in enumerate(_stream(11, 30000, 400, ooo=2500, step_ms=1000, n_wm=12)):
        mine = np.array([lib().fw_host_key_group(abi.KEYHASH_LONG, int(x), 0, 128) >= 64 for x in k])
        k, t, iv, dv = k[mine], t[mine], iv[mine], dv[mine]
        nseg, cap = 3, len(k) + 37
        cuts = np.sort(rng.integers(0, len(k) + 1, nseg - 1))
        parts = np.split(np.arange(len(k)), cuts)
        counts = np.array([len(p) for p in parts], np.int64)
        rows = rng.integers(-(1 << 62), 1 << 62, (nseg, cap, w)).astype(np.int64)  # garbage padding
        vals = [iv, dv.view(np.int64)][:cfg.n_value_cols]
        for s_, p_ in enumerate(parts):
            rows[s_, :len(p_), 0], rows[s_, :len(p_), 1] = k[p_], t[p_]
            for c, v in enumerate(vals):
                rows[s_, :len(p_), 2 + c] = v[p_]
        dvc = lambda a: torch.tensor(a, device="cuda")
        g.push_device_packed_segments(dvc(counts), dvc(rows.reshape(-1)), w)
        o.process_batch(k, t, vals)
        g.advance(wm)
        o.process_watermark(wm)
        _compare(_rows(g.results(reset=True), cfg, _double_cols(kw)), _rows(o.results(clear=True), cfg, _double_cols(kw)),
                 _double_cols(kw), f"{name} batch {bi}")
    assert g.stats()["error_flags"] == 0
    assert g.stats()["num_late_records_dropped"] == o.late_dropped
    g.close()


def test_partition_packed_equals_partition_by_dest():
    """fw_partition_packed writes exactly fw_partition_by_dest's per-destination row order into
    padded packed segments (and counts every row, also past the capacity)."""
    torch = _torch_cuda()
    import ctypes as C
    from flink_amd._native import check, lib
    L = lib()
    n, p = 50000, 4
    rng = np.random.default_rng(8)
    k = torch.tensor(rng.integers(0, 10**6, n), device="cuda")
    t = torch.tensor(rng.integers(0, 10**9, n), device="cuda")
    v = torch.tensor(rng.integers(-10**9, 10**9, n), device="cuda")
    ws = torch.empty(L.fw_partition_workspace_bytes(n, p), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    pk, pt, pv = torch.empty_like(k), torch.empty_like(t), torch.empty_like(v)
    c1 = torch.empty(p, dtype=torch.int64, device="cuda")
    vin = (C.c_void_p * abi.FW_MAX_COLS)(v.data_ptr())
    vout = (C.c_void_p * abi.FW_MAX_COLS)(pv.data_ptr())
    check(L.fw_partition_by_dest(k.data_ptr(), None, t.data_ptr(), vin, 1, n, abi.KEYHASH_BINROW_BIGINT, 128, p,
                                 pk.data_ptr(), pt.data_ptr(), vout, c1.data_ptr(), ws.data_ptr(), ws.numel(), s))
    cnt = c1.cpu().numpy()
    cap = int(cnt.max()) - 100  # the largest destination overflows its segment: its tail is dropped
    rows = torch.full((p * cap * 3,), -7, dtype=torch.int64, device="cuda")
    c2 = torch.empty(p, dtype=torch.int64, device="cuda")
    check(L.fw_partition_packed(k.data_ptr(), None, t.data_ptr(), vin, 1, n, abi.KEYHASH_BINROW_BIGINT, 128, p, cap,
                                rows.data_ptr(), c2.data_ptr(), ws.data_ptr(), ws.numel(), s))
    torch.cuda.synchronize()
    assert (c2.cpu().numpy() == cnt).all()
    seg = rows.view(p, cap, 3).cpu().numpy()
    ref = np.stack([pk.cpu().numpy(), pt.cpu().numpy(), pv.cpu().numpy()], axis=1)
    o = 0
    for d in range(p):
        m = min(int(cnt[d]), cap)
        assert (seg[d, :m] == ref[o:o + m]).all(), d
        assert (seg[d, m:] == -7).all(), d  # padding untouched
        o += int(cnt[d])


@pytest.mark.parametrize("delivery", ["kernel", "dma"])
@pytest.mark.parametrize("depth", [1, 2])
@pytest.mark.parametrize("name", ["sql_tumble_int_aggs", "sql_hop", "sql_tumble_double", "ds_sliding_max"])
def test_async_results_pipeline_matches_oracle(name, depth, delivery, monkeypatch):
    """fw_results_async / fw_results_ready: watermark b's rows are collected into pinned host memory
    while batch b + 1 is pushed (three pushes per watermark through the double-buffered staging)
    and read ``depth`` steps later (the oldest outstanding collection first) -- the same rows as
    the oracle's, watermark by watermark.  A fourth outstanding collection is refused.  ``dma``:
    the rows cross by hipMemcpyAsync on the D2H stream instead of the copy kernel (FW_AR_KERNEL=0:
    the early copy started by the next call, the wait before a buffer is reused, the synchronous
    copy in fw_results_ready)."""
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    if delivery == "dma":
        monkeypatch.setenv("FW_AR_KERNEL", "0")
    kw = CASES[name]
    cfg = _cfg(kw)
    dc = _double_cols(kw)
    o, g = OracleOperator(cfg), WindowAggHandle(cfg)
    pending = []
    for bi, (k, t, iv, dv, wm) in enumerate(_stream(zlib.crc32(name.encode()) % 997, 30000, 500, ooo=2 * kw["size_ms"],
                                                    step_ms=1500, n_wm=16)):
        vals = [iv, dv.view(np.int64)]
        o.process_batch(k, t, vals)
        for part in np.array_split(np.arange(len(k)), 3):
            g.push_host(k[part], t[part], [v[part] for v in vals])
        o.process_watermark(wm)
        g.advance(wm)
        want = _rows(o.results(clear=True), cfg, dc)
        if depth == 1 and pending:
            _compare(_rows(g.results_ready(), cfg, dc), pending.pop(0), dc, f"watermark before batch {bi}")
        g.results_async()
        pending.append(want)
        if depth == 2 and len(pending) > 2:
            _compare(_rows(g.results_ready(), cfg, dc), pending.pop(0), dc, f"watermark two before batch {bi}")
    if depth == 2:
        from flink_amd._native import FlinkWinError
        g.results_async()  # a third outstanding collection is allowed (nothing emitted since: no rows)
        with pytest.raises(FlinkWinError):
            g.results_async()
        pending.append(None)
    while pending:
        want = pending.pop(0)
        rows = _rows(g.results_ready(), cfg, dc)
        if want is None:
            assert len(rows) == 0
        else:
            _compare(rows, want, dc, "last watermarks")
    assert g.stats()["error_flags"] == 0 and g.stats()["num_late_records_dropped"] == o.late_dropped
    g.close()


@pytest.mark.parametrize("name", ["sql_tumble_int_aggs", "sql_tumble_double", "ds_sliding_max"])
def test_delta32_transfer_matches_words(name):
    """fw_commit_delta32: columns whose batch values span < 2^32 cross PCIe as 32-bit deltas and are
    widened on the device -- the same rows as 8-byte words through fw_commit, and the oracle's.  Odd
    push sizes (the widening's tail), and batches whose value column spans more (not packed): the
    mask changes from push to push."""
    import ctypes as C
    from flink_amd import _native, abi
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    kw = CASES[name]
    cfg = _cfg(kw)
    dc = _double_cols(kw)
    o, gw, gd = OracleOperator(cfg), WindowAggHandle(cfg), WindowAggHandle(cfg)
    for bi, (k, t, iv, dv, wm) in enumerate(_stream(zlib.crc32(name.encode()) % 991, 20000, 400, ooo=2 * kw["size_ms"],
                                                    step_ms=1500, n_wm=10)):
        if bi % 3 == 1:  # this batch's BIGINT values span > 2^32: that column goes as words
            iv = iv * (1 << 30) - (1 << 40)
        vals = [iv, dv.view(np.int64)]
        o.process_batch(k, t, vals)
        for part in np.split(np.arange(len(k)), [len(k) // 3 + 1, len(k) // 2 + 3]):
            gw.push_host(k[part], t[part], [v[part] for v in vals], delta32=False)
            gd.push_host(k[part], t[part], [v[part] for v in vals])
        o.process_watermark(wm)
        gw.advance(wm)
        gd.advance(wm)
        want = _rows(o.results(clear=True), cfg, dc)
        _compare(_rows(gw.results(reset=True), cfg, dc), want, dc, f"words, watermark {bi}")
        _compare(_rows(gd.results(reset=True), cfg, dc), want, dc, f"delta32, watermark {bi}")
    for g in (gw, gd):
        assert g.stats()["error_flags"] == 0 and g.stats()["num_late_records_dropped"] == o.late_dropped
    # a slot the operator does not have, or packed columns without bases: refused
    L = _native.lib()
    cols = abi.fw_host_cols()
    _native.check(L.fw_reserve(gd._h, 16, C.byref(cols)))
    bases = (C.c_int64 * (2 + abi.FW_MAX_COLS))()
    assert L.fw_commit_delta32(gd._h, 16, 1 << (2 + cfg.n_value_cols), bases) != 0
    assert L.fw_commit_delta32(gd._h, 16, 2, None) != 0
    _native.check(L.fw_commit(gd._h, 0))
    gw.close()
    gd.close()


@pytest.mark.parametrize("name", ["sql_tumble_int_aggs", "sql_hop", "sql_cumulate_countstar", "ds_sliding_max",
                                  "sql_tumble_double"])
def test_state_beyond_ingest_superbuckets_matches_oracle(name):
    """A state hint past the 16384 superbuckets the ingest histogram holds: the ingest partitions
    into 16384 and several merge passes share each ingest superbucket's partial rows, each keeping
    the keys that route to its own superbucket (KeySpace.pass_log2) -- the same results as the
    oracle, snapshot included."""
    kw = CASES[name]
    st = {}
    cfg = _cfg(kw, state_capacity=80_000_000, output_capacity=1 << 20)
    _run_both(cfg, _stream(zlib.crc32(name.encode()) % 991, 40000, 3000, ooo=2 * kw["size_ms"] + 1500,
                           step_ms=1500, n_wm=16), _double_cols(kw), split=2, snapshot_at=9, stats=st)
    assert st["num_superbuckets"] > 16384, st["num_superbuckets"]


@pytest.mark.parametrize("name", ["hop", "cumulate"])
def test_two_phase_device_step_matches_one_phase(name):
    """TwoPhaseWindowAgg.step_device: the LOCAL partials never reach the host -- collected on the
    device (fw_results_device), partitioned by their device-side count (fw_partition_packed_spill_dn)
    and ingested as packed segments by the GLOBAL operator -- and the results equal one one-phase
    oracle operator's (NOT NULL inputs: the GLOBAL fields are NOT NULL, the packed rows carry none)."""
    torch = _torch_cuda()
    from flink_amd.table.two_phase import TwoPhaseWindowAgg
    from oracle.oracle import OracleOperator
    kw = dict(TWO_PHASE_CASES[name])
    cfg = _cfg(kw)
    tp = TwoPhaseWindowAgg(cfg)
    assert tp.global_cfg.nullable_cols == 0
    o1 = OracleOperator(cfg)
    dc = _double_cols(kw)
    for bi, (k, t, iv, dv, wm) in enumerate(_stream(77 + len(name), 40000, 500, ooo=2 * kw["size_ms"], step_ms=1300,
                                                    n_wm=20)):
        vals = [iv, dv.view(np.int64)]
        tp.process_batch_device(torch.tensor(k, device="cuda"), torch.tensor(t, device="cuda"),
                                [torch.tensor(v, device="cuda") for v in vals])
        o1.process_batch(k, t, vals)
        assert tp.step_device(wm) == wm
        o1.process_watermark(wm)
        _compare(_rows(tp.glob.results(reset=True), cfg, dc), _rows(o1.results(clear=True), cfg, dc), dc,
                 f"{name} batch {bi}")
    assert tp.glob.stats()["error_flags"] == 0 and tp.local.stats()["error_flags"] == 0
    tp.close()


@pytest.mark.parametrize("n_keys", [3, 5000])
def test_ds_many_late_fire_rows_match_oracle(n_keys):
    """A burst of late elements within allowedLateness: each fires its window at once with the
    element added (EventTimeTrigger.onElement -> FIRE).  3 keys put ~2000 late rows into one
    superbucket (beyond the merge kernel's LDS list of 1024: the scan path), 5000 keys spread them
    (the LDS list path); every late row emits one window row, bit-exact with the oracle."""
    _torch_cuda()
    import time
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    kw = CASES["ds_tumble_lateness"]  # 4 s windows, 3 s lateness
    cfg = _cfg(kw)
    o, g = OracleOperator(cfg), WindowAggHandle(cfg)
    rng = np.random.default_rng(n_keys)
    t0 = 1_600_000_000_000
    n = 6000
    k = rng.integers(0, n_keys, n).astype(np.int64)
    t = (t0 + rng.integers(0, 8000, n)).astype(np.int64)
    iv = rng.integers(-1000, 1000, n).astype(np.int64)
    batches = [(k, t, iv, t0 + 8000)]
    # late elements into the fired windows [t0, t0+4000) and [t0+4000, t0+8000): cleanup at +3 s
    k2 = rng.integers(0, n_keys, n).astype(np.int64)
    t2 = (t0 + 4000 + rng.integers(0, 4000, n)).astype(np.int64)
    batches.append((k2, t2, rng.integers(-1000, 1000, n).astype(np.int64), t0 + 9000))
    batches.append((k2[:100], t2[:100] + 4000, iv[:100], t0 + 20000))
    dt = 0.0
    for bi, (kk, tt, vv, wm) in enumerate(batches):
        vals = [vv, np.zeros(len(kk), np.int64)]
        o.process_batch(kk, tt, vals)
        g.push_host(kk, tt, vals)
        o.process_watermark(wm)
        t_start = time.perf_counter()
        g.advance(wm)
        res = g.results(reset=True)
        dt = max(dt, time.perf_counter() - t_start)
        _compare(_rows(res, cfg, set()), _rows(o.results(clear=True), cfg, set()), set(), f"batch {bi}")
    assert g.stats()["error_flags"] == 0
    print(f"n_keys={n_keys}: slowest advance {dt * 1e3:.1f} ms")
    g.close()


def test_skipped_advance_keeps_watermark_through_snapshot():
    """An advance that crosses no slice end launches nothing (fw_advance's idle skip), yet the
    operator's currentWatermark is the new one: in stats, in a full snapshot and in a key-group
    blob (the union-list watermark state each subtask contributes)."""
    _torch_cuda()
    from flink_amd.runtime.handle import WindowAggHandle
    cfg = _cfg(CASES["sql_tumble_int_aggs"], key_hash=abi.KEYHASH_BINROW_BIGINT)
    g = WindowAggHandle(cfg)
    t0 = 1_600_000_000_000  # a multiple of the 10 s window
    k = np.arange(1000, dtype=np.int64)
    g.push_host(k, t0 + k, [k, k])
    g.advance(t0 + 10_000)      # fires [t0, t0 + 10 s)
    g.advance(t0 + 12_345)      # crosses no slice end: skipped
    assert g.stats()["current_watermark"] == t0 + 12_345
    blob = g.snapshot()
    h = WindowAggHandle(cfg)
    h.restore(blob)
    assert h.stats()["current_watermark"] == t0 + 12_345
    _, wm = g.snapshot_key_groups()
    assert wm == t0 + 12_345
    for x in (g, h):
        x.close()


@pytest.mark.parametrize("layout", ["runs", "cells"])
def test_restore_into_same_handle_drops_pending_pushes(layout, monkeypatch):
    """A restore drops the pushes still pending in the handle (the reference restores into a fresh
    operator: nothing buffered survives).  With runs, the dropped push's sub-run fill counters must
    go too, or the next flush folds its stale rows."""
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    monkeypatch.setenv("FW_RUNS", "1" if layout == "runs" else "0")
    kw = CASES["sql_tumble_int_aggs"]
    cfg = _cfg(kw)
    batches = _stream(4242, 120_000, 3000, ooo=2500, step_ms=3000, n_wm=6)
    o, g = OracleOperator(cfg), WindowAggHandle(cfg)

    def step(bi, push_oracle=True):
        k, t, iv, dv, wm = batches[bi]
        vals = [iv, dv.view(np.int64)]
        g.push_host(k, t, vals)
        if push_oracle:
            o.process_batch(k, t, vals)

    for bi in range(3):
        step(bi)
        wm = batches[bi][4]
        o.process_watermark(wm)
        g.advance(wm)
        _compare(_rows(g.results(reset=True), cfg, set()), _rows(o.results(clear=True), cfg, set()), set(), f"batch {bi}")
    blob = g.snapshot()
    o.snapshot_restore()
    step(3, push_oracle=False)  # pending in the handle, then dropped by the restore
    g.restore(blob)
    for bi in range(4, 6):
        step(bi)
        wm = batches[bi][4]
        o.process_watermark(wm)
        g.advance(wm)
        _compare(_rows(g.results(reset=True), cfg, set()), _rows(o.results(clear=True), cfg, set()), set(), f"batch {bi}")
    assert g.stats()["error_flags"] == 0
    g.close()


# HOP block state in the narrow layouts (k_merge_hopb: a superbucket whose every slot word with data
# fits int16 / int32 is written back as 5 / 7 words instead of 11, 7 / 11 instead of 19) and back: some batches carry values
# past 2^31 (and sums that pass it by accumulation), so superbuckets switch layouts from flush to flush;
# a snapshot / restore in the middle reads narrow and wide superbuckets back.  COUNT(*) + SUM and
# COUNT(*) + MIN (whose empty slots hold the identity Long.MAX_VALUE, restored on load).
@pytest.mark.parametrize("agg", [abi.AGG_SUM, abi.AGG_MIN, abi.AGG_MAX])
@pytest.mark.parametrize("narrow", ["2", "1", "0"])
def test_hop_block_state_narrow_and_wide_layouts(agg, narrow, monkeypatch):
    monkeypatch.setenv("FW_HB_NARROW", narrow)
    kw = dict(window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=2000, count_star_index=0,
              aggs=[(abi.AGG_COUNT_STAR, 0, I64), (agg, 0, I64)])
    batches = _stream(4242 + agg, 24000, 400, ooo=12000, step_ms=4500, n_wm=24)
    out = []
    for b, (k, t, iv, dv, wm) in enumerate(batches):
        iv = iv.copy()
        if b % 6 == 2:  # a few keys with values past int32
            sel = (k // 7919) % 7 == 0
            iv[sel] = iv[sel] * (1 << 33) + (1 << 40)
        elif b % 6 == 4:  # sums past int32 by accumulation (each value < 2^31)
            iv[:] = (1 << 30) + iv
        out.append((k, t, iv, dv, wm))
    for snap in (None, 11):
        _run_both(_cfg(kw), out, _double_cols(kw), snapshot_at=snap)
