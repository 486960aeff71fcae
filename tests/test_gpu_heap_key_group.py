"""GPU parity of the heap keyed-state backend's key-group format (flinkwin.h
fw_snapshot_key_group_heap / fw_restore_key_group_heap).

A handle runs part of a stream, writes every key group in the heap backend's bytes, and the parsed
contents must equal the oracle's keyed state at the same cut: one window-aggs entry per (key,
namespace) with the aggregates' buffer fields, and the event-time timers (timestamp, key,
namespace).  The blobs then restore into fresh handles -- at the same or another parallelism --
and the run continues against the oracle.  The byte layout is restated in tests/heap_format.py
from the Java writers; no Flink build is available, so the format is parity unpinned while its
contents and the restore are checked."""
import numpy as np
import pytest

from flink_amd import abi
from heap_format import acc_field_types, parse_key_group
from parity_common import CASES, F64, I32, I64, _cfg, _compare, _double_cols, _rows, _stream, _torch_cuda

pytestmark = pytest.mark.gpu

HEAP_CASES = {
    # TUMBLE: counts, nullable SUM, DOUBLE MIN/MAX word groups, AVG(DOUBLE), COUNT(col)
    "tumble_mixed_nullable": dict(window_kind=abi.WIN_TUMBLE, size_ms=5000, nullable_cols=[0, 1],
                                  aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MIN, 1, F64),
                                        (abi.AGG_COUNT, 0, I64)]),
    "tumble_avg_nullable": dict(window_kind=abi.WIN_TUMBLE, size_ms=5000, nullable_cols=[0, 1],
                                aggs=[(abi.AGG_AVG, 1, F64), (abi.AGG_MAX, 0, I64), (abi.AGG_COUNT, 1, F64),
                                      (abi.AGG_SUM, 1, F64)]),
    "tumble_int_offset": dict(window_kind=abi.WIN_TUMBLE, size_ms=7000, offset_ms=-2500, value_col_types=[I32, F64],
                              aggs=[(abi.AGG_SUM, 0, I32), (abi.AGG_MAX, 0, I32), (abi.AGG_AVG, 0, I32)]),
    # HOP with block state (k_merge_hopb) and HOP with slice entries (DOUBLE MAX: word groups)
    "hop_blocks": CASES["sql_hop_offset"],
    "hop_slices": CASES["sql_hop"],
    "cumulate": CASES["sql_cumulate_countstar"],
    "cumulate_nocount": CASES["sql_cumulate_nocount"],
    # GLOBAL phase: the value columns are LOCAL accumulator fields (count, DOUBLE max), rows at slice ends
    "global_tumble": dict(window_kind=abi.WIN_TUMBLE, size_ms=4000, agg_phase=abi.PHASE_GLOBAL, nullable_cols=[1],
                          aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_MAX, 1, F64)]),
    "tumble_shift_zone": dict(window_kind=abi.WIN_TUMBLE, size_ms=3600000, shift_zone="America/Los_Angeles",
                              aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_MIN, 0, I64)]),
}

IDS = (3, 1, 2)  # window-aggs, event timers, processing timers: written in id order


def _norm_fields(vals, types, nm):
    out = []
    for j, (x, t) in enumerate(zip(vals, types)):
        x = int(x) - (1 << 64) if int(x) >= 1 << 63 else int(x)
        if (nm >> j) & 1:
            x = 0
        elif t == I32:
            x = ((x & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000
        out.append(x)
    return out


def _fields_equal(a, b, types):
    for x, y, t in zip(a, b, types):
        if t == F64:
            xd, yd = np.int64(x).view(np.float64), np.int64(y).view(np.float64)
            if np.isnan(xd) and np.isnan(yd):
                continue
            if xd != pytest.approx(yd, rel=1e-9, abs=0.0):
                return False
        elif x != y:
            return False
    return True


def _heap_stream(kw, seed):
    if kw.get("shift_zone"):
        t0, step, ooo = 1_667_718_000_000, 1_200_000, 2_400_000  # across the 2022-11-06 09:00Z DST end
    else:
        t0, step, ooo = 0, 1200, 2500
    batches = _stream(seed, 36000, 900, ooo=ooo, step_ms=step, n_wm=14)
    if t0:
        batches = [(k, t - 1_600_000_000_000 + t0, iv, dv, wm - 1_600_000_000_000 + t0) for k, t, iv, dv, wm in batches]
    rng = np.random.default_rng(seed + 1)
    nulls = None
    if kw.get("nullable_cols"):
        nulls = [{c: (rng.random(len(b[0])) < 0.2).astype(np.uint8) for c in kw["nullable_cols"]} for b in batches]
    if kw.get("agg_phase") == abi.PHASE_GLOBAL:  # local rows: slice-end timestamps, counts >= 1
        size = kw["size_ms"]
        batches = [(k, (t // size + 1) * size, np.abs(iv) + 1, dv, wm) for k, t, iv, dv, wm in batches]
    if kw.get("value_col_types", [I64])[0] == I32:
        batches = [(k, t, (iv * 2_000_003) % (1 << 31) - (1 << 30), dv, wm) for k, t, iv, dv, wm in batches]
    return batches, nulls


def _check_against_oracle(cfg, blobs, o, hopb):
    types = acc_field_types(cfg)
    from oracle.oracle import key_group
    want_states, want_timers = o.keyed_state()
    got_states, got_timers = [], []
    for kg, blob in blobs.items():
        k2, st, tm, n_proc = parse_key_group(blob, cfg, IDS)
        assert k2 == kg and n_proc == 0
        for s in st:
            assert key_group(cfg.key_hash, s[0], 128) == kg, "state entry in a foreign key group"
        got_states += st
        got_timers += tm
    got = sorted((k, ns, _norm_fields(v, types, nm), nm) for k, ns, v, nm in got_states)
    want = sorted((k, ns, _norm_fields(v, types, nm), nm) for k, ns, v, nm in want_states)
    assert [(k, ns, nm) for k, ns, _, nm in got] == [(k, ns, nm) for k, ns, _, nm in want]
    for a, b in zip(got, want):
        assert _fields_equal(a[2], b[2], types), f"accumulator of {a[:2]}: {a[2]} != {b[2]}"
    want_t = sorted(want_timers)
    if hopb:  # block state leaves out chain timers at empty windows (they fire without output)
        live = {}
        for k, ns, _, _ in want_states:
            live.setdefault(k, []).append(ns)
        size = cfg.size_ms
        want_t = [t for t in want_t if any(t[2] - size < ns <= t[2] for ns in live.get(t[1], []))]
    assert sorted(got_timers) == want_t
    return len(got), len(got_timers)


@pytest.mark.parametrize("case", sorted(HEAP_CASES))
@pytest.mark.parametrize("p_to", [1, 3])
def test_heap_key_groups_match_oracle_state_and_restore(case, p_to):
    """Cut after 8 watermarks: the heap-format key groups hold exactly the oracle's keyed state
    and timers; restored at parallelism p_to the run continues bit-exact with the oracle."""
    _torch_cuda()
    from flink_amd.runtime.handle import WindowAggHandle
    from oracle.oracle import OracleOperator
    kw = dict(HEAP_CASES[case])
    dcols = _double_cols(kw)
    cfg = _cfg(kw, key_hash=abi.KEYHASH_BINROW_BIGINT)
    batches, nulls = _heap_stream(kw, 71 + len(case))
    o, g = OracleOperator(cfg), WindowAggHandle(cfg)
    cut = 8
    hs, cfgs = [g], [cfg]
    for bi, (k, t, iv, dv, wm) in enumerate(batches):
        if bi == cut:
            o.flush()  # prepareSnapshotPreBarrier: the buffer is flushed into the state
            blobs = {kg: g.snapshot_key_group_heap(kg, IDS) for kg in range(128)}
            n_st, n_tm = _check_against_oracle(cfg, blobs, o, case == "hop_blocks")
            assert n_st > 100 and (n_tm > 0 or kw["window_kind"] == abi.WIN_HOP)
            wm_cut = g.stats()["current_watermark"]
            g.close()
            cfgs = [_cfg(kw, key_hash=abi.KEYHASH_BINROW_BIGINT, parallelism=p_to, subtask_index=i) for i in range(p_to)]
            hs = [WindowAggHandle(c) for c in cfgs]
            for h in hs:
                lo, hi = h.key_group_range()
                for kg in range(lo, hi + 1):
                    h.restore_key_group_heap(blobs[kg], IDS)
                h.initialize_watermark(wm_cut)
            o.snapshot_restore()
        vals = [iv, dv.view(np.int64)]
        nb = nulls[bi] if nulls is not None else None
        o.process_batch(k, t, vals, nb)
        if len(hs) == 1:
            hs[0].push_host(k, t, vals, nulls=nb)
        else:
            dest = np.array(_dest(k, len(hs)))
            for i, h in enumerate(hs):
                m = dest == i
                if m.any():
                    h.push_host(k[m], t[m], [v[m] for v in vals], nulls=None if nb is None else {c: f[m] for c, f in nb.items()})
        o.process_watermark(wm)
        got = []
        for h in hs:
            h.advance(wm)
            got += _rows(h.results(reset=True), cfgs[0], dcols)
        _compare(sorted(got), _rows(o.results(clear=True), cfgs[0], dcols), dcols, f"{case} p_to={p_to} batch {bi}")
    assert all(h.stats()["error_flags"] == 0 for h in hs)
    for h in hs:
        h.close()


def _dest(keys, p):
    from flink_amd._native import lib
    out = []
    for k in keys.tolist():
        kg = lib().fw_host_key_group(abi.KEYHASH_BINROW_BIGINT, int(k), 0, 128)
        out.append(kg * p // 128)
    return out


def test_heap_key_group_round_trip_is_identity():
    """snapshot -> restore -> snapshot writes the same entries (as sets: the heap backend's
    iteration order is its hash table's), for every layout family, including empty key groups."""
    _torch_cuda()
    from flink_amd.runtime.handle import WindowAggHandle
    for case in ("tumble_mixed_nullable", "hop_blocks", "hop_slices", "cumulate"):
        kw = HEAP_CASES[case]
        cfg = _cfg(kw, key_hash=abi.KEYHASH_BINROW_BIGINT)
        batches, nulls = _heap_stream(kw, 5)
        g = WindowAggHandle(cfg)
        for bi, (k, t, iv, dv, wm) in enumerate(batches[:6]):
            g.push_host(k, t, [iv, dv.view(np.int64)], nulls=None if nulls is None else nulls[bi])
            g.advance(wm)
        g.results(reset=True)
        a = {kg: g.snapshot_key_group_heap(kg, IDS) for kg in range(128)}
        h = WindowAggHandle(cfg)
        h.initialize_watermark(g.stats()["current_watermark"])
        for blob in a.values():
            h.restore_key_group_heap(blob, IDS)
        b = {kg: h.snapshot_key_group_heap(kg, IDS) for kg in range(128)}
        for kg in range(128):
            pa, pb = parse_key_group(a[kg], cfg, IDS), parse_key_group(b[kg], cfg, IDS)
            assert sorted(map(repr, pa[1])) == sorted(map(repr, pb[1])), f"{case} kg {kg} states"
            assert sorted(pa[2]) == sorted(pb[2]), f"{case} kg {kg} timers"
        g.close()
        h.close()


def test_heap_key_group_rejects_bad_input():
    _torch_cuda()
    from flink_amd._native import FlinkWinError
    from flink_amd.runtime.handle import WindowAggHandle
    cfg = _cfg(HEAP_CASES["tumble_mixed_nullable"], key_hash=abi.KEYHASH_BINROW_BIGINT)
    g = WindowAggHandle(cfg)
    k = np.arange(500, dtype=np.int64)
    g.push_host(k, np.full(500, 1_600_000_000_000, np.int64), [k, k], nulls={0: np.zeros(500, np.uint8), 1: np.zeros(500, np.uint8)})
    blobs = {kg: g.snapshot_key_group_heap(kg, IDS) for kg in range(128)}
    full = max(blobs.values(), key=len)
    h = WindowAggHandle(cfg)
    with pytest.raises(FlinkWinError):
        h.restore_key_group_heap(full[:-3], IDS)  # truncated
    with pytest.raises(FlinkWinError):
        h.restore_key_group_heap(full, (7, 1, 2))  # unknown state id
    h.restore_key_group_heap(full, IDS)
    with pytest.raises(FlinkWinError):
        h.restore_key_group_heap(full, IDS)  # the key group already holds state
    ds = WindowAggHandle(_cfg(CASES["ds_tumble_sum"], key_hash=abi.KEYHASH_LONG))
    with pytest.raises(FlinkWinError):  # DataStream WindowOperator state is not this layout
        ds.snapshot_key_group_heap(0, IDS)
    for x in (g, h, ds):
        x.close()
