"""GPU parity of the DataStream WindowOperator's heap key-group bytes (flink_amd/datastream/heap_state.py
over flinkwin.h fw_ds_snapshot_key_group / fw_ds_restore_key_group).

A record-shaped operator runs part of a stream; every key group is written in the heap backend's
bytes ("window-contents": TimeWindow namespace, key, value1 with the aggregated field set;
"window-timers": flipped timestamp, key, namespace).  Parsed back, the contents must be the oracle's
window states at the cut -- the record is the window's first element with the window's current
aggregate -- and the timers its timer set.  The key groups then restore into fresh operators at
parallelism 1 or 3 and the run continues record for record against the oracle.  DoubleSerializer
writes doubleToLongBits, so a NaN aggregate crosses the savepoint as the canonical NaN, as it does in
the reference; NaN payloads are compared as NaN.  Byte layout: parity unpinned (no Flink build here)."""
import struct
import zlib

import numpy as np
import pytest

from flink_amd import abi

pytestmark = pytest.mark.gpu

T0 = 1_600_000_000_000
IDS = (4, 2, 3)  # window-contents, event-time window-timers, processing-time window-timers
_SPECIAL = np.array([0x7FF8000000000000, 0xFFF8000000000001, 0x7FF00000DEADBEEF, 0x8000000000000000, 0],
                    dtype=np.uint64).view(np.int64)

CASES = {
    # (window, allowed lateness, aggregation, value column)
    "tumble_sum_long": (("tumble", 3000, 0), 0, ("sum", "LONG"), 2),
    "tumble_min_double_lateness": (("tumble", 2000, 0), 1500, ("min", "DOUBLE"), 3),
    "sliding_max_double_lateness": (("sliding", 3000, 1000), 2000, ("max", "DOUBLE"), 3),
    "sliding_nondiv_sum_long": (("sliding", 3500, 1000), 0, ("sum", "LONG"), 2),
    # minBy / maxBy: the state holds the extremal element itself
    "sliding_maxby_long_last": (("sliding", 3000, 1000), 1000, ("maxBy", "LONG", False), 2),
    "tumble_minby_double_first": (("tumble", 2000, 0), 0, ("minBy", "DOUBLE"), 3),
}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _batches(seed, n_wm=16, per=1500, n_keys=400, step_ms=1000, ooo=2500):
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_wm):
        base = T0 + b * step_ms
        ts = (base + rng.integers(0, step_ms, per) - rng.integers(0, ooo, per)).astype(np.int64)
        keys = rng.integers(0, n_keys, per).astype(np.int64) * 7919 - 100_000
        iv = rng.integers(-10**6, 10**6, per).astype(np.int64)
        dv = (rng.random(per) * 100.0).view(np.int64).copy()
        sp = rng.random(per) < 0.2
        dv[sp] = _SPECIAL[rng.integers(0, len(_SPECIAL), int(sp.sum()))]
        out.append((keys, ts, iv, dv, base + step_ms - ooo // 3))
    return out


def _operator(case, p=1, i=0):
    from flink_amd.datastream.heap_state import TupleSerializer
    from flink_amd.datastream.window_operator import WindowOperator
    from flink_amd.datastream.windowing import EventTimeTrigger, SlidingEventTimeWindows, TumblingEventTimeWindows
    (kind, size, slide), late, agg, _ = CASES[case]
    assigner = TumblingEventTimeWindows.of(size) if kind == "tumble" else SlidingEventTimeWindows.of(size, slide)
    ser = TupleSerializer.of("LONG", "DOUBLE" if agg[1] == "DOUBLE" else "LONG", "STRING")
    return WindowOperator(assigner, EventTimeTrigger(), agg, key_type="LONG", state_capacity=1 << 16,
                          max_batch_rows=1 << 14, output_capacity=1 << 18, allowed_lateness=late, field=1,
                          parallelism=p, subtask_index=i, record_serializer=ser).open()


def _canon(bits, dbl):
    """value bits as compared across a savepoint: DoubleSerializer writes doubleToLongBits"""
    if dbl and np.isnan(np.int64(bits).view(np.float64)):
        return 0x7FF8000000000000
    return int(bits)


def _field_bits(v, dbl):
    return struct.unpack("<q", struct.pack("<d", v))[0] if dbl else int(v)


def _kg(key):
    from flink_amd._native import lib
    return lib().fw_host_key_group(abi.KEYHASH_LONG, int(key), 0, 128)


def _check_cut(case, blobs, o, elements, dbl):
    from flink_amd.datastream.heap_state import KEY_SERIALIZERS, TupleSerializer, read_key_group
    (kind, size, slide), late, agg, _ = CASES[case]
    ser = TupleSerializer.of("LONG", "DOUBLE" if dbl else "LONG", "STRING")
    want_states, want_timers = o.ds_keyed_state()
    got_states, got_timers = {}, set()
    for kg, blob in blobs.items():
        k2, contents, timers = read_key_group(blob, IDS, KEY_SERIALIZERS["LONG"], ser)
        assert k2 == kg
        for key, st, end, rec in contents:
            assert _kg(key) == kg, "window-contents entry in a foreign key group"
            assert end - st == size and (key, end) not in got_states
            got_states[(key, end)] = rec
        for ts, key, st, end in timers:
            assert _kg(key) == kg and end - st == size
            got_timers.add((ts, key, end))
    assert sorted(got_states) == sorted(want_states), "window-contents (key, window) set differs from the oracle"
    for kw, rec in got_states.items():
        vbits, first = want_states[kw]
        e = elements[first]
        assert rec[0] == e[0] and rec[2] == e[2], f"window {kw}: not value1 (the first element)"
        assert _canon(_field_bits(rec[1], dbl), dbl) == _canon(vbits, dbl), f"window {kw}: aggregate differs"
    assert got_timers == set(want_timers), "window-timers differ from the oracle's timer set"
    return len(got_states), len(got_timers)


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("p_to", [1, 3])
def test_ds_heap_key_groups_match_oracle_and_restore(case, p_to):
    from oracle.oracle import OracleOperator
    vcol = CASES[case][3]
    dbl = vcol == 3
    ops = [_operator(case)]
    o = OracleOperator(ops[0].cfg)
    elements = {}  # oracle arrival ordinal -> element (key, field, tag)
    cut, dropped = 8, 0
    for b, (k, t, iv, dv, wm) in enumerate(_batches(zlib.crc32(case.encode()) % 1000)):
        if b == cut:
            blobs = {kg: ops[0].snapshot_key_group_heap(kg, IDS) for kg in range(128)}
            n_st, n_tm = _check_cut(case, blobs, o, elements, dbl)
            assert n_st > 100 and n_tm > 100
            dropped = ops[0].num_late_records_dropped
            ops[0].close()
            ops = [_operator(case, p_to, i) for i in range(p_to)]
            for op in ops:
                lo, hi = op.handle.key_group_range()
                for kg in range(lo, hi + 1):
                    assert op.restore_key_group_heap(blobs[kg], IDS) == kg
            o.snapshot_restore()
        v = iv if vcol == 2 else dv
        recs = []
        for i in range(len(k)):
            fv = int(v[i]) if vcol == 2 else struct.unpack("<d", struct.pack("<q", int(v[i])))[0]
            rec = (int(k[i]), fv, f"e{b}.{i}")
            recs.append(rec)
            elements[(b << 32) | i] = rec
        dest = np.array([_kg(x) * len(ops) // 128 for x in k.tolist()])
        for i, op in enumerate(ops):
            m = np.nonzero(dest == i)[0]
            if len(m):
                op.process_batch(k[m], t[m], v[m], records=[recs[j] for j in m.tolist()])
        o.process_batch(k, t, [v])
        got = []
        for op in ops:
            r = op.process_watermark(wm)
            got += [(kk, we, _canon(val, dbl), rec[0], _canon(_field_bits(rec[1], dbl), dbl), rec[2])
                    for kk, we, val, rec in zip(r["key"].tolist(), r["window_end"].tolist(), r["value"].tolist(),
                                                r["records"])]
        o.process_watermark(wm)
        want = o.results(clear=True)
        exp = []
        for kk, we, val, fo in zip(want["key"].tolist(), want["window_end"].tolist(), want["values"][0].tolist(),
                                   want["first_ord"].tolist()):
            e = elements[fo]
            exp.append((kk, we, _canon(val, dbl), e[0], _canon(val, dbl), e[2]))
        assert sorted(got) == sorted(exp), f"{case} p_to={p_to} batch {b}: records differ from the oracle"
    end = T0 + 10**9
    for op in ops:
        op.process_watermark(end)
        assert op.handle.stats()["live_state_entries"] == 0
        assert not op._retained, "first elements still retained after every window was cleared"
    o.process_watermark(end)
    assert dropped + sum(op.num_late_records_dropped for op in ops) == o.late_dropped
    for op in ops:
        op.close()


def test_ds_heap_round_trip_and_rejects_bad_input():
    """snapshot -> restore -> snapshot writes the same contents and timers; foreign key groups,
    truncated bytes and non-window namespaces are refused"""
    from flink_amd._native import FlinkWinError
    from flink_amd.datastream.heap_state import KEY_SERIALIZERS, TupleSerializer, read_key_group
    case = "sliding_max_double_lateness"
    op = _operator(case)
    for b, (k, t, iv, dv, wm) in enumerate(_batches(7, n_wm=6)):
        recs = [(int(k[i]), float(np.int64(dv[i]).view(np.float64)), f"r{b}.{i}") for i in range(len(k))]
        op.process_batch(k, t, dv, records=recs)
        op.process_watermark(wm)
    a = {kg: op.snapshot_key_group_heap(kg, IDS) for kg in range(128)}
    op2 = _operator(case)
    for blob in a.values():
        op2.restore_key_group_heap(blob, IDS)
    b2 = {kg: op2.snapshot_key_group_heap(kg, IDS) for kg in range(128)}
    ser = TupleSerializer.of("LONG", "DOUBLE", "STRING")
    for kg in range(128):
        pa = read_key_group(a[kg], IDS, KEY_SERIALIZERS["LONG"], ser)
        pb = read_key_group(b2[kg], IDS, KEY_SERIALIZERS["LONG"], ser)
        assert sorted(map(repr, pa[1])) == sorted(map(repr, pb[1])), f"kg {kg} contents"
        assert sorted(pa[2]) == sorted(pb[2]), f"kg {kg} timers"
    full = max(a.items(), key=lambda kv: len(kv[1]))
    op3 = _operator(case, 2, 0)
    lo, hi = op3.handle.key_group_range()
    foreign = next(kg for kg in range(128) if not lo <= kg <= hi and len(a[kg]) > 20)
    with pytest.raises(FlinkWinError):
        op3.restore_key_group_heap(a[foreign], IDS)  # a key group this subtask does not own
    with pytest.raises(ValueError):
        op3.restore_key_group_heap(full[1][:-3], IDS)  # truncated
    for x in (op, op2, op3):
        x.close()


def _reference_heap_fixture():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "heap_ds_reduce_event_time_flink2.2.json")) as f:
        fx = json.load(f)
    sid = fx["state_ids"]
    ids = (sid["window-contents"], sid["_timer_state/event_window-timers"], sid["_timer_state/processing_window-timers"])
    return fx, ids, bytes.fromhex(fx["key_groups"][0]["hex"])


def _string_operator(max_p):
    from flink_amd.datastream.heap_state import TupleSerializer
    from flink_amd.datastream.window_operator import WindowOperator
    from flink_amd.datastream.windowing import EventTimeTrigger, TumblingEventTimeWindows
    return WindowOperator(TumblingEventTimeWindows.of(3000), EventTimeTrigger(), ("sum", "INT"), key_type="STRING",
                          max_parallelism=max_p, state_capacity=1 << 12, max_batch_rows=1 << 12,
                          output_capacity=1 << 12, field=1, record_serializer=TupleSerializer.of("STRING", "INT")).open()


@pytest.mark.parametrize("extra", [False, True], ids=["reference_continuation", "plus_new_string_key"])
def test_reference_heap_snapshot_restores_into_gpu_operator(extra):
    """The reference's own heap-backend key group (WindowOperatorMigrationTest.writeReducingEventTimeWindowsSnapshot
    :365-443: String keys, Tuple2<String, Integer> sums, max parallelism 1) restored into the GPU operator
    continues exactly as testRestoreReducingEventTimeWindows (:445-514) asserts: (key1, 3) and (key2, 3) at
    watermark 2999, nothing at 3999 / 4999, (key2, 2) at 5999.  With ``extra`` a new String key's element
    arrives after the restore (routed by String.hashCode like the restored windows) and fires with key2's
    window.  Writing the state back after the first watermark reproduces the reference's remaining entry."""
    from flink_amd.datastream import heap_state as hs
    fx, ids, blob = _reference_heap_fixture()
    op = _string_operator(fx["operator"]["max_parallelism"])
    assert op.restore_key_group_heap(blob, ids) == 0
    if extra:
        op.process_batch(["key3"], np.array([4500], np.int64), np.array([1], np.int64), records=[("key3", 1)])
    for wm, want in fx["continuation"]:
        got = op.process_watermark(wm)
        recs = sorted((r[0], r[1], int(t)) for r, t in zip(got["records"], got["timestamp"]))
        want = sorted(tuple(x) for x in want) + ([("key3", 1, 5999)] if extra and wm == 5999 else [])
        assert recs == sorted(want), f"watermark {wm}"
        assert all(isinstance(k, str) for k in got["key"])
        if wm == 2999 and not extra:  # left: key2's [3000, 6000) with its timer, as the reference holds it
            kser, vser = hs.KEY_SERIALIZERS["STRING"], hs.TupleSerializer.of("STRING", "INT")
            _, contents, timers = hs.read_key_group(op.snapshot_key_group_heap(0, ids), ids, kser, vser)
            assert contents == [("key2", 3000, 6000, ("key2", 2))]
            assert timers == [(5999, "key2", 3000, 6000)]
    assert op.handle.stats()["live_state_entries"] == 0
    assert not op._retained
    op.close()


def test_string_keys_route_by_java_hash_across_subtasks():
    """STRING keys at max parallelism 128 over 3 subtasks: a key group written by one STRING-keyed operator
    restores only into the subtask owning it (computeKeyGroupRangeForOperatorIndex), where the keys' windows
    land by String.hashCode and fire with their sums."""
    from flink_amd.datastream.heap_state import TupleSerializer, java_string_hash
    from flink_amd.datastream.window_operator import WindowOperator
    from flink_amd.datastream.windowing import EventTimeTrigger, TumblingEventTimeWindows
    from flink_amd import _native
    import ctypes as C

    def op(p=1, i=0):
        return WindowOperator(TumblingEventTimeWindows.of(3000), EventTimeTrigger(), ("sum", "INT"), key_type="STRING",
                              parallelism=p, subtask_index=i, state_capacity=1 << 14, max_batch_rows=1 << 14,
                              output_capacity=1 << 14, field=1, record_serializer=TupleSerializer.of("STRING", "INT")).open()
    rng = np.random.default_rng(5)
    names = [f"user-{i}-é" for i in range(300)]
    keys = [names[j] for j in rng.integers(0, len(names), 4000)]
    t3 = 1_599_999_999_000  # a multiple of the 3 s window: one window holds every element
    ts = (t3 + rng.integers(0, 3000, 4000)).astype(np.int64)
    vals = rng.integers(0, 100, 4000).astype(np.int64)
    a = op()
    a.process_batch(keys, ts, vals, records=[(k, int(v)) for k, v in zip(keys, vals)])
    a.process_watermark(t3 - 1)
    kg_of = {}
    for n in set(keys):
        kg_of[n] = _native.lib().fw_host_key_group(abi.KEYHASH_PRECOMPUTED, 0, java_string_hash(n), 128)
    want = {}
    for k, v in zip(keys, vals):
        want[k] = want.get(k, 0) + int(v)
    blobs = {kg: a.snapshot_key_group_heap(kg) for kg in sorted(set(kg_of.values()))}
    got = {}
    for i in range(3):
        b = op(3, i)
        for kg, blob in blobs.items():
            lo, hi = (i * 128 + 2) // 3, ((i + 1) * 128 - 1) // 3
            if lo <= kg <= hi:
                b.restore_key_group_heap(blob)
            else:
                with pytest.raises(Exception):
                    b.restore_key_group_heap(blob)
        r = b.process_watermark(t3 + 2999)
        for rec in r["records"]:
            assert rec[0] not in got
            got[rec[0]] = rec[1]
        b.close()
    a.close()
    assert got == want


@pytest.mark.parametrize("shaped", [True, False], ids=["record_shaped", "key_value"])
def test_string_key_snapshot_restores_into_fresh_operator(shaped):
    """snapshot_state / initialize_state of a STRING-keyed operator: the device blob holds
    interned ids, so the snapshot carries the id -> String table and a fresh operator resumes with the
    same Strings -- a String first seen after the restore gets a new id, not one of the restored ones."""
    from flink_amd.datastream.heap_state import TupleSerializer
    from flink_amd.datastream.window_operator import WindowOperator
    from flink_amd.datastream.windowing import EventTimeTrigger, TumblingEventTimeWindows

    def op():
        kw = dict(field=1, record_serializer=TupleSerializer.of("STRING", "INT")) if shaped else {}
        return WindowOperator(TumblingEventTimeWindows.of(3000), EventTimeTrigger(), ("sum", "INT"), key_type="STRING",
                              state_capacity=1 << 12, max_batch_rows=1 << 12, output_capacity=1 << 12, **kw).open()
    rng = np.random.default_rng(11)
    names = [f"k{i}" for i in range(40)]
    keys = [names[j] for j in rng.integers(0, 40, 500)]
    ts = rng.integers(0, 6000, 500).astype(np.int64)
    vals = rng.integers(0, 50, 500).astype(np.int64)
    recs = lambda ks, vs: [(k, int(v)) for k, v in zip(ks, vs)] if shaped else None
    a = op()
    a.process_batch(keys[:300], ts[:300], vals[:300], records=recs(keys[:300], vals[:300]))
    blob = a.snapshot_state()
    a.close()
    b = op()  # fresh: no Strings interned yet
    b.initialize_state(blob)
    late_keys = keys[300:] + ["new-key"]
    late_ts = np.concatenate([ts[300:], np.array([100], np.int64)])
    late_vals = np.concatenate([vals[300:], np.array([7], np.int64)])
    b.process_batch(late_keys, late_ts, late_vals, records=recs(late_keys, late_vals))
    got = {}
    for wm in (2999, 5999):
        r = b.process_watermark(wm)
        for k, v, t in zip(r["key"], r["value"], r["timestamp"]):
            got[(k, int(t))] = int(np.int32(np.int64(v)))
    want = {}
    for k, t, v in zip(keys + ["new-key"], np.concatenate([ts, [100]]), np.concatenate([vals, [7]])):
        e = (k, (int(t) // 3000) * 3000 + 2999)
        want[e] = want.get(e, 0) + int(v)
    assert got == want
    b.close()


def test_precomputed_hash_round_trip_needs_hashes_refilled():
    """fw_ds_snapshot_key_group reports key_hash 0 for FW_KEYHASH_PRECOMPUTED handles:
    restoring the unmodified array into a fresh handle is refused for a key group that hash 0 does not
    route to; with the keys' hashes filled back in the same array restores and fires the same sums."""
    from flink_amd.datastream.heap_state import java_string_hash
    from flink_amd.datastream.window_operator import WindowOperator
    from flink_amd.datastream.windowing import EventTimeTrigger, TumblingEventTimeWindows
    from flink_amd._native import FlinkWinError
    from flink_amd import _native

    def op():
        return WindowOperator(TumblingEventTimeWindows.of(3000), EventTimeTrigger(), ("sum", "INT"), key_type="STRING",
                              state_capacity=1 << 12, max_batch_rows=1 << 12, output_capacity=1 << 12).open()
    kg0 = _native.lib().fw_host_key_group(abi.KEYHASH_PRECOMPUTED, 0, 0, 128)
    names = [n for n in (f"s{i}" for i in range(400))
             if _native.lib().fw_host_key_group(abi.KEYHASH_PRECOMPUTED, 0, java_string_hash(n), 128) != kg0]
    kg = _native.lib().fw_host_key_group(abi.KEYHASH_PRECOMPUTED, 0, java_string_hash(names[0]), 128)
    keys = [n for n in names if _native.lib().fw_host_key_group(abi.KEYHASH_PRECOMPUTED, 0, java_string_hash(n), 128) == kg]
    a = op()
    a.process_batch(keys * 3, np.array([100, 200, 300] * len(keys), np.int64)[:3 * len(keys)],
                    np.arange(3 * len(keys), dtype=np.int64))
    w = a.handle.ds_key_group_windows(kg)
    assert len(w) == len(keys) and (w["key_hash"] == 0).all()
    b = op()
    with pytest.raises(FlinkWinError):
        b.handle.ds_restore_key_group_windows(kg, w, a.handle.push_seq)
    b.close()
    c = op()
    w2 = w.copy()
    w2["key_hash"] = [java_string_hash(a._kstr[int(k)]) for k in w["key"]]
    c.handle.ds_restore_key_group_windows(kg, w2, a.handle.push_seq)
    c.handle.advance(2999)
    r = c.handle.results(reset=True)
    want = {}
    for i, k in enumerate(keys * 3):
        want[int(a._kid[k])] = want.get(int(a._kid[k]), 0) + i
    assert dict(zip(r["key"].tolist(), [int(np.int32(np.int64(v))) for v in r["values"][0]])) == want
    c.close()
    a.close()
