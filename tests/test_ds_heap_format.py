"""Host-side checks of the DataStream heap key-group writer/reader (flink_amd/datastream/heap_state.py):
the basic serializers' bytes as the Java writers produce them (LongSerializer / IntSerializer
big-endian, DoubleSerializer doubleToLongBits, StringValue.writeString's variable-length lengths and
UTF-16 code units, TupleSerializer's fields in order), TimerSerializer's flipped timestamps, and a
write -> read round trip of one key group.  Byte parity is pinned by the reference's own heap-backend
snapshot of a WindowOperator (tests/golden/heap_ds_reduce_event_time_flink2.2.json, extracted by
tests/golden/make_heap_golden.py): parsed, and written back byte for byte.""" 
import struct

import numpy as np
import pytest

from flink_amd import abi
from flink_amd.datastream import heap_state as hs
from flink_amd.runtime.handle import DS_WINDOW_DTYPE


def _bytes(ser, v):
    out = hs._Out()
    ser.serialize(v, out)
    return bytes(out.b)


def test_basic_serializers_write_java_bytes():
    assert _bytes(hs.LongSerializer(), -2) == b"\xff" * 7 + b"\xfe"
    assert _bytes(hs.IntSerializer(), 0x01020304) == b"\x01\x02\x03\x04"
    assert _bytes(hs.DoubleSerializer(), 1.0) == struct.pack(">d", 1.0)
    nan_payload = struct.unpack("<d", struct.pack("<Q", 0x7FF00000DEADBEEF))[0]
    assert _bytes(hs.DoubleSerializer(), nan_payload) == bytes.fromhex("7ff8000000000000")  # doubleToLongBits
    assert _bytes(hs.BooleanSerializer(), True) == b"\x01"
    # StringValue.writeString: length + 1 as a 7-bit varint (0 = null), then each UTF-16 unit likewise
    assert _bytes(hs.StringSerializer(), "ab") == b"\x03ab"
    assert _bytes(hs.StringSerializer(), None) == b"\x00"
    assert _bytes(hs.StringSerializer(), "é") == b"\x02\xe9\x01"
    # a supplementary character is two UTF-16 units (0xD83D 0xDE00), each a 3-byte varint
    assert _bytes(hs.StringSerializer(), "\U0001F600") == bytes([0x03, 0xBD, 0xB0, 0x03, 0x80, 0xBC, 0x03])
    long_s = "x" * 200
    assert _bytes(hs.StringSerializer(), long_s)[:2] == bytes([(201 & 0x7F) | 0x80, 201 >> 7])
    for s in ["", "plain", "été", "\U0001F600 emoji", "x" * 300]:
        inp = hs._In(_bytes(hs.StringSerializer(), s))
        assert hs.StringSerializer().deserialize(inp) == s and inp.done()
    t = hs.TupleSerializer.of("LONG", "DOUBLE", "STRING")
    assert _bytes(t, (5, 2.5, "z")) == struct.pack(">q", 5) + struct.pack(">d", 2.5) + b"\x02z"
    with pytest.raises(ValueError):
        _bytes(t, (1, 2.0))


def test_key_group_write_read_round_trip():
    size, late = 3000, 1000

    def cleanup(end):
        return end - 1 + late

    w = np.zeros(4, DS_WINDOW_DTYPE)
    w["key"] = [7, 7, -3, 9]
    w["window_end"] = [3000, 6000, 3000, 9000]
    w["flags"] = [abi.DSW_CONTENTS | abi.DSW_CLEANUP, abi.DSW_CONTENTS | abi.DSW_TRIGGER | abi.DSW_CLEANUP,
                  abi.DSW_CONTENTS | abi.DSW_TRIGGER | abi.DSW_CLEANUP, abi.DSW_TRIGGER]
    recs = [(7, 1.5, "a"), (7, -2.0, "b"), (-3, 0.25, "c"), None]
    ser = hs.TupleSerializer.of("LONG", "DOUBLE", "STRING")
    ids = (5, 1, 2)
    blob = hs.write_key_group(42, ids, w, recs, hs.LongSerializer(), ser, size, cleanup)
    assert blob[:4] == struct.pack(">i", 42) and blob[4:6] == struct.pack(">h", 1)  # states in id order
    kg, contents, timers = hs.read_key_group(blob, ids, hs.LongSerializer(), ser)
    assert kg == 42
    assert sorted(contents) == sorted([(7, 0, 3000, recs[0]), (7, 3000, 6000, recs[1]), (-3, 0, 3000, recs[2])])
    want_t = {(3999, 7, 0, 3000), (5999, 7, 3000, 6000), (6999, 7, 3000, 6000), (2999, -3, 0, 3000),
              (3999, -3, 0, 3000), (8999, 9, 6000, 9000)}
    assert set(timers) == want_t
    # TimerSerializer: writeLong(flipSignBit(ts)) -- a negative timestamp sorts below a positive one bytewise
    out = hs._Out()
    out.u64((-5) ^ (1 << 63))
    assert bytes(out.b)[0] < 0x80
    back, kept = hs.windows_of(contents, timers, size, cleanup, lambda r: struct.unpack("<q", struct.pack("<d", r[1]))[0],
                               11 << 32)
    by = {(int(r["key"]), int(r["window_end"])): r for r in back}
    assert sorted(by) == sorted(zip(w["key"].tolist(), w["window_end"].tolist()))
    for r0 in w:
        r = by[(int(r0["key"]), int(r0["window_end"]))]
        assert int(r["flags"]) == int(r0["flags"])
    assert sorted(kept.values(), key=repr) == sorted([x for x in recs if x], key=repr)
    assert all((o >> 32) == 11 for o in kept)
    with pytest.raises(ValueError):
        hs.read_key_group(blob[:-1], ids, hs.LongSerializer(), ser)
    with pytest.raises(ValueError):
        hs.read_key_group(blob, (6, 1, 2), hs.LongSerializer(), ser)  # unknown state id
    with pytest.raises(ValueError):  # a timer that is neither the trigger nor the cleanup time
        hs.windows_of([], [(1234, 7, 0, 3000)], size, cleanup, lambda r: 0, 0)


def _reference_fixture():
    import json
    import os
    p = os.path.join(os.path.dirname(__file__), "golden", "heap_ds_reduce_event_time_flink2.2.json")
    with open(p) as f:
        fx = json.load(f)
    ids = fx["state_ids"]
    # (window-contents, event-time window-timers, processing-time window-timers)
    order = (ids["window-contents"], ids["_timer_state/event_window-timers"], ids["_timer_state/processing_window-timers"])
    return fx, order, bytes.fromhex(fx["key_groups"][0]["hex"])


def test_reference_heap_snapshot_parses_and_writes_back_byte_for_byte():
    """The reference's own heap-backend bytes (WindowOperatorMigrationTest.java:365-443, extracted by
    tests/golden/make_heap_golden.py): a tumbling 3 s WindowOperator whose ReducingState holds
    Tuple2<String, Integer> sums keyed by the String f0.  read_key_group must find exactly the state the
    writer left after watermark 1999 (elements of WindowOperatorMigrationTest.java:411-418), and writing
    those entries back in the blob's own order must reproduce the reference bytes byte for byte -- the
    StringSerializer keys and records, IntSerializer, TimeWindow.Serializer namespaces, flipped timer
    timestamps and the per-state framing."""
    fx, ids, blob = _reference_fixture()
    kser, vser = hs.KEY_SERIALIZERS["STRING"], hs.TupleSerializer.of("STRING", "INT")
    order = []
    kg, contents, timers = hs.read_key_group(blob, ids, kser, vser, order=order)
    assert kg == fx["key_groups"][0]["key_group"] == 0
    assert sorted(contents) == [("key1", 0, 3000, ("key1", 3)), ("key2", 0, 3000, ("key2", 3)),
                                ("key2", 3000, 6000, ("key2", 2))]
    assert sorted(timers) == [(2999, "key1", 0, 3000), (2999, "key2", 0, 3000), (5999, "key2", 3000, 6000)]
    assert sorted(order) == sorted(ids)
    assert hs.write_key_group_entries(kg, ids, contents, timers, kser, vser, state_order=order) == blob
    # as device windows (String keys interned to ids, routed by String.hashCode), then written back in
    # the library's canonical order (ids ascending, timers sorted): the same state
    names = sorted({k for k, *_ in contents})
    key_id = lambda k: (names.index(k), hs.java_string_hash(k))  # noqa: E731
    w, kept = hs.windows_of(contents, timers, 3000, lambda end: end - 1, lambda r: r[1], 7 << 32, key_id=key_id)
    full = abi.DSW_CONTENTS | abi.DSW_TRIGGER | abi.DSW_CLEANUP  # allowedLateness 0: one timer is both
    assert [(names[int(r["key"])], int(r["window_end"]), int(r["flags"]), int(r["key_hash"])) for r in w] == \
        [("key1", 3000, full, 3288498), ("key2", 3000, full, 3288499), ("key2", 6000, full, 3288499)]
    recs = [kept.get(int(r["first_ord"])) for r in w]
    canon = hs.write_key_group(kg, ids, w, recs, kser, vser, 3000, lambda end: end - 1, key_of=lambda i: names[i])
    assert len(canon) == len(blob)
    kg2, c2, t2 = hs.read_key_group(canon, ids, kser, vser)
    assert (kg2, sorted(c2), sorted(t2)) == (kg, sorted(contents), sorted(timers))


def test_java_string_hash():
    # String.hashCode (JLS 15.8 / java.lang.String): "" -> 0, "a" -> 97, "key1", surrogate pairs as units
    assert hs.java_string_hash("") == 0 and hs.java_string_hash("a") == 97
    assert hs.java_string_hash("key1") == 3288498
    assert hs.java_string_hash("polygenelubricants") == -2147483648  # the classic Integer.MIN_VALUE hash
    assert hs.java_string_hash("\U0001F600") == 0xD83D * 31 + 0xDE00
