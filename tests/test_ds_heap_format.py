"""Host-side checks of the DataStream heap key-group writer/reader (flink_amd/datastream/heap_state.py):
the basic serializers' bytes as the Java writers produce them (LongSerializer / IntSerializer
big-endian, DoubleSerializer doubleToLongBits, StringValue.writeString's variable-length lengths and
UTF-16 code units, TupleSerializer's fields in order), TimerSerializer's flipped timestamps, and a
write -> read round trip of one key group.  Byte layout restated from the Java writers: parity
unpinned (no Flink build in this image)."""
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
