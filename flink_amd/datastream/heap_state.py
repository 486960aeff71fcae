"""The DataStream WindowOperator's keyed state in the heap keyed-state backend's key-group bytes.

A heap-backend savepoint writes, per key group (HeapSnapshotStrategy.java:161-172): writeInt(keyGroup),
then per registered state in id order writeShort(stateId) and that state's key-group data:

  "window-contents"  the window's ReducingState (WindowOperatorBuilder.java:81), written by
                     CopyOnWriteStateMapSnapshot.writeState (:127-149): writeInt(n), then per entry
                     namespace (TimeWindow.Serializer: writeLong(start), writeLong(end),
                     TimeWindow.java:159-162), key (the key serializer), value (the record type's
                     serializer: value1 -- the window's first element -- with the aggregated field set,
                     SumAggregator.java:66-76 / ComparableAggregator.java:83-104)
  "window-timers"    the event-time and processing-time timer queues of the operator's timer service
                     (WindowOperator.java:232; InternalTimerServiceImpl.snapshotTimersForKeyGroup :360):
                     writeInt(n), then per timer TimerSerializer.serialize (:147-152):
                     writeLong(flipSignBit(timestamp)), key, namespace

The device side (flinkwin.h fw_ds_snapshot_key_group / fw_ds_restore_key_group) moves one record per
(key, window): its field value, its first element's arrival ordinal and which timers it holds; the
operator shim keeps the first elements themselves (window_operator.py), so the bytes are assembled
here.  Byte parity is pinned by the reference's own heap-backend snapshot of this operator
(WindowOperatorMigrationTest.java:365-443, String keys, Tuple2<String, Integer> records;
tests/golden/heap_ds_reduce_event_time_flink2.2.json): parsed, then written back byte for byte
(tests/test_ds_heap_format.py), and restored into the GPU operator, which continues with the
reference test's own expected records (tests/test_gpu_ds_heap_key_group.py).
"""
import struct

import numpy as np

from .. import abi
from ..runtime.handle import DS_WINDOW_DTYPE

_FLIP = 1 << 63


class _Out:
    def __init__(self):
        self.b = bytearray()

    def i16(self, v):
        self.b += struct.pack(">h", v)

    def i32(self, v):
        self.b += struct.pack(">i", v)

    def i64(self, v):
        self.b += struct.pack(">q", v)

    def u64(self, v):
        self.b += struct.pack(">Q", v & 0xFFFFFFFFFFFFFFFF)

    def raw(self, x):
        self.b += x


class _In:
    def __init__(self, b):
        self.b, self.at = memoryview(b), 0

    def take(self, n):
        if self.at + n > len(self.b):
            raise ValueError("heap key-group data truncated")
        x = self.b[self.at:self.at + n]
        self.at += n
        return bytes(x)

    def i16(self):
        return struct.unpack(">h", self.take(2))[0]

    def i32(self):
        return struct.unpack(">i", self.take(4))[0]

    def i64(self):
        return struct.unpack(">q", self.take(8))[0]

    def u64(self):
        return struct.unpack(">Q", self.take(8))[0]

    def done(self):
        return self.at >= len(self.b)


# ---- serializers of the basic types (flink-core typeutils.base) --------------------------------
class LongSerializer:        # LongSerializer.serialize: writeLong
    def serialize(self, v, out):
        out.i64(int(v))

    def deserialize(self, inp):
        return inp.i64()


class IntSerializer:         # IntSerializer.serialize: writeInt
    def serialize(self, v, out):
        out.i32(int(v))

    def deserialize(self, inp):
        return inp.i32()


class DoubleSerializer:      # DoubleSerializer -> DataOutputSerializer.writeDouble: doubleToLongBits
    def serialize(self, v, out):
        d = float(v)
        out.raw(struct.pack(">d", float("nan")) if d != d else struct.pack(">d", d))

    def deserialize(self, inp):
        return struct.unpack(">d", inp.take(8))[0]


class BooleanSerializer:     # BooleanSerializer.serialize: writeBoolean
    def serialize(self, v, out):
        out.raw(b"\x01" if v else b"\x00")

    def deserialize(self, inp):
        return inp.take(1) != b"\x00"


def _varint(out, x):
    while x >= 0x80:
        out.raw(bytes([(x & 0x7F) | 0x80]))
        x >>= 7
    out.raw(bytes([x]))


def _read_varint(inp):
    x, shift = 0, 0
    while True:
        c = inp.take(1)[0]
        x |= (c & 0x7F) << shift
        if c < 0x80:
            return x
        shift += 7


class StringSerializer:      # StringSerializer -> StringValue.writeString (StringValue.java:799-860)
    def serialize(self, v, out):
        if v is None:
            out.raw(b"\x00")
            return
        units = np.frombuffer(str(v).encode("utf-16-le"), np.uint16)  # Java chars: UTF-16 code units
        _varint(out, len(units) + 1)  # 0 marks null
        for c in units.tolist():
            _varint(out, c)

    def deserialize(self, inp):
        n = _read_varint(inp)
        if n == 0:
            return None
        units = np.array([_read_varint(inp) for _ in range(n - 1)], np.uint16)
        return units.tobytes().decode("utf-16-le")


class TupleSerializer:       # TupleSerializer.serialize (:135-144): the fields in order, no null flags
    def __init__(self, fields):
        self.fields = list(fields)

    def serialize(self, v, out):
        if len(v) != len(self.fields):
            raise ValueError(f"record arity {len(v)} != {len(self.fields)}")
        for f, x in zip(self.fields, v):
            f.serialize(x, out)

    def deserialize(self, inp):
        return tuple(f.deserialize(inp) for f in self.fields)

    @staticmethod
    def of(*types):
        """TupleSerializer.of("LONG", "DOUBLE", "STRING", ...)"""
        m = {"LONG": LongSerializer, "INT": IntSerializer, "DOUBLE": DoubleSerializer, "STRING": StringSerializer,
             "BOOLEAN": BooleanSerializer}
        return TupleSerializer([m[t]() for t in types])


# StringSerializer keys: WindowedStream over keyBy(String field), e.g. the reference's own
# WindowOperatorMigrationTest (Tuple2<String, Integer> keyed by f0)
KEY_SERIALIZERS = {"LONG": LongSerializer(), "INT": IntSerializer(), "STRING": StringSerializer()}


def java_string_hash(s):
    """String.hashCode (JLS): s[0]*31^(n-1) + ... + s[n-1] over the UTF-16 code units, int32 wrap"""
    h = 0
    for u in np.frombuffer(str(s).encode("utf-16-le"), np.uint16).tolist():
        h = (31 * h + u) & 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


# ---- key-group bytes ----------------------------------------------------------------------------
def write_key_group_entries(kg, ids, contents, timers, key_ser, value_ser, state_order=None):
    """The key group's bytes from explicit entry lists, written in list order: contents [(key, start,
    end, record)] and event timers [(ts, key, start, end)].  The reference writes its states in the
    iteration order of a HashMap over StateUID (HeapSnapshotStrategy.java:161-172: the order varies with
    the JVM's enum identity hashes), the window-contents entries in CopyOnWriteStateMap bucket order and
    the timers in heap-array order; none of those orders carries meaning (the restore reads any), so
    ``state_order`` (default: id order) and the list orders are the caller's choice."""
    out = _Out()
    out.i32(kg)
    for sid in (state_order if state_order is not None else sorted(ids)):
        out.i16(sid)
        if sid == ids[0]:
            out.i32(len(contents))
            for key, start, end, rec in contents:
                out.i64(start)
                out.i64(end)
                key_ser.serialize(key, out)
                value_ser.serialize(rec, out)
        elif sid == ids[1]:
            out.i32(len(timers))
            for ts, key, start, end in timers:
                out.u64(ts ^ _FLIP)  # MathUtils.flipSignBit
                key_ser.serialize(key, out)
                out.i64(start)
                out.i64(end)
        elif sid == ids[2]:
            out.i32(0)  # event-time windows register no processing-time timers
        else:
            raise ValueError(f"state id {sid} is not one of {ids}")
    return bytes(out.b)


def write_key_group(kg, ids, windows, records, key_ser, value_ser, size, cleanup_time, key_of=None):
    """windows: DS_WINDOW_DTYPE rows; records[i]: the state value (record) of windows[i] when it holds
    contents.  ids = (window-contents, event window-timers, processing window-timers) state ids.
    key_of: the key object of a device key (a String key's interned id -> the String; default int)."""
    key_of = key_of or int
    contents = [(key_of(int(w["key"])), int(w["window_end"]) - size, int(w["window_end"]), r)
                for w, r in zip(windows, records) if int(w["flags"]) & abi.DSW_CONTENTS]
    timers = set()
    for w in windows:
        key, end, fl = key_of(int(w["key"])), int(w["window_end"]), int(w["flags"])
        if fl & abi.DSW_TRIGGER:
            timers.add((end - 1, key, end - size, end))
        if fl & abi.DSW_CLEANUP:
            timers.add((cleanup_time(end), key, end - size, end))
    return write_key_group_entries(kg, ids, contents, sorted(timers), key_ser, value_ser)


def read_key_group(blob, ids, key_ser, value_ser, order=None):
    """-> (key_group, contents [(key, start, end, record)], event timers [(ts, key, start, end)]), each
    in the blob's order; ``order`` (a list) receives the state ids in the order the blob holds them"""
    inp = _In(blob)
    kg = inp.i32()
    contents, timers, seen = [], [], set()
    while not inp.done():
        sid = inp.i16()
        n = inp.i32()
        if sid in seen or sid not in ids:
            raise ValueError(f"unexpected state id {sid} in key group {kg}")
        seen.add(sid)
        if order is not None:
            order.append(sid)
        for _ in range(n):
            if sid == ids[0]:
                st, end = inp.i64(), inp.i64()
                key = key_ser.deserialize(inp)
                contents.append((key, st, end, value_ser.deserialize(inp)))
            elif sid == ids[1]:
                ts = inp.u64() ^ _FLIP
                ts = ts - (1 << 64) if ts >= 1 << 63 else ts
                key = key_ser.deserialize(inp)
                st, end = inp.i64(), inp.i64()
                timers.append((ts, key, st, end))
            else:
                raise ValueError("processing-time timers in an event-time window operator")
    return kg, contents, timers


def windows_of(contents, timers, size, cleanup_time, field_bits, first_ord0, key_id=None):
    """heap contents + timers -> DS_WINDOW_DTYPE rows (first elements numbered from first_ord0) and
    the records they retain.  key_id: key object -> (device key, key hash) for keys the device does not
    hash itself (a String key: its interned id and String.hashCode); default: the key is the device key."""
    rows = {}
    for key, st, end, rec in contents:
        if end - st != size:
            raise ValueError(f"namespace [{st}, {end}) is not a window of size {size}")
        if (key, end) in rows:
            raise ValueError(f"duplicate window-contents entry ({key}, [{st}, {end}))")
        rows[(key, end)] = [abi.DSW_CONTENTS, rec]
    for ts, key, st, end in timers:
        if end - st != size:
            raise ValueError(f"timer namespace [{st}, {end}) is not a window of size {size}")
        ent = rows.setdefault((key, end), [0, None])
        if ts == end - 1:
            ent[0] |= abi.DSW_TRIGGER
        if ts == cleanup_time(end):
            ent[0] |= abi.DSW_CLEANUP
        if ts != end - 1 and ts != cleanup_time(end):
            raise ValueError(f"timer {ts} is neither window [{st}, {end})'s trigger nor its cleanup time")
    out = np.zeros(len(rows), DS_WINDOW_DTYPE)
    kept = {}
    for i, ((key, end), (fl, rec)) in enumerate(sorted(rows.items(), key=lambda kv: kv[0])):
        dk, kh = key_id(key) if key_id is not None else (key, 0)
        out[i]["key"], out[i]["key_hash"], out[i]["window_end"], out[i]["flags"] = dk, kh, end, fl
        out[i]["first_ord"] = -1
        if rec is not None:
            o = first_ord0 + len(kept)
            out[i]["value"] = field_bits(rec)
            out[i]["first_ord"] = o
            kept[o] = rec
    return out, kept
