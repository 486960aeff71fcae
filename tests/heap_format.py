"""Reader of the heap keyed-state backend's key-group bytes, as the tests check them.

A restatement of the Java writers, independent of the library's C++ (flinkwin.h
fw_snapshot_key_group_heap): HeapSnapshotStrategy.java:161-172 writes writeInt(keyGroup) and per
state writeShort(id) + the state's key-group writer; a ValueState map writes writeInt(n) and n x
(namespace, key, value) (CopyOnWriteStateMapSnapshot.writeState :127-149); a timer queue writes
writeInt(n) and n x TimerSerializer records (flipSignBit(timestamp), key, namespace; :147-152).
Namespaces are LongSerializer (8 B big-endian); keys and accumulators are BinaryRowData
(BinaryRowDataSerializer: writeInt(length) + the bytes -- a null bit set of
((arity + 63 + 8) / 64) * 8 bytes whose first byte is the RowKind and whose bit i + 8 marks field
i NULL, then one little-endian 8-byte slot per fixed-length field, an INT in its low 4 bytes).
No Flink build is available here, so the byte format itself is "parity unpinned": the tests pin
the CONTENTS against the oracle's keyed state and the round trip against continued execution."""
import struct

from flink_amd import abi


def bitset_bytes(arity):
    return ((arity + 63 + 8) // 64) * 8


def acc_field_types(cfg):
    """The accumulator row's field types: COUNT(*) / COUNT: BIGINT; SUM / MIN / MAX: the
    aggregate's type; AVG: (sum BIGINT|DOUBLE, count BIGINT)."""
    out = []
    for g in range(cfg.n_aggs):
        a = cfg.aggs[g]
        if a.kind in (abi.AGG_COUNT_STAR, abi.AGG_COUNT):
            out.append(abi.T_I64)
        elif a.kind == abi.AGG_AVG:
            out += [abi.T_F64 if a.type == abi.T_F64 else abi.T_I64, abi.T_I64]
        else:
            out.append(a.type)
    return out


class _R:
    def __init__(self, b):
        self.b, self.at = b, 0

    def take(self, n):
        if self.at + n > len(self.b):
            raise ValueError("truncated")
        v = self.b[self.at:self.at + n]
        self.at += n
        return v

    def i32(self):
        return struct.unpack(">i", self.take(4))[0]

    def i16(self):
        return struct.unpack(">h", self.take(2))[0]

    def i64(self):
        return struct.unpack(">q", self.take(8))[0]

    def row(self):
        return self.take(self.i32())


def decode_row(raw, types):
    """BinaryRowData of fixed-length fields -> ([signed int64 / DOUBLE bits as int64], null mask)."""
    n = len(types)
    bs = bitset_bytes(n)
    assert len(raw) == bs + 8 * n, "accumulator row length"
    assert raw[0] == 0, "RowKind INSERT"
    vals, nm = [], 0
    for j, t in enumerate(types):
        if raw[(j + 8) // 8] >> ((j + 8) % 8) & 1:
            nm |= 1 << j
            vals.append(0)
            assert raw[bs + 8 * j:bs + 8 * j + 8] == b"\0" * 8, "a NULL field's slot is zeroed"
            continue
        if t == abi.T_I32:
            vals.append(struct.unpack_from("<i", raw, bs + 8 * j)[0])
            assert raw[bs + 8 * j + 4:bs + 8 * j + 8] == b"\0" * 4, "INT high bytes"
        else:
            vals.append(struct.unpack_from("<q", raw, bs + 8 * j)[0])
    return vals, nm


def decode_key(raw, key_hash):
    """A one-field BIGINT / INT key row -> the key; a key row image stays bytes."""
    if key_hash == abi.KEYHASH_KEYROW:
        return bytes(raw)
    assert len(raw) == 16 and raw[:8] == b"\0" * 8, "one-field key row, not NULL"
    if key_hash == abi.KEYHASH_BINROW_INT:
        assert raw[12:16] == b"\0" * 4
        return struct.unpack_from("<i", raw, 8)[0]
    return struct.unpack_from("<q", raw, 8)[0]


def parse_key_group(blob, cfg, ids=(0, 1, 2)):
    """-> (key_group, states [(key, namespace, fields, null_mask)], event timers
    [(timestamp, key, namespace)], number of processing-time timers)."""
    r = _R(blob)
    kg = r.i32()
    types = acc_field_types(cfg)
    states, timers, n_proc = [], [], None
    seen = []
    while r.at < len(blob):
        sid = r.i16()
        seen.append(sid)
        n = r.i32()
        if sid == ids[0]:
            for _ in range(n):
                ns = r.i64()
                key = decode_key(r.row(), cfg.key_hash)
                vals, nm = decode_row(r.row(), types)
                states.append((key, ns, vals, nm))
        elif sid == ids[1]:
            for _ in range(n):
                ts = r.i64() ^ -(1 << 63)  # MathUtils.flipSignBit
                key = decode_key(r.row(), cfg.key_hash)
                timers.append((ts, key, r.i64()))
        elif sid == ids[2]:
            n_proc = n
        else:
            raise ValueError(f"unknown state id {sid}")
    assert seen == sorted(ids), "every state once, in id order"
    return kg, states, timers, n_proc
