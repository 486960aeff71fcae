"""CPU check of tests/heap_format.py, the reader the heap key-group GPU tests parse with: a key
group written by hand from the Java writers' layout (HeapSnapshotStrategy.java:161-172,
CopyOnWriteStateMapSnapshot.writeState :127-149, TimerSerializer.serialize :147-152,
BinaryRowData: null bits of ((arity + 63 + 8) / 64) * 8 bytes, field i NULL at bit i + 8, 8-byte
little-endian slots) reads back field by field."""
import struct

import pytest

from flink_amd import abi
from heap_format import bitset_bytes, decode_row, parse_key_group


def _row(fields, types):
    bs = bitset_bytes(len(fields))
    b = bytearray(bs + 8 * len(fields))
    for j, (v, t) in enumerate(zip(fields, types)):
        if v is None:
            b[(j + 8) // 8] |= 1 << ((j + 8) % 8)
        elif t == abi.T_I32:
            struct.pack_into("<i", b, bs + 8 * j, v)
        else:
            struct.pack_into("<q", b, bs + 8 * j, v)
    return struct.pack(">i", len(b)) + bytes(b)


def _key(k):
    return struct.pack(">i", 16) + b"\0" * 8 + struct.pack("<q", k)


def test_bitset_width_follows_binary_row_data():
    assert [bitset_bytes(n) for n in (1, 56, 57, 120, 121)] == [8, 8, 16, 16, 24]


def test_decode_row_nulls_and_int_fields():
    types = [abi.T_I64, abi.T_I32, abi.T_F64]
    vals, nm = decode_row(_row([7, -5, None], types)[4:], types)
    assert vals == [7, -5, 0] and nm == 0b100


def test_parse_hand_written_key_group():
    cfg = abi.make_config(window_kind=abi.WIN_TUMBLE, size_ms=1000, value_col_types=[abi.T_I32],
                          aggs=[(abi.AGG_COUNT_STAR, 0, abi.T_I64), (abi.AGG_SUM, 0, abi.T_I32),
                                (abi.AGG_AVG, 0, abi.T_I32)], key_hash=abi.KEYHASH_BINROW_BIGINT)
    types = [abi.T_I64, abi.T_I32, abi.T_I64, abi.T_I64]  # count, sum, avg (sum, count)
    ids = (5, 2, 9)
    blob = struct.pack(">i", 17)
    blob += struct.pack(">h", 2) + struct.pack(">i", 1)  # event timers first: ids ascending
    blob += struct.pack(">q", (2999 ^ -(1 << 63))) + _key(-3) + struct.pack(">q", 3000)
    blob += struct.pack(">h", 5) + struct.pack(">i", 2)
    blob += struct.pack(">q", 3000) + _key(-3) + _row([4, None, 10, 4], types)
    blob += struct.pack(">q", 2000) + _key(11) + _row([1, -2, -2, 1], types)
    blob += struct.pack(">h", 9) + struct.pack(">i", 0)
    kg, states, timers, n_proc = parse_key_group(blob, cfg, ids)
    assert kg == 17 and n_proc == 0
    assert states == [(-3, 3000, [4, 0, 10, 4], 0b10), (11, 2000, [1, -2, -2, 1], 0)]
    assert timers == [(2999, -3, 3000)]
    with pytest.raises(AssertionError):  # states out of id order
        parse_key_group(struct.pack(">i", 17) + struct.pack(">h", 9) + struct.pack(">i", 0)
                        + struct.pack(">h", 2) + struct.pack(">i", 0) + struct.pack(">h", 5) + struct.pack(">i", 0), cfg, ids)
