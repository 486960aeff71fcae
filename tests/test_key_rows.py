"""Key rows for VARCHAR / composite keys: the host RowData -> columnar
encoder and BinaryRowData.hashCode (BinaryRowData.java:459 -> MurmurHashUtils.hashBytesByWords
:70-170) over the row image BinaryRowWriter builds (BinaryRowWriter.java:39-122,
AbstractBinaryWriter.java:83-106,242-348).  The library's streamed hash (fw_host_key_row_hash,
the code the device kernel runs) is checked against the oracle's byte-image restatement, and
single-field rows against the fixed 16-byte key-row hash used for BIGINT / INT keys.  Hash parity
is pinned as DESIGN.md section 2 says: the public Murmur3 vector plus independent restatements."""
import ctypes as C

import numpy as np
import pytest

from flink_amd import abi
from flink_amd._native import lib
from flink_amd.table.key_rows import KeyRowColumns, decode_key_row
from oracle import oracle as O

ALPHABET = "abcxyz0123é漢"


def _rand_str(rng, maxlen):
    return "".join(rng.choice(list(ALPHABET)) for _ in range(int(rng.integers(0, maxlen + 1))))


def _rand_rows(rng, types, n, null_p=0.1):
    rows = []
    for _ in range(n):
        r = []
        for t in types:
            if rng.random() < null_p:
                r.append(None)
            elif abi.KEY_FIELD_KINDS[t] == abi.KF_STRING:
                r.append(_rand_str(rng, 30) if t != "VARBINARY" else bytes(rng.integers(0, 256, rng.integers(0, 20)).astype(np.uint8)))
            elif t == "DOUBLE":
                r.append(float(rng.normal() * 1e6))
            elif t == "FLOAT":
                r.append(float(np.float32(rng.normal())))
            elif t == "BOOLEAN":
                r.append(bool(rng.integers(0, 2)))
            elif t == "TINYINT":
                r.append(int(rng.integers(-128, 128)))
            elif t == "SMALLINT":
                r.append(int(rng.integers(-32768, 32768)))
            elif t in ("INT", "DATE"):
                r.append(int(rng.integers(-2**31, 2**31)))
            else:
                r.append(int(rng.integers(-2**63, 2**63, dtype=np.int64)))
        rows.append(tuple(r))
    return rows


KEY_SHAPES = [("VARCHAR",), ("BIGINT", "VARCHAR"), ("VARCHAR", "INT", "VARCHAR"),
              ("BOOLEAN", "TINYINT", "SMALLINT", "INT", "BIGINT", "DOUBLE", "FLOAT", "DATE"),
              ("VARBINARY", "TIMESTAMP"), ("CHAR", "VARCHAR", "VARCHAR", "VARCHAR", "VARCHAR", "VARCHAR", "VARCHAR", "BIGINT")]


def test_fw_key_field_layout():
    assert C.sizeof(abi.fw_key_field) == 40


@pytest.mark.parametrize("types", KEY_SHAPES, ids=["-".join(t) for t in KEY_SHAPES])
def test_host_key_row_hash_matches_oracle(types):
    rng = np.random.default_rng(len(types) * 7 + len(types[0]))
    rows = _rand_rows(rng, types, 600)
    cols = KeyRowColumns.from_rows(rows, types)
    got = cols.hash_host()
    want = O.key_row_hash(cols.fields(), len(types), len(rows))
    assert np.array_equal(got, want)


def test_string_length_boundaries():
    """0..17-byte strings cross the 7-byte inline / variable-part boundary and the 4- and 8-byte
    word boundaries of the streamed hash."""
    rows = [("x" * n,) for n in range(18)] + [("é" * n, "ab" * n) for n in range(9)]
    for shape in (("VARCHAR",), ("VARCHAR", "VARCHAR")):
        sel = [r for r in rows if len(r) == len(shape)]
        cols = KeyRowColumns.from_rows(sel, shape)
        assert np.array_equal(cols.hash_host(), O.key_row_hash(cols.fields(), len(shape), len(sel)))


def test_single_fixed_field_equals_binrow_key_hash():
    """A one-field BIGINT / INT key row is the 16-byte row FW_KEYHASH_BINROW_* hashes."""
    rng = np.random.default_rng(3)
    ks = [0, -1, 1, 2**63 - 1, -2**63] + [int(x) for x in rng.integers(-2**63, 2**63, 200, dtype=np.int64)]
    cols = KeyRowColumns.from_rows([(k,) for k in ks], ("BIGINT",))
    want = [O.java_key_hash(abi.KEYHASH_BINROW_BIGINT, k) for k in ks]
    assert cols.hash_host().tolist() == want
    ki = [int(x) for x in rng.integers(-2**31, 2**31, 200)]
    cols = KeyRowColumns.from_rows([(k,) for k in ki], ("INT",))
    assert cols.hash_host().tolist() == [O.java_key_hash(abi.KEYHASH_BINROW_INT, k) for k in ki]


def test_null_field_row_differs_from_empty_string():
    cols = KeyRowColumns.from_rows([(None,), ("",)], ("VARCHAR",))
    h = cols.hash_host()
    assert h[0] != h[1]
    assert np.array_equal(h, O.key_row_hash(cols.fields(), 1, 2))


def test_invalid_key_field_descriptions_rejected():
    L = lib()
    cols = KeyRowColumns.from_rows([("a",)], ("VARCHAR",))
    f = cols.fields()
    out = np.empty(1, dtype=np.int32)
    assert L.fw_host_key_row_hash(f, 0, 1, out.ctypes.data) == abi.FW_E_INVALID
    assert L.fw_host_key_row_hash(f, abi.FW_MAX_KEY_FIELDS + 1, 1, out.ctypes.data) == abi.FW_E_INVALID
    f[0].kind = 3
    assert L.fw_host_key_row_hash(f, 1, 1, out.ctypes.data) == abi.FW_E_INVALID
    f[0].kind = abi.KF_FIXED8  # no fixed column
    assert L.fw_host_key_row_hash(f, 1, 1, out.ctypes.data) == abi.FW_E_INVALID


@pytest.mark.parametrize("types", KEY_SHAPES, ids=["-".join(t) for t in KEY_SHAPES])
def test_key_row_images_match_oracle_and_round_trip(types):
    """The library's BinaryRowWriter images (fw_host_key_row_images, the code k_kr_images runs) are
    byte-identical to the oracle's, hash (fw_host_key_row_image_hash, what k_kr_intern runs) like
    the columnar hash, and decode back to the rows (BinaryRowData getters)."""
    rng = np.random.default_rng(31 + len(types))
    rows = _rand_rows(rng, types, 400)
    cols = KeyRowColumns.from_rows(rows, types)
    off, img = cols.images_host()
    want = O.key_row_images(cols.fields(), len(types), len(rows))
    got = [img[off[i]:off[i + 1]].tobytes() for i in range(len(rows))]
    assert got == want
    L = lib()
    h = [L.fw_host_key_row_image_hash(np.frombuffer(g, np.uint64).ctypes.data, len(g)) for g in got]
    assert h == cols.hash_host().tolist()
    for r, g in zip(rows, got):
        d = decode_key_row(g, types)
        for t, x, y in zip(types, r, d):
            if t == "FLOAT" and x is not None:
                assert np.float32(x) == np.float32(y)
            elif t == "BOOLEAN" and x is not None:
                assert bool(x) == y
            else:
                assert x == y, (types, r, d)


def test_key_row_identity_is_the_image_bytes():
    """BinaryRowData.equals compares bytes: -0.0 and 0.0 are different DOUBLE keys, equal strings
    are one key whatever Python object carried them, and NULL differs from the empty string."""
    cols = KeyRowColumns.from_rows([(0.0,), (-0.0,), (0.0,)], ("DOUBLE",))
    off, img = cols.images_host()
    g = [img[off[i]:off[i + 1]].tobytes() for i in range(3)]
    assert g[0] == g[2] and g[0] != g[1]
    cols = KeyRowColumns.from_rows([("ab",), (b"ab",), (None,), ("",)], ("VARBINARY",))
    off, img = cols.images_host()
    g = [img[off[i]:off[i + 1]].tobytes() for i in range(4)]
    assert g[0] == g[1] and g[2] != g[3]


def test_host_partition_routes_precomputed_hash_like_oracle():
    import torch
    from flink_amd.runtime.exchange import KeyByExchange
    rng = np.random.default_rng(11)
    rows = _rand_rows(rng, ("VARCHAR", "BIGINT"), 500, null_p=0.05)
    cols = KeyRowColumns.from_rows(rows, ("VARCHAR", "BIGINT"))
    h = cols.hash_host()
    ex = KeyByExchange(abi.KEYHASH_PRECOMPUTED, 128)
    ex.world = 4  # routing only (no collective): 4 destinations
    key = torch.arange(len(rows), dtype=torch.int64)
    pk, pt, pv, counts = ex.partition(key, key.clone(), [], key_hash=torch.from_numpy(h))
    dest = [O.operator_index(128, 4, O.key_group(abi.KEYHASH_PRECOMPUTED, 0, 128, pre=int(x))) for x in h]
    assert counts.tolist() == np.bincount(dest, minlength=4).tolist()
    assert pk.tolist() == sorted(range(len(rows)), key=lambda i: dest[i])
    with pytest.raises(ValueError):
        ex.partition(key, key.clone(), [])


def test_eligibility_of_key_rows():
    from flink_amd.table.slice_assigners import SliceAssigners
    from flink_amd.table.window_agg import is_gpu_eligible
    a = SliceAssigners.tumbling(2, 1000)
    aggs = [("COUNT_STAR", 0, "BIGINT")]
    assert is_gpu_eligible(a, aggs, ["BIGINT"], key_type=("VARCHAR", "BIGINT"))[0]
    ok, why = is_gpu_eligible(a, aggs, ["BIGINT"], key_type=("VARCHAR", "DECIMAL"))
    assert not ok and "DECIMAL" in why
    assert not is_gpu_eligible(a, aggs, ["BIGINT"], key_type=("VARCHAR",) * 9)[0]
