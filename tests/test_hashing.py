"""Key hashing / key-group assignment: oracle vs an independent pure-Python MurmurHash3_x86_32
(the public algorithm) and the one public known-answer vector.  No reference test pins
MathUtils.murmurHash values, so this is a cross-pin, not a reference pin."""
import struct

import numpy as np
import pytest

from flink_amd import abi
from oracle import oracle as O


def murmur3_x86_32(data: bytes, seed: int) -> int:
    c1, c2 = 0xCC9E2D51, 0x1B873593
    h = seed & 0xFFFFFFFF
    n = len(data) // 4
    for i in range(n):
        k = struct.unpack_from("<I", data, 4 * i)[0]
        k = (k * c1) & 0xFFFFFFFF
        k = ((k << 15) | (k >> 17)) & 0xFFFFFFFF
        k = (k * c2) & 0xFFFFFFFF
        h ^= k
        h = ((h << 13) | (h >> 19)) & 0xFFFFFFFF
        h = (h * 5 + 0xE6546B64) & 0xFFFFFFFF
    assert len(data) % 4 == 0
    h ^= len(data)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def s32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def flink_murmur(code):  # MathUtils.murmurHash = abs(murmur3_32(LE int, seed 0)), MIN -> 0
    h = s32(murmur3_x86_32(struct.pack("<i", s32(code)), 0))
    if h >= 0:
        return h
    return -h if h != -(1 << 31) else 0


def test_public_vector():
    # MurmurHash3_x86_32 of four zero bytes with seed 0 = 0x2362F9DE (public test vector)
    assert murmur3_x86_32(b"\0\0\0\0", 0) == 0x2362F9DE
    assert O.murmur_hash(0) == 0x2362F9DE


def test_murmur_matches_independent_restatement():
    rng = np.random.default_rng(1)
    vals = list(rng.integers(-(1 << 31), 1 << 31, 2000)) + [0, 1, -1, 42, (1 << 31) - 1, -(1 << 31)]
    for v in vals:
        assert O.murmur_hash(int(v)) == flink_murmur(int(v))


@pytest.mark.parametrize("kind", [abi.KEYHASH_BINROW_BIGINT, abi.KEYHASH_BINROW_INT])
def test_binary_row_hash(kind):
    rng = np.random.default_rng(2)
    for k in list(rng.integers(-(1 << 62), 1 << 62, 500)) + [0, 1, -1]:
        k = int(k) if kind == abi.KEYHASH_BINROW_BIGINT else int(np.int32(np.int64(k) & 0x7FFFFFFF))
        if kind == abi.KEYHASH_BINROW_BIGINT:
            row = b"\0" * 8 + struct.pack("<q", k)
        else:
            row = b"\0" * 8 + struct.pack("<i", k) + b"\0" * 4
        want = s32(murmur3_x86_32(row, 42))  # hashBytesByWords seed 42 + fmix(h ^ 16)
        assert O.java_key_hash(kind, k) == want


def test_long_hashcode():
    for k in [0, 1, -1, 1 << 40, -(1 << 40) + 7, (1 << 63) - 1]:
        want = s32((k ^ ((k & 0xFFFFFFFFFFFFFFFF) >> 32)) & 0xFFFFFFFF)
        assert O.java_key_hash(abi.KEYHASH_LONG, k) == want


def test_key_group_ranges_partition_all_groups():
    for max_p in (128, 256, 1000):
        for p in (1, 2, 3, 4, 7, 8):
            seen = []
            for i in range(p):
                s, e = O.key_group_range(max_p, p, i)
                seen.extend(range(s, e + 1))
                for kg in range(s, e + 1):
                    assert O.operator_index(max_p, p, kg) == i
            assert seen == list(range(max_p))


def test_self_computed_key_groups():
    # values recorded in SURVEY.md 8c from a scratch restatement (self-computed, not reference)
    assert [O.key_group(abi.KEYHASH_INT, h, 128) for h in (0, 1, 42, -1)] == [94, 86, 29, 80]


def test_batched_operator_indices_match_scalar():
    """or_operator_indices (the bench's CPU-baseline keyBy) = key_group + operator_index per key."""
    keys = np.random.default_rng(5).integers(-2**63, 2**63 - 1, 2000, dtype=np.int64)
    for kind in (abi.KEYHASH_BINROW_BIGINT, abi.KEYHASH_LONG):
        for p in (1, 3, 16):
            got = O.operator_indices(kind, keys, 128, p)
            want = [O.operator_index(128, p, O.key_group(kind, int(k), 128)) for k in keys]
            assert got.tolist() == want
