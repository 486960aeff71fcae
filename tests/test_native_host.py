"""CPU-side checks of the native library: it loads, exports every symbol include/flinkwin.h
declares, and its host-side restatements (the code the kernels run) agree with the oracle.
No device call is made here."""
import re

import numpy as np
import pytest

from flink_amd import _native, abi
from oracle import oracle as O

HEADER = __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "include", "flinkwin.h")


def test_library_loads_and_exports_header_symbols():
    L = _native.lib()
    text = open(HEADER).read()
    declared = set(re.findall(r"^\s*(?:int|int32_t|int64_t|void\s*\*|const char\s*\*)\s+(fw_\w+)\s*\(", text, re.M))
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert set(_native.EXPORTED) == declared
    assert L.fw_abi_version() == abi.FW_ABI_VERSION


STRUCTS = ["fw_config", "fw_agg_desc", "fw_host_cols", "fw_result", "fw_stats", "fw_late_rows", "fw_ordinal_events",
           "fw_kernel_times", "fw_key_field", "fw_gen_params"]


def test_struct_layouts_match_header(tmp_path):
    """Every ctypes mirror in flink_amd/abi.py has the size and field offsets the C compiler gives
    include/flinkwin.h's struct (what a JNI / FFI binding must reproduce)."""
    import ctypes as C
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "flinkwin.h"', 'int main(void) {']
    for st in STRUCTS:
        lines.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f, _ in getattr(abi, st)._fields_:
            lines.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(root, "include"), "-o", str(exe), str(src)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines())
    for st in STRUCTS:
        cls = getattr(abi, st)
        assert int(got[st]) == C.sizeof(cls), st
        for f, _ in cls._fields_:
            assert int(got[f"{st}.{f}"]) == getattr(cls, f).offset, f"{st}.{f}"


def test_window_start_matches_oracle():
    L = _native.lib()
    rng = np.random.default_rng(7)
    for _ in range(20000):
        size = int(rng.choice([1, 2, 3, 7, 1000, 3600000, 86400000, int(rng.integers(1, 1 << 40))]))
        off = int(rng.integers(-size + 1, size)) if size > 1 else 0
        ts = int(rng.integers(-(1 << 62), 1 << 62))
        assert L.fw_host_window_start(ts, off, size) == O.window_start_with_offset(ts, off, size)
    for ts in (-(1 << 63), (1 << 63) - 1, 0, -1):
        assert L.fw_host_window_start(ts, 0, 1000) == O.window_start_with_offset(ts, 0, 1000)


def test_next_trigger_watermark_matches_oracle():
    L = _native.lib()
    for wm in (-(1 << 63), -1, 0, 999, 1000, 1999, (1 << 63) - 1, 1599998400000):
        for iv in (1, 1000, 2000, 60000):
            assert L.fw_host_next_trigger_watermark(wm, iv) == O.next_trigger_watermark(wm, iv)


@pytest.mark.parametrize("kind", [abi.KEYHASH_LONG, abi.KEYHASH_INT, abi.KEYHASH_BINROW_BIGINT, abi.KEYHASH_BINROW_INT])
def test_key_group_matches_oracle(kind):
    L = _native.lib()
    rng = np.random.default_rng(kind)
    for k in list(rng.integers(-(1 << 63), (1 << 63) - 1, 3000)) + [0, 1, -1]:
        for mp in (128, 1000):
            assert L.fw_host_key_group(kind, int(k), 0, mp) == O.key_group(kind, int(k), mp)


def test_invalid_configs_fail_without_device():
    # argument validation happens before any device call
    from flink_amd.runtime.handle import WindowAggHandle
    with pytest.raises(_native.FlinkWinError, match="Hopping window requires a COUNT"):
        WindowAggHandle(abi.make_config(window_kind=abi.WIN_HOP, size_ms=3000, slide_ms=1000,
                                        aggs=[(abi.AGG_SUM, 0, abi.T_I64)], value_col_types=[abi.T_I64]))
    with pytest.raises(_native.FlinkWinError, match="integral multiple"):
        WindowAggHandle(abi.make_config(window_kind=abi.WIN_CUMULATE, size_ms=3000, slide_ms=700,
                                        aggs=[(abi.AGG_SUM, 0, abi.T_I64)], value_col_types=[abi.T_I64]))


def test_device_count_without_gpu_is_zero_not_an_error():
    # fw_device_count never throws: on a host without a visible HIP device it reports 0, which is
    # what FlinkWin.available() relies on to keep the Java path.
    import torch
    n = _native.lib().fw_device_count()
    assert n >= 0
    if not torch.cuda.is_available():
        assert n == 0


def test_error_flag_bits_match_header():
    text = open(HEADER).read()
    declared = {m[0]: int(m[1]) for m in re.findall(r"#define FW_ERRF_(\w+) (\d+)", text)}
    assert declared == abi.ERRF


def test_delta32_encode_round_trip_and_range_flag():
    """fw_delta32_encode (host helper of fw_commit_delta32): the deltas widen back to the words
    (base + delta, the device kernel's rule), and a value outside [base, base + 2^32) is flagged."""
    L = _native.lib()
    rng = np.random.default_rng(7)
    src = rng.integers(-(1 << 40), 1 << 40, 1001, dtype=np.int64)
    src = (src % (1 << 31)) + 1_599_998_400_000  # event times within 2^31 ms of a base
    base = int(src[0]) - (1 << 31)
    dst = np.zeros(len(src), np.uint32)
    assert L.fw_delta32_encode(src.ctypes.data, len(src), base, dst.ctypes.data) == 0
    assert np.array_equal(dst.astype(np.int64) + base, src)
    # INT64 extremes wrap modulo 2^64 on both sides
    ext = np.array([np.iinfo(np.int64).max, np.iinfo(np.int64).max - 5], np.int64)
    d2 = np.zeros(2, np.uint32)
    assert L.fw_delta32_encode(ext.ctypes.data, 2, int(ext[1]), d2.ctypes.data) == 0
    assert list(d2) == [5, 0]
    bad = src.copy()
    bad[500] = base + (1 << 32)
    assert L.fw_delta32_encode(bad.ctypes.data, len(bad), base, dst.ctypes.data) == 1
    bad[500] = base - 1
    assert L.fw_delta32_encode(bad.ctypes.data, len(bad), base, dst.ctypes.data) == 1
    assert L.fw_delta32_encode(src.ctypes.data, 0, base, dst.ctypes.data) == 0
