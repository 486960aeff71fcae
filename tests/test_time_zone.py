"""TIMESTAMP_LTZ shift time zones (TimeWindowUtil.java:52-211) on the host: the library's plan +
arithmetic (fw_host_time_op, the code the kernels run) and the oracle's restatement against the
reference's DST known answers (*SliceAssignerTest.testDstSaving, America/Los_Angeles) and against
each other on random instants across zone transitions.  No device use."""
import ctypes as C

import numpy as np
import pytest

from fixture_runner import load_kats
from flink_amd import _native, abi
from flink_amd.table.time_zone import ShiftZone
from oracle.oracle import OracleOperator

DST_KATS = [k for k in load_kats() if k["op"] == "dst_slice"]


def _cfg(kind, size, slide, zone):
    return abi.make_config(window_kind=abi.WINDOW_NAMES[kind], size_ms=size, slide_ms=slide,
                           aggs=[(abi.AGG_COUNT_STAR, 0, abi.T_I64)], count_star_index=0, shift_zone=zone)


def _lib_op(cfg, what, x):
    out = C.c_int64()
    _native.check(_native.lib().fw_host_time_op(C.byref(cfg), what, int(x), C.byref(out)))
    return out.value


def test_zone_tables():
    la, sh = ShiftZone.of("America/Los_Angeles"), ShiftZone.of("Asia/Shanghai")
    assert la.use_dst and not sh.use_dst
    assert la.offset_at(1615716000000) == -7 * 3600000 and la.offset_at(1615712400000) == -8 * 3600000
    assert sh.offset_at(0) == 8 * 3600000


@pytest.mark.parametrize("kat", DST_KATS, ids=[k["src"].split("/")[-1] for k in DST_KATS])
def test_dst_slice_known_answers(kat):
    kind, size, slide, _ = kat["assigner"]
    cfg = _cfg(kind, size, slide, kat["zone"])
    orc = OracleOperator(cfg)
    for epoch, (start, end) in kat["cases"]:
        se = _lib_op(cfg, 3, epoch)
        assert (se, _lib_op(cfg, 4, se)) == (end, start), epoch
        assert (orc.time_op(3, epoch), orc.time_op(4, end)) == (end, start), epoch


@pytest.mark.parametrize("zone", ["America/Los_Angeles", "Europe/Berlin", "Asia/Shanghai", "Australia/Lord_Howe"])
def test_library_matches_oracle_across_transitions(zone):
    """toUtcTimestampMills / toEpochMillsForTimer / getNextTriggerWatermark / slice ends of the
    library against the oracle's ZoneRules restatement, densely around every transition of
    2015-2030 (Lord Howe shifts by 30 minutes)."""
    z = ShiftZone.of(zone)
    cfg = _cfg("HOP", 4 * 3600000, 1800000, zone)
    orc = OracleOperator(cfg)
    rng = np.random.default_rng(5)
    trans = [u for u in z.utc[1:] if 1420070400000 <= u <= 1893456000000] or [1600000000000]
    for t in trans:
        for d in list(rng.integers(-3 * 3600000, 3 * 3600000, 60)) + [-1, 0, 1, 3599999, 3600000, -3600000]:
            x = int(t + d)
            for what in (0, 1, 2, 3):
                assert _lib_op(cfg, what, x) == orc.time_op(what, x), (zone, what, x)


def test_utc_zone_is_identity():
    cfg = _cfg("TUMBLE", 3600000, 0, None)
    for x in (-5, 0, 1615716000000, (1 << 63) - 1):
        assert _lib_op(cfg, 0, x) == x and _lib_op(cfg, 1, x) == x
