"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper around oracle/liboracle.so, the CPU restatement of the reference window
operators (see flinkwin_oracle.cpp for the file:line map).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from flink_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int32
        L.or_create.restype = vp
        L.or_create.argtypes = [C.POINTER(abi.fw_config)]
        L.or_destroy.argtypes = [vp]
        L.or_initialize_watermark.argtypes = [vp, i64]
        L.or_process_batch.restype = i64
        L.or_process_batch.argtypes = [vp, i64, vp, vp, vp, i32, vp]
        L.or_process_watermark.argtypes = [vp, i64]
        L.or_flush.argtypes = [vp]
        L.or_snapshot_restore.argtypes = [vp]
        L.or_num_value_columns.restype = i32
        L.or_num_value_columns.argtypes = [vp]
        for f in ("or_late_dropped", "or_state_size", "or_timer_count", "or_num_results",
                  "or_current_watermark"):
            getattr(L, f).restype = i64
            getattr(L, f).argtypes = [vp]
        L.or_get_results.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.or_state_dump.restype = i64
        L.or_state_dump.argtypes = [vp, vp, vp, vp, vp, i64]
        L.or_ds_state_dump.restype = i64
        L.or_ds_state_dump.argtypes = [vp, vp, vp, vp, vp, i64]
        L.or_timer_dump.restype = i64
        L.or_timer_dump.argtypes = [vp, vp, vp, vp, i64]
        L.or_clear_results.argtypes = [vp]
        L.or_get_first.argtypes = [vp, vp]
        L.or_num_side_rows.restype = i64
        L.or_num_side_rows.argtypes = [vp]
        L.or_take_side_rows.argtypes = [vp, vp, vp, vp, vp, vp]
        L.or_time_op.restype = i64
        L.or_time_op.argtypes = [vp, i32, i64]
        L.or_murmur_hash.restype = i32
        L.or_murmur_hash.argtypes = [i32]
        L.or_java_key_hash.restype = i32
        L.or_java_key_hash.argtypes = [i32, i64, i32]
        L.or_key_row_hash.argtypes = [C.POINTER(abi.fw_key_field), i32, i64, vp]
        L.or_key_row_image.restype = i64
        L.or_key_row_image.argtypes = [C.POINTER(abi.fw_key_field), i32, i64, vp, i64]
        L.or_key_group.restype = i32
        L.or_key_group.argtypes = [i32, i64, i32, i32]
        L.or_operator_index.restype = i32
        L.or_operator_index.argtypes = [i32, i32, i32]
        L.or_key_group_range.argtypes = [i32, i32, i32, C.POINTER(i32), C.POINTER(i32)]
        L.or_operator_indices.argtypes = [i32, vp, i64, i32, i32, i32, vp]
        L.or_window_start_with_offset.restype = i64
        L.or_window_start_with_offset.argtypes = [i64, i64, i64]
        L.or_next_trigger_watermark.restype = i64
        L.or_next_trigger_watermark.argtypes = [i64, i64]
        L.or_generate.argtypes = [C.POINTER(abi.fw_gen_params), vp, i64, i64, vp, vp, vp]
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class OracleOperator:
    """One reference window operator subtask (SQL WindowAggOperator or DataStream
    WindowOperator), driven record-by-record exactly as the reference harness does."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.h = lib().or_create(C.byref(cfg))
        if not self.h:
            raise RuntimeError("oracle create failed")

    def close(self):
        if self.h:
            lib().or_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def initialize_watermark(self, wm):
        lib().or_initialize_watermark(self.h, int(wm))

    def process_batch(self, keys, ts, values, nulls=None):
        """``nulls``: {value column: per-row flags, non-zero = SQL NULL}."""
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        n = len(keys)
        ncols = len(values)
        vals = np.zeros((max(ncols, 1), n), dtype=np.uint64)
        for c, v in enumerate(values):
            v = np.asarray(v)
            vals[c] = v.view(np.uint64) if v.dtype in (np.float64, np.int64, np.uint64) else v.astype(np.int64).view(np.uint64)
        nul = None
        if nulls:
            nul = np.zeros((max(ncols, 1), n), dtype=np.uint8)
            for c, f in nulls.items():
                nul[c] = np.asarray(f).astype(np.uint8) != 0
        return lib().or_process_batch(self.h, n, _ptr(keys), _ptr(ts), _ptr(vals), ncols, _ptr(nul))

    def process_watermark(self, wm):
        lib().or_process_watermark(self.h, int(wm))

    def flush(self):
        lib().or_flush(self.h)

    def snapshot_restore(self):
        lib().or_snapshot_restore(self.h)

    @property
    def late_dropped(self):
        return lib().or_late_dropped(self.h)

    @property
    def state_size(self):
        return lib().or_state_size(self.h)

    def keyed_state(self):
        """(key, namespace, fields[nf], null_mask) of every window state entry, and (timestamp, key,
        namespace) of every event-time timer -- the contents a heap backend would snapshot."""
        L = lib()
        n = L.or_state_dump(self.h, None, None, None, None, 0)
        key, ns = np.zeros(n, np.int64), np.zeros(n, np.int64)
        fields = np.zeros((n, 2 * abi.FW_MAX_AGGS), np.uint64)
        nm = np.zeros(n, np.uint32)
        L.or_state_dump(self.h, _ptr(key), _ptr(ns), _ptr(fields), _ptr(nm), n)
        m = L.or_timer_dump(self.h, None, None, None, 0)
        ts, tk, tn = np.zeros(m, np.int64), np.zeros(m, np.int64), np.zeros(m, np.int64)
        L.or_timer_dump(self.h, _ptr(ts), _ptr(tk), _ptr(tn), m)
        nf = L.or_num_value_columns(self.h) if self.cfg.agg_phase == abi.PHASE_LOCAL else sum(
            2 if self.cfg.aggs[g].kind == abi.AGG_AVG else 1 for g in range(self.cfg.n_aggs))
        states = [(int(key[i]), int(ns[i]), [int(x) for x in fields[i, :nf]], int(nm[i])) for i in range(n)]
        timers = [(int(ts[i]), int(tk[i]), int(tn[i])) for i in range(m)]
        return states, timers

    def ds_keyed_state(self):
        """DataStream: {(key, window end): (value bits, first element ordinal)} of every window state,
        and the (timestamp, key, window end) event-time timers."""
        L = lib()
        n = L.or_ds_state_dump(self.h, None, None, None, None, 0)
        key, end, first = np.zeros(n, np.int64), np.zeros(n, np.int64), np.zeros(n, np.int64)
        val = np.zeros(n, np.uint64)
        L.or_ds_state_dump(self.h, _ptr(key), _ptr(end), _ptr(val), _ptr(first), n)
        states = {(int(key[i]), int(end[i])): (int(val[i].astype(np.int64)), int(first[i])) for i in range(n)}
        _, timers = self.keyed_state()
        return states, timers

    def results(self, clear=True):
        L = lib()
        n = L.or_num_results(self.h)
        na = L.or_num_value_columns(self.h)
        key = np.empty(n, np.int64)
        ws = np.empty(n, np.int64)
        we = np.empty(n, np.int64)
        vals = np.empty((max(na, 1), n), np.uint64)
        nm = np.empty(n, np.uint32)
        ep = np.empty(n, np.int64)
        first = np.empty(n, np.int64)
        if n:
            L.or_get_results(self.h, _ptr(key), _ptr(ws), _ptr(we), _ptr(vals), _ptr(nm), _ptr(ep))
            L.or_get_first(self.h, _ptr(first))
        if clear:
            L.or_clear_results(self.h)
        return {"key": key, "window_start": ws, "window_end": we,
                "values": [vals[a].view(np.int64) for a in range(na)], "null_mask": nm, "epoch": ep,
                "first_ord": first}


    def side_output(self):
        """Late side-output rows since the last call (consumed): key, ts, values, push, row."""
        L = lib()
        n = L.or_num_side_rows(self.h)
        nv = max(self.cfg.n_value_cols, 1)
        key, ts, push, row = (np.empty(n, np.int64) for _ in range(4))
        vals = np.zeros((nv, n), np.uint64)
        if n:
            L.or_take_side_rows(self.h, _ptr(key), _ptr(ts), _ptr(vals), _ptr(push), _ptr(row))
        return {"key": key, "ts": ts, "values": [vals[c].view(np.int64) for c in range(self.cfg.n_value_cols)],
                "push_seq": push, "row": row}

    def time_op(self, what, x):
        return lib().or_time_op(self.h, int(what), int(x))


def murmur_hash(code):
    return lib().or_murmur_hash(int(np.int32(code)))


def java_key_hash(kind, key, pre=0):
    return lib().or_java_key_hash(kind, int(key), int(pre))


def key_row_hash(fields, n_fields, n):
    """BinaryRowData.hashCode of n key rows from host fw_key_field columns (byte-image restatement)."""
    import numpy as np
    out = np.empty(n, dtype=np.int32)
    lib().or_key_row_hash(fields, n_fields, n, out.ctypes.data)
    return out


def key_row_images(fields, n_fields, n):
    """Each key row's BinaryRowWriter image (bytes), the byte-image restatement behind key_row_hash."""
    out = []
    buf = C.create_string_buffer(1 << 16)
    for i in range(n):
        ln = lib().or_key_row_image(fields, n_fields, i, buf, len(buf))
        out.append(buf.raw[:ln])
    return out


def key_group(kind, key, max_p, pre=0):
    return lib().or_key_group(kind, int(key), int(pre), max_p)


def operator_index(max_p, p, kg):
    return lib().or_operator_index(max_p, p, kg)


def operator_indices(kind, keys, max_p, p, pre=0):
    """Subtask of every key at parallelism p (a keyBy's channel selection, vectorised)."""
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    out = np.empty(len(keys), dtype=np.int32)
    lib().or_operator_indices(kind, _ptr(keys), len(keys), int(pre), max_p, p, _ptr(out))
    return out


def key_group_range(max_p, p, idx):
    s, e = C.c_int32(), C.c_int32()
    lib().or_key_group_range(max_p, p, idx, C.byref(s), C.byref(e))
    return s.value, e.value


def window_start_with_offset(ts, off, size):
    return lib().or_window_start_with_offset(int(ts), int(off), int(size))


def next_trigger_watermark(wm, interval):
    return lib().or_next_trigger_watermark(int(wm), int(interval))


def generate(gp, i0, n, zipf_cdf=None):
    key = np.empty(n, np.int64)
    ts = np.empty(n, np.int64)
    val = np.empty(n, np.int64)
    lib().or_generate(C.byref(gp), _ptr(zipf_cdf), int(i0), int(n), _ptr(key), _ptr(ts), _ptr(val))
    return key, ts, val


def zipf_cdf(n, s):
    """Inverse-CDF table for Zipf(s) over n keys."""
    w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return cdf
