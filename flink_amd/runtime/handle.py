"""Python wrapper of one libflinkwin operator handle (one Flink operator subtask).

The handle is single-threaded like Flink's mailbox thread (MailboxProcessor.java:58-91).
"""
import ctypes as C

import numpy as np

from .. import abi
from .._native import check, lib

# fw_ds_window (flinkwin.h), one (key, window) of a DataStream key group
DS_WINDOW_DTYPE = np.dtype([("key", np.int64), ("window_end", np.int64), ("value", np.int64),
                            ("first_ord", np.int64), ("flags", np.int32), ("key_hash", np.int32)])


def _np_view(ptr, n, dtype):
    if n == 0:
        return np.empty(0, dtype)
    ct = {np.int64: C.c_int64, np.int32: C.c_int32, np.uint32: C.c_uint32, np.uint64: C.c_uint64, np.uint8: C.c_uint8}[dtype]
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(n,))


class WindowAggHandle:
    def __init__(self, cfg: abi.fw_config):
        self.cfg = cfg
        self._h = C.c_void_p()
        check(lib().fw_create(C.byref(cfg), C.byref(self._h)))
        self.n_aggs = abi.result_columns(cfg)  # result value columns
        self.push_seq = 0  # fw_commit / fw_push_device* calls so far (arrival ordinals: push_seq << 32 | row)
        self._ext = None  # torch view of the handle's stream + two reusable ordering events

    # ---- stream ordering of device-resident inputs: the handle's stream waits for the producer's
    # current stream before the ingest reads the columns, and the producer's later work waits for
    # the ingest (no record_stream: the handle's stream dies with the handle, before torch frees the
    # tensors).  The stream view and events are created once per handle: a push is on the per-step
    # hot path, where creating them every time costs more host time than the launch itself.
    def _begin_read(self, device):
        import torch
        if self._ext is None or self._ext[0] != device:
            self._ext = (device, torch.cuda.ExternalStream(self.stream_ptr, device=device),
                         torch.cuda.Event(), torch.cuda.Event())
        cur = torch.cuda.current_stream(device)
        self._ext[2].record(cur)
        self._ext[1].wait_event(self._ext[2])
        return cur

    def _end_read(self, cur):
        self._ext[3].record(self._ext[1])
        cur.wait_event(self._ext[3])

    # ---- lifecycle
    def close(self):
        self._ext = None
        if self._h:
            lib().fw_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream_ptr(self):
        return lib().fw_get_stream(self._h)

    def sync(self):
        check(lib().fw_sync(self._h))

    def initialize_watermark(self, wm):
        check(lib().fw_initialize_watermark(self._h, int(wm)))

    # ---- ingest
    def push_host(self, keys, ts, values=(), key_hashes=None, nulls=None, delta32=True):
        """Host columns -> pinned staging -> device (fw_reserve / fw_commit).  ``nulls`` maps a
        nullable value column to its per-row null flags (bool / uint8, non-zero = SQL NULL).
        ``delta32``: a column whose batch values span < 2^32 crosses PCIe as 32-bit deltas from its
        minimum (fw_commit_delta32, as the JNI shim packs event times and bounded ids); the device
        sees the same 8-byte words either way."""
        keys = np.asarray(keys, dtype=np.int64)
        n = len(keys)
        cap = self.cfg.max_batch_rows
        for o in range(0, n, cap):
            m = min(cap, n - o)
            cols = abi.fw_host_cols()
            check(lib().fw_reserve(self._h, m, C.byref(cols)))
            mask, bases = 0, (C.c_int64 * (2 + abi.FW_MAX_COLS))()

            def put(slot, ptr, col):
                nonlocal mask
                if delta32:
                    lo, hi = int(col.min()), int(col.max())
                    if hi - lo < (1 << 32):
                        np.subtract(col, np.int64(lo), out=_np_view(ptr, m, np.uint32), casting="unsafe")
                        mask |= 1 << slot
                        bases[slot] = lo
                        return
                _np_view(ptr, m, np.int64)[:] = col
            if m:
                put(0, cols.key, keys[o:o + m])
                put(1, cols.ts, np.asarray(ts, dtype=np.int64)[o:o + m])
                if key_hashes is not None:
                    _np_view(cols.key_hash, m, np.int32)[:] = np.asarray(key_hashes, dtype=np.int32)[o:o + m]
                for c, v in enumerate(values):
                    v = np.asarray(v)
                    if v.dtype == np.float64:
                        v = v.view(np.int64)
                    put(2 + c, cols.values[c], v.astype(np.int64, copy=False)[o:o + m])
                for c in range(self.cfg.n_value_cols):
                    if self.cfg.nullable_cols >> c & 1:
                        nf = np.zeros(n, np.uint8) if nulls is None or c not in nulls else \
                            np.asarray(nulls[c]).astype(np.uint8, copy=False)
                        _np_view(cols.nulls[c], m, np.uint8)[:] = nf[o:o + m]
            if mask:
                check(lib().fw_commit_delta32(self._h, m, mask, bases))
            else:
                check(lib().fw_commit(self._h, m))
            self.push_seq += 1

    def push_host_key_rows(self, offsets, images, ts, values=(), nulls=None):
        """FW_KEYHASH_KEYROW: host key-row images (row i = images[offsets[i]:offsets[i + 1]], the
        key's BinaryRowData bytes) through the pinned staging of fw_reserve / fw_commit -- the path
        the JNI shim takes."""
        offsets = np.asarray(offsets, dtype=np.int64)
        images = np.asarray(images, dtype=np.uint8)
        n = len(offsets) - 1
        cap = self.cfg.max_batch_rows
        for o in range(0, n, cap):
            m = min(cap, n - o)
            cols = abi.fw_host_cols()
            check(lib().fw_reserve(self._h, m, C.byref(cols)))
            if m:
                off = offsets[o:o + m + 1] - offsets[o]
                if off[-1] > cols.key_row_bytes_cap:
                    raise ValueError("key rows exceed the staging bytes (key_row_max_bytes per row)")
                _np_view(cols.key_row_offsets, m + 1, np.int64)[:] = off
                _np_view(cols.key_row_bytes, int(off[-1]), np.uint8)[:] = images[offsets[o]:offsets[o + m]]
                _np_view(cols.ts, m, np.int64)[:] = np.asarray(ts, dtype=np.int64)[o:o + m]
                for c, v in enumerate(values):
                    v = np.asarray(v)
                    if v.dtype == np.float64:
                        v = v.view(np.int64)
                    _np_view(cols.values[c], m, np.int64)[:] = v.astype(np.int64, copy=False)[o:o + m]
                for c in range(self.cfg.n_value_cols):
                    if self.cfg.nullable_cols >> c & 1:
                        nf = np.zeros(n, np.uint8) if nulls is None or c not in nulls else \
                            np.asarray(nulls[c]).astype(np.uint8, copy=False)
                        _np_view(cols.nulls[c], m, np.uint8)[:] = nf[o:o + m]
            check(lib().fw_commit(self._h, m))
            self.push_seq += 1

    def push_device_key_rows(self, offsets, images, ts, values=(), nulls=None):
        """FW_KEYHASH_KEYROW: device-resident key-row images (int64 offsets tensor of n + 1, uint8
        bytes tensor, 8-byte aligned rows)."""
        n = ts.numel()
        if n == 0:
            return
        cur = self._begin_read(ts.device)
        arr = (C.c_void_p * abi.FW_MAX_COLS)()
        for c, v in enumerate(values):
            arr[c] = v.data_ptr()
        nul = (C.c_void_p * abi.FW_MAX_COLS)()
        for c, v in (nulls or {}).items():
            nul[c] = v.data_ptr()
        check(lib().fw_push_device_key_rows(self._h, n, offsets.data_ptr(), images.data_ptr(), ts.data_ptr(), arr, nul))
        self.push_seq += 1
        self._end_read(cur)

    def push_device(self, keys, ts, values=(), key_hashes=None, nulls=None, producer_synced=False):
        """Device-resident columns (torch cuda tensors, int64 / float64; ``nulls``: {column:
        uint8 tensor}).  The handle's stream waits for the producer's current stream before
        reading them -- unless ``producer_synced``: the caller guarantees the columns are complete
        (synchronised) and stay unmodified until the handle has read them (the C-ABI contract of
        fw_push_device, as a JNI shim calls it), and no stream events are recorded."""
        n = keys.numel()
        if n == 0:
            return
        if producer_synced:
            arr = (C.c_void_p * abi.FW_MAX_COLS)(*[v.data_ptr() for v in values])
            nul = (C.c_void_p * abi.FW_MAX_COLS)()
            for c, v in (nulls or {}).items():
                nul[c] = v.data_ptr()
            check(lib().fw_push_device(self._h, n, keys.data_ptr(), ts.data_ptr(),
                                       key_hashes.data_ptr() if key_hashes is not None else None, arr, nul))
            self.push_seq += 1
            return
        cur = self._begin_read(keys.device)
        arr = (C.c_void_p * abi.FW_MAX_COLS)()
        for c, v in enumerate(values):
            arr[c] = v.data_ptr()
        nul = (C.c_void_p * abi.FW_MAX_COLS)()
        for c, v in (nulls or {}).items():
            nul[c] = v.data_ptr()
        check(lib().fw_push_device(self._h, n, keys.data_ptr(), ts.data_ptr(),
                                   key_hashes.data_ptr() if key_hashes is not None else None, arr, nul))
        self.push_seq += 1
        self._end_read(cur)

    def push_device_segments(self, seg_counts, keys, ts, values=(), key_hashes=None, nulls=None):
        """A padded exchange receive buffer (KeyByExchange.exchange_padded): len(seg_counts)
        segments of keys.numel() // len(seg_counts) rows; segment s holds seg_counts[s] valid rows
        (a device int64 tensor -- no host round trip)."""
        p = seg_counts.numel()
        n = keys.numel()
        if p == 0 or n == 0:
            return
        cur = self._begin_read(keys.device)
        arr = (C.c_void_p * abi.FW_MAX_COLS)()
        for c, v in enumerate(values):
            arr[c] = v.data_ptr()
        nul = (C.c_void_p * abi.FW_MAX_COLS)()
        for c, v in (nulls or {}).items():
            nul[c] = v.data_ptr()
        check(lib().fw_push_device_segments(self._h, p, n // p, seg_counts.data_ptr(), keys.data_ptr(), ts.data_ptr(),
                                            key_hashes.data_ptr() if key_hashes is not None else None, arr, nul))
        self.push_seq += 1
        self._end_read(cur)

    def push_device_packed_segments(self, seg_counts, rows, row_words):
        """A packed padded exchange receive buffer (KeyByExchange.exchange_packed): len(seg_counts)
        segments of rows.numel() // (len(seg_counts) * row_words) packed rows (key, ts, value
        words); segment s holds seg_counts[s] valid rows (a device int64 tensor)."""
        p = seg_counts.numel()
        if p == 0 or rows.numel() == 0:
            return
        cur = self._begin_read(rows.device)
        check(lib().fw_push_device_packed_segments(self._h, p, rows.numel() // (p * row_words), seg_counts.data_ptr(),
                                                   rows.data_ptr(), int(row_words)))
        self.push_seq += 1
        self._end_read(cur)

    # ---- progress / output
    def advance(self, wm):
        check(lib().fw_advance(self._h, int(wm)))

    def advance_device(self, wm_tensor):
        """fw_advance_device: the watermark is the first element of a device int64 tensor (e.g. the
        device-side watermark valve of KeyByExchange); the handle's stream waits for the producer's
        current stream first."""
        cur = self._begin_read(wm_tensor.device)
        check(lib().fw_advance_device(self._h, wm_tensor.data_ptr()))
        self._end_read(cur)

    def flush(self):
        check(lib().fw_flush(self._h))

    def results(self, reset=True):
        r = abi.fw_result()
        check(lib().fw_results(self._h, C.byref(r), 1))
        n = r.n
        out = {
            "key": _np_view(r.key, n, np.int64).copy(),
            "window_start": _np_view(r.window_start, n, np.int64).copy(),
            "window_end": _np_view(r.window_end, n, np.int64).copy(),
            "values": [_np_view(r.values[a], n, np.int64).copy() for a in range(self.n_aggs)],
            "null_mask": _np_view(r.null_mask, n, np.uint32).copy(),
        }
        if self.cfg.ds_first_ordinals:  # DataStream: arrival ordinal of each window's first element
            out["first_ord"] = _np_view(r.first_ord, n, np.int64).copy()
        if self.cfg.key_hash == abi.KEYHASH_KEYROW:  # each row's key row (BinaryRowData image)
            lens = _np_view(r.key_row_len, n, np.int32)
            img = _np_view(r.key_row_bytes, n * r.key_row_stride, np.uint8)
            st = r.key_row_stride
            out["key_rows"] = [img[i * st:i * st + int(lens[i])].tobytes() for i in range(n)]
        if reset:
            self.reset_results()
        return out

    def result_segments(self):
        """fw_results_device_segments: the rows emitted since the last collection where the merge
        wrote them (no compaction), consumed.  Returns the device description (n_segments, seg_cap,
        counts pointer, column pointers) as the ABI struct; segments_to_host() reads it back."""
        seg = abi.fw_result_segments()
        check(lib().fw_results_device_segments(self._h, C.byref(seg)))
        return seg

    def _window_starts(self, window_end):
        """ABI v10: segments carry no window_start; it is SliceAssigner.getWindowStart(window_end),
        computed by the library's own host helper (fw_host_time_op 4) once per distinct window end
        (the LOCAL phase's rows are slices: start = end)."""
        if self.cfg.agg_phase == abi.PHASE_LOCAL or window_end.size == 0:
            return window_end.copy()
        ends, inv = np.unique(window_end, return_inverse=True)
        starts = np.empty_like(ends)
        v = C.c_int64()
        for i, e in enumerate(ends.tolist()):
            check(lib().fw_host_time_op(C.byref(self.cfg), 4, int(e), C.byref(v)))
            starts[i] = v.value
        return starts[inv.reshape(-1)]

    def segments_to_host(self, seg):
        """The rows of a result_segments() description as the dict results() returns (host copies,
        after the handle's stream drains; for tests and tools -- a device consumer reads the
        segments in place)."""
        self.sync()
        cols = {"key": seg.cols.key, "window_end": seg.cols.window_end}
        out = {k: [] for k in cols}
        out["values"] = [[] for _ in range(self.n_aggs)]
        out["null_mask"] = []
        ds = bool(self.cfg.ds_first_ordinals)
        if ds:
            out["first_ord"] = []
        if seg.n_segments:
            counts = _np_view(seg.counts, int(seg.n_segments), np.int32).copy()
            total = int(seg.cols.n)
            for sidx, c in enumerate(counts.tolist()):
                if c <= 0:
                    continue
                r0 = sidx * int(seg.seg_cap)
                for k, ptr in cols.items():
                    out[k].append(_np_view(ptr, total, np.int64)[r0:r0 + c].copy())
                for a in range(self.n_aggs):
                    out["values"][a].append(_np_view(seg.cols.values[a], total, np.int64)[r0:r0 + c].copy())
                out["null_mask"].append(_np_view(seg.cols.null_mask, total, np.uint32)[r0:r0 + c].copy())
                if ds:
                    out["first_ord"].append(_np_view(seg.cols.first_ord, total, np.int64)[r0:r0 + c].copy())

        def cat(xs, dt):
            return np.concatenate(xs) if xs else np.empty(0, dt)
        res = {k: cat(out[k], np.int64) for k in cols}
        res["window_start"] = self._window_starts(res["window_end"])
        res["values"] = [cat(v, np.int64) for v in out["values"]]
        res["null_mask"] = cat(out["null_mask"], np.uint32)
        if ds:
            res["first_ord"] = cat(out["first_ord"], np.int64)
        return res

    def results_async(self):
        """Queue the collection of the rows emitted since the last collection into pinned host
        memory (fw_results_async); they count as consumed.  results_ready() returns them."""
        check(lib().fw_results_async(self._h))

    def results_ready(self, copy=True):
        """The rows of the OLDEST outstanding results_async() (waits for them; up to three may be
        outstanding): the dict results() returns.  With copy=False the arrays are views of the
        handle's pinned buffers, valid until the third results_async() after that one."""
        r = abi.fw_result()
        check(lib().fw_results_ready(self._h, C.byref(r)))
        n = r.n
        cp = (lambda a: a.copy()) if copy else (lambda a: a)
        v = lambda p, t: cp(_np_view(p, n, t)) if n else np.zeros(0, dtype=t)
        out = {"key": v(r.key, np.int64), "window_start": v(r.window_start, np.int64),
               "window_end": v(r.window_end, np.int64),
               "values": [v(r.values[a], np.int64) for a in range(self.n_aggs)],
               "null_mask": v(r.null_mask, np.uint32)}
        if self.cfg.ds_first_ordinals:
            out["first_ord"] = v(r.first_ord, np.int64)
        return out

    def device_results_async(self, device):
        """The rows emitted since the last collection as device tensors, WITHOUT a host round trip
        (fw_results_device): returns (n, key, window_start, window_end, [values], null_mask) where n is
        a one-element device int64 tensor and the columns are views of output_capacity rows (only the
        first n are rows).  The rows count as consumed; the caller's current stream is ordered after
        the collection, and the views stay valid until the handle collects results again."""
        import torch
        r = abi.fw_result()
        dn = C.c_void_p()
        check(lib().fw_results_device(self._h, C.byref(r), C.byref(dn)))
        cap = int(r.n)
        cur = self._begin_read(device)  # (the handle stream also waits for the caller's earlier work)
        self._end_read(cur)             # the caller's stream waits for the collection

        class _View:
            def __init__(self, ptr, n, typestr):
                self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                                 "version": 3, "strides": None}

        def t(ptr, n=cap, typestr="<i8"):
            return torch.as_tensor(_View(C.cast(ptr, C.c_void_p).value, n, typestr), device=device)
        return (t(dn.value, 1), t(r.key), t(r.window_start), t(r.window_end),
                [t(r.values[a]) for a in range(self.n_aggs)], t(r.null_mask, typestr="<i4"))

    def device_results(self):
        """(n, fw_result with device pointers) -- for device-side sinks."""
        r = abi.fw_result()
        check(lib().fw_results(self._h, C.byref(r), 0))
        return r.n, r

    def device_result_tensors(self, device):
        """This watermark's results as torch tensors on `device` (zero-copy views of the handle's
        result buffers, valid until the next call on the handle): key, window_start, window_end,
        [values], null_mask (int64)."""
        import torch
        n, r = self.device_results()

        class _View:  # __cuda_array_interface__ over a device pointer
            def __init__(self, ptr, typestr):
                self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                                 "version": 3, "strides": None}

        def t(ptr, typestr="<i8"):
            if n == 0:
                return torch.empty(0, dtype=torch.int64 if typestr == "<i8" else torch.int32, device=device)
            return torch.as_tensor(_View(C.cast(ptr, C.c_void_p).value, typestr), device=device)
        return (t(r.key), t(r.window_start), t(r.window_end), [t(r.values[a]) for a in range(self.n_aggs)],
                t(r.null_mask, "<i4").to(torch.int64))

    def reset_results(self):
        check(lib().fw_results_reset(self._h))

    def late_records(self):
        """The late side output since the last call (DataStream, late_side_output): key, ts,
        values (per value column), push_seq, row -- consumed (WindowOperator.sideOutput)."""
        r = abi.fw_late_rows()
        check(lib().fw_late_records(self._h, C.byref(r)))
        n = r.n
        return {"key": _np_view(r.key, n, np.int64).copy(), "ts": _np_view(r.ts, n, np.int64).copy(),
                "values": [_np_view(r.values[c], n, np.int64).copy() for c in range(self.cfg.n_value_cols)],
                "push_seq": _np_view(r.push_seq, n, np.int64).copy(), "row": _np_view(r.row, n, np.int64).copy()}

    def first_element_events(self):
        """DataStream with ds_first_ordinals: (retain, release) arrival ordinals since the last call
        (fw_first_element_events) -- the first elements a shim must keep / may drop."""
        r = abi.fw_ordinal_events()
        check(lib().fw_first_element_events(self._h, C.byref(r)))
        return (_np_view(r.retain, r.n_retain, np.int64).copy(), _np_view(r.release, r.n_release, np.int64).copy())

    def stats(self):
        s = abi.fw_stats()
        check(lib().fw_get_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in abi.fw_stats._fields_}

    # ---- device timing (hipEvents around each launch on the handle stream)
    def set_profiling(self, enable=True, mode="device"):
        """Per-launch timing of the ingest and merge/fire kernels: mode "device" (in-kernel clock
        stamps, nothing added to the stream) or "events" (hipEvents around each launch)."""
        m = {"device": 1, "events": 2, "events_all": 3}[mode]
        check(lib().fw_set_profiling(self._h, m if enable else 0))

    def kernel_times(self):
        """{kind: (ms, launches)} accumulated since set_profiling(True)."""
        t = abi.fw_kernel_times()
        check(lib().fw_get_kernel_times(self._h, C.byref(t)))
        names = {abi.KT_PARTITION: "partition", abi.KT_SCAN: "scan", abi.KT_REDUCE: "reduce",
                 abi.KT_MERGE: "merge", abi.KT_OTHER: "other"}
        out = {n: (t.ms[k], t.launches[k]) for k, n in names.items()}
        out["merge_phase_cycles"] = list(t.merge_phase_cycles)
        return out

    # ---- checkpoint
    def snapshot(self) -> bytes:
        size = C.c_int64()
        check(lib().fw_snapshot(self._h, None, 0, C.byref(size)))
        buf = C.create_string_buffer(size.value)
        check(lib().fw_snapshot(self._h, buf, size.value, C.byref(size)))
        return buf.raw[:size.value]

    # ---- key-group-partitioned checkpoint (rescaling)
    def key_group_range(self):
        """computeKeyGroupRangeForOperatorIndex(maxP, p, subtask) (KeyGroupRangeAssignment.java:93-106),
        inclusive bounds."""
        mp, p, i = self.cfg.max_parallelism, self.cfg.parallelism, self.cfg.subtask_index
        return (i * mp + p - 1) // p, ((i + 1) * mp - 1) // p

    def snapshot_key_groups(self):
        """{key_group: blob} for every owned key group, plus this subtask's watermark (the entry it
        contributes to the operator's union-list watermark state)."""
        lo, hi = self.key_group_range()
        out = {}
        for kg in range(lo, hi + 1):
            size = C.c_int64()
            check(lib().fw_snapshot_key_group(self._h, kg, None, 0, C.byref(size)))
            buf = C.create_string_buffer(size.value)
            check(lib().fw_snapshot_key_group(self._h, kg, buf, size.value, C.byref(size)))
            out[kg] = buf.raw[:size.value]
        return out, self.stats()["current_watermark"]

    def restore_key_groups(self, blobs, watermarks):
        """Restore the owned key groups found in `blobs` ({key_group: blob}, any source parallelism).
        SQL: the watermark becomes the min of the union list (WindowAggOperator.initializeState
        :183-206).  DataStream: the WindowOperator keeps no watermark state; its timer service
        starts again at Long.MIN_VALUE (InternalTimerServiceImpl.java:72)."""
        lo, hi = self.key_group_range()
        for kg, blob in blobs.items():
            if lo <= kg <= hi:
                self.restore_key_group_blob(blob)
        wms = list(watermarks)
        if wms and self.cfg.api == abi.API_SQL:
            self.initialize_watermark(min(wms))

    def restore_key_group_blob(self, blob: bytes):
        """One key group's blob; raises if this subtask does not own it or the layout differs."""
        buf = C.create_string_buffer(blob, len(blob))
        check(lib().fw_restore_key_group(self._h, buf, len(blob)))
        self.push_seq = max(self.push_seq, _snapshot_push_seq(blob))

    def ds_key_group_windows(self, kg: int):
        """DataStream: the (key, window) states and timers of key group `kg` (flinkwin.h
        fw_ds_snapshot_key_group; flushes first) as a structured numpy array."""
        n = C.c_int64()
        check(lib().fw_ds_snapshot_key_group(self._h, kg, None, 0, C.byref(n)))
        arr = (abi.fw_ds_window * max(n.value, 1))()
        check(lib().fw_ds_snapshot_key_group(self._h, kg, arr, n.value, C.byref(n)))
        out = np.zeros(n.value, DS_WINDOW_DTYPE)
        if n.value:
            out[:] = np.frombuffer(bytes(arr)[:n.value * C.sizeof(abi.fw_ds_window)], DS_WINDOW_DTYPE)
        return out

    def ds_restore_key_group_windows(self, kg: int, windows, next_push_seq: int):
        """DataStream: adds key group `kg`'s windows (DS_WINDOW_DTYPE records); first-element
        ordinals lie below push `next_push_seq`, where this handle's ordinals then continue."""
        w = np.ascontiguousarray(np.asarray(windows, DS_WINDOW_DTYPE))
        arr = (abi.fw_ds_window * max(len(w), 1)).from_buffer_copy(w.tobytes() or bytes(C.sizeof(abi.fw_ds_window)))
        check(lib().fw_ds_restore_key_group(self._h, kg, arr, len(w), next_push_seq))
        self.push_seq = max(self.push_seq, next_push_seq)

    def snapshot_key_group_heap(self, kg: int, ids=(0, 1, 2)) -> bytes:
        """Key group `kg` in the heap keyed-state backend's byte format (flinkwin.h
        fw_snapshot_key_group_heap); ids = (window-aggs, event timers, processing timers) state ids."""
        sid = abi.fw_heap_state_ids(*ids, 0)
        size = C.c_int64()
        check(lib().fw_snapshot_key_group_heap(self._h, kg, C.byref(sid), None, 0, C.byref(size)))
        buf = C.create_string_buffer(max(size.value, 1))
        check(lib().fw_snapshot_key_group_heap(self._h, kg, C.byref(sid), buf, size.value, C.byref(size)))
        return buf.raw[:size.value]

    def restore_key_group_heap(self, blob: bytes, ids=(0, 1, 2)):
        """Adds one key group written in the heap backend's format (by this library or by a heap
        backend) to this handle."""
        sid = abi.fw_heap_state_ids(*ids, 0)
        buf = C.create_string_buffer(blob, max(len(blob), 1))
        check(lib().fw_restore_key_group_heap(self._h, buf, len(blob), C.byref(sid)))

    def restore(self, blob: bytes):
        buf = C.create_string_buffer(blob, len(blob))
        check(lib().fw_restore(self._h, buf, len(blob)))
        self.push_seq = max(self.push_seq, _snapshot_push_seq(blob))


def _snapshot_push_seq(blob):
    """The push counter a snapshot blob carries (SnapHeader / KgHeader .push_seq, the last field)."""
    import struct
    off = {0x464c4b57494e3033: 8 + 16 + 32 + 8, 0x464c4b574b473033: 8 + 24 + 32 + 8}.get(struct.unpack_from("<Q", blob, 0)[0])
    return struct.unpack_from("<q", blob, off)[0] if off is not None else 0
