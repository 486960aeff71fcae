"""keyBy exchange between operator subtasks, one rank per GPU.

Replaces the reference's record routing + network shuffle for a keyed window operator:
KeyGroupStreamPartitioner.selectChannel (flink-runtime/.../streaming/runtime/partitioner/
KeyGroupStreamPartitioner.java:55-65, destination = computeOperatorIndexForKeyGroup(maxP, p,
assignToKeyGroup(key)), KeyGroupRangeAssignment.java:63-127) followed by
ChannelSelectorRecordWriter.emit (flink-runtime/.../io/network/api/writer/
ChannelSelectorRecordWriter.java:54) over Netty, and the receiving side's
StatusWatermarkValve.inputWatermark (min over input channels, StatusWatermarkValve.java:153).

Here a columnar batch is counting-sorted by destination subtask, then moved with an all-to-all
(RCCL over xGMI for device batches; gloo for host batches).  Partitioning runs where the batch
lives: device batches on the GPU (fw_partition_by_dest), host-staged batches with the library's
host routine (fw_host_assign_key_groups) - the reference routes records on the sending task's CPU
too.  Both use the same key-group code the kernels run.

exchange_packed is the per-step device path: the partition kernel writes every row's columns
side by side (key, ts, values) straight into fixed-size per-destination segments
(fw_partition_packed_spill), the rows travel as ONE all-to-all of that buffer, the row counts as a
second small all-to-all that stays on the device, and the receiving operator reads the packed
rows in place and skips each segment's padding itself (fw_push_device_packed_segments).  The
segment size comes from the batch itself (its even share plus headroom), never from later data:
rows past a destination's segment go to a spill region, and an overflow round sends them when
any subtask had some (the subtasks agree on it in the same host all-reduce as the watermark valve,
after waiting only for their own partition kernel, not for the all-to-all in flight).  exchange_padded does the same with one all-to-all per column (for
configurations whose key-hash or NULL-flag columns do not fit the packed rows).  The watermark
valve runs on the host (a gloo group over CPU tensors), as Flink's StatusWatermarkValve does on
the receiving task, so it never waits on the GPU stream.
"""
import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from .. import abi
from .._native import check, lib


class KeyByExchange:
    def __init__(self, key_hash_kind, max_parallelism=128, group=None, force_collectives=False):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.kind = key_hash_kind
        self.max_p = max_parallelism
        self._ws = None
        self._cpu_group = None
        # the packed exchange's collectives (all-to-all, valve all-reduce, overflow round) run when
        # there is more than one subtask; force_collectives runs them for one subtask too, so the
        # RCCL branches execute on a one-GPU box (tests/test_gpu_multirank.py)
        self.collectives = self.world > 1 or (force_collectives and dist.is_initialized())
        if self.collectives and dist.get_backend(group) != "gloo":
            # the watermark valve's host-side group over the same ranks (collective creation:
            # every rank builds the exchange at the same point)
            ranks = dist.get_process_group_ranks(group) if group is not None else None
            self._cpu_group = dist.new_group(ranks=ranks, backend="gloo")
        self._max_count = None  # running max of rows per destination (padded exchanges), on the device
        self.spill_rounds = 0
        self._dn_share = 1 << 16  # largest per-destination share of the last exchange, agreed by all subtasks
        self._share_known = False  # _dn_share comes from an agreed exchange (not the initial guess)
        # packed segments: the previous exchange's agreed largest share plus this headroom (rows past a
        # segment take the overflow round, so a tight headroom costs a spill round, never rows)
        self.headroom = 0.03

    # ---- routing ------------------------------------------------------------------------
    def partition(self, key, ts, values, key_hash=None):
        """Rows grouped by destination subtask (ascending).  Returns (key, ts, values, counts)
        with counts[d] = rows for subtask d; rows keep their input order within a destination
        (fw_partition_by_dest's scatter is stable).  ``key_hash`` (int32 per row) routes
        FW_KEYHASH_PRECOMPUTED keys, e.g. VARCHAR keys hashed by fw_key_row_hash."""
        p = self.world
        if self.kind == abi.KEYHASH_PRECOMPUTED and key_hash is None:
            raise ValueError("precomputed-hash keys need their key_hash column")
        if key.is_cuda:
            return self._partition_device(key, ts, values, key_hash)
        n = key.numel()
        dest = np.empty(n, dtype=np.int32)
        kn = np.ascontiguousarray(key.numpy())
        kh = None if key_hash is None else np.ascontiguousarray(key_hash.numpy().astype(np.int32, copy=False))
        check(lib().fw_host_assign_key_groups(kn.ctypes.data, None if kh is None else kh.ctypes.data, n, self.kind,
                                              self.max_p, p, None, dest.ctypes.data))
        order = torch.from_numpy(np.argsort(dest, kind="stable"))
        counts = torch.from_numpy(np.bincount(dest, minlength=p).astype(np.int64))
        return key[order], ts[order], [v[order] for v in values], counts

    def _partition_device(self, key, ts, values, key_hash=None):
        p, n, dev = self.world, key.numel(), key.device
        L = lib()
        ws = L.fw_partition_workspace_bytes(n, p)
        if self._ws is None or self._ws.numel() < ws or self._ws.device != dev:
            self._ws = torch.empty(max(ws, 256), dtype=torch.uint8, device=dev)
        pk, pt = torch.empty_like(key), torch.empty_like(ts)
        pv = [torch.empty_like(v) for v in values]
        counts = torch.empty(p, dtype=torch.int64, device=dev)
        vin = (C.c_void_p * abi.FW_MAX_COLS)(*[v.data_ptr() for v in values])
        vout = (C.c_void_p * abi.FW_MAX_COLS)(*[v.data_ptr() for v in pv])
        kh = None if key_hash is None else key_hash.to(torch.int32).contiguous()
        check(L.fw_partition_by_dest(key.data_ptr(), None if kh is None else kh.data_ptr(), ts.data_ptr(), vin,
                                     len(values), n, self.kind,
                                     self.max_p, p, pk.data_ptr(), pt.data_ptr(), vout, counts.data_ptr(),
                                     self._ws.data_ptr(), self._ws.numel(),
                                     torch.cuda.current_stream(dev).cuda_stream))
        return pk, pt, pv, counts

    # ---- exchange -----------------------------------------------------------------------
    def exchange(self, key, ts, values, key_hash=None):
        """Send every row to the subtask owning its key group; returns this subtask's rows
        (grouped by source rank, each source's rows in their partitioned order).  With
        ``key_hash`` (precomputed-hash keys) the hash travels with its row and the result is
        (key, ts, values, key_hash)."""
        if key_hash is None:
            return self._exchange(key, ts, list(values), None)
        # the hash moves as one more 8-byte column
        k, t, v = self._exchange(key, ts, list(values) + [key_hash.to(torch.int64)], key_hash)
        return k, t, v[:-1], v[-1].to(torch.int32)

    def _exchange(self, key, ts, values, routing_hash):
        if self.world == 1:
            return key, ts, list(values)
        pk, pt, pv, counts = self.partition(key, ts, values, routing_hash)
        # gloo moves host tensors only: device batches are staged through host memory (used to
        # rehearse the N > 1 path on one GPU; RCCL moves device memory directly over xGMI)
        stage = key.is_cuda and dist.get_backend(self.group) != "nccl"
        cols = [pk, pt] + pv
        if stage:
            counts, cols = counts.cpu(), [c.cpu() for c in cols]
        rc = torch.empty_like(counts)
        dist.all_to_all_single(rc, counts, group=self.group)
        send, recv = counts.tolist(), rc.tolist()
        n = sum(recv)
        out = []
        for col in cols:
            r = torch.empty(n, dtype=col.dtype, device=col.device)
            dist.all_to_all_single(r, col, recv, send, group=self.group)
            out.append(r.to(key.device) if stage else r)
        return out[0], out[1], out[2:]

    def exchange_padded(self, key, ts, values, capacity):
        """Device batches, no host round trip: every destination's rows travel in a fixed-size
        segment of ``capacity`` rows (one equal-split all-to-all per column), the row counts in
        one small all-to-all that stays on the device.  Returns (key, ts, values, recv_counts):
        columns of p segments of ``capacity`` rows, segment s holding the first recv_counts[s]
        rows subtask s sent here -- the layout fw_push_device_segments ingests.  A destination
        with more rows than ``capacity`` is detected by check_capacity()."""
        p, n, dev = self.world, key.numel(), key.device
        pk, pt, pv, counts = self.partition(key, ts, values)
        if p == 1:
            return pk, pt, pv, counts
        cap = int(capacity)
        starts = torch.cumsum(counts, 0) - counts
        j = torch.arange(cap, device=dev)
        src = (starts[:, None] + j[None, :]).clamp_(max=max(n - 1, 0)).reshape(-1)
        # gloo moves host tensors only (the one-GPU rehearsal stages through host memory)
        stage = key.is_cuda and dist.get_backend(self.group) != "nccl"
        mv = (lambda x: x.cpu()) if stage else (lambda x: x)
        back = (lambda x: x.to(dev)) if stage else (lambda x: x)
        rc = torch.empty_like(mv(counts))
        dist.all_to_all_single(rc, mv(counts), group=self.group)
        out = []
        for col in [pk, pt] + list(pv):
            send = mv(col.index_select(0, src))  # segment d = the rows for subtask d, padded to cap
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send, group=self.group)
            out.append(back(recv))
        rc = back(rc)
        self._note_counts(counts, cap)  # validated lazily, off the hot path
        return out[0], out[1], out[2:], rc

    @staticmethod
    def segment_capacity(n_rows, world, headroom=0.25):
        """The padded segment size for a batch of n_rows: its even share plus headroom (rows past
        it take the overflow round, so this never has to bound the batch)."""
        return int(n_rows / max(world, 1) * (1.0 + headroom)) + 1024

    def exchange_packed(self, key, ts, values, capacity=None, watermark=None):
        """Like exchange_padded, with the rows packed: returns (rows, recv_counts, row_words, spill,
        watermark) where rows is p segments of ``capacity`` rows of row_words = 2 + len(values)
        int64 words (key, ts, value bits), segment s holding the first recv_counts[s] rows subtask s
        sent here -- the buffer fw_push_device_packed_segments ingests.  One all-to-all for the
        rows, one for the counts.  Rows past a destination's segment come in ``spill`` (packed
        rows, None when no subtask overflowed).  ``watermark``: this subtask's input watermark;
        the returned one is the valve's minimum over all subtasks (StatusWatermarkValve)."""
        px = self.exchange_packed_async(key, ts, values, capacity)
        spill, wm = px.finish(watermark)
        return px.rows, px.recv_counts, px.row_words, spill, wm

    def exchange_packed_async(self, key, ts, values, capacity=None, n_dev=None):
        """The packed exchange in two halves, so the caller can queue the ingest of the received
        segments before the host waits: this call enqueues the partition and both all-to-alls and
        returns a PackedExchange (rows, recv_counts, row_words); its finish(watermark) waits for
        this subtask's partition kernel only, agrees on the overflow round and the watermark with
        the other subtasks (one host all-reduce) and returns (spill, watermark).  ``n_dev``: a
        one-element device int64 tensor holding the row count (the columns are only its bound, e.g.
        fw_results_device's): the rows are partitioned without a host round trip, and the segment
        size comes from the largest share the previous such exchange saw (rows past it take the
        overflow round)."""
        p, n, dev = self.world, key.numel(), key.device
        w = 2 + len(values)
        if capacity is not None:
            cap = int(capacity)
        elif self._share_known:  # the last agreed share + headroom: padding is ~3 %, not 25 % + 1024 rows
            cap = max(int(self._dn_share * (1.0 + self.headroom)) + 64, 64)
        elif n_dev is not None:
            cap = int(self._dn_share * 1.25) + 1024
        else:
            cap = self.segment_capacity(n, p)
        vals64 = [v.view(torch.int64) if v.dtype == torch.float64 else v for v in values]
        if key.is_cuda:
            L = lib()
            ws = L.fw_partition_workspace_bytes(n, p)
            if self._ws is None or self._ws.numel() < ws or self._ws.device != dev:
                self._ws = torch.empty(max(ws, 256), dtype=torch.uint8, device=dev)
            send = torch.empty(p * cap * w, dtype=torch.int64, device=dev)
            spill = torch.empty(max(n, 1) * w, dtype=torch.int64, device=dev)
            counts = torch.empty(p, dtype=torch.int64, device=dev)
            vin = (C.c_void_p * abi.FW_MAX_COLS)(*[v.data_ptr() for v in vals64])
            if n_dev is None:
                check(L.fw_partition_packed_spill(key.data_ptr(), None, ts.data_ptr(), vin, len(values), n, self.kind,
                                                  self.max_p, p, cap, send.data_ptr(), spill.data_ptr(),
                                                  counts.data_ptr(), self._ws.data_ptr(), self._ws.numel(),
                                                  torch.cuda.current_stream(dev).cuda_stream))
            else:
                check(L.fw_partition_packed_spill_dn(key.data_ptr(), None, ts.data_ptr(), vin, len(values), n,
                                                     n_dev.data_ptr(), self.kind, self.max_p, p, cap, send.data_ptr(),
                                                     spill.data_ptr(), counts.data_ptr(), self._ws.data_ptr(),
                                                     self._ws.numel(), torch.cuda.current_stream(dev).cuda_stream))
            counts_h = torch.empty(p, dtype=torch.int64, pin_memory=True)
            counts_h.copy_(counts, non_blocking=True)
            part_done = torch.cuda.Event()
            part_done.record(torch.cuda.current_stream(dev))
            counts_d = counts
        else:  # host batch: the host partition, then the same padded layout
            pk, pt, pv, counts = self.partition(key, ts, vals64)
            send = torch.zeros(p * cap * w, dtype=torch.int64)
            rows = torch.stack([pk, pt] + list(pv), dim=1) if n else torch.zeros((0, w), dtype=torch.int64)
            seg = send.view(p, cap, w)
            sp = []
            o = 0
            for d, c in enumerate(counts.tolist()):
                m = min(c, cap)
                seg[d, :m] = rows[o:o + m]
                sp.append(rows[o + m:o + c])
                o += c
            spill = torch.cat(sp).reshape(-1) if sp else torch.zeros(0, dtype=torch.int64)
            counts_h, part_done, counts_d = counts, None, counts
        stage = key.is_cuda and self.collectives and dist.get_backend(self.group) != "nccl"
        mv = (lambda x: x.cpu()) if stage else (lambda x: x)
        back = (lambda x: x.to(dev)) if stage else (lambda x: x)
        if self.collectives:
            rc = torch.empty_like(mv(counts))
            dist.all_to_all_single(rc, mv(counts), group=self.group)
            s_ = mv(send)
            recv = torch.empty_like(s_)
            dist.all_to_all_single(recv, s_, group=self.group)
            recv, rc = back(recv), back(rc)
        else:
            recv, rc = send, counts
        return PackedExchange(self, recv, rc, w, cap, spill, counts_h, part_done, mv, back, counts_d)

    def _agree(self, overflow, watermark, share=0):
        """One host all-reduce for the overflow decision, the watermark valve's minimum and the
        largest per-destination share."""
        wm = None if watermark is None else int(watermark)
        if not self.collectives:
            return overflow, wm, int(share)
        g = self.group if self._cpu_group is None else self._cpu_group
        # ~w (= -w - 1) reverses the int64 order with no overflow (-Long.MIN_VALUE would): MAX of ~w is ~MIN
        t = torch.tensor([1 if overflow else 0, ~wm if wm is not None else 0, int(share)], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
        return bool(t[0].item()), (None if wm is None else ~int(t[1].item())), int(t[2].item())

    def _note_counts(self, counts, cap):
        """Keep the running max of rows per destination on the device (check_capacity)."""
        m = counts.max() if counts.numel() else torch.zeros((), dtype=torch.int64, device=counts.device)
        self._max_count = m if self._max_count is None or self._max_count.device != m.device else torch.maximum(self._max_count, m)
        self._cap_min = cap if getattr(self, "_cap_min", None) is None else min(self._cap_min, cap)

    def check_capacity(self):
        """Raises if exchange_padded dropped rows: some destination of some batch since the first
        exchange got more rows than its segment (running max; exchange_packed never drops -- its
        overflow round sends them)."""
        if self._max_count is not None:
            m, cap = int(self._max_count), self._cap_min
            if m > cap:
                raise RuntimeError(f"padded exchange: {m} rows for one subtask > capacity {cap}")

    def global_max(self, x):
        """Max of a host integer over all subtasks (e.g. the padded exchange's capacity, which
        every subtask must agree on)."""
        if self.world == 1:
            return int(x)
        t = torch.tensor([int(x)], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group if self._cpu_group is None else self._cpu_group)
        return int(t.item())

    def global_watermark(self, w):
        """StatusWatermarkValve: the combined watermark is the min over all input channels.  Runs
        on the host (gloo over CPU tensors): the watermark is a host value, like the valve's."""
        if self.world == 1:
            return int(w)
        g = self.group if self._cpu_group is None else self._cpu_group
        t = torch.tensor([int(w)], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=g)
        return int(t.item())


class PackedExchange:
    """One step's packed keyBy exchange in flight (KeyByExchange.exchange_packed_async).

    Two ways to close it: finish(watermark) -- the host waits for this subtask's partition kernel and
    agrees on the overflow round, the watermark and the next segment size in one host all-reduce --
    or, with no host wait, finish_device(watermark, prev) + settle() one step later: the same three
    values travel in one DEVICE all-reduce (RCCL), the valve's watermark stays in device memory for
    fw_advance_device, and a step with overflow holds the watermark at the previous one until its
    spill rows, sent by settle() before the next step's rows, are in."""

    def __init__(self, ex, rows, recv_counts, row_words, cap, spill, counts_h, part_done, mv, back, counts_d=None):
        self.ex, self.rows, self.recv_counts, self.row_words = ex, rows, recv_counts, row_words
        self._cap, self._spill, self._counts_h, self._part_done = cap, spill, counts_h, part_done
        self._mv, self._back, self._counts_d = mv, back, counts_d
        self._agreed = None  # finish_device's all-reduced [overflow, ~watermark, share] (device)
        self.agreed_watermark = None  # settle(): the valve's minimum watermark of this step (host)
        self._agreed_h = self._agreed_ev = None  # its pinned host mirror and the event that fills it

    def finish(self, watermark=None):
        """The overflow round and the watermark valve: waits for this subtask's partition kernel
        only (the all-to-all and whatever the caller queued after it stay in flight)."""
        ex = self.ex
        if self._part_done is not None:
            self._part_done.synchronize()
        cnt = self._counts_h.tolist()
        over = [max(0, c - self._cap) for c in cnt]
        # the next device-counted exchange sizes its segments from the largest share any subtask
        # sent this time: every subtask must pick the same segment size, so it rides in the same
        # all-reduce as the overflow decision and the watermark
        any_over, wm, share = ex._agree(sum(over) > 0, watermark, max(cnt) if cnt else 0)
        ex._dn_share, ex._share_known = share, True
        return self._spill_round(any_over, over), wm

    def finish_device(self, watermark, prev_watermark):
        """The device-side valve (StatusWatermarkValve.java:153: min over the input channels): this
        subtask's overflow flag, ~watermark and largest per-destination share go into ONE all-reduce
        (MAX) on the device -- RCCL on the stream, nothing waits on the host.  Returns a one-element
        device int64 tensor: the minimum watermark, or ``prev_watermark`` (device tensor) when any
        subtask overflowed its segments -- its spill rows are sent by settle() at the start of the next
        step, and the watermark must not pass them before.  settle() must be called before the next
        exchange (it also agrees on the next device-counted segment size)."""
        ex = self.ex
        dev = self._counts_d.device
        if self._counts_d.is_cuda and 0 < self._counts_d.numel() <= 64:  # one kernel for the three words
            t = torch.empty(3, dtype=torch.int64, device=dev)
            check(lib().fw_valve_local(self._counts_d.data_ptr(), self._counts_d.numel(), int(self._cap), int(watermark),
                                       t.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
        else:
            t = torch.stack([(self._counts_d > self._cap).any().to(torch.int64),
                             torch.full((), ~int(watermark), dtype=torch.int64, device=dev),
                             self._counts_d.max() if self._counts_d.numel() else torch.zeros((), dtype=torch.int64, device=dev)])
        if ex.collectives:
            if self._counts_d.is_cuda and dist.get_backend(ex.group) == "nccl":
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ex.group)
            else:  # gloo moves host tensors (the one-GPU rehearsal and the CPU tests)
                g = ex._cpu_group if ex._cpu_group is not None else ex.group
                th = t.cpu()
                dist.all_reduce(th, op=dist.ReduceOp.MAX, group=g)
                t = th.to(dev)
        self._agreed = t
        self._agreed_h = self._agreed_ev = None
        if t.is_cuda:  # settle() reads a pinned mirror behind an event: no stream-wide sync
            self._agreed_h = torch.empty(3, dtype=torch.int64, pin_memory=True)
            self._agreed_h.copy_(t, non_blocking=True)
            self._agreed_ev = torch.cuda.Event()
            self._agreed_ev.record(torch.cuda.current_stream(dev))
        if t.is_cuda:  # nothing advanced yet (prev None): an overflowing first step holds at Long.MIN_VALUE
            wm = torch.empty(1, dtype=torch.int64, device=dev)
            check(lib().fw_valve_select(t.data_ptr(), None if prev_watermark is None else prev_watermark.data_ptr(),
                                        wm.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
            return wm
        if prev_watermark is None:
            prev_watermark = torch.full((1,), -(1 << 63), dtype=torch.int64, device=dev)
        return torch.where(t[0:1] > 0, prev_watermark, torch.bitwise_not(t[1:2]))

    def settle(self):
        """The host half of finish_device, one step late: reads the agreed values (waits only for this
        step's all-reduce, long done while the next step's work is queued behind it), sets the next
        device-counted segment size, and runs the overflow round if any subtask overflowed.  Returns the
        spill rows for this subtask (device, packed) or None.  When it returns spill rows, the step's
        watermark was held at the previous one: the caller pushes the rows, then advances to
        ``agreed_watermark`` (TwoPhaseWindowAgg.settle does)."""
        t = self._agreed
        if t is None:
            return None
        self._agreed = None
        if self._agreed_ev is not None:  # waits for this step's all-reduce only (the stream runs on)
            self._agreed_ev.synchronize()
            t = self._agreed_h
        any_over, nwm, share = (int(x) for x in t.tolist())
        self.agreed_watermark = ~nwm
        self.ex._dn_share, self.ex._share_known = share, True
        over = None
        if any_over:
            cnt = self._counts_h.tolist()
            over = [max(0, c - self._cap) for c in cnt]
        return self._spill_round(bool(any_over), over)

    def _spill_round(self, any_over, over):
        """Rows past their destination's segment, exchanged with host-known split sizes."""
        ex, w = self.ex, self.row_words
        out_spill = None
        if any_over:
            ex.spill_rounds += 1
            if not ex.collectives:
                out_spill = self._spill[:over[0] * w] if over[0] else None
            else:
                g = ex._cpu_group if ex._cpu_group is not None else ex.group
                sc = torch.tensor(over, dtype=torch.int64)
                rsc = torch.empty_like(sc)
                dist.all_to_all_single(rsc, sc, group=g)
                rin = rsc.tolist()
                total = sum(over)
                src = self._mv(self._spill[:total * w] if total else self._spill[:0])
                dst = torch.empty(sum(rin) * w, dtype=torch.int64, device=src.device)
                dist.all_to_all_single(dst, src, [r * w for r in rin], [o * w for o in over], group=ex.group)
                out_spill = self._back(dst) if sum(rin) else None
        return out_spill
