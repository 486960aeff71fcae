"""Two-phase (local/global) window aggregation: the plan TwoStageOptimizedWindowAggregateRule
(flink-table-planner/.../rules/physical/stream/TwoStageOptimizedWindowAggregateRule.java:80-109)
picks for mergeable aggregates on rowtime windows.

    source subtask --> LocalSlicingWindowAggOperator (LocalAggCombiner, no state, no timers)
                   --> keyBy exchange of (key, accumulator fields, sliceEnd) rows
                   --> WindowAggOperator with GlobalAggCombiner (merge into state, timers, fire)

Here one LOCAL handle per source subtask (owning every key group: it runs before the keyBy) and
one GLOBAL handle per operator subtask.  Between them only the local partials travel -- one row
per (key, slice) per local flush instead of one per record (LocalAggCombiner.java:69-97) -- which
is what makes the phase split pay on the all-to-all for skewed keys.  The local partials never
leave the device: the LOCAL handle's result buffers are read as device tensors, routed by
fw_partition_by_dest, moved by the all-to-all (RCCL over xGMI), and pushed into the GLOBAL handle.
"""
import torch

from .. import abi
from ..runtime.handle import WindowAggHandle


class TwoPhaseWindowAgg:
    def __init__(self, cfg, exchange=None, device=None, local_state_capacity=None):
        """cfg: the one-phase SQL operator configuration of this subtask (its parallelism and
        subtask_index are the GLOBAL operator's).  exchange: a KeyByExchange for parallelism > 1.
        local_state_capacity: the LOCAL operator's sizing hint (it sees every key group; default the
        GLOBAL operator's)."""
        if cfg.api != abi.API_SQL:
            raise ValueError("two-phase window aggregation is a SQL plan")
        if cfg.key_hash == abi.KEYHASH_PRECOMPUTED:
            raise ValueError("two-phase plan needs device-hashable keys (partial rows carry no key hash)")
        if any(cfg.aggs[i].kind not in (abi.AGG_COUNT_STAR, abi.AGG_COUNT, abi.AGG_SUM, abi.AGG_MIN, abi.AGG_MAX,
                                         abi.AGG_AVG) for i in range(cfg.n_aggs)):
            raise ValueError("every aggregate must be mergeable")
        local = abi.make_config(
            api=cfg.api, window_kind=cfg.window_kind, size_ms=cfg.size_ms, slide_ms=cfg.slide_ms,
            offset_ms=cfg.offset_ms, aggs=[(cfg.aggs[i].kind, cfg.aggs[i].input_col, cfg.aggs[i].type)
                                           for i in range(cfg.n_aggs)],
            count_star_index=cfg.count_star_index,
            value_col_types=[cfg.value_col_types[c] for c in range(cfg.n_value_cols)],
            key_hash=cfg.key_hash, max_parallelism=cfg.max_parallelism, parallelism=1, subtask_index=0,
            device=cfg.device, state_capacity=local_state_capacity or cfg.state_capacity, max_batch_rows=cfg.max_batch_rows,
            output_capacity=cfg.output_capacity,
            nullable_cols=[c for c in range(cfg.n_value_cols) if cfg.nullable_cols >> c & 1],
            agg_phase=abi.PHASE_LOCAL)
        self.local_cfg = local
        self.global_cfg = abi.global_config(local, parallelism=cfg.parallelism, subtask_index=cfg.subtask_index,
                                            state_capacity=cfg.state_capacity,
                                            max_batch_rows=max(cfg.max_batch_rows, cfg.output_capacity))
        self.local = WindowAggHandle(local)
        self.glob = WindowAggHandle(self.global_cfg)
        self.exchange = exchange
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.n_fields = abi.result_columns(local)
        self.nullable_fields = [j for j in range(self.n_fields) if self.global_cfg.nullable_cols >> j & 1]

    def close(self):
        self.local.close()
        self.glob.close()

    # ---- LocalSlicingWindowAggOperator.processElement, per columnar batch
    def process_batch(self, keys, ts, values=(), nulls=None):
        self.local.push_host(keys, ts, values, nulls=nulls)

    def process_batch_device(self, keys, ts, values=(), nulls=None):
        self.local.push_device(keys, ts, values, nulls=nulls)

    # ---- local flush -> exchange -> global processElement, then the global watermark
    def local_partials(self, watermark):
        """Advance the LOCAL phase; returns its partial rows as device tensors (key, slice_end,
        [fields], null_mask), copied out of the handle's result buffers."""
        self.local.advance(watermark)
        key, _, se, fields, nm = self.local.device_result_tensors(self.device)
        out = key.clone(), se.clone(), [f.clone() for f in fields], nm.clone()
        self.local.reset_results()
        return out

    def global_ingest(self, key, se, fields, nm):
        nulls = {j: ((nm >> j) & 1).to(torch.uint8) for j in self.nullable_fields}
        self.glob.push_device(key, se, fields, nulls=nulls)

    def process_watermark(self, watermark, global_watermark=None):
        """Returns the GLOBAL operator's rows for this watermark (host dict)."""
        key, se, fields, nm = self.local_partials(watermark)
        if self.exchange is not None:
            key, se, cols = self.exchange.exchange(key, se, fields + [nm])
            fields, nm = cols[:-1], cols[-1]
        self.global_ingest(key, se, fields, nm)
        self.glob.advance(watermark if global_watermark is None else global_watermark)
        return self.glob.results(reset=True)

    def step_device_valve(self, watermark):
        """step_device with the watermark valve on the device (PackedExchange.finish_device): no host
        wait on this step's GPU work; the previous step's overflow round and segment-size agreement are
        settled first (one step late).  Returns the valve's watermark as a one-element device tensor.
        Call settle() after the last step."""
        from ..runtime.exchange import KeyByExchange
        if self.global_cfg.nullable_cols:
            raise ValueError("step_device moves packed rows, which carry no NULL flags: NOT NULL inputs only")
        if self.exchange is None:
            self.exchange = KeyByExchange(self.global_cfg.key_hash, self.global_cfg.max_parallelism)
        self.settle()
        self.local.advance(watermark)
        n, key, _, se, fields, _ = self.local.device_results_async(self.device)
        px = self.exchange.exchange_packed_async(key, se, fields, n_dev=n)
        self.glob.push_device_packed_segments(px.recv_counts, px.rows, px.row_words)
        wm = px.finish_device(watermark, getattr(self, "_wm_dev", None))
        self._wm_dev = wm
        self._px = px
        self.glob.advance_device(wm)
        return wm

    def settle(self):
        """The previous device-valve step's overflow round: its spill rows reach the GLOBAL operator
        before any later watermark, and the watermark that step held back (finish_device keeps the
        previous one while rows are in flight) is issued after them, so the last step needs no extra
        advance from the caller."""
        px = getattr(self, "_px", None)
        if px is None:
            return
        self._px = None
        spill = px.settle()
        if spill is not None:
            n_sp = spill.numel() // px.row_words
            self.glob.push_device_packed_segments(torch.tensor([n_sp], dtype=torch.int64, device=self.device), spill,
                                                  px.row_words)
            self.glob.advance(px.agreed_watermark)

    def step_device(self, watermark):
        """One watermark interval of the plan with the partials kept on the device and no host round
        trip before the exchange: the LOCAL advance, its partial rows collected on the device
        (fw_results_device: the count stays a device value), the packed partition by that count and
        the all-to-all (KeyByExchange.exchange_packed_async, n_dev), the GLOBAL ingest of the received
        segments queued, then the overflow round and the watermark valve in one host all-reduce, and
        the GLOBAL advance.  Returns the valve's watermark; the GLOBAL rows stay in its handle."""
        from ..runtime.exchange import KeyByExchange
        if self.global_cfg.nullable_cols:
            raise ValueError("step_device moves packed rows, which carry no NULL flags: NOT NULL inputs only")
        if self.exchange is None:
            self.exchange = KeyByExchange(self.global_cfg.key_hash, self.global_cfg.max_parallelism)
        self.local.advance(watermark)
        n, key, _, se, fields, _ = self.local.device_results_async(self.device)
        px = self.exchange.exchange_packed_async(key, se, fields, n_dev=n)
        self.glob.push_device_packed_segments(px.recv_counts, px.rows, px.row_words)
        spill, wm = px.finish(watermark)
        if spill is not None:
            n_sp = spill.numel() // px.row_words
            self.glob.push_device_packed_segments(torch.tensor([n_sp], dtype=torch.int64, device=self.device), spill,
                                                  px.row_words)
        self.glob.advance(wm)
        return wm

    def flush(self):
        """prepareSnapshotPreBarrier of both operators: the local buffer is emitted downstream
        (LocalSlicingWindowAggOperator.java:133-135), then the global buffer is flushed."""
        self.local.flush()
        key, _, se, fields, nm = self.local.device_result_tensors(self.device)
        key, se, fields, nm = key.clone(), se.clone(), [f.clone() for f in fields], nm.clone()
        self.local.reset_results()
        if self.exchange is not None:
            key, se, cols = self.exchange.exchange(key, se, fields + [nm])
            fields, nm = cols[:-1], cols[-1]
        self.global_ingest(key, se, fields, nm)
        self.glob.flush()

    @property
    def num_late_records_dropped(self):
        return self.glob.stats()["num_late_records_dropped"]
