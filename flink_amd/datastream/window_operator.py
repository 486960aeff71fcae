"""GPU-backed drop-in for the DataStream WindowOperator on its eligible subset.

WindowOperatorBuilder.buildWindowOperator (flink-runtime/.../windowing/WindowOperatorBuilder.java:432-446)
would return this operator iff: the assigner is TumblingEventTimeWindows or
SlidingEventTimeWindows (any size and slide), the trigger is EventTimeTrigger, there is no
evictor, and the function is a built-in field aggregation (SumAggregator / ComparableAggregator
for min/max and -- record-shaped -- minBy/maxBy with either tie rule, WindowedStream.java:660-880)
on a numeric field.  Any allowedLateness and a
late-data side output (sideOutputLateData) are supported.  Anything else stays on the reference
WindowOperator.

Semantics (WindowOperator.java:293-682): per element, every window that is not late (cleanupTime =
maxTimestamp + allowedLateness > watermark) gets the value; a window the watermark has not
reached gets a timer at window.maxTimestamp(), one it has already passed fires again at once with
the element added (EventTimeTrigger.onElement).  A watermark fires (key, window) timers and emits
(key, aggregate) with record timestamp window.maxTimestamp(); the window state is cleared at its
cleanup time.  Elements late for all their windows go to the late side output when one is set,
else they are counted in numLateRecordsDropped.

Output records.  SumAggregator.reduce (SumAggregator.java:66-76) and ComparableAggregator.reduce
(ComparableAggregator.java:83-104) return value1 -- the window's FIRST element, copied -- with the
aggregated field set, so every non-aggregated field of an output record comes from the first
element.  With ``field`` set the operator is record-shaped: ``process_batch(..., records=...)``
takes the elements themselves, the device tracks each window's first arrival ordinal
(ds_first_ordinals) and tells the operator which elements to keep (fw_first_element_events);
``process_watermark`` then returns the reference's records.
"""
import json
import struct

import numpy as np

from .. import abi
from ..runtime.handle import WindowAggHandle
from ..runtime.options import gpu_enabled
from . import heap_state
from .windowing import EventTimeTrigger, SlidingEventTimeWindows, TumblingEventTimeWindows

_AGG = {"sum": abi.AGG_SUM, "min": abi.AGG_MIN, "max": abi.AGG_MAX, "count": abi.AGG_COUNT_STAR,
        "minBy": abi.AGG_MINBY, "maxBy": abi.AGG_MAXBY}
_BY = ("minBy", "maxBy")
# STRING keys (keyBy a String field): the operator interns each String to a dense int64 id -- the
# device key -- and hands the device its String.hashCode, which routes it exactly as
# KeyGroupRangeAssignment.assignToKeyGroup(key) does (FW_KEYHASH_PRECOMPUTED).  Ids are never
# reused: the table holds every distinct String the operator has seen (and is saved with each
# snapshot), so its host memory grows with the stream's key cardinality, not with the live windows.
# A stream with unbounded String cardinality should stay on the reference operator.
_KEY = {"LONG": abi.KEYHASH_LONG, "INT": abi.KEYHASH_INT, "HOST_HASHED": abi.KEYHASH_PRECOMPUTED,
        "STRING": abi.KEYHASH_PRECOMPUTED}
_TYPE = {"LONG": abi.T_I64, "INT": abi.T_I32, "DOUBLE": abi.T_F64}


def _enc_field(x):
    """a record field for the snapshot's JSON side: floats by their bits (a NaN keeps its payload,
    which minBy / maxBy hand back inside the element)"""
    return {"f64": struct.unpack("<q", struct.pack("<d", x))[0]} if isinstance(x, float) else x


def _dec_field(x):
    return struct.unpack("<d", struct.pack("<q", x["f64"]))[0] if isinstance(x, dict) and "f64" in x else x


def is_gpu_eligible(assigner, trigger, aggregation, *, evictor=None, allowed_lateness=0,
                    late_data_output_tag=None, conf=None):
    """WindowOperatorBuilder.buildWindowOperator's seam.  ``conf``: the job configuration
    (runtime/options.py): ``gpu.window-agg.enabled`` must be true; None = the GPU operator was chosen."""
    if conf is not None and not gpu_enabled(conf):
        return False, "gpu.window-agg.enabled is false"
    if not isinstance(assigner, (TumblingEventTimeWindows, SlidingEventTimeWindows)):
        return False, "assigner is not Tumbling/SlidingEventTimeWindows"
    if isinstance(assigner, SlidingEventTimeWindows) and assigner.size < assigner.slide:
        return False, "sliding windows with gaps (size < slide)"
    if not isinstance(trigger, EventTimeTrigger):
        return False, "custom trigger"
    if evictor is not None:
        return False, "evictor"
    if allowed_lateness < 0:
        return False, "The allowed lateness cannot be negative."
    if aggregation[0] not in _AGG or aggregation[1] not in _TYPE:
        return False, "not a built-in field aggregation"
    if len(aggregation) > 2 and (aggregation[0] not in _BY or not isinstance(aggregation[2], bool)):
        return False, "only minBy / maxBy take a first/last flag"
    return True, ""


class WindowOperator:
    def __init__(self, assigner, trigger, aggregation, key_type="LONG", max_parallelism=128,
                 parallelism=1, subtask_index=0, device=0, state_capacity=1 << 20,
                 max_batch_rows=1 << 22, output_capacity=1 << 22, allowed_lateness=0,
                 late_data_output_tag=None, field=None, record_serializer=None):
        """``field``: position of the aggregated field in the records (``sum(field)``, ...); given,
        the operator emits whole records (value1.copy() with the field set), else (key, agg).
        ``record_serializer``: the records' TypeSerializer restatement (heap_state.TupleSerializer,
        ...), for the heap backend's key-group bytes."""
        ok, why = is_gpu_eligible(assigner, trigger, aggregation, allowed_lateness=allowed_lateness,
                                  late_data_output_tag=late_data_output_tag)
        if not ok:
            raise ValueError(f"not eligible for the GPU window operator: {why}")
        fn, ftype = aggregation[:2]
        if fn in _BY and field is None:
            raise ValueError("minBy / maxBy emit whole elements: a record-shaped operator (field=...) is needed")
        # minBy / maxBy(field, first): ties go to the first element unless first is False
        by_flags = abi.AGGF_LAST if fn in _BY and len(aggregation) > 2 and not aggregation[2] else 0
        sliding = isinstance(assigner, SlidingEventTimeWindows)
        self.assigner = assigner
        self.aggregation = aggregation
        t = _TYPE[ftype]
        self.cfg = abi.make_config(
            api=abi.API_DATASTREAM, window_kind=abi.WIN_HOP if sliding else abi.WIN_TUMBLE,
            size_ms=assigner.size, slide_ms=assigner.slide if sliding else 0,
            offset_ms=assigner.offset, aggs=[(_AGG[fn], 0, t, by_flags)], count_star_index=-1,
            value_col_types=[t], key_hash=_KEY[key_type], max_parallelism=max_parallelism,
            parallelism=parallelism, subtask_index=subtask_index, device=device,
            state_capacity=state_capacity, max_batch_rows=max_batch_rows,
            output_capacity=output_capacity, allowed_lateness_ms=allowed_lateness,
            late_side_output=late_data_output_tag is not None, ds_first_ordinals=field is not None)
        self.late_data_output_tag = late_data_output_tag
        self.field = field
        self.key_type = key_type
        self.allowed_lateness = allowed_lateness
        self.record_serializer = record_serializer
        self.handle = None
        self._pending = {}   # push_seq -> records of that push (not yet flushed into state)
        self._retained = {}  # arrival ordinal -> [record, windows whose first element it is]
        self._wm = -(1 << 63)
        self._kid, self._kstr, self._khash = {}, [], []  # STRING keys: String <-> device id, hashCode

    def open(self):
        self.handle = WindowAggHandle(self.cfg)
        return self

    def close(self):
        if self.handle is not None:
            self.handle.close()
            self.handle = None

    def _intern(self, key):
        """STRING key -> (device id, String.hashCode)"""
        i = self._kid.get(key)
        if i is None:
            i = self._kid[key] = len(self._kstr)
            self._kstr.append(key)
            self._khash.append(heap_state.java_string_hash(key))
        return i, self._khash[i]

    def _key_objects(self, ids):
        """device keys -> the operator's keys (the Strings of a STRING-keyed operator)"""
        if self.key_type != "STRING":
            return ids
        return np.array([self._kstr[int(i)] for i in ids], dtype=object)

    def _intern_batch(self, keys):
        """a batch of STRING keys -> (device ids, String.hashCodes): each distinct String of the batch is
        looked up once.  The table grows with the distinct Strings the operator has seen (ids are not
        reused: a long-running, high-cardinality String stream holds every String it ever saw)."""
        uniq, inv = np.unique(np.asarray([str(k) for k in keys], dtype=object), return_inverse=True)
        ids = np.empty(len(uniq), np.int64)
        hashes = np.empty(len(uniq), np.int32)
        for i, k in enumerate(uniq.tolist()):
            ids[i], hashes[i] = self._intern(k)
        return ids[inv], hashes[inv]

    def process_batch(self, keys, timestamps, values, key_hashes=None, records=None):
        """processElement for a batch; ``records``: the elements themselves (record-shaped
        operator), kept until the device says which ones are first elements of a window.  A
        STRING-keyed operator takes its keys as Python strings."""
        seq0 = self.handle.push_seq
        if self.key_type == "STRING":
            keys, key_hashes = self._intern_batch(keys) if len(keys) else (np.empty(0, np.int64), np.empty(0, np.int32))
        self.handle.push_host(keys, timestamps, [values], key_hashes)
        self._keep(seq0, records, len(keys))

    def process_batch_device(self, keys, timestamps, values, key_hashes=None, records=None):
        if self.key_type == "STRING":
            raise ValueError("a STRING-keyed operator interns its keys on the host (process_batch)")
        seq0 = self.handle.push_seq
        self.handle.push_device(keys, timestamps, [values], key_hashes)
        self._keep(seq0, records, keys.numel())

    def _keep(self, seq0, records, n):
        if self.field is None:
            return
        if records is None or len(records) != n:
            raise ValueError("a record-shaped operator needs the batch's records")
        cap = self.cfg.max_batch_rows
        for i, seq in enumerate(range(seq0, self.handle.push_seq)):  # one push per max_batch_rows rows
            self._pending[seq] = records[i * cap:(i + 1) * cap] if self.handle.push_seq - seq0 > 1 else records

    def _element(self, ord_):
        rec = self._retained.get(int(ord_))
        if rec is not None:
            return rec[0]
        return self._pending[int(ord_) >> 32][int(ord_) & 0xFFFFFFFF]

    def _first_elements(self, first_ord, flushed):
        """The retain events (records -> kept), the results' first elements, then the releases."""
        retain, release = self.handle.first_element_events()
        for o in retain.tolist():
            ent = self._retained.get(o)
            if ent is None:
                self._retained[o] = [self._element(o), 1]
            else:
                ent[1] += 1
        firsts = [self._element(o) for o in first_ord.tolist()]
        for o in release.tolist():
            ent = self._retained[o]
            ent[1] -= 1
            if ent[1] == 0:
                del self._retained[o]
        if flushed:  # every pushed row is in the state now: the batches are no longer needed
            self._pending.clear()
        return firsts

    def process_watermark(self, watermark):
        """Fires all (key, window) timers <= watermark; returns {key, value, timestamp} (and, for
        a record-shaped operator, "records": value1.copy() with the aggregated field set)."""
        self.handle.advance(watermark)
        r = self.handle.results(reset=True)
        out = {"key": self._key_objects(r["key"]), "value": r["values"][0], "timestamp": r["window_end"] - 1,
               "window_start": r["window_start"], "window_end": r["window_end"],
               "values": r["values"], "null_mask": r["null_mask"]}
        if self.field is not None:
            flushed = watermark > self._wm
            out["first_ord"] = r["first_ord"]
            firsts = self._first_elements(r["first_ord"], flushed)
            if self.aggregation[0] in _BY:  # the extremal element itself
                out["records"] = firsts
            else:
                vals = self._field_values(r["values"][0])
                out["records"] = [tuple(f[:self.field]) + (v,) + tuple(f[self.field + 1:]) for f, v in zip(firsts, vals)]
        self._wm = max(self._wm, watermark)
        return out

    def _field_values(self, words):
        fn, ftype = self.aggregation[:2]
        if ftype == "DOUBLE" and fn != "count":
            return [struct.unpack("<d", struct.pack("<q", int(w)))[0] for w in words]
        if ftype == "INT" and fn != "count":
            return [int(np.int32(np.int64(w))) for w in words]
        return [int(w) for w in words]

    def side_output(self):
        """Records routed to the late-data side output since the last call
        (WindowOperator.sideOutput): {key, timestamp, value, push_seq, row}."""
        r = self.handle.late_records()
        return {"key": self._key_objects(r["key"]), "timestamp": r["ts"], "value": r["values"][0], "push_seq": r["push_seq"],
                "row": r["row"]}

    def snapshot_state(self) -> bytes:
        """The device blob; a record-shaped operator appends the first elements it keeps (the
        reference's window state holds them: HeapReducingState's value is value1), a STRING-keyed
        one the Strings behind its device key ids (the blob holds ids)."""
        if self.field is None and self.key_type != "STRING":
            return self.handle.snapshot()
        if self.field is not None:
            self.handle.flush()                          # prepareSnapshotPreBarrier
            self._first_elements(np.empty(0, np.int64), True)  # the flush's retains; batches flushed
        blob = self.handle.snapshot()
        side = {"retained": [[o, [_enc_field(x) for x in r], c] for o, (r, c) in self._retained.items()]}
        if self.key_type == "STRING":
            side["strings"] = self._kstr
        return struct.pack("<q", len(blob)) + blob + json.dumps(side).encode()

    def initialize_state(self, blob: bytes):
        if self.field is None and self.key_type != "STRING":
            self.handle.restore(blob)
            return
        n = struct.unpack_from("<q", blob, 0)[0]
        self.handle.restore(blob[8:8 + n])
        side = json.loads(blob[8 + n:].decode())
        self._retained = {o: [tuple(_dec_field(x) for x in r), c] for o, r, c in side["retained"]}
        self._pending.clear()
        if self.key_type == "STRING":  # the same ids as the snapshotting operator's
            self._kstr = list(side["strings"])
            self._kid = {k: i for i, k in enumerate(self._kstr)}
            self._khash = [heap_state.java_string_hash(k) for k in self._kstr]

    # ---- the heap keyed-state backend's key-group bytes (heap_state.py) -------------------------
    def _cleanup_time(self, end):
        """WindowOperator.cleanupTime (:670-677): maxTimestamp + allowedLateness, Long.MAX_VALUE on overflow"""
        t = end - 1 + self.allowed_lateness
        return t if t < (1 << 63) else (1 << 63) - 1

    def _heap_serializers(self, record_serializer):
        if self.field is None:
            raise ValueError("the heap key-group format holds records: a record-shaped operator (field=...) is needed")
        if self.key_type not in heap_state.KEY_SERIALIZERS:
            raise ValueError(f"the heap key-group format needs LONG, INT or STRING keys, not {self.key_type}")
        ser = record_serializer or self.record_serializer
        if ser is None:
            raise ValueError("no record serializer (record_serializer=...)")
        return heap_state.KEY_SERIALIZERS[self.key_type], ser

    def snapshot_key_group_heap(self, key_group, ids=(0, 1, 2), record_serializer=None) -> bytes:
        """Key group ``key_group`` as a heap-backend savepoint writes it: the "window-contents"
        states (value1 with the field set) and the "window-timers" queues; ids = (window-contents,
        event-time timers, processing-time timers) state ids."""
        kser, vser = self._heap_serializers(record_serializer)
        self.handle.flush()                                # prepareSnapshotPreBarrier
        self._first_elements(np.empty(0, np.int64), True)  # the flush's retains; batches flushed
        w = self.handle.ds_key_group_windows(key_group)
        vals = self._field_values(w["value"])
        f = self.field
        recs = []
        for row, v in zip(w, vals):
            if int(row["flags"]) & abi.DSW_CONTENTS:
                first = self._element(int(row["first_ord"]))
                by = self.aggregation[0] in _BY  # minBy / maxBy: the state holds the element itself
                recs.append(first if by else tuple(first[:f]) + (v,) + tuple(first[f + 1:]))
            else:
                recs.append(None)
        key_of = (lambda i: self._kstr[i]) if self.key_type == "STRING" else None
        return heap_state.write_key_group(key_group, ids, w, recs, kser, vser, self.assigner.size, self._cleanup_time,
                                          key_of=key_of)

    def restore_key_group_heap(self, blob: bytes, ids=(0, 1, 2), record_serializer=None):
        """Adds one key group written in the heap backend's bytes (by this operator or a heap-backend
        WindowOperator) to this subtask, which must own it.  Each restored state's record becomes
        the window's retained first element (its field already holds the aggregate)."""
        kser, vser = self._heap_serializers(record_serializer)
        kg, contents, timers = heap_state.read_key_group(blob, ids, kser, vser)
        fn, ftype = self.aggregation[:2]
        f = self.field

        def field_bits(rec):
            v = rec[f]
            if ftype == "DOUBLE" and fn != "count":
                return struct.unpack("<q", struct.pack("<d", float(v)))[0]
            return int(v)

        base = self.handle.push_seq
        key_id = (lambda k: self._intern(str(k))) if self.key_type == "STRING" else None
        w, kept = heap_state.windows_of(contents, timers, self.assigner.size, self._cleanup_time, field_bits, base << 32,
                                        key_id=key_id)
        self.handle.ds_restore_key_group_windows(kg, w, base + 1)
        for o, rec in kept.items():
            self._retained[o] = [rec, 1]
        return kg

    @property
    def num_late_records_dropped(self):
        return self.handle.stats()["num_late_records_dropped"]

    def output_records(self, res):
        fn, ftype = self.aggregation[:2]
        vals = res["value"]
        if ftype == "DOUBLE" and fn != "count":
            vals = vals.view(np.float64)
        elif ftype == "INT" and fn != "count":
            vals = vals.astype(np.int32)
        return [(k if isinstance(k, str) else int(k), v.item(), int(t)) for k, v, t in zip(res["key"], vals, res["timestamp"])]
