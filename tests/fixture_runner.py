"""Replays a golden event script (tests/golden/*.json) through an operator adapter and checks
the per-watermark output multiset, as the reference harness does with
assertOutputEqualsSorted (TestHarnessUtil / RowDataHarnessAssertor)."""
import glob
import json
import os

import numpy as np

from flink_amd import abi

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixtures():
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.json"))):
        with open(p) as fh:
            d = json.load(fh)
        if isinstance(d, dict) and "steps" in d:
            out.append(d)
    return out


def load_kats():
    with open(os.path.join(GOLDEN_DIR, "slice_assigner_kats.json")) as fh:
        return json.load(fh)


def fixture_config(fx, **overrides):
    c = fx["config"]
    kh = c.get("key_hash", "PRECOMPUTED")
    kw = dict(
        api=abi.API_SQL if c["api"] == "SQL" else abi.API_DATASTREAM,
        window_kind=abi.WINDOW_NAMES[c["window"]],
        size_ms=c["size_ms"], slide_ms=c.get("slide_ms", 0), offset_ms=c.get("offset_ms", 0),
        aggs=[(abi.AGG_NAMES[k], col, abi.TYPE_NAMES[t]) for k, col, t in c["aggs"]],
        count_star_index=c.get("count_star_index", -1),
        value_col_types=[abi.TYPE_NAMES[t] for t in c["value_cols"]],
        key_hash=getattr(abi, "KEYHASH_" + kh),
        state_capacity=1 << 14, max_batch_rows=1 << 12, output_capacity=1 << 12,
        nullable_cols=c.get("nullable_cols", []),
        allowed_lateness_ms=c.get("allowed_lateness_ms", 0),
        late_side_output=c.get("late_side_output", False),
        shift_zone=c.get("shift_zone"),
    )
    kw.update(overrides)
    return abi.make_config(**kw)


def _bits(x):
    return int(np.float64(x).view(np.int64)) if isinstance(x, float) else int(x)


def _row_tuple(key, ws, we, vals, nulls, compare, is_ds):
    # a NULL compares as None whatever its value word holds
    vs = tuple(None if (nulls >> a) & 1 else _bits(vals[a]) for a in compare)
    return (int(key), None if is_ds else int(ws), int(we)) + vs


def replay(fx, op, check_late=True):
    """op: adapter with process_batch(keys, ts, hashes, values) -> None,
    process_watermark(wm) -> dict of result columns, snapshot_restore(), late_dropped."""
    cfg = fx["config"]
    keys = fx["keys"]
    is_ds = cfg["api"] == "DATASTREAM"
    n_aggs = len(cfg["aggs"])
    compare = cfg.get("compare_aggs", list(range(n_aggs)))
    pend = []

    def drain():
        if not pend:
            return
        k = np.array([keys[e["key"]]["id"] for e in pend], np.int64)
        h = np.array([keys[e["key"]]["hash"] for e in pend], np.int32)
        t = np.array([e["ts"] for e in pend], np.int64)
        ncols = len(pend[0]["values"])
        vals = [np.array([_bits(e["values"][c]) for e in pend], np.int64) for c in range(ncols)]
        nulls = None
        if any("nulls" in e for e in pend):
            nulls = {c: np.array([e.get("nulls", [0] * ncols)[c] for e in pend], np.uint8) for c in range(ncols)}
        op.process_batch(k, t, h, vals, nulls)
        pend.clear()

    def rows_of(res):
        return [_row_tuple(res["key"][i], res["window_start"][i], res["window_end"][i],
                           [res["values"][a][i] for a in range(n_aggs)], int(res["null_mask"][i]), compare, is_ds)
                for i in range(len(res["key"]))]

    def expected(rows):
        # expected rows list only the compared aggregates, in compare order
        return sorted(_row_tuple(keys[r["key"]]["id"], r.get("window_start", 0), r["window_end"],
                                 _expand(r["values"], compare, n_aggs), _null_mask(r, compare), compare, is_ds)
                      for r in rows)

    collected = []  # rows of watermarks without a per-watermark expectation (checked by "check")
    for step_no, st in enumerate(fx["steps"]):
        if st["op"] == "element":
            pend.append(st)
            continue
        drain()
        if st["op"] == "snapshot_restore":
            op.snapshot_restore()
            continue
        if st["op"] == "check":
            got, want = sorted(collected), expected(st["expect"])
            assert got == want, f"{fx['name']}: step {step_no}: got {got} want {want}"
            collected.clear()
            continue
        assert st["op"] == "watermark"
        res = op.process_watermark(st["wm"])
        if "expect" not in st:
            collected += rows_of(res)
            continue
        got, want = sorted(rows_of(res)), expected(st["expect"])
        assert got == want, f"{fx['name']}: watermark {st['wm']} (step {step_no}): got {got} want {want}"
    drain()
    assert not collected, f"{fx['name']}: unchecked rows {collected}"
    if "side_output" in fx:  # late side output: multiset of (key, ts, values)
        so = op.side_output()
        got = sorted((int(so["key"][i]), int(so["ts"][i])) + tuple(int(v[i]) for v in so["values"])
                     for i in range(len(so["key"])))
        want = sorted((keys[r["key"]]["id"], r["ts"]) + tuple(_bits(v) for v in r["values"]) for r in fx["side_output"])
        assert got == want, f"{fx['name']}: side output {got} != {want}"
    if check_late and fx["late_dropped"] is not None:
        assert op.late_dropped == fx["late_dropped"], \
            f"{fx['name']}: late dropped {op.late_dropped} != {fx['late_dropped']}"


def _expand(values, compare, n_aggs):
    full = [0] * n_aggs
    for v, a in zip(values, compare):
        full[a] = v
    return full


def _null_mask(r, compare):
    m = 0
    for flag, a in zip(r.get("nulls", []), compare):
        m |= (1 << a) if flag else 0
    return m


class OracleAdapter:
    def __init__(self, fx):
        from oracle.oracle import OracleOperator
        self.op = OracleOperator(fixture_config(fx))

    def process_batch(self, k, t, h, vals, nulls=None):
        self.op.process_batch(k, t, vals, nulls)

    def process_watermark(self, w):
        self.op.process_watermark(w)
        return self.op.results(clear=True)

    def snapshot_restore(self):
        self.op.snapshot_restore()

    def side_output(self):
        return self.op.side_output()

    @property
    def late_dropped(self):
        return self.op.late_dropped


class GpuAdapter:
    """Drives the HIP operator (libflinkwin via flink_amd) through a fixture."""

    def __init__(self, fx, **overrides):
        from flink_amd.runtime.handle import WindowAggHandle
        self._cls = WindowAggHandle
        self.cfg = fixture_config(fx, **overrides)
        self.h = WindowAggHandle(self.cfg)
        self.dropped_before = 0
        self._side = []

    def process_batch(self, k, t, h, vals, nulls=None):
        self.h.push_host(k, t, vals, key_hashes=h, nulls=nulls)

    def process_watermark(self, w):
        self.h.advance(w)
        return self.h.results(reset=True)

    def snapshot_restore(self):
        side = self.h.late_records() if self.cfg.late_side_output else None
        blob = self.h.snapshot()
        self.h.close()
        self.h = self._cls(self.cfg)
        self.h.restore(blob)
        if side is not None:
            self._side.append(side)

    _side = None

    def side_output(self):
        parts = (self._side or []) + [self.h.late_records()]
        return {"key": np.concatenate([p["key"] for p in parts]), "ts": np.concatenate([p["ts"] for p in parts]),
                "values": [np.concatenate([p["values"][c] for p in parts]) for c in range(len(parts[0]["values"]))]}

    @property
    def late_dropped(self):
        return self.h.stats()["num_late_records_dropped"]


class TwoPhaseOracleAdapter:
    """The reference's two-phase plan on the CPU: LocalSlicingWindowAggOperator -> (one subtask,
    no exchange) -> WindowAggOperator with GlobalAggCombiner."""

    def __init__(self, fx):
        from oracle.oracle import OracleOperator
        self._cls = OracleOperator
        one = fixture_config(fx)
        self.local_cfg = fixture_config(fx, agg_phase=abi.PHASE_LOCAL)
        self.global_cfg = abi.global_config(self.local_cfg)
        self.local, self.glob = OracleOperator(self.local_cfg), OracleOperator(self.global_cfg)
        self.n = one.n_aggs

    def process_batch(self, k, t, h, vals, nulls=None):
        self.local.process_batch(k, t, vals, nulls)

    def _forward(self):
        r = self.local.results(clear=True)
        if len(r["key"]):
            nm = r["null_mask"].astype(np.int64)
            self.glob.process_batch(r["key"], r["window_end"], r["values"],
                                    {j: (nm >> j) & 1 for j in range(len(r["values"]))})

    def process_watermark(self, w):
        self.local.process_watermark(w)
        self._forward()
        self.glob.process_watermark(w)
        return self.glob.results(clear=True)

    def snapshot_restore(self):
        self.local.flush()      # LocalSlicingWindowAggOperator.prepareSnapshotPreBarrier
        self._forward()
        self.local.snapshot_restore()
        self.glob.snapshot_restore()

    @property
    def late_dropped(self):
        return self.glob.late_dropped


class TwoPhaseGpuAdapter:
    """The two-phase plan on the GPU (flink_amd.table.two_phase.TwoPhaseWindowAgg); a snapshot
    flushes the local buffer downstream, then checkpoints and restores the GLOBAL operator."""

    def __init__(self, fx):
        from flink_amd.runtime.handle import WindowAggHandle
        from flink_amd.table.two_phase import TwoPhaseWindowAgg
        # one subtask: key groups do not change results, so the fixture's key ids hash as LONG
        # (a two-phase plan needs device-hashable keys: partial rows carry no Java hash)
        self.tp = TwoPhaseWindowAgg(fixture_config(fx, key_hash=abi.KEYHASH_LONG))
        self._handle = WindowAggHandle

    def process_batch(self, k, t, h, vals, nulls=None):
        self.tp.local.push_host(k, t, vals, nulls=nulls)

    def process_watermark(self, w):
        return self.tp.process_watermark(w)

    def snapshot_restore(self):
        self.tp.flush()
        blob = self.tp.glob.snapshot()
        self.tp.glob.close()
        self.tp.glob = self._handle(self.tp.global_cfg)
        self.tp.glob.restore(blob)

    @property
    def late_dropped(self):
        return self.tp.num_late_records_dropped
