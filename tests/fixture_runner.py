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
            out.append(json.load(fh))
    return out


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
    )
    kw.update(overrides)
    return abi.make_config(**kw)


def _row_tuple(key, ws, we, vals, compare, is_ds):
    vs = tuple(int(vals[a]) for a in compare)
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
        vals = [np.array([e["values"][c] for e in pend], np.int64) for c in range(ncols)]
        op.process_batch(k, t, h, vals)
        pend.clear()

    for step_no, st in enumerate(fx["steps"]):
        if st["op"] == "element":
            pend.append(st)
            continue
        drain()
        if st["op"] == "snapshot_restore":
            op.snapshot_restore()
            continue
        assert st["op"] == "watermark"
        res = op.process_watermark(st["wm"])
        got = sorted(_row_tuple(res["key"][i], res["window_start"][i], res["window_end"][i],
                                [res["values"][a][i] for a in range(n_aggs)], compare, is_ds)
                     for i in range(len(res["key"])))
        # expected rows list only the compared aggregates, in compare order
        want = sorted(_row_tuple(keys[r["key"]]["id"], r.get("window_start", 0), r["window_end"],
                                 _expand(r["values"], compare, n_aggs), compare, is_ds)
                      for r in st["expect"])
        assert got == want, f"{fx['name']}: watermark {st['wm']} (step {step_no}): got {got} want {want}"
    drain()
    if check_late:
        assert op.late_dropped == fx["late_dropped"], \
            f"{fx['name']}: late dropped {op.late_dropped} != {fx['late_dropped']}"


def _expand(values, compare, n_aggs):
    full = [0] * n_aggs
    for v, a in zip(values, compare):
        full[a] = v
    return full


class OracleAdapter:
    def __init__(self, fx):
        from oracle.oracle import OracleOperator
        self.op = OracleOperator(fixture_config(fx))

    def process_batch(self, k, t, h, vals):
        self.op.process_batch(k, t, vals)

    def process_watermark(self, w):
        self.op.process_watermark(w)
        return self.op.results(clear=True)

    def snapshot_restore(self):
        self.op.snapshot_restore()

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

    def process_batch(self, k, t, h, vals):
        self.h.push_host(k, t, vals, key_hashes=h)

    def process_watermark(self, w):
        self.h.advance(w)
        return self.h.results(reset=True)

    def snapshot_restore(self):
        blob = self.h.snapshot()
        self.h.close()
        self.h = self._cls(self.cfg)
        self.h.restore(blob)

    @property
    def late_dropped(self):
        return self.h.stats()["num_late_records_dropped"]
