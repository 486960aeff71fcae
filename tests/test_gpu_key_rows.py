"""VARCHAR / composite keys on the device.  fw_key_row_hash computes
BinaryRowData.hashCode (BinaryRowData.java:459 -> MurmurHashUtils.hashBytesByWords :70-170) of
each key row from its columns (strings as offsets + bytes); the window operator routes by it
(FW_KEYHASH_PRECOMPUTED) and keys its state by dictionary ids.  Checked on an MI355X against the
oracle's byte-image restatement, the golden fixtures with their string keys, and a randomized
stream at parallelism 2 (a wrong hash would route a row to a subtask that does not own its key
group, which the device flags)."""
import numpy as np
import pytest

from fixture_runner import load_fixtures, replay
from test_key_rows import KEY_SHAPES, _rand_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("types", KEY_SHAPES, ids=["-".join(t) for t in KEY_SHAPES])
def test_device_key_row_hash_matches_host_and_oracle(types):
    import torch
    from flink_amd.table.key_rows import KeyRowColumns
    from oracle import oracle as O
    rng = np.random.default_rng(100 + len(types))
    rows = _rand_rows(rng, types, 3000)
    cols = KeyRowColumns.from_rows(rows, types)
    want = O.key_row_hash(cols.fields(), len(types), len(rows))
    got = cols.to(torch.device("cuda", 0)).hash_device().cpu().numpy()
    assert np.array_equal(got, want)
    assert np.array_equal(cols.hash_host(), want)


def test_device_key_row_hash_large_batch():
    """A 2^20-row VARCHAR batch: every row's hash equals the host restatement."""
    import torch
    from flink_amd.table.key_rows import KeyRowColumns
    rng = np.random.default_rng(5)
    n = 1 << 20
    lens = rng.integers(0, 40, n).astype(np.int32)
    off = np.zeros(n + 1, np.int32)
    np.cumsum(lens, out=off[1:])
    data = np.concatenate([rng.integers(0, 256, int(off[-1])).astype(np.uint8), np.zeros(4, np.uint8)])
    cols = KeyRowColumns(["VARCHAR"], [None], [off], [data], [None], n)
    dev = torch.device("cuda", 0)
    got = cols.to(dev).hash_device().cpu().numpy()
    assert np.array_equal(got, cols.hash_host())


SQL = [f for f in load_fixtures() if f["config"]["api"] == "SQL" and not f.get("two_phase_only")]


class VarcharKeyAdapter:
    """The fixture's string keys as one-field VARCHAR key rows through WindowAggOperator."""

    def __init__(self, fx):
        from test_gpu_api_layer import _slice_assigner
        from flink_amd.table.window_agg import WindowAggOperator
        c = fx["config"]
        self.names = {v["id"]: k for k, v in fx["keys"].items()}
        self.ids = {k: v["id"] for k, v in fx["keys"].items()}
        self.kw = dict(assigner=_slice_assigner(c), aggs=[tuple(a) for a in c["aggs"]], value_types=c["value_cols"],
                       count_star_index=c.get("count_star_index", -1), key_type=("VARCHAR",),
                       state_capacity=1 << 14, max_batch_rows=1 << 12, output_capacity=1 << 12,
                       nullable_cols=c.get("nullable_cols", []))
        self.op = WindowAggOperator(**self.kw).open()

    def process_batch(self, k, t, h, vals, nulls=None):
        self.op.process_batch([(self.names[int(x)],) for x in k], t, vals, nulls=nulls)

    def process_watermark(self, w):
        res = self.op.process_watermark(w)
        res["key"] = np.array([self.ids[self.op.keys.decode(x)[0]] for x in res["key"]], np.int64)
        return res

    def snapshot_restore(self):
        from flink_amd.table.window_agg import WindowAggOperator
        self.op.prepare_snapshot_pre_barrier()
        blob = self.op.snapshot_state()
        keys = self.op.keys
        self.op.close()
        self.op = WindowAggOperator(**self.kw).open()
        self.op.keys = keys  # the dictionary is host state restored with the operator
        self.op.initialize_state(blob)

    @property
    def late_dropped(self):
        return self.op.num_late_records_dropped


@pytest.mark.parametrize("fx", SQL, ids=[f["name"] for f in SQL])
def test_fixtures_with_varchar_key_rows(fx):
    op = VarcharKeyAdapter(fx)
    try:
        replay(fx, op)
    finally:
        op.op.close()


def test_composite_key_rows_two_subtasks_vs_oracle():
    """(BIGINT, VARCHAR) keys, HOP windows, parallelism 2: rows go to the subtask the oracle's
    key-row hash assigns; each subtask's device-computed hash must agree (else the device flags
    a foreign key group) and the union of results equals one oracle operator."""
    from flink_amd import abi
    from flink_amd.table.key_rows import KeyDictionary, KeyRowColumns
    from flink_amd.table.slice_assigners import SliceAssigners
    from flink_amd.table.window_agg import WindowAggOperator
    from oracle import oracle as O
    rng = np.random.default_rng(21)
    types = ("BIGINT", "VARCHAR")
    universe = _rand_rows(rng, types, 300, null_p=0.05)
    aggs = [("COUNT_STAR", 0, "BIGINT"), ("SUM", 0, "BIGINT"), ("MAX", 0, "BIGINT")]
    kw = dict(assigner=SliceAssigners.hopping(0, 3000, 1000), aggs=aggs, value_types=["BIGINT"],
              count_star_index=0, key_type=types, parallelism=2, state_capacity=1 << 14,
              max_batch_rows=1 << 14, output_capacity=1 << 16)
    ops = [WindowAggOperator(subtask_index=i, **kw).open() for i in range(2)]
    ids = KeyDictionary()
    ocfg = abi.make_config(api=abi.API_SQL, window_kind=abi.WIN_HOP, size_ms=3000, slide_ms=1000,
                           aggs=[(abi.AGG_NAMES[k], c, abi.TYPE_NAMES[t]) for k, c, t in aggs], count_star_index=0,
                           value_col_types=[abi.T_I64], key_hash=abi.KEYHASH_PRECOMPUTED)
    orc = O.OracleOperator(ocfg)
    try:
        t0 = 1_600_000_000_000
        for b in range(12):
            sel = rng.integers(0, len(universe), 2000)
            rows = [universe[i] for i in sel]
            ts = t0 + b * 700 + rng.integers(-1500, 1500, len(rows))
            val = rng.integers(-1000, 1000, len(rows)).astype(np.int64)
            kc = KeyRowColumns.from_rows(rows, types)  # keeps the columns alive while hashing
            h = O.key_row_hash(kc.fields(), 2, len(rows))
            dest = np.array([O.operator_index(128, 2, O.key_group(abi.KEYHASH_PRECOMPUTED, 0, 128, pre=int(x)))
                             for x in h])
            for d in range(2):
                m = dest == d
                if m.any():
                    ops[d].process_batch([r for r, keep in zip(rows, m) if keep], ts[m], [val[m]])
            orc.process_batch(ids.encode(rows), ts, [val])
            wm = t0 + b * 700 - 1600
            got = []
            for op in ops:
                res = op.process_watermark(wm)
                got += [op.keys.decode(k) + (int(ws), int(we)) + tuple(int(v[i]) for v in res["values"])
                        for i, (k, ws, we) in enumerate(zip(res["key"], res["window_start"], res["window_end"]))]
            orc.process_watermark(wm)
            r = orc.results(clear=True)
            want = [ids.decode(k) + (int(ws), int(we)) + tuple(int(v[i]) for v in r["values"])
                    for i, (k, ws, we) in enumerate(zip(r["key"], r["window_start"], r["window_end"]))]
            assert sorted(got, key=repr) == sorted(want, key=repr), f"batch {b}"
        assert all(op.handle.stats()["error_flags"] == 0 for op in ops)
    finally:
        for op in ops:
            op.close()
        orc.close()
