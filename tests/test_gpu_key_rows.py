"""VARCHAR / composite keys on the device, through the ABI only.
fw_key_row_hash computes BinaryRowData.hashCode (BinaryRowData.java:459 -> MurmurHashUtils
.hashBytesByWords :70-170) of each key row from its columns; fw_key_row_images writes the rows'
BinaryRowData images; a FW_KEYHASH_KEYROW operator takes the images (pinned staging, as the JNI shim
copies each key row) and interns them in an HBM table keyed by the bytes (BinaryRowDataKeySelector
.getKey :54, RecordsWindowBuffer.addElement :81-104), routing by their hashCode.  Checked on an
MI355X against the oracle: hashes and images, the golden fixtures with their string keys (with a
snapshot/restore through the operator alone), a randomized stream at parallelism 2 (a wrong hash
routes a row to a subtask that does not own its key group, which the device flags), a p -> p'
key-group restore, and the collection of key rows no state holds any more."""
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


@pytest.mark.parametrize("types", KEY_SHAPES, ids=["-".join(t) for t in KEY_SHAPES])
def test_device_key_row_images_match_oracle(types):
    import torch
    from flink_amd.table.key_rows import KeyRowColumns
    from oracle import oracle as O
    rng = np.random.default_rng(200 + len(types))
    rows = _rand_rows(rng, types, 2000)
    cols = KeyRowColumns.from_rows(rows, types)
    off, img = cols.to(torch.device("cuda", 0)).images_device()
    off, img = off.cpu().numpy(), img.cpu().numpy()
    assert [img[off[i]:off[i + 1]].tobytes() for i in range(len(rows))] == O.key_row_images(cols.fields(), len(types), len(rows))


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
        from flink_amd.table.key_rows import decode_key_row
        res = self.op.process_watermark(w)
        res["key"] = np.array([self.ids[decode_key_row(x, ("VARCHAR",))[0]] for x in res["key_rows"]], np.int64)
        return res

    def snapshot_restore(self):
        # through the operator alone: the blob carries the key rows its state uses
        from flink_amd.table.window_agg import WindowAggOperator
        self.op.prepare_snapshot_pre_barrier()
        blob = self.op.snapshot_state()
        self.op.close()
        self.op = WindowAggOperator(**self.kw).open()
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
    from flink_amd.table.key_rows import KeyRowColumns
    from flink_amd.table.slice_assigners import SliceAssigners
    from flink_amd.table.window_agg import WindowAggOperator
    from oracle import oracle as O
    rng = np.random.default_rng(21)
    types = ("BIGINT", "VARCHAR")
    universe = _rand_rows(rng, types, 300, null_p=0.05)
    aggs = [("COUNT_STAR", 0, "BIGINT"), ("SUM", 0, "BIGINT"), ("MAX", 0, "BIGINT")]
    kw = dict(assigner=SliceAssigners.hopping(0, 3000, 1000), aggs=aggs, value_types=["BIGINT"],
              count_star_index=0, key_type=types, parallelism=2, state_capacity=1 << 14,
              max_batch_rows=1 << 14, output_capacity=1 << 16, key_row_max_bytes=256)
    ops = [WindowAggOperator(subtask_index=i, **kw).open() for i in range(2)]
    ids = _OracleKeys()
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
                got += op.output_rows(res)
            orc.process_watermark(wm)
            r = orc.results(clear=True)
            want = [ids.decode(k) + tuple(int(v[i]) for v in r["values"]) + (int(ws), int(we))
                    for i, (k, ws, we) in enumerate(zip(r["key"], r["window_start"], r["window_end"]))]
            assert sorted(got, key=repr) == sorted(want, key=repr), f"batch {b}"
        assert all(op.handle.stats()["error_flags"] == 0 for op in ops)
    finally:
        for op in ops:
            op.close()
        orc.close()


class _OracleKeys:
    """Test-side ids for the oracle, which keys on int64: one per distinct key row."""

    def __init__(self):
        self.ids, self.rows = {}, []

    def encode(self, rows):
        out = np.empty(len(rows), np.int64)
        for i, r in enumerate(rows):
            k = self.ids.get(r)
            if k is None:
                k = self.ids[r] = len(self.rows)
                self.rows.append(r)
            out[i] = k
        return out

    def decode(self, k):
        return self.rows[int(k)]


def _route(rows, types, p):
    from flink_amd import abi
    from flink_amd.table.key_rows import KeyRowColumns
    from oracle import oracle as O
    kc = KeyRowColumns.from_rows(rows, types)
    h = O.key_row_hash(kc.fields(), len(types), len(rows))
    return np.array([O.operator_index(128, p, O.key_group(abi.KEYHASH_PRECOMPUTED, 0, 128, pre=int(x))) for x in h])


@pytest.mark.parametrize("p_from,p_to,fmt", [(2, 3, "own"), (3, 1, "own"), (2, 3, "heap")])
def test_key_row_rescale_restore_by_key_group(p_from, p_to, fmt):
    """(VARCHAR, BIGINT) keys, CUMULATE: checkpoint at parallelism p_from, restore the key groups
    at p_to through the ABI (each blob carries its key rows; the restoring subtask interns them and
    routes each by its hashCode), continue; the union of results equals one oracle restarted at the
    same cut.  fmt "heap": the key groups travel in the heap backend's bytes
    (fw_snapshot_key_group_heap: key = the key row's BinaryRowData image)."""
    from flink_amd import abi
    from flink_amd.table.slice_assigners import SliceAssigners
    from flink_amd.table.window_agg import WindowAggOperator
    from oracle import oracle as O
    rng = np.random.default_rng(7 + p_from)
    types = ("VARCHAR", "BIGINT")
    universe = _rand_rows(rng, types, 400, null_p=0.05)
    aggs = [("COUNT_STAR", 0, "BIGINT"), ("SUM", 0, "BIGINT"), ("MIN", 0, "BIGINT")]
    kw = dict(assigner=SliceAssigners.cumulative(0, 4000, 1000), aggs=aggs, value_types=["BIGINT"],
              count_star_index=0, key_type=types, state_capacity=1 << 14, max_batch_rows=1 << 13,
              output_capacity=1 << 16, key_row_max_bytes=256)
    ocfg = abi.make_config(api=abi.API_SQL, window_kind=abi.WIN_CUMULATE, size_ms=4000, slide_ms=1000,
                           aggs=[(abi.AGG_NAMES[k], c, abi.TYPE_NAMES[t]) for k, c, t in aggs], count_star_index=0,
                           value_col_types=[abi.T_I64], key_hash=abi.KEYHASH_PRECOMPUTED)
    orc = O.OracleOperator(ocfg)
    ids = _OracleKeys()
    ops = [WindowAggOperator(parallelism=p_from, subtask_index=i, **kw).open() for i in range(p_from)]
    t0 = 1_600_000_000_000
    try:
        for b in range(16):
            if b == 8:  # checkpoint, rescale, restore
                blobs, wms = {}, []
                for op in ops:
                    op.prepare_snapshot_pre_barrier()
                    bl, wm_ = op.handle.snapshot_key_groups()
                    if fmt == "heap":
                        bl = {kg: op.handle.snapshot_key_group_heap(kg) for kg in bl}
                    blobs.update(bl)
                    wms.append(wm_)
                    op.close()
                ops = [WindowAggOperator(parallelism=p_to, subtask_index=i, **kw).open() for i in range(p_to)]
                for op in ops:
                    if fmt == "heap":
                        lo, hi = op.handle.key_group_range()
                        for kg in range(lo, hi + 1):
                            op.handle.restore_key_group_heap(blobs[kg])
                        op.handle.initialize_watermark(min(wms))
                    else:
                        op.handle.restore_key_groups(blobs, wms)
                orc.snapshot_restore()
            p = len(ops)
            rows = [universe[i] for i in rng.integers(0, len(universe), 1500)]
            ts = t0 + b * 600 + rng.integers(-1200, 1200, len(rows))
            val = rng.integers(-1000, 1000, len(rows)).astype(np.int64)
            dest = _route(rows, types, p)
            for d in range(p):
                m = dest == d
                if m.any():
                    ops[d].process_batch([r for r, keep in zip(rows, m) if keep], ts[m], [val[m]])
            orc.process_batch(ids.encode(rows), ts, [val])
            wm = t0 + b * 600 - 1300
            got = []
            for op in ops:
                got += op.output_rows(op.process_watermark(wm))
            orc.process_watermark(wm)
            r = orc.results(clear=True)
            want = [ids.decode(k) + tuple(int(v[i]) for v in r["values"]) + (int(ws), int(we))
                    for i, (k, ws, we) in enumerate(zip(r["key"], r["window_start"], r["window_end"]))]
            assert sorted(got, key=repr) == sorted(want, key=repr), f"batch {b}"
        assert all(op.handle.stats()["error_flags"] == 0 for op in ops)
    finally:
        for op in ops:
            op.close()
        orc.close()


def test_key_rows_no_state_holds_are_collected():
    """A stream whose keys change every few windows: the table keeps only the key rows some state
    entry, pending partial or unread result holds -- collections run, the ids are reused, the
    table never fills although 10x its capacity of distinct keys pass -- and the results stay
    bit-exact against the oracle."""
    from flink_amd import abi
    from flink_amd.table.slice_assigners import SliceAssigners
    from flink_amd.table.window_agg import WindowAggOperator
    from oracle import oracle as O
    rng = np.random.default_rng(3)
    types = ("VARCHAR",)
    aggs = [("COUNT_STAR", 0, "BIGINT"), ("MAX", 0, "BIGINT")]
    op = WindowAggOperator(SliceAssigners.tumbling(0, 2000), aggs, ["BIGINT"], count_star_index=0, key_type=types,
                           state_capacity=2048, max_batch_rows=512, output_capacity=1 << 14).open()
    ocfg = abi.make_config(api=abi.API_SQL, window_kind=abi.WIN_TUMBLE, size_ms=2000,
                           aggs=[(abi.AGG_NAMES[k], c, abi.TYPE_NAMES[t]) for k, c, t in aggs], count_star_index=0,
                           value_col_types=[abi.T_I64], key_hash=abi.KEYHASH_PRECOMPUTED)
    orc = O.OracleOperator(ocfg)
    ids = _OracleKeys()
    t0 = 1_600_000_000_000
    distinct = 0
    max_live = 0
    try:
        for b in range(120):
            gen = b // 3  # a new key population every 3 watermarks
            rows = [(f"k{gen}-{int(x)}",) for x in rng.integers(0, 700, 500)]
            distinct += 0 if b % 3 else 700
            ts = t0 + b * 1000 + rng.integers(0, 1000, len(rows))
            val = rng.integers(0, 10**6, len(rows)).astype(np.int64)
            op.process_batch(rows, ts, [val])
            orc.process_batch(ids.encode(rows), ts, [val])
            wm = t0 + b * 1000 + 999
            got = op.output_rows(op.process_watermark(wm))
            orc.process_watermark(wm)
            r = orc.results(clear=True)
            want = [ids.decode(k) + tuple(int(v[i]) for v in r["values"]) + (int(ws), int(we))
                    for i, (k, ws, we) in enumerate(zip(r["key"], r["window_start"], r["window_end"]))]
            assert sorted(got, key=repr) == sorted(want, key=repr), f"batch {b}"
            st = op.handle.stats()
            assert st["error_flags"] == 0, f"batch {b}: {st}"
            max_live = max(max_live, st["key_rows"])
        st = op.handle.stats()
        assert st["key_row_collections"] > 0
        assert distinct > 4 * (2048 + 8 * 512) and max_live <= 2048 + 8 * 512
    finally:
        op.close()
        orc.close()


def test_key_row_longer_than_the_limit_is_a_device_error():
    from flink_amd._native import FlinkWinError
    from flink_amd.table.slice_assigners import SliceAssigners
    from flink_amd.table.window_agg import WindowAggOperator
    op = WindowAggOperator(SliceAssigners.tumbling(0, 2000), [("COUNT_STAR", 0, "BIGINT")], ["BIGINT"],
                           key_type=("VARCHAR",), state_capacity=1024, max_batch_rows=64, output_capacity=1024,
                           key_row_max_bytes=32).open()
    try:
        with pytest.raises((FlinkWinError, ValueError)):
            op.process_batch([("x" * 100,)], np.array([1_600_000_000_000]), [np.array([1])])
            op.process_watermark(1_600_000_010_000)
    finally:
        op.close()
