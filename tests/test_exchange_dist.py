"""N > 1 path on CPU: world-size-2 `gloo` run of the keyBy exchange (flink_amd/runtime/exchange.py).

Each rank is one operator subtask (parallelism 2, maxParallelism 128).  It generates its slice
of every global batch (the bench's layout), routes rows to the owner of their key group through
KeyByExchange (host partitioner + all_to_all_single; a third of the batches through the padded
exchange -- fixed-size segments per destination, counts exchanged separately -- and a third
through the packed padded exchange the bench times, one buffer of (key, ts, value) rows),
min-reduces the watermark (StatusWatermarkValve), and feeds a per-subtask operator.  Every batch is routed through the
exchange, so the test checks three things:
  * every received row belongs to this subtask's key-group range
    (KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex, :93-106);
  * no row is lost or duplicated;
  * the union of the two subtasks' window results equals one unsharded operator's results.
The per-subtask operator here is the CPU oracle: this test covers the exchange and the
key-group sharding on CPU.  The GPU operator behind the same sharding is covered by
test_gpu_parity.py::test_sharded_subtasks_match_unsharded_oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flink_amd import abi

WORLD = 2
T0 = 1_600_000_000_000


def _stream(rank, batch, n):
    rng = np.random.default_rng(1000 * batch + rank)
    k = rng.integers(0, 4000, n).astype(np.int64)
    t = (T0 + batch * 3000 + rng.integers(-2500, 3000, n)).astype(np.int64)
    v = rng.integers(-10**6, 10**6, n).astype(np.int64)
    return k, t, v


def _cfg(parallelism, subtask):
    return abi.make_config(window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=2000, count_star_index=0,
                           aggs=[(abi.AGG_COUNT_STAR, 0, abi.T_I64), (abi.AGG_SUM, 0, abi.T_I64),
                                 (abi.AGG_MAX, 0, abi.T_I64)],
                           value_col_types=[abi.T_I64], key_hash=abi.KEYHASH_BINROW_BIGINT,
                           max_parallelism=128, parallelism=parallelism, subtask_index=subtask)


def _rows(r):
    return sorted(zip(r["key"].tolist(), r["window_end"].tolist(), *[v.tolist() for v in r["values"]]))


def _worker(rank, port, n_batches, n, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from flink_amd.runtime.exchange import KeyByExchange
        from oracle.oracle import OracleOperator, key_group, key_group_range

        ex = KeyByExchange(abi.KEYHASH_BINROW_BIGINT, 128)
        lo, hi = key_group_range(128, WORLD, rank)
        op = OracleOperator(_cfg(WORLD, rank))
        rows, received = [], 0
        for b in range(n_batches):
            k, t, v = _stream(rank, b, n)
            my_wm = T0 + b * 3000 - 3000 + 500 * rank  # ranks propose different watermarks
            wm = None
            if b % 3 == 0:
                rk, rt, rv = ex.exchange(torch.from_numpy(k), torch.from_numpy(t), [torch.from_numpy(v)])
            elif b % 3 == 2:  # the bench's packed padded exchange: one buffer of (key, ts, value) rows
                # segments of a quarter batch on odd steps: the overflow round carries the rest
                cap = n // 4 if b % 2 else n
                packed, rc, w, spill, wm = ex.exchange_packed(torch.from_numpy(k), torch.from_numpy(t),
                                                              [torch.from_numpy(v)], cap, watermark=my_wm)
                assert w == 3 and packed.numel() == WORLD * cap * w
                seg = packed.view(WORLD, cap, w)
                keep = torch.arange(cap)[None, :] < rc[:, None]
                rk, rt, rv = seg[..., 0][keep], seg[..., 1][keep], [seg[..., 2][keep]]
                assert (spill is not None) == bool(b % 2)
                if spill is not None:
                    sp = spill.view(-1, w)
                    rk, rt, rv = torch.cat([rk, sp[:, 0]]), torch.cat([rt, sp[:, 1]]), [torch.cat([rv[0], sp[:, 2]])]
            else:  # the padded exchange: fixed segments + device-side counts, one all-to-all per column
                cap = n  # a subtask never gets more than all of one sender's rows
                pk, pt, pv, rc = ex.exchange_padded(torch.from_numpy(k), torch.from_numpy(t), [torch.from_numpy(v)], cap)
                assert pk.numel() == WORLD * cap
                keep = (torch.arange(WORLD * cap) % cap) < rc.repeat_interleave(cap)
                rk, rt, rv = pk[keep], pt[keep], [pv[0][keep]]
                ex.check_capacity()
            received += rk.numel()
            kgs = {key_group(abi.KEYHASH_BINROW_BIGINT, int(x), 128) for x in np.unique(rk.numpy())}
            assert all(lo <= g <= hi for g in kgs), f"rank {rank}: foreign key group"
            op.process_batch(rk.numpy(), rt.numpy(), [rv[0].numpy()])
            # the valve takes the min (agreed with the overflow decision in exchange_packed)
            if wm is None:
                wm = ex.global_watermark(my_wm)
            assert wm == T0 + b * 3000 - 3000
            op.process_watermark(wm)
            rows += _rows(op.results())
        op.process_watermark(T0 + n_batches * 3000 + 60000)
        rows += _rows(op.results())
        out_q.put((rank, received, rows, op.late_dropped))
        op.close()
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_two_subtasks_union_equals_unsharded():
    from oracle.oracle import OracleOperator

    n_batches, n = 8, 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, n_batches, n, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert sum(r[1] for r in res) == WORLD * n_batches * n  # nothing lost or duplicated
    got = sorted(row for r in res for row in r[2])

    # one unsharded subtask over the same global stream and watermarks
    op = OracleOperator(_cfg(1, 0))
    want = []
    for b in range(n_batches):
        cols = [_stream(r, b, n) for r in range(WORLD)]
        op.process_batch(*[np.concatenate([c[i] for c in cols]) for i in (0, 1)], [np.concatenate([c[2] for c in cols])])
        op.process_watermark(T0 + b * 3000 - 3000)
        want += _rows(op.results())
    op.process_watermark(T0 + n_batches * 3000 + 60000)
    want += _rows(op.results())
    assert sum(r[3] for r in res) == op.late_dropped
    assert len(got) > 1000 and got == sorted(want)
    op.close()


def _worker_two_phase(rank, port, n_batches, n, out_q):
    """Two-phase plan on CPU: oracle LOCAL per source subtask -> keyBy exchange of the partial rows
    (key, slice end, accumulator fields, null mask) -> oracle GLOBAL per subtask."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from flink_amd.runtime.exchange import KeyByExchange
        from oracle.oracle import OracleOperator, key_group, key_group_range

        ex = KeyByExchange(abi.KEYHASH_BINROW_BIGINT, 128)
        lo, hi = key_group_range(128, WORLD, rank)
        one = _cfg(WORLD, rank)
        local_cfg = abi.make_config(window_kind=one.window_kind, size_ms=one.size_ms, slide_ms=one.slide_ms,
                                    count_star_index=one.count_star_index,
                                    aggs=[(one.aggs[i].kind, one.aggs[i].input_col, one.aggs[i].type) for i in range(one.n_aggs)],
                                    value_col_types=[abi.T_I64], key_hash=abi.KEYHASH_BINROW_BIGINT,
                                    agg_phase=abi.PHASE_LOCAL)
        glob_cfg = abi.global_config(local_cfg, parallelism=WORLD, subtask_index=rank)
        local, glob = OracleOperator(local_cfg), OracleOperator(glob_cfg)
        rows, partials = [], 0
        for b in range(n_batches):
            k, t, v = _stream(rank, b, n)
            local.process_batch(k, t, [v])
            wm = ex.global_watermark(T0 + b * 3000 - 3000 + 500 * rank)
            local.process_watermark(wm)
            r = local.results()
            nf = len(r["values"])
            rk, rse, cols = ex.exchange(torch.from_numpy(r["key"]), torch.from_numpy(r["window_end"]),
                                        [torch.from_numpy(x) for x in r["values"]] +
                                        [torch.from_numpy(r["null_mask"].astype(np.int64))])
            partials += rk.numel()
            kgs = {key_group(abi.KEYHASH_BINROW_BIGINT, int(x), 128) for x in np.unique(rk.numpy())}
            assert all(lo <= g <= hi for g in kgs), f"rank {rank}: foreign key group"
            nm = cols[-1].numpy()
            glob.process_batch(rk.numpy(), rse.numpy(), [c.numpy() for c in cols[:nf]],
                               {j: (nm >> j) & 1 for j in range(nf)})
            glob.process_watermark(wm)
            rows += _rows(glob.results())
        local.process_watermark(T0 + n_batches * 3000 + 60000)
        r = local.results()
        rk, rse, cols = ex.exchange(torch.from_numpy(r["key"]), torch.from_numpy(r["window_end"]),
                                    [torch.from_numpy(x) for x in r["values"]] +
                                    [torch.from_numpy(r["null_mask"].astype(np.int64))])
        nm = cols[-1].numpy()
        glob.process_batch(rk.numpy(), rse.numpy(), [c.numpy() for c in cols[:-1]],
                           {j: (nm >> j) & 1 for j in range(len(cols) - 1)})
        glob.process_watermark(T0 + n_batches * 3000 + 60000)
        rows += _rows(glob.results())
        out_q.put((rank, partials, rows, glob.late_dropped))
        local.close()
        glob.close()
    finally:
        dist.destroy_process_group()


def test_gloo_two_phase_union_equals_one_phase():
    """LocalSlicingWindowAggOperator + GlobalAggCombiner across two subtasks (only partial rows on
    the wire) produce exactly the one-phase results of one unsharded operator."""
    from oracle.oracle import OracleOperator

    n_batches, n = 8, 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_two_phase, args=(r, port, n_batches, n, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = sorted(row for r in res for row in r[2])
    assert sum(r[1] for r in res) < WORLD * n_batches * n  # fewer partial rows than records on the wire
    op = OracleOperator(_cfg(1, 0))
    want = []
    for b in range(n_batches):
        cols = [_stream(r, b, n) for r in range(WORLD)]
        op.process_batch(*[np.concatenate([c[i] for c in cols]) for i in (0, 1)], [np.concatenate([c[2] for c in cols])])
        op.process_watermark(T0 + b * 3000 - 3000)
        want += _rows(op.results())
    op.process_watermark(T0 + n_batches * 3000 + 60000)
    want += _rows(op.results())
    assert len(got) > 1000 and got == sorted(want)
    op.close()


def _worker_device_valve(rank, port, n_batches, n, out_q):
    """PackedExchange.finish_device + settle (the device-side watermark valve, here on CPU tensors):
    every row arrives once (segment or one-step-late overflow round), the watermark is the minimum
    proposal, held at the previous one on a step whose overflow round is still outstanding."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from flink_amd.runtime.exchange import KeyByExchange
        from oracle.oracle import key_group, key_group_range

        ex = KeyByExchange(abi.KEYHASH_BINROW_BIGINT, 128)
        lo, hi = key_group_range(128, WORLD, rank)
        got, wms, agreed, prev_px, prev_wm = [], [], [], None, None
        LMIN = -(1 << 63)

        def take(rows_, w):
            sp = rows_.view(-1, w)
            got.extend(zip(sp[:, 0].tolist(), sp[:, 1].tolist(), sp[:, 2].tolist()))

        for b in range(n_batches):
            if prev_px is not None:
                spill = prev_px.settle()
                agreed.append(prev_px.agreed_watermark)
                if spill is not None:
                    take(spill, prev_px.row_words)
            k, t, v = _stream(rank, b, n)
            cap = n // 4 if b % 2 else n  # odd steps overflow
            px = ex.exchange_packed_async(torch.from_numpy(k), torch.from_numpy(t), [torch.from_numpy(v)], cap)
            seg = px.rows.view(WORLD, cap, px.row_words)
            keep = torch.arange(cap)[None, :] < px.recv_counts.clamp(max=cap)[:, None]
            take(seg[keep].reshape(-1), px.row_words)
            # step 0: rank 0 proposes Long.MIN_VALUE (no watermark yet), which the valve must carry
            wm = px.finish_device(LMIN if b == 0 and rank == 0 else T0 + b * 3000 - 3000 + 500 * rank, prev_wm)
            wms.append(int(wm.item()))
            prev_px, prev_wm = px, wm
        spill = prev_px.settle()
        agreed.append(prev_px.agreed_watermark)
        if spill is not None:
            take(spill, prev_px.row_words)
        assert agreed == [LMIN] + [T0 + b * 3000 - 3000 for b in range(1, n_batches)]
        assert all(lo <= key_group(abi.KEYHASH_BINROW_BIGINT, int(x), 128) <= hi for x in {r[0] for r in got})
        out_q.put((rank, sorted(got), wms, ex.spill_rounds))
    finally:
        dist.destroy_process_group()


def test_gloo_device_valve_holds_watermark_until_overflow_round():
    from oracle.oracle import operator_indices
    n_batches, n = 6, 2000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_device_valve, args=(r, port, n_batches, n, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every row reached its key group's subtask exactly once
    for r in range(WORLD):
        want = []
        for b in range(n_batches):
            for src in range(WORLD):
                k, t, v = _stream(src, b, n)
                m = operator_indices(abi.KEYHASH_BINROW_BIGINT, k, 128, WORLD) == r
                want += zip(k[m].tolist(), t[m].tolist(), v[m].tolist())
        assert res[r][1] == sorted(want)
    # the valve: rank 0's proposal (the minimum), held at the previous value on the overflowing steps
    assert res[0][2] == res[1][2]
    expect = [T0 + b * 3000 - 3000 if b % 2 == 0 else T0 + (b - 1) * 3000 - 3000 for b in range(n_batches)]
    expect[0] = expect[1] = -(1 << 63)  # step 0 is Long.MIN_VALUE; step 1 overflows and holds it
    assert res[0][2] == expect
    assert res[0][3] == n_batches // 2


def _worker_rank_load(rank, port, n_batches, n, out_q):
    """bench.rank_load on CPU: each rank routes its slice of every batch by destination subtask
    (the oracle's computeKeyGroupRangeForOperatorIndex) and the collective returns the job-wide shares."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import bench
        from oracle.oracle import operator_indices
        owned = torch.zeros(WORLD, dtype=torch.int64)
        for b in range(n_batches):
            k, _, _ = _stream(rank, b, n)
            owned += torch.bincount(torch.from_numpy(operator_indices(abi.KEYHASH_BINROW_BIGINT, k, 128, WORLD)).long(),
                                    minlength=WORLD)
        out_q.put((rank, bench.rank_load(owned, 0.5 + rank, 100 * (rank + 1), WORLD)))
    finally:
        dist.destroy_process_group()


def test_bench_rank_load_fields_sum_to_all_events():
    """The N > 1 BENCH line's per-rank block (bench.rank_load): present on every
    rank, the per-subtask event shares sum to N * B * steps, the imbalance is max / mean of them, and
    every rank's wall clock and ingested partials are gathered."""
    n_batches, n = 3, 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_rank_load, args=(r, port, n_batches, n, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    r = res[0]
    ev = r["events_owned_per_rank"]
    assert len(ev) == WORLD and sum(ev) == r["events_total"] == WORLD * n_batches * n
    assert min(ev) > 0 and r["key_group_imbalance_max_over_mean"] == pytest.approx(max(ev) / (sum(ev) / WORLD))
    assert r["rank_elapsed_s"] == [0.5, 1.5] and r["partials_ingested_per_rank"] == [100, 200]


SIZES_GROWING = [2000, 2600, 3400, 4400, 5700, 1500]  # +30 % a step, then a small step


def _worker_growing_shares(rank, port, out_q):
    """The device-counted packed exchange with the segment size LEARNED (capacity=None: the previous
    step's agreed largest share + KeyByExchange.headroom): batches growing ~30 % a step overflow their
    segments on every step after the first, so the overflow round and the held watermark repeat on
    consecutive steps (settle-time advance under repeated overflow)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from flink_amd.runtime.exchange import KeyByExchange

        ex = KeyByExchange(abi.KEYHASH_BINROW_BIGINT, 128)
        got, wms, agreed, caps, prev_px, prev_wm = [], [], [], [], None, None

        def take(rows_, w):
            sp = rows_.view(-1, w)
            got.extend(zip(sp[:, 0].tolist(), sp[:, 1].tolist(), sp[:, 2].tolist()))

        for b, n in enumerate(SIZES_GROWING):
            if prev_px is not None:
                spill = prev_px.settle()
                agreed.append(prev_px.agreed_watermark)
                if spill is not None:
                    take(spill, prev_px.row_words)
            k, t, v = _stream(rank, b, n)
            px = ex.exchange_packed_async(torch.from_numpy(k), torch.from_numpy(t), [torch.from_numpy(v)])
            cap = px.rows.numel() // (WORLD * px.row_words)
            caps.append(cap)
            seg = px.rows.view(WORLD, cap, px.row_words)
            keep = torch.arange(cap)[None, :] < px.recv_counts.clamp(max=cap)[:, None]
            take(seg[keep].reshape(-1), px.row_words)
            wm = px.finish_device(T0 + b * 3000 - 3000 + 500 * rank, prev_wm)
            wms.append(int(wm.item()))
            prev_px, prev_wm = px, wm
        spill = prev_px.settle()
        agreed.append(prev_px.agreed_watermark)
        if spill is not None:
            take(spill, prev_px.row_words)
        out_q.put((rank, sorted(got), wms, agreed, caps, ex.spill_rounds))
    finally:
        dist.destroy_process_group()


def test_gloo_learned_segments_repeated_overflow():
    from oracle.oracle import operator_indices
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_growing_shares, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # row parity: every row reached its key group's subtask exactly once, through 4 overflow rounds
    for r in range(WORLD):
        want = []
        for b, n in enumerate(SIZES_GROWING):
            for src in range(WORLD):
                k, t, v = _stream(src, b, n)
                m = operator_indices(abi.KEYHASH_BINROW_BIGINT, k, 128, WORLD) == r
                want += zip(k[m].tolist(), t[m].tolist(), v[m].tolist())
        assert res[r][1] == sorted(want)
    wm = [T0 + b * 3000 - 3000 for b in range(len(SIZES_GROWING))]
    for r in range(WORLD):
        _, _, wms, agreed, caps, spills = res[r]
        assert caps == res[0][4]  # every subtask picked the same (learned) segment size
        assert caps[1] < caps[2] < caps[3] < caps[4]  # ... tracking the growing share
        assert spills == 4  # steps 1..4 overflowed, step 5 (small) did not
        assert agreed == wm  # the valve's minimum every step
        # the device watermark holds at the last non-overflowing step's, then catches up
        assert wms == [wm[0]] * 5 + [wm[5]]
