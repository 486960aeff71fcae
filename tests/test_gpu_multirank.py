"""The N > 1 HIP path across real ranks: two spawned processes, one operator subtask each
(parallelism 2, maxParallelism 128), a gloo process group, both on the one GPU of the box.

Every rank runs the bench's step functions on its own WindowAggHandle(s):
  * one-phase: KeyByExchange.exchange_packed_async (fw_partition_packed_spill + the packed
    all-to-all) -> fw_push_device_packed_segments -> PackedExchange.finish (overflow round and the
    watermark valve) -> the overflow round's spill push -> fw_advance.  Every other step uses
    segments of a quarter of the even share, so the overflow round runs;
  * two-phase: TwoPhaseWindowAgg.step_device (LOCAL advance -> fw_results_device ->
    fw_partition_packed_spill_dn by the device-side row count -> all-to-all -> GLOBAL ingest ->
    valve -> GLOBAL advance), with the segment size forced small on some steps so the partial rows
    spill too.
Ranks propose different watermarks; the valve takes their minimum (StatusWatermarkValve.java:153).

The union of the ranks' window results must equal ONE unsharded oracle operator over the same
global stream and the valve's watermarks: integers, window bounds and MIN/MAX bit-exact, DOUBLE
SUM/AVG within 1e-9 relative.  Reference seams: KeyGroupStreamPartitioner.java:55-65,
KeyGroupRangeAssignment.java:93-127, TwoStageOptimizedWindowAggregateRule.java:80-109.

The children initialise the GPU themselves (spawn start method: nothing of the parent's GPU state
is inherited) and exchange through host memory (gloo stages device tensors); the driver's N > 1
runs use RCCL, whose only difference is the transport of the same buffers.
"""
import os
import socket

import numpy as np
import pytest

from flink_amd import abi

from parity_common import REL_TOL

pytestmark = pytest.mark.gpu

WORLD = 2
T0 = 1_600_000_000_000
STEP = 3000
I64, F64 = abi.T_I64, abi.T_F64

SCENARIOS = {
    # one-phase keyBy of raw rows, HOP with the hidden COUNT(*) (uniform keys)
    "one_phase_hop": dict(plan="one", dist="uniform",
                          kw=dict(window_kind=abi.WIN_HOP, size_ms=6000, slide_ms=2000, count_star_index=0,
                                  aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64), (abi.AGG_MAX, 0, I64)],
                                  value_col_types=[I64])),
    # one-phase TUMBLE over DOUBLE (CFG4's aggregates)
    "one_phase_tumble_double": dict(plan="one", dist="uniform",
                                    kw=dict(window_kind=abi.WIN_TUMBLE, size_ms=5000,
                                            aggs=[(abi.AGG_SUM, 0, F64), (abi.AGG_AVG, 0, F64), (abi.AGG_MAX, 0, F64)],
                                            value_col_types=[F64])),
    # two-phase CUMULATE, COUNT(*) / SUM / MIN / MAX over Zipf keys (CFG5's plan)
    "two_phase_cumulate_zipf": dict(plan="two", dist="zipf",
                                    kw=dict(window_kind=abi.WIN_CUMULATE, size_ms=12000, slide_ms=3000, count_star_index=0,
                                            aggs=[(abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_SUM, 0, I64),
                                                  (abi.AGG_MIN, 0, I64), (abi.AGG_MAX, 0, I64)],
                                            value_col_types=[I64])),
    # two-phase HOP over Zipf keys
    "two_phase_hop_zipf": dict(plan="two", dist="zipf",
                               kw=dict(window_kind=abi.WIN_HOP, size_ms=8000, slide_ms=2000, count_star_index=1,
                                       aggs=[(abi.AGG_SUM, 0, I64), (abi.AGG_COUNT_STAR, 0, I64), (abi.AGG_MIN, 0, I64)],
                                       value_col_types=[I64])),
    # two-phase TUMBLE SUM / AVG(DOUBLE) (CFG4's plan at N > 1)
    "two_phase_tumble_double": dict(plan="two", dist="uniform",
                                    kw=dict(window_kind=abi.WIN_TUMBLE, size_ms=6000,
                                            aggs=[(abi.AGG_SUM, 0, F64), (abi.AGG_AVG, 0, F64)],
                                            value_col_types=[F64])),
}
# the same steps with the watermark valve on the device (PackedExchange.finish_device -> one device
# all-reduce of (overflow, watermark, share) -> fw_advance_device; overflow rounds settled one step
# late, the watermark held at the previous one meanwhile)
for _n in ("one_phase_hop", "one_phase_tumble_double", "two_phase_cumulate_zipf", "two_phase_hop_zipf"):
    SCENARIOS[_n + "_device_valve"] = dict(SCENARIOS[_n], valve="device")
# segments sized as the bench sizes them -- the previous step's agreed largest share plus a headroom
# (KeyByExchange.headroom) -- with the headroom negative, so every step after the first overflows its
# segments and the overflow round carries the rest (host and device valves)
for _n, _v in (("one_phase_hop_share_sizing", "host"), ("one_phase_tumble_double_share_sizing_device_valve", "device")):
    SCENARIOS[_n] = dict(SCENARIOS["one_phase_hop" if "hop" in _n else "one_phase_tumble_double"], valve=_v,
                         cap="share", headroom=-0.15)
N_BATCHES = 9
N_ROWS = 24000  # per rank per batch


def _stream(dist_kind, value_type, rank, batch, n):
    """Rank `rank`'s slice of global batch `batch`: out-of-order timestamps around the batch's
    interval (some records late for the valve's watermark), uniform or Zipf keys."""
    rng = np.random.default_rng(7919 * batch + 31 * rank + 5)
    if dist_kind == "zipf":
        k = (rng.zipf(1.3, n) % 20000).astype(np.int64) * 104729 - 7
    else:
        k = rng.integers(0, 6000, n).astype(np.int64) * 7919 + 13
    t = (T0 + batch * STEP + rng.integers(-2500, STEP, n)).astype(np.int64)
    if value_type == F64:
        v = (rng.random(n) * 1000.0).view(np.int64)
    else:
        v = rng.integers(-10**6, 10**6, n).astype(np.int64)
    return k, t, v


def _proposed_wm(batch, rank):
    return T0 + batch * STEP - STEP + 700 * rank  # the valve's minimum is rank 0's


FINAL_WM = T0 + N_BATCHES * STEP + 120_000


def _cfg(kw, parallelism, subtask, **extra):
    d = dict(kw)
    d.update(key_hash=abi.KEYHASH_BINROW_BIGINT, max_parallelism=128, parallelism=parallelism,
             subtask_index=subtask, state_capacity=1 << 16, max_batch_rows=1 << 17, output_capacity=1 << 18)
    d.update(extra)
    return abi.make_config(**d)


def _rows(res, n_aggs):
    return [(int(res["key"][i]), int(res["window_start"][i]), int(res["window_end"][i]),
             tuple(int(res["values"][a][i]) for a in range(n_aggs)), int(res["null_mask"][i]))
            for i in range(len(res["key"]))]


def _worker(rank, port, name, out_q, world=WORLD, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        if backend == "nccl":  # RCCL: the device all-to-all and the device valve's all-reduce
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        from flink_amd.runtime.exchange import KeyByExchange
        from flink_amd.runtime.handle import WindowAggHandle
        from flink_amd.table.two_phase import TwoPhaseWindowAgg

        sc = SCENARIOS[name]
        kw = sc["kw"]
        vt = kw["value_col_types"][0]
        cfg = _cfg(kw, world, rank)
        n_aggs = cfg.n_aggs
        ex = KeyByExchange(abi.KEYHASH_BINROW_BIGINT, 128, force_collectives=backend == "nccl")
        share_sizing = sc.get("cap") == "share"
        if share_sizing:
            ex.headroom = sc["headroom"]
        rows, wms, received = [], [], 0
        device_valve = sc.get("valve") == "device"
        if sc["plan"] == "one" and device_valve:
            h = WindowAggHandle(cfg)
            px_prev, wm_prev = None, None

            def settle(px):
                nonlocal received
                spill = px.settle()
                if spill is not None:
                    n_sp = spill.numel() // px.row_words
                    received += n_sp
                    h.push_device_packed_segments(torch.tensor([n_sp], dtype=torch.int64, device=dev), spill,
                                                  px.row_words)
            for b in range(N_BATCHES):
                if px_prev is not None:
                    settle(px_prev)
                k, t, v = (torch.from_numpy(x).to(dev) for x in _stream(sc["dist"], vt, rank, b, N_ROWS))
                cap = None if share_sizing else ex.segment_capacity(N_ROWS, world) if b % 2 == 0 else N_ROWS // (4 * world)
                px = ex.exchange_packed_async(k, t, [v], capacity=cap)
                h.push_device_packed_segments(px.recv_counts, px.rows, px.row_words)
                received += int(px.recv_counts.clamp(max=px._cap).sum())
                wm_t = px.finish_device(_proposed_wm(b, rank), wm_prev)
                h.advance_device(wm_t)
                px_prev, wm_prev = px, wm_t
                wms.append(int(wm_t.item()))  # (the test reads it back; the step itself never waits)
                rows += _rows(h.results(), n_aggs)
            settle(px_prev)
            h.advance(FINAL_WM)
            rows += _rows(h.results(), n_aggs)
            st = h.stats()
            h.close()
        elif sc["plan"] == "one":
            h = WindowAggHandle(cfg)
            for b in range(N_BATCHES):
                k, t, v = (torch.from_numpy(x).to(dev) for x in _stream(sc["dist"], vt, rank, b, N_ROWS))
                # odd steps: segments of a quarter of the even share -> the overflow round carries the rest
                cap = None if share_sizing else ex.segment_capacity(N_ROWS, world) if b % 2 == 0 else N_ROWS // (4 * world)
                px = ex.exchange_packed_async(k, t, [v], capacity=cap)
                h.push_device_packed_segments(px.recv_counts, px.rows, px.row_words)
                spill, wm = px.finish(watermark=_proposed_wm(b, rank))
                received += int(px.recv_counts.clamp(max=px._cap).sum())  # rows past a segment come in the spill
                if spill is not None:
                    n_sp = spill.numel() // px.row_words
                    received += n_sp
                    h.push_device_packed_segments(torch.tensor([n_sp], dtype=torch.int64, device=dev), spill,
                                                  px.row_words)
                h.advance(wm)
                wms.append(wm)
                rows += _rows(h.results(), n_aggs)
            h.advance(FINAL_WM)
            rows += _rows(h.results(), n_aggs)
            st = h.stats()
            h.close()
        else:
            tp = TwoPhaseWindowAgg(cfg, exchange=ex, device=dev, local_state_capacity=1 << 17)
            for b in range(N_BATCHES + 1):
                if b < N_BATCHES:
                    k, t, v = (torch.from_numpy(x).to(dev) for x in _stream(sc["dist"], vt, rank, b, N_ROWS))
                    tp.local.push_device(k, t, [v])
                if b % 3 == 1:  # segments far below the partials' share: their overflow round runs
                    if device_valve:
                        tp.settle()  # (it sets the agreed share; overridden for this step)
                    ex._dn_share = 64
                wm_prop = _proposed_wm(b, rank) if b < N_BATCHES else FINAL_WM
                if device_valve:
                    wm = int(tp.step_device_valve(wm_prop).item())
                else:
                    wm = tp.step_device(wm_prop)
                wms.append(wm)
                rows += _rows(tp.glob.results(), n_aggs)
            if device_valve:  # the last step's overflow round, then its watermark
                tp.settle()
                tp.glob.advance(FINAL_WM)
                rows += _rows(tp.glob.results(), n_aggs)
            st = tp.glob.stats()
            st["error_flags"] |= tp.local.stats()["error_flags"]
            tp.close()
        torch.cuda.synchronize()
        lo, hi = (rank * 128 + world - 1) // world, ((rank + 1) * 128 - 1) // world
        out_q.put((rank, dict(rows=rows, wms=wms, received=received, spill_rounds=ex.spill_rounds,
                              backend=dist.get_backend(), collectives=ex.collectives,
                              late=st["num_late_records_dropped"], err=st["error_flags"], kg=(lo, hi))))
    except Exception as e:  # reported to the parent, which fails the test with it
        import traceback
        out_q.put((rank, dict(error=f"{type(e).__name__}: {e}\n{traceback.format_exc()}")))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(name, world=WORLD, backend="gloo"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, name, q, world, backend)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=180) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert "error" not in res[r], f"rank {r}: {res[r]['error']}"
    for p in procs:
        assert p.exitcode == 0
    return res


def _oracle_rows(name, wms, world=WORLD):
    """One unsharded operator (parallelism 1) over the global stream and the valve's watermarks."""
    from oracle.oracle import OracleOperator
    sc = SCENARIOS[name]
    kw = sc["kw"]
    vt = kw["value_col_types"][0]
    op = OracleOperator(_cfg(kw, 1, 0))
    want = []
    for b in range(N_BATCHES):
        cols = [_stream(sc["dist"], vt, r, b, N_ROWS) for r in range(world)]
        op.process_batch(np.concatenate([c[0] for c in cols]), np.concatenate([c[1] for c in cols]),
                         [np.concatenate([c[2] for c in cols])])
        op.process_watermark(wms[b])
        want += _rows(op.results(clear=True), op.cfg.n_aggs)
    op.process_watermark(FINAL_WM)
    want += _rows(op.results(clear=True), op.cfg.n_aggs)
    late = op.late_dropped
    op.close()
    return want, late


def _compare(got, want, double_cols, ctx):
    got, want = sorted(got), sorted(want)
    assert len(got) == len(want), f"{ctx}: {len(got)} rows vs oracle {len(want)}"
    for g, w in zip(got, want):
        assert g[:3] == w[:3] and g[4] == w[4], f"{ctx}: {g} vs {w}"
        for a, (x, y) in enumerate(zip(g[3], w[3])):
            if a in double_cols:
                xd, yd = float(np.int64(x).view(np.float64)), float(np.int64(y).view(np.float64))
                assert xd == pytest.approx(yd, rel=REL_TOL, abs=0.0), f"{ctx}: agg {a} {xd} vs {yd}"
            else:
                assert x == y, f"{ctx}: agg {a} {x} != {y} ({g} vs {w})"


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_two_ranks_union_equals_unsharded_oracle(name):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.oracle import key_group
    res = _run_ranks(name)
    sc = SCENARIOS[name]
    # the ranks agreed on every watermark: the valve's minimum, rank 0's proposal -- or, with the device
    # valve, the previous watermark held while an overflow round is outstanding
    assert res[0]["wms"] == res[1]["wms"]
    wms = res[0]["wms"][:N_BATCHES]
    if sc.get("valve") == "device":
        held = [b for b in range(N_BATCHES) if wms[b] != _proposed_wm(b, 0)]
        assert held and all(wms[b] == (wms[b - 1] if b else -(1 << 63)) for b in held)
    else:
        assert wms == [_proposed_wm(b, 0) for b in range(N_BATCHES)]
    assert all(res[r]["err"] == 0 for r in range(WORLD))
    # the overflow rounds ran (the spill path is exercised), on both ranks alike
    assert res[0]["spill_rounds"] > 0 and res[0]["spill_rounds"] == res[1]["spill_rounds"]
    if sc["plan"] == "one":  # every raw row arrived exactly once
        assert res[0]["received"] + res[1]["received"] == WORLD * N_BATCHES * N_ROWS
    # each rank emitted only keys of its own key-group range
    for r in range(WORLD):
        lo, hi = res[r]["kg"]
        kgs = {key_group(abi.KEYHASH_BINROW_BIGINT, row[0], 128) for row in res[r]["rows"]}
        assert all(lo <= g <= hi for g in kgs), f"rank {r}: foreign key group"
    want, late = _oracle_rows(name, res[0]["wms"][:N_BATCHES])
    got = res[0]["rows"] + res[1]["rows"]
    kw = sc["kw"]
    double_cols = {a for a, (k, c, t) in enumerate(kw["aggs"]) if t == F64 and k in (abi.AGG_SUM, abi.AGG_AVG)}
    assert len(want) > 2000
    _compare(got, want, double_cols, name)
    if sc["plan"] == "one":  # (two-phase: the GLOBAL operator counts late partial rows, not records)
        assert res[0]["late"] + res[1]["late"] == late


# The RCCL branches of the exchange on hardware: one rank over the nccl backend (RCCL) on the box's one
# GPU -- RCCL does not put two ranks on one device, so the two-rank scenarios above run over gloo.
# force_collectives keeps the collectives a single subtask would skip: the packed all-to-all moves
# device buffers unstaged through RCCL, the device valve's all-reduce runs in RCCL and
# fw_advance_device reads its result, and the overflow round's device all-to-all runs too; with one
# subtask the all-to-all is the rank's own segment, the forced-small segments still overflow, and
# the results must equal the unsharded oracle.
RCCL_SCENARIOS = ["one_phase_hop_device_valve", "one_phase_tumble_double_share_sizing_device_valve",
                  "two_phase_cumulate_zipf_device_valve", "one_phase_hop"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", RCCL_SCENARIOS)
def test_rccl_single_rank_exchange_equals_oracle(name):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run_ranks(name, world=1, backend="nccl")
    assert res[0]["backend"] == "nccl" and res[0]["collectives"]  # the RCCL branches ran
    sc = SCENARIOS[name]
    wms = res[0]["wms"][:N_BATCHES]
    if sc.get("valve") == "device":
        held = [b for b in range(N_BATCHES) if wms[b] != _proposed_wm(b, 0)]
        assert all(wms[b] == (wms[b - 1] if b else -(1 << 63)) for b in held)
    else:
        assert wms == [_proposed_wm(b, 0) for b in range(N_BATCHES)]
    assert res[0]["err"] == 0
    assert res[0]["spill_rounds"] > 0
    if sc["plan"] == "one":
        assert res[0]["received"] == N_BATCHES * N_ROWS
    want, late = _oracle_rows(name, wms, world=1)
    kw = sc["kw"]
    double_cols = {a for a, (k, c, t) in enumerate(kw["aggs"]) if t == F64 and k in (abi.AGG_SUM, abi.AGG_AVG)}
    assert len(want) > 1000
    _compare(res[0]["rows"], want, double_cols, name)
    if sc["plan"] == "one":
        assert res[0]["late"] == late
