#!/usr/bin/env python3
"""Windowed keyed-aggregation benchmark (BASELINE.json metric: windowed-agg events/sec, whole
node, at 1/2/4/8 GPUs, + % of HBM peak of the segmented-reduce kernel).

One "step" = one watermark interval of the hot path: ingest one batch of B = 2^22 synthetic
Nexmark-shaped events already resident in HBM (slice assignment + LDS segmented reduce), then
processWatermark (flush into the HBM slice table + fire/emit due windows).  Default workload is
CFG2 (Nexmark Q7-style TUMBLE 10 s MAX(price) GROUP BY auction, 10^6 auctions) for 24 steps
= 100.7 M events, the configuration BASELINE.json quotes the metric on (configs[1]).

N > 1 (torchrun, one rank per GPU, RCCL): every rank generates its slice of each global batch,
routes rows to the key-group owner with fw_partition_packed + one packed padded all-to-all over
xGMI (the keyBy exchange; the row counts stay on the device and the operator reads the packed rows
in place, skipping the padding itself),
min-reduces the watermark on the device (--valve device, the default: one RCCL all-reduce whose
result fw_advance_device reads from device memory; --valve host keeps a host gloo all-reduce for
A/B), then runs its own operator subtask -- no host synchronisation inside a step.  Weak scaling: per-GPU events, keys and event rate stay fixed as
N grows.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

B = 1 << 22                    # events per watermark interval
T0 = 1_599_998_400_000         # hour-aligned UTC start
J = 4000                       # out-of-orderness (nexmark.sql WATERMARK -4 s)
HBM_PEAK_GBPS = 8000.0         # MI355X HBM3E spec (MI355X_MICROARCH.md)

WORKLOADS = {
    # name: (description, window, aggs, keys per GPU, rate per GPU, value kind, key dist, input B/event)
    # state_per_key: the operator's capacity hint, (key, slice) entries per key at the PEAK of a
    # flush (live entries plus the batch's new slices before firing expires the old ones; live after
    # a step: CFG2 0.94, CFG3 5.3, CFG4 0.90, CFG5 1.24); a step that outgrows it fails loudly.  The
    # planner fills 75 % of a superbucket's table at the hint; the fullest superbucket's peak
    # (fw_stats.peak_superbucket_entries, round 5) lands at 72 % (CFG2), 76 % (CFG3), 69 % (CFG4), 94 %
    # (CFG5) and 74 % (cfg4_10m) of its table
    "cfg2": dict(desc="Nexmark Q7-style TUMBLE(10 s) MAX(price) GROUP BY auction",
                 window=("TUMBLE", 10_000, 0), aggs=[("MAX", 0, "BIGINT")], count_star=-1,
                 keys=1_000_000, key_base=1000, rate=1_000_000, value_kind=0, dist=0, w_in=24,
                 value_cols=["BIGINT"], nw=1, state_per_key=2),
    "cfg3": dict(desc="Nexmark Q5-style HOP(2 s slide, 10 s size) COUNT(*) GROUP BY auction",
                 window=("HOP", 10_000, 2_000), aggs=[("COUNT_STAR", 0, "BIGINT")], count_star=0,
                 keys=1_000_000, key_base=1000, rate=1_000_000, value_kind=0, dist=0, w_in=16,
                 value_cols=[], nw=1, state_per_key=8),
    "cfg4": dict(desc="TUMBLE(10 s) SUM(v), AVG(v) DOUBLE over 10^7 keys (1.25 M per GPU at N=8)",
                 window=("TUMBLE", 10_000, 0), aggs=[("SUM", 0, "DOUBLE"), ("AVG", 0, "DOUBLE")],
                 count_star=-1, keys=1_250_000, key_base=0, rate=1_000_000, value_kind=1, dist=0, w_in=24,
                 value_cols=["DOUBLE"], nw=2, state_per_key=2),
    # CFG4's full key space on ONE GPU (10^7 keys, sharded over 8 GPUs in cfg4).  At 10^6
    # events/s a 10 s window sees ~63 % of the 10^7 keys, so a flush's peak is ~1.24 entries per key
    # (the fired window + the next one's first seconds; measured: 1508 entries in the fullest of 8192
    # superbuckets), not CFG4's ~2.3 (1.25 M keys: every key in both windows).  Hint 1.25: 8192
    # superbuckets (hint 2 planned 16384 at 39 % of their tables: merge 1070 -> 639 us per flush)
    "cfg4_10m": dict(desc="TUMBLE(10 s) SUM(v), AVG(v) DOUBLE over 10^7 keys on one GPU",
                     window=("TUMBLE", 10_000, 0), aggs=[("SUM", 0, "DOUBLE"), ("AVG", 0, "DOUBLE")],
                     count_star=-1, keys=10_000_000, key_base=0, rate=1_000_000, value_kind=1, dist=0, w_in=24,
                     keys_fixed=True, value_cols=["DOUBLE"], nw=2, state_per_key=1.25),
    "cfg5": dict(desc="CUMULATE(1 min step, 1 h) COUNT(*), SUM, MIN, MAX, Zipf(1.1) keys",
                 window=("CUMULATE", 3_600_000, 60_000),
                 aggs=[("COUNT_STAR", 0, "BIGINT"), ("SUM", 0, "BIGINT"), ("MIN", 0, "BIGINT"), ("MAX", 0, "BIGINT")],
                 count_star=0, keys=1_000_000, key_base=0, rate=27_778, value_kind=2, dist=1, w_in=24,
                 zipf_s=1.1, keys_fixed=True, value_cols=["BIGINT"], nw=4, state_per_key=3),
}


def chunk_rows(wl):
    # rows per k_ingest chunk (fw_internal.h ig_block * ig_rpt): 4096 up to 4 accumulator words
    return 4096 if wl["nw"] <= 4 else 2048


def watermark(b, rate_per_gpu):
    # W_b = T0 + floor((b+1) * B * 1000 / R) - J - 1 (per-GPU rate; N ranks x B events per step)
    return T0 + ((b + 1) * B * 1000) // rate_per_gpu - J - 1


def build_config(wl, world, rank, keys_total, out_cap):
    from flink_amd import abi
    kind, size, slide = wl["window"]
    return abi.make_config(
        api=abi.API_SQL, window_kind=abi.WINDOW_NAMES[kind], size_ms=size, slide_ms=slide,
        aggs=[(abi.AGG_NAMES[k], c, abi.TYPE_NAMES[t]) for k, c, t in wl["aggs"]],
        count_star_index=wl["count_star"],
        value_col_types=[abi.TYPE_NAMES[t] for t in wl["value_cols"]],
        key_hash=abi.KEYHASH_BINROW_BIGINT, max_parallelism=128, parallelism=world,
        subtask_index=rank,
        # this subtask's share of the keys (key-group range), with headroom for shard imbalance
        state_capacity=int(keys_total * wl["state_per_key"] / world * (1.0 if world == 1 else 1.25)),
        max_batch_rows=2 * B, output_capacity=out_cap)


def gen_params(wl, world, zipf_ptr):
    from flink_amd import abi
    keys_total = wl["keys"] if wl.get("keys_fixed") else wl["keys"] * world
    return abi.fw_gen_params(seed=42, t0_ms=T0, rate_per_s=wl["rate"] * world, ooo_ms=J,
                             key_base=wl["key_base"], key_count=keys_total, key_dist=wl["dist"],
                             value_kind=wl["value_kind"], zipf_cdf=zipf_ptr), keys_total


def cpu_baseline(wl, sample_events, threads=1):
    """Oracle (CPU restatement) on the first `sample_events` events of the same stream with the
    same watermarks; returns events/s of the record + watermark processing.  threads > 1 runs the
    sample as a keyBy at parallelism `threads` does: every thread is one subtask (its own oracle
    operator) fed the rows of its key-group range (KeyGroupRangeAssignment), pre-partitioned
    before the timed region; the oracle's C calls release the GIL, so the subtasks run in
    parallel and the rate is the sample over the slowest subtask's wall clock."""
    import threading
    from flink_amd import abi
    from oracle import oracle as O
    zcdf = O.zipf_cdf(wl["keys"], wl["zipf_s"]) if wl["dist"] == 1 else None
    gp = abi.fw_gen_params(seed=42, t0_ms=T0, rate_per_s=wl["rate"], ooo_ms=J, key_base=wl["key_base"],
                           key_count=wl["keys"], key_dist=wl["dist"], value_kind=wl["value_kind"], zipf_cdf=None)
    p = max(1, int(threads))
    steps = max(1, sample_events // B)
    ops = [O.OracleOperator(build_config(wl, p, i, wl["keys"], 1 << 22)) for i in range(p)]
    nvc = ops[0].cfg.n_value_cols
    shards = [[] for _ in range(p)]
    for b in range(steps):
        k, t, v = O.generate(gp, b * B, B, zcdf)
        dest = O.operator_indices(abi.KEYHASH_BINROW_BIGINT, k, 128, p) if p > 1 else np.zeros(len(k), np.int32)
        for i in range(p):
            m = dest == i
            shards[i].append((k[m], t[m], v[m]))
    n_out = [0] * p
    err = []

    def run(i):
        try:
            op = ops[i]
            for b, (k, t, v) in enumerate(shards[i]):
                op.process_batch(k, t, [v] if nvc else [])
                op.process_watermark(watermark(b, wl["rate"]))
                n_out[i] += len(op.results(clear=True)["key"])
        except Exception as e:  # surfaced below
            err.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(p)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    for op in ops:
        op.close()
    if err:
        raise err[0]
    return steps * B / dt, steps * B, dt, sum(n_out)


def rank_load(owned, elapsed_s, partials, world):
    """N > 1 per-rank load, collective over the job's process group (after the timed region).
    owned: int64 tensor [world] of THIS rank's timed rows by destination subtask (its share of the
    keyBy), on the collective's device; returns the job-wide per-subtask event counts, their max/mean
    (the key-group imbalance that bounds linear scaling), every rank's timed wall clock and the
    partial rows its operator ingested."""
    import torch
    import torch.distributed as dist
    dist.all_reduce(owned)
    mine = torch.tensor([float(elapsed_s), float(partials)], dtype=torch.float64, device=owned.device)
    allr = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    ev = [int(x) for x in owned.cpu().tolist()]
    mean = sum(ev) / world
    return {"events_owned_per_rank": ev, "events_total": sum(ev),
            "key_group_imbalance_max_over_mean": max(ev) / mean if mean else None,
            "rank_elapsed_s": [float(x[0]) for x in allr],
            "partials_ingested_per_rank": [int(x[1]) for x in allr],
            "note": "events owned = rows of the timed batches whose key group the subtask owns "
                    "(computeKeyGroupRangeForOperatorIndex); gathered after the timed region"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--force-collectives", action="store_true",
                    help="rehearsal: run one rank (torch.distributed.run --nproc-per-node 1) through the N > 1 "
                         "code path and its collectives (RCCL with --dist-backend nccl)")
    ap.add_argument("--cpu-sample", type=int, default=4 * B, help="events for the CPU baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="CPU baseline subtasks (threads), capped at the usable CPUs; 16 = the GPU box's "
                         "CPU share per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic summary (tools/traffic.py); default: newest profiles/r*/traffic_<workload>.json")
    ap.add_argument("--calibrate-traffic", action="store_true",
                    help="launch fw_assign_key_groups over 2^28 keys before timing: a known-byte "
                         "8-B/lane read (2 GiB) + 4-B/lane write (1 GiB) that calibrates FETCH_SIZE/WRITE_SIZE")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-staged end-to-end leg (N=1 only)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="diagnostic: time the steps without the per-launch hipEvents (no roofline)")
    ap.add_argument("--e2e-steps", type=int, default=8)
    ap.add_argument("--e2e-transfer", default="delta32", choices=["delta32", "words"],
                    help="end-to-end leg: columns spanning < 2^32 per batch cross PCIe as 32-bit deltas "
                         "(fw_commit_delta32), or every column as 8-byte words (fw_commit)")
    ap.add_argument("--state-per-key", type=float, default=None,
                    help="capacity hint override: (key, slice) entries per key at a flush's peak")
    ap.add_argument("--e2e-depth", type=int, default=2, choices=[1, 2],
                    help="end-to-end leg: read each watermark's rows 1 or 2 watermarks after collecting them "
                         "(fw_results_ready returns the oldest outstanding collection; 2 keeps the collection "
                         "off the host's critical path)")
    ap.add_argument("--kernel-timing", default="device", choices=["device", "events"],
                    help="per-launch kernel timing: in-kernel device-clock stamps (default) or hipEvents")
    ap.add_argument("--plan", default="auto", choices=["auto", "one", "two"],
                    help="one- or two-phase window aggregation; auto: two-phase for cfg4/cfg5 at N>1 (partials on "
                         "the wire), one-phase otherwise")
    ap.add_argument("--valve", default="device", choices=["device", "host"],
                    help="N>1: the watermark valve / overflow agreement as one device all-reduce read by "
                         "fw_advance_device (no host wait per step), or on the host (gloo all-reduce after "
                         "waiting for the partition kernel)")
    ap.add_argument("--sink", default="segments", choices=["segments", "compact", "discard"],
                    help="each watermark's result rows: handed over as per-superbucket device segments where "
                         "the merge wrote them (fw_results_device_segments; the timed loop reads no row, so this "
                         "costs what dropping them costs), compacted into contiguous device columns "
                         "(fw_results_device: one more read and write of every row), or dropped (fw_results_reset)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, one rank per GPU).  gloo is a rehearsal of the N>1 path on a "
                         "one-GPU box: ranks share the GPUs round robin and the exchange is staged "
                         "through host memory; never used for reported numbers")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: launch N>1 with torch.distributed.run")
    if args.dist_backend == "nccl":
        gpu = local
    else:  # rehearsal only: several ranks may share one GPU
        gpu = local % torch.cuda.device_count()
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    # --force-collectives: one rank through the N > 1 code path (process group, packed exchange and
    # valve collectives, per-rank load), so the RCCL branches run on a one-GPU box; never the value
    dpath = world > 1 or args.force_collectives
    if dpath:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from flink_amd import _native, abi
    from flink_amd.runtime.handle import WindowAggHandle
    L = _native.lib()
    wl = dict(WORKLOADS[args.workload])
    if args.state_per_key is not None:
        wl["state_per_key"] = args.state_per_key
    nv = len(wl["value_cols"])

    # ---------------- synthetic input, resident in HBM before timing --------------------
    zipf_t = None
    if wl["dist"] == 1:
        w = 1.0 / np.power(np.arange(1, wl["keys"] + 1, dtype=np.float64), wl["zipf_s"])
        cdf = np.cumsum(w)
        cdf /= cdf[-1]
        zipf_t = torch.tensor(cdf, device=dev)
    gp, keys_total = gen_params(wl, world, zipf_t.data_ptr() if zipf_t is not None else None)
    total_steps = args.warmup + args.steps
    gk = torch.empty((total_steps, B), dtype=torch.int64, device=dev)
    gt = torch.empty_like(gk)
    gv = torch.empty_like(gk)
    s = torch.cuda.current_stream(dev).cuda_stream
    for b in range(total_steps):
        i0 = (b * world + rank) * B     # this rank's slice of global batch b
        _native.check(L.fw_generate(C.byref(gp), i0, B, gk[b].data_ptr(), gt[b].data_ptr(), gv[b].data_ptr(), s))
    torch.cuda.synchronize(dev)

    # ---------------- keyBy exchange (N > 1): device partition + RCCL all-to-all ------------
    from flink_amd.runtime.exchange import KeyByExchange
    ex = KeyByExchange(abi.KEYHASH_BINROW_BIGINT, 128, force_collectives=args.force_collectives)

    def exchange(b):
        """Untimed helper (G_b count): the plain exchange, exact row counts."""
        if not dpath:
            return gk[b], gt[b], gv[b]
        k, t, v = ex.exchange(gk[b], gt[b], [gv[b]] if nv else [])
        return k, t, (v[0] if nv else None)

    # the timed keyBy exchange is the packed padded one: segments of the previous step's agreed
    # largest per-destination share + 3 % (KeyByExchange.headroom; the first step: the batch's even
    # share + 25 %), rows past a segment in an overflow round; the overflow decision, the next share
    # and the watermark valve share one all-reduce per step
    def push_step(b, handle):
        """Ingest step b; returns the watermark to advance to (the valve's minimum over subtasks)."""
        if not dpath:
            if isinstance(handle, WindowAggHandle):
                # the batches were generated and synchronised before the timed region: the C-ABI
                # push as a JNI shim makes it, without torch stream events
                handle.push_device(gk[b], gt[b], [gv[b]] if nv else [], producer_synced=True)
            else:
                handle.push_device(gk[b], gt[b], [gv[b]] if nv else [])
            return watermark(b, wl["rate"])
        if args.valve == "device":
            # the device-side valve: the previous step's overflow round (settled one step late: its
            # all-reduce is long done), then partition + all-to-all + ingest + ONE device all-reduce of
            # (overflow, watermark, share) + fw_advance_device -- no host wait on this step's GPU work
            vs = handle.__dict__.setdefault("_valve", {"px": None, "wm": None})
            if vs["px"] is not None:
                spill = vs["px"].settle()
                if spill is not None:
                    n_sp = spill.numel() // vs["px"].row_words
                    handle.push_device_packed_segments(torch.tensor([n_sp], dtype=torch.int64, device=dev), spill,
                                                       vs["px"].row_words)
            px = ex.exchange_packed_async(gk[b], gt[b], [gv[b]] if nv else [])
            handle.push_device_packed_segments(px.recv_counts, px.rows, px.row_words)
            wm = px.finish_device(watermark(b, wl["rate"]), vs["wm"])
            vs.update(px=px, wm=wm)
            return wm
        # the received segments' ingest is queued before the host waits for the partition's
        # counts (overflow round + watermark valve), so the GPU stays busy through that host step
        px = ex.exchange_packed_async(gk[b], gt[b], [gv[b]] if nv else [])
        handle.push_device_packed_segments(px.recv_counts, px.rows, px.row_words)
        spill, wm = px.finish(watermark=watermark(b, wl["rate"]))
        if spill is not None:
            n_sp = spill.numel() // px.row_words
            handle.push_device_packed_segments(torch.tensor([n_sp], dtype=torch.int64, device=dev), spill, px.row_words)
        return wm

    out_cap = 2 * keys_total // world + (1 << 20)
    if wl["window"][0] == "CUMULATE":
        # every step of every active key's window fires; a 2^22 batch spans ~151 s = up to 3 steps
        out_cap = 4 * keys_total + (1 << 20)

    two_phase = args.plan == "two" or (args.plan == "auto" and world > 1 and args.workload in ("cfg4", "cfg5"))

    class TwoPhaseOp:
        """The two-phase plan (TwoStageOptimizedWindowAggregateRule.java:80-109, Flink's default for these
        mergeable aggregates) on this rank: a LOCAL operator over the rank's own batch, its partial rows
        exchanged on the device (TwoPhaseWindowAgg.step_device), the GLOBAL operator of this subtask."""

        def __init__(self, cfg):
            from flink_amd.table.two_phase import TwoPhaseWindowAgg
            # the LOCAL operator sees every key group: its flush table is sized for all keys
            self.tp = TwoPhaseWindowAgg(cfg, exchange=ex, device=dev,
                                        local_state_capacity=int(keys_total * wl["state_per_key"]))

        def step(self, b):
            self.tp.local.push_device(gk[b], gt[b], [gv[b]] if nv else [])
            sink(self.tp.glob)
            if args.valve == "device":
                self.tp.step_device_valve(watermark(b, wl["rate"]))
            else:
                self.tp.step_device(watermark(b, wl["rate"]))

        def settle(self):
            self.tp.settle()

        def set_profiling(self, *a, **k):
            self.tp.local.set_profiling(*a, **k)
            self.tp.glob.set_profiling(*a, **k)

        def sync(self):
            self.tp.local.sync()
            self.tp.glob.sync()

        def stats(self):  # the GLOBAL operator's state and merges, the LOCAL operator's ingest
            st, sl = self.tp.glob.stats(), self.tp.local.stats()
            for f in ("partials_emitted", "partial_bytes_written", "compact_chunks"):
                st[f] = sl[f]
            st["error_flags"] |= sl["error_flags"]
            return st

        def kernel_times(self):
            kl, kg = self.tp.local.kernel_times(), self.tp.glob.kernel_times()
            out = {"reduce": kl["reduce"], "merge": kg["merge"]}
            out.update({"local_" + k: v for k, v in kl.items() if k not in ("reduce", "merge_phase_cycles")})
            out.update({"global_" + k: v for k, v in kg.items() if k not in ("merge", "merge_phase_cycles")})
            return out

        def close(self):
            self.tp.close()

    def make_op(cfg):
        return TwoPhaseOp(cfg) if two_phase else WindowAggHandle(cfg)

    sink_res, sink_dn, sink_seg = abi.fw_result(), C.c_void_p(), abi.fw_result_segments()

    def sink(h):
        """the previous watermark's rows, consumed on the device through the C-ABI call itself (no
        torch views): as segments in place, compacted, or dropped"""
        if args.sink == "segments":
            _native.check(L.fw_results_device_segments(h._h, C.byref(sink_seg)))
        elif args.sink == "compact":
            _native.check(L.fw_results_device(h._h, C.byref(sink_res), C.byref(sink_dn)))
        else:
            h.reset_results()

    def run(first, nsteps, handle):
        for b in range(first, first + nsteps):
            if two_phase:
                handle.step(b)
                continue
            wm = push_step(b, handle)
            sink(handle)
            if torch.is_tensor(wm):
                handle.advance_device(wm)
            else:
                handle.advance(wm)
        # the device valve's last overflow round (settled one step late)
        if two_phase:
            handle.settle()
        elif getattr(handle, "_valve", None) and handle._valve["px"] is not None:
            spill = handle._valve["px"].settle()
            if spill is not None:
                n_sp = spill.numel() // handle._valve["px"].row_words
                handle.push_device_packed_segments(torch.tensor([n_sp], dtype=torch.int64, device=dev), spill,
                                                   handle._valve["px"].row_words)
            handle._valve["px"] = None

    if args.calibrate_traffic:
        # same access width as k_ingest's column loads (global_load_dwordx2 per lane), sized far
        # past the 256 MiB Infinity Cache so every byte comes from HBM
        nc = 1 << 28
        ck = torch.zeros(nc, dtype=torch.int64, device=dev)
        cd = torch.empty(nc, dtype=torch.int32, device=dev)
        _native.check(L.fw_assign_key_groups(ck.data_ptr(), None, nc, abi.KEYHASH_LONG, 128, 8,
                                             None, cd.data_ptr(), s))
        torch.cuda.synchronize(dev)
        del ck, cd

    # G_b of SURVEY.md 8d: distinct (key, slice) groups of each timed batch (exact, untimed; no
    # event of the synthetic stream is late, so every row's group is (key, its own slice))
    interval = wl["window"][2] if wl["window"][0] != "TUMBLE" else wl["window"][1]
    if wl["window"][0] == "HOP":
        import math
        interval = math.gcd(wl["window"][1], wl["window"][2])
    groups = []
    for b in range(args.warmup, total_steps):
        # one-phase: the batch this subtask ingests after the exchange; two-phase: the LOCAL
        # operator's own batch (its k_ingest is the segmented reduce measured below)
        k, t = (gk[b], gt[b]) if two_phase else exchange(b)[:2]
        sl = torch.div(t, interval, rounding_mode="floor")
        sl = sl - sl.min()
        groups.append(int(torch.unique(k * (int(sl.max()) + 1) + sl).numel()))
        del k, t, sl
    torch.cuda.synchronize(dev)

    cfg = build_config(wl, world, rank, keys_total, out_cap)
    # warmup on its own operator instance (first batches of the same stream)
    if args.warmup:
        hw = make_op(cfg)
        run(0, args.warmup, hw)
        hw.sync()
        hw.close()
    h = make_op(cfg)
    torch.cuda.synchronize(dev)
    if dpath:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # per-launch kernel times over the timed region: in-kernel device-clock stamps (block 0's start
    # -> the grid's last workgroup's end) by default; --kernel-timing events puts hipEvents around
    # every launch on the operator's stream instead (they idle the stream ~7 us per launch)
    h.set_profiling(not args.no_kernel_events, mode=args.kernel_timing)
    t0 = time.perf_counter()
    run(args.warmup, args.steps, h)
    t_issued = time.perf_counter() - t0  # host time to enqueue the K steps
    h.sync()
    torch.cuda.synchronize(dev)
    if dpath:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    elapsed_own = elapsed
    if dpath:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    st = h.stats()
    kt = h.kernel_times()
    if st["error_flags"]:
        raise SystemExit(f"device error flags {st['error_flags']}")

    # ---------------- N > 1: per-rank load (after the timed region) ---------------------------
    # key-group skew limits linearity, so the line reports each subtask's share of the
    # timed events -- the rows whose key group it owns (KeyGroupRangeAssignment
    # .computeKeyGroupRangeForOperatorIndex :93-106, as KeyGroupStreamPartitioner.selectChannel routes
    # them) -- and every rank's own timed wall clock; the shares sum to N * B * steps
    ranks = None
    if dpath:
        cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        owned = torch.zeros(world, dtype=torch.int64, device=dev)
        kg_b = torch.empty(B, dtype=torch.int32, device=dev)
        dst_b = torch.empty(B, dtype=torch.int32, device=dev)
        for b in range(args.warmup, total_steps):
            _native.check(L.fw_assign_key_groups(gk[b].data_ptr(), None, B, abi.KEYHASH_BINROW_BIGINT, 128, world,
                                                 kg_b.data_ptr(), dst_b.data_ptr(), s))
            owned += torch.bincount(dst_b.long(), minlength=world)
        ranks = rank_load(owned.to(cdev), elapsed_own, st["partials_emitted"], world)

    n_total = args.steps * B * world
    value = n_total / elapsed
    if args.no_kernel_events:
        if rank == 0:
            print(json.dumps({"diagnostic": "no per-launch events", "value": value,
                              "ms_per_step": elapsed / args.steps * 1e3}), flush=True)
        h.close()
        return
    # ---------------- roofline of the segmented-reduce (ingest) kernel ----------------------
    # algorithmic bytes per launch: N_b * sum(w_in) + G_b * w_partial, with
    # w_partial = key + slice + accumulator words (8 B each) and G_b the distinct (key, slice)
    # groups of the batch (counted exactly above)
    red_ms, red_n = kt["reduce"]
    w_partial = 8 * (2 + wl["nw"])
    rows_per_launch = n_total / world / red_n
    g_per_launch = sum(groups) / len(groups)
    bytes_per_launch = rows_per_launch * wl["w_in"] + g_per_launch * w_partial
    avg_reduce_s = red_ms / red_n / 1e3
    achieved = bytes_per_launch / avg_reduce_s / 1e9
    # ---------------- the flush + fire kernel -------------------------------------------------
    # algorithmic bytes over the timed region, from device counters (fw_stats): the distinct groups
    # of the batches those flushes merged (G_b * w_partial), the state entries the launches loaded
    # and wrote back (counted per superbucket on the device: only launches that flush or fire move
    # state), and the fired windows' output rows; per launch = total / launches.  Beside it, what
    # the flushes really read: every partial row the ingest wrote (partials_merged * w_partial).
    mg_ms, mg_n = kt["merge"]
    w_entry = 8 * (3 + wl["nw"])
    # an emitted row as the merge writes it: key, window_end, one word per aggregate, the NULL mask
    # (no window_start since ABI v10: readers derive it from window_end)
    w_out = 8 * (2 + len(wl["aggs"])) + 4
    live = st["live_state_entries"]
    fired_total = st["num_fired_windows"]
    merged_share = st["partials_merged"] / max(st["partials_emitted"], 1)  # batches flushed by the end
    merge_total = (sum(groups) * merged_share * w_partial + st["state_entries_moved"] * w_entry
                   + fired_total * w_out)
    merge_bytes = merge_total / max(mg_n, 1)
    # partial bytes as written (compact chunks: (key, acc) or (key) rows + a rank byte, fw_internal.h PF_*)
    merge_read_total = (st["partial_bytes_merged"] + st["state_entries_moved"] * w_entry + fired_total * w_out)
    avg_merge_s = mg_ms / max(mg_n, 1) / 1e3
    traffic = traffic_m = None
    tpath = args.traffic_json
    if tpath is None:
        import glob
        found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"traffic_{args.workload}.json")))
        tpath = found[-1] if found else ""
    plan_name = "two-phase" if two_phase else "one-phase"
    traffic_src = None
    if tpath and os.path.exists(tpath):
        tj = json.load(open(tpath))
        # counters measured on this exact run shape only: same workload, GPU count and plan (files
        # written before round 6 carry neither field: tools/measure.sh ran them at N = 1, one-phase)
        if (tj.get("workload") == args.workload and tj.get("n_gpus", 1) == world
                and tj.get("plan", "one-phase") == plan_name and not (world == 1 and dpath)):
            traffic = tj.get("k_ingest_hbm_bytes_per_launch")
            traffic_m = tj.get("k_merge_fire_hbm_bytes_per_launch")
            traffic_src = os.path.relpath(tpath, ROOT) if tpath.startswith(ROOT) else tpath

    # ---------------- end-to-end leg (N = 1): host-staged, pipelined --------------------------
    # What the JNI shim does, pipelined the way the handle allows: the host fills
    # the operator's pinned staging columns (fw_reserve; 8 threads copying slices of the numpy
    # batch, standing for the shim's record serialisation), fw_commit moves them over PCIe on the
    # copy stream while the previous batch is still being ingested (two staging sets), and each
    # watermark's rows are collected into pinned host memory by fw_results_async and read
    # --e2e-depth steps later (fw_results_ready).  Reported beside the device-resident `value`, never as it.
    e2e = None
    if not dpath and not args.no_e2e and args.e2e_steps > 0:
        from concurrent.futures import ThreadPoolExecutor
        from flink_amd.runtime.handle import _np_view
        ns = min(args.e2e_steps, gk.shape[0])
        hk = [gk[b].cpu().numpy() for b in range(ns)]
        ht = [gt[b].cpu().numpy() for b in range(ns)]
        hv = [gv[b].cpu().numpy() for b in range(ns)]
        cfg_e = build_config(wl, 1, 0, keys_total, out_cap)
        he = WindowAggHandle(cfg_e)
        pool = ThreadPoolExecutor(8)
        parts = [(i * B // 8, (i + 1) * B // 8) for i in range(8)]

        def fill(dst, src):  # ctypes.memmove releases the GIL: the slices copy in parallel
            d = C.cast(dst, C.c_void_p).value
            return [pool.submit(C.memmove, d + 8 * a, src.ctypes.data + 8 * a, 8 * (e - a)) for a, e in parts]

        def fill_delta32(items):
            # as the shim serialises records: each column as 32-bit deltas from (its first value - 2^31),
            # range-checked in the same pass (fw_delta32_encode, 8 threads); a column with a value
            # outside that 2^32 window is written again as words
            mask, bases, pend = 0, (C.c_int64 * (2 + abi.FW_MAX_COLS))(), []
            for slot, dst, src in items:
                base = int(src[0]) - (1 << 31)
                if base < -(1 << 63):
                    pend.append((slot, dst, src, None))
                    continue
                d = C.cast(dst, C.c_void_p).value
                pend.append((slot, dst, src, base, [pool.submit(L.fw_delta32_encode, src.ctypes.data + 8 * a, e - a, base,
                                                                d + 4 * a) for a, e in parts]))
            fs = []
            for slot, dst, src, base, *f in pend:
                if base is not None and not any(x.result() for x in f[0]):
                    mask |= 1 << slot
                    bases[slot] = base
                else:
                    fs += fill(dst, src)
            return mask, bases, fs

        cols = abi.fw_host_cols()
        _native.check(L.fw_reserve(he._h, 0, C.byref(cols)))  # allocates the staging (untimed)
        _native.check(L.fw_commit(he._h, 0))
        he.results_async()  # allocates the pinned result buffers (untimed); nothing to collect yet
        he.results_ready(copy=False)
        depth = args.e2e_depth
        rows_out = 0
        delta_cols = 0
        t_reserve = t_fill = t_ready = t_commit = t_adv = t_async = 0.0
        te0 = time.perf_counter()
        for b in range(ns):
            t1 = time.perf_counter()
            cols = abi.fw_host_cols()
            _native.check(L.fw_reserve(he._h, B, C.byref(cols)))  # waits for the H2D two commits back
            t2 = time.perf_counter()
            if args.e2e_transfer == "delta32":
                # BIGINT columns are range-checked for packing; a DOUBLE column's bit patterns span the
                # whole word range, so the shim writes it as words without trying
                dbl = nv and wl["value_cols"][0] == "DOUBLE"
                mask, bases, fs = fill_delta32([(0, cols.key, hk[b]), (1, cols.ts, ht[b])] +
                                               ([(2, cols.values[0], hv[b])] if nv and not dbl else []))
                if dbl:
                    fs += fill(cols.values[0], hv[b])
            else:
                mask, fs = 0, fill(cols.key, hk[b]) + fill(cols.ts, ht[b]) + (fill(cols.values[0], hv[b]) if nv else [])
            for f in fs:
                f.result()
            t3 = time.perf_counter()
            if mask:
                _native.check(L.fw_commit_delta32(he._h, B, mask, bases))
                delta_cols |= mask
            else:
                _native.check(L.fw_commit(he._h, B))
            t3c = time.perf_counter()
            he.advance(watermark(b, wl["rate"]))
            t4 = time.perf_counter()
            he.results_async()  # watermark b's rows, collected while the next batches are ingested
            t5 = time.perf_counter()
            if b >= depth:
                rows_out += len(he.results_ready(copy=False)["key"])  # watermark b - depth's rows
            t_reserve += t2 - t1
            t_fill += t3 - t2
            t_commit += t3c - t3
            t_adv += t4 - t3c
            t_async += t5 - t4
            t_ready += time.perf_counter() - t5
        t6 = time.perf_counter()
        for _ in range(min(depth, ns)):
            rows_out += len(he.results_ready(copy=False)["key"])
        he.sync()
        te = time.perf_counter() - te0
        t_ready += time.perf_counter() - t6
        he.close()
        pool.shutdown()
        e2e = {"value": ns * B / te, "unit": "events/s", "steps": ns,
               "ms_per_step": te / ns * 1e3, "result_rows": rows_out,
               "host_ms_per_step": {"fill_pinned_8_threads": t_fill / ns * 1e3,
                                    "reserve_wait_h2d": t_reserve / ns * 1e3,
                                    "commit_enqueue_h2d_ingest": t_commit / ns * 1e3,
                                    "advance_enqueue": t_adv / ns * 1e3,
                                    "results_ready_wait": t_ready / ns * 1e3,
                                    "results_async_enqueue": t_async / ns * 1e3},
               "fill_GBps": ns * B * wl["w_in"] / max(t_fill, 1e-9) / 1e9,
               "path": "numpy batch -> pinned staging (fw_reserve, 8 fill threads) -> H2D on the copy stream, "
                       "overlapping the previous batch's ingest (fw_commit, or fw_commit_delta32 for columns spanning < 2^32) -> advance -> rows into pinned host "
                       f"memory (fw_results_async), read {depth} watermark(s) later (fw_results_ready)",
               "results_depth": depth, "transfer": args.e2e_transfer,
               "delta32_columns": [n for i, n in enumerate(["key", "ts", "value"]) if delta_cols >> i & 1]}

    cpu = None
    if rank == 0 and not dpath and not args.no_cpu_baseline:
        try:
            host_cpus = len(os.sched_getaffinity(0))
        except AttributeError:
            host_cpus = os.cpu_count()
        thr = max(1, min(args.cpu_threads, host_cpus))
        v, n, dt, _ = cpu_baseline(wl, args.cpu_sample, thr)
        cpu = {"value": v, "unit": "events/s", "cores": thr, "kind": "port",
               "host_nproc": host_cpus,
               "sample": f"first {n} events of the same {args.workload} stream through the C++ oracle "
                         f"(oracle/flinkwin_oracle.cpp) as a keyBy at parallelism {thr}: one thread and one "
                         f"operator per subtask over its key-group range (rows pre-partitioned, untimed), on a "
                         f"host with {host_cpus} usable CPUs, {dt:.1f} s wall; the reference Flink operator needs a JDK, absent here"}

    if rank == 0:
        line = {
            "metric": "windowed-agg events/sec (whole node) at 1/2/4/8 GPU + % of HBM peak",
            "value": value, "unit": "events/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64" if wl["value_kind"] != 1 else "f64",
            "data": "synthetic (SplitMix64 Nexmark-shaped generator, seed 42, device-resident)",
            "config": {"workload": f"{args.workload}: {wl['desc']}", "events_per_gpu_per_step": B,
                       "plan": "two-phase (LOCAL -> partials on the device exchange -> GLOBAL)" if two_phase else "one-phase",
                       "keys_total": keys_total, "rate_per_gpu_ev_s": wl["rate"],
                       "state_per_key_hint": wl["state_per_key"],
                       "parallelism": f"key-group sharded x{world}" + (
                           "" if not dpath else " + RCCL all-to-all" if args.dist_backend == "nccl"
                           else " + gloo all-to-all (rehearsal, shared GPU)"),
                       "max_parallelism": 128, "superbuckets": st["num_superbuckets"],
                       "result_sink": {"segments": "each watermark's rows left in the merge's device slabs and "
                                                   "handed over as per-superbucket segments "
                                                   "(fw_results_device_segments); no row is read in the timed loop",
                                       "compact": "each watermark's rows compacted into contiguous device columns "
                                                  "(fw_results_device)",
                                       "discard": "dropped (fw_results_reset)"}[args.sink],
                       "rehearsal": ("one rank through the N > 1 code path (--force-collectives): its "
                                     "all-to-all is the rank's own segment; not a scaling measurement")
                                    if world == 1 and dpath else None,
                       "exchange": None if not dpath else {
                           "kind": "packed padded all-to-all, segments of the previous step's agreed largest "
                                   "share + 3 % (first step: even share + 25 %)",
                           "watermark_valve": ("device all-reduce (overflow, watermark, share) -> fw_advance_device"
                                               if args.valve == "device" else "host gloo all-reduce"),
                           "segment_rows_first_step": ex.segment_capacity(B, world),
                           "agreed_share_rows": ex._dn_share if ex._share_known else None,
                           "overflow_rounds": ex.spill_rounds}},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "fw::k_ingest (K1 key group + K2 slice assign + K3 LDS segmented reduce, "
                                   "chunk-local superbucket sort)",
                         "algorithmic_bytes_per_launch": bytes_per_launch, "avg_launch_us": avg_reduce_s * 1e6,
                         "launch_timing": ("in-kernel device clock (block 0 start -> last workgroup end), "
                                           "every launch of the timed region" if args.kernel_timing == "device"
                                           else "hipEvents around every launch of the timed region"),
                         "launches": red_n, "distinct_groups_per_launch": g_per_launch,
                         "partials_written_per_launch": st["partials_emitted"] / red_n,
                         "partial_bytes_written_per_launch": st["partial_bytes_written"] / red_n,
                         "compact_chunk_share": st["compact_chunks"] / max(1, red_n * -(-int(rows_per_launch) // chunk_rows(wl))),
                         "counter_rate_GBps": (traffic / avg_reduce_s / 1e9) if traffic else None,
                         "traffic_over_algorithmic": (traffic / bytes_per_launch) if traffic else None},
            "roofline_merge": {"bound": "hbm", "kernel": "fw::k_merge_fire (K4 flush into the HBM slice table + "
                                                         "K5 timers / fire / emit)",
                               "achieved": merge_bytes / avg_merge_s / 1e9 if mg_n else None,
                               "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                               "frac": merge_bytes / avg_merge_s / 1e9 / HBM_PEAK_GBPS if mg_n else None,
                               "algorithmic_bytes_per_launch": merge_bytes,
                               "terms_per_launch": {
                                   "G_b_w_partial": sum(groups) * merged_share * w_partial / max(mg_n, 1),
                                   "state_entries_moved_w_entry": st["state_entries_moved"] * w_entry / max(mg_n, 1),
                                   "F_w_out": fired_total * w_out / max(mg_n, 1)},
                               "flush_launches": st["flush_launches"], "live_state_entries_end": live,
                               "superbuckets": st["num_superbuckets"],
                               "peak_superbucket_entries": st["peak_superbucket_entries"],
                               "superbucket_capacity": st["superbucket_capacity"],
                               "partial_bytes_read_per_launch": st["partial_bytes_merged"] / max(mg_n, 1),
                               "design_bytes_per_launch": merge_read_total / max(mg_n, 1),
                               "avg_launch_us": avg_merge_s * 1e6, "launches": mg_n, "traffic": traffic_m,
                               "counter_rate_GBps": (traffic_m / avg_merge_s / 1e9) if traffic_m else None,
                               "traffic_over_algorithmic": (traffic_m / merge_bytes) if traffic_m else None},
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "per_rank": ranks,
            "device_ms_per_step": {k: v[0] / args.steps for k, v in kt.items() if v[1]},
            "host_issue_ms_per_step": t_issued / args.steps * 1e3,
        }
        print(json.dumps(line), flush=True)
    h.close()
    if dpath:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
