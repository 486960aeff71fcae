"""Per-launch kernel timing of the operator (fw_set_profiling), the source of bench.py's roofline
launch times: the in-kernel device-clock stamps (FW_PROF_DEVICE, bench's default) and hipEvents
around each launch (FW_PROF_EVENTS) count the same launches and agree on their durations.  Run on
an MI355X."""
import ctypes as C

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(mode, steps=6, n=1 << 20):
    import torch
    import bench
    from flink_amd import _native
    from flink_amd.runtime.handle import WindowAggHandle
    wl = bench.WORKLOADS["cfg2"]
    gp, keys = bench.gen_params(wl, 1, None)
    dev = torch.device("cuda", 0)
    k = torch.empty(n, dtype=torch.int64, device=dev)
    t, v = torch.empty_like(k), torch.empty_like(k)
    cfg = bench.build_config(wl, 1, 0, keys, 1 << 22)
    h = WindowAggHandle(cfg)
    try:
        h.set_profiling(True, mode=mode)
        s = torch.cuda.current_stream(dev).cuda_stream
        for b in range(steps):
            _native.check(_native.lib().fw_generate(C.byref(gp), b * n, n, k.data_ptr(), t.data_ptr(),
                                                    v.data_ptr(), s))
            h.push_device(k, t, [v])
            h.advance(bench.T0 + ((b + 1) * n * 1000) // wl["rate"] - bench.J - 1)
        h.sync()
        return h.kernel_times()
    finally:
        h.close()


def test_device_stamps_and_events_time_the_same_launches(monkeypatch):
    monkeypatch.setenv("FW_SKIP_IDLE", "0")  # a merge launch per advance, idle or not
    dev = _run("device")
    ev = _run("events")
    for kind in ("reduce", "merge"):
        (ms_d, n_d), (ms_e, n_e) = dev[kind], ev[kind]
        assert n_d == n_e == 6, (kind, n_d, n_e)  # (advances that cross no slice end launch too)
        assert ms_d > 0 and ms_e > 0
    # an ingest launch over 2^20 rows does the same work in both runs; the stamps exclude the
    # dispatch ramp the events include, so they may read a little lower, never far off
    r = dev["reduce"][0] / ev["reduce"][0]
    assert 0.6 < r < 1.3, r


def test_profiling_off_records_nothing():
    import bench
    from flink_amd.runtime.handle import WindowAggHandle
    wl = bench.WORKLOADS["cfg2"]
    h = WindowAggHandle(bench.build_config(wl, 1, 0, 1000, 1 << 16))
    try:
        h.set_profiling(False)
        kt = h.kernel_times()
        assert kt["reduce"] == (0.0, 0) and kt["merge"] == (0.0, 0)
    finally:
        h.close()
