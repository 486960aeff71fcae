#!/usr/bin/env python3
"""Development timing tool: times fw::k_ingest with phases switched off (FW_ABLATE bits, see
fw_internal.h AB_*).  The ablations and phase stamps exist only in a diagnostic build of the
library (make -C flink_amd/csrc DIAG=1); the production build compiles them out.  Only pushes (<= 6 per handle, so no merge ever reads the ablated
partials); results are meaningless, only the per-kernel device times matter."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from flink_amd import _native  # noqa: E402
from flink_amd.runtime.handle import WindowAggHandle  # noqa: E402


def main():
    wl_name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    variants = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 3, 4, 6, 7]
    wl = bench.WORKLOADS[wl_name]
    dev = torch.device("cuda", 0)
    L = _native.lib()
    zipf_t = None
    if wl["dist"] == 1:
        import numpy as np
        w = 1.0 / np.power(np.arange(1, wl["keys"] + 1, dtype=np.float64), wl["zipf_s"])
        cdf = np.cumsum(w)
        zipf_t = torch.tensor(cdf / cdf[-1], device=dev)
    gp, keys_total = bench.gen_params(wl, 1, zipf_t.data_ptr() if zipf_t is not None else None)
    nb = 6
    gk = torch.empty((nb, bench.B), dtype=torch.int64, device=dev)
    gt, gv = torch.empty_like(gk), torch.empty_like(gk)
    s = torch.cuda.current_stream(dev).cuda_stream
    for b in range(nb):
        _native.check(L.fw_generate(C.byref(gp), b * bench.B, bench.B, gk[b].data_ptr(), gt[b].data_ptr(),
                                    gv[b].data_ptr(), s))
    torch.cuda.synchronize()
    cfg = bench.build_config(wl, 1, 0, keys_total, 1 << 22)
    out = {}
    for ab in variants:
        os.environ["FW_ABLATE"] = str(ab)
        times = []
        for rep in range(3):
            h = WindowAggHandle(cfg)
            # one push and a flush first: the timed pushes then open a flush epoch with measured
            # PF_PACK fields (fw_internal.h), as in the bench's steady state
            h.push_device(gk[0], gt[0], [gv[0]] if wl["value_cols"] else [])
            h.flush()
            h.set_profiling(True)
            for b in range(1, nb):
                h.push_device(gk[b], gt[b], [gv[b]] if wl["value_cols"] else [])
            ms, n = h.kernel_times()["reduce"]
            if rep and n:
                times.append(ms / n * 1e3)
            h.close()
        out[ab] = sum(times) / len(times) if times else float("nan")  # early-exit ablations: time with rocprofv3
        print(json.dumps({"workload": wl_name, "ablate": ab, "k_ingest_us": round(out[ab], 2)}), flush=True)
    os.environ.pop("FW_ABLATE", None)




def merge_main(wl_name, variants, steps=12):
    """Full push + advance loop; reports the merge kernel's average time per step."""
    wl = bench.WORKLOADS[wl_name]
    dev = torch.device("cuda", 0)
    L = _native.lib()
    zipf_t = None
    if wl["dist"] == 1:
        import numpy as np
        w = 1.0 / np.power(np.arange(1, wl["keys"] + 1, dtype=np.float64), wl["zipf_s"])
        cdf = np.cumsum(w)
        zipf_t = torch.tensor(cdf / cdf[-1], device=dev)
    gp, keys_total = bench.gen_params(wl, 1, zipf_t.data_ptr() if zipf_t is not None else None)
    gk = torch.empty((steps, bench.B), dtype=torch.int64, device=dev)
    gt, gv = torch.empty_like(gk), torch.empty_like(gk)
    s = torch.cuda.current_stream(dev).cuda_stream
    for b in range(steps):
        _native.check(L.fw_generate(C.byref(gp), b * bench.B, bench.B, gk[b].data_ptr(), gt[b].data_ptr(),
                                    gv[b].data_ptr(), s))
    torch.cuda.synchronize()
    out_cap = 2 * keys_total + (1 << 20)
    cfg = bench.build_config(wl, 1, 0, keys_total, out_cap)
    for ab in variants:
        os.environ["FW_ABLATE"] = str(ab)
        h = WindowAggHandle(cfg)
        try:
            for b in range(steps):
                if b == 3:
                    torch.cuda.synchronize()  # not h.sync(): ablated runs may set error bits
                    h.set_profiling(True)
                h.push_device(gk[b], gt[b], [gv[b]] if wl["value_cols"] else [])
                h.reset_results()
                h.advance(bench.watermark(b, wl["rate"]))
        except _native.FlinkWinError as e:  # ablated runs may overflow the state table
            print(json.dumps({"workload": wl_name, "ablate": ab, "error": str(e)}), flush=True)
            h.close()
            continue
        kt = h.kernel_times()  # reads times + stamps, no error check
        ms, n = kt["merge"]
        print(json.dumps({"workload": wl_name, "ablate": ab, "merge_ms_per_step": round(ms / (steps - 3), 4),
                          "reduce_us": round(kt["reduce"][0] / kt["reduce"][1] * 1e3, 2),
                          "phase_Mcycles": [round(x / 1e6, 1) for x in kt["merge_phase_cycles"][:8]],
                          "rounds": kt["merge_phase_cycles"][7], "fired": h.stats()["num_fired_windows"],
                          "errors": h.stats()["error_flags"]}), flush=True)
        h.close()
    os.environ.pop("FW_ABLATE", None)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "merge":
        merge_main(sys.argv[2], [int(x) for x in sys.argv[3].split(",")])
    else:
        main()
