"""ctypes binding of libflinkwin.so (the HIP/gfx950 library built in-tree from flink_amd/csrc).

There is no CPU fallback: if the library is missing or cannot be loaded this module raises,
so a GPU run can never silently take another path.
"""
import ctypes as C
import os

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libflinkwin.so")
if os.environ.get("FW_LIB_VARIANT"):  # development A/B builds (make OUT=../libflinkwin_<v>.so); never set by default
    LIB_PATH = os.path.join(_HERE, f"libflinkwin_{os.environ['FW_LIB_VARIANT']}.so")


class FlinkWinError(RuntimeError):
    """Raised for any non-zero libflinkwin status (the Java shim maps this to Exception)."""

    def __init__(self, code, msg):
        super().__init__(f"libflinkwin error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with `make -C flink_amd/csrc` "
                          "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int32
    P = C.POINTER
    sig = {
        "fw_create": (i32, [P(abi.fw_config), P(vp)]),
        "fw_destroy": (i32, [vp]),
        "fw_last_error": (C.c_char_p, []),
        "fw_abi_version": (i32, []),
        "fw_device_count": (i32, []),
        "fw_get_stream": (vp, [vp]),
        "fw_sync": (i32, [vp]),
        "fw_initialize_watermark": (i32, [vp, i64]),
        "fw_reserve": (i32, [vp, i64, P(abi.fw_host_cols)]),
        "fw_commit": (i32, [vp, i64]),
        "fw_commit_delta32": (i32, [vp, i64, C.c_uint32, P(C.c_int64)]),
        "fw_delta32_encode": (i32, [vp, i64, i64, vp]),
        "fw_push_device": (i32, [vp, i64, vp, vp, vp, vp, vp]),
        "fw_push_device_segments": (i32, [vp, i32, i64, vp, vp, vp, vp, vp, vp]),
        "fw_push_device_packed_segments": (i32, [vp, i32, i64, vp, vp, i32]),
        "fw_partition_packed": (i32, [vp, vp, vp, vp, i32, i64, i32, i32, i32, i64, vp, vp, vp, i64, vp]),
        "fw_partition_packed_spill": (i32, [vp, vp, vp, vp, i32, i64, i32, i32, i32, i64, vp, vp, vp, vp, i64, vp]),
        "fw_partition_packed_spill_dn": (i32, [vp, vp, vp, vp, i32, i64, vp, i32, i32, i32, i64, vp, vp, vp, vp, i64, vp]),
        "fw_valve_local": (i32, [vp, i32, i64, i64, vp, vp]),
        "fw_valve_select": (i32, [vp, vp, vp, vp]),
        "fw_advance": (i32, [vp, i64]),
        "fw_advance_device": (i32, [vp, vp]),
        "fw_flush": (i32, [vp]),
        "fw_results": (i32, [vp, P(abi.fw_result), i32]),
        "fw_results_reset": (i32, [vp]),
        "fw_results_async": (i32, [vp]),
        "fw_results_ready": (i32, [vp, P(abi.fw_result)]),
        "fw_results_device": (i32, [vp, P(abi.fw_result), P(vp)]),
        "fw_get_stats": (i32, [vp, P(abi.fw_stats)]),
        "fw_set_profiling": (i32, [vp, i32]),
        "fw_get_kernel_times": (i32, [vp, P(abi.fw_kernel_times)]),
        "fw_snapshot": (i32, [vp, vp, i64, P(i64)]),
        "fw_restore": (i32, [vp, vp, i64]),
        "fw_snapshot_key_group": (i32, [vp, i32, vp, i64, P(i64)]),
        "fw_restore_key_group": (i32, [vp, vp, i64]),
        "fw_snapshot_key_group_heap": (i32, [vp, i32, P(abi.fw_heap_state_ids), vp, i64, P(i64)]),
        "fw_restore_key_group_heap": (i32, [vp, vp, i64, P(abi.fw_heap_state_ids)]),
        "fw_ds_snapshot_key_group": (i32, [vp, i32, vp, i64, P(i64)]),
        "fw_results_device_segments": (i32, [vp, P(abi.fw_result_segments)]),
        "fw_ds_restore_key_group": (i32, [vp, i32, vp, i64, i64]),
        "fw_assign_key_groups": (i32, [vp, vp, i64, i32, i32, i32, vp, vp, vp]),
        "fw_partition_by_dest": (i32, [vp, vp, vp, vp, i32, i64, i32, i32, i32, vp, vp, vp, vp, vp, i64, vp]),
        "fw_key_row_hash": (i32, [P(abi.fw_key_field), i32, i64, vp, vp]),
        "fw_host_key_row_hash": (i32, [P(abi.fw_key_field), i32, i64, vp]),
        "fw_partition_workspace_bytes": (i64, [i64, i32]),
        "fw_generate": (i32, [P(abi.fw_gen_params), i64, i64, vp, vp, vp, vp]),
        "fw_host_key_group": (i32, [i32, i64, i32, i32]),
        "fw_host_assign_key_groups": (i32, [vp, vp, i64, i32, i32, i32, vp, vp]),
        "fw_host_window_start": (i64, [i64, i64, i64]),
        "fw_host_next_trigger_watermark": (i64, [i64, i64]),
        "fw_host_time_op": (i32, [P(abi.fw_config), i32, i64, P(i64)]),
        "fw_late_records": (i32, [vp, P(abi.fw_late_rows)]),
        "fw_first_element_events": (i32, [vp, P(abi.fw_ordinal_events)]),
        "fw_push_device_key_rows": (i32, [vp, i64, vp, vp, vp, vp, vp]),
        "fw_key_row_images": (i32, [P(abi.fw_key_field), i32, i64, vp, vp, vp]),
        "fw_host_key_row_image_lengths": (i32, [P(abi.fw_key_field), i32, i64, vp]),
        "fw_host_key_row_images": (i32, [P(abi.fw_key_field), i32, i64, vp, vp]),
        "fw_host_key_row_image_hash": (i32, [vp, i64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.fw_abi_version() != abi.FW_ABI_VERSION:
        raise ImportError("libflinkwin ABI version mismatch")
    _lib = L
    return L


# every symbol the public header declares (tests check they are exported)
EXPORTED = ["fw_create", "fw_destroy", "fw_last_error", "fw_abi_version", "fw_device_count", "fw_get_stream", "fw_sync",
            "fw_initialize_watermark", "fw_reserve", "fw_commit", "fw_commit_delta32", "fw_delta32_encode", "fw_push_device", "fw_push_device_segments", "fw_push_device_packed_segments", "fw_advance", "fw_advance_device",
            "fw_flush", "fw_results", "fw_results_reset", "fw_results_async", "fw_results_ready", "fw_results_device", "fw_get_stats", "fw_set_profiling",
            "fw_get_kernel_times", "fw_snapshot", "fw_restore", "fw_snapshot_key_group", "fw_restore_key_group",
            "fw_snapshot_key_group_heap", "fw_restore_key_group_heap", "fw_ds_snapshot_key_group", "fw_ds_restore_key_group", "fw_results_device_segments", "fw_key_row_hash", "fw_host_key_row_hash",
            "fw_assign_key_groups", "fw_partition_by_dest", "fw_partition_packed", "fw_partition_packed_spill", "fw_partition_packed_spill_dn", "fw_partition_workspace_bytes",
            "fw_valve_local", "fw_valve_select",
            "fw_generate", "fw_host_key_group", "fw_host_assign_key_groups", "fw_host_window_start",
            "fw_host_next_trigger_watermark", "fw_host_time_op", "fw_late_records", "fw_first_element_events",
            "fw_push_device_key_rows", "fw_key_row_images", "fw_host_key_row_image_lengths", "fw_host_key_row_images",
            "fw_host_key_row_image_hash"]


def check(rc):
    if rc != 0:
        msg = lib().fw_last_error()
        raise FlinkWinError(rc, msg.decode() if msg else "")
    return rc
