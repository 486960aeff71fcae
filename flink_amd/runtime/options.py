"""Job configuration switches of the GPU window aggregation (Config/flags).

The reference keeps its knobs as ``ConfigOption``s beside ``table.exec.*``
(flink-table/flink-table-api-java/.../config/ExecutionConfigOptions.java); the shim adds two, read by
both builder seams before anything touches a device:

* ``gpu.window-agg.enabled`` (default false): eligible window aggregations run on the GPU; off, every
  operator stays on the reference path unchanged.
* ``gpu.window-agg.device`` (default -1): the HIP device of a subtask's handle; -1 maps subtask
  ``i`` to device ``i % device_count`` (``fw_config.device``).

``conf`` is any mapping of option keys to values (Flink's ``Configuration.toMap()`` form: strings, or
already-typed values)."""
GPU_WINDOW_AGG_ENABLED = "gpu.window-agg.enabled"
GPU_WINDOW_AGG_DEVICE = "gpu.window-agg.device"
DEFAULTS = {GPU_WINDOW_AGG_ENABLED: False, GPU_WINDOW_AGG_DEVICE: -1}


def _bool(v):
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("true", "1", "yes"):
        return True
    if s in ("false", "0", "no"):
        return False
    raise ValueError(f"Could not parse value '{v}' for key '{GPU_WINDOW_AGG_ENABLED}'.")


def gpu_enabled(conf):
    """``gpu.window-agg.enabled`` of ``conf`` (default false)."""
    return _bool(conf.get(GPU_WINDOW_AGG_ENABLED, DEFAULTS[GPU_WINDOW_AGG_ENABLED]))


def gpu_device(conf, subtask_index, device_count):
    """The device of subtask ``subtask_index``: ``gpu.window-agg.device``, or -1 -> subtask modulo the
    visible devices."""
    d = int(conf.get(GPU_WINDOW_AGG_DEVICE, DEFAULTS[GPU_WINDOW_AGG_DEVICE]))
    if d >= 0:
        return d
    if device_count <= 0:
        raise ValueError("no GPU device visible")
    return subtask_index % device_count
