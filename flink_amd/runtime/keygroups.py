"""KeyGroupRangeAssignment mirror (flink-runtime/.../state/KeyGroupRangeAssignment.java).

Scalar helpers run on the host through the library's host entry points (the same code the
kernels run); bulk assignment runs on the device (fw_assign_key_groups).
"""
from .. import abi
from .._native import check, lib

DEFAULT_LOWER_BOUND_MAX_PARALLELISM = 1 << 7   # :32
UPPER_BOUND_MAX_PARALLELISM = 1 << 15


def compute_default_max_parallelism(operator_parallelism):
    """computeDefaultMaxParallelism (:137-147)."""
    p = operator_parallelism + operator_parallelism // 2
    r = 1
    while r < p:
        r <<= 1
    return min(max(r, DEFAULT_LOWER_BOUND_MAX_PARALLELISM), UPPER_BOUND_MAX_PARALLELISM)


def assign_to_key_group(key, max_parallelism, key_hash_kind=abi.KEYHASH_LONG, precomputed_hash=0):
    """assignToKeyGroup (:63) for the key.hashCode() defined by key_hash_kind."""
    return lib().fw_host_key_group(key_hash_kind, int(key), int(precomputed_hash), max_parallelism)


def compute_key_group_range_for_operator_index(max_parallelism, parallelism, operator_index):
    """computeKeyGroupRangeForOperatorIndex (:93-106) -> (start, end) inclusive."""
    if not (0 < parallelism <= max_parallelism):
        raise ValueError("Maximum parallelism must not be smaller than parallelism.")
    start = (operator_index * max_parallelism + parallelism - 1) // parallelism
    end = ((operator_index + 1) * max_parallelism - 1) // parallelism
    return start, end


def compute_operator_index_for_key_group(max_parallelism, parallelism, key_group):
    """computeOperatorIndexForKeyGroup (:124-127)."""
    return key_group * parallelism // max_parallelism


def assign_key_to_parallel_operator(key, max_parallelism, parallelism, key_hash_kind=abi.KEYHASH_LONG):
    """assignKeyToParallelOperator (:49)."""
    return compute_operator_index_for_key_group(
        max_parallelism, parallelism, assign_to_key_group(key, max_parallelism, key_hash_kind))


def assign_key_groups_device(keys, max_parallelism, parallelism, key_hash_kind, stream=None):
    """Bulk (kg, dest) for a cuda int64 tensor of keys."""
    import torch
    n = keys.numel()
    kg = torch.empty(n, dtype=torch.int32, device=keys.device)
    dest = torch.empty(n, dtype=torch.int32, device=keys.device)
    s = stream if stream is not None else torch.cuda.current_stream(keys.device).cuda_stream
    check(lib().fw_assign_key_groups(keys.data_ptr(), None, n, key_hash_kind, max_parallelism,
                                     parallelism, kg.data_ptr(), dest.data_ptr(), s))
    return kg, dest
