"""Host RowData -> columnar key rows for VARCHAR / composite keys.

The SQL window operator keys its state by the BinaryRowData the key projection writes
(BinaryRowDataKeySelector.getKey, flink-table-runtime/.../keyselector/BinaryRowDataKeySelector.java:54)
and routes records by that row's hashCode (BinaryRowData.java:459 -> MurmurHashUtils
.hashBytesByWords, KeyGroupStreamPartitioner.java:55-65).  For keys that are not a single
BIGINT / INT, this module turns the key rows of a batch into:

  * the key's identity in the window state: a dense int64 id per distinct key row
    (``KeyDictionary``; results come back as ids and are mapped back to the key rows), and
  * the key-row columns (``KeyRowColumns``: one 8-byte column per fixed-width field, offsets +
    bytes per string field, NULL flags) from which ``fw_key_row_hash`` computes the Java hash
    on the device (or ``fw_host_key_row_hash`` on the host for host-staged partitioning).

The handle then runs with ``FW_KEYHASH_PRECOMPUTED``: the hash decides key group, subtask and
superbucket exactly as the reference's key group does.
"""
import ctypes as C

import numpy as np

from .. import abi
from .._native import check, lib


def _fixed_bits(kind, sql_type, v):
    """The 8-byte column value whose low `kind` bytes BinaryRowWriter writes for v."""
    if sql_type == "DOUBLE":
        return int(np.float64(v).view(np.int64))
    if sql_type == "FLOAT":
        return int(np.float32(v).view(np.int32))
    if sql_type == "BOOLEAN":
        return 1 if v else 0
    return int(v)


class KeyRowColumns:
    """Columnar key rows of one batch.  ``types`` are SQL type names (abi.KEY_FIELD_KINDS)."""

    def __init__(self, types, fixed, offsets, data, nulls, n):
        self.types = list(types)
        self.kinds = [abi.KEY_FIELD_KINDS[t] for t in self.types]
        self.fixed, self.offsets, self.data, self.nulls, self.n = fixed, offsets, data, nulls, n

    @classmethod
    def from_rows(cls, rows, types):
        """rows: sequence of key tuples (str / bytes for string fields, numbers otherwise, None
        for NULL)."""
        types = list(types)
        if not 1 <= len(types) <= abi.FW_MAX_KEY_FIELDS:
            raise ValueError(f"key rows need 1..{abi.FW_MAX_KEY_FIELDS} fields")
        for t in types:
            if t not in abi.KEY_FIELD_KINDS:
                raise ValueError(f"key field type {t} is not supported on the GPU")
        n = len(rows)
        fixed, offsets, data, nulls = [], [], [], []
        for f, t in enumerate(types):
            kind = abi.KEY_FIELD_KINDS[t]
            nl = np.zeros(n, dtype=np.uint8)
            if kind == abi.KF_STRING:
                parts, off = [], np.zeros(n + 1, dtype=np.int32)
                pos = 0
                for i, r in enumerate(rows):
                    v = r[f]
                    if v is None:
                        nl[i] = 1
                        b = b""
                    else:
                        b = v.encode("utf-8") if isinstance(v, str) else bytes(v)
                    parts.append(b)
                    pos += len(b)
                    off[i + 1] = pos
                buf = np.frombuffer(b"".join(parts) + b"\0" * 4, dtype=np.uint8).copy()  # tail: dword reads
                fixed.append(None)
                offsets.append(off)
                data.append(buf)
            else:
                col = np.zeros(n, dtype=np.int64)
                for i, r in enumerate(rows):
                    if r[f] is None:
                        nl[i] = 1
                    else:
                        v = _fixed_bits(kind, t, r[f]) & 0xFFFFFFFFFFFFFFFF
                        col[i] = v - (1 << 64) if v >> 63 else v
                fixed.append(col)
                offsets.append(None)
                data.append(None)
            nulls.append(nl if nl.any() else None)
        return cls(types, fixed, offsets, data, nulls, n)

    def to(self, device):
        """A copy with every column as a torch tensor on `device` (for fw_key_row_hash)."""
        import torch

        def t(a):
            return None if a is None else torch.from_numpy(a).to(device)
        return KeyRowColumns(self.types, [t(a) for a in self.fixed], [t(a) for a in self.offsets],
                             [t(a) for a in self.data], [t(a) for a in self.nulls], self.n)

    def fields(self):
        """The fw_key_field array (pointers into this object's columns)."""
        arr = (abi.fw_key_field * len(self.kinds))()

        def ptr(a):
            if a is None:
                return None
            return a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data
        for f, k in enumerate(self.kinds):
            arr[f].kind = k
            arr[f].fixed = ptr(self.fixed[f])
            arr[f].offsets = ptr(self.offsets[f])
            arr[f].bytes = ptr(self.data[f])
            arr[f].nulls = ptr(self.nulls[f])
        return arr

    def hash_host(self):
        """BinaryRowData.hashCode per row (fw_host_key_row_hash; host columns)."""
        out = np.empty(self.n, dtype=np.int32)
        check(lib().fw_host_key_row_hash(self.fields(), len(self.kinds), self.n, out.ctypes.data))
        return out

    def hash_device(self, stream=None):
        """BinaryRowData.hashCode per row computed on the device (fw_key_row_hash); the columns
        must be cuda tensors (see ``to``).  Returns an int32 cuda tensor."""
        import torch
        dev = next(a.device for a in self.offsets + self.fixed if a is not None)
        out = torch.empty(self.n, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream if stream is None else stream
        check(lib().fw_key_row_hash(self.fields(), len(self.kinds), self.n, out.data_ptr(), C.c_void_p(s)))
        return out


class KeyDictionary:
    """Dense int64 ids for distinct key rows: the key's identity in the device window state."""

    def __init__(self):
        self._ids = {}
        self._rows = []

    def encode(self, rows):
        out = np.empty(len(rows), dtype=np.int64)
        ids, lst = self._ids, self._rows
        for i, r in enumerate(rows):
            r = tuple(r)
            k = ids.get(r)
            if k is None:
                k = ids[r] = len(lst)
                lst.append(r)
            out[i] = k
        return out

    def decode(self, key_id):
        return self._rows[int(key_id)]

    def __len__(self):
        return len(self._rows)
