"""Host RowData -> columnar key rows for VARCHAR / composite keys.

The SQL window operator keys its state by the BinaryRowData the key projection writes
(BinaryRowDataKeySelector.getKey, flink-table-runtime/.../keyselector/BinaryRowDataKeySelector.java:54)
and routes records by that row's hashCode (BinaryRowData.java:459 -> MurmurHashUtils
.hashBytesByWords, KeyGroupStreamPartitioner.java:55-65).  For keys that are not a single
BIGINT / INT, this module turns the key rows of a batch into:

  * the key-row columns (``KeyRowColumns``: one 8-byte column per fixed-width field, offsets +
    bytes per string field, NULL flags), and
  * the key rows' BinaryRowData images (``images_host`` / ``images_device``: the bytes
    BinaryRowWriter writes, what the reference's state keys on and BinaryRowData.equals compares).

A ``FW_KEYHASH_KEYROW`` handle takes the images (fw_reserve staging or fw_push_device_key_rows),
interns them in an HBM table (the key's identity is its bytes) and routes each by its
BinaryRowData.hashCode; results come back with their key rows (``decode_key_row``).  The
columnar hash (``fw_key_row_hash`` / ``fw_host_key_row_hash``) serves host-side partitioners.
"""
import struct

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
        """A copy with every column as a torch tensor on `device` (for fw_key_row_hash /
        images_device); the image offsets are computed from the host columns first."""
        import torch

        def t(a):
            return None if a is None else torch.from_numpy(a).to(device)
        out = KeyRowColumns(self.types, [t(a) for a in self.fixed], [t(a) for a in self.offsets],
                            [t(a) for a in self.data], [t(a) for a in self.nulls], self.n)
        out._img_off = self.image_offsets()
        return out

    def image_offsets(self):
        """Arrow offsets (n + 1) of the rows' BinaryRowData images (host columns)."""
        lens = np.empty(self.n, dtype=np.int64)
        check(lib().fw_host_key_row_image_lengths(self.fields(), len(self.kinds), self.n, lens.ctypes.data))
        off = np.zeros(self.n + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        return off

    def images_host(self):
        """(offsets, bytes) of the rows' BinaryRowData images (fw_host_key_row_images)."""
        off = self.image_offsets()
        buf = np.zeros(max(int(off[-1]) // 8, 1), dtype=np.uint64).view(np.uint8)  # 8-byte aligned
        check(lib().fw_host_key_row_images(self.fields(), len(self.kinds), self.n, off.ctypes.data, buf.ctypes.data))
        return off, buf[:int(off[-1])]

    def images_device(self, stream=None):
        """(offsets, bytes) cuda tensors: the images written on the device (fw_key_row_images);
        this object must come from ``to``."""
        import torch
        dev = next(a.device for a in self.offsets + self.fixed if a is not None)
        off = torch.from_numpy(self._img_off).to(dev)
        nb = int(self._img_off[-1])
        buf = torch.zeros(max(nb // 8, 1), dtype=torch.int64, device=dev).view(torch.uint8)
        s = torch.cuda.current_stream(dev).cuda_stream if stream is None else stream
        check(lib().fw_key_row_images(self.fields(), len(self.kinds), self.n, off.data_ptr(), buf.data_ptr(), C.c_void_p(s)))
        return off, buf

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


def decode_key_row(image, types):
    """A key row image (BinaryRowData bytes) back to a tuple of Python values by SQL type --
    BinaryRowData.getLong / getInt / getString... (NULL -> None)."""
    image = bytes(image)
    n = len(types)
    nb = ((n + 71) // 64) * 8
    hdr = int.from_bytes(image[:8], "little")
    out = []
    for f, t in enumerate(types):
        if (hdr >> (8 + f)) & 1:
            out.append(None)
            continue
        slot = image[nb + 8 * f:nb + 8 * f + 8]
        kind = abi.KEY_FIELD_KINDS[t]
        if kind == abi.KF_STRING:
            w = int.from_bytes(slot, "little")
            if w >> 63:  # inline: length in the high byte
                ln = (w >> 56) & 0x7F
                b = slot[:ln]
            else:
                o, ln = w >> 32, w & 0xFFFFFFFF
                b = image[o:o + ln]
            out.append(b.decode("utf-8") if t in ("VARCHAR", "CHAR", "STRING") else bytes(b))
        elif t == "DOUBLE":
            out.append(struct.unpack("<d", slot)[0])
        elif t == "FLOAT":
            out.append(struct.unpack("<f", slot[:4])[0])
        elif t == "BOOLEAN":
            out.append(slot[0] != 0)
        else:
            out.append(int.from_bytes(slot[:kind], "little", signed=True))
    return tuple(out)
