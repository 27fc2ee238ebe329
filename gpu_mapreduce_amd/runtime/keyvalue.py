"""Callback-facing KeyValue and value codecs.

`KeyValue` is what user map/reduce callbacks receive (MR-MPI's KeyValue*,
reference src/keyvalue.h:55-57). It wraps the native `HostKV` builder:
host-emitted pairs are packed into contiguous byte arrays in C++, device
batches (tensors produced on the GPU) are appended as-is, so a callback can
emit millions of pairs without per-pair Python objects by using
`add_tensors` / `add_kv`.

Encoding of Python objects to key/value bytes (`to_bytes`):
  bytes/bytearray/memoryview -> raw bytes
  str   -> UTF-8 + NUL terminator (the C-string convention the reference apps
           use, e.g. wordfreq's kv->add(word, strlen(word)+1, ...))
  int   -> 8-byte little-endian signed (use numpy scalars for other widths)
  float -> 8-byte IEEE double
  numpy scalar / array -> its raw bytes;  torch tensor -> its raw bytes
  None  -> b"" (NULL value)
"""
from __future__ import annotations

import struct

import numpy as np
import torch

from .._ext import C


def to_bytes(x) -> bytes:
    if x is None:
        return b""
    if isinstance(x, (bytes, bytearray, memoryview)):
        return bytes(x)
    if isinstance(x, str):
        return x.encode("utf-8") + b"\0"
    if isinstance(x, bool):
        return struct.pack("<i", int(x))
    if isinstance(x, int):
        return struct.pack("<q", x)
    if isinstance(x, float):
        return struct.pack("<d", x)
    if isinstance(x, np.generic):
        return x.tobytes()
    if isinstance(x, np.ndarray):
        return np.ascontiguousarray(x).tobytes()
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().contiguous().numpy().tobytes()
    raise TypeError(f"cannot encode {type(x).__name__} as key/value bytes")


def _byte_view(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    return t.view(torch.uint8).reshape(-1) if t.dtype != torch.uint8 else t.reshape(-1)


class KeyValue:
    """Append-only KV builder handed to map/reduce callbacks."""

    def __init__(self, device: str | None = None, native=None):
        self._h = native if native is not None else C.HostKV(device)
        self.device = self._h.device

    @classmethod
    def wrap(cls, native):
        """Python view of a native KeyValue handed to a callback by the engine."""
        return cls(native=native)

    # --- MR-MPI KeyValue::add(key, keybytes, value, valuebytes) ----------------
    def add(self, key, value=None):
        self._h.add(to_bytes(key), to_bytes(value))

    # --- add(n, keys, keybytes, values, valuebytes): fixed sizes --------------
    def add_multi_static(self, keys, values):
        ks = [to_bytes(k) for k in keys]
        vs = [to_bytes(v) for v in values]
        if not ks:
            return
        kb, vb = len(ks[0]), len(vs[0])
        if any(len(k) != kb for k in ks) or any(len(v) != vb for v in vs):
            raise ValueError("add_multi_static: keys/values must have uniform sizes")
        self._h.add_fixed(len(ks), b"".join(ks), kb, b"".join(vs), vb)

    # --- add(n, keys, keybytes[], values, valuebytes[]): variable sizes -------
    def add_multi_dynamic(self, keys, values):
        ks = [to_bytes(k) for k in keys]
        vs = [to_bytes(v) for v in values]
        self._h.add_var(b"".join(ks), [len(k) for k in ks], b"".join(vs), [len(v) for v in vs])

    # --- device fast paths ------------------------------------------------------
    def add_kv(self, kv):
        """Append a native KV batch (e.g. from a kernel) without host copies."""
        self._h.add_kv(kv)

    def enable_grouping(self):
        """Group pairs by key as they are added (call before the first add):
        a convert() right after this map then finds the group-by done
        (csrc/engine/grouper.h). Worth it when the map streams its input and
        the device would otherwise idle between batches."""
        self._h.enable_grouping()

    def reserve_grouping(self, rows: int, key_bytes: int, value_bytes: int, groups: int | None = None):
        """Capacity hint for the grouped arenas: sized once for the whole map
        (no regrow copies or hash-table rehash while the input streams).
        groups: distinct keys to size the hash table for (None: as many as
        rows — mostly distinct keys; 0: sized from a sample of the first
        part — keys that repeat, such as words)."""
        self._h.reserve_grouping(int(rows), int(key_bytes), int(value_bytes), -1 if groups is None else int(groups))

    @property
    def grouping(self) -> bool:
        return self._h.grouping

    def add_tensors(self, keys: torch.Tensor, values: torch.Tensor | None = None,
                    koff: torch.Tensor | None = None, voff: torch.Tensor | None = None):
        """Append n pairs from tensors. Fixed width: `keys` is [n, ...] and each
        row is one key (any dtype). Variable width: `keys` is a flat uint8 byte
        array and `koff` its int64 [n+1] offsets. Same for values; values=None
        means NULL values."""
        if koff is not None:
            n = koff.numel() - 1
        else:
            n = keys.shape[0] if keys.dim() > 0 else 1
        kd = _byte_view(keys)
        vd = _byte_view(values) if values is not None else torch.empty(0, dtype=torch.uint8, device=keys.device)
        if values is not None and voff is None and values.shape[0] != n:
            raise ValueError("add_tensors: keys and values must have the same number of rows")
        self._h.add_kv(C.make_kv(kd, koff, vd, voff, n, self.device))

    def size(self) -> int:
        return self._h.size()

    def finish(self):
        return self._h.finish()
