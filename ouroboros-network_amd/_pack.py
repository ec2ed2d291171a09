"""Host-side packing of batches into the structure-of-arrays layout the C ABI
takes (include/ouro_verify.h): fixed-size fields as contiguous (n, k) uint8
arrays, variable-length messages as one buffer addressed by (offset, length)."""
from __future__ import annotations

from typing import Iterable, Sequence, Tuple

import numpy as np


def as_rows(x, width: int, name: str) -> np.ndarray:
    """(n, width) C-contiguous uint8 from bytes rows / a 2-D array."""
    if isinstance(x, np.ndarray):
        a = np.ascontiguousarray(x, dtype=np.uint8)
        if a.ndim == 1:
            a = a.reshape(-1, width)
    else:
        rows = list(x)
        for r in rows:
            if len(r) != width:
                raise ValueError(f"{name}: every entry must be {width} bytes, got {len(r)}")
        a = np.frombuffer(b"".join(bytes(r) for r in rows), dtype=np.uint8).reshape(-1, width)
        a = np.ascontiguousarray(a)
    if a.shape[1:] != (width,):
        raise ValueError(f"{name}: expected shape (n, {width}), got {a.shape}")
    return a


def pack_messages(msgs: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Concatenate messages; returns (buffer, offsets u64, lengths u32)."""
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint32, count=len(msgs))
    offs = np.zeros(len(msgs), dtype=np.uint64)
    if len(msgs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bytes(m) for m in msgs) or b"\0", dtype=np.uint8)
    return np.ascontiguousarray(buf), offs, lens


def fixed_messages(rows: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(n, k) equal-length messages -> (buffer, offsets, lengths) without copying."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    n, k = rows.shape
    offs = np.arange(n, dtype=np.uint64) * np.uint64(k)
    lens = np.full(n, k, dtype=np.uint32)
    return rows.reshape(-1), offs, lens


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None else 0


def msgs_arg(msgs) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Accept list[bytes], (n, k) array, or a ready (buf, off, len) triple."""
    if isinstance(msgs, tuple) and len(msgs) == 3:
        buf, off, ln = msgs
        return (np.ascontiguousarray(buf, dtype=np.uint8),
                np.ascontiguousarray(off, dtype=np.uint64),
                np.ascontiguousarray(ln, dtype=np.uint32))
    if isinstance(msgs, np.ndarray) and msgs.ndim == 2:
        return fixed_messages(msgs)
    return pack_messages(list(msgs))


def ints(x: Iterable[int], dtype) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(list(x) if not isinstance(x, np.ndarray) else x,
                                           dtype=dtype))
