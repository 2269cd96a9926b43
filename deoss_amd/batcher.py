"""Coalescing executor for concurrent callers (``dm_batcher_*``).

Upload handlers (one goroutine / thread per request) each hash or process one object.  Called one
at a time, every request would keep only a handful of SIMDs busy; :class:`Batcher` accepts
blocking calls from any number of threads and turns whatever is queued into one batched GPU pass
(one leaf launch over every queued request's leaves, one tree per request).  Results are
identical to :meth:`MerkleContext.root_buffer` / :meth:`Processor.process_buffer`.  ctypes
releases the GIL during the call, so Python threads really wait in parallel.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

from ._lib import DM_ERR_EMPTY, DeossMerkleError, load_library

ROOT = 0
PROCESS = 1


class Batcher:
    def __init__(self, mode: int, unit: int, data_shards: int = 4, parity_shards: int = 8, device=0,
                 slots: int = 0, max_leaves: int = 0, max_bytes: int = 0, linger_us: int = 0):
        """device: a GPU ordinal, a list of them (slots per GPU), or None for every visible GPU."""
        self._L = load_library()
        h = ctypes.c_void_p()
        devs = None if device is None else ([device] if isinstance(device, int) else list(device))
        arr = (ctypes.c_int * len(devs))(*devs) if devs else None
        rc = self._L.dm_batcher_create(arr, len(devs) if devs else 0, mode, unit, data_shards, parity_shards, slots,
                                       max_leaves, max_bytes, linger_us, ctypes.byref(h))
        if rc != 0:
            raise DeossMerkleError(rc, f"dm_batcher_create: {self._L.dm_batcher_last_error().decode()}")
        self._h = h
        self.mode, self.unit = mode, unit
        self.k, self.m = data_shards, parity_shards

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.dm_batcher_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> None:
        if rc == 0:
            return
        if rc == DM_ERR_EMPTY:
            raise DeossMerkleError(rc, "Empty data")
        raise DeossMerkleError(rc, f"{what}: {self._L.dm_strerror(rc).decode()}: "
                                   f"{self._L.dm_batcher_last_error().decode()}")

    @staticmethod
    def _src(buf):
        """(pointer, length) of bytes, a ctypes array, or an (address, length) pair of host memory."""
        if isinstance(buf, tuple):
            return ctypes.c_void_p(buf[0]), buf[1], None
        if isinstance(buf, ctypes.Array):
            return buf, len(buf), buf
        keep = ctypes.create_string_buffer(bytes(buf), max(len(buf), 1))
        return keep, len(buf), keep

    def root(self, buf, want_leaves: bool = False) -> Tuple[Optional[bytes], bytes]:
        """NewHashTreeFromBuffer(buf, unit) through the batcher: (leaf digests or None, root)."""
        src, n, _keep = self._src(buf)
        nl = (n + self.unit - 1) // self.unit
        leaves = ctypes.create_string_buffer(max(32 * nl, 32)) if want_leaves else None
        root = ctypes.create_string_buffer(32)
        self._check(self._L.dm_batcher_root(self._h, src, n, leaves, root), "dm_batcher_root")
        return (leaves.raw[:32 * nl] if leaves is not None else None), root.raw

    def process(self, buf, want_frags: bool = False) -> Tuple[bytes, bytes, bytes, Optional[bytes]]:
        """FullProcessing of one object through the batcher: (segment digests, fragment digests,
        fid, fragments or None)."""
        src, n, _keep = self._src(buf)
        nseg = (n + self.unit - 1) // self.unit
        total = self.k + self.m
        seg = ctypes.create_string_buffer(max(32 * nseg, 32))
        frag = ctypes.create_string_buffer(max(32 * nseg * total, 32))
        fid = ctypes.create_string_buffer(32)
        frags = ctypes.create_string_buffer(nseg * total * (self.unit // self.k)) if (want_frags and nseg) else None
        self._check(self._L.dm_batcher_process(self._h, src, n, frags, seg, frag, fid), "dm_batcher_process")
        return seg.raw[:32 * nseg], frag.raw[:32 * nseg * total], fid.raw, (frags.raw if frags is not None else None)

    def stats(self) -> Tuple[int, int, int]:
        """(requests served, batches launched, largest batch in requests)."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self._L.dm_batcher_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
                    "dm_batcher_stats")
        return a.value, b.value, c.value
