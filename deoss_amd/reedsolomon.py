"""Python mirror of the klauspost/reedsolomon Encoder DeOSS fragments use (``dm_rs_*``).

cess-go-sdk (go.mod:8) codes every 32 MiB segment into ``chain.DataShards = 4`` data and
``chain.ParShards = 8`` parity fragments (``node/tracker.go:250,369``,
``node/fileHandler.go:250``) with ``github.com/klauspost/reedsolomon v1.12.4`` (``go.mod:65``).
:func:`New` mirrors ``reedsolomon.New(dataShards, parityShards)``; the returned
:class:`Encoder` has ``Split``, ``Encode``, ``Reconstruct`` and ``Verify`` with the same
argument meaning (a list of shards, ``None`` / empty for a missing one) and the same errors
(too few shards, short data).  Every byte is coded on the GPU (``rs_code_kernel``); there is no
CPU fallback.  Device-resident forms take raw device pointers and a HIP stream handle.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

from ._lib import DM_ERR_EMPTY, DeossMerkleError
from .merkle import MerkleContext

DATA_SHARDS = 4     # chain.DataShards
PAR_SHARDS = 8      # chain.ParShards


class ErrTooFewShards(DeossMerkleError):
    pass


class Encoder:
    def __init__(self, ctx: MerkleContext, data_shards: int, parity_shards: int):
        self._ctx = ctx
        self._L = ctx._L
        h = ctypes.c_void_p()
        rc = self._L.dm_rs_create(ctx._h, data_shards, parity_shards, ctypes.byref(h))
        ctx._check(rc, "dm_rs_create")
        self._h = h
        ctx._children.add(self)   # the context destroys this coder before itself
        self.data_shards = data_shards
        self.parity_shards = parity_shards
        self.total_shards = data_shards + parity_shards

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.dm_rs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> None:
        if rc == 0:
            return
        detail = (self._L.dm_last_error(self._ctx._h) or b"").decode()
        if "too few shards" in detail:
            raise ErrTooFewShards(rc, "too few shards given")
        if rc == DM_ERR_EMPTY:
            raise DeossMerkleError(rc, "not enough data to fill the number of requested shards")
        raise DeossMerkleError(rc, f"{what}: {self._L.dm_strerror(rc).decode()}: {detail}")

    def matrix(self) -> List[List[int]]:
        k, t = self.data_shards, self.total_shards
        out = ctypes.create_string_buffer(t * k)
        self._check(self._L.dm_rs_matrix(self._h, out), "dm_rs_matrix")
        return [list(out.raw[r * k:(r + 1) * k]) for r in range(t)]

    # -- klauspost Encoder API (host shards) ---------------------------------------------------
    def Split(self, data: bytes) -> List[bytes]:
        """Equal-size data shards (ceil(len / data)), the last zero-padded, plus empty parity."""
        if len(data) == 0:
            raise DeossMerkleError(DM_ERR_EMPTY, "not enough data to fill the number of requested shards")
        per = (len(data) + self.data_shards - 1) // self.data_shards
        b = bytes(data) + bytes(per * self.data_shards - len(data))
        return [b[i * per:(i + 1) * per] for i in range(self.data_shards)] + \
            [bytes(per) for _ in range(self.parity_shards)]

    def Encode(self, shards: List[bytes]) -> List[bytes]:
        """Fill shards[data:] with parity; returns the (new) shard list."""
        k, m = self.data_shards, self.parity_shards
        if len(shards) != self.total_shards:
            raise DeossMerkleError(-2, "too few shards given")
        n = len(shards[0])
        if any(len(s) != n for s in shards[:k]) or n == 0:
            raise DeossMerkleError(-2, "shard sizes do not match")
        ins = [ctypes.create_string_buffer(bytes(s), n) for s in shards[:k]]
        outs = [ctypes.create_string_buffer(n) for _ in range(m)]
        dp = (ctypes.c_void_p * k)(*[ctypes.addressof(b) for b in ins])
        pp = (ctypes.c_void_p * m)(*[ctypes.addressof(b) for b in outs])
        self._check(self._L.dm_rs_encode(self._h, dp, pp, n), "dm_rs_encode")
        return list(shards[:k]) + [b.raw for b in outs]

    def EncodeBuffer(self, data: bytes) -> List[bytes]:
        """Split + Encode of one segment in one call (dm_rs_encode_buffer)."""
        k, t = self.data_shards, self.total_shards
        if len(data) == 0:
            raise DeossMerkleError(DM_ERR_EMPTY, "not enough data to fill the number of requested shards")
        per = (len(data) + k - 1) // k
        out = ctypes.create_string_buffer(per * t)
        got = ctypes.c_uint64()
        src = ctypes.create_string_buffer(bytes(data), len(data))
        self._check(self._L.dm_rs_encode_buffer(self._h, src, len(data), out, ctypes.byref(got)),
                    "dm_rs_encode_buffer")
        assert got.value == per
        raw = out.raw
        return [raw[i * per:(i + 1) * per] for i in range(t)]

    def Reconstruct(self, shards: Sequence[Optional[bytes]]) -> List[bytes]:
        """Rebuild missing shards (None or empty); returns the complete list."""
        t = self.total_shards
        if len(shards) != t:
            raise DeossMerkleError(-2, "too few shards given")
        sizes = {len(s) for s in shards if s}
        if len(sizes) != 1:
            if not sizes:
                raise ErrTooFewShards(-2, "too few shards given")
            raise DeossMerkleError(-2, "shard sizes do not match")
        n = sizes.pop()
        bufs = [ctypes.create_string_buffer(bytes(s) if s else bytes(n), n) for s in shards]
        present = bytes(int(bool(s)) for s in shards)
        ptrs = (ctypes.c_void_p * t)(*[ctypes.addressof(b) for b in bufs])
        self._check(self._L.dm_rs_reconstruct(self._h, ptrs, present, n), "dm_rs_reconstruct")
        return [b.raw for b in bufs]

    def Verify(self, shards: Sequence[bytes]) -> bool:
        t = self.total_shards
        if len(shards) != t:
            raise DeossMerkleError(-2, "too few shards given")
        n = len(shards[0])
        bufs = [ctypes.create_string_buffer(bytes(s), max(n, 1)) for s in shards]
        ptrs = (ctypes.c_void_p * t)(*[ctypes.addressof(b) for b in bufs])
        ok = ctypes.c_int()
        self._check(self._L.dm_rs_verify(self._h, ptrs, n, ctypes.byref(ok)), "dm_rs_verify")
        return bool(ok.value)

    # -- device-resident forms -----------------------------------------------------------------
    def encode_device_async(self, data_ptr: int, data_stride: int, parity_ptr: int, parity_stride: int, shard: int,
                            nseg: int = 1, stream: int = 0) -> None:
        self._check(self._L.dm_rs_encode_device_async(self._h, data_ptr, data_stride, parity_ptr, parity_stride,
                                                       shard, nseg, stream), "dm_rs_encode_device_async")

    def reconstruct_device_async(self, shard_ptrs: Sequence[int], present: Sequence[bool], shard: int,
                                 stream: int = 0) -> None:
        t = self.total_shards
        ptrs = (ctypes.c_void_p * t)(*shard_ptrs)
        pres = bytes(int(bool(p)) for p in present)
        self._check(self._L.dm_rs_reconstruct_device_async(self._h, ptrs, pres, shard, stream),
                    "dm_rs_reconstruct_device_async")


def New(ctx: MerkleContext, data_shards: int = DATA_SHARDS, parity_shards: int = PAR_SHARDS) -> Encoder:
    """reedsolomon.New(dataShards, parityShards) on the context's first GPU."""
    return Encoder(ctx, data_shards, parity_shards)
