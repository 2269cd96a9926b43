"""Python host binding of the MI355X Merkle path (ctypes over include/deoss_merkle.h).

:class:`MerkleContext` owns a ``dm_ctx`` (one or more GPUs of this process) and exposes the
C-ABI entry points with Python types.  Device-resident entry points take raw device pointers
(ints) and a HIP stream handle, so they can be driven from ``torch`` tensors
(``t.data_ptr()``, ``torch.cuda.current_stream().cuda_stream``) without any torch type crossing
the boundary.  ``stream=0`` is HIP's null stream (torch's default stream): work is ordered with
torch's own kernels and copies on that stream.
"""
from __future__ import annotations

import ctypes
import weakref
from typing import List, Optional, Sequence, Tuple

from ._lib import DM_ERR_EMPTY, DeossMerkleError, load_library


class MerkleContext:
    def __init__(self, devices: Optional[Sequence[int]] = None, lanes: Optional[int] = None):
        """``lanes``: call lanes per GPU (``dm_create_lanes``); None = ``DEOSS_LANES``, else sized
        from free HBM (4 on an MI355X)."""
        self._L = load_library()
        h = ctypes.c_void_p()
        arr = (ctypes.c_int * len(devices))(*devices) if devices else None
        n = len(devices) if devices else 0
        if lanes is None:
            rc = self._L.dm_create(ctypes.byref(h), arr, n)
        else:
            rc = self._L.dm_create_lanes(ctypes.byref(h), arr, n, int(lanes))
        if rc != 0:
            raise DeossMerkleError(rc, f"dm_create: {self._L.dm_strerror(rc).decode()}")
        self._h = h
        # objects holding C handles that point into this context (dm_rs coders): closed first
        self._children = weakref.WeakSet()

    # -- lifecycle -------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            for child in list(getattr(self, "_children", ())):
                child.close()
            self._L.dm_destroy(self._h)
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

    @property
    def device_count(self) -> int:
        return self._L.dm_device_count(self._h)

    @property
    def lane_count(self) -> int:
        return self._L.dm_lane_count(self._h)

    @property
    def can_shard(self) -> bool:
        """Whether one object can be sharded over this context's GPUs (dm_can_shard): more than one
        GPU and RCCL communicators up.  A context whose RCCL init failed runs every call whole on
        one GPU."""
        return bool(self._L.dm_can_shard(self._h))

    def route_constants(self):
        """(all-gather microseconds, host bytes/s) this context's routing model uses
        (dm_route_constants): estimates, or DEOSS_ALLGATHER_US / DEOSS_HOST_BYTES_PER_S as set at
        dm_create."""
        ag, hb = ctypes.c_double(), ctypes.c_double()
        self._check(self._L.dm_route_constants(self._h, ctypes.byref(ag), ctypes.byref(hb)), "dm_route_constants")
        return ag.value, hb.value

    @staticmethod
    def keep_claimed(hip_device: int = 0) -> int:
        """Idle lane-buffer bytes every live context of this process may keep on that GPU
        (dm_keep_claimed): the per-GPU budget the default lane count is sized against."""
        out = ctypes.c_uint64()
        rc = load_library().dm_keep_claimed(hip_device, ctypes.byref(out))
        if rc != 0:
            raise DeossMerkleError(rc, "dm_keep_claimed failed")
        return out.value

    def _check(self, rc: int, what: str) -> None:
        if rc == 0:
            return
        if rc == DM_ERR_EMPTY:
            raise DeossMerkleError(rc, "Empty data")
        detail = (self._L.dm_last_error(self._h) or b"").decode()
        raise DeossMerkleError(rc, f"{what}: {self._L.dm_strerror(rc).decode()}: {detail}")

    # -- host-memory entry points ------------------------------------------------------------
    def new_hash_tree(self, paths: Sequence[str]) -> Tuple[List[bytes], bytes]:
        n = len(paths)
        arr = (ctypes.c_char_p * max(n, 1))(*[p.encode() for p in paths])
        leaf = ctypes.create_string_buffer(max(32 * n, 32))
        root = ctypes.create_string_buffer(32)
        rc = self._L.dm_new_hash_tree(self._h, arr, n, leaf, root)
        if rc != 0:
            if rc == DM_ERR_EMPTY:
                raise DeossMerkleError(rc, "Empty data")
            detail = (self._L.dm_last_error(self._h) or b"").decode()
            raise DeossMerkleError(rc, detail or self._L.dm_strerror(rc).decode())
        return [leaf.raw[32 * i:32 * i + 32] for i in range(n)], root.raw

    def root_chunks(self, chunks: Sequence[bytes]) -> Tuple[bytes, bytes]:
        """Returns (n*32 leaf digest bytes, root)."""
        n = len(chunks)
        ptrs = (ctypes.c_void_p * max(n, 1))()
        lens = (ctypes.c_uint64 * max(n, 1))()
        keep = []
        for i, c in enumerate(chunks):
            b = ctypes.create_string_buffer(bytes(c), max(len(c), 1))
            keep.append(b)
            ptrs[i] = ctypes.cast(b, ctypes.c_void_p)
            lens[i] = len(c)
        leaf = ctypes.create_string_buffer(max(32 * n, 32))
        root = ctypes.create_string_buffer(32)
        self._check(self._L.dm_root_chunks(self._h, ptrs, lens, n, leaf, root), "dm_root_chunks")
        return leaf.raw[:32 * n], root.raw

    def root_buffer_ptr(self, addr: int, length: int, chunk: int, want_leaves: bool = False
                        ) -> Tuple[Optional[bytes], bytes]:
        n = (length + chunk - 1) // chunk if length and chunk else 0
        leaf = ctypes.create_string_buffer(max(32 * n, 32)) if want_leaves else None
        root = ctypes.create_string_buffer(32)
        self._check(self._L.dm_root_buffer(self._h, ctypes.c_void_p(addr), length, chunk, leaf, root),
                    "dm_root_buffer")
        return (leaf.raw[:32 * n] if leaf is not None else None), root.raw

    def root_buffer(self, buf: bytes, chunk: int, want_leaves: bool = True) -> Tuple[Optional[bytes], bytes]:
        b = ctypes.create_string_buffer(bytes(buf), max(len(buf), 1))
        return self.root_buffer_ptr(ctypes.addressof(b), len(buf), chunk, want_leaves)

    def root_batch(self, objs: Sequence[bytes], chunk: int) -> List[bytes]:
        n = len(objs)
        ptrs = (ctypes.c_void_p * max(n, 1))()
        lens = (ctypes.c_uint64 * max(n, 1))()
        keep = []
        for i, o in enumerate(objs):
            b = ctypes.create_string_buffer(bytes(o), max(len(o), 1))
            keep.append(b)
            ptrs[i] = ctypes.cast(b, ctypes.c_void_p)
            lens[i] = len(o)
        roots = ctypes.create_string_buffer(max(32 * n, 32))
        self._check(self._L.dm_root_batch(self._h, ptrs, lens, n, chunk, roots), "dm_root_batch")
        return [roots.raw[32 * i:32 * i + 32] for i in range(n)]

    # -- device-resident entry points ---------------------------------------------------------
    def root_device(self, dev_ptr: int, length: int, chunk: int) -> bytes:
        root = ctypes.create_string_buffer(32)
        self._check(self._L.dm_root_device(self._h, ctypes.c_void_p(dev_ptr), length, chunk, root),
                    "dm_root_device")
        return root.raw

    def root_device_async(self, dev_ptr: int, length: int, chunk: int, dev_root: int,
                          dev_leaves: int = 0, stream: int = 0) -> None:
        self._check(self._L.dm_root_device_async(self._h, ctypes.c_void_p(dev_ptr), length, chunk,
                                                 ctypes.c_void_p(dev_root), ctypes.c_void_p(dev_leaves or None),
                                                 ctypes.c_void_p(stream or None)), "dm_root_device_async")

    def subtree_device_async(self, dev_ptr: int, length: int, chunk: int, levels: int, dev_nodes: int,
                             stream: int = 0) -> int:
        nout = ctypes.c_uint64()
        self._check(self._L.dm_subtree_device_async(self._h, ctypes.c_void_p(dev_ptr), length, chunk, levels,
                                                    ctypes.c_void_p(dev_nodes), ctypes.byref(nout),
                                                    ctypes.c_void_p(stream or None)), "dm_subtree_device_async")
        return nout.value

    def finish_device_async(self, dev_nodes: int, n: int, min_one_level: bool, dev_root: int,
                            stream: int = 0) -> None:
        self._check(self._L.dm_finish_device_async(self._h, ctypes.c_void_p(dev_nodes), n, int(min_one_level),
                                                   ctypes.c_void_p(dev_root), ctypes.c_void_p(stream or None)),
                    "dm_finish_device_async")

    def root_batch_device_async(self, dev_ptrs: Sequence[int], lens: Sequence[int], chunk: int, dev_roots: int,
                                stream: int = 0) -> None:
        n = len(dev_ptrs)
        ptrs = (ctypes.c_void_p * max(n, 1))(*dev_ptrs)
        ls = (ctypes.c_uint64 * max(n, 1))(*lens)
        self._check(self._L.dm_root_batch_device_async(self._h, ptrs, ls, n, chunk, ctypes.c_void_p(dev_roots),
                                                       ctypes.c_void_p(stream or None)),
                    "dm_root_batch_device_async")

    def fill_synthetic_async(self, dev_ptr: int, off: int, nbytes: int, seed: int, stream: int = 0) -> None:
        self._check(self._L.dm_fill_synthetic_async(self._h, ctypes.c_void_p(dev_ptr), off, nbytes, seed,
                                                    ctypes.c_void_p(stream or None)), "dm_fill_synthetic_async")

    def read_probe_async(self, dev_ptr: int, nbytes: int, dev_xor8: int, stream: int = 0) -> None:
        """HBM read-bandwidth probe: XOR of every 8-byte word of dev[0, nbytes) into dev_xor8."""
        self._check(self._L.dm_read_probe_async(self._h, ctypes.c_void_p(dev_ptr), nbytes, ctypes.c_void_p(dev_xor8),
                                                ctypes.c_void_p(stream or None)), "dm_read_probe_async")

    # -- tree levels and proofs (merkletree GetMerklePath / VerifyContent / VerifyTree) ----------
    def tree_node_count(self, n: int) -> int:
        return self._L.dm_tree_node_count(n)

    def tree_depth(self, n: int) -> int:
        return self._L.dm_tree_depth(n)

    def tree_levels(self, leaf_digests: bytes) -> bytes:
        """Levels 1 .. root over the leaf digests, level-major (the root is the last 32 bytes)."""
        n = len(leaf_digests) // 32
        if n == 0:
            raise DeossMerkleError(DM_ERR_EMPTY, "Empty data")
        out = ctypes.create_string_buffer(32 * self.tree_node_count(n))
        self._check(self._L.dm_tree_levels(self._h, bytes(leaf_digests), n, out), "dm_tree_levels")
        return out.raw

    def tree_root(self, leaf_digests: bytes) -> bytes:
        """Root of the tree over leaf digests (the fid of a list of segment digests)."""
        return self.tree_levels(leaf_digests)[-32:]

    def tree_levels_device_async(self, dev_leaves: int, n: int, dev_nodes: int, stream: int = 0) -> None:
        self._check(self._L.dm_tree_levels_device_async(self._h, ctypes.c_void_p(dev_leaves), n,
                                                        ctypes.c_void_p(dev_nodes), ctypes.c_void_p(stream or None)),
                    "dm_tree_levels_device_async")

    def merkle_paths(self, leaf_digests: bytes, indices: Sequence[int]) -> List[Tuple[List[bytes], List[int]]]:
        """GetMerklePath for each leaf index: (sibling digests, bits) with bits[i] = 1 when the
        sibling is the right child (merkletree's index convention)."""
        n = len(leaf_digests) // 32
        q = len(indices)
        depth = self.tree_depth(n)
        idx = (ctypes.c_uint64 * max(q, 1))(*indices)
        paths = ctypes.create_string_buffer(max(32 * depth * q, 32))
        bits = ctypes.create_string_buffer(max(depth * q, 1))
        self._check(self._L.dm_merkle_paths(self._h, bytes(leaf_digests), n, idx, q, paths, bits), "dm_merkle_paths")
        out = []
        for t in range(q):
            p = paths.raw[32 * depth * t:32 * depth * (t + 1)]
            out.append(([p[32 * l:32 * l + 32] for l in range(depth)], list(bits.raw[depth * t:depth * (t + 1)])))
        return out

    def merkle_paths_device_async(self, dev_leaves: int, dev_nodes: int, n: int, dev_idx: int, q: int,
                                  dev_paths: int, dev_bits: int, stream: int = 0) -> None:
        self._check(self._L.dm_merkle_paths_device_async(self._h, ctypes.c_void_p(dev_leaves),
                                                         ctypes.c_void_p(dev_nodes), n, ctypes.c_void_p(dev_idx), q,
                                                         ctypes.c_void_p(dev_paths), ctypes.c_void_p(dev_bits),
                                                         ctypes.c_void_p(stream or None)),
                    "dm_merkle_paths_device_async")

    def verify_paths(self, contents: Sequence[bytes], paths: Sequence[Sequence[bytes]], bits: Sequence[Sequence[int]],
                     roots: Sequence[bytes]) -> List[bool]:
        """ok[t]: SHA-256(contents[t]) folded with its path equals roots[t] (one root: shared)."""
        q = len(contents)
        if q == 0:
            return []
        depth = len(paths[0])
        if any(len(p) != depth for p in paths) or any(len(b) != depth for b in bits):
            raise DeossMerkleError(-2, "every path needs the same depth")
        ptrs = (ctypes.c_void_p * q)()
        lens = (ctypes.c_uint64 * q)()
        keep = []
        for i, c in enumerate(contents):
            b = ctypes.create_string_buffer(bytes(c), max(len(c), 1))
            keep.append(b)
            ptrs[i] = ctypes.cast(b, ctypes.c_void_p)
            lens[i] = len(c)
        pb = b"".join(b"".join(p) for p in paths)
        bb = bytes(x for bl in bits for x in bl)
        shared = len(roots) == 1
        rb = b"".join(roots)
        ok = ctypes.create_string_buffer(q)
        self._check(self._L.dm_verify_paths(self._h, ptrs, lens, q, pb, bb, depth, rb, 0 if shared else 32, ok),
                    "dm_verify_paths")
        return [bool(x) for x in ok.raw]

    def verify_paths_device_async(self, dev_contents: Sequence[int], lens: Sequence[int], q: int, dev_paths: int,
                                  dev_bits: int, depth: int, dev_roots: int, root_stride: int, dev_ok: int,
                                  stream: int = 0) -> None:
        ptrs = (ctypes.c_void_p * max(q, 1))(*dev_contents)
        ls = (ctypes.c_uint64 * max(q, 1))(*lens)
        self._check(self._L.dm_verify_paths_device_async(self._h, ptrs, ls, q, ctypes.c_void_p(dev_paths),
                                                         ctypes.c_void_p(dev_bits), depth, ctypes.c_void_p(dev_roots),
                                                         root_stride, ctypes.c_void_p(dev_ok),
                                                         ctypes.c_void_p(stream or None)),
                    "dm_verify_paths_device_async")

    def verify_object_device_async(self, dev_obj: int, length: int, chunk: int, dev_paths: int, dev_bits: int,
                                   depth: int, dev_roots: int, root_stride: int, dev_ok: int, stream: int = 0) -> None:
        """Every chunk of one object in HBM against its proof (uniform layout, no tables)."""
        self._check(self._L.dm_verify_object_device_async(self._h, ctypes.c_void_p(dev_obj), length, chunk,
                                                          ctypes.c_void_p(dev_paths), ctypes.c_void_p(dev_bits), depth,
                                                          ctypes.c_void_p(dev_roots), root_stride,
                                                          ctypes.c_void_p(dev_ok), ctypes.c_void_p(stream or None)),
                    "dm_verify_object_device_async")

    # -- streaming -------------------------------------------------------------------------------
    def open_stream(self, chunk: int) -> "MerkleStream":
        """Incremental root of one object written in pieces (hash while receiving)."""
        return MerkleStream(self, chunk)

    # -- tuning --------------------------------------------------------------------------------
    LEAF_KERNELS = {"auto": 0, "wide": 1, "latency": 2, "pair": 3, "quad": 4}

    def set_leaf_kernel(self, mode: str) -> None:
        """'auto' | 'wide' (one lane per leaf) | 'latency' (producer/consumer waves) |
        'pair' (producer/consumer with rounds packed on lane pairs) | 'quad' (rounds spread over
        eight lanes per leaf)."""
        self._check(self._L.dm_set_leaf_kernel(self._h, self.LEAF_KERNELS[mode]), "dm_set_leaf_kernel")

    def leaf_kernel_for(self, nleaves: int) -> str:
        """Leaf kernel ('wide' | 'latency' | 'pair' | 'quad') an object of nleaves uniform chunks runs with."""
        code = self._L.dm_leaf_kernel_for(self._h, nleaves)
        if code < 0:
            self._check(code, "dm_leaf_kernel_for")
        return {v: k for k, v in self.LEAF_KERNELS.items()}[code]

    # -- measurement ----------------------------------------------------------------------------
    def set_timing(self, enable: bool) -> None:
        self._check(self._L.dm_set_timing(self._h, int(enable)), "dm_set_timing")

    def timing_summary(self) -> Tuple[int, float, float, float]:
        """(timed calls, sum of K1 ms, sum of whole-call ms, max K1 ms) since set_timing(True)."""
        n = ctypes.c_uint64()
        a, b, m = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        self._check(self._L.dm_timing_summary(self._h, ctypes.byref(n), ctypes.byref(a), ctypes.byref(b),
                                              ctypes.byref(m)), "dm_timing_summary")
        return n.value, a.value, b.value, m.value

    def exchange_timing(self) -> Tuple[int, float, float, int]:
        """(sharded calls, sum of exchange us, max exchange us, G of the last one) since
        set_timing(True): the subtree-root all-gather (C1) of each sharded call."""
        n = ctypes.c_uint64()
        a, m = ctypes.c_double(), ctypes.c_double()
        g = ctypes.c_int()
        self._check(self._L.dm_exchange_timing(self._h, ctypes.byref(n), ctypes.byref(a), ctypes.byref(m),
                                               ctypes.byref(g)), "dm_exchange_timing")
        return n.value, a.value, m.value, g.value

    def last_call_devices(self) -> Tuple[List[int], List[int], int]:
        """Where this thread's last call on the context ran: (context device indices, HIP device
        ids, lane); ([], [], -1) before the first call."""
        cap = max(self.device_count, 1)
        devs, ids = (ctypes.c_int * cap)(), (ctypes.c_int * cap)()
        lane = ctypes.c_int()
        n = self._L.dm_last_call_devices(self._h, devs, ids, cap, ctypes.byref(lane))
        if n < 0:
            self._check(n, "dm_last_call_devices")
        n = min(n, cap)
        return list(devs[:n]), list(ids[:n]), lane.value


class MerkleStream:
    """dm_stream_*: write() pieces of any size, close() -> (leaf digests, root)."""

    def __init__(self, ctx: MerkleContext, chunk: int):
        self._ctx = ctx
        self._L = ctx._L
        h = ctypes.c_void_p()
        ctx._check(self._L.dm_stream_open(ctx._h, chunk, ctypes.byref(h)), "dm_stream_open")
        self._h = h
        self.chunk = chunk
        self.written = 0

    def _check(self, rc: int, what: str) -> None:
        if rc == 0:
            return
        if rc == DM_ERR_EMPTY:
            raise DeossMerkleError(rc, "Empty data")
        detail = (self._L.dm_stream_error(self._h) or b"").decode() if self._h else ""
        raise DeossMerkleError(rc, f"{what}: {self._L.dm_strerror(rc).decode()}: {detail}")

    def write(self, data) -> None:
        if isinstance(data, (bytes, bytearray)):
            buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
            self._check(self._L.dm_stream_write(self._h, buf, len(data)), "dm_stream_write")
            self.written += len(data)
        else:   # (address, length) of host memory
            addr, n = data
            self._check(self._L.dm_stream_write(self._h, ctypes.c_void_p(addr), n), "dm_stream_write")
            self.written += n

    def close(self, want_leaves: bool = False, leaf_cap: int = 0) -> Tuple[Optional[bytes], bytes]:
        cap = leaf_cap if leaf_cap else (-(-self.written // self.chunk) if want_leaves else 0)
        leaf = ctypes.create_string_buffer(max(32 * cap, 32)) if want_leaves else None
        n = ctypes.c_uint64()
        root = ctypes.create_string_buffer(32)
        h, self._h = self._h, None
        rc = self._L.dm_stream_close(h, leaf, cap if want_leaves else 0, ctypes.byref(n), root)
        if rc != 0:
            if rc == DM_ERR_EMPTY:
                raise DeossMerkleError(rc, "Empty data")
            detail = (self._L.dm_last_error(self._ctx._h) or b"").decode()
            raise DeossMerkleError(rc, f"dm_stream_close: {self._L.dm_strerror(rc).decode()}: {detail}")
        return (leaf.raw[:32 * min(n.value, cap)] if want_leaves else None), root.raw

    def abort(self) -> None:
        if self._h:
            self._L.dm_stream_abort(self._h)
            self._h = None

    def __del__(self):
        try:
            self.abort()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host memory from dm_host_alloc (visible to every GPU).  Objects held in it are
    hashed in place by the zero-copy host paths (dm_root_buffer / chunks / batch).  `array()` is a
    writable numpy view; free() (or garbage collection) releases it."""

    def __init__(self, nbytes: int):
        self._L = load_library()
        p = ctypes.c_void_p()
        rc = self._L.dm_host_alloc(nbytes, ctypes.byref(p))
        if rc != 0:
            raise DeossMerkleError(rc, (self._L.dm_last_error(None) or b"").decode() or "dm_host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self._fin = weakref.finalize(self, self._L.dm_host_free, ctypes.c_void_p(self.ptr))

    def array(self):
        import numpy as np
        return np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))

    def free(self) -> None:
        self._fin()
        self.ptr = None
