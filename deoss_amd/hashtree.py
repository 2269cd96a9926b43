"""Host-side mirror of DeOSS ``common/hashtree`` backed by the MI355X HIP path.

Mirrors the reference Go API (same names, argument meaning and error behaviour):

* ``NewHashTree(chunkPath)`` -- ``common/hashtree/types.go:19-39``: one leaf per file, each read
  whole; an empty list fails with ``"Empty data"``; open/read errors are returned as errors.
  Returns ``(tree, err)`` like the Go function.
* ``HashTreeContent`` -- ``common/hashtree/hashtree.go:18-35`` (``CalculateHash``, ``Equals``).
* ``MerkleTree`` / ``Node`` -- the parts of ``cbergoon/merkletree`` v0.2.0 the reference test reads:
  ``Leafs`` (n entries, n+1 when n is odd: the last leaf duplicated with ``dup=True``),
  ``MerkleRoot()`` and ``Root``; plus the proof API ``GetMerklePath(content)``,
  ``VerifyContent(content)`` and ``VerifyTree()``, whose levels, paths and
  proof folds run on the GPU (``dm_tree_levels``, ``dm_merkle_paths``, ``dm_verify_paths``).

Deviation (documented in DESIGN.md): interior nodes are not ``Node`` objects (the root comes from
the fused leaf kernel; the levels are built on the GPU the first time a proof asks for them);
``Root.Left``/``Right`` are ``None``.  ``Leafs[i].C.Equals`` compares chunk bytes when the
content was kept (``keep_content=True``) and digests otherwise.

Additive entry points: ``NewHashTreeFromBuffer(buf, chunkSize)`` (the upload-handler host
buffer path) and ``NewHashTreesBatch(objects, chunkSize)``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from ._lib import DeossMerkleError
from .merkle import MerkleContext

_default_ctx: Optional[MerkleContext] = None
_selected: Optional[List[int]] = None


def Init(devs: Sequence[int]) -> Optional[Exception]:
    """The Go package's Init(devs): the GPUs the default context spans (before first use)."""
    global _selected
    if _default_ctx is not None:
        return DeossMerkleError(-2, "hashtree: Init after first use")
    if not devs:
        return DeossMerkleError(-2, "hashtree: Init needs at least one device")
    _selected = list(devs)
    return None


def _device_list() -> List[int]:
    """Init(devs), else DEOSS_GPUS ("0,1,2,3" or "all"), else every visible GPU."""
    import os
    from ._lib import load_library
    if _selected:
        return _selected
    spec = os.environ.get("DEOSS_GPUS", "").strip()
    if spec and spec != "all":
        return [int(x) for x in spec.split(",") if x.strip()]
    return list(range(load_library().dm_gpu_count())) or [0]


def default_context() -> MerkleContext:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = MerkleContext(devices=_device_list())
    return _default_ctx


# NewHashTreeFromBuffer objects up to BATCH_LIMIT bytes go through a process-wide coalescing
# dm_batcher per chunk size, as the Go package does (go/hashtree/types_hip.go): concurrent callers
# share GPU passes instead of queueing one chain-latency pass each.  Larger
# objects take dm_root_buffer on the default context (ramped striped H2D, zero-copy when pinned, on
# its least-loaded GPU).  Only the first MAX_BATCHERS chunk sizes get a batcher (each holds worker
# contexts on every GPU); other sizes take dm_root_buffer too -- the bound of go/hashtree.
BATCH_LIMIT = 256 << 20
MAX_BATCHERS = 4
_batchers: dict = {}
_batch_lock = None


def _batcher(chunk: int):
    global _batch_lock
    import threading
    if _batch_lock is None:
        _batch_lock = threading.Lock()
    with _batch_lock:
        b = _batchers.get(chunk)
        if b is None and len(_batchers) >= MAX_BATCHERS:
            return None
        if b is None:
            import atexit
            from .batcher import ROOT, Batcher
            default_context()   # fixes the device list (Init after this point is refused)
            b = Batcher(ROOT, chunk, device=_device_list(), linger_us=2000)
            _batchers[chunk] = b
            if len(_batchers) == 1:
                atexit.register(_close_batchers)
        return b


def _close_batchers() -> None:
    for b in list(_batchers.values()):
        b.close()
    _batchers.clear()


class HashTreeContent:
    """Leaf payload (hashtree.go:18-20).  ``x`` holds the chunk bytes (or None if dropped)."""

    def __init__(self, x: Optional[bytes], digest: Optional[bytes] = None):
        self.x = x
        self._digest = digest

    def CalculateHash(self) -> Tuple[Optional[bytes], Optional[Exception]]:
        """SHA-256 of the chunk (hashtree.go:23-30), computed on the GPU."""
        if self._digest is not None:
            return self._digest, None
        try:
            leaves, _ = default_context().root_chunks([self.x or b""])
        except DeossMerkleError as e:
            return None, e
        self._digest = leaves[:32]
        return self._digest, None

    def Equals(self, other: "HashTreeContent") -> Tuple[bool, Optional[Exception]]:
        """hashtree.go:33-35 compares the contents; without kept bytes, compare digests."""
        if self.x is not None and other.x is not None:
            return self.x == other.x, None
        a, e1 = self.CalculateHash()
        b, e2 = other.CalculateHash()
        return a == b, e1 or e2


@dataclass
class Node:
    Hash: bytes
    C: Optional[HashTreeContent] = None
    leaf: bool = False
    dup: bool = False
    Left: Optional["Node"] = None
    Right: Optional["Node"] = None


@dataclass
class MerkleTree:
    Root: Node
    Leafs: List[Node] = field(default_factory=list)
    ctx: Optional[MerkleContext] = None

    def MerkleRoot(self) -> bytes:
        return self.Root.Hash

    def _ctx(self) -> MerkleContext:
        return self.ctx or default_context()

    def _digests(self) -> bytes:
        return b"".join(l.Hash for l in self.Leafs if not l.dup)

    def _find(self, content: HashTreeContent) -> Tuple[int, Optional[Exception]]:
        """Index of the first leaf whose content Equals `content` (-1: none), as merkletree scans."""
        for i, l in enumerate(self.Leafs):
            ok, err = l.C.Equals(content)
            if err is not None:
                return -1, err
            if ok:
                return i, None
        return -1, None

    def GetMerklePath(self, content: HashTreeContent
                      ) -> Tuple[Optional[List[bytes]], Optional[List[int]], Optional[Exception]]:
        """merkletree GetMerklePath: sibling digests leaf -> root and their indices (1 = the
        sibling is the right child); (None, None, None) when no leaf holds `content`."""
        i, err = self._find(content)
        if err is not None or i < 0:
            return None, None, err
        try:
            (path, bits), = self._ctx().merkle_paths(self._digests(), [i])
        except DeossMerkleError as e:
            return None, None, e
        return path, bits, None

    def VerifyContent(self, content: HashTreeContent) -> Tuple[bool, Optional[Exception]]:
        """merkletree VerifyContent: `content` is a leaf and its branch hashes up to the root."""
        i, err = self._find(content)
        if err is not None or i < 0:
            return False, err
        try:
            c = self._ctx()
            (path, bits), = c.merkle_paths(self._digests(), [i])
            data = content.x if content.x is not None else None
            if data is None:   # digest-only content: fold the stored digest instead of re-hashing
                return self._fold(content.CalculateHash()[0], path, bits) == self.Root.Hash, None
            return c.verify_paths([data], [path], [bits], [self.Root.Hash])[0], None
        except DeossMerkleError as e:
            return False, e

    def _fold(self, h: bytes, path: List[bytes], bits: List[int]) -> bytes:
        # digest-only proof fold: the tree over [h, sibling] pairs, one GPU level per step
        c = self._ctx()
        for sib, b in zip(path, bits):
            h = c.tree_root(h + sib if b == 1 else sib + h)
        return h

    def VerifyTree(self) -> Tuple[bool, Optional[Exception]]:
        """merkletree VerifyTree: every leaf re-hashed from its content, the root recomputed."""
        try:
            c = self._ctx()
            real = [l for l in self.Leafs if not l.dup]
            if all(l.C is not None and l.C.x is not None for l in real):
                _, root = c.root_chunks([l.C.x for l in real])
            else:
                root = c.tree_root(b"".join(l.C.CalculateHash()[0] for l in real))
            return root == self.Root.Hash, None
        except DeossMerkleError as e:
            return False, e


def _build(leaf_digests: bytes, root: bytes, contents: Sequence[Optional[bytes]],
           ctx: Optional[MerkleContext] = None) -> MerkleTree:
    n = len(leaf_digests) // 32
    leafs = [Node(Hash=leaf_digests[32 * i:32 * i + 32], C=HashTreeContent(contents[i], leaf_digests[32 * i:32 * i + 32]),
                  leaf=True) for i in range(n)]
    if n % 2 == 1:   # merkletree v0.2.0 buildWithContent: duplicate the last leaf
        last = leafs[-1]
        leafs.append(Node(Hash=last.Hash, C=last.C, leaf=True, dup=True))
    return MerkleTree(Root=Node(Hash=root), Leafs=leafs, ctx=ctx)


def NewHashTree(chunkPath: Sequence[str], ctx: Optional[MerkleContext] = None,
                keep_content: bool = False) -> Tuple[Optional[MerkleTree], Optional[Exception]]:
    """types.go:19-39 -- build the tree over whole files, one leaf per file."""
    if len(chunkPath) == 0:
        return None, DeossMerkleError(-1, "Empty data")
    c = ctx or default_context()
    try:
        leaves, root = c.new_hash_tree(list(chunkPath))
    except DeossMerkleError as e:
        return None, e
    contents: List[Optional[bytes]] = [None] * len(chunkPath)
    if keep_content:
        for i, p in enumerate(chunkPath):
            with open(p, "rb") as f:
                contents[i] = f.read()
    return _build(b"".join(leaves), root, contents, c), None


def NewHashTreeFromBuffer(buf: bytes, chunkSize: int, ctx: Optional[MerkleContext] = None
                          ) -> Tuple[Optional[MerkleTree], Optional[Exception]]:
    """Additive: the object buffer split into chunkSize chunks (last one short)."""
    if chunkSize <= 0:
        return None, DeossMerkleError(-2, f"hashtree: chunk size {chunkSize} must be positive")
    if len(buf) == 0:
        return None, DeossMerkleError(-1, "Empty data")
    c = ctx or default_context()
    try:
        b = _batcher(chunkSize) if ctx is None and len(buf) <= BATCH_LIMIT else None
        if b is not None:
            leaves, root = b.root(buf, want_leaves=True)
        else:
            leaves, root = c.root_buffer(buf, chunkSize, want_leaves=True)
    except DeossMerkleError as e:
        return None, e
    n = len(leaves) // 32
    return _build(leaves, root, [None] * n, c), None


def NewHashTreesBatch(objects: Sequence[bytes], chunkSize: int, ctx: Optional[MerkleContext] = None
                      ) -> Tuple[Optional[List[bytes]], Optional[Exception]]:
    """Additive: many independent objects, one root each."""
    c = ctx or default_context()
    try:
        return c.root_batch(list(objects), chunkSize), None
    except DeossMerkleError as e:
        return None, e


class Stream:
    """The Go package's hash-while-receiving Stream (go/hashtree/stream_hip.go) over dm_stream:
    ``Write(piece)`` any number of times, ``Close()`` -> ``(tree, err)`` equal to
    NewHashTreeFromBuffer over the concatenated bytes, ``Abort()``."""

    def __init__(self, st, chunk: int):
        self._st, self._chunk, self._received, self._err = st, chunk, 0, None

    def Write(self, p: bytes) -> Tuple[int, Optional[Exception]]:
        if self._st is None:
            return 0, DeossMerkleError(-2, "hashtree: write on a closed stream")
        if self._err is not None:
            return 0, self._err
        try:
            self._st.write(p)
        except DeossMerkleError as e:
            self._err = e
            return 0, e
        self._received += len(p)
        return len(p), None

    def Close(self) -> Tuple[Optional["MerkleTree"], Optional[Exception]]:
        if self._st is None:
            return None, DeossMerkleError(-2, "hashtree: stream already closed")
        st, self._st = self._st, None
        if self._err is not None:
            st.abort()
            return None, self._err
        n = -(-self._received // self._chunk)
        try:
            leaves, root = st.close(want_leaves=True, leaf_cap=n)
        except DeossMerkleError as e:
            return None, e
        return _build(leaves, root, [None] * n, st._ctx), None

    def Abort(self) -> None:
        if self._st is not None:
            self._st.abort()
            self._st = None


def NewStream(chunkSize: int, ctx: Optional[MerkleContext] = None) -> Tuple[Optional[Stream], Optional[Exception]]:
    """NewStream(chunkSize): chunkSize a positive multiple of 16 (DeOSS: chain.SegmentSize)."""
    if chunkSize <= 0 or chunkSize % 16:
        return None, DeossMerkleError(-2, f"hashtree: stream chunk size {chunkSize} must be a positive multiple of 16")
    c = ctx or default_context()
    try:
        return Stream(c.open_stream(chunkSize), chunkSize), None
    except DeossMerkleError as e:
        return None, e
