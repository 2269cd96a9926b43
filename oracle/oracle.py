"""CPU oracle for the DeOSS ``common/hashtree`` Merkle path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker (or the baseline being timed).  The product package
``deoss_amd`` never imports it.

Two restatements of the same algorithm live here:

* ``py_*``: pure Python over :mod:`hashlib` (OpenSSL FIPS 180-4 SHA-256, standing in for Go's
  ``crypto/sha256``).  Slow; used for small cases and to generate ``tests/golden`` fixtures.
* ``Oracle``: ctypes binding of ``oracle/merkle_oracle.c`` (scalar or SHA-NI SHA-256), fast
  enough for the full-size CPU baseline.

Reference semantics followed (paths relative to the reference repo):

* ``common/hashtree/hashtree.go:23-30`` -- leaf = SHA-256(chunk bytes).
* ``common/hashtree/types.go:19-39``    -- one leaf per chunk; empty list -> ``"Empty data"``.
* ``cbergoon/merkletree v0.2.0`` (``go.mod:10``; not vendored, restated) -- odd leaf count
  duplicates the last leaf; each level pairs (i, i+1) or (i, i) for a trailing odd node;
  node = SHA-256(left || right); stops at one node, after at least one level.

Reed-Solomon fragment coding (``py_rs_*`` and ``Oracle.rs_*`` over ``oracle/rs_oracle.c``):
``klauspost/reedsolomon v1.12.4`` (``go.mod:65``; not vendored, restated -- parity unpinned)
``New(4, 8)`` as the cess-go-sdk uses it for chain.DataShards / chain.ParShards
(``node/tracker.go:250,369``): GF(2^8) mod x^8+x^4+x^3+x^2+1, Vandermonde matrix times the
inverse of its top square, parity = matrix rows x data shards.  The Python restatement below
multiplies bitwise (no log tables) so the two restatements share no tables.

FullProcessing (``py_full_processing`` and ``Oracle.full_processing`` over
``oracle/process_oracle.c``): cess-go-sdk ``process.FullProcessing(file, "", savedir)``
(``go.mod:8``; not vendored, restated -- composition parity unpinned, see process_oracle.c):
32 MiB zero-padded segments, RS 4+8 fragments per segment, every segment / fragment named by
its SHA-256, fid = the hashtree root over the segments.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from typing import List, Optional, Sequence, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_merkle.so")


def py_sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def py_level(nodes: Sequence[bytes]) -> List[bytes]:
    """One merkletree v0.2.0 ``buildIntermediate`` level (right = i when i+1 == len)."""
    n = len(nodes)
    return [py_sha256(nodes[2 * j] + nodes[min(2 * j + 1, n - 1)]) for j in range((n + 1) // 2)]


def py_reduce(digests: Sequence[bytes], levels: int = -1) -> List[bytes]:
    """Reduce for exactly ``levels`` levels, or (levels=-1) to one node with at least one level."""
    cur = list(digests)
    done = 0
    while True:
        if levels >= 0 and done >= levels:
            break
        if levels < 0 and done >= 1 and len(cur) == 1:
            break
        cur = py_level(cur)
        done += 1
    return cur


def py_go_tree(chunks: Sequence[bytes]) -> Tuple[List[bytes], bytes]:
    """Literal restatement of merkletree v0.2.0 NewTree: returns (Leafs hashes incl. dup, root).

    buildWithContent appends a duplicate of the last leaf when the count is odd; buildIntermediate
    recurses until a level has exactly two nodes and returns their parent.
    """
    if len(chunks) == 0:
        raise ValueError("Empty data")
    leafs = [py_sha256(c) for c in chunks]
    if len(leafs) % 2 == 1:
        leafs.append(leafs[-1])
    nl = list(leafs)
    while True:
        nodes = []
        for i in range(0, len(nl), 2):
            left, right = i, i + 1
            if i + 1 == len(nl):
                right = i
            h = py_sha256(nl[left] + nl[right])
            nodes.append(h)
            if len(nl) == 2:
                return leafs, h
        nl = nodes


class _GoNode:
    """merkletree v0.2.0 Node: Parent / Left / Right / Hash / leaf / dup / C."""
    __slots__ = ("Parent", "Left", "Right", "Hash", "leaf", "dup", "C")

    def __init__(self, Hash, leaf=False, dup=False, C=None, Left=None, Right=None):
        self.Parent, self.Left, self.Right = None, Left, Right
        self.Hash, self.leaf, self.dup, self.C = Hash, leaf, dup, C


def py_go_tree_nodes(chunks: Sequence[bytes]) -> Tuple[List["_GoNode"], "_GoNode"]:
    """Literal merkletree v0.2.0 NewTree with Node objects and Parent pointers
    (buildWithContent + buildIntermediate), for GetMerklePath / VerifyContent restatements."""
    if len(chunks) == 0:
        raise ValueError("Empty data")
    leafs = [_GoNode(py_sha256(c), leaf=True, C=bytes(c)) for c in chunks]
    if len(leafs) % 2 == 1:
        last = leafs[-1]
        leafs.append(_GoNode(last.Hash, leaf=True, dup=True, C=last.C))
    nl = list(leafs)
    while True:
        nodes = []
        for i in range(0, len(nl), 2):
            left, right = i, i + 1
            if i + 1 == len(nl):
                right = i
            n = _GoNode(py_sha256(nl[left].Hash + nl[right].Hash), Left=nl[left], Right=nl[right])
            nodes.append(n)
            nl[left].Parent = n
            nl[right].Parent = n
            if len(nl) == 2:
                return leafs, n
        nl = nodes


def py_get_merkle_path(chunks: Sequence[bytes], content: bytes) -> Tuple[Optional[List[bytes]], Optional[List[int]]]:
    """merkletree v0.2.0 GetMerklePath(content): first leaf whose content Equals (HashTreeContent
    compares strings, hashtree.go:33-35), then up the Parent chain; index 1 when
    bytes.Equal(parent.Left.Hash, current.Hash) (sibling = Right), else 0 (sibling = Left)."""
    leafs, _ = py_go_tree_nodes(chunks)
    for cur in leafs:
        if cur.C == bytes(content):
            path, index = [], []
            parent = cur.Parent
            while parent is not None:
                if parent.Left.Hash == cur.Hash:
                    path.append(parent.Right.Hash)
                    index.append(1)
                else:
                    path.append(parent.Left.Hash)
                    index.append(0)
                cur, parent = parent, parent.Parent
            return path, index
    return None, None


def py_fold_path(leaf_digest: bytes, path: Sequence[bytes], index: Sequence[int]) -> bytes:
    """Root implied by a GetMerklePath proof: H(h || sib) for index 1, H(sib || h) for index 0."""
    h = leaf_digest
    for sib, b in zip(path, index):
        h = py_sha256(h + sib) if b == 1 else py_sha256(sib + h)
    return h


def py_root_chunks(chunks: Sequence[bytes]) -> Tuple[List[bytes], bytes]:
    if len(chunks) == 0:
        raise ValueError("Empty data")
    leaves = [py_sha256(c) for c in chunks]
    return leaves, py_reduce(leaves)[0]


def split_chunks(buf: bytes, chunk: int) -> List[bytes]:
    return [buf[i:i + chunk] for i in range(0, len(buf), chunk)]


def splitmix64_bytes(nbytes: int, seed: int, off: int = 0) -> bytes:
    """Synthetic object bytes (numpy): word[i] = splitmix64(seed ^ i), little-endian."""
    import numpy as np
    assert off % 8 == 0
    nw = (nbytes + 7) // 8
    i = np.arange(off // 8, off // 8 + nw, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) ^ i) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:nbytes]


def py_gf_mul(a: int, b: int) -> int:
    """GF(2^8) product, polynomial 0x11d, shift-and-add (klauspost galois.go restated)."""
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
        b >>= 1
    return r


def py_gf_pow(a: int, n: int) -> int:
    r = 1
    for _ in range(n):
        r = py_gf_mul(r, a)
    return r


def py_gf_inverse(m: List[List[int]]) -> List[List[int]]:
    k = len(m)
    w = [list(row) + [int(i == j) for j in range(k)] for i, row in enumerate(m)]
    for c in range(k):
        p = next(r for r in range(c, k) if w[r][c])
        w[c], w[p] = w[p], w[c]
        inv = next(x for x in range(1, 256) if py_gf_mul(w[c][c], x) == 1)
        w[c] = [py_gf_mul(v, inv) for v in w[c]]
        for r in range(k):
            if r != c and w[r][c]:
                f = w[r][c]
                w[r] = [v ^ py_gf_mul(f, u) for v, u in zip(w[r], w[c])]
    return [row[k:] for row in w]


def py_rs_matrix(data: int, total: int) -> List[List[int]]:
    """klauspost buildMatrix: vandermonde(total, data) x inverse(top data x data square)."""
    vm = [[py_gf_pow(r, c) for c in range(data)] for r in range(total)]
    inv = py_gf_inverse(vm[:data])
    out = []
    for r in range(total):
        row = []
        for c in range(data):
            acc = 0
            for t in range(data):
                acc ^= py_gf_mul(vm[r][t], inv[t][c])
            row.append(acc)
        out.append(row)
    return out


def _mul_table():
    import numpy as np
    t = np.zeros((256, 256), dtype=np.uint8)
    for a in range(256):
        for b in range(256):
            t[a, b] = py_gf_mul(a, b)
    return t


_MUL = None


def py_rs_code(rows: List[List[int]], inputs: Sequence[bytes]) -> List[bytes]:
    """out[i] = sum_j rows[i][j] * inputs[j] over GF(2^8), bytewise (numpy)."""
    import numpy as np
    global _MUL
    if _MUL is None:
        _MUL = _mul_table()
    ins = [np.frombuffer(bytes(x), dtype=np.uint8) for x in inputs]
    outs = []
    for row in rows:
        acc = np.zeros(len(ins[0]), dtype=np.uint8)
        for c, x in zip(row, ins):
            acc ^= _MUL[c][x]
        outs.append(acc.tobytes())
    return outs


def py_rs_split(buf: bytes, data: int) -> List[bytes]:
    """klauspost Split: perShard = ceil(len / data), the tail zero-padded."""
    per = (len(buf) + data - 1) // data
    b = bytes(buf) + bytes(per * data - len(buf))
    return [b[i * per:(i + 1) * per] for i in range(data)]


def py_rs_encode(data_shards: Sequence[bytes], parity: int) -> List[bytes]:
    k = len(data_shards)
    m = py_rs_matrix(k, k + parity)
    return py_rs_code(m[k:], data_shards)


def py_full_processing(buf: bytes, segment: int, data: int = 4, parity: int = 8
                       ) -> Tuple[List[bytes], List[List[bytes]], bytes, List[List[bytes]]]:
    """FullProcessing restated over hashlib + the bitwise RS restatement.

    Returns (segment digests, per-segment fragment digests (data first), fid, fragments)."""
    if len(buf) == 0:
        raise ValueError("empty file")
    nseg = (len(buf) + segment - 1) // segment
    padded = bytes(buf) + bytes(nseg * segment - len(buf))
    segs, frag_h, frags = [], [], []
    for s in range(nseg):
        seg = padded[s * segment:(s + 1) * segment]
        segs.append(py_sha256(seg))
        dshards = py_rs_split(seg, data)
        shards = list(dshards) + py_rs_encode(dshards, parity)
        frags.append(shards)
        frag_h.append([py_sha256(x) for x in shards])
    fid = py_reduce(segs)[0]   # NewHashTree(segment paths).MerkleRoot()
    return segs, frag_h, fid, frags


class Oracle:
    """ctypes binding of oracle/merkle_oracle.c and oracle/rs_oracle.c."""

    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(path)
        u64, vp, cp = ctypes.c_uint64, ctypes.c_void_p, ctypes.c_char_p
        L.or_sha256.argtypes = [vp, u64, vp]
        L.or_reduce.argtypes = [vp, u64, ctypes.c_int, vp]
        L.or_reduce.restype = u64
        L.or_root_chunks.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(u64), u64, vp, vp, ctypes.c_int]
        L.or_root_buffer.argtypes = [vp, u64, u64, vp, vp, ctypes.c_int]
        L.or_fill_splitmix.argtypes = [vp, u64, u64, u64]
        L.or_root_synthetic.argtypes = [u64, u64, u64, vp, vp, ctypes.c_int]
        L.or_root_synthetic_at.argtypes = [u64, u64, u64, u64, vp, vp, ctypes.c_int]
        L.or_set_backend.argtypes = [ctypes.c_int]
        L.or_rs_matrix.argtypes = [ctypes.c_int, ctypes.c_int, vp]
        L.or_rs_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                   ctypes.c_size_t, ctypes.c_int]
        L.or_rs_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), vp, ctypes.c_size_t,
                                        ctypes.c_int]
        L.or_full_processing.argtypes = [vp, u64, u64, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, ctypes.c_int]
        L.or_full_processing.restype = ctypes.c_int64
        self.L = L

    def backend(self) -> str:
        return {1: "scalar", 2: "sha-ni"}[self.L.or_backend()]

    def set_backend(self, name: str) -> None:
        self.L.or_set_backend({"auto": 0, "scalar": 1, "sha-ni": 0}[name])

    def sha256(self, b: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.or_sha256(b, len(b), out)
        return out.raw

    def reduce(self, digests: bytes, levels: int = -1) -> bytes:
        n = len(digests) // 32
        out = ctypes.create_string_buffer(max(32 * n, 32))
        m = self.L.or_reduce(digests, n, levels, out)
        return out.raw[:32 * m]

    def root_chunks(self, chunks: Sequence[bytes], nthreads: int = 1) -> Tuple[bytes, bytes]:
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
        rc = self.L.or_root_chunks(ptrs, lens, n, leaf, root, nthreads)
        if rc == -1:
            raise ValueError("Empty data")
        return leaf.raw[:32 * n], root.raw

    def root_buffer_ptr(self, addr: int, length: int, chunk: int, nthreads: int = 1,
                        want_leaves: bool = False) -> Tuple[Optional[bytes], bytes]:
        n = (length + chunk - 1) // chunk if length else 0
        leaf = ctypes.create_string_buffer(max(32 * n, 32)) if want_leaves else None
        root = ctypes.create_string_buffer(32)
        rc = self.L.or_root_buffer(ctypes.c_void_p(addr), length, chunk, leaf, root, nthreads)
        if rc == -1:
            raise ValueError("Empty data")
        if rc != 0:
            raise ValueError(f"or_root_buffer rc={rc}")
        return (leaf.raw[:32 * n] if leaf is not None else None), root.raw

    def root_buffer(self, buf: bytes, chunk: int, nthreads: int = 1) -> Tuple[bytes, bytes]:
        b = ctypes.create_string_buffer(bytes(buf), max(len(buf), 1))
        leaves, root = self.root_buffer_ptr(ctypes.addressof(b), len(buf), chunk, nthreads, True)
        return leaves, root

    def root_synthetic(self, length: int, chunk: int, seed: int, nthreads: int = 1,
                       want_leaves: bool = False, base: int = 0) -> Tuple[Optional[bytes], bytes]:
        """Root of bytes [base, base + length) of the splitmix64 stream `seed`, regenerated leaf by
        leaf (no whole-object buffer: the 1 TiB configs[3] check; base > 0: one GPU's share)."""
        n = (length + chunk - 1) // chunk if length else 0
        leaf = ctypes.create_string_buffer(max(32 * n, 32)) if want_leaves else None
        root = ctypes.create_string_buffer(32)
        rc = self.L.or_root_synthetic_at(base, length, chunk, seed, leaf, root, nthreads)
        if rc == -1:
            raise ValueError("Empty data")
        if rc != 0:
            raise ValueError(f"or_root_synthetic rc={rc} (chunk must be a multiple of 64, length of 8)")
        return (leaf.raw[:32 * n] if leaf is not None else None), root.raw

    def fill_splitmix_ptr(self, addr: int, off: int, nbytes: int, seed: int) -> None:
        assert off % 8 == 0 and nbytes % 8 == 0
        self.L.or_fill_splitmix(ctypes.c_void_p(addr), off, nbytes, seed)

    def splitmix_bytes(self, nbytes: int, seed: int, off: int = 0) -> bytes:
        n8 = (nbytes + 7) // 8 * 8
        b = ctypes.create_string_buffer(max(n8, 8))
        self.fill_splitmix_ptr(ctypes.addressof(b), off, n8, seed)
        return b.raw[:nbytes]

    # -- Reed-Solomon (oracle/rs_oracle.c) ----------------------------------------------------
    def rs_matrix(self, data: int, total: int) -> List[List[int]]:
        out = ctypes.create_string_buffer(total * data)
        if self.L.or_rs_matrix(data, total, out) != 0:
            raise ValueError("invalid shard counts")
        return [list(out.raw[r * data:(r + 1) * data]) for r in range(total)]

    def rs_encode_ptrs(self, data: int, parity: int, dptrs: Sequence[int], pptrs: Sequence[int], shard: int,
                       nthreads: int = 1) -> None:
        d = (ctypes.c_void_p * data)(*dptrs)
        p = (ctypes.c_void_p * parity)(*pptrs)
        if self.L.or_rs_encode(data, parity, d, p, shard, nthreads) != 0:
            raise ValueError("or_rs_encode failed")

    def rs_encode(self, data_shards: Sequence[bytes], parity: int, nthreads: int = 1) -> List[bytes]:
        k, n = len(data_shards), len(data_shards[0])
        ins = [ctypes.create_string_buffer(bytes(x), max(n, 1)) for x in data_shards]
        outs = [ctypes.create_string_buffer(max(n, 1)) for _ in range(parity)]
        self.rs_encode_ptrs(k, parity, [ctypes.addressof(b) for b in ins], [ctypes.addressof(b) for b in outs],
                            n, nthreads)
        return [b.raw[:n] for b in outs]

    def rs_reconstruct(self, data: int, parity: int, shards: Sequence[Optional[bytes]], shard: int) -> List[bytes]:
        """Rebuild the shards given as None (klauspost Reconstruct semantics)."""
        total = data + parity
        bufs = [ctypes.create_string_buffer(bytes(x) if x is not None else bytes(shard), max(shard, 1))
                for x in shards]
        present = bytes(int(x is not None) for x in shards)
        ptrs = (ctypes.c_void_p * total)(*[ctypes.addressof(b) for b in bufs])
        rc = self.L.or_rs_reconstruct(data, parity, ptrs, present, shard, 1)
        if rc == -2:
            raise ValueError("too few shards")
        if rc != 0:
            raise ValueError("or_rs_reconstruct failed")
        return [b.raw[:shard] for b in bufs]

    # -- FullProcessing (oracle/process_oracle.c) ----------------------------------------------
    def full_processing_ptr(self, addr: int, length: int, segment: int, data: int = 4, parity: int = 8,
                            want_frags: bool = False, nthreads: int = 1):
        """Returns (segment digests bytes, fragment digests bytes, fid, fragments bytes or None)."""
        nseg = (length + segment - 1) // segment if length else 0
        total = data + parity
        seg = ctypes.create_string_buffer(max(32 * nseg, 32))
        frag = ctypes.create_string_buffer(max(32 * nseg * total, 32))
        fid = ctypes.create_string_buffer(32)
        fr = ctypes.create_string_buffer(nseg * total * (segment // data)) if want_frags else None
        rc = self.L.or_full_processing(ctypes.c_void_p(addr), length, segment, data, parity, seg, frag, fid, fr,
                                       nthreads)
        if rc == -1:
            raise ValueError("empty file")
        if rc < 0:
            raise ValueError(f"or_full_processing rc={rc}")
        return seg.raw[:32 * nseg], frag.raw[:32 * nseg * total], fid.raw, (fr.raw if fr is not None else None)

    def full_processing(self, buf: bytes, segment: int, data: int = 4, parity: int = 8, want_frags: bool = False,
                        nthreads: int = 1):
        b = ctypes.create_string_buffer(bytes(buf), max(len(buf), 1))
        return self.full_processing_ptr(ctypes.addressof(b), len(buf), segment, data, parity, want_frags, nthreads)
