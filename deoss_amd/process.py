"""Python mirror of cess-go-sdk ``process.FullProcessing`` backed by the GPU pipeline (``dm_process_*``).

DeOSS computes every file id ("fid") and fragment name with
``process.FullProcessing(file, cipher, savedir) ([]chain.SegmentDataInfo, fid string, error)``
from cess-go-sdk (``go.mod:8``; not vendored): ``node/objectHandler.go:168``,
``node/fileHandler.go:771``, ``node/filesHandler.go:201``, ``node/resumeHandler.go:326``,
``node/tracker.go:767-769`` and the fragment download path ``node/fileHandler.go:964,997``.
:func:`FullProcessing` keeps that signature and result shape:

* the file is cut into ``SEGMENT_SIZE`` (chain.SegmentSize, 32 MiB) segments, the last one
  zero-padded;
* each segment becomes ``DATA_SHARDS + PAR_SHARDS`` fragments of ``FRAGMENT_SIZE`` (8 MiB) with
  the klauspost Reed-Solomon coder, written to ``savedir/<hex SHA-256 of the fragment>``;
* ``SegmentDataInfo.SegmentHash`` is ``savedir/<hex SHA-256 of the segment>`` and
  ``SegmentDataInfo.FragmentHash`` the fragment paths, data fragments first (the handlers open
  them by path and match ``filepath.Base`` against a requested hash, ``node/fileHandler.go:967-969``);
* the fid is the hex ``common/hashtree`` root over the segments.

Coding, hashing and the tree run on the GPU; there is no CPU fallback.  Segment files are written
too (the zero-padded segment = its data fragments in order), so every returned path exists.
:meth:`Processor.FullProcessing` is one ``dm_full_processing`` call: the library reads the file,
and fragment writes overlap the reads and the GPU's hashing.
Deviation: a non-empty ``cipher`` is rejected (the AES branch is not implemented).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

from ._lib import DM_ERR_EMPTY, DM_ERR_INVALID, DM_ERR_IO, DeossMerkleError
from .merkle import MerkleContext
from .reedsolomon import DATA_SHARDS, PAR_SHARDS, Encoder

SEGMENT_SIZE = 32 << 20                       # chain.SegmentSize
FRAGMENT_SIZE = SEGMENT_SIZE // DATA_SHARDS   # chain.FragmentSize (8 MiB; node/tracker.go:250 "96M")
WINDOW_SEGMENTS = 8                           # segments per GPU call (256 MiB of file + 768 MiB of fragments; the Go shim bounds the segments in flight by DEOSS_PROCESS_MEM_GIB)


def _write_segments() -> bool:
    """Segment files are written unless DEOSS_SKIP_SEGMENT_FILES=1 (as in the Go shim: DeOSS itself
    only opens fragment paths, node/fileHandler.go:967-969)."""
    return os.environ.get("DEOSS_SKIP_SEGMENT_FILES") != "1"


@dataclass
class SegmentDataInfo:
    """chain.SegmentDataInfo: the segment's path name and its fragments' path names."""
    SegmentHash: str = ""
    FragmentHash: List[str] = field(default_factory=list)


class Processor:
    """One GPU pipeline (``dm_rs`` coder + context) for FullProcessing calls."""

    def __init__(self, ctx: Optional[MerkleContext] = None, data_shards: int = DATA_SHARDS,
                 parity_shards: int = PAR_SHARDS, segment: int = SEGMENT_SIZE):
        self.ctx = ctx or MerkleContext()
        self.enc = Encoder(self.ctx, data_shards, parity_shards)
        self.segment = segment
        self.k, self.m = data_shards, parity_shards
        self.frag = segment // data_shards

    def close(self) -> None:
        self.enc.close()

    def _check(self, rc: int, what: str) -> None:
        if rc == DM_ERR_EMPTY:
            raise DeossMerkleError(rc, "Empty data")
        self.enc._check(rc, what)

    # -- raw pipeline ----------------------------------------------------------------------------
    def process_buffer(self, buf, want_frags: bool = True) -> Tuple[bytes, bytes, bytes, Optional[bytes]]:
        """One ``dm_process_buffer`` call: (segment digests, fragment digests, fid, fragments)."""
        n = len(buf)
        nseg = (n + self.segment - 1) // self.segment if n else 0
        total = self.k + self.m
        seg = ctypes.create_string_buffer(max(32 * nseg, 32))
        frag = ctypes.create_string_buffer(max(32 * nseg * total, 32))
        fid = ctypes.create_string_buffer(32)
        frags = ctypes.create_string_buffer(nseg * total * self.frag) if (want_frags and nseg) else None
        src = buf if isinstance(buf, ctypes.Array) else ctypes.create_string_buffer(bytes(buf), max(n, 1))
        L = self.ctx._L
        self._check(L.dm_process_buffer(self.enc._h, src, n, self.segment, frags, seg, frag, fid),
                    "dm_process_buffer")
        return seg.raw[:32 * nseg], frag.raw[:32 * nseg * total], fid.raw, (frags.raw if frags is not None else None)

    def process_batch(self, bufs, want_frags: bool = False):
        """``dm_process_batch``: many objects in one pass; list of (seg digests, frag digests, fid,
        fragments or None) per object."""
        n = len(bufs)
        if n == 0:
            return []
        total = self.k + self.m
        srcs, segs, frs, fragss = [], [], [], []
        ptrs = (ctypes.c_void_p * n)()
        lens = (ctypes.c_uint64 * n)()
        sp = (ctypes.c_void_p * n)()
        fp = (ctypes.c_void_p * n)()
        gp = (ctypes.c_void_p * n)()
        for i, b in enumerate(bufs):
            nseg = (len(b) + self.segment - 1) // self.segment
            src = ctypes.create_string_buffer(bytes(b), max(len(b), 1))
            srcs.append(src)
            ptrs[i] = ctypes.addressof(src)
            lens[i] = len(b)
            segs.append(ctypes.create_string_buffer(max(32 * nseg, 32)))
            frs.append(ctypes.create_string_buffer(max(32 * nseg * total, 32)))
            sp[i] = ctypes.addressof(segs[-1])
            fp[i] = ctypes.addressof(frs[-1])
            if want_frags and nseg:
                fragss.append(ctypes.create_string_buffer(nseg * total * self.frag))
                gp[i] = ctypes.addressof(fragss[-1])
            else:
                fragss.append(None)
                gp[i] = None
        fids = ctypes.create_string_buffer(32 * n)
        self._check(self.ctx._L.dm_process_batch(self.enc._h, ptrs, lens, n, self.segment, gp, sp, fp, fids),
                    "dm_process_batch")
        out = []
        for i, b in enumerate(bufs):
            nseg = (len(b) + self.segment - 1) // self.segment
            out.append((segs[i].raw[:32 * nseg], frs[i].raw[:32 * nseg * total], fids.raw[32 * i:32 * i + 32],
                        fragss[i].raw if fragss[i] is not None else None))
        return out

    def process_device_async(self, obj_ptr: int, length: int, parity_ptr: int, seg_hash_ptr: int,
                             frag_hash_ptr: int, fid_ptr: int, stream: int = 0) -> None:
        """``dm_process_device_async``: object already in HBM (room for whole segments)."""
        self._check(self.ctx._L.dm_process_device_async(self.enc._h, obj_ptr, length, self.segment, parity_ptr,
                                                        seg_hash_ptr or None, frag_hash_ptr or None, fid_ptr,
                                                        stream), "dm_process_device_async")

    # -- FullProcessing ----------------------------------------------------------------------------
    def full_processing_file(self, file: str, savedir: str, segment_files: Optional[bool] = None
                             ) -> Tuple[bytes, bytes, bytes]:
        """One ``dm_full_processing`` call: the library reads ``file``, writes every fragment (and
        segment) to ``savedir/<hex SHA-256>`` and returns (segment digests, fragment digests, fid)."""
        L = self.ctx._L
        if segment_files is None:
            segment_files = _write_segments()
        try:
            size = os.stat(file).st_size
        except OSError:
            size = 0
        cap = max(1, (size + self.segment - 1) // self.segment)
        total = self.k + self.m
        for _ in range(2):   # a FIFO / a file that grew: retry once with the count the library saw
            seg = ctypes.create_string_buffer(32 * cap)
            frag = ctypes.create_string_buffer(32 * cap * total)
            fid = ctypes.create_string_buffer(32)
            nseg = ctypes.c_uint64(0)
            rc = L.dm_full_processing(self.enc._h, os.fsencode(file), os.fsencode(savedir), self.segment,
                                      1 if segment_files else 0, seg, frag, cap, ctypes.byref(nseg), fid)
            if rc == DM_ERR_INVALID and nseg.value > cap:
                cap = nseg.value
                continue
            if rc == DM_ERR_IO:   # file errors keep Go's text ("open <path>: no such file or directory")
                raise DeossMerkleError(rc, (L.dm_last_error(None) or b"").decode())
            self._check(rc, "dm_full_processing")
            n = nseg.value
            return seg.raw[:32 * n], frag.raw[:32 * n * total], fid.raw
        raise DeossMerkleError(DM_ERR_INVALID, "dm_full_processing: file size changed during the call")

    def fragment_lookup(self, file: str, fragment_hash: str, want_bytes: bool = True
                        ) -> Optional[Tuple[int, int, Optional[bytes]]]:
        """``dm_fragment_lookup``: the fragment of ``file`` named ``fragment_hash`` (hex SHA-256), as
        the download handler finds it (node/fileHandler.go:962-979) -- without writing any file.
        Returns (segment index, fragment index, fragment bytes or None), or None when no fragment of
        the file has that name."""
        L = self.ctx._L
        want = bytes.fromhex(fragment_hash)
        if len(want) != 32:
            raise ValueError("fragment hash must be 32 bytes of hex")
        out = ctypes.create_string_buffer(self.frag) if want_bytes else None
        found, seg_i, frag_i = ctypes.c_int(0), ctypes.c_uint64(0), ctypes.c_int(0)
        rc = L.dm_fragment_lookup(self.enc._h, os.fsencode(file), self.segment, want, out, self.frag if out else 0,
                                  ctypes.byref(found), ctypes.byref(seg_i), ctypes.byref(frag_i))
        if rc == DM_ERR_IO:
            raise DeossMerkleError(rc, (L.dm_last_error(None) or b"").decode())
        self._check(rc, "dm_fragment_lookup")
        if not found.value:
            return None
        return seg_i.value, frag_i.value, (out.raw if out is not None else None)

    def FullProcessing(self, file: str, cipher: str, savedir: str
                       ) -> Tuple[Optional[List[SegmentDataInfo]], str, Optional[Exception]]:
        """FullProcessing in one library call (``dm_full_processing``: reads, coding, hashing and
        fragment writes overlapped)."""
        if cipher:
            return None, "", DeossMerkleError(DM_ERR_INVALID, "cipher is not supported by the GPU pipeline")
        try:
            segd, fragd, fid = self.full_processing_file(file, savedir)
        except (OSError, DeossMerkleError) as e:
            return None, "", e
        total = self.k + self.m
        info = []
        for s in range(len(segd) // 32):
            names = [os.path.join(savedir, fragd[32 * (s * total + j):32 * (s * total + j + 1)].hex())
                     for j in range(total)]
            info.append(SegmentDataInfo(os.path.join(savedir, segd[32 * s:32 * s + 32].hex()), names))
        return info, fid.hex(), None

    def NewProcessingStream(self, savedir: str, segment_files: Optional[bool] = None) -> "ProcessingStream":
        """FullProcessing while the body arrives: write() the pieces, close() -> (info, fid)."""
        return ProcessingStream(self, savedir, segment_files)

    def FullProcessingWindows(self, file: str, cipher: str, savedir: str
                              ) -> Tuple[Optional[List[SegmentDataInfo]], str, Optional[Exception]]:
        """The window path (the Go shim's shape before dm_full_processing): read a window of
        ``WINDOW_SEGMENTS`` segments, one ``dm_process_buffer`` call, write its fragments, repeat.
        Kept as the A/B baseline of ``bench.py --workload fullprocessing``."""
        if cipher:
            return None, "", DeossMerkleError(DM_ERR_INVALID, "cipher is not supported by the GPU pipeline")
        try:
            size = os.path.getsize(file)
        except OSError as e:
            return None, "", e
        if size == 0:
            return None, "", DeossMerkleError(-1, "Empty data")
        os.makedirs(savedir, exist_ok=True)
        info: List[SegmentDataInfo] = []
        seg_digests = []
        window = WINDOW_SEGMENTS * self.segment
        total = self.k + self.m
        try:
            with open(file, "rb") as f:
                while True:
                    buf = f.read(window)
                    if not buf:
                        break
                    segd, fragd, fid, frags = self.process_buffer(buf, want_frags=True)
                    for s in range(len(segd) // 32):
                        seg_digests.append(segd[32 * s:32 * s + 32])
                        names = []
                        for j in range(total):
                            t = s * total + j
                            path = os.path.join(savedir, fragd[32 * t:32 * t + 32].hex())
                            if not os.path.exists(path):
                                with open(path, "wb") as out:
                                    out.write(frags[t * self.frag:(t + 1) * self.frag])
                            names.append(path)
                        seg_path = os.path.join(savedir, segd[32 * s:32 * s + 32].hex())
                        if not os.path.exists(seg_path):   # data fragments in order = the padded segment
                            with open(seg_path, "wb") as out:
                                out.write(frags[s * total * self.frag:(s * total + self.k) * self.frag])
                        info.append(SegmentDataInfo(seg_path, names))
                    if len(buf) < window:
                        break
        except (OSError, DeossMerkleError) as e:
            return None, "", e
        if len(seg_digests) * self.segment > window:   # several windows: tree over all segments
            fid = self.ctx.tree_root(b"".join(seg_digests))
        return info, fid.hex(), None


class ProcessingStream:
    """FullProcessing while the upload body arrives (``dm_pstream_*``): ``write()`` pieces of any
    size beside the handler's own file write, ``close()`` -> (SegmentDataInfo list, hex fid) with
    every fragment and segment file in ``savedir`` -- the same results as
    ``FullProcessing(file, "", savedir)`` on the same bytes, without reading the file again."""

    def __init__(self, proc: "Processor", savedir: str, segment_files: Optional[bool] = None):
        self._p = proc
        self._L = proc.ctx._L
        self.savedir = savedir
        self.written = 0
        self.device_bytes = self.peak_device_bytes = 0
        h = ctypes.c_void_p()
        if segment_files is None:
            segment_files = _write_segments()
        rc = self._L.dm_pstream_open(proc.enc._h, proc.segment, os.fsencode(savedir), 1 if segment_files else 0,
                                     ctypes.byref(h))
        self._raise(rc, "dm_pstream_open")
        self._h = h

    def _raise(self, rc: int, what: str) -> None:
        if rc == 0:
            return
        detail = (self._L.dm_last_error(None) or b"").decode()
        if rc == DM_ERR_EMPTY:
            raise DeossMerkleError(rc, "Empty data")
        if rc == DM_ERR_IO:
            raise DeossMerkleError(rc, detail)
        raise DeossMerkleError(rc, f"{what}: {self._L.dm_strerror(rc).decode()}: {detail}")

    def write(self, data) -> int:
        """One piece: bytes-like, or (address, length) of host memory."""
        if self._h is None:
            raise DeossMerkleError(DM_ERR_INVALID, "stream is closed")
        if isinstance(data, tuple):
            addr, n = data
            ptr = ctypes.c_void_p(addr)
        elif isinstance(data, bytes):
            n, ptr = len(data), ctypes.c_char_p(data)   # no copy
        else:
            mv = memoryview(data).cast("B")
            n = mv.nbytes
            ptr = ctypes.c_char_p(mv.tobytes()) if (mv.readonly or n == 0) else (ctypes.c_char * n).from_buffer(mv)
        rc = self._L.dm_pstream_write(self._h, ptr, n)
        if rc != 0:
            self.abort()
            self._raise(rc, "dm_pstream_write")
        self.written += n
        return n

    def close(self) -> Tuple[List[SegmentDataInfo], str]:
        if self._h is None:
            raise DeossMerkleError(DM_ERR_INVALID, "stream is closed")
        p = self._p
        total = p.k + p.m
        cap = max(1, (self.written + p.segment - 1) // p.segment)
        seg = ctypes.create_string_buffer(32 * cap)
        frag = ctypes.create_string_buffer(32 * cap * total)
        fid = ctypes.create_string_buffer(32)
        nseg = ctypes.c_uint64(0)
        self.device_bytes, self.peak_device_bytes = self.stats()
        h, self._h = self._h, None
        self._raise(self._L.dm_pstream_close(h, seg, frag, cap, ctypes.byref(nseg), fid), "dm_pstream_close")
        n = nseg.value
        info = []
        for s in range(n):
            names = [os.path.join(self.savedir, frag.raw[32 * (s * total + j):32 * (s * total + j + 1)].hex())
                     for j in range(total)]
            info.append(SegmentDataInfo(os.path.join(self.savedir, seg.raw[32 * s:32 * s + 32].hex()), names))
        self.segment_digests = seg.raw[:32 * n]
        self.fragment_digests = frag.raw[:32 * n * total]
        return info, fid.raw.hex()

    def stats(self) -> Tuple[int, int]:
        """(device bytes the stream holds now, the most it has held): chunk buffers in use or spare,
        bounded by DEOSS_PS_DEVICE_CAP (default 16 GiB), not by the body size."""
        if self._h is None:
            return self.device_bytes, self.peak_device_bytes
        cur, peak = ctypes.c_uint64(), ctypes.c_uint64()
        self._raise(self._L.dm_pstream_stats(self._h, ctypes.byref(cur), ctypes.byref(peak)), "dm_pstream_stats")
        return cur.value, peak.value

    def abort(self) -> None:
        if self._h is not None:
            self._L.dm_pstream_abort(self._h)
            self._h = None

    def __del__(self):
        try:
            self.abort()
        except Exception:
            pass


_default: Optional[Processor] = None


def FullProcessing(file: str, cipher: str, savedir: str
                   ) -> Tuple[Optional[List[SegmentDataInfo]], str, Optional[Exception]]:
    """process.FullProcessing(file, cipher, savedir) on the default GPU pipeline."""
    global _default
    if _default is None:
        try:
            _default = Processor()
        except DeossMerkleError as e:   # no GPU: the Go shape (nil, "", err), as gpu() fails in Go
            return None, "", e
    return _default.FullProcessing(file, cipher, savedir)


def FindFragment(fpath: str, fragment_hash: str) -> Tuple[Optional[bytes], Optional[Exception]]:
    """process.FindFragment (go/process/process_hip.go) on the default GPU pipeline: the fragment
    of ``fpath`` named ``fragment_hash``, or (None, None) when the file has no such fragment."""
    global _default
    # file names are lower-case hex SHA-256 (node/fileHandler.go:968): any other spelling names no
    # fragment, as the handler's string comparison would find none
    try:
        ok = len(fragment_hash) == 64 and bytes.fromhex(fragment_hash).hex() == fragment_hash
    except ValueError:
        ok = False
    if not ok:
        return None, None
    try:
        if _default is None:
            _default = Processor()
        hit = _default.fragment_lookup(fpath, fragment_hash)
    except (DeossMerkleError, ValueError) as e:
        return None, e
    return (hit[2] if hit else None), None


def FullProcessingFiles(files: List[str], cipher: str, savedir: str
                        ) -> Tuple[List[Optional[List[SegmentDataInfo]]], List[str], List[Optional[Exception]]]:
    """process.FullProcessingFiles (go/process/process_hip.go; the batch upload PUT /files,
    node/filesHandler.go:197-207): every file's FullProcessing at once, results in file order; an
    empty path is skipped (None, "", None)."""
    from concurrent.futures import ThreadPoolExecutor
    n = len(files)
    infos: List[Optional[List[SegmentDataInfo]]] = [None] * n
    fids, errs = [""] * n, [None] * n

    def one(i):
        infos[i], fids[i], errs[i] = FullProcessing(files[i], cipher, savedir)

    global _default
    todo = [i for i in range(n) if files[i]]
    if todo and _default is None:   # the default pipeline, made once before the calls start
        try:
            _default = Processor()
        except DeossMerkleError as e:   # no GPU: every call fails the Go way
            return [None] * n, [""] * n, [e if files[i] else None for i in range(n)]
    with ThreadPoolExecutor(max(1, min(16, len(todo)))) as ex:
        list(ex.map(one, todo))
    return infos, fids, errs
