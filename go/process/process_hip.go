//go:build hip

// Package process is a GPU-backed stand-in for cess-go-sdk core/process.FullProcessing (DeOSS
// go.mod:8), the call every upload handler makes to get the file id and the fragment names
// (node/objectHandler.go:168, node/fileHandler.go:771, node/filesHandler.go:201,
// node/resumeHandler.go:326, node/tracker.go:767-769) and the fragment download path re-runs
// (node/fileHandler.go:964,997).  Same signature and result shape; segmenting, Reed-Solomon 4 + 8
// coding, the SHA-256 names and the fid tree run on the MI355X (include/deoss_merkle.h): calls
// from concurrent handler goroutines go through one dm_batcher, which coalesces whatever is
// queued into one batched GPU pass (dm_batcher_process); files larger than one window (8
// segments) go through dm_full_processing on a per-GPU pipeline, which reads the file, writes
// every fragment and segment file itself and overlaps those writes with the GPU's coding and
// hashing (one GPU pass per 32 GiB of file, no Go memory for the data).  Go memory of the small
// path is bounded process-wide: 1 GiB per window in flight, DEOSS_PROCESS_MEM_GIB (default 8)
// windows at once across every upload, buffers pooled.  Swap it in by changing the handlers' import of
// github.com/CESSProject/cess-go-sdk/core/process to this package (INTEGRATION.md).
// Deviation: cipher must be "" (the AES branch is not implemented; INTEGRATION.md).  Segment and
// fragment files are both written to savedir under their hex SHA-256.  Build with `-tags hip`,
// CGO_ENABLED=1.
package process

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../deoss_amd -ldeoss_merkle -Wl,-rpath,${SRCDIR}/../../deoss_amd
#include <stdlib.h>
#include "deoss_merkle.h"
*/
import "C"

import (
	"encoding/hex"
	"errors"
	"io"
	"os"
	"path/filepath"
	"runtime"
	"strconv"
	"sync"
	"sync/atomic"
	"unsafe"

	"github.com/CESSProject/cess-go-sdk/chain"
)

// windowSegments segments go to the GPU per call: 8 x 32 MiB of file plus 8 x 12 x 8 MiB of
// fragments = 1 GiB of Go memory per window.  A large file runs several windows at once (they
// meet in the same dm_batcher pass, so the GPU still sees one wide batch), and every window in
// flight, across all goroutines, holds one slot of the process-wide memory budget.
const windowSegments = 8

var (
	once    sync.Once
	ctx     *C.dm_ctx     // tree levels over the segment digests of multi-window files
	batcher *C.dm_batcher // FullProcessing requests from every goroutine
	initEr  error
	slots   chan struct{} // window budget: DEOSS_PROCESS_MEM_GIB (default 8) GiB / 1 GiB per window
	bufs    sync.Pool     // *windowBuf, reused across calls
	pipes   chan *C.dm_rs // large files: one dm_full_processing pipeline per GPU
	coders  []*C.dm_rs    // the same pipelines, for streams (NewWriter picks one round robin)
	nextW   atomic.Uint64
	// writeSegments: SegmentHash paths exist as files (the zero-padded segment bytes), like the
	// fragment paths; DEOSS_SKIP_SEGMENT_FILES=1 skips them (DeOSS itself only opens fragments).
	writeSegments = os.Getenv("DEOSS_SKIP_SEGMENT_FILES") != "1"
)

type windowBuf struct {
	data, frags, segd, fragd []byte
}

func gpu() error {
	once.Do(func() {
		budget := 8
		if v, err := strconv.Atoi(os.Getenv("DEOSS_PROCESS_MEM_GIB")); err == nil && v > 0 {
			budget = v
		}
		slots = make(chan struct{}, budget)
		seg, total := uint64(chain.SegmentSize), uint64(chain.DataShards+chain.ParShards)
		frag := seg / uint64(chain.DataShards)
		bufs.New = func() any {
			return &windowBuf{data: make([]byte, windowSegments*seg), frags: make([]byte, windowSegments*total*frag),
				segd: make([]byte, 32*windowSegments), fragd: make([]byte, 32*windowSegments*total)}
		}
		if rc := C.dm_create(&ctx, nil, 0); rc != C.DM_OK {
			initEr = errors.New(C.GoString(C.dm_strerror(rc)))
			return
		}
		ngpu := int(C.dm_gpu_count())
		pipes = make(chan *C.dm_rs, ngpu)
		for g := 0; g < ngpu; g++ {
			var pc *C.dm_ctx
			var rs *C.dm_rs
			dev := C.int(g)
			if rc := C.dm_create(&pc, &dev, 1); rc != C.DM_OK {
				initEr = errors.New(C.GoString(C.dm_strerror(rc)))
				return
			}
			if rc := C.dm_rs_create(pc, C.int(chain.DataShards), C.int(chain.ParShards), &rs); rc != C.DM_OK {
				initEr = errors.New(C.GoString(C.dm_strerror(rc)))
				return
			}
			pipes <- rs
			coders = append(coders, rs)
		}
		// every visible GPU, 2 worker slots each, 4096 leaves per batch, 2 ms linger (DESIGN.md §6.9)
		if rc := C.dm_batcher_create(nil, 0, C.DM_BATCH_PROCESS, C.uint64_t(chain.SegmentSize), C.int(chain.DataShards),
			C.int(chain.ParShards), 0, 0, 0, 2000, &batcher); rc != C.DM_OK {
			initEr = errors.New(C.GoString(C.dm_batcher_last_error()))
		}
	})
	return initEr
}

// batcherError must run on the goroutine's OS thread that made the call (the message is
// thread-local in the library): callers hold runtime.LockOSThread around the pair.
func batcherError(rc C.int) error {
	if rc == C.DM_ERR_EMPTY {
		return errors.New("Empty data")
	}
	if msg := C.GoString(C.dm_batcher_last_error()); msg != "" {
		return errors.New(msg)
	}
	return errors.New(C.GoString(C.dm_strerror(rc)))
}

func ctxError(rc C.int) error {
	if msg := C.GoString(C.dm_last_error(ctx)); msg != "" {
		return errors.New(msg)
	}
	return errors.New(C.GoString(C.dm_strerror(rc)))
}

// window is one GPU call's worth of the file: segments [first, first+nseg).
type window struct {
	first, nseg uint64
	n           int // file bytes in the window
	buf         *windowBuf
	fid         [32]byte
	err         error
}

// runWindow reads the window's bytes at its file offset, codes + hashes them through the batcher
// and writes its fragments to savedir; the caller holds one budget slot.
func runWindow(f *os.File, w *window, savedir string) {
	seg := uint64(chain.SegmentSize)
	total := uint64(chain.DataShards + chain.ParShards)
	frag := seg / uint64(chain.DataShards)
	b := bufs.Get().(*windowBuf)
	w.buf = b
	data := b.data[:w.n]
	if _, err := f.ReadAt(data, int64(w.first*seg)); err != nil && err != io.EOF {
		w.err = err
		return
	}
	runtime.LockOSThread()
	rc := C.dm_batcher_process(batcher, unsafe.Pointer(&data[0]), C.uint64_t(w.n), unsafe.Pointer(&b.frags[0]),
		(*C.uint8_t)(unsafe.Pointer(&b.segd[0])), (*C.uint8_t)(unsafe.Pointer(&b.fragd[0])),
		(*C.uint8_t)(unsafe.Pointer(&w.fid[0])))
	if rc != C.DM_OK {
		w.err = batcherError(rc)
	}
	runtime.UnlockOSThread()
	if w.err != nil {
		return
	}
	for t := uint64(0); t < w.nseg*total; t++ { // fragments go to disk before the buffer is reused
		p := filepath.Join(savedir, hex.EncodeToString(b.fragd[32*t:32*t+32]))
		if _, err := os.Stat(p); err != nil {
			if err = os.WriteFile(p, b.frags[t*frag:(t+1)*frag], os.ModePerm); err != nil {
				w.err = err
				return
			}
		}
	}
	if !writeSegments {
		return
	}
	// SegmentHash names a file too: the zero-padded segment, i.e. its data fragments in order
	for s := uint64(0); s < w.nseg; s++ {
		p := filepath.Join(savedir, hex.EncodeToString(b.segd[32*s:32*s+32]))
		if _, err := os.Stat(p); err != nil {
			first := s * total * frag
			if err = os.WriteFile(p, b.frags[first:first+seg], os.ModePerm); err != nil {
				w.err = err
				return
			}
		}
	}
}

// FullProcessing cuts file into chain.SegmentSize segments (the last zero-padded), codes each into
// chain.DataShards + chain.ParShards fragments written to savedir/<hex SHA-256>, and returns the
// segment / fragment path names and the fid (hex hashtree root over the segments).
func FullProcessing(file string, cipher string, savedir string) ([]chain.SegmentDataInfo, string, error) {
	if cipher != "" {
		return nil, "", errors.New("process: cipher is not supported by the GPU pipeline")
	}
	if err := gpu(); err != nil {
		return nil, "", err
	}
	f, err := os.Open(file)
	if err != nil {
		return nil, "", err
	}
	defer f.Close()
	st, err := f.Stat()
	if err != nil {
		return nil, "", err
	}
	size := uint64(st.Size())
	if size == 0 {
		return nil, "", errors.New("Empty data")
	}
	if err = os.MkdirAll(savedir, 0755); err != nil {
		return nil, "", err
	}
	seg := uint64(chain.SegmentSize)
	total := chain.DataShards + chain.ParShards
	nsegAll := (size + seg - 1) / seg
	if nsegAll > windowSegments {
		return fullProcessingLarge(file, savedir, nsegAll)
	}
	var wins []*window
	for first := uint64(0); first < nsegAll; first += windowSegments {
		nseg := min(uint64(windowSegments), nsegAll-first)
		wins = append(wins, &window{first: first, nseg: nseg, n: int(min(nseg*seg, size-first*seg))})
	}
	var wg sync.WaitGroup
	for _, w := range wins { // windows run concurrently within the budget and batch together on the GPU
		slots <- struct{}{}
		wg.Add(1)
		go func(w *window) {
			defer wg.Done()
			defer func() { <-slots }()
			runWindow(f, w, savedir)
		}(w)
	}
	wg.Wait()
	info := make([]chain.SegmentDataInfo, 0, nsegAll)
	segDigests := make([]byte, 0, 32*nsegAll)
	var firstErr error
	for _, w := range wins {
		if w.err != nil && firstErr == nil {
			firstErr = w.err
		}
		if firstErr == nil {
			b := w.buf
			for s := uint64(0); s < w.nseg; s++ {
				names := make([]string, total)
				for j := 0; j < total; j++ {
					t := s*uint64(total) + uint64(j)
					names[j] = filepath.Join(savedir, hex.EncodeToString(b.fragd[32*t:32*t+32]))
				}
				info = append(info, chain.SegmentDataInfo{
					SegmentHash:  filepath.Join(savedir, hex.EncodeToString(b.segd[32*s:32*s+32])),
					FragmentHash: names,
				})
			}
			segDigests = append(segDigests, b.segd[:32*w.nseg]...)
		}
		if w.buf != nil {
			bufs.Put(w.buf)
			w.buf = nil
		}
	}
	if firstErr != nil {
		return nil, "", firstErr
	}
	fid := wins[0].fid
	if len(wins) > 1 { // several windows: the fid is the tree over every segment
		nodes := make([]byte, 32*uint64(C.dm_tree_node_count(C.uint64_t(len(info)))))
		runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
		defer runtime.UnlockOSThread()
		if rc := C.dm_tree_levels(ctx, (*C.uint8_t)(unsafe.Pointer(&segDigests[0])), C.uint64_t(len(info)),
			(*C.uint8_t)(unsafe.Pointer(&nodes[0]))); rc != C.DM_OK {
			return nil, "", ctxError(rc)
		}
		copy(fid[:], nodes[len(nodes)-32:])
	}
	return info, hex.EncodeToString(fid[:]), nil
}

// fullProcessingLarge: one dm_full_processing call on a free per-GPU pipeline.  The library reads
// the file, writes every fragment and segment file to savedir/<hex SHA-256> (data fragments while
// the file is still being read, parity fragments while the leaf kernel hashes) and returns the
// digests and the fid.
func fullProcessingLarge(file, savedir string, nseg uint64) ([]chain.SegmentDataInfo, string, error) {
	total := uint64(chain.DataShards + chain.ParShards)
	rs := <-pipes
	defer func() { pipes <- rs }()
	for attempt := 0; ; attempt++ {
		segd := make([]byte, 32*nseg)
		fragd := make([]byte, 32*nseg*total)
		var fid [32]byte
		var got C.uint64_t
		cfile, cdir := C.CString(file), C.CString(savedir)
		flags := C.int(C.DM_FP_SEGMENT_FILES)
		if !writeSegments {
			flags = 0
		}
		runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
		rc := C.dm_full_processing(rs, cfile, cdir, C.uint64_t(chain.SegmentSize), flags,
			(*C.uint8_t)(unsafe.Pointer(&segd[0])), (*C.uint8_t)(unsafe.Pointer(&fragd[0])), C.uint64_t(nseg), &got,
			(*C.uint8_t)(unsafe.Pointer(&fid[0])))
		var err error
		if rc != C.DM_OK {
			if msg := C.GoString(C.dm_last_error(nil)); msg != "" {
				err = errors.New(msg)
			} else {
				err = errors.New(C.GoString(C.dm_strerror(rc)))
			}
		}
		runtime.UnlockOSThread()
		C.free(unsafe.Pointer(cfile))
		C.free(unsafe.Pointer(cdir))
		if rc == C.DM_ERR_INVALID && uint64(got) > nseg && attempt == 0 { // the file grew since Stat
			nseg = uint64(got)
			continue
		}
		if err != nil {
			return nil, "", err
		}
		info := make([]chain.SegmentDataInfo, 0, nseg)
		for s := uint64(0); s < uint64(got); s++ {
			names := make([]string, total)
			for j := uint64(0); j < total; j++ {
				t := s*total + j
				names[j] = filepath.Join(savedir, hex.EncodeToString(fragd[32*t:32*t+32]))
			}
			info = append(info, chain.SegmentDataInfo{
				SegmentHash:  filepath.Join(savedir, hex.EncodeToString(segd[32*s:32*s+32])),
				FragmentHash: names,
			})
		}
		return info, hex.EncodeToString(fid[:]), nil
	}
}
