//go:build hip

// Package process is a GPU-backed stand-in for cess-go-sdk core/process.FullProcessing (DeOSS
// go.mod:8), the call every upload handler makes to get the file id and the fragment names
// (node/objectHandler.go:168, node/fileHandler.go:771, node/filesHandler.go:201,
// node/resumeHandler.go:326, node/tracker.go:767-769) and the fragment download path re-runs
// (node/fileHandler.go:964,997).  Same signature and result shape; segmenting, Reed-Solomon 4 + 8
// coding, the SHA-256 names and the fid tree run on the MI355X (include/deoss_merkle.h):
//   - files of up to one window (8 segments = 256 MiB), the common upload: one call through a
//     process-wide dm_batcher, which coalesces whatever concurrent handler goroutines have queued
//     into one batched GPU pass (dm_batcher_process); Go memory is bounded process-wide (1 GiB
//     per call in flight, DEOSS_PROCESS_MEM_GIB (default 8) at once, buffers pooled);
//   - larger files: dm_full_processing on a lane of a per-GPU pipeline, which reads the file, writes every
//     fragment and segment file itself and overlaps those writes with the GPU's coding and hashing
//     (one GPU pass per 32 GiB of file, no Go memory for the data);
//   - cipher != "" (an encrypted upload, the Cipher header of node/objectHandler.go:102 and
//     node/fileHandler.go:705): the SDK's own FullProcessing, unchanged -- its AES scheme is not
//     restated here, so those uploads keep exactly the SDK's results.
// Swap it in by changing the handlers' import of github.com/CESSProject/cess-go-sdk/core/process to
// this package (INTEGRATION.md).  Segment and fragment files are both written to savedir under
// their hex SHA-256.  Build with `-tags hip`, CGO_ENABLED=1, PKG_CONFIG_PATH=<checkout>/deoss_amd.
package process

/*
#cgo pkg-config: deoss_merkle
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
	sdkprocess "github.com/CESSProject/cess-go-sdk/core/process"
)

// windowSegments: files of up to this many segments go to the GPU in one batcher call (at most
// 8 x 32 MiB of file plus 8 x 12 x 8 MiB of fragments = 1 GiB of Go memory).  Every call in
// flight, across all goroutines, holds its segments' share of the process-wide memory budget
// (128 MiB per segment), so a 1 MiB upload holds 1/64 of the default budget, not a whole window,
// and up to 64 small uploads reach the batcher together.  Larger files take dm_full_processing
// (no Go memory for the data).
const windowSegments = 8

var (
	once       sync.Once
	batcher    *C.dm_batcher // FullProcessing requests from every goroutine
	initEr     error
	budgetMu   sync.Mutex
	budgetCond = sync.NewCond(&budgetMu)
	budgetFree int                          // segments: DEOSS_PROCESS_MEM_GIB (default 8) GiB / 128 MiB
	bufs       [windowSegments + 1]sync.Pool // *windowBuf for n segments, reused across calls
	pipes   chan *C.dm_rs // large files: each GPU's pipeline, once per call lane of its context
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
		seg, total := uint64(chain.SegmentSize), uint64(chain.DataShards+chain.ParShards)
		frag := seg / uint64(chain.DataShards)
		perSeg := seg + total*frag // Go bytes one segment of a window holds
		budgetFree = int(uint64(budget) << 30 / perSeg)
		if budgetFree < windowSegments {
			budgetFree = windowSegments // one full window always fits
		}
		for n := 1; n <= windowSegments; n++ {
			k := uint64(n)
			bufs[n].New = func() any {
				return &windowBuf{data: make([]byte, k*seg), frags: make([]byte, k*total*frag),
					segd: make([]byte, 32*k), fragd: make([]byte, 32*k*total)}
			}
		}
		ngpu := int(C.dm_gpu_count())
		if ngpu <= 0 {
			initEr = errors.New(C.GoString(C.dm_strerror(C.DM_ERR_NODEV)))
			return
		}
		pipes = make(chan *C.dm_rs, ngpu*8)
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
			// one token per call lane: a coder's calls run on its context's lanes (own staging each),
			// so that many large uploads share the GPU side by side (DEOSS_LANES; 4 per MI355X by default)
			for l := 0; l < int(C.dm_lane_count(pc)); l++ {
				pipes <- rs
			}
			coders = append(coders, rs)
		}
		// every visible GPU, 4 worker slots each (the library default), 4096 leaves per batch, 2 ms
		// linger (DESIGN.md §6.9)
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

// acquireBudget blocks until n segments of the Go memory budget are free and takes them.
func acquireBudget(n int) {
	budgetMu.Lock()
	for budgetFree < n {
		budgetCond.Wait()
	}
	budgetFree -= n
	budgetMu.Unlock()
}

func releaseBudget(n int) {
	budgetMu.Lock()
	budgetFree += n
	budgetMu.Unlock()
	budgetCond.Broadcast()
}

// window is one batcher call: the whole file, nseg <= windowSegments segments.
type window struct {
	nseg uint64
	n    int // file bytes
	buf  *windowBuf
	fid  [32]byte
	err  error
}

// runWindow reads the file, codes + hashes it through the batcher and writes its fragments to
// savedir; the caller holds one budget slot.
func runWindow(f *os.File, w *window, savedir string) {
	seg := uint64(chain.SegmentSize)
	total := uint64(chain.DataShards + chain.ParShards)
	frag := seg / uint64(chain.DataShards)
	b := bufs[w.nseg].Get().(*windowBuf)
	w.buf = b
	data := b.data[:w.n]
	// every byte must come from this file: a pooled buffer still holds an earlier upload's bytes,
	// so a file shorter than its Stat size (truncated or rewritten since) is an error, as in
	// dm_full_processing ("unexpected EOF"), never a silently stale tail
	if n, err := f.ReadAt(data, 0); n != w.n {
		if err == nil || err == io.EOF {
			err = io.ErrUnexpectedEOF
		}
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
	if cipher != "" { // encrypted upload: the SDK's own pipeline (AES before coding), unchanged
		return sdkprocess.FullProcessing(file, cipher, savedir)
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
	total := uint64(chain.DataShards + chain.ParShards)
	nseg := (size + seg - 1) / seg
	if nseg > windowSegments {
		return fullProcessingLarge(file, savedir, nseg)
	}
	w := &window{nseg: nseg, n: int(size)}
	acquireBudget(int(nseg))
	runWindow(f, w, savedir)
	releaseBudget(int(nseg))
	defer func() {
		if w.buf != nil {
			bufs[nseg].Put(w.buf)
		}
	}()
	if w.err != nil {
		return nil, "", w.err
	}
	b := w.buf
	info := make([]chain.SegmentDataInfo, 0, nseg)
	for s := uint64(0); s < nseg; s++ {
		names := make([]string, total)
		for j := uint64(0); j < total; j++ {
			t := s*total + j
			names[j] = filepath.Join(savedir, hex.EncodeToString(b.fragd[32*t:32*t+32]))
		}
		info = append(info, chain.SegmentDataInfo{
			SegmentHash:  filepath.Join(savedir, hex.EncodeToString(b.segd[32*s:32*s+32])),
			FragmentHash: names,
		})
	}
	return info, hex.EncodeToString(w.fid[:]), nil
}

// FullProcessingFiles (additive, for the batch upload PUT /files, node/filesHandler.go:197-207,
// which calls FullProcessing once per file from one goroutine): every file's FullProcessing at
// once, so small files share batched GPU passes (the process-wide batcher coalesces concurrent
// calls) instead of paying one segment chain (~0.5 s) each in turn, and large files run on the
// pipeline lanes side by side.  Results in file order, each exactly FullProcessing(files[i],
// cipher, savedir); an empty path is skipped (nil, "", nil), as the handler skips failed files.
func FullProcessingFiles(files []string, cipher string, savedir string) ([][]chain.SegmentDataInfo, []string, []error) {
	infos := make([][]chain.SegmentDataInfo, len(files))
	fids := make([]string, len(files))
	errs := make([]error, len(files))
	var wg sync.WaitGroup
	for i := range files {
		if files[i] == "" {
			continue
		}
		wg.Add(1)
		go func(i int) {
			defer wg.Done()
			infos[i], fids[i], errs[i] = FullProcessing(files[i], cipher, savedir)
		}(i)
	}
	wg.Wait()
	return infos, fids, errs
}

// fullProcessingLarge: one dm_full_processing call on a free pipeline lane.  The library reads
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

// FindFragment (additive, for the fragment download handler, node/fileHandler.go:962-979): the
// fragment of the file at fpath whose name is fragmentHash (hex SHA-256), found without writing
// every fragment to a cache directory first (dm_fragment_lookup: the file is RS-coded and its
// fragments hashed on the GPU window by window, and the scan stops at the window holding the name).
// Returns (nil, nil) when no fragment of the file has that name, as the handler's scan falls
// through to the chain.  The first match in (segment, index) order wins, as in the handler.
func FindFragment(fpath, fragmentHash string) ([]byte, error) {
	// The handler compares fragmentHash with file names, which are lower-case hex SHA-256
	// (node/fileHandler.go:968): any other spelling (upper case, wrong length, not hex) names no
	// fragment, so it is not found -- never decoded into a digest that would match one.
	want, err := hex.DecodeString(fragmentHash)
	if err != nil || len(want) != 32 || hex.EncodeToString(want) != fragmentHash {
		return nil, nil
	}
	if err := gpu(); err != nil {
		return nil, err
	}
	rs := <-pipes
	defer func() { pipes <- rs }()
	out := make([]byte, uint64(chain.SegmentSize)/uint64(chain.DataShards))
	cpath := C.CString(fpath)
	defer C.free(unsafe.Pointer(cpath))
	var found, idx C.int
	var seg C.uint64_t
	runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
	defer runtime.UnlockOSThread()
	rc := C.dm_fragment_lookup(rs, cpath, C.uint64_t(chain.SegmentSize), (*C.uint8_t)(unsafe.Pointer(&want[0])),
		unsafe.Pointer(&out[0]), C.uint64_t(len(out)), &found, &seg, &idx)
	if rc != C.DM_OK {
		if rc == C.DM_ERR_EMPTY {
			return nil, errors.New("Empty data")
		}
		if msg := C.GoString(C.dm_last_error(nil)); msg != "" {
			return nil, errors.New(msg)
		}
		return nil, errors.New(C.GoString(C.dm_strerror(rc)))
	}
	if found == 0 {
		return nil, nil
	}
	return out, nil
}
