//go:build hip

package process

/*
#include <stdlib.h>
#include "deoss_merkle.h"
*/
import "C"

import (
	"encoding/hex"
	"errors"
	"path/filepath"
	"runtime"
	"unsafe"

	"github.com/CESSProject/cess-go-sdk/chain"
	sdkprocess "github.com/CESSProject/cess-go-sdk/core/process"
)

// Writer is FullProcessing while the upload body arrives (dm_pstream_*, include/deoss_merkle.h).
// The handlers save the body with io.Copy (node/objectHandler.go:248-266 saveObjectToFile,
// node/fileHandler.go:899-937) and then run FullProcessing(fpath, cipher, cacheDir) over the saved
// file (node/objectHandler.go:168, node/fileHandler.go:771), reading it again.  With a Writer the
// handler copies the body into io.MultiWriter(f, w): whole segments are copied to the GPU, coded,
// hashed and their fragment files written to savedir while later bytes are still being received;
// Close returns the same ([]chain.SegmentDataInfo, fid, error) as FullProcessing on the saved file.
// A Writer is used by one goroutine; Close or Abort must be called exactly once.  Device memory
// is bounded per Writer (DEOSS_PS_DEVICE_CAP, default 16 GiB), whatever the body size.
type Writer struct {
	st      *C.dm_pstream
	savedir string
	n       uint64
	// an encrypted upload (NewWriterFor with a cipher): the bytes only go to the handler's file,
	// and Close runs the SDK's FullProcessing(fpath, cipher, savedir) over it
	sdkFile, sdkCipher string
	sdkOpen            bool
}

// NewWriterFor is the handler-shaped form: fpath is the file the handler saves the body to (beside
// this Writer, through io.MultiWriter), cipher its Cipher header.  With cipher "" it is NewWriter;
// with a cipher the Writer only counts the bytes and Close returns the SDK's
// FullProcessing(fpath, cipher, savedir) over the saved file -- the handler must have written and
// closed fpath before Close.  So one code path serves plain and encrypted uploads.
func NewWriterFor(fpath, cipher, savedir string) (*Writer, error) {
	if cipher == "" {
		return NewWriter(savedir)
	}
	return &Writer{savedir: savedir, sdkFile: fpath, sdkCipher: cipher, sdkOpen: true}, nil
}

// NewWriter opens a streaming FullProcessing into savedir (FullProcessing(fpath, "", savedir)).
func NewWriter(savedir string) (*Writer, error) {
	if err := gpu(); err != nil {
		return nil, err
	}
	// a stream keeps its own HIP streams and buffers and only briefly locks its coder's context at
	// Close, so it shares the per-GPU pipelines round robin instead of holding one
	rs := coders[nextW.Add(1)%uint64(len(coders))]
	cdir := C.CString(savedir)
	defer C.free(unsafe.Pointer(cdir))
	flags := C.int(C.DM_FP_SEGMENT_FILES)
	if !writeSegments {
		flags = 0
	}
	w := &Writer{savedir: savedir}
	runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
	defer runtime.UnlockOSThread()
	if rc := C.dm_pstream_open(rs, C.uint64_t(chain.SegmentSize), cdir, flags, &w.st); rc != C.DM_OK {
		return nil, lastError(rc)
	}
	return w, nil
}

func lastError(rc C.int) error {
	if rc == C.DM_ERR_EMPTY {
		return errors.New("Empty data")
	}
	if msg := C.GoString(C.dm_last_error(nil)); msg != "" {
		return errors.New(msg)
	}
	return errors.New(C.GoString(C.dm_strerror(rc)))
}

// Write implements io.Writer.  The bytes are copied before it returns (p may be reused).
func (w *Writer) Write(p []byte) (int, error) {
	if w.sdkOpen {
		w.n += uint64(len(p))
		return len(p), nil
	}
	if w.st == nil {
		return 0, errors.New("process: write on a closed Writer")
	}
	if len(p) == 0 {
		return 0, nil
	}
	runtime.LockOSThread()
	rc := C.dm_pstream_write(w.st, unsafe.Pointer(&p[0]), C.uint64_t(len(p)))
	var err error
	if rc != C.DM_OK {
		err = lastError(rc)
	}
	runtime.UnlockOSThread()
	if err != nil {
		w.Abort()
		return 0, err
	}
	w.n += uint64(len(p))
	return len(p), nil
}

// Close finishes the last segment and returns FullProcessing's results for everything written.
func (w *Writer) Close() ([]chain.SegmentDataInfo, string, error) {
	if w.sdkOpen {
		w.sdkOpen = false
		return sdkprocess.FullProcessing(w.sdkFile, w.sdkCipher, w.savedir)
	}
	if w.st == nil {
		return nil, "", errors.New("process: Writer already closed")
	}
	seg := uint64(chain.SegmentSize)
	total := uint64(chain.DataShards + chain.ParShards)
	nseg := (w.n + seg - 1) / seg
	segd := make([]byte, 32*max(nseg, 1))
	fragd := make([]byte, 32*max(nseg, 1)*total)
	var fid [32]byte
	var got C.uint64_t
	st := w.st
	w.st = nil
	runtime.LockOSThread()
	rc := C.dm_pstream_close(st, (*C.uint8_t)(unsafe.Pointer(&segd[0])), (*C.uint8_t)(unsafe.Pointer(&fragd[0])),
		C.uint64_t(max(nseg, 1)), &got, (*C.uint8_t)(unsafe.Pointer(&fid[0])))
	var err error
	if rc != C.DM_OK {
		err = lastError(rc)
	}
	runtime.UnlockOSThread()
	if err != nil {
		return nil, "", err
	}
	info := make([]chain.SegmentDataInfo, 0, nseg)
	for s := uint64(0); s < uint64(got); s++ {
		names := make([]string, total)
		for j := uint64(0); j < total; j++ {
			t := s*total + j
			names[j] = filepath.Join(w.savedir, hex.EncodeToString(fragd[32*t:32*t+32]))
		}
		info = append(info, chain.SegmentDataInfo{
			SegmentHash:  filepath.Join(w.savedir, hex.EncodeToString(segd[32*s:32*s+32])),
			FragmentHash: names,
		})
	}
	return info, hex.EncodeToString(fid[:]), nil
}

// Abort drops the stream; no file it started is left in savedir.
func (w *Writer) Abort() {
	w.sdkOpen = false
	if w.st != nil {
		C.dm_pstream_abort(w.st)
		w.st = nil
	}
}
