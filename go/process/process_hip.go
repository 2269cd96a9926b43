//go:build hip

// Package process is a GPU-backed stand-in for cess-go-sdk core/process.FullProcessing (DeOSS
// go.mod:8), the call every upload handler makes to get the file id and the fragment names
// (node/objectHandler.go:168, node/fileHandler.go:771, node/filesHandler.go:201,
// node/resumeHandler.go:326, node/tracker.go:767-769) and the fragment download path re-runs
// (node/fileHandler.go:964,997).  Same signature and result shape; segmenting, Reed-Solomon 4 + 8
// coding, the SHA-256 names and the fid tree run on the MI355X (include/deoss_merkle.h): calls
// from concurrent handler goroutines go through one dm_batcher, which coalesces whatever is
// queued into one batched GPU pass (dm_batcher_process), and dm_tree_levels builds the fid of
// files larger than one window.  Swap it in by changing the handlers' import of
// github.com/CESSProject/cess-go-sdk/core/process to this package (INTEGRATION.md).
// Deviations: cipher must be "" (the AES branch is not implemented), and segment files are not
// written (their bytes are the data fragments in order).  Build with `-tags hip`, CGO_ENABLED=1.
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
	"sync"
	"unsafe"

	"github.com/CESSProject/cess-go-sdk/chain"
)

// windowSegments is the number of segments coded per GPU call (2 GiB of file at 32 MiB).
const windowSegments = 64

var (
	once    sync.Once
	ctx     *C.dm_ctx     // tree levels over the segment digests of multi-window files
	batcher *C.dm_batcher // FullProcessing requests from every goroutine
	initEr  error
)

func gpu() error {
	once.Do(func() {
		if rc := C.dm_create(&ctx, nil, 0); rc != C.DM_OK {
			initEr = errors.New(C.GoString(C.dm_strerror(rc)))
			return
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
	if st.Size() == 0 {
		return nil, "", errors.New("Empty data")
	}
	if err = os.MkdirAll(savedir, 0755); err != nil {
		return nil, "", err
	}
	seg := uint64(chain.SegmentSize)
	total := chain.DataShards + chain.ParShards
	frag := seg / uint64(chain.DataShards)
	wsize := windowSegments * seg // a small upload reads into a buffer of its own size
	if uint64(st.Size()) < wsize {
		wsize = uint64(st.Size())
	}
	window := make([]byte, wsize)
	var info []chain.SegmentDataInfo
	var segDigests []byte
	var fid [32]byte
	for {
		n, rerr := io.ReadFull(f, window)
		if n == 0 {
			if rerr == io.EOF && len(info) == 0 {
				return nil, "", errors.New("Empty data")
			}
			break
		}
		nseg := (uint64(n) + seg - 1) / seg
		frags := make([]byte, nseg*uint64(total)*frag)
		segd := make([]byte, 32*nseg)
		fragd := make([]byte, 32*nseg*uint64(total))
		runtime.LockOSThread()
		rc := C.dm_batcher_process(batcher, unsafe.Pointer(&window[0]), C.uint64_t(n), unsafe.Pointer(&frags[0]),
			(*C.uint8_t)(unsafe.Pointer(&segd[0])), (*C.uint8_t)(unsafe.Pointer(&fragd[0])),
			(*C.uint8_t)(unsafe.Pointer(&fid[0])))
		var perr error
		if rc != C.DM_OK {
			perr = batcherError(rc)
		}
		runtime.UnlockOSThread()
		if perr != nil {
			return nil, "", perr
		}
		for s := uint64(0); s < nseg; s++ {
			names := make([]string, total)
			for j := 0; j < total; j++ {
				t := s*uint64(total) + uint64(j)
				p := filepath.Join(savedir, hex.EncodeToString(fragd[32*t:32*t+32]))
				if _, err := os.Stat(p); err != nil {
					if err = os.WriteFile(p, frags[t*frag:(t+1)*frag], os.ModePerm); err != nil {
						return nil, "", err
					}
				}
				names[j] = p
			}
			info = append(info, chain.SegmentDataInfo{
				SegmentHash:  filepath.Join(savedir, hex.EncodeToString(segd[32*s:32*s+32])),
				FragmentHash: names,
			})
		}
		segDigests = append(segDigests, segd...)
		if rerr != nil { // short final window
			break
		}
	}
	if len(info) > windowSegments { // several windows: the fid is the tree over every segment
		nodes := make([]byte, 32*uint64(C.dm_tree_node_count(C.uint64_t(len(info)))))
		if rc := C.dm_tree_levels(ctx, (*C.uint8_t)(unsafe.Pointer(&segDigests[0])), C.uint64_t(len(info)),
			(*C.uint8_t)(unsafe.Pointer(&nodes[0]))); rc != C.DM_OK {
			return nil, "", ctxError(rc)
		}
		copy(fid[:], nodes[len(nodes)-32:])
	}
	return info, hex.EncodeToString(fid[:]), nil
}
