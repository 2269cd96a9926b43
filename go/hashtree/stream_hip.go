//go:build hip

// Hash-while-receiving (SURVEY.md 8f #1).  The upload handlers copy the request body to a temp
// file and hash it afterwards (node/objectHandler.go:248-266 saveObjectToFile,
// node/fileHandler.go:899-937 saveFormFile).  A Stream is an io.Writer over dm_stream_*: every
// whole chunk is hashed on the GPU while later bytes are still arriving, so the Merkle tree is
// ready one chunk after the body ends.  Typical use, keeping the temp file the handler still needs:
//
//	hs, err := hashtree.NewStream(chunkSize)
//	...
//	length, err := io.Copy(io.MultiWriter(f, hs), c.Request.Body)
//	if err != nil { hs.Abort(); ... }
//	tree, err := hs.Close() // == NewHashTreeFromBuffer(body, chunkSize) / NewHashTree(chunk files)
package hashtree

/*
#include <stdlib.h>
#include "deoss_merkle.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"

	"github.com/cbergoon/merkletree"
)

// Stream hashes one object whose bytes arrive in pieces of any size.  It is used by one goroutine
// at a time; many streams may be open at once (they share the package's GPU context).
type Stream struct {
	c        *C.dm_ctx
	st       *C.dm_stream
	chunk    uint64
	received uint64
	err      error
}

// NewStream opens a stream that splits the object into chunkSize-byte leaves (a positive multiple
// of 16; DeOSS segments are chain.SegmentSize = 32 MiB).
func NewStream(chunkSize int) (*Stream, error) {
	if chunkSize <= 0 || chunkSize%16 != 0 {
		return nil, fmt.Errorf("hashtree: stream chunk size %d must be a positive multiple of 16", chunkSize)
	}
	c, err := gpu()
	if err != nil {
		return nil, err
	}
	s := &Stream{c: c, chunk: uint64(chunkSize)}
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	if rc := C.dm_stream_open(c, C.uint64_t(chunkSize), &s.st); rc != C.DM_OK {
		return nil, rcError(c, rc)
	}
	runtime.SetFinalizer(s, func(x *Stream) { x.Abort() })
	return s, nil
}

// Write copies p into the library's pinned staging (p is not retained) and launches leaf hashing
// for every chunk it completes.  After an error the stream only accepts Abort.
func (s *Stream) Write(p []byte) (int, error) {
	if s.st == nil {
		return 0, errors.New("hashtree: write on a closed stream")
	}
	if s.err != nil {
		return 0, s.err
	}
	if len(p) == 0 {
		return 0, nil
	}
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	if rc := C.dm_stream_write(s.st, unsafe.Pointer(&p[0]), C.uint64_t(len(p))); rc != C.DM_OK {
		s.err = rcError(s.c, rc)
		return 0, s.err
	}
	s.received += uint64(len(p))
	return len(p), nil
}

// Close waits for the last leaves, builds the tree and frees the stream.  Nothing written ->
// "Empty data" (types.go:21).  The result is the tree NewHashTree builds over the same chunks.
func (s *Stream) Close() (*merkletree.MerkleTree, error) {
	if s.st == nil {
		return nil, errors.New("hashtree: stream already closed")
	}
	st := s.st
	s.st = nil
	runtime.SetFinalizer(s, nil)
	if s.err != nil {
		C.dm_stream_abort(st)
		return nil, s.err
	}
	n := (s.received + s.chunk - 1) / s.chunk
	leaves := make([]byte, 32*max(n, 1))
	root := make([]byte, 32)
	var got C.uint64_t
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	rc := C.dm_stream_close(st, (*C.uint8_t)(unsafe.Pointer(&leaves[0])), C.uint64_t(n), &got,
		(*C.uint8_t)(unsafe.Pointer(&root[0])))
	if rc != C.DM_OK {
		return nil, rcError(s.c, rc)
	}
	if uint64(got) != n {
		return nil, fmt.Errorf("hashtree: stream closed with %d leaves, expected %d", uint64(got), n)
	}
	return buildTree(leaves[:32*n], root)
}

// Abort discards the stream (e.g. the client went away mid-body).
func (s *Stream) Abort() {
	if s.st != nil {
		C.dm_stream_abort(s.st)
		s.st = nil
		runtime.SetFinalizer(s, nil)
	}
}
