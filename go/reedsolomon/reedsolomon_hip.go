//go:build hip

// Package reedsolomon is a GPU-backed stand-in for the subset of
// github.com/klauspost/reedsolomon v1.12.4 (DeOSS go.mod:65) that cess-go-sdk uses to code each
// segment into chain.DataShards + chain.ParShards fragments (node/tracker.go:250,369).  Same
// constructor, method set and errors for New / Split / Encode / Reconstruct / Verify; the bytes
// are coded by the MI355X library through include/deoss_merkle.h (dm_rs_*).  Only the default
// matrix (no options) is provided.  Build with `-tags hip` and CGO_ENABLED=1; swap it in with a
// go.mod `replace github.com/klauspost/reedsolomon => <this dir>` (INTEGRATION.md).
package reedsolomon

/*
#cgo pkg-config: deoss_merkle
#include <stdlib.h>
#include "deoss_merkle.h"
*/
import "C"

import (
	"errors"
	"runtime"
	"sync"
	"unsafe"
)

// Errors with klauspost's texts.
var (
	ErrInvShardNum  = errors.New("cannot create Encoder with less than one data shard or less than zero parity shards")
	ErrMaxShardNum  = errors.New("cannot create Encoder with more than 256 data+parity shards")
	ErrTooFewShards = errors.New("too few shards given")
	ErrShortData    = errors.New("not enough data to fill the number of requested shards")
	ErrShardSize    = errors.New("shard sizes do not match")
	ErrShardNoData  = errors.New("no shard data")
	ErrNotSupported = errors.New("operation not supported")
)

// Option is accepted for signature compatibility; no option changes the coding here.
type Option func()

// Encoder is the method subset of klauspost's Encoder that DeOSS's SDK calls.
type Encoder interface {
	Encode(shards [][]byte) error
	Verify(shards [][]byte) (bool, error)
	Reconstruct(shards [][]byte) error
	ReconstructData(shards [][]byte) error
	Split(data []byte) ([][]byte, error)
}

var (
	ctxOnce sync.Once
	ctx     *C.dm_ctx
	ctxErr  error
)

func gpu() (*C.dm_ctx, error) {
	ctxOnce.Do(func() {
		if rc := C.dm_create(&ctx, nil, 0); rc != C.DM_OK {
			ctxErr = errors.New(C.GoString(C.dm_strerror(rc)))
		}
	})
	return ctx, ctxErr
}

type rsGPU struct {
	h            *C.dm_rs
	data, parity int
}

// New creates an Encoder for dataShards + parityShards (1..8 each on the GPU path).
func New(dataShards, parityShards int, opts ...Option) (Encoder, error) {
	if dataShards <= 0 || parityShards < 0 {
		return nil, ErrInvShardNum
	}
	if dataShards+parityShards > 256 {
		return nil, ErrMaxShardNum
	}
	if dataShards > 8 || parityShards > 8 || parityShards == 0 {
		return nil, ErrNotSupported
	}
	c, err := gpu()
	if err != nil {
		return nil, err
	}
	r := &rsGPU{data: dataShards, parity: parityShards}
	runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
	defer runtime.UnlockOSThread()
	if rc := C.dm_rs_create(c, C.int(dataShards), C.int(parityShards), &r.h); rc != C.DM_OK {
		return nil, errors.New(C.GoString(C.dm_last_error(c)))
	}
	runtime.SetFinalizer(r, func(x *rsGPU) { C.dm_rs_destroy(x.h) })
	return r, nil
}

func (r *rsGPU) check(shards [][]byte, needAll bool) (int, error) {
	if len(shards) != r.data+r.parity {
		return 0, ErrTooFewShards
	}
	size := 0
	for _, s := range shards {
		if len(s) == 0 {
			if needAll {
				return 0, ErrShardNoData
			}
			continue
		}
		if size == 0 {
			size = len(s)
		} else if len(s) != size {
			return 0, ErrShardSize
		}
	}
	if size == 0 {
		return 0, ErrShardNoData
	}
	return size, nil
}

// cPtrs puts the shard base pointers into C memory for the call; the shards are pinned
// (runtime.Pinner, Go >= 1.21) so C memory may hold their addresses until unpinned.
func cPtrs(shards [][]byte, pin *runtime.Pinner) (unsafe.Pointer, []unsafe.Pointer) {
	n := len(shards)
	arr := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
	view := unsafe.Slice((*unsafe.Pointer)(arr), n)
	for i, s := range shards {
		if len(s) > 0 {
			pin.Pin(&s[0])
			view[i] = unsafe.Pointer(&s[0])
		} else {
			view[i] = nil
		}
	}
	return arr, view
}

// Encode fills shards[data:] (allocated by the caller, as klauspost requires) with parity.
func (r *rsGPU) Encode(shards [][]byte) error {
	size, err := r.check(shards, false)
	if err != nil {
		return err
	}
	for i := 0; i < r.data+r.parity; i++ {
		if len(shards[i]) != size {
			return ErrShardSize
		}
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	arr, view := cPtrs(shards, &pin)
	defer C.free(arr)
	runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
	defer runtime.UnlockOSThread()
	rc := C.dm_rs_encode(r.h, (*unsafe.Pointer)(unsafe.Pointer(&view[0])), (*unsafe.Pointer)(unsafe.Pointer(&view[r.data])),
		C.uint64_t(size))
	runtime.KeepAlive(shards)
	if rc != C.DM_OK {
		return errors.New(C.GoString(C.dm_last_error(ctx)))
	}
	return nil
}

// Verify reports whether the parity shards match the data shards.
func (r *rsGPU) Verify(shards [][]byte) (bool, error) {
	size, err := r.check(shards, true)
	if err != nil {
		return false, err
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	arr, view := cPtrs(shards, &pin)
	defer C.free(arr)
	var ok C.int
	runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
	defer runtime.UnlockOSThread()
	rc := C.dm_rs_verify(r.h, (*unsafe.Pointer)(unsafe.Pointer(&view[0])), C.uint64_t(size), &ok)
	runtime.KeepAlive(shards)
	if rc != C.DM_OK {
		return false, errors.New(C.GoString(C.dm_last_error(ctx)))
	}
	return ok != 0, nil
}

// Reconstruct rebuilds every missing (nil / empty) shard; it allocates them like klauspost.
func (r *rsGPU) Reconstruct(shards [][]byte) error {
	size, err := r.check(shards, false)
	if err != nil {
		return err
	}
	present := make([]byte, len(shards))
	have := 0
	for i, s := range shards {
		if len(s) > 0 {
			present[i] = 1
			have++
		}
	}
	if have == len(shards) {
		return nil
	}
	if have < r.data {
		return ErrTooFewShards
	}
	for i := range shards {
		if present[i] == 0 {
			shards[i] = make([]byte, size)
		}
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	arr, view := cPtrs(shards, &pin)
	defer C.free(arr)
	cp := C.CBytes(present)
	defer C.free(cp)
	runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
	defer runtime.UnlockOSThread()
	rc := C.dm_rs_reconstruct(r.h, (*unsafe.Pointer)(unsafe.Pointer(&view[0])), (*C.uint8_t)(cp), C.uint64_t(size))
	runtime.KeepAlive(shards)
	if rc != C.DM_OK {
		return errors.New(C.GoString(C.dm_last_error(ctx)))
	}
	return nil
}

// ReconstructData rebuilds the missing data shards (parity shards are rebuilt too).
func (r *rsGPU) ReconstructData(shards [][]byte) error { return r.Reconstruct(shards) }

// Split slices data into equal data shards (the last zero-padded) plus zeroed parity shards.
func (r *rsGPU) Split(data []byte) ([][]byte, error) {
	if len(data) == 0 {
		return nil, ErrShortData
	}
	per := (len(data) + r.data - 1) / r.data
	buf := make([]byte, per*(r.data+r.parity))
	copy(buf, data)
	out := make([][]byte, r.data+r.parity)
	for i := range out {
		out[i] = buf[i*per : (i+1)*per : (i+1)*per]
	}
	return out, nil
}
