//go:build hip

// Drop-in replacement for DeOSS common/hashtree/hashtree.go (reference lines 18-35) when built
// with `-tags hip` and CGO_ENABLED=1.  The leaf digest is computed by the MI355X library
// (include/deoss_merkle.h) and carried inside the content, so merkletree's CalculateHash calls
// return it instead of re-hashing the chunk on the CPU.
package hashtree

import (
	"bytes"
	"crypto/sha256"

	"github.com/cbergoon/merkletree"
)

// HashTreeContent implements the Content interface provided by merkletree
// and represents the content stored in the tree.
type HashTreeContent struct {
	x      string // chunk bytes (kept only when the caller asked for them)
	digest []byte // SHA-256(x) from the GPU leaf kernel
}

// CalculateHash returns the GPU leaf digest; without one it hashes x like the reference.
func (t HashTreeContent) CalculateHash() ([]byte, error) {
	if t.digest != nil {
		return append([]byte(nil), t.digest...), nil
	}
	h := sha256.New()
	if _, err := h.Write([]byte(t.x)); err != nil {
		return nil, err
	}
	return h.Sum(nil), nil
}

// Equals compares contents when both are held, digests otherwise (documented deviation:
// the reference compares x only, common/hashtree/hashtree.go:33-35).
func (t HashTreeContent) Equals(other merkletree.Content) (bool, error) {
	o := other.(HashTreeContent)
	if t.digest == nil || o.digest == nil {
		return t.x == o.x, nil
	}
	return bytes.Equal(t.digest, o.digest), nil
}
