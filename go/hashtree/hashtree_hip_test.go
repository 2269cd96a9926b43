//go:build hip

package hashtree

import (
	"crypto/sha256"
	"encoding/hex"
	"os"
	"path/filepath"
	"testing"

	"github.com/stretchr/testify/assert"
)

// Same assertions as the reference common/hashtree/hashtree_test.go:20-82, through the GPU.
func TestNewHashTreeGPU(t *testing.T) {
	contents := []string{"content_one", "content_two", "content_three", "content_four"}
	var hashes [][32]byte
	dir := t.TempDir()
	var chunks []string
	for _, c := range contents {
		hashes = append(hashes, sha256.Sum256([]byte(c)))
		p := filepath.Join(dir, c)
		assert.NoError(t, os.WriteFile(p, []byte(c), 0o644))
		chunks = append(chunks, p)
	}
	five := sha256.Sum256(append(hashes[0][:], hashes[1][:]...))
	six := sha256.Sum256(append(hashes[2][:], hashes[3][:]...))
	root := sha256.Sum256(append(five[:], six[:]...))

	mtree, err := NewHashTree(chunks)
	assert.NoError(t, err)
	assert.Equal(t, 4, len(mtree.Leafs))
	for i := range contents {
		assert.Equal(t, hex.EncodeToString(hashes[i][:]), hex.EncodeToString(mtree.Leafs[i].Hash))
	}
	assert.Equal(t, "b513419286835c1e36fa520b86cbf37650db82e73f510f0e6a699cc0505f1151", hex.EncodeToString(mtree.MerkleRoot()))
	assert.Equal(t, hex.EncodeToString(root[:]), hex.EncodeToString(mtree.MerkleRoot()))

	_, err = NewHashTree(nil)
	assert.EqualError(t, err, "Empty data")
}
