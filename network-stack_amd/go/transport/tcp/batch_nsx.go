//go:build nsx

// Batch entry points over the MI355X library: many segments per cgo call,
// checksummed on the GPU(s). Segments are densely packed into one pinned
// (DMA-registered) C buffer — Go heap memory is not DMA-registered and C may
// not retain Go pointers — and handed to nsx_csum_ragged_host, which shards
// them over the node's GPUs (no collective) and pipelines H2D → kernel → D2H.
package tcp

/*
#include "nsx_csum.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"
)

// PinnedBatch is a reusable pinned staging area for segment bytes. A transport
// can serialize segments straight into Bytes() (unsafe.Slice over C memory)
// and avoid a copy.
type PinnedBatch struct {
	base    unsafe.Pointer
	buf     []byte
	offsets []uint64
}

// NewPinnedBatch allocates capacity bytes of pinned host memory.
func NewPinnedBatch(capacity int) (*PinnedBatch, error) {
	var p unsafe.Pointer
	if rc := C.nsx_alloc_pinned(C.size_t(capacity), &p); rc != C.NSX_OK {
		return nil, fmt.Errorf("nsx_alloc_pinned: %s", C.GoString(C.nsx_strerror(rc)))
	}
	return &PinnedBatch{base: p, buf: unsafe.Slice((*byte)(p), capacity), offsets: []uint64{0}}, nil
}

// Append copies one serialized segment (e.g. segment.bytes(), tcp.go:98-128)
// into the batch.
func (b *PinnedBatch) Append(seg []byte) error {
	at := b.offsets[len(b.offsets)-1]
	if at+uint64(len(seg)) > uint64(len(b.buf)) {
		return errors.New("pinned batch full")
	}
	copy(b.buf[at:], seg)
	b.offsets = append(b.offsets, at+uint64(len(seg)))
	return nil
}

// Reset empties the batch for reuse.
func (b *PinnedBatch) Reset() { b.offsets = b.offsets[:1] }

// Free releases the pinned memory.
func (b *PinnedBatch) Free() {
	if b.base != nil {
		C.nsx_free_pinned(b.base)
		b.base, b.buf = nil, nil
	}
}

// pseudoPartial is the integer sum of a pseudo-header's big-endian 16-bit
// words (the d_prefix_partial convention of nsx_csum.h); pseudo-headers have
// even length (12 B IPv4, 40 B IPv6).
func pseudoPartial(ph []byte) uint32 {
	var s uint32
	for i := 0; i+1 < len(ph); i += 2 {
		s += uint32(ph[i])<<8 | uint32(ph[i+1])
	}
	return s
}

// Checksum returns the raw sum of every segment in the batch, each over
// pseudo[i] ‖ segment i when pseudo is non-nil (len(pseudo) == segments):
// the batch form of computeChecksum (tcp.go:72-95). numGPUs 0 = auto: one GPU
// per 64 MiB of batch, up to all visible (nsx_csum.h, host-resident batches).
func (b *PinnedBatch) Checksum(pseudo [][]byte, numGPUs int) ([]uint16, error) {
	n := len(b.offsets) - 1
	out := make([]uint16, n)
	if n == 0 {
		return out, nil
	}
	var partial *C.uint32_t
	if pseudo != nil {
		if len(pseudo) != n {
			return nil, errors.New("pseudo-header count != segment count")
		}
		parts := make([]uint32, n)
		for i, ph := range pseudo {
			if len(ph)%2 != 0 {
				return nil, errors.New("pseudo-header of odd length")
			}
			parts[i] = pseudoPartial(ph)
		}
		partial = (*C.uint32_t)(unsafe.Pointer(&parts[0]))
	}
	rc := C.nsx_csum_ragged_host((*C.uint8_t)(b.base), (*C.uint64_t)(unsafe.Pointer(&b.offsets[0])), C.uint64_t(n),
		partial, (*C.uint16_t)(unsafe.Pointer(&out[0])), C.int(numGPUs))
	if rc != C.NSX_OK {
		return nil, fmt.Errorf("nsx_csum_ragged_host: %s", C.GoString(C.nsx_strerror(rc)))
	}
	return out, nil
}

// ChecksumSegments checksums segs (each already serialized) on the GPU(s).
func ChecksumSegments(segs [][]byte, pseudo [][]byte, numGPUs int) ([]uint16, error) {
	total := 0
	for _, s := range segs {
		total += len(s)
	}
	b, err := NewPinnedBatch(total + 1)
	if err != nil {
		return nil, err
	}
	defer b.Free()
	for _, s := range segs {
		if err := b.Append(s); err != nil {
			return nil, err
		}
	}
	return b.Checksum(pseudo, numGPUs)
}
