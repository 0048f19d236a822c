//go:build nsx

// Sender-side batch build over the MI355X library (SURVEY.md §8 f1). A Go
// transport's send loop — per segment bytes() (tcp.go:98-128), the checksum
// over its ipPseudoHeader (tcp.go:72-95) stored as ^sum in bytes 16-17
// (tcp.go:110, :68-71), then Write into the pipe or socket
// (transport/pipe/pipe.go:92-124) — becomes one nsx_tcp_build_host call: the
// segments' header fields, serialised options, payloads and pseudo-header
// partials are staged in one pinned (DMA-registered) block, the GPU(s) build
// every wire image, and the images come back into the same block, ready to be
// written. C never retains a Go pointer: everything the call reads is in the
// pinned block except the raw-sum slice it fills during the call.
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

// BuiltSegments holds a batch's wire images in pinned host memory.
type BuiltSegments struct {
	base   unsafe.Pointer
	block  []byte
	out    []byte
	outOff []uint64
	wire   []int
	// Raw is the raw sum of each image taken with its checksum field zero; the
	// field holds ^Raw[i], so a receiver re-summing pseudo[i] ‖ image gets
	// 0xFFFF (tcp.go:70).
	Raw []uint16
}

// Len returns the number of segments in the batch.
func (b *BuiltSegments) Len() int { return len(b.wire) }

// Image returns segment i's wire image: a view into pinned memory, valid until
// Free, byte for byte what s.bytes() returns after s.checksum = ^Raw[i].
func (b *BuiltSegments) Image(i int) []byte {
	o := b.outOff[i]
	return b.out[o : o+uint64(b.wire[i])]
}

// Free releases the pinned memory.
func (b *BuiltSegments) Free() {
	if b.base != nil {
		C.nsx_free_pinned(b.base)
		b.base, b.block, b.out = nil, nil, nil
	}
}

func alignUp(x, a uint64) uint64 { return (x + a - 1) &^ (a - 1) }

// BuildSegments builds the wire images of segs on the GPU(s). Each segment's
// header fields are used as they are — offset included, as bytes() expects
// (tcp.go:97); s.checksum is ignored, the sum being taken with the field zero
// as the sender must (tcp.go:68) — and its options are serialised by
// option.bytes() (tcp.go:225-231) and padded as bytes() pads them
// (tcp.go:118-121). pseudo[i] is segment i's ipPseudoHeader (even length), or
// pseudo is nil for none. numGPUs 0 = auto: one GPU per 64 MiB of images, up
// to all visible (nsx_csum.h, host-resident batches).
func BuildSegments(segs []segment, pseudo [][]byte, numGPUs int) (*BuiltSegments, error) {
	n := len(segs)
	if pseudo != nil && len(pseudo) != n {
		return nil, errors.New("pseudo-header count != segment count")
	}
	b := &BuiltSegments{outOff: make([]uint64, n+1), wire: make([]int, n), Raw: make([]uint16, n)}
	if n == 0 {
		return b, nil
	}
	// sizes: serialised options, payloads, 4-aligned image slots (nsx_tcp_layout_host's rule)
	optLen := make([]uint64, n)
	var nOpt, nData uint64
	for i, s := range segs {
		if pseudo != nil && len(pseudo[i])%2 != 0 {
			return nil, errors.New("pseudo-header of odd length")
		}
		for _, op := range s.options {
			optLen[i] += uint64(len(op.bytes()))
		}
		nOpt += optLen[i]
		nData += uint64(len(s.data))
		b.wire[i] = int(C.nsx_tcp_wire_len(C.uint64_t(optLen[i]), C.uint64_t(len(s.data))))
		b.outOff[i+1] = b.outOff[i] + alignUp(uint64(b.wire[i]), 4)
	}
	nOut := b.outOff[n]
	un := uint64(n)
	// one pinned block: the 8 header field arrays (nsx_tcp_hdr_soa order below), data/opt/out offsets,
	// partials, option bytes, payload bytes, images
	sizes := []uint64{2 * un, 2 * un, 4 * un, 4 * un, un, un, 2 * un, 2 * un,
		8 * (un + 1), 8 * (un + 1), 8 * (un + 1), 4 * un, nOpt + 1, nData + 1, nOut}
	at := make([]uint64, len(sizes)+1)
	for k, sz := range sizes {
		at[k+1] = alignUp(at[k]+sz, 64)
	}
	var p unsafe.Pointer
	if rc := C.nsx_alloc_pinned(C.size_t(at[len(sizes)]), &p); rc != C.NSX_OK {
		return nil, fmt.Errorf("nsx_alloc_pinned: %s", C.GoString(C.nsx_strerror(rc)))
	}
	b.base = p
	b.block = unsafe.Slice((*byte)(p), at[len(sizes)])
	region := func(k int) unsafe.Pointer { return unsafe.Pointer(&b.block[at[k]]) }
	srcPort := unsafe.Slice((*uint16)(region(0)), n)
	dstPort := unsafe.Slice((*uint16)(region(1)), n)
	seqNum := unsafe.Slice((*uint32)(region(2)), n)
	ackNum := unsafe.Slice((*uint32)(region(3)), n)
	offset := unsafe.Slice((*uint8)(region(4)), n)
	control := unsafe.Slice((*uint8)(region(5)), n)
	window := unsafe.Slice((*uint16)(region(6)), n)
	urgentPtr := unsafe.Slice((*uint16)(region(7)), n)
	dataOff := unsafe.Slice((*uint64)(region(8)), n+1)
	optOff := unsafe.Slice((*uint64)(region(9)), n+1)
	outOff := unsafe.Slice((*uint64)(region(10)), n+1)
	parts := unsafe.Slice((*uint32)(region(11)), n)
	opts := unsafe.Slice((*byte)(region(12)), nOpt+1)
	data := unsafe.Slice((*byte)(region(13)), nData+1)
	b.out = unsafe.Slice((*byte)(region(14)), nOut)
	var d, o uint64
	for i, s := range segs {
		srcPort[i], dstPort[i], seqNum[i], ackNum[i] = s.srcPort, s.dstPort, s.seqNum, s.ackNum
		offset[i], control[i], window[i], urgentPtr[i] = s.offset, s.control.byte(), s.window, s.urgentPtr
		dataOff[i], optOff[i], outOff[i] = d, o, b.outOff[i]
		for _, op := range s.options {
			o += uint64(copy(opts[o:], op.bytes()))
		}
		d += uint64(copy(data[d:], s.data))
		if pseudo != nil {
			parts[i] = pseudoPartial(pseudo[i])
		}
	}
	dataOff[n], optOff[n], outOff[n] = d, o, nOut

	var h C.nsx_tcp_hdr_soa
	h.src_port = (*C.uint16_t)(region(0))
	h.dst_port = (*C.uint16_t)(region(1))
	h.seq_num = (*C.uint32_t)(region(2))
	h.ack_num = (*C.uint32_t)(region(3))
	h.offset = (*C.uint8_t)(region(4))
	h.control = (*C.uint8_t)(region(5))
	h.window = (*C.uint16_t)(region(6))
	h.urgent_ptr = (*C.uint16_t)(region(7))
	var partial *C.uint32_t
	if pseudo != nil {
		partial = (*C.uint32_t)(region(11))
	}
	var optOffs *C.uint64_t
	if nOpt > 0 {
		optOffs = (*C.uint64_t)(region(9))
	}
	rc := C.nsx_tcp_build_host(&h, (*C.uint8_t)(region(12)), optOffs, (*C.uint8_t)(region(13)),
		(*C.uint64_t)(region(8)), partial, C.uint64_t(n), (*C.uint8_t)(region(14)), (*C.uint64_t)(region(10)),
		(*C.uint16_t)(unsafe.Pointer(&b.Raw[0])), C.int(numGPUs))
	if rc != C.NSX_OK {
		b.Free()
		return nil, fmt.Errorf("nsx_tcp_build_host: %s", C.GoString(C.nsx_strerror(rc)))
	}
	return b, nil
}
