//go:build nsx

// Receive-side batch verification over the MI355X library: received IPv4
// datagrams (or IPv6 packets) carrying TCP are packed into pinned staging and
// checked in one GPU pass (nsx_rx_ipv4_tcp_verify_host /
// nsx_rx_ipv6_tcp_verify_host): the IPv4 header checksum, the pseudo-header
// built from the header's own addresses (ip.Addr.Raw(), network/ip/v4/ipv4.go:15,
// network/ip/v6/ipv6.go:16; ip.NextProtoTCP, network/ip/protocols.go:8), and
// computeChecksum(pseudo) == 0xFFFF over the segment (tcp.go:70, :72-95).
package tcp

/*
#include "nsx_csum.h"
*/
import "C"

import (
	"fmt"
	"unsafe"
)

// Verify reports, per frame appended to the batch, whether it is a well-formed
// unfragmented IPv4 datagram (ipver 4) or IPv6 packet (ipver 6) carrying a TCP
// segment of at least minSegmentLength bytes (tcp.go:131) whose checksums
// verify. A receive loop keeps one PinnedBatch and, per batch of frames read
// from its socket or pipe, Resets, Appends and Verifies: its pinned block is
// reused. numGPUs 0 = auto (nsx_csum.h, host-resident batches).
func (b *PinnedBatch) Verify(ipver int, numGPUs int) ([]bool, error) {
	n := b.Len()
	ok := make([]bool, n)
	if n == 0 {
		return ok, nil
	}
	w := (n + 63) / 64
	if cap(b.mask) < w {
		b.mask = make([]uint64, w)
	}
	b.mask = b.mask[:w]
	base, offs := (*C.uint8_t)(b.arena.base), (*C.uint64_t)(unsafe.Pointer(&b.offsets[0]))
	words := (*C.uint64_t)(unsafe.Pointer(&b.mask[0]))
	var rc C.int
	switch ipver {
	case 4:
		rc = C.nsx_rx_ipv4_tcp_verify_host(base, offs, C.uint64_t(n), words, C.int(numGPUs))
	case 6:
		rc = C.nsx_rx_ipv6_tcp_verify_host(base, offs, C.uint64_t(n), words, C.int(numGPUs))
	default:
		return nil, fmt.Errorf("ipver %d: 4 or 6", ipver)
	}
	if rc != C.NSX_OK {
		return nil, fmt.Errorf("nsx_rx_ipv%d_tcp_verify_host: %s", ipver, C.GoString(C.nsx_strerror(rc)))
	}
	for i := range ok {
		ok[i] = b.mask[i/64]>>(uint(i)%64)&1 == 1
	}
	return ok, nil
}

// VerifyDatagrams reports, per received datagram, whether it is a well-formed
// unfragmented IPv4 datagram carrying a TCP segment of at least
// minSegmentLength bytes (tcp.go:131) whose header and TCP checksums both
// verify: the one-shot form of PinnedBatch.Verify (pins a block for this call
// only). numGPUs 0 = auto: one GPU per 64 MiB of batch, up to all visible.
func VerifyDatagrams(frames [][]byte, numGPUs int) ([]bool, error) {
	return verifyFrames(frames, numGPUs, 4)
}

// VerifyPackets6 is VerifyDatagrams for IPv6 packets whose fixed header is
// followed directly by TCP (Next Header 6): the TCP checksum over the RFC 8200
// pseudo-header must verify (IPv6 has no header checksum).
func VerifyPackets6(frames [][]byte, numGPUs int) ([]bool, error) {
	return verifyFrames(frames, numGPUs, 6)
}

func verifyFrames(frames [][]byte, numGPUs int, ipver int) ([]bool, error) {
	total := 0
	for _, f := range frames {
		total += len(f)
	}
	b, err := NewPinnedBatch(total + 1)
	if err != nil {
		return nil, err
	}
	defer b.Free()
	for _, f := range frames {
		if err := b.Append(f); err != nil {
			return nil, err
		}
	}
	return b.Verify(ipver, numGPUs)
}
