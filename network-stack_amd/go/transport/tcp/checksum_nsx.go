//go:build nsx

// cgo binding of transport/tcp's checksum to the MI355X library
// (include/nsx_csum.h). Drop this file into transport/tcp/ of
// oneee-playground/network-stack and build with `-tags nsx`; see INTEGRATION.md.
//
// checksum16 keeps computeChecksum's exact semantics (tcp.go:72-95): raw
// one's-complement sum over ipPseudoHeader ‖ segment, odd tail zero-padded,
// never fails. It runs on the host CPU (nsx_csum16): one cgo call per segment
// must not drive the GPU. Batches go through ChecksumSegments (batch_nsx.go).
package tcp

/*
#cgo LDFLAGS: -lnsx_csum
#include "nsx_csum.h"
*/
import "C"

import (
	"fmt"
	"unsafe"
)

func bytesPtr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// checksum16 is the body of segment.computeChecksum (tcp.go:72-95) without the
// append(ipPseudoHeader, s.bytes()...) concatenation (tcp.go:73): the C ABI
// takes the two spans separately, so the caller's backing array is never
// written. Go memory is only read for the duration of the call (cgo rules).
func checksum16(ipPseudoHeader, seg []byte) uint16 {
	var sum C.uint16_t
	rc := C.nsx_csum16(bytesPtr(ipPseudoHeader), C.size_t(len(ipPseudoHeader)),
		bytesPtr(seg), C.size_t(len(seg)), &sum)
	if rc != C.NSX_OK {
		// computeChecksum has no error path; nsx_csum16 only fails on nil
		// pointers with nonzero lengths, which Go slices cannot produce.
		panic(fmt.Sprintf("nsx_csum16: %s", C.GoString(C.nsx_strerror(rc))))
	}
	return uint16(sum)
}
