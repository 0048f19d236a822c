//go:build !nsx

// Pure-Go twin of checksum_nsx.go for builds without the MI355X library: the
// reference's own loop (tcp.go:73-94), unchanged in behaviour.
package tcp

func checksum16(ipPseudoHeader, seg []byte) uint16 {
	input := append(append([]byte{}, ipPseudoHeader...), seg...)
	if len(input)%2 == 1 {
		input = append(input, byte(0))
	}
	sum := uint16(0)
	for idx := 0; idx < len(input); idx += 2 {
		v := uint16(input[idx])<<8 + uint16(input[idx+1])
		v += sum
		if sum > v {
			v++
		}
		sum = v
	}
	return sum
}
