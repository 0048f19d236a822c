// Reads a segment blob and its offsets (argv[1] blob, argv[2] text file of n+1 offsets), parses every segment
// with the C++ mirror's parse_segment (network-stack_amd/include/nsx/tcp.hpp, tcp.go:130-185) and prints one
// line per segment: status src dst seq ack offset control window checksum urgent data_off n_options, the
// status numbered as nsx_tcp_parse_dev's (0 ok, 1 short, 2 offset, 3 option range, 4 option kind).
#include <cstdio>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "nsx/tcp.hpp"

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    std::ifstream fb(argv[1], std::ios::binary);
    const std::vector<uint8_t> blob((std::istreambuf_iterator<char>(fb)), std::istreambuf_iterator<char>());
    std::ifstream fo(argv[2]);
    std::vector<unsigned long long> offs;
    for (unsigned long long v; fo >> v;) offs.push_back(v);
    for (size_t i = 0; i + 1 < offs.size(); ++i) {
        const std::vector<uint8_t> raw(blob.begin() + (long)offs[i], blob.begin() + (long)offs[i + 1]);
        nsx::tcp::Segment s;
        std::string err;
        int status = 0;
        if (!nsx::tcp::parse_segment(raw, s, err)) {
            status = err == "segment too short" ? 1 : err == "advertised data offset too long" ? 2
                     : err == "option out of range" ? 3 : err == "unknown option kind" ? 4 : 9;
            s = nsx::tcp::Segment{};
        }
        const unsigned long long data_off = status ? 0ull : offs[i] + (unsigned long long)s.offset * 4u;
        std::printf("%d %u %u %u %u %u %u %u %u %u %llu %zu\n", status, s.src_port, s.dst_port, s.seq_num,
                    s.ack_num, s.offset, s.control.byte(), s.window, s.checksum, s.urgent_ptr, data_off,
                    s.options.size());
    }
    return 0;
}
