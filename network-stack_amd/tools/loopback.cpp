// nsx_loopback — config 1 of BASELINE.json ("64×1500 B TCP segments over
// transport/pipe loopback") and the f4 feed: a sender thread
// serialises TCP segments with the nsx::tcp mirror (checksum field = ~raw over
// the IPv4 pseudo-header, tcp.go:68-71), writes them through an nsx::pipe
// loopback (transport/pipe/pipe.go semantics); the receiver frames exactly
// seg_len bytes per segment (io.ReadFull) and verifies every checksum:
//   --mode host   per-segment nsx_csum16 on arrival (computeChecksum's path)
//   --mode batch  frames land in pinned memory; one nsx_csum_fixed_host call
//                 (GPU) verifies the whole batch — the transport feeding batches.
// Prints one JSON line.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "nsx/pipe.hpp"
#include "nsx/tcp.hpp"

int main(int argc, char** argv) {
    int nseg = 64, seg_len = 1500, reps = 200, corrupt = -1;
    std::string mode = "host";
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        if (k == "--segments") nseg = std::atoi(argv[i + 1]);
        else if (k == "--seg-len") seg_len = std::atoi(argv[i + 1]);
        else if (k == "--reps") reps = std::atoi(argv[i + 1]);
        else if (k == "--mode") mode = argv[i + 1];
        else if (k == "--corrupt") corrupt = std::atoi(argv[i + 1]);  // flip a bit of segment K in transit
    }
    if (seg_len < 20 || corrupt >= nseg || nseg < 1 || reps < 1 || (mode != "host" && mode != "batch")) {
        std::fprintf(stderr, "usage: nsx_loopback [--segments N] [--seg-len L>=20] [--reps R] [--mode host|batch]\n");
        return 2;
    }
    // Build the segments once (sender side of tcp.go: field zero, sum, store ~sum).
    std::mt19937_64 rng(0x1071);
    std::vector<std::vector<uint8_t>> wire(nseg), pseudo(nseg);
    std::vector<uint32_t> partial(nseg);
    for (int i = 0; i < nseg; ++i) {
        nsx::tcp::Segment s;
        s.src_port = (uint16_t)rng();
        s.dst_port = 443;
        s.seq_num = (uint32_t)rng();
        s.ack_num = (uint32_t)rng();
        s.control.ack = true;
        s.window = 65535;
        s.data.resize(seg_len - 20);
        for (auto& b : s.data) b = (uint8_t)rng();
        s.offset = s.compute_offset();
        const uint8_t src[4] = {10, 0, 0, 1}, dst[4] = {10, 0, 0, 2};
        pseudo[i] = nsx::tcp::ipv4_pseudo_header(src, dst, 6, (uint16_t)seg_len);
        for (size_t k = 0; k + 1 < pseudo[i].size(); k += 2) partial[i] += (uint32_t)pseudo[i][k] << 8 | pseudo[i][k + 1];
        s.checksum = nsx_field(s.compute_checksum(pseudo[i]));
        wire[i] = s.bytes();
    }
    uint8_t* frames = nullptr;
    if (mode == "batch") {
        void* p = nullptr;
        const int rc = nsx_alloc_pinned((size_t)nseg * seg_len, &p);
        if (rc != NSX_OK) {
            std::printf("{\"error\": \"%s\"}\n", nsx_strerror(rc));
            return 1;
        }
        frames = static_cast<uint8_t*>(p);
    }
    std::vector<uint8_t> frame(seg_len);
    std::vector<uint16_t> raw(nseg);
    long bad = 0;
    double best = 1e30, total = 0;
    for (int r = 0; r < reps; ++r) {
        auto ends = nsx::pipe::make_pipe("client", "server");
        nsx::pipe::End& c1 = ends.first;
        nsx::pipe::End& c2 = ends.second;
        const auto t0 = std::chrono::steady_clock::now();
        std::thread writer([&] {
            for (int i = 0; i < nseg; ++i) {
                size_t n = 0;
                if (c1.write(wire[i].data(), wire[i].size(), &n) != nsx::pipe::Err::kOk) return;
            }
        });
        for (int i = 0; i < nseg; ++i) {
            uint8_t* dst = frames ? frames + (size_t)i * seg_len : frame.data();
            if (c2.read_full(dst, seg_len) != nsx::pipe::Err::kOk) { ++bad; break; }
            if (i == corrupt) dst[seg_len / 2] ^= 0x10;
            if (!frames) {
                uint16_t sum = 0;
                nsx_csum16(pseudo[i].data(), pseudo[i].size(), dst, seg_len, &sum);
                if (!nsx_verify(sum)) ++bad;
            }
        }
        if (frames) {
            const int rc = nsx_csum_fixed_host(frames, seg_len, seg_len, nseg, partial.data(), raw.data(), 1);
            if (rc != NSX_OK) {
                std::printf("{\"error\": \"%s\"}\n", nsx_strerror(rc));
                return 1;
            }
            for (int i = 0; i < nseg; ++i) bad += !nsx_verify(raw[i]);
        }
        writer.join();
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        best = dt < best ? dt : best;
        total += dt;
    }
    if (frames) nsx_free_pinned(frames);
    const double bytes = (double)nseg * seg_len;
    std::printf("{\"config\": \"config1: %d x %dB TCP segments over nsx::pipe loopback\", \"mode\": \"%s\", "
                "\"reps\": %d, \"bad\": %ld, \"corrupt\": %d, \"best_us_per_batch\": %.2f, \"mean_us_per_batch\": %.2f, "
                "\"us_per_segment\": %.3f, \"MB_per_s_best\": %.1f}\n",
                nseg, seg_len, mode.c_str(), reps, bad, corrupt, best * 1e6, total / reps * 1e6, best * 1e6 / nseg,
                bytes / best / 1e6);
    return bad == (corrupt >= 0 ? reps : 0) ? 0 : 1;
}
