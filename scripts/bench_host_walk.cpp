// Times host_walk (urlearning-cpp_amd/csrc/host_walk.h) on bitsets dumped by
// a wide-layer scoring call (ULG_DUMP_HOSTWALK=dir: hostwalk_<i>_L<L>_p<ph>_q<q>.bin,
// the skip words then the hi words of one handed-over replay).  CPU only.
//   g++ -O2 -std=c++17 -Iurlearning-cpp_amd/csrc scripts/bench_host_walk.cpp -o scripts/bin/bench_host_walk
//   scripts/bin/bench_host_walk dir/hostwalk_*.bin
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "host_walk.h"

int main(int argc, char **argv) {
    double total = 0.0;
    for (int a = 1; a < argc; ++a) {
        const std::string fn = argv[a];
        int idx, L, ph, q;
        const char *base = std::strrchr(fn.c_str(), '/');
        base = base ? base + 1 : fn.c_str();
        if (std::sscanf(base, "hostwalk_%d_L%d_p%d_q%d.bin", &idx, &L, &ph, &q) != 4) continue;
        const size_t nw = ((size_t)1 << q) >> 6;
        std::vector<uint64_t> buf(2 * nw);
        FILE *f = std::fopen(fn.c_str(), "rb");
        if (!f || std::fread(buf.data(), 8, buf.size(), f) != buf.size()) { std::fprintf(stderr, "bad %s\n", base); return 1; }
        std::fclose(f);
        std::vector<uint64_t> skip(nw);
        double best = 1e9;
        bool dom = false, err = false;
        for (int r = 0; r < 20; ++r) {
            std::memcpy(skip.data(), buf.data(), nw * 8);
            const auto t0 = std::chrono::steady_clock::now();
            dom = ulg::host_walk(L, ph, skip.data(), buf.data() + nw, &err);
            best = std::min(best, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        uint64_t its = 0, nc = 0;
        std::memcpy(skip.data(), buf.data(), nw * 8);
        (void)ulg::host_walk(L, ph, skip.data(), buf.data() + nw, &err, &its, &nc);
        std::printf("%-40s L=%2d ph=%d q=%2d dom=%d err=%d best_us=%.1f iters=%llu nbr=%llu ns/iter=%.1f\n", base, L, ph,
                    q, (int)dom, (int)err, best, (unsigned long long)its, (unsigned long long)nc, best * 1e3 / (double)its);
        total += best;
    }
    std::printf("total_us %.1f\n", total);
    return 0;
}
