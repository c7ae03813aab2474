// Times host_walk.h's replay on wide-layer bitsets dumped by
// ULG_DUMP_HOSTWALK=<dir> (hostwalk_<i>_L<L>_p<phase>_q<q>.bin: nw skip words,
// then nw hi words): decision, iterations, neighbour reads and ns per
// iteration, best of R runs (each on a fresh copy of skip).
//
//   g++ -O2 -march=native -std=c++17 -I urlearning-cpp_amd/csrc -o /tmp/hwb scripts/host_walk_bench.cpp
//   /tmp/hwb gpurun_out/hw/hostwalk_*.bin
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "host_walk.h"

int main(int argc, char **argv) {
    double tot_ns = 0, tot_it = 0;
    for (int i = 1; i < argc; ++i) {
        int idx, L, ph, q;
        const char *b = std::strrchr(argv[i], '/');
        b = b ? b + 1 : argv[i];
        if (std::sscanf(b, "hostwalk_%d_L%d_p%d_q%d.bin", &idx, &L, &ph, &q) != 4) continue;
        const size_t nw = ((size_t)1 << q) >> 6;
        std::vector<uint64_t> bits(2 * nw);
        FILE *f = std::fopen(argv[i], "rb");
        if (!f) continue;
        const size_t got = std::fread(bits.data(), 8, 2 * nw, f);
        std::fclose(f);
        if (got != 2 * nw) continue;
        double best = 1e30;
        uint64_t it = 0, nc = 0;
        bool dom = false, err = false;
        for (int r = 0; r < 5; ++r) {
            std::vector<uint64_t> skip(bits.begin(), bits.begin() + nw);
            const auto t0 = std::chrono::steady_clock::now();
            dom = ulg::host_walk(L, ph, skip.data(), bits.data() + nw, &err, &it, &nc);
            const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
            if (ns < best) best = ns;
        }
        tot_ns += best;
        tot_it += (double)it;
        std::printf("%-28s q=%2d %s iters=%7llu nbr=%7llu %.1f ns/iter%s\n", b, q, dom ? "hit  " : "store",
                    (unsigned long long)it, (unsigned long long)nc, best / (double)it, err ? " ERR" : "");
    }
    std::printf("total %.0f iterations, %.1f ns/iter\n", tot_it, tot_ns / tot_it);
    return 0;
}
