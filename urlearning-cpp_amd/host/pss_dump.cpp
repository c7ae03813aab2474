// pss_dump -- prints what the drop-in .pss reader (io.cpp read_pss, the
// parallel restatement of ScoreCache::read, score_cache.cpp:55-160) loads:
//   names <name_0> ... <name_{n-1}>
//   <variable> <parent set as u64> <cost as float bits, hex>
// one line per stored entry, variables in order.  Used by the CPU tests to
// check the reader against the oracle's sequential one on quirky files.
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <string>

#include "io.h"

int main(int argc, char **argv) {
    if (argc != 2) {
        std::fprintf(stderr, "usage: pss_dump file.pss\n");
        return 2;
    }
    ulgio::PssData p;
    std::string err;
    if (!ulgio::read_pss(argv[1], p, err)) {
        std::fprintf(stderr, "pss_dump: %s\n", err.c_str());
        return 1;
    }
    std::printf("names");
    for (const std::string &s : p.names) std::printf(" %s", s.c_str());
    std::printf("\n");
    const int n = (int)p.names.size();
    for (int v = 0; v < n; ++v)
        for (int64_t i = p.offsets[v]; i < p.offsets[v + 1]; ++i) {
            uint32_t bits;
            std::memcpy(&bits, &p.costs[i], 4);
            std::printf("%d %" PRIu64 " %08x\n", v, p.sets[i], bits);
        }
    return 0;
}
