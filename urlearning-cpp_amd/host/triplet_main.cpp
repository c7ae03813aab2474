// triplet_astar -- the reference's triplet_astar command line
// (astar/triplet_astar.cpp:1624-1687, driver :991-1622) on the MI355X path:
// the .pss score cache is read on the host, the best-score lattice and every
// cluster's static pattern database are built on the GPU, and ulg_triplet_astar
// runs the orientation driver with one exact-order A* per distinct cluster.
//
//   triplet_astar <in.pss> [-k skeleton] [-n netFile] [-a 2]
//
// As in the reference, netFile is created empty (its network write-out is
// commented out) and netFile.csv receives the MEC matrix directed_graph
// ((i,j) = 1 iff i -> j; both set = undirected) (:1601-1613).
// Post-processing flags (-f/-i/-l/-w/--adaptive) are accepted and unused, as
// in the reference's driver.
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/ulg.h"
#include "cli_common.h"
#include "io.h"

int main(int argc, char **argv) {
    ulgcli::Args args(
        {
            {"k", "skeleton", true, "", "The file containing the edges of a skeleton"},
            {"f", "scoring_function", true, "", "The scoring function to use in post-processing (unused)"},
            {"i", "raw_inputFile", true, "", "The raw data file (unused)"},
            {"l", "lambda", true, "", "The lambda in Lasso (unused)"},
            {"", "adaptive", false, "", "Use adaptive Lasso (unused)"},
            {"w", "scoreType", true, "1", "Score type (unused)"},
            {"b", "bestScore", true, "list", "BestScore calculator: list, bitwise or tree"},
            {"e", "heuristic", true, "static", "Heuristic type: static"},
            {"a", "argument", true, "2", "Number of static pattern databases"},
            {"p", "pc_{i-1}", true, "", "Ancestor-only variables (unsupported)"},
            {"s", "scc_i", true, "", "Variables to add in the search (unsupported)"},
            {"r", "runningTime", true, "0", "The maximum running time for the algorithm.  0 means no running time."},
            {"n", "netFile", true, "", "The file to which the learned network is written."},
            {"", "device", true, "0", "HIP device to use."},
            {"h", "help", false, "", "Show this help message."},
        },
        {"scoreFile"});
    std::string err;
    if (!args.parse(argc, argv, err)) {
        std::fprintf(stderr, "triplet_astar: %s\n", err.c_str());
        return 2;
    }
    if (args.has("help") || argc == 1 || !args.has("scoreFile")) {
        args.usage(argv[0], "Learn a Markov equivalence class with triplet A* on an MI355X.  Example usage: triplet_astar iris.pss");
        return args.has("help") || argc == 1 ? 0 : 2;
    }
    // -r: the reference's watchdog over the whole driver (triplet_astar.cpp:
    // 1674-1681); after it fires every A* ends without a goal (:139-142,355),
    // so the MEC written depends on the clock, as in the reference
    const int running_time = std::atoi(args.get("runningTime").c_str());
    if (running_time > 0) std::printf("Maximum running time: %d\n", running_time);
    std::string bs = args.get("bestScore");
    if (bs != "list" && bs != "bitwise" && bs != "tree") {
        std::fprintf(stderr, "triplet_astar: Invalid BestScore calculator type: '%s'\n", bs.c_str());
        return 2;
    }
    if (args.get("heuristic") != "static") {
        std::fprintf(stderr, "triplet_astar: only the static pattern database heuristic is on this path\n");
        return 2;
    }
    if (!args.get("pc_{i-1}").empty() || !args.get("scc_i").empty()) {
        std::fprintf(stderr, "triplet_astar: -p/-s (ancestor / scc subsets) are not supported on this path\n");
        return 2;
    }
    const int pd = std::atoi(args.get("argument").c_str());
    ulgio::PssData p;
    const double t0 = ulgcli::now_s();
    if (!ulgio::read_pss(args.get("scoreFile"), p, err)) {
        std::fprintf(stderr, "triplet_astar: %s\n", err.c_str());
        return 1;
    }
    const int n = (int)p.names.size();
    if (n < 1) {
        std::fprintf(stderr, "triplet_astar: no variables in '%s'\n", args.get("scoreFile").c_str());
        return 1;
    }
    std::vector<uint64_t> rows;
    bool good = false;
    const std::string skel = args.get("skeleton");
    if (!skel.empty()) {
        int nv = 0;
        good = ulgio::read_skeleton(skel, n, rows, nv);
        if (good) rows.resize(std::max<size_t>(rows.size(), (size_t)n));
    }
    const double tr = ulgcli::now_s();
    const int dev = std::atoi(args.get("device").c_str());
    ulg_ctx *ctx = nullptr;
    if (ulg_create(&dev, 1, &ctx) != ULG_OK) {
        std::fprintf(stderr, "triplet_astar: no usable HIP device %d\n", dev);
        return 1;
    }
    const double t1 = ulgcli::now_s();
    int rc = ulg_search_load(ctx, n, p.offsets.data(), p.sets.data(), p.costs.data());
    if (rc == ULG_OK && running_time > 0) rc = ulg_set_option(ctx, "time_limit_ms", (int64_t)running_time * 1000);
    const double t2 = ulgcli::now_s();
    std::vector<int> dg((size_t)n * n, 0);
    int64_t stats[3] = {0, 0, 0};
    if (rc == ULG_OK) rc = ulg_triplet_astar(ctx, good ? rows.data() : nullptr, pd, dg.data(), stats);
    const double t3 = ulgcli::now_s();
    if (rc != ULG_OK) {
        std::fprintf(stderr, "triplet_astar: %s\n", ulg_last_error(ctx));
        ulg_destroy(ctx);
        return 1;
    }
    int64_t out_of_time = 0;
    if (running_time > 0) ulg_get_info(ctx, "out_of_time", &out_of_time);
    ulg_destroy(ctx);
    if (out_of_time) std::printf("Out of time\n");
    std::printf("A* runs %lld (distinct clusters %lld), nodes expanded %lld\n", (long long)stats[0],
                (long long)stats[1], (long long)stats[2]);
    std::printf("Timing: read .pss %.3f s, HIP init %.3f s, GPU best-score tables %.3f s, triplet search %.3f s\n",
                tr - t0, t1 - tr, t2 - t1, t3 - t2);
    std::fprintf(stderr,
                 "ulg_metrics {\"tool\": \"triplet_astar\", \"n\": %d, \"runs\": %lld, \"distinct\": %lld, "
                 "\"expanded\": %lld, \"read_s\": %.6f, \"init_s\": %.6f, \"tables_s\": %.6f, \"search_s\": %.6f}\n",
                 n, (long long)stats[0], (long long)stats[1], (long long)stats[2], tr - t0, t1 - tr, t2 - t1, t3 - t2);
    const std::string net = args.get("netFile");
    if (!net.empty()) {
        std::string csv;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                csv += std::to_string(dg[(size_t)i * n + j]);
                csv += (j == n - 1) ? "\n" : ",";
            }
        if (!ulgio::write_text(net, "") || !ulgio::write_text(net + ".csv", csv)) {
            std::fprintf(stderr, "triplet_astar: cannot write '%s'\n", net.c_str());
            return 1;
        }
    }
    return 0;
}
