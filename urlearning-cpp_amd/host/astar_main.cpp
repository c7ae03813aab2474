// astar -- the reference's astar command line (astar/astar_main.cpp) on the
// MI355X path: the .pss score cache is read on the host, the best-score
// lattice tables and the static pattern database are built on the GPU, and
// the search runs either in the reference's exact pop order (--mode exact,
// default: the reference's DAG bit for bit) or as the GPU layer-synchronous
// order-graph search (--mode gpu: an optimal DAG, expansions/s path).
//
//   astar <in.pss> [-k skeleton] [-n netFile] [-a 2] [--mode exact|gpu]
//
// The reference's post-processing (-f/-i/-l/-w/--adaptive, astar_main.cpp:
// 482-491) only prints and is skipped; -b accepts list, bitwise
// and tree (all give the list calculator's answer); -e accepts static only.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ulg.h"
#include "cli_common.h"
#include "io.h"

int main(int argc, char **argv) {
    ulgcli::Args args(
        {
            {"k", "skeleton", true, "", "The file containing the edges of a skeleton"},
            {"f", "scoring_function", true, "", "Post-processing scoring function (skipped)"},
            {"i", "raw_inputFile", true, "", "Raw data file for post-processing (skipped)"},
            {"l", "lambda", true, "", "Lambda for post-processing (skipped)"},
            {"", "adaptive", false, "", "Post-processing flag (skipped)"},
            {"w", "scoreType", true, "1", "Post-processing score type (skipped)"},
            {"b", "bestScore", true, "list", "BestScore calculator: list, bitwise or tree"},
            {"e", "heuristic", true, "static", "Heuristic type: static"},
            {"a", "argument", true, "2", "Number of static pattern databases"},
            {"p", "pc_{i-1}", true, "", "Variables which can only be used as ancestors (CSV of indices; with -s)"},
            {"s", "scc_i", true, "", "Variables which will be added in the search (CSV of indices; blank: all)"},
            {"r", "runningTime", true, "0", "The maximum running time (s) for the algorithm (exact mode).  0 means no running time."},
            {"n", "netFile", true, "", "The file to which the learned network is written."},
            {"", "mode", true, "exact", "exact (reference pop order) or gpu (GPU order-graph search)"},
            {"", "device", true, "0", "HIP device to use."},
            {"h", "help", false, "", "Show this help message."},
        },
        {"scoreFile"});
    std::string err;
    if (!args.parse(argc, argv, err)) {
        std::fprintf(stderr, "astar: %s\n", err.c_str());
        return 2;
    }
    if (args.has("help") || argc == 1 || !args.has("scoreFile")) {
        args.usage(argv[0], "Learn an optimal Bayesian network using A* on an MI355X.  Example usage: astar iris.pss -n iris_net");
        return args.has("help") || argc == 1 ? 0 : 2;
    }
    std::string bs = args.get("bestScore");
    if (bs != "list" && bs != "bitwise" && bs != "tree") {
        std::fprintf(stderr, "astar: Invalid BestScore calculator type: '%s'\n", bs.c_str());
        return 2;
    }
    if (args.get("heuristic") != "static") {
        std::fprintf(stderr, "astar: only the static pattern database heuristic is on this path\n");
        return 2;
    }
    const std::string mode = args.get("mode");
    if (mode != "exact" && mode != "gpu") {
        std::fprintf(stderr, "astar: --mode must be exact or gpu\n");
        return 2;
    }
    const int pd = std::atoi(args.get("argument").c_str());
    ulgio::PssData p;
    const double t0 = ulgcli::now_s();
    if (!ulgio::read_pss(args.get("scoreFile"), p, err)) {
        std::fprintf(stderr, "astar: %s\n", err.c_str());
        return 1;
    }
    const int n = (int)p.names.size();
    if (n < 1) {
        std::fprintf(stderr, "astar: no variables in '%s'\n", args.get("scoreFile").c_str());
        return 1;
    }
    // astar_main.cpp:590-598: no -s means every variable (and -p is ignored)
    uint64_t ancestors = 0, scc = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    if (!args.get("scc_i").empty()) {
        scc = 0;
        if (!ulgcli::set_from_csv(args.get("scc_i"), scc) || !ulgcli::set_from_csv(args.get("pc_{i-1}"), ancestors)) {
            std::fprintf(stderr, "astar: Invalid csv string: '%s' / '%s'\n", args.get("scc_i").c_str(),
                         args.get("pc_{i-1}").c_str());
            return 1;
        }
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
        std::fprintf(stderr, "astar: no usable HIP device %d\n", dev);
        return 1;
    }
    const double t1 = ulgcli::now_s();
    int rc = ulg_search_load(ctx, n, p.offsets.data(), p.sets.data(), p.costs.data());
    const double t2 = ulgcli::now_s();
    std::vector<uint64_t> vpar(n);
    std::vector<int> order(n);
    float cost = 0.0f;
    int64_t expanded = 0;
    std::vector<char> text(1 << 20);
    const int running_time = std::atoi(args.get("runningTime").c_str());
    if (running_time > 0) {
        std::printf("Maximum running time: %d\n", running_time);  // astar_main.cpp:698
        if (rc == ULG_OK) rc = ulg_set_option(ctx, "time_limit_ms", (int64_t)running_time * 1000);
    }
    if (rc == ULG_OK)
        rc = ulg_astar_scc(ctx, good ? rows.data() : nullptr, pd, mode == "gpu" ? ULG_ASTAR_GPU : ULG_ASTAR_EXACT,
                           ancestors, scc, vpar.data(), order.data(), &cost, &expanded, text.data(),
                           (int64_t)text.size());
    const double t3 = ulgcli::now_s();
    if (rc != ULG_OK) {
        std::fprintf(stderr, "astar: %s\n", ulg_last_error(ctx));
        ulg_destroy(ctx);
        return 1;
    }
    int64_t oot = 0;
    ulg_get_info(ctx, "out_of_time", &oot);
    ulg_destroy(ctx);
    if (oot) {
        // astar_main.cpp:136,535-540: the loop ended without a goal
        std::printf("Out of time\n");
        std::printf("No solution found.\n");
        std::printf("Nodes expanded: %lld\n", (long long)expanded);
        // a component finished before the watchdog keeps its netFile
        const std::string net = args.get("netFile");
        if (!net.empty() && text[0] && (!ulgio::write_text(net, std::string(text.data())) ||
                                        !ulgio::write_net_csv(net + ".csv", vpar, n))) {
            std::fprintf(stderr, "astar: cannot write '%s'\n", net.c_str());
            return 1;
        }
        return 0;
    }
    std::printf("Found solution: %f\n", (double)cost);
    std::printf("Nodes expanded: %lld\n", (long long)expanded);
    std::printf("Timing: read .pss %.3f s, HIP init %.3f s, GPU best-score tables %.3f s, search (%s) %.3f s (%.3g expansions/s)\n",
                tr - t0, t1 - tr, t2 - t1, mode.c_str(), t3 - t2, (double)expanded / (t3 - t2));
    // one machine-readable line on stderr (stdout keeps the reference's text)
    std::fprintf(stderr,
                 "ulg_metrics {\"tool\": \"astar\", \"mode\": \"%s\", \"n\": %d, \"cost\": %.6f, \"expanded\": %lld, "
                 "\"read_s\": %.6f, \"init_s\": %.6f, \"tables_s\": %.6f, \"search_s\": %.6f, \"expansions_per_s\": %.6g}\n",
                 mode.c_str(), n, (double)cost, (long long)expanded, tr - t0, t1 - tr, t2 - t1, t3 - t2,
                 (double)expanded / (t3 - t2));
    const std::string net = args.get("netFile");
    if (!net.empty()) {
        std::string txt(text.data());
        if (mode == "gpu") {
            // netFile text from the GPU result (same layout, astar_main.cpp:192-212)
            txt = "NumVars " + std::to_string(n) + "\n";
            for (int v = 0; v < n; ++v) {
                txt += "Var " + std::to_string(order[v] + 1) + ", parents";
                for (int i = 0; i < n; ++i)
                    if ((vpar[order[v]] >> i) & 1ull) txt += ", " + std::to_string(i + 1);
                txt += "\n";
            }
        }
        if (!ulgio::write_text(net, txt) || !ulgio::write_net_csv(net + ".csv", vpar, n)) {
            std::fprintf(stderr, "astar: cannot write '%s'\n", net.c_str());
            return 1;
        }
    }
    return 0;
}
