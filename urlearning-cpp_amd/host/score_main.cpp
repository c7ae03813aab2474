// score -- the reference's score command line (score/score_main.cpp) on the
// MI355X path: the input CSV is read on the host, every cBIC parent set is
// scored by libulg.so on one GPU, and the .pss score cache is written in the
// reference's exact text format.
//
//   score <in.csv> <out.pss> -f cBIC --lambda L [-k skeleton] [-p k] [-s] [-d ,]
//
// Options that only matter for other scoring functions or for the reference's
// AD-tree (-m, -e, -w, -a, -o, --enableDeCamposPruning) are accepted; -e
// still feeds the "META ess" header line as in score_main.cpp:388.
#include <cctype>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/ulg.h"
#include "cli_common.h"
#include "io.h"

int main(int argc, char **argv) {
    using ulgcli::Opt;
    ulgcli::Args args(
        {
            {"d", "delimiter", true, ",", "The delimiter of the input file."},
            {"l", "lambda", true, "0.5", "The lambda (BIC penalty weight)."},
            {"a", "adaptive", false, "", "Use adaptive Lasso (not on this path)."},
            {"w", "scoreType", true, "1", "which score (not on this path)"},
            {"c", "constraints", true, "", "The file specifying constraints on the scores (unsupported)."},
            {"k", "skeleton", true, "", "The file specifying the skeleton superstructure"},
            {"m", "rMin", true, "5", "The minimum number of records in the AD-tree nodes (unused by cBIC)."},
            {"f", "function", true, "BIC", "The scoring function to use (cBIC)."},
            {"e", "ess", true, "1", "The equivalent sample size (written to META ess)."},
            {"p", "maxParents", true, "0", "The maximum number of parents for any variable. A value less than 1 means no limit."},
            {"t", "threads", true, "1", "Host threads in the reference; the GPU scores every variable at once."},
            {"r", "time", true, "-1", "The maximum amount of time (s) to use for each variable (every variable is scored at once: the budget of the whole call, checked after each layer). A value less than 1 means no limit."},
            {"s", "hasHeader", false, "", "Add this flag if the first line of the input file gives the variable names."},
            {"o", "doNotPrune", false, "", "No effect (the reference's pruning is disabled, score_main.cpp:167-171)."},
            {"", "enableDeCamposPruning", false, "", "No effect for cBIC."},
            {"", "device", true, "0", "HIP device to use."},
            {"h", "help", false, "", "Show this help message."},
        },
        {"input", "output"});
    std::string err;
    if (!args.parse(argc, argv, err)) {
        std::fprintf(stderr, "score: %s\n", err.c_str());
        return 2;
    }
    if (args.has("help") || argc == 1 || !args.has("input") || !args.has("output")) {
        args.usage(argv[0], "Compute the scores for a csv file on an MI355X.  Example usage: score iris.csv iris.pss -f cBIC --lambda 2");
        return args.has("help") || argc == 1 ? 0 : 2;
    }
    std::string sf = args.get("function");
    for (char &ch : sf) ch = (char)std::tolower((unsigned char)ch);
    if (sf != "cbic") {
        std::fprintf(stderr, "score: scoring function '%s' is not on this path; use -f cBIC\n", args.get("function").c_str());
        return 2;
    }
    if (!args.get("constraints").empty()) {
        std::fprintf(stderr, "score: constraint files (-c) are not supported on this path\n");
        return 2;
    }
    const std::string input = args.get("input"), output = args.get("output");
    const char delim = args.get("delimiter").empty() ? ',' : args.get("delimiter")[0];
    const bool has_header = args.has("hasHeader");
    const double lambda = std::atof(args.get("lambda").c_str());
    int maxp = std::atoi(args.get("maxParents").c_str());

    ulgio::RecordStats rs;
    if (!ulgio::record_stats(input, delim, has_header, rs)) {
        std::fprintf(stderr, "score: cannot read '%s'\n", input.c_str());
        return 1;
    }
    std::vector<double> data;
    int64_t N = 0;
    int ncols = 0;
    if (!ulgio::load_numeric_csv(input, data, N, ncols)) {
        std::fprintf(stderr, "score: cannot load '%s'\n", input.c_str());
        return 1;
    }
    const int n = (int)rs.names.size();
    if (n != ncols || n < 1 || n > 63) {
        std::fprintf(stderr, "score: %d record columns vs %d numeric columns (n must be 1..63)\n", n, ncols);
        return 1;
    }
    if (maxp > n || maxp < 1) maxp = n - 1;  // score_main.cpp:296-298
    // candidates: 2-hop skeleton neighbourhood; no -k = every variable
    std::vector<uint64_t> cands(n, n >= 64 ? ~0ull : ((1ull << n) - 1ull));
    const std::string skel = args.get("skeleton");
    if (!skel.empty()) {
        std::vector<uint64_t> rows;
        int nv = 0;
        if (ulgio::read_skeleton(skel, n, rows, nv)) {
            for (int v = 0; v < n; ++v) cands[v] = ulgio::candidates(rows, n, v);
        } else {
            // an unreadable -k leaves the default Skeleton(1) whose get_neighbors is {0}
            for (int v = 0; v < n; ++v) cands[v] = 1ull;
        }
    }
    const int dev = std::atoi(args.get("device").c_str());
    ulg_ctx *ctx = nullptr;
    if (ulg_create(&dev, 1, &ctx) != ULG_OK) {
        std::fprintf(stderr, "score: no usable HIP device %d\n", dev);
        return 1;
    }
    const double t0 = ulgcli::now_s();
    int rc = ulg_cbic_load(ctx, data.data(), N, n, lambda);
    std::vector<int> vars(n);
    for (int v = 0; v < n; ++v) vars[v] = v;
    int64_t stored = 0, scored = 0;
    const int running_time = std::atoi(args.get("time").c_str());
    if (running_time > 0) {
        std::printf("I am using a timer in the calculation function.\n");  // score_calculator.cpp:40
        if (rc == ULG_OK) rc = ulg_set_option(ctx, "time_limit_ms", (int64_t)running_time * 1000);
    }
    if (rc == ULG_OK) rc = ulg_cbic_score(ctx, vars.data(), n, cands.data(), maxp, &stored, &scored);
    int64_t oot = 0, done_layer = 0;
    if (rc == ULG_OK && running_time > 0) {
        ulg_get_info(ctx, "out_of_time", &oot);
        ulg_get_info(ctx, "highest_completed_layer", &done_layer);
        if (oot) std::printf("Out of time\n");  // score_calculator.cpp:28-31
    }
    const double t1 = ulgcli::now_s();
    if (rc != ULG_OK) {
        std::fprintf(stderr, "score: %s\n", ulg_last_error(ctx));
        ulg_destroy(ctx);
        return 1;
    }
    ulgio::PssHeader h;
    h.input_file = input;
    h.num_records = rs.num_records;
    h.parent_limit = maxp;
    h.score_type = sf;
    {
        // boost::lexical_cast<std::string>(float)
        char buf[64];
        std::snprintf(buf, sizeof buf, "%.9g", (double)std::strtof(args.get("ess").c_str(), nullptr));
        h.ess = buf;
    }
    const std::string header = ulgio::pss_header_text(h);
    std::vector<const char *> cnames(n);
    for (int v = 0; v < n; ++v) cnames[v] = rs.names[v].c_str();
    const char *text = nullptr;
    int64_t len = 0;
    rc = ulg_pss_format(ctx, header.c_str(), cnames.data(), rs.arity.data(), &text, &len);
    const double t2 = ulgcli::now_s();
    if (rc != ULG_OK) {
        std::fprintf(stderr, "score: %s\n", ulg_last_error(ctx));
        ulg_destroy(ctx);
        return 1;
    }
    if (!ulgio::write_bytes(output, text, len)) {
        std::fprintf(stderr, "score: cannot write '%s'\n", output.c_str());
        ulg_destroy(ctx);
        return 1;
    }
    ulg_destroy(ctx);
    const double t3 = ulgcli::now_s();
    std::printf("URLearning (MI355X), Score Calculator: n=%d N=%lld k=%d lambda=%g\n", n, (long long)N, maxp, lambda);
    if (oot) std::printf("Scoring stopped after layer %lld of %d (-r %d s)\n", (long long)done_layer, maxp, running_time);
    std::printf("Parent sets scored: %lld, stored: %lld, GPU scoring %.3f s (%.3g sets/s), GPU .pss format %.3f s, "
                "file write %.3f s (%lld bytes)\n",
                (long long)scored, (long long)stored, t1 - t0, (double)scored / (t1 - t0), t2 - t1, t3 - t2,
                (long long)len);
    std::fprintf(stderr,
                 "ulg_metrics {\"tool\": \"score\", \"n\": %d, \"N\": %lld, \"k\": %d, \"lambda\": %g, "
                 "\"scored\": %lld, \"stored\": %lld, \"score_s\": %.6f, \"sets_per_s\": %.6g, \"format_s\": %.6f, "
                 "\"write_s\": %.6f, \"bytes\": %lld, \"out_of_time\": %d}\n",
                 n, (long long)N, maxp, lambda, (long long)scored, (long long)stored, t1 - t0,
                 (double)scored / (t1 - t0), t2 - t1, t3 - t2, (long long)len, (int)oot);
    return 0;
}
