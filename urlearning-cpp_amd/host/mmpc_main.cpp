// mmpc -- writes the skeleton file the reference's score / astar /
// triplet_astar take with -k (README.md:16 expects it from an MMPC run
// outside the package; format read by Skeleton::read_matrix_file,
// base/skeleton.cpp:19-105): an n x n 0/1 matrix, row i column j = 1 iff
// edge i-j.  The data go through the same loader as `score` (mlpack/Armadillo
// csv semantics), the Gram matrix is built on the GPU (MFMA f64) and every
// Fisher-z test runs on the GPU (ulg_mmpc).
//
//   mmpc <in.csv> <skeleton.csv> [--alpha 0.05] [--max-cond K] [--diagonal]
//
// --diagonal also sets the diagonal, as the README's all-ones example does
// (it changes triplet_astar's degenerate triples, tests/golden/README.md).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/ulg.h"
#include "cli_common.h"
#include "io.h"

int main(int argc, char **argv) {
    ulgcli::Args args(
        {
            {"", "alpha", true, "0.05", "Significance level of the Fisher-z tests"},
            {"", "max-cond", true, "-1", "Largest conditioning set (-1: no cap below 24)"},
            {"", "diagonal", false, "", "Set the diagonal of the skeleton matrix"},
            {"", "device", true, "0", "HIP device to use."},
            {"h", "help", false, "", "Show this help message."},
        },
        {"input", "output"});
    std::string err;
    if (!args.parse(argc, argv, err)) {
        std::fprintf(stderr, "mmpc: %s\n", err.c_str());
        return 2;
    }
    if (args.has("help") || argc == 1 || !args.has("input") || !args.has("output")) {
        args.usage(argv[0], "MMPC skeleton for the score/astar/triplet_astar -k option.  Example usage: mmpc data.csv skeleton.csv");
        return args.has("help") || argc == 1 ? 0 : 2;
    }
    const double alpha = std::atof(args.get("alpha").c_str());
    const int max_cond = std::atoi(args.get("max-cond").c_str());
    std::vector<double> data;
    int64_t N = 0;
    int n = 0;
    if (!ulgio::load_numeric_csv(args.get("input"), data, N, n) || n < 1 || n > 63) {
        std::fprintf(stderr, "mmpc: cannot load '%s' (1..63 columns)\n", args.get("input").c_str());
        return 1;
    }
    const int dev = std::atoi(args.get("device").c_str());
    ulg_ctx *ctx = nullptr;
    if (ulg_create(&dev, 1, &ctx) != ULG_OK) {
        std::fprintf(stderr, "mmpc: no usable HIP device %d\n", dev);
        return 1;
    }
    const double t0 = ulgcli::now_s();
    std::vector<uint64_t> rows(n, 0);
    int rc = ulg_cbic_load(ctx, data.data(), N, n, 0.0);
    if (rc == ULG_OK) rc = ulg_mmpc(ctx, alpha, max_cond, rows.data());
    const double t1 = ulgcli::now_s();
    if (rc != ULG_OK) {
        std::fprintf(stderr, "mmpc: %s\n", ulg_last_error(ctx));
        ulg_destroy(ctx);
        return 1;
    }
    ulg_destroy(ctx);
    std::string text;
    int edges = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            const bool e = ((rows[i] >> j) & 1ull) || (i == j && args.has("diagonal"));
            edges += (j > i) && ((rows[i] >> j) & 1ull);
            text += e ? '1' : '0';
            text += (j == n - 1) ? '\n' : ',';
        }
    if (!ulgio::write_text(args.get("output"), text)) {
        std::fprintf(stderr, "mmpc: cannot write '%s'\n", args.get("output").c_str());
        return 1;
    }
    std::printf("MMPC (MI355X): n=%d N=%lld alpha=%g edges=%d, Gram + tests %.3f s\n", n, (long long)N, alpha, edges,
                t1 - t0);
    return 0;
}
