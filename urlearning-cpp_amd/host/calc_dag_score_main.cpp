// calc_dag_score -- the reference's DAG scorer (astar/calc_dag_score.cpp)
// on the MI355X path: the .pss is read on the host, the best-score lattice is
// built on the GPU, and every lookup of every DAG -- getScore(parents) for
// each row and for each column of the transposed ("alt") reading -- goes to
// the device in one batched ulg_bestscore_query.
//
//   calc_dag_score <in.pss> <dag.csv> [<dag.csv> ...]
//
// Output (calc_dag_score.cpp:160-175), one line for all models:
//   "<NAME>  <score>  edges <E>  " for the first DAG, then
//   "<NAME>  <score>  edges <E> remove <R> " for the others, where NAME is the
//   file's basename cut at ".csv" and upper-cased, score = min(row-wise total,
//   transposed total) and R the matching quirk of :166.  An unreadable score
//   file gives zero scores (the reference's NULL calculators); an unreadable
//   DAG file prints "Invalid model file" and counts as empty.
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/ulg.h"
#include "io.h"

namespace {

// boost::char_separator<char>(", \n\r") tokens of one line, through atof
std::vector<double> dag_tokens(const std::string &line) {
    std::vector<double> out;
    size_t i = 0;
    const char *sep = ", \n\r";
    while (i < line.size()) {
        while (i < line.size() && std::strchr(sep, line[i])) ++i;
        if (i >= line.size()) break;
        const size_t b = i;
        while (i < line.size() && !std::strchr(sep, line[i])) ++i;
        out.push_back(std::atof(line.substr(b, i - b).c_str()));
    }
    return out;
}

struct Dag {
    std::string name;
    bool ok = false;
    int variableCount = 0;
    std::vector<uint64_t> rows;  // parents of row v
    std::vector<uint64_t> alt;   // transposed reading
    int num_edges = 0;
};

Dag read_dag(const char *path) {
    Dag d;
    const char *base = std::strrchr(path, '/');
    d.name = base ? base + 1 : path;
    const size_t dot = d.name.find(".csv");
    if (dot != std::string::npos) d.name = d.name.substr(0, dot);
    for (char &ch : d.name) ch = (char)std::toupper((unsigned char)ch);
    std::ifstream in(path);
    if (!in.good()) {
        std::fprintf(stderr, "Invalid model file %s\n", path);
        return d;
    }
    d.ok = true;
    std::string line;
    std::getline(in, line);
    d.variableCount = (int)dag_tokens(line).size();
    const int vc = std::min(d.variableCount, 64);
    d.alt.assign(vc, 0);
    std::vector<std::vector<int>> edges(64, std::vector<int>(64, 0));
    int v = 0;
    do {
        const std::vector<double> tok = dag_tokens(line);
        uint64_t par = 0;
        for (size_t i = 0; i < tok.size() && i < 64; ++i)
            if (std::fabs((float)tok[i]) > 1e-5f) {
                par |= 1ull << i;
                if ((int)i < vc) d.alt[i] |= 1ull << v;
                edges[v][i] = edges[i][v] = 1;
            }
        d.rows.push_back(par);
        ++v;
    } while (std::getline(in, line) && v < d.variableCount && v < 64);
    for (int i = 0; i < vc; ++i)
        for (int j = i + 1; j < vc; ++j) d.num_edges += edges[i][j];
    return d;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: calc_dag_score <in.pss> <dag.csv>...\n");
        return 2;
    }
    std::vector<Dag> dags;
    for (int m = 2; m < argc; ++m) dags.push_back(read_dag(argv[m]));
    ulg_ctx *ctx = nullptr;
    int n = 0;
    {
        std::ifstream probe(argv[1]);
        if (probe.good()) {
            ulgio::PssData p;
            std::string err;
            if (!ulgio::read_pss(argv[1], p, err)) {
                std::fprintf(stderr, "calc_dag_score: %s\n", err.c_str());
                return 1;
            }
            n = (int)p.names.size();
            const int dev = 0;
            if (ulg_create(&dev, 1, &ctx) != ULG_OK) {
                std::fprintf(stderr, "calc_dag_score: no usable HIP device\n");
                return 1;
            }
            if (ulg_search_load(ctx, n, p.offsets.data(), p.sets.data(), p.costs.data()) != ULG_OK) {
                std::fprintf(stderr, "calc_dag_score: %s\n", ulg_last_error(ctx));
                ulg_destroy(ctx);
                return 1;
            }
        }
    }
    // one batched lookup for every (variable, parent set) of every DAG
    std::vector<int> qv;
    std::vector<uint64_t> qs;
    for (const Dag &d : dags) {
        if (!ctx || !d.ok) continue;
        if (d.variableCount > n) {
            std::fprintf(stderr, "calc_dag_score: %d columns in a DAG over %d scored variables\n", d.variableCount, n);
            ulg_destroy(ctx);
            return 1;
        }
        for (size_t v = 0; v < d.rows.size(); ++v) { qv.push_back((int)v); qs.push_back(d.rows[v]); }
        for (size_t i = 0; i < d.alt.size(); ++i) { qv.push_back((int)i); qs.push_back(d.alt[i]); }
    }
    std::vector<float> qc(qv.size());
    std::vector<uint64_t> qp(qv.size());
    if (ctx && !qv.empty() &&
        ulg_bestscore_query(ctx, (int64_t)qv.size(), qv.data(), qs.data(), qc.data(), qp.data()) != ULG_OK) {
        std::fprintf(stderr, "calc_dag_score: %s\n", ulg_last_error(ctx));
        ulg_destroy(ctx);
        return 1;
    }
    size_t q = 0;
    for (size_t m = 0; m < dags.size(); ++m) {
        const Dag &d = dags[m];
        float total = 0.0f, alt = 0.0f;
        int rm = 0, rma = 0;
        if (ctx && d.ok) {
            for (size_t v = 0; v < d.rows.size(); ++v, ++q) {
                total += qc[q];
                rm += __builtin_popcountll(d.rows[v] ^ qp[q]);
            }
            for (size_t i = 0; i < d.alt.size(); ++i, ++q) {
                alt += qc[q];
                rma += __builtin_popcountll(d.alt[i] ^ qp[q]);
            }
        }
        const float score = total > alt ? alt : total;
        const int to_remove = total > alt ? rm : rma;
        if (m == 0) std::printf("%s  %f  edges %d  ", d.name.c_str(), (double)score, d.num_edges);
        else std::printf("%s  %f  edges %d remove %d ", d.name.c_str(), (double)score, d.num_edges, to_remove);
    }
    std::printf("\n");
    if (ctx) ulg_destroy(ctx);
    return 0;
}
