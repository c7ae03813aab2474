// io.h -- host-side text formats of the drop-in surface: the data CSV, the
// skeleton file, the .pss score cache, and the A* network outputs.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ulgio {

// mlpack::data::Load(file, m, fatal=true, transpose=false) over Armadillo's
// csv_ascii (scoring_function/BIC_OLS.cpp:48): rows = lines, cols = max
// tokens per line, every token through strtod, unconvertible tokens 0 (a
// header row becomes a row of zeros).  Column-major N x n.
bool load_numeric_csv(const std::string &path, std::vector<double> &colmajor, int64_t &N, int &n);

// RecordFile + BayesianNetwork::initialize (base/record_file.h:39-54,
// base/bayesian_network.cpp:25-42, base/variable.h:58-64): names and
// per-column distinct-token counts ("META arity").
struct RecordStats {
    int64_t num_records = 0;
    std::vector<std::string> names;
    std::vector<int> arity;
};
bool record_stats(const std::string &path, char delim, bool has_header, RecordStats &out);

// Skeleton::read_matrix_file / read_arc_list_file (base/skeleton.cpp:19-105).
// Returns false if the file cannot be opened.  rows[i] bit j = edge i-j.
bool read_skeleton(const std::string &path, int n_expected, std::vector<uint64_t> &rows, int &num_vertices);
// 2-hop candidate sets N(v) U N(N(v)) (score/score_main.cpp:146-153)
uint64_t candidates(const std::vector<uint64_t> &rows, int n, int v);

// .pss writer (score/score_main.cpp:173-203 per variable, :383-400 header)
struct PssHeader {
    std::string input_file;
    int64_t num_records = 0;
    int parent_limit = 0;
    std::string score_type;
    std::string ess = "1";
};
// The META block the .pss starts with (score_main.cpp:383-389), blank line
// included; the per-variable blocks come from ulg_pss_format.
std::string pss_header_text(const PssHeader &h);
bool write_bytes(const std::string &path, const char *data, int64_t len);

// ScoreCache::read (score_cache/score_cache.cpp:55-160): two passes with the
// reference's case-insensitive "var " / "meta" substring tests; costs are
// -1 * atof(score); a repeated parent set keeps its first position and its
// last value (FloatMap operator[] semantics).
struct PssData {
    std::vector<std::string> names;
    std::vector<int64_t> offsets;
    std::vector<uint64_t> sets;
    std::vector<float> costs;
};
bool read_pss(const std::string &path, PssData &out, std::string &err);

// netFile text and netFile.csv (astar/astar_main.cpp:192-212, 518-533)
bool write_net_csv(const std::string &path, const std::vector<uint64_t> &vpar, int n);
bool write_text(const std::string &path, const std::string &text);

}  // namespace ulgio
