// io.cpp -- see io.h.
#include "io.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <unordered_map>
#include <unordered_set>

namespace ulgio {

namespace {

std::string trim(const std::string &s) {
    size_t b = 0, e = s.size();
    while (b < e && std::isspace((unsigned char)s[b])) ++b;
    while (e > b && std::isspace((unsigned char)s[e - 1])) --e;
    return s.substr(b, e - b);
}

// boost::split(out, s, is_any_of(delims), token_compress_on)
std::vector<std::string> split_compress(const std::string &s, const std::string &delims) {
    std::vector<std::string> out;
    std::string cur;
    bool in_delim = false;
    for (char ch : s) {
        if (delims.find(ch) != std::string::npos) {
            if (!in_delim) out.push_back(cur);
            cur.clear();
            in_delim = true;
        } else {
            cur.push_back(ch);
            in_delim = false;
        }
    }
    out.push_back(cur);
    return out;
}

bool icontains(const std::string &line, const char *needle) {
    std::string a = line, b = needle;
    std::transform(a.begin(), a.end(), a.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    std::transform(b.begin(), b.end(), b.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    return a.find(b) != std::string::npos;
}

}  // namespace

bool load_numeric_csv(const std::string &path, std::vector<double> &colmajor, int64_t &N, int &n) {
    std::ifstream in(path);
    if (!in) return false;
    std::vector<std::string> lines;
    std::string line;
    int cols = 0;
    while (std::getline(in, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        cols = std::max(cols, (int)std::count(line.begin(), line.end(), ',') + 1);
        lines.push_back(line);
    }
    if (lines.empty() || cols == 0) return false;
    N = (int64_t)lines.size();
    n = cols;
    colmajor.assign((size_t)(N * n), 0.0);
    for (int64_t r = 0; r < N; ++r) {
        const std::string &s = lines[r];
        size_t pos = 0;
        int c = 0;
        while (true) {
            const size_t comma = s.find(',', pos);
            const std::string tok = s.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
            char *end = nullptr;
            const double v = std::strtod(tok.c_str(), &end);
            if (end != tok.c_str()) colmajor[(size_t)c * N + r] = v;
            ++c;
            if (comma == std::string::npos) break;
            pos = comma + 1;
        }
    }
    return true;
}

bool record_stats(const std::string &path, char delim, bool has_header, RecordStats &out) {
    std::ifstream in(path);
    if (!in) return false;
    std::string line;
    std::vector<std::string> header;
    std::vector<std::unordered_set<std::string>> seen;
    bool first = true;
    size_t ncols = 0;
    out.num_records = 0;
    const std::string d(1, delim);
    while (std::getline(in, line)) {
        const std::vector<std::string> tok = split_compress(trim(line), d);
        if (first && has_header) {
            header = tok;
            first = false;
            continue;
        }
        if (first || ncols == 0) {
            if (ncols == 0) ncols = tok.size();
            seen.resize(std::max(seen.size(), tok.size()));
        }
        first = false;
        if (seen.size() < tok.size()) seen.resize(tok.size());
        for (size_t c = 0; c < tok.size(); ++c) seen[c].insert(tok[c]);
        ++out.num_records;
    }
    out.names.clear();
    out.arity.clear();
    for (size_t c = 0; c < ncols; ++c) {
        out.names.push_back(has_header && c < header.size() ? header[c] : "Variable_" + std::to_string(c));
        out.arity.push_back((int)seen[c].size());
    }
    return true;
}

bool read_skeleton(const std::string &path, int n_expected, std::vector<uint64_t> &rows, int &num_vertices) {
    std::ifstream in(path);
    if (!in) return false;
    rows.assign(64, 0);
    std::string line;
    const bool arc = path.size() >= 4 && path.compare(path.size() - 4, 4, ".arc") == 0;
    auto add_edge = [&](int i, int j) {
        if (i >= 0 && i < 64 && j >= 0 && j < 64) {
            rows[i] |= 1ull << j;
            rows[j] |= 1ull << i;
        }
    };
    if (arc) {
        num_vertices = n_expected;
        while (std::getline(in, line)) {
            std::vector<std::string> tok;
            for (const std::string &t : split_compress(line, ","))
                if (!t.empty()) tok.push_back(t);
            if (tok.size() < 2 || tok[0].size() < 2 || tok[1].size() < 2) continue;
            add_edge(std::atoi(tok[0].c_str() + 2) - 1, std::atoi(tok[1].c_str() + 2) - 1);
        }
    } else {
        int row = 0;
        num_vertices = 0;
        while (std::getline(in, line)) {
            // boost::char_separator(", \n\r"): empty tokens dropped
            int col = 0;
            std::string tok;
            auto flush = [&]() {
                if (tok.empty()) return;
                if (tok == "TRUE" || std::fabs(std::atof(tok.c_str())) > 0.05) add_edge(row, col);
                ++col;
                tok.clear();
            };
            for (char ch : line) {
                if (ch == ',' || ch == ' ' || ch == '\n' || ch == '\r') flush();
                else tok.push_back(ch);
            }
            flush();
            if (row == 0) num_vertices = col;
            ++row;
        }
    }
    rows.resize(std::max(num_vertices, n_expected));
    return true;
}

uint64_t candidates(const std::vector<uint64_t> &rows, int n, int v) {
    uint64_t nb = rows[v];
    for (int j = 0; j < n; ++j)
        if (((rows[v] >> j) & 1ull) && j != v) nb |= rows[j];
    return nb;
}

bool write_pss(const std::string &path, const PssHeader &h, const std::vector<std::string> &names,
               const std::vector<int> &arity, const std::vector<int64_t> &offsets, const std::vector<uint64_t> &sets,
               const std::vector<float> &scores) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::vector<char> buf(1 << 22);
    std::setvbuf(f, buf.data(), _IOFBF, buf.size());
    std::fprintf(f, "META pss_version = 0.1\nMETA input_file=%s\nMETA num_records=%lld\n", h.input_file.c_str(),
                 (long long)h.num_records);
    std::fprintf(f, "META parent_limit=%d\nMETA score_type=%s\nMETA ess=%s\n\n", h.parent_limit, h.score_type.c_str(),
                 h.ess.c_str());
    const int n = (int)names.size();
    for (int v = 0; v < n; ++v) {
        std::fprintf(f, "VAR %s\n", names[v].c_str());
        std::fprintf(f, "META arity=%d\n", arity[v]);
        for (int64_t i = offsets[v]; i < offsets[v + 1]; ++i) {
            std::fprintf(f, "%f ", (double)scores[i]);
            uint64_t s = sets[i];
            while (s) {
                const int p = __builtin_ctzll(s);
                s &= s - 1;
                std::fputs(names[p].c_str(), f);
                std::fputc(' ', f);
            }
            std::fputc('\n', f);
        }
        std::fputc('\n', f);
    }
    return std::fclose(f) == 0;
}

bool read_pss(const std::string &path, PssData &out, std::string &err) {
    std::ifstream in(path);
    if (!in) {
        err = "Could not open the score cache file: '" + path + "'";
        return false;
    }
    std::string line;
    std::unordered_map<std::string, int> index;
    out.names.clear();
    bool started = false;
    // pass 1: META block, then the variable names (score_cache.cpp:69-129)
    while (std::getline(in, line)) {
        if (line.empty() || line[0] == '#') continue;
        if (!started) {
            if (icontains(line, "var ")) started = true;
            else {
                if (!icontains(line, "meta")) {
                    err = "Error while parsing META information of network.  Expected META line or Variable.  Line: '" + line + "'";
                    return false;
                }
                const std::vector<std::string> kv = split_compress(trim(line.size() > 4 ? line.substr(4) : ""), "=");
                if (kv.size() != 2) {
                    err = "Error while parsing META information of network.  Too many tokens.  Line: '" + line + "'";
                    return false;
                }
                continue;
            }
        }
        if (icontains(line, "var ")) {
            const std::vector<std::string> tok = split_compress(trim(line), " ");
            if (tok.size() < 2) continue;
            if (index.count(tok[1])) {
                err = "Duplicate variable name: '" + tok[1] + "'.";
                return false;
            }
            index[tok[1]] = (int)out.names.size();
            out.names.push_back(tok[1]);
        }
    }
    const int n = (int)out.names.size();
    if (n > 63) {
        err = "more than 63 variables";
        return false;
    }
    // pass 2: parent sets (score_cache.cpp:135-159)
    in.clear();
    in.seekg(0);
    std::vector<std::vector<uint64_t>> sets(n);
    std::vector<std::vector<float>> costs(n);
    std::vector<std::unordered_map<uint64_t, size_t>> pos(n);
    int cur = -1;
    while (std::getline(in, line)) {
        if (line.empty() || line[0] == '#' || icontains(line, "meta")) continue;
        const std::vector<std::string> tok = split_compress(trim(line), " ");
        if (icontains(line, "var ")) {
            auto it = tok.size() >= 2 ? index.find(tok[1]) : index.end();
            cur = it == index.end() ? 0 : it->second;  // nameToIndex[] default-inserts 0
            continue;
        }
        if (cur < 0) continue;
        const float cost = -1 * std::atof(tok[0].c_str());
        uint64_t ps = 0;
        for (size_t i = 1; i < tok.size(); ++i) {
            auto it = index.find(tok[i]);
            ps |= 1ull << (it == index.end() ? 0 : it->second);
        }
        auto p = pos[cur].find(ps);
        if (p != pos[cur].end()) {
            costs[cur][p->second] = cost;
            continue;
        }
        pos[cur][ps] = sets[cur].size();
        sets[cur].push_back(ps);
        costs[cur].push_back(cost);
    }
    out.offsets.assign(n + 1, 0);
    out.sets.clear();
    out.costs.clear();
    for (int v = 0; v < n; ++v) {
        out.offsets[v + 1] = out.offsets[v] + (int64_t)sets[v].size();
        out.sets.insert(out.sets.end(), sets[v].begin(), sets[v].end());
        out.costs.insert(out.costs.end(), costs[v].begin(), costs[v].end());
    }
    return true;
}

bool write_net_csv(const std::string &path, const std::vector<uint64_t> &vpar, int n) {
    std::ofstream f(path, std::ios::trunc);
    if (!f) return false;
    for (int v = 0; v < n; ++v) {
        std::string row;
        for (int i = 0; i < n; ++i) {
            row += ((vpar[v] >> i) & 1ull) ? '1' : '0';
            row += (i == n - 1) ? '\n' : ',';
        }
        f << row;
    }
    return (bool)f;
}

bool write_text(const std::string &path, const std::string &text) {
    std::ofstream f(path, std::ios::trunc);
    if (!f) return false;
    f << text;
    return (bool)f;
}

}  // namespace ulgio
