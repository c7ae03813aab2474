// io.cpp -- see io.h.
#include "io.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <fstream>
#include <thread>
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

std::string pss_header_text(const PssHeader &h) {
    return "META pss_version = 0.1\nMETA input_file=" + h.input_file + "\nMETA num_records=" +
           std::to_string(h.num_records) + "\nMETA parent_limit=" + std::to_string(h.parent_limit) +
           "\nMETA score_type=" + h.score_type + "\nMETA ess=" + h.ess + "\n\n";
}

bool write_bytes(const std::string &path, const char *data, int64_t len) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = len == 0 || std::fwrite(data, 1, (size_t)len, f) == (size_t)len;
    return (std::fclose(f) == 0) && ok;
}

// ---- .pss reader ----------------------------------------------------------
// The file is read whole and its lines are handled by host threads: pass 1
// collects the variable names in order, pass 2 parses every chunk of lines
// into per-variable runs, and a final step merges the runs of each variable
// in file order with the duplicate rule.  Line classification, tokens and the
// atof conversion are the reference's (score_cache.cpp:55-160), so the
// result is identical to a sequential read.
namespace {

inline char lower(char ch) { return (ch >= 'A' && ch <= 'Z') ? (char)(ch - 'A' + 'a') : ch; }

bool icontains_sv(const char *b, const char *e, const char *needle, size_t nl) {
    if ((size_t)(e - b) < nl) return false;
    for (const char *p = b; p + nl <= e; ++p) {
        size_t k = 0;
        while (k < nl && lower(p[k]) == needle[k]) ++k;
        if (k == nl) return true;
    }
    return false;
}

// split_compress(trim(line), " ") as [begin, end) pairs
void tokens(const char *b, const char *e, std::vector<std::pair<const char *, const char *>> &out) {
    out.clear();
    while (b < e && std::isspace((unsigned char)*b)) ++b;
    while (e > b && std::isspace((unsigned char)e[-1])) --e;
    const char *cur = b;
    bool in_delim = false;
    for (const char *p = b; p < e; ++p) {
        if (*p == ' ') {
            if (!in_delim) out.emplace_back(cur, p);
            cur = p + 1;
            in_delim = true;
        } else {
            if (in_delim) cur = p;
            in_delim = false;
        }
    }
    out.emplace_back(in_delim ? e : cur, e);
}

int worker_count() {
    const char *env = std::getenv("ULG_THREADS");
    if (!env || !*env) env = std::getenv("OMP_NUM_THREADS");
    int t = env && *env ? std::atoi(env) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 64));
}

struct Entry {
    uint64_t set;
    float cost;
};

}  // namespace

bool read_pss(const std::string &path, PssData &out, std::string &err) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) {
        err = "Could not open the score cache file: '" + path + "'";
        return false;
    }
    std::string buf;
    {
        std::fseek(f, 0, SEEK_END);
        const long sz = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        buf.resize(sz > 0 ? (size_t)sz : 0);
        if (sz > 0 && std::fread(&buf[0], 1, (size_t)sz, f) != (size_t)sz) {
            std::fclose(f);
            err = "Could not read the score cache file: '" + path + "'";
            return false;
        }
        std::fclose(f);
    }
    const char *B = buf.data(), *E = B + buf.size();
    // line starts (std::getline: '\n'-terminated, a last unterminated line counts)
    const int T = worker_count();
    std::vector<const char *> cut(T + 1);
    cut[0] = B;
    cut[T] = E;
    for (int t = 1; t < T; ++t) {
        const char *p = B + (buf.size() * (size_t)t) / (size_t)T;
        if (p < cut[t - 1]) p = cut[t - 1];
        const char *nl = (const char *)std::memchr(p, '\n', (size_t)(E - p));
        cut[t] = nl ? nl + 1 : E;
    }
    auto for_lines = [](const char *b, const char *e, auto &&fn) {
        while (b < e) {
            const char *nl = (const char *)std::memchr(b, '\n', (size_t)(e - b));
            const char *le = nl ? nl : e;
            fn(b, le);
            b = nl ? nl + 1 : e;
        }
    };
    // pass 1a: every "var " line (skipping empty and '#' lines), per chunk
    std::vector<std::vector<const char *>> var_lines(T);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for_lines(cut[t], cut[t + 1], [&](const char *b, const char *e) {
                    if (b == e || *b == '#') return;
                    if (icontains_sv(b, e, "var ", 4)) var_lines[t].push_back(b);
                });
            });
        for (auto &x : th) x.join();
    }
    // pass 1b: the META block before the first variable (score_cache.cpp:69-106)
    const char *first_var = E;
    for (int t = 0; t < T; ++t)
        if (!var_lines[t].empty()) { first_var = var_lines[t][0]; break; }
    {
        bool bad = false;
        for_lines(B, first_var, [&](const char *b, const char *e) {
            if (bad || b == e || *b == '#') return;
            const std::string line(b, e);
            if (!icontains(line, "meta")) {
                err = "Error while parsing META information of network.  Expected META line or Variable.  Line: '" + line + "'";
                bad = true;
                return;
            }
            const std::vector<std::string> kv = split_compress(trim(line.size() > 4 ? line.substr(4) : ""), "=");
            if (kv.size() != 2) {
                err = "Error while parsing META information of network.  Too many tokens.  Line: '" + line + "'";
                bad = true;
            }
        });
        if (bad) return false;
    }
    // pass 1c: names in file order
    std::unordered_map<std::string, int> index;
    out.names.clear();
    std::vector<std::pair<const char *, const char *>> tok;
    for (int t = 0; t < T; ++t)
        for (const char *b : var_lines[t]) {
            const char *e = (const char *)std::memchr(b, '\n', (size_t)(E - b));
            tokens(b, e ? e : E, tok);
            if (tok.size() < 2) continue;
            const std::string name(tok[1].first, tok[1].second);
            if (index.count(name)) {
                err = "Duplicate variable name: '" + name + "'.";
                return false;
            }
            index[name] = (int)out.names.size();
            out.names.push_back(name);
        }
    const int n = (int)out.names.size();
    if (n > 63) {
        err = "more than 63 variables";
        return false;
    }
    // pass 2: the variable each chunk starts in, then every entry line
    std::vector<int> start_var(T, -1);
    auto var_of_line = [&](const char *b, const char *e) {
        std::vector<std::pair<const char *, const char *>> tk;
        tokens(b, e, tk);
        if (tk.size() < 2) return 0;  // nameToIndex[] default-inserts 0
        auto it = index.find(std::string(tk[1].first, tk[1].second));
        return it == index.end() ? 0 : it->second;
    };
    {
        int cur = -1;
        for (int t = 0; t < T; ++t) {
            start_var[t] = cur;
            // the last "var " line of this chunk that pass 2 would act on (no "meta" in it)
            for (auto it = var_lines[t].rbegin(); it != var_lines[t].rend(); ++it) {
                const char *b = *it;
                const char *e = (const char *)std::memchr(b, '\n', (size_t)(E - b));
                if (!e) e = E;
                if (icontains_sv(b, e, "meta", 4)) continue;
                cur = var_of_line(b, e);
                break;
            }
        }
    }
    std::vector<std::vector<std::vector<Entry>>> runs(T, std::vector<std::vector<Entry>>(n > 0 ? n : 1));
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                int cur = start_var[t];
                std::vector<std::pair<const char *, const char *>> tk;
                std::string name;
                for_lines(cut[t], cut[t + 1], [&](const char *b, const char *e) {
                    if (b == e || *b == '#' || icontains_sv(b, e, "meta", 4)) return;
                    if (icontains_sv(b, e, "var ", 4)) {
                        cur = var_of_line(b, e);
                        return;
                    }
                    if (cur < 0) return;
                    tokens(b, e, tk);
                    // atof(tok[0]): strtod stops at the token's end (a space, the
                    // line end or the buffer's NUL) exactly where atof on the copy would
                    const float cost = -1 * std::atof(std::string(tk[0].first, tk[0].second).c_str());
                    uint64_t ps = 0;
                    for (size_t i = 1; i < tk.size(); ++i) {
                        name.assign(tk[i].first, tk[i].second);
                        auto it = index.find(name);
                        ps |= 1ull << (it == index.end() ? 0 : it->second);
                    }
                    runs[t][cur].push_back(Entry{ps, cost});
                });
            });
        for (auto &x : th) x.join();
    }
    // merge per variable in file order: a repeated set keeps its first
    // position and its last value (FloatMap operator[] semantics)
    std::vector<std::vector<uint64_t>> sets(n);
    std::vector<std::vector<float>> costs(n);
    {
        std::atomic<int> next{0};
        std::vector<std::thread> th;
        for (int t = 0; t < std::min(T, std::max(n, 1)); ++t)
            th.emplace_back([&] {
                for (int v = next++; v < n; v = next++) {
                    size_t cnt = 0;
                    for (int c = 0; c < T; ++c) cnt += runs[c][v].size();
                    std::unordered_map<uint64_t, size_t> pos;
                    pos.reserve(cnt * 2);
                    sets[v].reserve(cnt);
                    costs[v].reserve(cnt);
                    for (int c = 0; c < T; ++c)
                        for (const Entry &x : runs[c][v]) {
                            auto ins = pos.emplace(x.set, sets[v].size());
                            if (!ins.second) {
                                costs[v][ins.first->second] = x.cost;
                                continue;
                            }
                            sets[v].push_back(x.set);
                            costs[v].push_back(x.cost);
                        }
                }
            });
        for (auto &x : th) x.join();
    }
    out.offsets.assign(n + 1, 0);
    for (int v = 0; v < n; ++v) out.offsets[v + 1] = out.offsets[v] + (int64_t)sets[v].size();
    out.sets.resize((size_t)out.offsets[n]);
    out.costs.resize((size_t)out.offsets[n]);
    for (int v = 0; v < n; ++v) {
        std::copy(sets[v].begin(), sets[v].end(), out.sets.begin() + out.offsets[v]);
        std::copy(costs[v].begin(), costs[v].end(), out.costs.begin() + out.offsets[v]);
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
