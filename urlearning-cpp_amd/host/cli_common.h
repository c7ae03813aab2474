// cli_common.h -- boost::program_options-like argument handling shared by the
// command lines (short "-x v" / "-xv", long "--name v" / "--name=v", and
// positional arguments).
#pragma once

#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace ulgcli {

struct Opt {
    std::string shortname, longname;
    bool takes_value;
    std::string def;
    std::string help;
};

class Args {
public:
    Args(std::vector<Opt> opts, std::vector<std::string> positional) : opts_(std::move(opts)), pos_names_(std::move(positional)) {}

    bool parse(int argc, char **argv, std::string &err) {
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i];
            if (a.size() > 1 && a[0] == '-') {
                const Opt *o = nullptr;
                std::string val;
                bool has_val = false;
                if (a[1] == '-') {
                    std::string name = a.substr(2);
                    const size_t eq = name.find('=');
                    if (eq != std::string::npos) {
                        val = name.substr(eq + 1);
                        name = name.substr(0, eq);
                        has_val = true;
                    }
                    for (const Opt &x : opts_)
                        if (x.longname == name) o = &x;
                } else {
                    const std::string name = a.substr(1, 1);
                    for (const Opt &x : opts_)
                        if (x.shortname == name) o = &x;
                    if (o && a.size() > 2) {
                        val = a.substr(2);
                        has_val = true;
                    }
                }
                if (!o) {
                    err = "unrecognised option '" + a + "'";
                    return false;
                }
                if (o->takes_value && !has_val) {
                    if (i + 1 >= argc) {
                        err = "the required argument for option '--" + o->longname + "' is missing";
                        return false;
                    }
                    val = argv[++i];
                }
                vals_[o->longname] = o->takes_value ? val : "1";
                seen_.insert(o->longname);
            } else {
                if (pos_.size() >= pos_names_.size()) {
                    err = "too many positional options";
                    return false;
                }
                pos_.push_back(a);
            }
        }
        for (size_t i = 0; i < pos_.size(); ++i) {
            vals_[pos_names_[i]] = pos_[i];
            seen_.insert(pos_names_[i]);
        }
        return true;
    }
    bool has(const std::string &name) const { return seen_.count(name) > 0; }
    std::string get(const std::string &name) const {
        auto it = vals_.find(name);
        if (it != vals_.end()) return it->second;
        for (const Opt &o : opts_)
            if (o.longname == name) return o.def;
        return "";
    }
    void usage(const char *prog, const char *what) const {
        std::printf("%s\nUsage: %s", what, prog);
        for (const std::string &p : pos_names_) std::printf(" <%s>", p.c_str());
        std::printf(" [options]\n");
        for (const Opt &o : opts_)
            std::printf("  %s%s--%s%s  %s%s\n", o.shortname.empty() ? "" : "-", o.shortname.empty() ? "" : (o.shortname + " [ ").c_str(),
                        o.longname.c_str(), o.shortname.empty() ? "" : " ]", o.help.c_str(),
                        o.def.empty() ? "" : (" (=" + o.def + ")").c_str());
    }

private:
    std::vector<Opt> opts_;
    std::vector<std::string> pos_names_;
    std::vector<std::string> pos_;
    std::map<std::string, std::string> vals_;
    std::set<std::string> seen_;
};

// setFromCsv (typedefs.h:737-754): comma-separated variable indices, split
// with adjacent separators compressed; a token that atoi reads as 0 without
// starting with '0' (an empty leading/trailing token included) is an error.
inline bool set_from_csv(const std::string &csv, uint64_t &vs) {
    if (csv.empty()) return true;
    size_t i = 0;
    while (true) {
        size_t j = csv.find(',', i);
        const std::string tok = csv.substr(i, j == std::string::npos ? std::string::npos : j - i);
        const int var = std::atoi(tok.c_str());
        if ((var == 0 && (tok.empty() || tok[0] != '0')) || var < 0 || var >= 64) return false;
        vs |= 1ull << var;
        if (j == std::string::npos) break;
        while (j < csv.size() && csv[j] == ',') ++j;
        i = j;
    }
    return true;
}

inline double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace ulgcli
