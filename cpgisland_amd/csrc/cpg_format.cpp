// cpg_format.cpp — the reference's byte-exact text outputs, host side:
//   * island lines  String.format("%d %d %d %f %f\n", ...)   CpGIslandFinder.java:287-288
//   * trained model Double.toString(x) per value, " " after every matrix entry,
//                   newLine() after each row group                          :207-224
// Java renders a double from its shortest round-tripping decimal digits (FloatingDecimal /
// Double.toString); %f then rounds those digits HALF_UP to 6 fraction digits (not the exact
// binary value, as C's printf does).  The digits come from std::to_chars (shortest
// round-trip); locale: root ('.' separator).

#include <charconv>
#include <cmath>
#include <cstring>
#include <string>

#include "cpg_internal.h"

namespace {

// shortest round-trip digits of |x| (x finite, != 0): value = 0.d1d2...dn x 10^e10
void shortest(double x, std::string& digits, int& e10) {
    char b[64];
    const auto r = std::to_chars(b, b + sizeof b, std::fabs(x), std::chars_format::scientific);
    *r.ptr = 0;
    digits.clear();
    const char* p = b;
    for (; *p && *p != 'e'; ++p)
        if (*p >= '0' && *p <= '9') digits.push_back(*p);
    e10 = std::atoi(p + 1) + 1;   // d.ddd e X  ->  0.dddd x 10^(X+1)
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
}

// java.util.Formatter "%f": shortest digits rounded HALF_UP to 6 fraction digits
std::string java_f6(double x) {
    if (std::isnan(x)) return "NaN";
    if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
    std::string out = std::signbit(x) ? "-" : "";
    if (x == 0.0) return out + "0.000000";
    std::string d;
    int e;
    shortest(x, d, e);
    // fixed digits: integer part (at least "0"), then fraction digits
    std::string ip, fp;
    if (e > 0) {
        for (int k = 0; k < e; ++k) ip.push_back(k < (int)d.size() ? d[k] : '0');
        if ((int)d.size() > e) fp = d.substr(e);
    } else {
        ip = "0";
        fp.assign(-e, '0');
        fp += d;
    }
    if (fp.size() > 6) {
        const bool up = fp[6] >= '5';
        fp.resize(6);
        if (up) {   // carry through fraction and integer digits
            std::string all = ip + fp;
            int k = (int)all.size() - 1;
            for (; k >= 0; --k) {
                if (all[k] == '9') {
                    all[k] = '0';
                } else {
                    ++all[k];
                    break;
                }
            }
            if (k < 0) all.insert(all.begin(), '1');
            ip = all.substr(0, all.size() - 6);
            fp = all.substr(all.size() - 6);
        }
    }
    fp.resize(6, '0');
    return out + ip + "." + fp;
}

// Double.toString: decimal for 1e-3 <= |x| < 1e7, else d.dddE[-]n; at least one fraction digit
std::string java_dtoa(double x) {
    if (std::isnan(x)) return "NaN";
    if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
    std::string out = std::signbit(x) ? "-" : "";
    if (x == 0.0) return out + "0.0";
    std::string d;
    int e;
    shortest(x, d, e);
    const double ax = std::fabs(x);
    if (ax >= 1e-3 && ax < 1e7) {
        std::string ip, fp;
        if (e > 0) {
            for (int k = 0; k < e; ++k) ip.push_back(k < (int)d.size() ? d[k] : '0');
            if ((int)d.size() > e) fp = d.substr(e);
        } else {
            ip = "0";
            fp.assign(-e, '0');
            fp += d;
        }
        if (fp.empty()) fp = "0";
        return out + ip + "." + fp;
    }
    std::string m = d.substr(0, 1) + "." + (d.size() > 1 ? d.substr(1) : std::string("0"));
    return out + m + "E" + std::to_string(e - 1);
}

int put(std::string& acc, char* buf, int64_t cap, int64_t* nbytes) {
    *nbytes = (int64_t)acc.size();
    if ((int64_t)acc.size() > cap)
        return cpg::set_error(CPG_E_CAPACITY, "text needs %lld bytes", (long long)acc.size());
    if (!acc.empty()) std::memcpy(buf, acc.data(), acc.size());
    return CPG_OK;
}

}  // namespace

extern "C" {

int cpg_format_islands(const cpg_island* recs, int64_t n, char* buf, int64_t cap,
                       int64_t* nbytes) {
    if (!nbytes || n < 0 || (n > 0 && !recs) || (cap > 0 && !buf) || cap < 0)
        return cpg::set_error(CPG_E_INVALID, "cpg_format_islands: bad argument");
    std::string acc;
    acc.reserve((size_t)n * 48);
    for (int64_t i = 0; i < n; ++i) {
        const cpg_island& r = recs[i];
        acc += std::to_string(r.beg1);
        acc += ' ';
        acc += std::to_string(r.end1);
        acc += ' ';
        acc += std::to_string(r.len);
        acc += ' ';
        acc += java_f6(r.cg);
        acc += ' ';
        acc += java_f6(r.oe);
        acc += '\n';
    }
    return put(acc, buf, cap, nbytes);
}

int cpg_format_model(const cpg_model* m, char* buf, int64_t cap, int64_t* nbytes) {
    if (!m || !nbytes || (cap > 0 && !buf) || cap < 0)
        return cpg::set_error(CPG_E_INVALID, "cpg_format_model: bad argument");
    std::string acc;
    for (int i = 0; i < 8; ++i) {
        acc += java_dtoa(m->pi[i]);
        acc += '\n';
        for (int j = 0; j < 8; ++j) {
            acc += java_dtoa(m->a[i][j]);
            acc += ' ';
        }
        acc += '\n';
        for (int k = 0; k < 4; ++k) {
            acc += java_dtoa(m->b[i][k]);
            acc += ' ';
        }
        acc += '\n';
    }
    return put(acc, buf, cap, nbytes);
}

}  // extern "C"
