// dem_io.cpp -- DEM ingest: the planner reads its DEM as comma-separated
// text, `array([[float(num) for num in line.split(',')] for line in file])`
// (Coupled_motion_planner.py:1098-1099) -- a Python float() per value, minutes for a 16k^2 DEM.
// Here: the file is read once, cut into line-aligned chunks, and the chunks are parsed by host
// threads with std::from_chars (correctly rounded, like Python's float(), so the values are
// bit-identical).  Host code: no GPU, no context.
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/eikonal.h"

namespace {

thread_local std::string g_io_err;

int io_err(int code, const std::string& msg) {
    g_io_err = msg;
    return code;
}

bool blank(const char* b, const char* e) {
    for (; b < e; ++b)
        if (*b != ' ' && *b != '\t' && *b != '\r') return false;
    return true;
}

// values of one line [b, e): comma-separated, surrounding blanks allowed (Python's float() strips)
int parse_line(const char* b, const char* e, double* out, int64_t want, int64_t* got) {
    int64_t n = 0;
    const char* p = b;
    while (p <= e) {
        const char* q = static_cast<const char*>(memchr(p, ',', (size_t)(e - p)));
        if (!q) q = e;
        const char* s = p;
        const char* t = q;
        while (s < t && (*s == ' ' || *s == '\t')) ++s;
        while (t > s && (t[-1] == ' ' || t[-1] == '\t' || t[-1] == '\r')) --t;
        if (s < t && *s == '+') ++s;  // from_chars does not take a leading '+'
        double v = 0;
        const auto r = std::from_chars(s, t, v);
        if (r.ec == std::errc::result_out_of_range && r.ptr == t) {
            // Python's float() gives +-inf on overflow and 0 / a subnormal on underflow, where
            // from_chars reports the range error: glibc's strtod (correctly rounded too) does that
            const std::string tok(s, t);
            char* end = nullptr;
            v = strtod(tok.c_str(), &end);
            if (end != tok.c_str() + tok.size()) return EIK_ERR_ARG;
        } else if (r.ec != std::errc() || r.ptr != t) {
            return EIK_ERR_ARG;
        }
        if (out && n < want) out[n] = v;
        ++n;
        if (q == e) break;
        p = q + 1;
    }
    *got = n;
    return EIK_OK;
}

}  // namespace

extern "C" {

const char* eik_io_last_error(void) { return g_io_err.c_str(); }

int eik_load_dem_txt(const char* path, double* out, int64_t cap, int64_t* H, int64_t* W, int nthreads) {
    if (!path || !H || !W) return io_err(EIK_ERR_ARG, "NULL argument");
    FILE* f = fopen(path, "rb");
    if (!f) return io_err(EIK_ERR_ARG, std::string("cannot open ") + path);
    std::string buf;
    if (fseek(f, 0, SEEK_END) == 0) {
        const long sz = ftell(f);
        if (sz > 0) {
            buf.resize((size_t)sz);
            fseek(f, 0, SEEK_SET);
            if (fread(&buf[0], 1, (size_t)sz, f) != (size_t)sz) {
                fclose(f);
                return io_err(EIK_ERR_ARG, "short read");
            }
        }
    }
    fclose(f);
    // line starts (trailing blank lines are ignored; the reference would fail on them)
    std::vector<size_t> starts;
    size_t pos = 0;
    const size_t n = buf.size();
    while (pos < n) {
        const char* nl = static_cast<const char*>(memchr(buf.data() + pos, '\n', n - pos));
        const size_t end = nl ? (size_t)(nl - buf.data()) : n;
        if (!blank(buf.data() + pos, buf.data() + end)) starts.push_back(pos);
        pos = end + 1;
    }
    const int64_t rows = (int64_t)starts.size();
    if (rows == 0) return io_err(EIK_ERR_ARG, "empty DEM");
    auto line_end = [&](int64_t r) {
        const char* b = buf.data() + starts[r];
        const char* nl = static_cast<const char*>(memchr(b, '\n', n - starts[r]));
        return nl ? nl : buf.data() + n;
    };
    int64_t cols = 0;
    int rc = parse_line(buf.data() + starts[0], line_end(0), nullptr, 0, &cols);
    if (rc) return io_err(rc, "row 0: not a comma-separated list of numbers");
    *H = rows;
    *W = cols;
    if (!out) return EIK_OK;  // size query
    if (cap < rows * cols) return io_err(EIK_ERR_ARG, "output buffer too small");
    int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
    if (nt < 1) nt = 1;
    if (nt > 64) nt = 64;
    if (nt > rows) nt = (int)rows;
    std::vector<int> status(nt, EIK_OK);
    std::vector<int64_t> bad(nt, -1);
    auto work = [&](int t) {
        for (int64_t r = rows * t / nt; r < rows * (t + 1) / nt; ++r) {
            int64_t got = 0;
            const int e = parse_line(buf.data() + starts[r], line_end(r), out + r * cols, cols, &got);
            if (e || got != cols) {
                status[t] = EIK_ERR_ARG;
                bad[t] = r;
                return;
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (int t = 0; t < nt; ++t)
        if (status[t]) return io_err(EIK_ERR_ARG, "row " + std::to_string(bad[t]) + ": bad number or ragged row");
    return EIK_OK;
}

}  // extern "C"
