// Keypoints TSV rows (ResultWriterStep.__process_csv,
// M/pipeline/write_results_step.py:54-73, which writes them with
// pandas.DataFrame.to_csv(sep="\t", index=False)) formatted natively, so the
// result writer's thread formats a chunk without holding the Python GIL.
// The bytes are pandas': float64 fields are Python's repr of the value (the
// shortest string that round-trips: std::to_chars' shortest scientific
// digits, laid out positionally for 1e-4 <= |x| < 1e16 and as d.ddde+XX
// otherwise), NaN an empty field, bools True / False, integers decimal.
#include <charconv>
#include <cmath>
#include <cstring>

#include "common.h"

namespace {

// Python repr of a finite or infinite double (NaN handled by the caller)
int repr_double(double x, char *o) {
    if (std::isinf(x)) {
        const char *s = x < 0 ? "-inf" : "inf";
        const int n = (int)std::strlen(s);
        std::memcpy(o, s, n);
        return n;
    }
    char sci[40];
    const auto r = std::to_chars(sci, sci + sizeof(sci), x, std::chars_format::scientific);
    const char *p = sci, *end = r.ptr;
    int n = 0;
    if (*p == '-') {
        o[n++] = '-';
        ++p;
    }
    char dig[24];
    int nd = 0;
    while (p < end && *p != 'e') {
        if (*p != '.') dig[nd++] = *p;
        ++p;
    }
    int e10 = 0;  // "e+16" / "e-05" (to_chars writes no terminating NUL)
    if (p < end) {
        const bool neg = p[1] == '-';
        for (const char *q = p + 2; q < end; ++q) e10 = 10 * e10 + (*q - '0');
        if (neg) e10 = -e10;
    }
    const int decpt = e10 + 1;            // digits d1 d2 ... with the point after decpt of them
    if (decpt <= -4 || decpt > 16) {      // d[.ddd]e+XX (two exponent digits at least)
        o[n++] = dig[0];
        if (nd > 1) {
            o[n++] = '.';
            std::memcpy(o + n, dig + 1, nd - 1);
            n += nd - 1;
        }
        o[n++] = 'e';
        o[n++] = e10 < 0 ? '-' : '+';
        const int ae = e10 < 0 ? -e10 : e10;
        if (ae < 10) o[n++] = '0';
        const auto re = std::to_chars(o + n, o + n + 8, ae);
        n = (int)(re.ptr - o);
    } else if (decpt <= 0) {  // 0.000ddd
        o[n++] = '0';
        o[n++] = '.';
        for (int i = 0; i < -decpt; ++i) o[n++] = '0';
        std::memcpy(o + n, dig, nd);
        n += nd;
    } else if (decpt < nd) {  // ddd.ddd
        std::memcpy(o + n, dig, decpt);
        n += decpt;
        o[n++] = '.';
        std::memcpy(o + n, dig + decpt, nd - decpt);
        n += nd - decpt;
    } else {  // ddd000.0
        std::memcpy(o + n, dig, nd);
        n += nd;
        for (int i = nd; i < decpt; ++i) o[n++] = '0';
        o[n++] = '.';
        o[n++] = '0';
    }
    return n;
}

}  // namespace

extern "C" int64_t mdx_format_tsv_rows(const void *const *cols, const int *kinds, int ncols, int64_t nrows, char *out,
                                       int64_t cap) {
    MDX_REQUIRE(cols && kinds && out && ncols > 0 && nrows >= 0, "mdx_format_tsv_rows: bad arguments");
    for (int c = 0; c < ncols; ++c)
        MDX_REQUIRE(cols[c] && kinds[c] >= 0 && kinds[c] <= 2, "mdx_format_tsv_rows: column %d: bad pointer or kind",
                    c);
    int64_t n = 0;
    constexpr int FIELD = 40;  // longest field: "-1.2345678901234567e-308" (24) / an int64 (20)
    for (int64_t r = 0; r < nrows; ++r) {
        MDX_REQUIRE(n + (int64_t)ncols * FIELD + 1 <= cap, "mdx_format_tsv_rows: output buffer too small");
        for (int c = 0; c < ncols; ++c) {
            if (c) out[n++] = '\t';
            if (kinds[c] == 0) {
                const double v = reinterpret_cast<const double *>(cols[c])[r];
                if (!std::isnan(v)) n += repr_double(v, out + n);
            } else if (kinds[c] == 1) {
                const bool v = reinterpret_cast<const uint8_t *>(cols[c])[r] != 0;
                const char *s = v ? "True" : "False";
                const int l = v ? 4 : 5;
                std::memcpy(out + n, s, l);
                n += l;
            } else {
                const auto re = std::to_chars(out + n, out + n + 24, reinterpret_cast<const int64_t *>(cols[c])[r]);
                n = re.ptr - out;
            }
        }
        out[n++] = '\n';
    }
    return n;
}
