// mmio.hip — native MatrixMarket reader (host code): the `.mtx` -> CSR path the reference takes with
// scipy.io.mmread(path).tocsr() (examples/DHTestProblem.py:27-28) for the TestMatrices/DH-Matrix-*.mtx
// inputs of configs[0] (and any coordinate file).
//
// Result = mmread(...).tocsr(): coordinate entries, symmetric / skew-symmetric files expanded to both
// triangles (diagonal once, skew mirrored negated), pattern entries 1.0, integer entries as f64; rows
// sorted by column and duplicate entries summed (COO -> CSR canonicalisation), explicit zeros kept.
// Values are parsed with strtod (correctly rounded, as the reference's reader).
#include "psk_internal.hpp"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <string>
#include <vector>

namespace psk {
namespace {

struct MMFile {
    int64_t nrows = 0, ncols = 0, entries = 0;
    enum Field { kReal, kInteger, kPattern } field = kReal;
    enum Sym { kGeneral, kSymmetric, kSkew } sym = kGeneral;
    std::string text;   // whole file
    size_t body = 0;    // offset of the first entry line
};

std::string lower(std::string s) {
    for (auto &ch : s) ch = (char)std::tolower((unsigned char)ch);
    return s;
}

int mm_open(const char *path, MMFile &f) {
    if (!path) return fail(PSK_ERR_ARG, "MatrixMarket: NULL path");
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return fail(PSK_ERR_ARG, std::string("MatrixMarket: cannot open ") + path);
    std::fseek(fp, 0, SEEK_END);
    const long sz = std::ftell(fp);
    std::fseek(fp, 0, SEEK_SET);
    f.text.resize(sz > 0 ? (size_t)sz : 0);
    const size_t got = sz > 0 ? std::fread(&f.text[0], 1, (size_t)sz, fp) : 0;
    std::fclose(fp);
    if ((long)got != sz) return fail(PSK_ERR_ARG, std::string("MatrixMarket: short read of ") + path);
    size_t pos = 0;
    auto next_line = [&](std::string &line) {
        if (pos >= f.text.size()) return false;
        size_t e = f.text.find('\n', pos);
        if (e == std::string::npos) e = f.text.size();
        line.assign(f.text, pos, e - pos);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        pos = e + 1;
        return true;
    };
    std::string line;
    if (!next_line(line)) return fail(PSK_ERR_ARG, "MatrixMarket: empty file");
    char b[5][64] = {};
    if (std::sscanf(line.c_str(), "%63s %63s %63s %63s %63s", b[0], b[1], b[2], b[3], b[4]) != 5 ||
        lower(b[0]) != "%%matrixmarket" || lower(b[1]) != "matrix")
        return fail(PSK_ERR_ARG, "MatrixMarket: bad banner");
    if (lower(b[2]) != "coordinate") return fail(PSK_ERR_UNSUPPORTED, "MatrixMarket: only coordinate format");
    const std::string fld = lower(b[3]), sym = lower(b[4]);
    if (fld == "real" || fld == "double") f.field = MMFile::kReal;
    else if (fld == "integer") f.field = MMFile::kInteger;
    else if (fld == "pattern") f.field = MMFile::kPattern;
    else return fail(PSK_ERR_UNSUPPORTED, "MatrixMarket: field " + fld + " not supported (real/integer/pattern)");
    if (sym == "general") f.sym = MMFile::kGeneral;
    else if (sym == "symmetric") f.sym = MMFile::kSymmetric;
    else if (sym == "skew-symmetric") f.sym = MMFile::kSkew;
    else return fail(PSK_ERR_UNSUPPORTED, "MatrixMarket: symmetry " + sym + " not supported");
    while (next_line(line)) {
        size_t k = line.find_first_not_of(" \t");
        if (k == std::string::npos || line[k] == '%') continue;
        long long r = 0, c = 0, e = 0;
        if (std::sscanf(line.c_str(), "%lld %lld %lld", &r, &c, &e) != 3 || r < 0 || c < 0 || e < 0)
            return fail(PSK_ERR_ARG, "MatrixMarket: bad size line");
        f.nrows = r;
        f.ncols = c;
        f.entries = e;
        f.body = pos;
        // an entry takes at least 4 bytes ("r c\n"; 3 on an unterminated last line): a size line
        // claiming more entries than the body can hold is refused here, before anything is sized
        // from it (scripts/asan_host.sh: a 9e18-entry header made the reserve below throw through
        // the C ABI)
        if (e > (long long)((pos < f.text.size() ? f.text.size() - pos : 0) / 3 + 1))
            return fail(PSK_ERR_ARG, "MatrixMarket: fewer entries than the size line says");
        if (r >= INT32_MAX || c >= INT32_MAX) return fail(PSK_ERR_UNSUPPORTED, "MatrixMarket: int32 CSR required");
        return PSK_OK;
    }
    return fail(PSK_ERR_ARG, "MatrixMarket: missing size line");
}

int64_t nnz_max(const MMFile &f) { return f.sym == MMFile::kGeneral ? f.entries : 2 * f.entries; }

// parse the entries into expanded COO
int mm_coo(const MMFile &f, std::vector<int64_t> &ri, std::vector<int64_t> &ci, std::vector<double> &va) {
    ri.reserve(nnz_max(f));
    ci.reserve(nnz_max(f));
    va.reserve(nnz_max(f));
    const char *p = f.text.c_str() + f.body, *end = f.text.c_str() + f.text.size();
    int64_t seen = 0;
    while (p < end && seen < f.entries) {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
        if (p >= end) break;
        if (*p == '%') {   // comment line inside the body
            while (p < end && *p != '\n') ++p;
            continue;
        }
        char *q;
        const long long r = std::strtoll(p, &q, 10);
        if (q == p) return fail(PSK_ERR_ARG, "MatrixMarket: bad entry (row)");
        p = q;
        const long long c = std::strtoll(p, &q, 10);
        if (q == p) return fail(PSK_ERR_ARG, "MatrixMarket: bad entry (column)");
        p = q;
        double v = 1.0;
        if (f.field != MMFile::kPattern) {
            v = std::strtod(p, &q);
            if (q == p) return fail(PSK_ERR_ARG, "MatrixMarket: bad entry (value)");
            p = q;
        }
        while (p < end && *p != '\n') ++p;   // ignore anything else on the line
        if (r < 1 || r > f.nrows || c < 1 || c > f.ncols) return fail(PSK_ERR_ARG, "MatrixMarket: index out of range");
        ri.push_back(r - 1);
        ci.push_back(c - 1);
        va.push_back(v);
        if (f.sym != MMFile::kGeneral && r != c) {
            ri.push_back(c - 1);
            ci.push_back(r - 1);
            va.push_back(f.sym == MMFile::kSkew ? -v : v);
        }
        ++seen;
    }
    if (seen != f.entries) return fail(PSK_ERR_ARG, "MatrixMarket: fewer entries than the size line says");
    return PSK_OK;
}

// COO -> canonical CSR (per-row column sort, duplicates summed in stored order after the sort)
int mm_csr(const MMFile &f, std::vector<int32_t> &rp, std::vector<int32_t> &cols, std::vector<double> &vals) {
    if (f.nrows >= INT32_MAX || f.ncols >= INT32_MAX || nnz_max(f) > kMaxNnz)
        return fail(PSK_ERR_UNSUPPORTED, "MatrixMarket: int32 CSR required");
    std::vector<int64_t> ri, ci;
    std::vector<double> va;
    PSK_TRY(mm_coo(f, ri, ci, va));
    const int64_t n = f.nrows, m = (int64_t)ri.size();
    std::vector<int64_t> cnt(n + 1, 0);
    for (int64_t k = 0; k < m; ++k) cnt[ri[k] + 1]++;
    for (int64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    std::vector<int64_t> perm(m), fillp(cnt.begin(), cnt.end() - 1);
    for (int64_t k = 0; k < m; ++k) perm[fillp[ri[k]]++] = k;   // stable: file order within a row
    rp.assign(n + 1, 0);
    cols.clear();
    vals.clear();
    cols.reserve(m);
    vals.reserve(m);
    for (int64_t i = 0; i < n; ++i) {
        auto b = perm.begin() + cnt[i], e = perm.begin() + cnt[i + 1];
        std::stable_sort(b, e, [&](int64_t x, int64_t y) { return ci[x] < ci[y]; });
        for (auto it = b; it != e; ++it) {
            if (it != b && ci[*it] == cols.back()) {
                vals.back() += va[*it];
                continue;
            }
            cols.push_back((int32_t)ci[*it]);
            vals.push_back(va[*it]);
        }
        rp[i + 1] = (int32_t)cols.size();
    }
    return PSK_OK;
}

}  // namespace
}  // namespace psk

using namespace psk;

extern "C" int psk_mm_info(const char *path, int64_t *nrows, int64_t *ncols, int64_t *nnz_max_out) {
    MMFile f;
    PSK_TRY(mm_open(path, f));
    if (nrows) *nrows = f.nrows;
    if (ncols) *ncols = f.ncols;
    if (nnz_max_out) *nnz_max_out = nnz_max(f);
    return PSK_OK;
}

extern "C" int psk_mm_read(const char *path, int32_t *rowptr, int32_t *colidx, double *vals, int64_t *nnz) {
    if (!rowptr || !nnz) return fail(PSK_ERR_ARG, "psk_mm_read: NULL argument");
    MMFile f;
    PSK_TRY(mm_open(path, f));
    std::vector<int32_t> rp, cols;
    std::vector<double> va;
    PSK_TRY(mm_csr(f, rp, cols, va));
    std::copy(rp.begin(), rp.end(), rowptr);
    if (!cols.empty() && (!colidx || !vals)) return fail(PSK_ERR_ARG, "psk_mm_read: NULL colidx/vals");
    std::copy(cols.begin(), cols.end(), colidx);
    std::copy(va.begin(), va.end(), vals);
    *nnz = (int64_t)cols.size();
    return PSK_OK;
}

extern "C" int psk_csr_create_mm(const char *path, psk_csr **out) {
    if (!out) return fail(PSK_ERR_ARG, "psk_csr_create_mm: NULL out");
    MMFile f;
    PSK_TRY(mm_open(path, f));
    std::vector<int32_t> rp, cols;
    std::vector<double> va;
    PSK_TRY(mm_csr(f, rp, cols, va));
    return psk_csr_create_rect(f.nrows, f.ncols, (int64_t)cols.size(), rp.data(), cols.data(), va.data(), PSK_HOST,
                               out);
}
