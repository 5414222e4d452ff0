// Legacy VTK unstructured-grid reader: the on-disk format behind the reference's
// `vtk_loader_to_torch` (`solver/element.py:39-90`, which goes through pyvista's pv.read). Host code: a file
// is parsed once into points (fp64 [N,3]) and the legacy count-prefixed cell array ([n0, i.., n1, j.., ...],
// what pyvista exposes as `mesh.cells`), plus the VTK cell types.
//
// Supported: "# vtk DataFile Version 2.x-5.x", ASCII or BINARY (big-endian), DATASET UNSTRUCTURED_GRID with
//   POINTS n {float|double|int|...}
//   CELLS n size                  (<= 4.x: count-prefixed int32 array)
//   CELLS n_off n_conn + OFFSETS <type> + CONNECTIVITY <type>   (5.x)
//   CELL_TYPES n
// Anything after CELL_TYPES (POINT_DATA, CELL_DATA, FIELD ...) is ignored. Errors are reported through
// fem_last_error() with FEM_EARG, never by aborting.
#include <algorithm>
#include <cctype>
#include <new>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace fem {
void set_error(const char* fmt, ...);
}

namespace {

struct Reader {
    std::vector<char> buf;
    size_t pos = 0;
    bool binary = false;

    bool eof() const { return pos >= buf.size(); }

    void skip_space() {
        while (pos < buf.size() && std::isspace((unsigned char)buf[pos])) ++pos;
    }

    std::string token() {
        skip_space();
        size_t b = pos;
        while (pos < buf.size() && !std::isspace((unsigned char)buf[pos])) ++pos;
        return std::string(buf.data() + b, pos - b);
    }

    std::string line() {
        size_t b = pos;
        while (pos < buf.size() && buf[pos] != '\n') ++pos;
        std::string s(buf.data() + b, pos - b);
        if (pos < buf.size()) ++pos;
        if (!s.empty() && s.back() == '\r') s.pop_back();
        return s;
    }

    // after a header line in BINARY mode the payload starts right after the line's newline
    void to_next_line() {
        while (pos < buf.size() && buf[pos] != '\n') ++pos;
        if (pos < buf.size()) ++pos;
    }
};

int type_size(const std::string& t, bool* is_float) {
    *is_float = false;
    if (t == "float") {
        *is_float = true;
        return 4;
    }
    if (t == "double") {
        *is_float = true;
        return 8;
    }
    if (t == "int" || t == "unsigned_int" || t == "vtktypeint32") return 4;
    if (t == "long" || t == "unsigned_long" || t == "vtktypeint64" || t == "vtkIdType") return 8;
    if (t == "short" || t == "unsigned_short") return 2;
    if (t == "char" || t == "unsigned_char" || t == "bit") return 1;
    return 0;
}

template <typename T>
T load_be(const char* p) {
    unsigned char b[sizeof(T)];
    for (size_t i = 0; i < sizeof(T); ++i) b[i] = (unsigned char)p[sizeof(T) - 1 - i];
    T v;
    std::memcpy(&v, b, sizeof(T));
    return v;
}

// read `n` values of type `t` as doubles (points) or int64 (indices)
bool read_values(Reader& r, const std::string& t, int64_t n, std::vector<double>* fv, std::vector<int64_t>* iv) {
    bool is_float = false;
    const int sz = type_size(t, &is_float);
    if (!sz) {
        fem::set_error("vtk: unsupported data type '%s'", t.c_str());
        return false;
    }
    if (n < 0 || (uint64_t)n > (uint64_t)(r.buf.size() - std::min(r.pos, r.buf.size()))) {   // >= 1 byte per value
        fem::set_error("vtk: %lld values announced, more than the file holds", (long long)n);
        return false;
    }
    if (fv) fv->resize((size_t)n);
    if (iv) iv->resize((size_t)n);
    if (r.binary) {
        r.to_next_line();
        if (r.pos + (size_t)n * sz > r.buf.size()) {
            fem::set_error("vtk: binary block of %lld x %d bytes runs past the end of the file", (long long)n, sz);
            return false;
        }
        const char* p = r.buf.data() + r.pos;
        const bool uns = t.rfind("unsigned", 0) == 0;
        auto put = [&](int64_t i, double d, int64_t k) {
            if (fv) (*fv)[(size_t)i] = d;
            if (iv) (*iv)[(size_t)i] = k;
        };
        // one tight loop per stored type (the type test is hoisted out of the element loop)
        if (is_float && sz == 8) {
            for (int64_t i = 0; i < n; ++i) { const double d = load_be<double>(p + 8 * i); put(i, d, (int64_t)d); }
        } else if (is_float) {
            for (int64_t i = 0; i < n; ++i) { const double d = load_be<float>(p + 4 * i); put(i, d, (int64_t)d); }
        } else if (sz == 8) {
            for (int64_t i = 0; i < n; ++i) {
                const int64_t k = uns ? (int64_t)load_be<uint64_t>(p + 8 * i) : load_be<int64_t>(p + 8 * i);
                put(i, (double)k, k);
            }
        } else if (sz == 4) {
            for (int64_t i = 0; i < n; ++i) {
                const int64_t k = uns ? (int64_t)load_be<uint32_t>(p + 4 * i) : (int64_t)load_be<int32_t>(p + 4 * i);
                put(i, (double)k, k);
            }
        } else if (sz == 2) {
            for (int64_t i = 0; i < n; ++i) {
                const int64_t k = uns ? (int64_t)load_be<uint16_t>(p + 2 * i) : (int64_t)load_be<int16_t>(p + 2 * i);
                put(i, (double)k, k);
            }
        } else {
            for (int64_t i = 0; i < n; ++i) {
                const int64_t k = uns ? (int64_t)(unsigned char)p[i] : (int64_t)(signed char)p[i];
                put(i, (double)k, k);
            }
        }
        r.pos += (size_t)n * sz;
        return true;
    }
    for (int64_t i = 0; i < n; ++i) {
        const std::string s = r.token();
        if (s.empty()) {
            fem::set_error("vtk: file ends after %lld of %lld values", (long long)i, (long long)n);
            return false;
        }
        char* end = nullptr;
        if (fv) {
            double d = std::strtod(s.c_str(), &end);
            if (*end) {
                fem::set_error("vtk: bad number '%s'", s.c_str());
                return false;
            }
            if (is_float && sz == 4) d = (double)(float)d;   // a `float` array holds float32 values (VTK)
            (*fv)[(size_t)i] = d;
        }
        if (iv) {
            const long long k = std::strtoll(s.c_str(), &end, 10);
            if (*end) {
                fem::set_error("vtk: bad integer '%s'", s.c_str());
                return false;
            }
            (*iv)[(size_t)i] = k;
        }
    }
    return true;
}

std::string upper(std::string s) {
    for (auto& c : s) c = (char)std::toupper((unsigned char)c);
    return s;
}

}  // namespace

struct fem_vtk {
    std::vector<double> points;   // [3 n_points]
    std::vector<int64_t> cells;   // legacy count-prefixed array
    std::vector<int64_t> types;   // [n_cells]
    int64_t n_cells = 0;
};

extern "C" {

static int vtk_read(const char* path, fem_vtk** out);

int fem_vtk_read(const char* path, fem_vtk** out) {
    *out = nullptr;
    try {
        return vtk_read(path, out);
    } catch (const std::bad_alloc&) {
        fem::set_error("vtk: out of host memory reading '%s'", path);
        return 5;
    }
}

static int vtk_read(const char* path, fem_vtk** out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        fem::set_error("vtk: cannot open '%s'", path);
        return 5;
    }
    Reader r;
    std::fseek(f, 0, SEEK_END);
    const long len = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    r.buf.resize(len > 0 ? (size_t)len : 0);
    const size_t got = len > 0 ? std::fread(r.buf.data(), 1, (size_t)len, f) : 0;
    std::fclose(f);
    if ((long)got != len) {
        fem::set_error("vtk: short read on '%s'", path);
        return 5;
    }
    const std::string magic = r.line();
    if (magic.rfind("# vtk DataFile Version", 0) != 0) {
        fem::set_error("vtk: '%s' is not a legacy VTK file (header '%s')", path, magic.c_str());
        return 5;
    }
    double version = 0;
    std::sscanf(magic.c_str() + std::strlen("# vtk DataFile Version"), "%lf", &version);
    (void)r.line();   // title
    const std::string mode = upper(r.token());
    if (mode != "ASCII" && mode != "BINARY") {
        fem::set_error("vtk: expected ASCII or BINARY, got '%s'", mode.c_str());
        return 5;
    }
    r.binary = mode == "BINARY";
    fem_vtk* v = new fem_vtk();
    bool have_points = false, have_cells = false;
    int64_t n_points = 0;
    auto fail = [&]() {
        delete v;
        return 5;
    };
    while (true) {
        const std::string kw = upper(r.token());
        if (kw.empty()) break;
        if (kw == "DATASET") {
            const std::string ds = upper(r.token());
            if (ds != "UNSTRUCTURED_GRID") {
                fem::set_error("vtk: dataset '%s' is not supported (UNSTRUCTURED_GRID only)", ds.c_str());
                return fail();
            }
        } else if (kw == "POINTS") {
            n_points = std::strtoll(r.token().c_str(), nullptr, 10);
            const std::string t = r.token();
            if (n_points < 0 || !read_values(r, t, 3 * n_points, &v->points, nullptr)) return fail();
            have_points = true;
        } else if (kw == "CELLS") {
            const int64_t a = std::strtoll(r.token().c_str(), nullptr, 10);
            const int64_t b = std::strtoll(r.token().c_str(), nullptr, 10);
            if (version < 5.0) {
                v->n_cells = a;
                if (a < 0 || b < 0 || !read_values(r, "int", b, nullptr, &v->cells)) return fail();
            } else {
                // OFFSETS <type> (a values) then CONNECTIVITY <type> (b values)
                std::vector<int64_t> off, conn;
                if (upper(r.token()) != "OFFSETS") {
                    fem::set_error("vtk 5.x: OFFSETS expected after CELLS");
                    return fail();
                }
                const std::string to = r.token();
                if (!read_values(r, to, a, nullptr, &off)) return fail();
                if (upper(r.token()) != "CONNECTIVITY") {
                    fem::set_error("vtk 5.x: CONNECTIVITY expected after OFFSETS");
                    return fail();
                }
                const std::string tc = r.token();
                if (!read_values(r, tc, b, nullptr, &conn)) return fail();
                v->n_cells = a > 0 ? a - 1 : 0;
                v->cells.reserve((size_t)(v->n_cells + b));
                for (int64_t c = 0; c < v->n_cells; ++c) {
                    const int64_t o0 = off[(size_t)c], o1 = off[(size_t)c + 1];
                    if (o0 < 0 || o1 < o0 || o1 > b) {
                        fem::set_error("vtk 5.x: bad OFFSETS entry %lld", (long long)c);
                        return fail();
                    }
                    v->cells.push_back(o1 - o0);
                    for (int64_t k = o0; k < o1; ++k) v->cells.push_back(conn[(size_t)k]);
                }
            }
            have_cells = true;
        } else if (kw == "CELL_TYPES") {
            const int64_t n = std::strtoll(r.token().c_str(), nullptr, 10);
            if (n < 0 || !read_values(r, "int", n, nullptr, &v->types)) return fail();
            break;   // the geometry is complete; attribute sections are not needed
        } else if (kw == "METADATA") {
            // 5.x metadata block: the keyword's line, then lines up to the first blank one
            (void)r.line();
            while (!r.eof()) {
                const std::string l = r.line();
                if (l.find_first_not_of(" \t") == std::string::npos) break;
            }
        } else if (kw == "POINT_DATA" || kw == "CELL_DATA" || kw == "FIELD") {
            break;
        } else {
            fem::set_error("vtk: unexpected keyword '%s'", kw.c_str());
            return fail();
        }
    }
    if (!have_points || !have_cells) {
        fem::set_error("vtk: '%s' lacks %s", path, have_points ? "CELLS" : "POINTS");
        return fail();
    }
    // validate the count-prefixed walk and the node ids
    size_t p = 0;
    for (int64_t c = 0; c < v->n_cells; ++c) {
        if (p >= v->cells.size() || v->cells[p] < 0 || p + 1 + (size_t)v->cells[p] > v->cells.size()) {
            fem::set_error("vtk: cell array is inconsistent at cell %lld", (long long)c);
            return fail();
        }
        for (int64_t k = 1; k <= v->cells[p]; ++k)
            if (v->cells[p + k] < 0 || v->cells[p + k] >= n_points) {
                fem::set_error("vtk: cell %lld references point %lld of %lld", (long long)c,
                               (long long)v->cells[p + k], (long long)n_points);
                return fail();
            }
        p += 1 + (size_t)v->cells[p];
    }
    *out = v;
    return 0;
}

int fem_vtk_sizes(const fem_vtk* v, int64_t* n_points, int64_t* n_cells, int64_t* cells_len, int64_t* n_types) {
    *n_points = (int64_t)v->points.size() / 3;
    *n_cells = v->n_cells;
    *cells_len = (int64_t)v->cells.size();
    *n_types = (int64_t)v->types.size();
    return 0;
}

int fem_vtk_copy(const fem_vtk* v, double* points, int64_t* cells, int64_t* types) {
    if (points && !v->points.empty()) std::memcpy(points, v->points.data(), v->points.size() * sizeof(double));
    if (cells && !v->cells.empty()) std::memcpy(cells, v->cells.data(), v->cells.size() * sizeof(int64_t));
    if (types && !v->types.empty()) std::memcpy(types, v->types.data(), v->types.size() * sizeof(int64_t));
    return 0;
}

void fem_vtk_free(fem_vtk* v) { delete v; }

}  // extern "C"
