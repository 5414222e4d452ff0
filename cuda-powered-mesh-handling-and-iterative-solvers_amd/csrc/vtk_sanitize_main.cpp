// Host sanitizer harness for the legacy-VTK reader (vtk.cpp), SURVEY.md §5 ("-fsanitize=address host builds"):
// `make -C csrc vtk-asan` links vtk.cpp with this driver under AddressSanitizer + UndefinedBehaviorSanitizer
// (g++, host code only -- no GPU code is involved). For every path on the command line it runs the reader exactly as
// the library's C-ABI does for `element.read_vtk` (fem_vtk_read -> fem_vtk_sizes -> fem_vtk_copy -> fem_vtk_free) and
// prints one line:  <rc> <n_points> <n_cells> <cells_len> <n_types> <checksum> | <error message>
// tests/test_vtk_sanitize.py writes the reader's round-trip and malformed files and checks the lines and that the
// sanitizers reported nothing (any report aborts the process with a non-zero status).
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../include/fem355.h"

namespace fem {
static char g_err[1024];
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace fem

extern "C" const char* fem_last_error(void) { return fem::g_err; }

// the message on one printable line (file bytes quoted in it may be anything)
static const char* printable(const char* m) {
    static char out[sizeof(fem::g_err)];
    size_t k = 0;
    for (; m[k] && k + 1 < sizeof(out); ++k) out[k] = (m[k] >= 32 && m[k] < 127) ? m[k] : '?';
    out[k] = 0;
    return out;
}

int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
        fem::g_err[0] = 0;
        fem_vtk* v = nullptr;
        const int rc = fem_vtk_read(argv[i], &v);
        if (rc != FEM_OK) {
            std::printf("%d 0 0 0 0 0 | %s\n", rc, printable(fem_last_error()));
            continue;
        }
        int64_t np = 0, nc = 0, nl = 0, nt = 0;
        fem_vtk_sizes(v, &np, &nc, &nl, &nt);
        std::vector<double> pts((size_t)(np * 3));
        std::vector<int64_t> cells((size_t)nl), types((size_t)nt);
        const int rc2 = fem_vtk_copy(v, pts.data(), cells.data(), types.data());
        fem_vtk_free(v);
        // order-sensitive checksum of everything the reader returned
        double cs = 0.0;
        for (size_t k = 0; k < pts.size(); ++k) cs = cs * 1.000001 + pts[k];
        for (size_t k = 0; k < cells.size(); ++k) cs = cs * 1.000001 + (double)cells[k];
        for (size_t k = 0; k < types.size(); ++k) cs = cs * 1.000001 + (double)types[k];
        std::printf("%d %lld %lld %lld %lld %.17g | %s\n", rc2, (long long)np, (long long)nc, (long long)nl,
                    (long long)nt, cs, printable(fem_last_error()));
    }
    return 0;
}
