/* Probe and layout-experiment kernels (tools/lab/libfem355_lab.so). NOT part of the product library: these
 * entry points measured layout and memory-system questions whose answers shaped the production kernels
 * (DESIGN.md §4, §8b, §8c). The library links against libfem355.so for its error plumbing. */
#pragma once
#include <stdint.h>

#include "../../include/fem355.h"

#ifdef __cplusplus
extern "C" {
#endif

/* W-byte-per-lane copy / read probes (W = 8, 16, 32), the lane-paired SELL-64 layout (two consecutive entries of a
 * row per 16-byte value load + 4-byte column load) and its SpMV (tools/spmv_layout.py) */
int fem_lab_copy(int width, int read_only, const double* src, double* dst, int64_t n, int grid, fem_stream_t stream);
int fem_lab_sell_pair(int64_t nrows, const int64_t* slice_ptr, const double* vals, const int16_t* dcols,
                      double* vals_out, int16_t* dcols_out, fem_stream_t stream);
int fem_lab_spmv16_pair(int u, int grid, int64_t nrows, const int64_t* slice_ptr, const int16_t* dcols,
                        const double* vals, const double* x, double* y, fem_stream_t stream);
/* persistent-geometry SpMV probe (paired bs = 1 layout): one workgroup of `threads` per CU pinned by lds_bytes of
 * dynamic LDS, contiguous slice ranges per wave (tools/persist_probe.py) */
int fem_lab_spmv_persist(int threads, int u, int grid, int64_t lds_bytes, int64_t nrows, const int64_t* slice_ptr,
                         const int16_t* dcols, const double* vals, const double* x, double* y, fem_stream_t stream);
/* bs = 3 layout probes (sell_pair3.hpp): layout 1 plane-paired values, 2 entry-paired values + int32 column pairs
 * (tools/spmv3_layout.py) */
int fem_lab_sell3_layout(int layout, int64_t nrows, const int64_t* slice_ptr, const double* vals,
                         const int16_t* dcols, double* vals_out, int16_t* dcols_out, fem_stream_t stream);
int fem_lab_spmv3(int layout, int u, int nt, int grid, int64_t nrows, const int64_t* slice_ptr, const int16_t* dcols,
                  const double* vals, const double* x, double* y, fem_stream_t stream);
/* tools/sym_probe.py: the production bs = 1 paired copy with slice-uniform deltas and the persistent-geometry SpMV
 * over it; a symmetric-storage SpMV (upper triangle only, lower entries re-read from the rows they mirror) */
int fem_lab_sell_uniform(int64_t nrows, const int64_t* slice_ptr, const double* vals, const int16_t* dcols,
                         double* vals_out, int16_t* dcols_out, int16_t* ucol, int32_t* uoff, fem_stream_t stream);
int fem_lab_spmv_persist_uni(int grid, int64_t lds_bytes, int64_t nrows, const int64_t* slice_ptr,
                             const int16_t* pcols, const double* pvals, const int32_t* uoff, const int16_t* ucol,
                             const double* x, double* y, fem_stream_t stream);
int fem_lab_spmv_gather(int mode, int grid, int64_t lds_bytes, int64_t nrows, const int64_t* slice_ptr,
                        const double* pvals, const int32_t* uoff, const int16_t* ucol, const double* x, double* y,
                        fem_stream_t stream);
int fem_lab_spmv_sym(int grid, int64_t lds_bytes, int64_t nrows, const int64_t* uptr, const int32_t* ulist,
                     const int16_t* udel, const int32_t* lptr, const int32_t* ldel, const int32_t* lbase,
                     const double* uvals, const double* x, double* y, fem_stream_t stream);

#ifdef __cplusplus
}
#endif
