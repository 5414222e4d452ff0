/*
 * fem355 C-ABI — MI355X (gfx950) FEM assembly + Jacobi-PCG.
 *
 * Drop-in boundary for the hot path of sml2004/CUDA-powered-mesh-handling-and-Iterative-solvers
 * (reference @ 2025-04-18; citations are reference-relative file:line). The reference is pure
 * Python/PyTorch, so its "FFI" is its module-level function surface; each entry point below names the
 * reference function whose device work it replaces. The Python mirror of that surface is
 * `cuda-powered-mesh-handling-and-iterative-solvers_amd/{element,solver}.py` (ctypes, `_capi.py`).
 *
 * Conventions
 *   - every pointer is caller-owned DEVICE memory (torch tensors' data_ptr()), except where marked [host];
 *   - coordinates / values are fp64; connectivity is int64 row-major [M, npe] (torch.long, as the reference);
 *   - graph indices (incidence, CSR/SELL pattern) are int32, offsets into value arrays int64;
 *   - dof = dpn * node + component (`solver/element.py:451`); dpn (= block size bs) is 1 or 3;
 *   - every call is asynchronous on `stream` (a hipStream_t; 0 = legacy default) unless marked [sync];
 *   - return value: FEM_OK or one of the FEM_E* codes; fem_last_error() gives a message.
 *
 * Matrix format (the "ELL-blocked" global matrix): SELL-64 with bs x bs blocks. Rows (nodes) are cut into
 * slices of 64; slice s has width w_s = max row length in the slice; entry (s, k, lane) holds block
 * column cols[slice_ptr[s] + 64*k + lane] and its bs*bs values at
 *   vals[bs*bs*slice_ptr[s] + 64*(bs*bs*k + rc) + lane],  rc = r*bs + c (row-major in the block).
 * Padding entries have col = own row and zero values. Columns of a row are ascending.
 */
#ifndef FEM355_H
#define FEM355_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* fem_stream_t; /* hipStream_t */

enum {
    FEM_OK = 0,
    FEM_EBADTYPE = 1,   /* unsupported element type  -> ValueError (`solver/element.py:427`) */
    FEM_ESINGULAR = 2,  /* singular element, index in *bad_idx -> ValueError (`solver/element.py:857-858`) */
    FEM_EHIP = 3,       /* HIP runtime error -> RuntimeError */
    FEM_ERCCL = 4,      /* RCCL error -> RuntimeError */
    FEM_EARG = 5,       /* bad argument / capacity exceeded */
    FEM_ESTATE = 6,     /* a device-side invariant was found broken (e.g. FEM_PCG_BAD_WINDOW) -> RuntimeError */
};

/* status words of the (P)CG state, mirrored on the host as the reference's print strings
 * (`solver/solver.py:187-198,210-218,226-227,805-811`) */
enum {
    FEM_PCG_RUNNING = 0,
    FEM_PCG_CONVERGED = 1,
    FEM_PCG_MAXITER = 2,
    FEM_PCG_BREAKDOWN = 3,  /* pAp < eps or pAp < 0  (`solver/solver.py:187-192`) */
    FEM_PCG_ALPHA_NAN = 4,  /* (`solver/solver.py:196-198`) */
    FEM_PCG_BETA_NAN = 5,   /* (`solver/solver.py:214-218`) */
    FEM_PCG_SYNC_TIMEOUT = 6, /* persistent schedule: an in-launch wait gave up (seconds without progress); the
                               * iterate is not meaningful -> RuntimeError */
    FEM_PCG_BAD_WINDOW = 7,   /* persistent / fused schedules: a workgroup's gather window lay outside the u-flag
                               * array (an internal invariant broken upstream). The kernel never indexes past the
                               * array; it ends the launch, and fem_pcg_poll / fem_pcg_solve return FEM_ESTATE */
};

/* CG_CONSTRAINED: constrained_conjugate_gradient_solver / new_constrained_conjugate_gradient_solver
 * (`solver/solver.py:512-600`, `:702-759`): the CG_STABLE arithmetic without zeroing x, plus the projections
 * of fem_pcg_set_constraints after every x update */
enum { FEM_MODE_CG_STABLE = 0, FEM_MODE_PCG = 1, FEM_MODE_CG_CONSTRAINED = 2 };
enum { FEM_KIND_ELASTIC = 0, FEM_KIND_POISSON = 1, FEM_KIND_MASS = 2 };
enum { FEM_ISO_SUM = 0, FEM_ISO_STACK = 1, FEM_ISO_VOLUME = 2, FEM_ISO_MASS = 3 };

const char* fem_last_error(void);                 /* [host] message of the last failing call */
int fem_version(void);                            /* [host] ABI version (100 * major + minor) */

/* ------------------------------------------------------------------ element stiffness (L1)
 * fem_tet4_ke: c3d4 element matrices.
 *   kind = FEM_KIND_ELASTIC: Ke [M,12,12] = B^T D B V   — replaces compute_c3d4_K_matrix
 *          (`solver/element.py:883-903`, with B `:835-881`, D `:282-306`, V `:514-541`).
 *   kind = FEM_KIND_POISSON: Ke [M,4,4] = kappa V G G^T (derived P1 Laplacian; no reference function,
 *          SURVEY §8(a) a15); `E` is used as kappa.
 *   Singular check |det[1 x y z]| < 1e-12 -> FEM_ESINGULAR, *bad_idx [device int64] = first bad element
 *   (initialise it to M). */
int fem_tet4_ke(const double* coords, const int64_t* conn, int64_t M, double E, double nu, int kind,
                double* Ke, int64_t* bad_idx, fem_stream_t stream);

/* c3d4 geometry: vol [M] = |det|/6 (compute_tetrahedral_volumes, `solver/element.py:514-541`), grads [M,4,3]
 * (rows of inv([1 x y z]), `:851-866`), B [M,6,12] (compute_c3d4_B_matrix, `:835-881`); outputs may be NULL.
 * kind FEM_KIND_MASS of fem_tet4_ke gives the consistent P1 mass [M,12,12] = rho V (1+delta_ab)/20 (x) I3 with
 * E = rho (compute_c3d4_M_matrix, called at `solver_example.ipynb:221`; no source exists: parity unpinned). */
int fem_tet4_geom(const double* coords, const int64_t* conn, int64_t M, double* vol, double* grads, double* B,
                  int64_t* bad_idx, fem_stream_t stream);

/* fem_iso_ke: isoparametric solids c3d8 / c3d6 / c3d10 (npe = 8 / 6 / 10). The natural derivatives dN
 * [n_ip, npe, 3] and weights w [n_ip] are evaluated on the host exactly as the reference does (its quirks:
 * c3d10 weights summing to 0.45, the float32 line points of c3d6), then
 *   mode FEM_ISO_SUM    : Ke[M,d,d]      = sum_q w_q detJ_q B_q^T D B_q   (signed detJ)
 *   mode FEM_ISO_STACK  : Ke[n_ip,M,d,d] = detJ_q B_q^T D B_q            (`single=False`, Q6)
 *   mode FEM_ISO_VOLUME : Ke[M,d,d]      = B^T D B * wedge volume, one point (c3d6 single=True)
 * Replaces compute_c3d8_K_matrix (`solver/element.py:1754-1803`), compute_c3d6_K_matrix (`:2631-2676`),
 * compute_c3d10_K_matrix (`:1191-1239`). */
int fem_iso_ke(const double* coords, const int64_t* conn, int64_t M, int npe, double E, double nu,
               const double* dN, const double* w, int n_ip, int mode, double* Ke, fem_stream_t stream);
/* fem_iso_ke_sym: the same K_e (modes FEM_ISO_SUM / FEM_ISO_VOLUME) in the packed symmetric form of the internal
 * assembly path: per element only the upper 3x3 blocks (a <= b), row-major over the upper triangle (block (a, b) at
 * (a npe - a (a - 1) / 2 + b - a) * 9, entries r * 3 + c), fem_ke_sym_stride(npe) doubles per element (9 npe (npe + 1)
 * / 2 rounded up to even: c3d10 496 of 900, c3d8 324 of 576, c3d6 190 of 324). The upper blocks equal fem_iso_ke's
 * bit for bit. Consumed by fem_assemble_from_ke_sym; the reference-named functions keep the full [M, d, d]. */
int fem_ke_sym_stride(int npe);
int fem_iso_ke_sym(const double* coords, const int64_t* conn, int64_t M, int npe, double E, double nu,
                   const double* dN, const double* w, int n_ip, int mode, double* Kp, fem_stream_t stream);
/* fem_iso_mass: consistent mass of c3d8 / c3d6 / c3d10 (npe = 8 / 6 / 10) — no reference function exists (the
 * reference notebook calls a compute_c3d4_M_matrix defined nowhere, `solver_example.ipynb:221`): parity unpinned.
 *   Me[M, 3 npe, 3 npe], block (a,b) = rho sum_q w_q |detJ_q| N_a(q) N_b(q) I3
 * Nv [n_ip, npe] shape values and dN [n_ip, npe, 3] natural derivatives at the n_ip (<= 32) points, w [n_ip] weights
 * (element.py picks rules exact for N_a N_b on affine elements). */
int fem_iso_mass(const double* coords, const int64_t* conn, int64_t M, int npe, double rho, const double* Nv,
                 const double* dN, const double* w, int n_ip, double* Me, fem_stream_t stream);
/* the same consistent mass as its scalar factor: Ms [M, npe, npe] with M_e = Ms (x) I3 (block (a, b) = Ms[a][b] I3,
 * the values of fem_iso_mass's diagonal entries bit for bit) -- 1/9 of the bytes; assembled as a bs = 1 matrix on the
 * same node pattern it is the global M_s of M = M_s (x) I3 */
int fem_iso_mass_scalar(const double* coords, const int64_t* conn, int64_t M, int npe, double rho, const double* Nv,
                        const double* dN, const double* w, int n_ip, double* Ms, fem_stream_t stream);
/* J [M,3,3] (J[i][k] = sum_j dN[j][i] x_j[k]), global gradients [M,npe,3] and B [M,6,3npe] of an isoparametric
 * element at one point with natural derivatives dN [npe,3]; outputs may be NULL. Replaces compute_c3d8_Jacobian /
 * _shape_gradients / _B_matrix (`solver/element.py:1601-1694`) and the c3d6 (`:2482-2568`) / c3d10
 * (`:1026-1125`) equivalents. */
int fem_iso_geom(const double* coords, const int64_t* conn, int64_t M, int npe, const double* dN, double* J,
                 double* grads, double* B, fem_stream_t stream);

/* ------------------------------------------------------------------ mesh graph (pattern build)
 * Node -> (element, local) incidence, deterministic (entries sorted ascending by e*npe+local; a stable radix sort
 * of (node, slot) pairs). work: a device workspace of fem_incidence_work_bytes(M*npe, N)
 * bytes (256-aligned), or NULL to allocate it stream-ordered inside the call. */
int64_t fem_incidence_work_bytes(int64_t total, int64_t N);
int64_t fem_scan_work_len(int64_t n);
/* inc_ptr [N+1], inc [M*npe] */
int fem_incidence(const int64_t* conn, int64_t M, int npe, int64_t N, int32_t* inc_ptr, int32_t* inc,
                  int32_t* work, fem_stream_t stream);
/* the same with the connectivity check of the reference's indexing (IndexError in torch) folded in: *bad [device
 * int32] = 1 if any node id is outside [0, N) (such slots are left out), else 0 -- read it before using the result */
int fem_incidence_checked(const int64_t* conn, int64_t M, int npe, int64_t N, int32_t* inc_ptr, int32_t* inc,
                          int32_t* work, int32_t* bad, fem_stream_t stream);

/* Node-graph CSR pattern (block pattern for any dpn): the coalesced COO pattern of the reference's global
 * assembly (`subdivision.ipynb:118-139`) at node granularity. Two passes:
 *   fem_graph_count : row_len [N]  (unique neighbours incl. self; rows of any length, the widest by a selection
 *                     kernel); *overflow [device int, may be NULL] = 1 if some row has a neighbour more than 32767
 *                     rows away (16-bit column deltas do not fit), else 0
 *   fem_graph_fill  : colidx [nnz] sorted per row, diagpos [N] (position of the diagonal; -1 for a node no element touches)
 * rowptr [N+1] is the exclusive scan of row_len (fem_scan_i32). */
int fem_graph_count(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                    int32_t* row_len, int32_t* overflow, fem_stream_t stream);
int fem_graph_fill(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                   const int32_t* rowptr, int32_t* colidx, int32_t* diagpos, fem_stream_t stream);
/* Same pattern in (typically) one pass: rows of at most 32 neighbours from at most 384 candidates are gathered,
 * deduplicated and sorted once by a wave-private kernel into tmp [fem_graph_tmp_len(N)] (int32); the rest fall
 * back to the two-pass kernels above (LDS hash up to 512 neighbours, selection beyond). fem_graph_count2 writes row_len; fem_graph_fill2 copies / fills the rows. */
int64_t fem_graph_tmp_len(int64_t N);
int fem_graph_count2(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                     int32_t* row_len, int32_t* tmp, int32_t* overflow, fem_stream_t stream);
int fem_graph_fill2(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                    const int32_t* rowptr, const int32_t* tmp, int32_t* colidx, int32_t* diagpos,
                    fem_stream_t stream);
/* fem_graph_fill2 + fem_sell_fill + fem_sell_delta16 in one pass over the slices (slice_ptr from fem_sell_widths +
 * fem_scan_i64): colidx, diagpos, SELL cols, the 16-bit deltas dcols [slice_ptr[S]] (0 where they do not fit,
 * *overflow [device int] = 1 then: keep the int32 cols) and csr2sell (may be NULL: fem_sell_csr2sell forms it on
 * demand) -- the same arrays as the three calls. dcols / overflow may be NULL (fem_graph_count2's overflow already
 * told the caller whether the deltas fit). */
int fem_graph_sell_fill(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                        const int32_t* rowptr, const int32_t* tmp, const int64_t* slice_ptr, int32_t* colidx,
                        int32_t* diagpos, int32_t* cols, int16_t* dcols, int64_t* csr2sell, int32_t* overflow,
                        fem_stream_t stream);
/* fem_graph_sell_fill without csr2sell / overflow, plus the bs = 1 solver layout of fem_sell_sl_pattern (pcols, ucol,
 * uoff, and for G > 0 the persistent schedule's gather windows win[2 G]) formed in the same slice pass from the deltas
 * it writes -- the same arrays as fem_sell_sl_pattern, without its separate pass over the deltas. Needs the 16-bit
 * deltas (no neighbour more than 32767 rows away). */
int fem_graph_sell_fill_sl(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                           const int32_t* rowptr, const int32_t* tmp, const int64_t* slice_ptr, int32_t* colidx,
                           int32_t* diagpos, int32_t* cols, int16_t* dcols, int G, int16_t* pcols, int16_t* ucol,
                           int32_t* uoff, int32_t* win, fem_stream_t stream);
/* exclusive scan of int32 counts -> out[n+1] (out[n] = total); work: int32 [fem_scan_work_len(n)] */
int fem_scan_i32(const int32_t* in, int64_t n, int32_t* out, int32_t* work, fem_stream_t stream);

/* CSR pattern -> SELL-64 pattern. slice_ptr [S+1] int64 (entries, i.e. 64*sum of widths); cols [slice_ptr[S]].
 *   fem_sell_widths: width [S] int64 = 64 * max row length in the slice (scan it with fem_scan_i64)
 *   fem_sell_fill  : cols (padding = own row) and the CSR->SELL entry map csr2sell [nnz] int64 */
int fem_sell_widths(const int32_t* rowptr, int64_t nrows, int64_t* width, fem_stream_t stream);
/* the pattern's sizes for the build's one device-to-host read, in one launch: out5 = {nnz = rowptr[N], SELL entries
 * = slice_ptr[S], *bad (fem_incidence_checked; 0 if NULL), *ovf (fem_graph_count2; 0 if NULL), widest slice =
 * max width[s]} (int64, device) */
int fem_graph_sizes(const int32_t* rowptr, const int64_t* slice_ptr, const int64_t* width, int64_t N,
                    const int32_t* bad, const int32_t* ovf, int64_t* out5, fem_stream_t stream);
/* the CSR -> SELL entry map (as fem_sell_fill writes it) from rowptr and slice_ptr alone */
int fem_sell_csr2sell(const int32_t* rowptr, int64_t nrows, const int64_t* slice_ptr, int64_t* csr2sell,
                      fem_stream_t stream);
int fem_scan_i64(const int64_t* in, int64_t n, int64_t* out, int64_t* work, fem_stream_t stream);
int fem_sell_fill(const int32_t* rowptr, const int32_t* colidx, int64_t nrows, const int64_t* slice_ptr,
                  int32_t* cols, int64_t* csr2sell, fem_stream_t stream);

/* Reverse Cuthill-McKee renumbering of the nodes (opt-in; no reference counterpart -- the reference keeps the file
 * order of `vtk_loader_to_torch`, `solver/element.py:39-90`, which this undoes for the assembled operator) over the
 * node-graph CSR pattern rowptr / colidx above: perm [N] (new -> old), inv [N] (old -> new). Deterministic: level-
 * synchronous Cuthill-McKee from the lowest-(degree, id) node, a level's nodes grouped by their parent's CM index,
 * a parent's children in ascending id; further components from their lowest-id node; nodes no element touches last;
 * the CM order reversed. work: int32 [fem_rcm_work_len(N)]; *levels_out (may be NULL): level steps
 * launched. One host round trip per 48 levels. */
int64_t fem_rcm_work_len(int64_t N);
int fem_rcm(const int32_t* rowptr, const int32_t* colidx, int64_t N, int32_t* perm, int32_t* inv, int32_t* work,
            int* levels_out, fem_stream_t stream);

/* ------------------------------------------------------------------ global assembly (values)
 * Deterministic row-gather: every block row sums its contributions in ascending element order.
 * fem_assemble_from_ke: values from element matrices Ke [M, npe*bs, npe*bs] (the solver-entry path: the
 *   reference hands K[M,d,d] to its CG, `solver/solver.py:144`).
 * fem_assemble_tet4  : values of the c3d4 elastic (bs=3) / Poisson (bs=1) operator computed on the fly
 *   from coordinates (K_e never materialised). E is kappa for Poisson.
 * Both write SELL values (vals must be zeroed by the caller). */
int fem_assemble_from_ke(const double* Ke, const int64_t* conn, int npe, int bs, const int32_t* inc_ptr,
                         const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                         const int64_t* csr2sell, const int64_t* slice_ptr, double* vals, fem_stream_t stream);
/* fem_assemble_from_ke with the sizes the caller already knows (nnz = block-CSR entries, ent = SELL entries; -1:
 * read from the device) and store != 0 for a matrix whose values were never written: every SELL value is written
 * (padding zeroed), so the caller skips zeroing the matrix and the kernels skip reading it. Same values bit for bit
 * as zeroing + fem_assemble_from_ke (`solver/solver.py:144`'s K handoff, as above). */
int fem_assemble_from_ke_ex(const double* Ke, const int64_t* conn, int npe, int bs, const int32_t* inc_ptr,
                            const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                            const int64_t* csr2sell, const int64_t* slice_ptr, int64_t nnz, int64_t ent, int store,
                            double* vals, fem_stream_t stream);
/* fem_assemble_from_ke_ex with the widest SELL slice in block columns (max_width > 0, from the pattern build): bs = 3
 * then runs the tile form -- the rows of a slice summed together in LDS and written straight into the SELL planes
 * (no block-CSR buffer, csr2sell unused and may be NULL). Same values bit for bit. max_width <= 0: as _ex. */
int fem_assemble_from_ke_ex2(const double* Ke, const int64_t* conn, int npe, int bs, const int32_t* inc_ptr,
                             const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                             const int64_t* csr2sell, const int64_t* slice_ptr, int64_t nnz, int64_t ent, int store,
                             int max_width, double* vals, fem_stream_t stream);
int fem_assemble_tet4(const double* coords, const int64_t* conn, double E, double nu, int bs,
                      const int32_t* inc_ptr, const int32_t* inc, int64_t N, const int32_t* rowptr,
                      const int32_t* colidx, const int64_t* csr2sell, const int64_t* slice_ptr, double* vals,
                      int64_t* bad_idx, fem_stream_t stream);
/* fem_assemble_tet4 with store != 0 for a matrix whose values were never written: every SELL value is written
 * (padding zeroed) and nothing is read, so the caller skips zeroing it. Same values bit for bit as zeroing +
 * fem_assemble_tet4 (csr2sell is not read by the default accumulator kernel; pass it for FEM355_ASM_ROWS). */
int fem_assemble_tet4_ex(const double* coords, const int64_t* conn, double E, double nu, int bs,
                         const int32_t* inc_ptr, const int32_t* inc, int64_t N, const int32_t* rowptr,
                         const int32_t* colidx, const int64_t* csr2sell, const int64_t* slice_ptr, int store,
                         double* vals, int64_t* bad_idx, fem_stream_t stream);
/* fem_assemble_tet4_ex with the pattern's widest slice (max over slices of (slice_ptr[s+1] - slice_ptr[s]) / 64;
 * 0 = unknown): a P1 pattern of at most 16 columns per row takes the 16-column accumulator window (one sweep per
 * slice, less LDS per workgroup). Same values bit for bit whatever max_width says. */
int fem_assemble_tet4_ex2(const double* coords, const int64_t* conn, double E, double nu, int bs,
                          const int32_t* inc_ptr, const int32_t* inc, int64_t N, const int32_t* rowptr,
                          const int32_t* colidx, const int64_t* csr2sell, const int64_t* slice_ptr, int store,
                          int max_width, double* vals, int64_t* bad_idx, fem_stream_t stream);

/* SELL -> CSR values (export / testing): csr_vals [nnz*bs*bs] row-major blocks. */
int fem_sell_to_csr_vals(const double* vals, int bs, const int32_t* rowptr, int64_t nrows,
                         const int64_t* csr2sell, const int64_t* slice_ptr, double* csr_vals,
                         fem_stream_t stream);

/* Jacobi: w[i] = 1/A_ii (inf -> 0, `solver/solver.py:830-831`), w[i] = 0 where mask[i] != 0 (fixed DOFs);
 * mask may be NULL. diag read through diagpos (diagpos < 0: diagonal 0, so w = 0 as the reference's inf -> 0);
 * csr2sell may be NULL (the diagonal's SELL entry is then formed from rowptr and slice_ptr). */
int fem_jacobi(const double* vals, int bs, const int32_t* rowptr, const int32_t* diagpos,
               const int64_t* csr2sell, const int64_t* slice_ptr, int64_t nrows, const uint8_t* mask,
               double* w, fem_stream_t stream);

/* diag [nrows*bs] = the block diagonals' diagonal entries; w = 1/diag (inf -> 0, 0 where mask) — the two halves
 * of fem_jacobi, split so a distributed caller can halo-sum the diagonal in between (fem_halo_sum). */
int fem_sell_diag(const double* vals, int bs, const int32_t* diagpos, const int64_t* csr2sell, int64_t nrows,
                  double* diag, fem_stream_t stream);
int fem_jacobi_from_diag(const double* diag, int64_t n, const uint8_t* mask, double* w, fem_stream_t stream);

/* ------------------------------------------------------------------ element-by-element operator
 * y = sum_e P_e^T K_e P_e u — replaces compute_nodal_forces (`solver/element.py:429-464`), deterministic
 * (ascending element order per dof, like the CPU index_add). Ke [M, npe*dpn, npe*dpn]. */
int fem_ebe_apply(const double* Ke, const int64_t* conn, int npe, int dpn, const int32_t* inc_ptr,
                  const int32_t* inc, int64_t N, const double* u, double* y, fem_stream_t stream);
/* diag_K of compute_diagonal_preconditioner (`solver/solver.py:814-833`) before inversion:
 * colzero = 1 reproduces the reference's column-0 slice (`:828`, quirk Q1), 0 the true diagonal. */
int fem_ebe_diag(const double* Ke, const int64_t* conn, int npe, int dpn, const int32_t* inc_ptr,
                 const int32_t* inc, int64_t N, int colzero, double* diag, fem_stream_t stream);
/* out[i] = 1/in[i], inf -> 0 */
int fem_invert_diag(const double* in, int64_t n, double* out, fem_stream_t stream);

/* ------------------------------------------------------------------ stress recovery (post-solve)
 * strain = B u_e, stress = D strain (isotropic D of `solver/element.py:282-306`), tensor rows xx xy xz / xy yy yz /
 * xz yz zz, von Mises. u [N,3]. Outputs sig [.., 3, 3] and vm [..] may each be NULL. */
/* compute_c3d4_element_stress (`solver/element.py:905-937`): sig [M,3,3], vm [M]; bad_idx (nullable, preset to M)
 * receives the lowest element index with |det| < 1e-12 (the reference's B-matrix ValueError, `:857-858`). */
int fem_tet4_stress(const double* coords, const int64_t* conn, int64_t M, const double* u, double E, double nu,
                    double* sig, double* vm, int64_t* bad_idx, fem_stream_t stream);
/* compute_c3d8/c3d6/c3d10_element_stress (`:1696-1752`, `:2570-2629`, `:1127-1189`) at n_ip points with natural
 * derivative tables dN [n_ip, npe, 3] (npe 6, 8, 10) and weights w [n_ip]. layout 0: sum_q w_q sig_q -> [M,3,3] and
 * sum_q w_q vm_q -> [M] (single=True); 1: [M,n_ip,3,3] / [M,n_ip] (c3d8/c3d6 single=False); 2: [n_ip,M,3,3] /
 * [n_ip,M] (c3d10 single=False). */
int fem_iso_stress(const double* coords, const int64_t* conn, int64_t M, int npe, const double* u, double E, double nu,
                   const double* dN, const double* w, int n_ip, int layout, double* sig, double* vm,
                   fem_stream_t stream);
/* compute_stress_tensor (`:308-330`): Voigt [M,6] (xx, yy, zz, xy, yz, xz) -> [M,3,3] */
int fem_voigt_to_tensor(const double* voigt, int64_t M, double* tensor, fem_stream_t stream);
/* compute_von_mises_stress (`:332-353`): [M,3,3] -> [M] */
int fem_von_mises(const double* tensor, int64_t M, double* vm, fem_stream_t stream);
/* compute_node_vm_stress (`:466-504`): out[n] = mean of ev[e] over the incidence of node n (0 if none), summed in
 * ascending element order (the reference's sequential index_add); inc from fem_incidence of the same [M,npe] */
int fem_node_average(const double* ev, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N, double* out,
                     fem_stream_t stream);
/* compute_c3d4_surface_forces (`:3343-3362`): out [M,F,3] = sig_e n_ef for normals [M,F,3], sig [M,3,3] */
int fem_face_forces(const double* normals, const double* sig, int64_t M, int F, double* out, fem_stream_t stream);
/* compute_c3d4_shared_face_forces_sum (`:3364-3382`): out [S,3] = ff[e0,f0] + ff[e1,f1], idx [S,2,2] (validated by
 * the caller), ff [M,F,3] */
int fem_shared_face_sum(const int64_t* idx, const double* face_forces, int F, int64_t S, double* out,
                        fem_stream_t stream);

/* ------------------------------------------------------------------ mesh topology
 * Face / edge grouping: every element face of table ftab [F, fpn] (local node indices, element-major flat id
 * e * F + f) is keyed by its sorted node ids and radix-sorted once (stable), which reproduces torch.unique(dim=0)
 * row order and the reference's pairing order (`solver/element.py:543-579,707-762,1293-1334,1474-1532,2234-2283,
 * 2687-2713`). N bounds the node ids (< 2^32); F <= 12, fpn <= 4, M * F < 2^31. [sync] */
typedef struct fem_topo fem_topo;
int fem_topo_create(const int64_t* conn, int64_t M, int npe, const int32_t* ftab, int F, int fpn, int64_t N,
                    fem_stream_t stream, fem_topo** out);
/* number of distinct faces, of faces occurring once (surfaces) and of faces occurring exactly twice (shared) */
int fem_topo_counts(const fem_topo* t, int64_t* n_unique, int64_t* n_single, int64_t* n_pair);
/* shared faces [n_pair, 2, 2] = ((e0, f0), (e1, f1)) in key order, e0 * F + f0 < e1 * F + f1
 * (identify_*_shared_faces) */
int fem_topo_pairs(fem_topo* t, int64_t* out);
/* distinct sorted node tuples [n_unique, fpn] in lexicographic order (element_to_edge) */
int fem_topo_unique(fem_topo* t, int64_t* out);
/* faces occurring once, in face-major order fs * M + e of a caller table of Fs rows: stab [Fs, fpn] gives the
 * output node order, smap [Fs] the context row with the same node set, xtab [Fs] (nullable) the extra node
 * (compute_*_surface_faces_with_*_node). faces [count, fpn], extra [count] may be NULL to only count. [sync] */
int fem_topo_boundary(fem_topo* t, const int64_t* conn, int Fs, const int32_t* smap, const int32_t* stab,
                      const int32_t* xtab, int64_t* faces, int64_t* extra, int64_t* count);
void fem_topo_destroy(fem_topo* t);
/* out [M * T, spe] = conn[:, tab] (c3d8_to_c3d4 `:1555-1581`, c3d6_to_c3d4 `:2424-2446`, c3d10_to_c3d4 `:963-993`) */
int fem_sub_elements(const int64_t* conn, int64_t M, int npe, const int32_t* tab, int T, int spe, int64_t* out,
                     fem_stream_t stream);
/* per element face normals [M, F, 3]: (p[e1] - p[e0]) x (p[e2] - p[e0]) * scale for edges [F, 3]; unit: normalise;
 * flip: negate when dot(n, x[extra] - mean(x[cen[f][0..ncen[f])])) > 0 (cen is [F, 4]).
 * compute_tetrahedral_normals_and_area `:652-705`, compute_hexahedral_normals_and_area `:1418-1472`,
 * compute_wedge_normals_and_area `:2377-2422` */
int fem_element_face_normals(const double* coords, const int64_t* conn, int64_t M, int npe, const int32_t* edges,
                             const int32_t* cen, const int32_t* ncen, const int32_t* extra, int F, double scale,
                             int flip, int unit, double* out, fem_stream_t stream);
/* outward unit normals of surface faces [K, fpn] with extra nodes [K]; second edge to vertex v2
 * (compute_tetrahdral_surface_normals `:581-619`, compute_hexahedral_surface_normals `:1336-1374`,
 * compute_wedge_surface_normals `:2285-2338`) */
int fem_surface_normals(const double* coords, const int64_t* faces, const int64_t* extra, int64_t K, int fpn, int v2,
                        double* out, fem_stream_t stream);

/* ------------------------------------------------------------------ mesh input
 * Legacy VTK unstructured grid (ASCII / BINARY, file versions 2.x-5.x) -> points [N,3] fp64, the count-prefixed
 * cell array pyvista exposes as mesh.cells, and the VTK cell types: the file side of vtk_loader_to_torch
 * (`solver/element.py:39-90`). [host] — plain host memory, no device needed. */
typedef struct fem_vtk fem_vtk;
int fem_vtk_read(const char* path, fem_vtk** out);
int fem_vtk_sizes(const fem_vtk* v, int64_t* n_points, int64_t* n_cells, int64_t* cells_len, int64_t* n_types);
int fem_vtk_copy(const fem_vtk* v, double* points, int64_t* cells, int64_t* types);
void fem_vtk_free(fem_vtk* v);

/* ------------------------------------------------------------------ dof-level CSR layer (SURVEY §8(b) names)
 * The assembled-matrix view of the reference (`subdivision.ipynb:118-139`: rows dof_i, cols dof_j, K_e values
 * row-major, coalesced), dof = dpn * node + comp. [sync] where noted; temporaries are stream-ordered.
 * fem_solid_ke: c3d8 / c3d6 / c3d10 element matrices (type = nodes per element 8 / 6 / 10) from natural points
 *   ip [n_ip,3] and weights w [n_ip] (device); single = 1: sum_q w_q detJ_q B^T D B (c3d6: B at (1/3,1/3,0) times
 *   the wedge volume, ip ignored), single = 0: the per-point stack [n_ip,M,d,d] (c3d6: the weighted sum)
 *   (`solver/element.py:1754-1803`, `:2631-2676`, `:1191-1239`). */
int fem_solid_ke(int type, const double* coords, const int64_t* conn, int64_t M, double E, double nu, const double* ip,
                 const double* w, int n_ip, int single, double* Ke, fem_stream_t stream);
/* [sync] dof CSR pattern: rowptr [n_nodes*dpn+1], *nnz_out; with colidx (nnz, sorted per row) and diagpos
 * [n_nodes*dpn] (nullable) also the columns. Call once with colidx = NULL to size colidx. */
int fem_csr_pattern(const int64_t* conn, int64_t M, int npe, int dofs_per_node, int64_t n_nodes, int32_t* rowptr,
                    int32_t* colidx, int32_t* diagpos, int64_t* nnz_out, fem_stream_t stream);
/* vals += coalesce(P_e^T K_e P_e), Ke [M, npe*dpn, npe*dpn], summed per entry in ascending (element, local) order */
int fem_csr_fill(const double* Ke, const int64_t* conn, int64_t M, int npe, int dpn, int64_t n_nodes,
                 const int32_t* rowptr, const int32_t* colidx, double* vals, fem_stream_t stream);
/* y = A x on the dof CSR (n rows) */
int fem_spmv_csr(const int32_t* rowptr, const int32_t* colidx, const double* vals, const double* x, double* y,
                 int64_t n, fem_stream_t stream);
/* [sync] one-shot solve on the dof CSR: mode FEM_MODE_CG_STABLE (`solver/solver.py:144-229`; fixed_mask dofs held
 * at zero) or FEM_MODE_PCG (`:766-812`; z = dinv r, fixed_mask dofs get dinv = 0). x: initial guess in, solution out;
 * res_hist_out [max_iter] (nullable) receives sqrt(r.z) per iteration. */
int fem_pcg_csr(const int32_t* rowptr, const int32_t* colidx, const double* vals, int64_t n, const double* b,
                double* x, const double* dinv, const uint8_t* fixed_mask, double tol, int max_iter, double eps,
                int mode, int* iters_out, int* status_out, double* res_hist_out, fem_stream_t stream);

/* ------------------------------------------------------------------ SpMV (L2)
 * y = A x on the SELL-64 matrix (nrows block rows of size bs). */
int fem_spmv(int64_t nrows, int bs, const int64_t* slice_ptr, const int32_t* cols, const double* vals,
             const double* x, double* y, fem_stream_t stream);
/* 16-bit column deltas: dcols[e] = cols[e] - row (SELL layout); *overflow [device int32, zeroed] = 1 when a
 * delta exceeds +-32767 (then keep the int32 columns). Halves the index stream of every SpMV: 10 instead of
 * 12 bytes per scalar nonzero on banded (e.g. line-numbered or RCM-ordered) meshes. */
int fem_sell_delta16(const int32_t* cols, int64_t nrows, const int64_t* slice_ptr, int16_t* dcols, int32_t* overflow,
                     fem_stream_t stream);
int fem_spmv16(int64_t nrows, int bs, const int64_t* slice_ptr, const int16_t* dcols, const double* vals,
               const double* x, double* y, fem_stream_t stream);
/* measurement entry points (bench.py stream_ceiling): the HBM copy-ceiling probe dst = src and the read-only
 * probe (16-byte loads summed, *out written only to keep the loads alive) over n doubles (n even, 16-byte
 * aligned); grid <= 0: default. */
int fem_stream_copy(const double* src, double* dst, int64_t n, int grid, fem_stream_t stream);
int fem_stream_read(const double* src, double* out, int64_t n, int grid, fem_stream_t stream);

/* ------------------------------------------------------------------ (P)CG (L3)
 * One solve context over a SELL matrix. The whole iteration runs on the device: SpMV + p.q reduction,
 * update + r.z reduction, p/x update; scalars, guards and the stop test live in a device state word,
 * so the host only polls between chunks of iterations.
 *   mode FEM_MODE_CG_STABLE: stable_conjugate_gradient_solver (`solver/solver.py:144-229`), w = free mask
 *        (1 free / 0 fixed), alpha = rs/(pAp+eps), beta = rs_new/(rs_old+eps), stop sqrt(r.r) < tol
 *   mode FEM_MODE_PCG: preconditioned_conjugate_gradient_solver (`solver/solver.py:766-812`), w = M_inv,
 *        no eps, no guards, stop sqrt(r.z) < tol
 * b, x, w are [n = nrows*bs]; x holds u_init on entry and u on exit. hist [max_iter] (may be NULL)
 * receives sqrt(r.z) (sqrt(r.r) for CG) after each iteration. */
typedef struct fem_pcg fem_pcg;   /* opaque */
int fem_pcg_create(int64_t nrows, int bs, const int64_t* slice_ptr, const int32_t* cols, const double* vals,
                   const double* b, double* x, const double* w, int mode, double tol, double eps,
                   double* hist, int64_t hist_len, fem_stream_t stream, fem_pcg** out);
/* initial residual r0 = b - A x0 (+ masking in CG mode), z0, p0, r0.z0 */
int fem_pcg_start(fem_pcg* s);
/* enqueue k iterations (no host sync); iterations after a stop are no-ops on the device */
int fem_pcg_iterate(fem_pcg* s, int k);
/* [sync] read iteration count, status and last r.z (or r.r). Guard stops (FEM_PCG_BREAKDOWN / _ALPHA_NAN) report
 * the reference's printed iteration; every other status the completed iterations. Returns FEM_ESTATE (status
 * FEM_PCG_BAD_WINDOW, message in fem_last_error) when a launch found a gather window outside its flag array */
int fem_pcg_poll(fem_pcg* s, int* iters, int* status, double* rz);
/* [debug, test-only] overwrite logical workgroup L's gather window with [lo, hi] in the active schedule's window
 * array (persistent or fused; call after fem_pcg_start): the fault-injection knob behind the FEM_PCG_BAD_WINDOW
 * test. FEM_EARG when the context has no window array */
int fem_pcg_debug_window(fem_pcg* s, int L, int lo, int hi);
/* [sync] diagnostic of a FEM_PCG_SYNC_TIMEOUT: the give-up site code (persistent kernel: 1 grid barrier, 2 u-flag
 * window, 3 rank sums of the DIST build, + 16 * epoch; merged update k_pcg_update2: 4 + 16 * launch since start),
 * 0 for any other status */
int fem_pcg_sync_site(fem_pcg* s, int* site);
/* [sync] out6 = {rz (rs_old), pq (p.Ap), alpha, beta, rz_new, completed iterations} for the host messages */
int fem_pcg_scalars(fem_pcg* s, double* out6);
/* [sync] run to completion: start + chunks of `chunk` iterations until stop or max_iter (persistent schedule:
 * cooperative launches, deferred-schedule re-solve from x0 after a FEM_PCG_SYNC_TIMEOUT) */
int fem_pcg_solve(fem_pcg* s, int max_iter, int chunk, int* iters, int* status, double* rz);
/* kernel schedule: 0 = 3-kernel (SpMV+p.q / r update+r.z / x,p update; the context default), 1 = fused (p formed
 * inside the SpMV from r, w and the previous p; 2 kernels per iteration), 2 = deferred (each kernel finishes the
 * previous kernel's block partials itself: no grid atomics, state banked by launch parity), 3 = persistent
 * (pcg_persist.hpp: the single-reduction iteration as one cooperative launch per chunk, CG state of every row held in
 * registers / LDS of its owning wave, slices past 7 per wave streamed from HBM in the same launch; bs = 1 with
 * 16-bit columns and FEM_TUNE_PAIR, single GPU; otherwise fem_pcg_start falls back to 2; bs = 3: pcg_persist3.hpp,
 * 2 slices per wave on chip, past that the same overflow build), 4 = auto (3 where it applies -- for bs = 3 only
 * while the state fits on chip, else 0). Element-partitioned and constrained contexts accept only 0 (4 maps to 0). */
int fem_pcg_set_schedule(fem_pcg* s, int sched);
/* the SELL entry count of the context's matrix, which MUST equal slice_ptr[nslices] (known to the caller from the
 * pattern build; the paired copy is sized from it): spares fem_pcg_start the device-to-host read (a host sync)
 * before it builds that copy. Optional; without it fem_pcg_start reads the count itself. */
int fem_pcg_set_entries(fem_pcg* s, int64_t entries);
/* the schedule the context runs (valid after fem_pcg_start: 3 may have fallen back to 2) */
int fem_pcg_get_schedule(fem_pcg* s);
/* [sync] over the slices [s_begin, s_end) of the context's matrix (s_end < 0: to the last): the slices stored with
 * slice-uniform deltas (FEM_TUNE_PK_UNI; valid after fem_pcg_start), the slice count, and the column-index bytes one
 * SpMV over those slices reads (padding included) */
int fem_pcg_uniform_slices(fem_pcg* s, int64_t s_begin, int64_t s_end, int64_t* uniform, int64_t* nslices,
                           int64_t* index_bytes);
/* ------------------------------------------------------------------ solver layout
 * The matrix stored straight in the layout the PCG schedules read, so a solve converts nothing and the matrix is
 * resident once. bs = 1: lane-paired SELL entries (entry k of lane l of a slice of width w at 128 (k / 2) + 2 l + k % 2,
 * the odd tail at 128 (w / 2) + l), and in every slice whose rows take their columns at one sorted list of offsets
 * (slice-uniform) those offsets stored once, the rows' missing offsets holding value 0. bs = 3: the plane-paired
 * layout A (entry E = slice base + 64 k + lane: values (2t, 2t + 1) at 9 (E - lane) + 128 t + 2 lane, value 8 at
 * 9 (E - lane) + 512 + lane), columns the plain 16-bit deltas.
 *   fem_sell_sl_pattern : from the plain 16-bit deltas (fem_graph_sell_fill): pcols [entries] paired deltas, uoff
 *                         [nslices] (-1: per-lane deltas), ucol [2 (entries / 64) + 2] lists; with G > 0 also the
 *                         persistent schedule's gather windows win [2 G] for a G-workgroup grid (G = CUs rounded
 *                         down to a multiple of 8). bs = 3 reads only the windows
 *   fem_assemble_tet4_sl: the c3d4 values (bs = 1: Poisson, kappa = E; bs = 3: elasticity E, nu) into svals
 *                         [entries bs^2] in that layout (store != 0: every value written; else added) --
 *                         fem_assemble_tet4_ex2's sums, bit for bit, at other positions; uoff / ucol unused for bs = 3
 *   fem_assemble_from_ke_sl: bs = 3 stored element matrices (npe 4 / 6 / 8 / 10, the pattern's widest slice
 *                         max_width) into layout A -- fem_assemble_from_ke_ex2's sums, bit for bit
 *   fem_jacobi_sl       : fem_jacobi of such a matrix;  fem_spmv_sl: y = A x (bs = 3: pcols = the plain deltas);
 *   fem_sell_sl_unpair  : its plain SELL values
 *   fem_pcg_set_layout  : a context (16-bit columns set) reads the caller's svals (bs = 1 also pcols / uoff / ucol)
 *                         and windows (nullable) instead of building its own paired copy: no conversion at
 *                         fem_pcg_start; the arrays must outlive the context; vals of fem_pcg_create is then not read. */
int fem_sell_sl_pattern(int64_t nrows, const int64_t* slice_ptr, const int16_t* dcols, int G, int16_t* pcols,
                        int16_t* ucol, int32_t* uoff, int32_t* win, fem_stream_t stream);
int fem_assemble_tet4_sl(const double* coords, const int64_t* conn, double E, double nu, int bs,
                         const int32_t* inc_ptr, const int32_t* inc, int64_t N, const int32_t* rowptr,
                         const int32_t* colidx, const int64_t* slice_ptr, const int32_t* uoff, const int16_t* ucol,
                         int store, int max_width, double* svals, int64_t* bad_idx, fem_stream_t stream);
int fem_assemble_from_ke_sl(const double* Ke, const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc,
                            int64_t N, const int32_t* rowptr, const int32_t* colidx, const int64_t* slice_ptr,
                            int store, int max_width, double* svals, fem_stream_t stream);
/* bs = 3 assembly from packed symmetric K_e (fem_iso_ke_sym; the tile form of fem_assemble_from_ke_ex2 / _sl): block
 * (a, b) read from the upper block, (b, a) from its transpose, in the same (incidence, b) order -- the same sums as
 * from the full K_e whose lower blocks mirror the upper ones. layout_a = 1: vals is the bs = 3 solver layout (as
 * fem_assemble_from_ke_sl), 0: the plain planes. Internal path of configs[4] (`solver/element.py:1191-1239,1754-1803`
 * K_e, `subdivision.ipynb:118-139` COO assembly semantics). */
int fem_assemble_from_ke_sym(const double* Kp, const int64_t* conn, int npe, const int32_t* inc_ptr,
                             const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                             const int64_t* slice_ptr, int store, int max_width, int layout_a, double* vals,
                             fem_stream_t stream);
/* Stiffness and mass of one element family in one pass (configs[4]'s internal path): the bs = 3 K_e [M, 3 npe, 3 npe]
 * into layout A svals (fem_assemble_from_ke_sl's sums, bit for bit) and the scalar Me [M, npe, npe] (the consistent
 * mass factor M_s of M = M_s (x) I3) into the plain bs = 1 SELL values mvals of the same pattern
 * (fem_assemble_from_ke_ex2's bs = 1 sums, bit for bit); store != 0: both fresh (every value written), else both added.
 * One column search and one incidence walk for both matrices. Replaces the two assembly calls a caller of the
 * reference would make over `compute_K_matrix` (`solver/element.py:419-427`) and a mass matrix of the same mesh
 * (`solver_example.ipynb:216,221`), with the COO semantics of `subdivision.ipynb:118-139`. */
int fem_assemble_from_ke_mass_sl(const double* Ke, const double* Me, const int64_t* conn, int npe,
                                 const int32_t* inc_ptr, const int32_t* inc, int64_t N, const int32_t* rowptr,
                                 const int32_t* colidx, const int64_t* slice_ptr, int store, int max_width,
                                 double* svals, double* mvals, fem_stream_t stream);
int fem_jacobi_sl(const double* svals, int bs, const int32_t* rowptr, const int32_t* diagpos,
                  const int64_t* slice_ptr, const int32_t* uoff, const int16_t* ucol, int64_t nrows,
                  const uint8_t* mask, double* w, fem_stream_t stream);
int fem_spmv_sl(int64_t nrows, int bs, const int64_t* slice_ptr, const int16_t* pcols, const double* svals,
                const int32_t* uoff, const int16_t* ucol, const double* x, double* y, fem_stream_t stream);
int fem_sell_sl_unpair(int64_t nrows, int bs, const int64_t* slice_ptr, const int16_t* dcols, const int32_t* uoff,
                       const int16_t* ucol, const int32_t* rowptr, const double* svals, double* vals,
                       fem_stream_t stream);
int fem_pcg_set_layout(fem_pcg* s, const double* svals, const int16_t* pcols, const int32_t* uoff,
                       const int16_t* ucol, const int32_t* win, int G);
/* [host] the persistent build the context's launches run (valid after fem_pcg_start; all 0 when the schedule is not
 * 3): register slots per wave (bs = 1: 1, 2, 4 or 7; bs = 3: 2), 1 for the overflow build, and the packed
 * assignment's slices per wave (0: the even spread) */
int fem_pcg_persist_build(fem_pcg* s, int* slots, int* overflow, int* pack);
/* 1 in *on when the started context runs the pipelined persistent iteration (FEM_TUNE_PK_GV), else 0 */
int fem_pcg_pipelined(fem_pcg* s, int* on);
/* persistent schedule only: k iterations of the instrumented kernel build; host_out[G * 8] = per-workgroup shader-clock
 * sums of the phases (u wait, SpMV, block sum, barrier + partial sums, step, update + drain + flag, launch prologue,
 * launch epilogue), then host_out[G * 8 + G * 16] = every wave's own SpMV clock sum; *grid = G */
int fem_pcg_persist_profile(fem_pcg* s, int k, unsigned long long* host_out, int* grid);
/* CG_CONSTRAINED projections applied to x once at fem_pcg_start (after r0 = b - A x0) and after every x update:
 *   order 0 (`enforce_constraints`, `solver/solver.py:478-510`): x[rbe2_slave] = x[rbe2_master] (all gathered
 *           before any is written), then x[spc_dof] = spc_val.  G must be 0.
 *   order 1 (`new_enforce_constraints`, `:665-700`): SPC, then RBE2, then for every RBE3 group g in order
 *           x[r3_master[g]] = sum_{e in [r3_ptr[g], r3_ptr[g+1])} r3_w[e] x[r3_slave[e]] / (r3_wsum[g] + 1e-30).
 * All indices are flat dofs (node * dpn + dof) in [0, n); r3_ptr is a CSR offset array with r3_ptr[0] = 0 (one
 * group per (RBE3, dof) pair: `:685-698`). The residual masking of SPC dofs and RBE2 slaves (`r[...] = 0`) is the
 * context's 0/1 weight vector w. All arrays are device-resident and must outlive the context.
 * [sync] validates every index once; FEM_EARG on a bad index, a non-constrained / distributed / graph context. */
int fem_pcg_set_constraints(fem_pcg* s, int order, int64_t R, const int64_t* rbe2_slave, const int64_t* rbe2_master,
                            int64_t S, const int64_t* spc_dof, const double* spc_val, int64_t G,
                            const int64_t* r3_ptr, const int64_t* r3_master, const double* r3_wsum,
                            const int64_t* r3_slave, const double* r3_w);
/* [sync] the same projections applied once to x [n] (stream-ordered), and r [n] (nullable) zeroed at the SPC dofs
 * and RBE2 slaves: `enforce_constraints` / `new_enforce_constraints` as standalone calls
 * (`solver/solver.py:478-510`, `:665-700`). */
int fem_enforce_constraints(double* x, double* r, int64_t n, int order, int64_t R, const int64_t* rbe2_slave,
                            const int64_t* rbe2_master, int64_t S, const int64_t* spc_dof, const double* spc_val,
                            int64_t G, const int64_t* r3_ptr, const int64_t* r3_master, const double* r3_wsum,
                            const int64_t* r3_slave, const double* r3_w, fem_stream_t stream);
/* tuning flags (default FEM_TUNE_REVERSE | FEM_TUNE_PAIR | FEM_TUNE_PK_SC1 | FEM_TUNE_PK_PACK | FEM_TUNE_PK_UNI |
 * FEM_TUNE_UPD1): the SpMV of every schedule sweeps each XCD's slice range backwards on
 * odd iterations, so the matrix tail read last (still in the MI355X's 256 MB memory-side cache) is read first by
 * the next sweep: 67 -> 57 us per SpMV on the 10M Poisson matrix. Results depend on the flags only through the
 * order of the per-block p.q partials (deterministic for a given flag set). */
enum { FEM_TUNE_REVERSE = 1, FEM_TUNE_PAIR = 2, FEM_TUNE_PK_SC1 = 4, FEM_TUNE_PK_PACK = 8, FEM_TUNE_C1F = 16,
       FEM_TUNE_PK_COOP = 32, FEM_TUNE_DIST_FINE = 64, FEM_TUNE_PK_UNI = 128, FEM_TUNE_PK_WIDE = 256,
       FEM_TUNE_DIST_DROP = 512, FEM_TUNE_UPD1 = 1024, FEM_TUNE_U2_HOLD = 2048, FEM_TUNE_U2_SMALL = 4096,
       FEM_TUNE_MF_GATHER = 8192, FEM_TUNE_PK_GV = 16384 };
/* FEM_TUNE_PK_GV (opt-in, set before fem_pcg_start): persistent schedule, bs = 1, single GPU, PCG mode, systems of at
 * most 2 slices per wave (~2M rows on 256 CUs: the 1M-tet cube, a rank share of the 10M one) -- the pipelined
 * (Ghysels-Vanroose) Jacobi-PCG, whose grid reduction runs under the next SpMV (csrc/pcg_persist_gv.hpp). Its
 * iterates leave the single-reduction ones at rounding level (recurrences for M^-1 r and A M^-1 r); other contexts
 * ignore the flag. fem_pcg_pipelined reports whether the started context runs it. */
/* FEM_TUNE_MF_GATHER (A/B): on the element-chunk operator, q = A p is summed from the slots by a gather launch and
 * read by the merged update, instead of the update summing each dof's slots itself (the default; same bits). */
/* FEM_TUNE_U2_HOLD / FEM_TUNE_U2_SMALL (tests only): the merged update's give-up path -- workgroup 0 arrives only after
 * every other workgroup's bounded wait ran out, so the launch must end with FEM_PCG_SYNC_TIMEOUT, no x / p update
 * anywhere and the give-up site 4 (+ 16 * launch); and its grid capped at 8 workgroups, so a small system reaches the
 * loops past the register-cached elements. */
/* FEM_TUNE_UPD1 (default): single-GPU 3-kernel schedule (bs = 3 past the persistent kernel's capacity) -- the r / z
 * update and the x / p update run as ONE launch with every workgroup resident (k_pcg_update2: the last workgroup
 * finishes r.z and releases the others), z kept in registers in between: 8 vector streams per iteration instead of
 * 10. Same recurrences; p = z + beta p rounds z before the add (the two-kernel form may fuse it). */
/* FEM_TUNE_DIST_DROP: fault injection for the multi-GPU failure chain (tests only): the rank publishes no u row and
 * no flag to the other ranks, so their launches give up (FEM_PCG_SYNC_TIMEOUT) within the bounded waits */
/* FEM_TUNE_PK_WIDE: persistent schedule (bs = 1, single GPU) -- keep the 7-slot build when every wave owns at most
 * one slice (by default such systems, e.g. 1M tets, run a one-slot build with 8 lane pairs in flight; A/B switch) */
/* FEM_TUNE_PK_UNI (default): bs = 1 paired copies also record, per 64-row slice whose rows take their columns at one
 * common sorted list of offsets (rows lacking an offset get a zero value there), that list once (sell_pair.hpp
 * k_sell_uniform); the persistent schedule then reads those slices' deltas with wave-uniform loads: 10 -> 8 bytes
 * per matrix entry (every slice of the Kuhn cubes). Same products in the same order per row (+-0 terms between). */
/* FEM_TUNE_DIST_FINE (set before fem_pcg_set_rows): the distributed persistent comm block (u, flags, rank sums) in
 * fine-grained device memory (hipDeviceMallocFinegrained) instead of hipMalloc's coarse-grained memory -- the
 * variant bench.py tries when the coarse-grained one fails its self-check on a multi-GPU node. */
/* FEM_TUNE_PK_COOP: persistent schedule — every launch is a hipLaunchCooperativeKernel (the runtime guarantees that
 * all workgroups are resident at once, or fails the launch). fem_pcg_solve always launches cooperatively and, should
 * a launch still end with FEM_PCG_SYNC_TIMEOUT, re-solves from the saved x0 on the deferred schedule; without the
 * flag fem_pcg_iterate / fem_pcg_profile use plain launches (residency from the occupancy check) and report the
 * timeout status. */
/* FEM_TUNE_C1F: distributed single-reduction contexts run each iteration as ONE launch (k_cg1_fused: step, update,
 * u hand-off to the neighbouring workgroups by flags, SpMV, pack, one two-value grid reduction) instead of
 * k_cg1_update + k_cg1_spmv. */
/* FEM_TUNE_PK_PACK (default): persistent schedule only — each workgroup gives its waves ceil(max slices per
 * workgroup / 16) slices each in order (the last busy wave takes the remainder) instead of spreading them evenly:
 * at 10M 15 waves x 7 slices all stream to the end of the SpMV phase instead of 7-slice waves finishing alone
 * (54.0 -> 51.6 us per iteration; 3M tets 21.6 -> 19.3; equal at 1M and 6M). Same per-row arithmetic, so the
 * iterates change only through the order of the u.v partials. */
/* FEM_TUNE_PK_SC1 (default): persistent schedule only — the u gathers are sc1 (agent-coherent) loads instead of
 * plain loads behind an agent acquire per workgroup and iteration (whose L2 invalidations cost the other workgroups
 * of the XCD their gather window): 58.8 -> 55.9 us per 10M Poisson iteration, bit-identical iterates. */
/* FEM_TUNE_PAIR (default): contexts with 16-bit columns keep a copy of the matrix read with 16-byte value loads,
 * rebuilt from vals / cols16 by every fem_pcg_start: bs = 1 lane-paired (two entries per load, sell_pair.hpp; +257 MB
 * on the 10M Poisson matrix), bs = 3 plane-paired (values 0..7 of a block as four 16-byte loads, sell_pair3.hpp
 * layout A; +1.85 GB on the 10M elasticity matrix). Same products, same summation order per row as the plain layout. */
int fem_pcg_set_tuning(fem_pcg* s, int flags);
/* run the SpMV of this context on 16-bit column deltas (NULL: back to the int32 columns) */
int fem_pcg_set_cols16(fem_pcg* s, const int16_t* dcols);
/* apply the deferred x update of the fused schedule after the last iteration (fem_pcg_solve does this) */
int fem_pcg_finish(fem_pcg* s);
/* capture `k` iterations in a hipGraph and use it for fem_pcg_iterate calls with that k (0 disables) */
int fem_pcg_use_graph(fem_pcg* s, int k);
/* [sync] enqueue k iterations like fem_pcg_iterate, bracketing every `every`-th iteration's three kernels
 * with hip events on the solver stream; ms[0..2] = summed device ms of SpMV+dot / update / p-x update over the
 * n[0..2] sampled launches (bench.py's live per-kernel timing inside its timed region) */
int fem_pcg_profile(fem_pcg* s, int k, int every, double* ms, int* n);
void fem_pcg_destroy(fem_pcg* s);
/* ------------------------------------------------------------------ multi-GPU persistent schedule (rows partitioned)
 * The persistent schedule across ranks (one process per GPU, or several contexts of one process on one GPU for
 * validation): every rank holds the SELL rows of the global matrix it owns (global row / column numbering, all
 * vectors global-length) and runs ONE persistent launch per chunk over its own slices; the u rows another rank
 * gathers are written straight into that rank's comm block (system-scope stores over xGMI + a system release +
 * an epoch flag per workgroup), and the per-iteration sums go rank -> every rank the same way, summed in rank
 * order (bit-identical scalars everywhere). No collective library call inside an iteration. bs = 1 only.
 *   fem_pcg_set_rows  : rank `rank` of `nranks` (<= 8) owns the global slices [split[rank], split[rank+1]) of the
 *                       context's matrix; grid = workgroups of this rank's launches (0: one per CU; a multiple of
 *                       8: several ranks sharing one GPU); allocates the comm block and the gather windows.
 *   fem_pcg_comm_block: [host] the rank's comm block (device memory from hipMalloc: exportable with fem_ipc_handle)
 *   fem_pcg_col_window: [sync] min / max global column of the own rows (exchange between the ranks)
 *   fem_pcg_set_peers : every rank's comm block as mapped in THIS process (own entry ignored) and column window
 *   then fem_pcg_start on EVERY rank, a host barrier over the ranks, and fem_pcg_iterate / fem_pcg_profile /
 *   fem_pcg_poll with the same k on every rank (the first launch after a start forms r0 = b - A x0, u0 and r0.u0
 *   itself). fem_pcg_solve refuses such a context (it cannot place the barrier).
 * fem_ipc_handle / fem_ipc_open / fem_ipc_close: 64-byte hipIpcMemHandle of a device allocation, and its mapping in
 * another process (hipIpcMemLazyEnablePeerAccess). */
int fem_pcg_set_rows(fem_pcg* s, int nranks, int rank, const int64_t* slice_split, int grid);
int fem_pcg_comm_block(fem_pcg* s, void** base, int64_t* bytes);
int fem_pcg_col_window(fem_pcg* s, int64_t* lo, int64_t* hi);
int fem_pcg_set_peers(fem_pcg* s, void* const* bases, const int64_t* need_lo, const int64_t* need_hi);
/* [sync] diagnostics of a distributed persistent context into host_out[n]: which 0 = gather windows [G] first /
 * [G] last global workgroup + the column window, 1 = u-flag of every global workgroup in this rank's comm block,
 * 2 = publication table [G][nranks][2], 3 = rank epoch lines, 4 = local sync words (18 lines' first words) */
int fem_pcg_dist_debug(fem_pcg* s, int which, int32_t* host_out, int64_t n);
/* [host] a stream whose kernels run only on the CUs with cu % nparts == part (hipExtStreamCreateWithCUMask: its own
 * hardware queue) -- several emulated ranks of one process then run their persistent launches side by side */
int fem_stream_create_cu(int part, int nparts, void** stream);
int fem_stream_destroy(void* stream);
/* distributed persistent contexts: every later launch runs the phase-clock build (pcg_persist.hpp PROF) into dev_buf
 * ([G][8] phase sums, then [G][16] per-wave SpMV sums, as fem_pcg_persist_profile); NULL turns it off */
int fem_pcg_set_prof(fem_pcg* s, unsigned long long* dev_buf);
int fem_ipc_handle(void* ptr, char* out64);
int fem_ipc_open(const char* h64, void** ptr);
int fem_ipc_close(void* ptr);
/* [host] free the buffers that destroyed bs = 1 contexts left in the library's recycling cache (capped at
 * FEM355_PCG_CACHE_MB, default 1024 MB; invisible to torch's allocator); returns the MB released */
int fem_pcg_release_cache(void);
/* [host, sync] free the per-stream scratch buffers the library keeps between calls and trim its private stream-
 * ordered pools (capped at 256 MB of retained memory each) to zero; called by the Python layer at exit */
int fem_release_scratch(void);

/* ------------------------------------------------------------------ multi-GPU (element partition, RCCL)
 * One process per GPU. Every rank holds the SELL matrix of ITS elements over its local nodes (unassembled at
 * nodes shared with other ranks) and the global interface list: imap [nI] = local row of global interface node j
 * (-1 if the rank has no copy), ipos [nrows] = interface index of a local row (-1 interior), own [nrows] = 1 on
 * the rows the rank owns (owner = lowest rank touching the node). Each iteration then adds, on the device
 * stream: ONE all-reduce of the compact interface vector of A p (nI*bs doubles) with this rank's p.q partial
 * appended (p . q_rank over all local rows sums to p.q exactly), and one scalar all-reduce of r.z over owned
 * rows. The reference has no multi-device code; this replaces its
 * single-GPU region-growing split (`subdivision.ipynb:194-297`) with a deterministic partition.
 *   fem_comm_unique_id: [host] 128-byte RCCL id from rank 0 (broadcast it with any host transport)
 *   fem_comm_init     : [sync] communicator of this rank on the current HIP device */
int fem_comm_unique_id(char* out128);
int fem_comm_init(int nranks, int rank, const char* id128, void** comm);
int fem_comm_destroy(void* comm);
int fem_allreduce_sum(void* comm, double* buf, int64_t n, fem_stream_t stream);
/* v[interface rows] <- sum over ranks (buf: [nI*bs] scratch) = pack, all-reduce, unpack */
int fem_halo_pack(const double* v, int bs, const int32_t* imap, int64_t nI, double* buf, fem_stream_t stream);
int fem_halo_unpack(double* v, int bs, const int32_t* ipos, int64_t nrows, const double* buf, fem_stream_t stream);
int fem_halo_sum(void* comm, double* v, int bs, const int32_t* imap, int64_t nI, const int32_t* ipos, int64_t nrows,
                 double* buf, fem_stream_t stream);
/* switch a (P)CG context to the distributed iteration (enable=1; 3-kernel schedule, no graph). With comm = NULL
 * the exchanges are left to the caller, who drives the iteration phase by phase (below). */
int fem_pcg_set_dist(fem_pcg* s, int enable, void* comm, int64_t nI, const int32_t* imap, const int32_t* ipos,
                     const uint8_t* own);
/* Distributed iteration variant (call after fem_pcg_set_dist; resets on every fem_pcg_set_dist):
 *   0: the two-reduction PCG above (halo + p.q all-reduce, then the r.z all-reduce; six kernels per iteration)
 *   1: single reduction (Chronopoulos-Gear form of the same PCG): v = A u with u = z carried alongside r, so r.z,
 *      u.v and the interface rows of v ride in ONE all-reduce per iteration (three kernels). Same stop test and
 *      guards; rounding differs from variant 0 (N>1 contract: u within 1e-10, iterations within +-2).
 *      Phases: start 10 | sum | 20 | sum; iteration 4 | sum (buffer: fem_pcg_dist_buffer of that phase). */
int fem_pcg_set_dist_variant(fem_pcg* s, int variant);
/* neighbour exchange for the single-reduction variant (call after fem_pcg_set_dist_variant(s, 1)): the per-iteration
 * all-reduce of [interface rows | g | d] becomes ONE grouped ncclSend/ncclRecv with each of the npeer other ranks
 * (every other rank: the [g, d] pair travels to all). Message i (to and from peer_rank[i], peer_cnt[i] doubles) =
 * [g, d | bs values of each node shared with that rank, ascending global interface index]; the slot layout is the
 * same in both directions. csrc[J * nranks + r] (device int32, J over the nI global interface nodes) = offset of node
 * J's component 0 in the slot of rank r (-1: this rank, -2: r does not touch J or this rank does not); ssrc[r]
 * (device int32) = offset of rank r's [g, d] pair (-1: this rank). The SpMV kernel writes straight into the send
 * slots, the step/update kernels sum the received slots in rank order 0..nranks-1, so shared dofs stay
 * bit-identical across ranks. The maps stay owned by the caller (fem355.dist.p2p_maps builds them). */
int fem_pcg_set_p2p(fem_pcg* s, int nranks, int npeer, const int* peer_rank, const int64_t* peer_cnt,
                    const int32_t* csrc, const int32_t* ssrc);
/* the neighbour-exchange staging buffers (psend / precv, total doubles) */
int fem_pcg_p2p_buffers(fem_pcg* s, double** psend, double** precv, int64_t* total);
/* group path (all P ranks' contexts in one process, ctx[r] = rank r): every rank's message to each peer copied into
 * that peer's receive slot (what the grouped ncclSend/ncclRecv moves) */
int fem_p2p_deliver(fem_pcg* const* ctx, int P, fem_stream_t stream);
/* Phase-driven distributed iteration (what fem_pcg_start/iterate do around ncclAllReduce): phases 10, 11, 12
 * start the solve, phases 0..3 are one iteration; after a phase whose fem_pcg_dist_buffer is non-empty (10, 11:
 * start; 0: interface rows of A p + the p.q partial; 2: the r.z partial) that buffer must be summed over all ranks. Used to validate the distributed kernels with several
 * partitions in ONE process on one GPU (RCCL refuses two ranks on one device). */
int fem_pcg_dist_phase(fem_pcg* s, int phase);
int fem_pcg_dist_buffer(fem_pcg* s, int phase, double** ptr, int64_t* n);
/* dev_ptr_array: DEVICE array of P device pointers; sums the P buffers (rank order) into each of them */
int fem_group_allreduce(double* const* dev_ptr_array, int P, int64_t n, fem_stream_t stream);

/* ------------------------------------------------------------------ element-chunk operator (matrix-free c3d4)
 * y = K x of the c3d4 stiffness (kind FEM_KIND_ELASTIC, bs = 3: K_e of compute_c3d4_K_matrix, `solver/element.py:
 * 883-903`) or the P1 Laplacian (FEM_KIND_POISSON, bs = 1, kappa = E) formed element by element from the vertex
 * coordinates in every application -- the reference's element-by-element product `compute_nodal_forces`
 * (`solver/element.py:429-464`) without K_e in memory. Elements in Morton order, cut into chunks of <= 512 elements /
 * <= 256 nodes; per chunk a fixed-order sum per local node into a slot, per node a fixed-order sum of its slots
 * (deterministic). coords [N,3] and conn [M,4] (int64) must stay alive and unchanged while the operator is used.
 * FEM_ESINGULAR (*bad_idx = smallest element with |det| < 1e-12, `solver/element.py:857-858`), FEM_EARG for a node
 * outside [0, N). */
typedef struct fem_mf fem_mf;
int fem_mf_create(const double* coords, const int64_t* conn, int64_t M, int64_t N, int kind, double E, double nu,
                  int64_t* bad_idx, fem_stream_t stream, fem_mf** out);
int fem_mf_destroy(fem_mf* m);
/* y = K x ([N*bs] each; y overwritten) */
int fem_mf_apply(fem_mf* m, const double* x, double* y, fem_stream_t stream);
/* d = diag(K) [N*bs] (the exact diagonal) */
int fem_mf_diag(fem_mf* m, double* d, fem_stream_t stream);
/* debug builds only (-DFEM_MF_SPCHECK=1, tools/mf_spcheck.py): the stand-alone applications also carry each slot
 * position through the chunk walk's prefetch records and compare it at every store with the one read under the chunk;
 * out8 = {stores checked, mismatches, first mismatch (chunk << 16 | thread), carried, expected, walk step}, counters
 * reset. FEM_EARG in a normal build. */
int fem_mf_spcheck(uint64_t* out8);
/* out6 = {chunks, slots, bs, static bytes streamed per application, M, N} */
int fem_mf_info(fem_mf* m, int64_t* out6);
/* device copies of the layout (each nullable): Morton element order [M], chunk element offsets and slot offsets
 * [chunks + 1], slot nodes [slots] */
int fem_mf_order(fem_mf* m, int32_t* eorder, int32_t* cptr, int32_t* sbase, int32_t* cnode, fem_stream_t stream);
/* the context's operator becomes m (nrows = N, bs = m's; create the context with NULL slice_ptr / cols / vals):
 * K1 = the chunk kernel with the p.q reduction + the slot gather, then the merged update; modes PCG and CG_STABLE
 * (FEM_EARG for CG_CONSTRAINED, and fem_pcg_set_constraints refuses an operator context), schedule 0. The context
 * allocates its own slot buffer, so contexts (and fem_mf_apply / fem_mf_diag, which use the operator's) may run on
 * different streams at once. Distributed contexts (fem_pcg_set_dist, element partitions: m = the rank's own
 * elements over its local nodes) run the single-reduction iteration (variant 1, all-reduce or neighbour exchange,
 * not fused): per iteration k_cg1_update, the rank's chunks into the slots, and the slot gather that packs the
 * interface rows and the [g, d] pair -- BASELINE configs[3] with no assembled matrix (`solver/element.py:429-464`
 * per partition, `subdivision.ipynb:248-279`). */
int fem_pcg_set_operator_mf(fem_pcg* s, fem_mf* m);

#ifdef __cplusplus
}
#endif
#endif /* FEM355_H */
