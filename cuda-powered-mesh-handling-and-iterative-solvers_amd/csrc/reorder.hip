// Reverse Cuthill-McKee node renumbering on the device (opt-in; SURVEY §7: meshes arrive in file order through
// `vtk_loader_to_torch`, `solver/element.py:39-90`, and a file-ordered numbering gives the SELL slices scattered
// gathers and int32 columns).
//
// Level-synchronous Cuthill-McKee over the node graph (CSR rowptr / colidx, diagonal included): the next level is
// every unvisited neighbour of the current level; each such node's parent is its visited neighbour with the
// smallest CM index (atomicMin -> order-independent), and the children of a parent are numbered in their CSR
// order (ascending node id -- the id stands in for CM's degree key, so no sort is needed and the order is unique).
// Per level two launches, a wave per frontier node where a node's row is walked: k_cm_count counts every frontier
// node's children (the frontier split into one contiguous chunk per workgroup) and its last workgroup scans the
// chunk totals and advances the level (or starts the next component); k_cm_write numbers each chunk's children and
// marks the next level and its parents from them (k_cm_expand, for the start node only, marks level 1 alone). Levels run in
// batches without host round trips; the state words say when the last component is done. The sweep starts at the
// lowest-(degree, id) node (a boundary node: fewest neighbours); further components start at their lowest-id node;
// nodes no element touches go last. RCM = the reversed CM order.
#include <algorithm>

#include "common.hpp"

namespace fem {

enum { CM_B = 0, CM_E, CM_L, CM_CURSOR, CM_DONE, CM_LASTB, CM_TICKET, CM_WORDS = 16 };

__device__ __forceinline__ int cm_deg(const int32_t* rowptr, int64_t i) { return rowptr[i + 1] - rowptr[i]; }

// marks of level L + 1 from the frontier nodes [lo, hi) (CM indices), wave w of nw per node
__device__ __forceinline__ void cm_expand_range(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
                                                const int32_t* __restrict__ order, int32_t* __restrict__ level,
                                                int32_t* __restrict__ par, int lo, int hi, int L, int w, int nw) {
    const int lane = threadIdx.x & 63;
    for (int p = lo + w; p < hi; p += nw) {
        // device-coherent: in k_cm_write<true> another wave of this workgroup has just written order[p]
        const int u = __hip_atomic_load(order + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int q = rowptr[u] + lane; q < rowptr[u + 1]; q += 64) {
            const int v = colidx[q];
            const int lv = level[v];
            if (lv == -1 || lv == L + 1) {
                level[v] = L + 1;
                atomicMin(&par[v], p);
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_cm_expand(const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ colidx,
                                                   const int32_t* __restrict__ order, int32_t* __restrict__ level,
                                                   int32_t* __restrict__ par, const int32_t* __restrict__ st) {
    if (st[CM_DONE]) return;
    const int b = st[CM_B], e = st[CM_E], L = st[CM_L];
    // wave per frontier node: the row's neighbours in parallel
    const int lane = threadIdx.x & 63;
    for (int64_t p = b + ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)); p < e; p += (int64_t)gridDim.x * 4) {
        const int u = order[p];
        for (int q = rowptr[u] + lane; q < rowptr[u + 1]; q += 64) {
            const int v = colidx[q];
            const int lv = level[v];
            if (lv == -1 || lv == L + 1) {
                level[v] = L + 1;
                atomicMin(&par[v], (int)p);
            }
        }
    }
}

// block-wide exclusive scan of one int per thread (NT threads, NT / 64 <= 16 waves), total in *tot
template <int NT>
__device__ __forceinline__ int cm_scan_block(int v, int* lds, int* tot) {
    constexpr int NW = NT / 64;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    __syncthreads();
    if (lane == 63) lds[w] = x;
    __syncthreads();
    if (t < NW) {
        int s = lds[t];
        for (int o = 1; o < NW; o <<= 1) {
            const int y = __shfl_up(s, o, 64);
            if (t >= o) s += y;
        }
        lds[16 + t] = s;
    }
    __syncthreads();
    *tot = lds[16 + NW - 1];
    return x - v + (w > 0 ? lds[16 + w - 1] : 0);
}

// Count and write split the frontier [b, e) the same way: workgroup g of CM_G takes the contiguous chunk
// [b + g c, b + (g + 1) c), c = ceil(nf / CM_G), so the children of a chunk are numbered contiguously and only the
// CM_G chunk totals need a grid-wide scan (by the count kernel's last workgroup); each write workgroup scans its own
// chunk's counts.
constexpr int CM_G = 256;      // workgroups of k_cm_count / k_cm_write
constexpr int CM_NT = 1024;    // their threads
constexpr int CM_CHUNK = 4096; // chunk counts a write workgroup scans per round (LDS)

__device__ __forceinline__ void cm_chunk(int nf, int g, int* lo, int* hi) {
    const int c = (nf + CM_G - 1) / CM_G;
    *lo = min(g * c, nf);
    *hi = min(*lo + c, nf);
}

// the scan step of a level, by the count kernel's last workgroup: exclusive scan of the CM_G chunk totals (CM order)
// -> off[g], the next level's bounds; an empty frontier starts the next component (lowest-id unvisited node with
// neighbours) or finishes. part is read with device-coherent loads (written by the other workgroups).
__device__ void cm_scan_step(const int32_t* __restrict__ rowptr, int64_t N, int32_t* __restrict__ order,
                             int32_t* __restrict__ cm, int32_t* __restrict__ level, const int32_t* __restrict__ part,
                             int32_t* __restrict__ off, int32_t* __restrict__ st, int* lds, int* found) {
    const int b = st[CM_B], e = st[CM_E], L = st[CM_L];
    const int t = threadIdx.x;
    if (e == b) {
        if (t == 0) *found = INT_MAX;
        __syncthreads();
        for (int64_t c = st[CM_CURSOR]; c < N; c += 16 * CM_NT) {
#pragma unroll 4
            for (int j = 0; j < 16; ++j) {
                const int64_t i = c + j * CM_NT + t;
                if (i < N && level[i] == -1 && cm_deg(rowptr, i) > 0) atomicMin(found, (int)i);
            }
            __syncthreads();
            const bool hit = *found != INT_MAX;
            __syncthreads();   // every thread has read `found` before the next round's atomics
            if (hit) break;
        }
        __syncthreads();
        if (t == 0) {
            const int r = *found;
            if (r == INT_MAX) {
                st[CM_DONE] = 1;
            } else {
                order[e] = r;
                cm[r] = e;
                level[r] = 0;
                st[CM_CURSOR] = r + 1;
                st[CM_E] = e + 1;
                st[CM_L] = 0;
            }
        }
        return;
    }
    const int v = t < CM_G ? __hip_atomic_load(part + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    int running;
    const int ex = cm_scan_block<CM_NT>(v, lds, &running);
    if (t < CM_G) off[t] = ex;
    if (t == 0) {
        st[CM_B] = e;
        st[CM_E] = e + running;
        st[CM_L] = L + 1;
        st[CM_LASTB] = b;   // the level just numbered from (k_cm_write's parents)
    }
}

// children of frontier node p (CM index): unvisited-at-L neighbours whose parent is p; wave per frontier node of the
// workgroup's chunk. The chunk total goes to part[g]; the last workgroup to finish (ticket) runs the level's scan
// step, so a level takes three launches
__global__ void __launch_bounds__(CM_NT) k_cm_count(const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ colidx, int64_t N,
                                                    int32_t* __restrict__ order, int32_t* __restrict__ cm,
                                                    int32_t* __restrict__ level, const int32_t* __restrict__ par,
                                                    int32_t* __restrict__ cnt, int32_t* __restrict__ part,
                                                    int32_t* __restrict__ off, int32_t* __restrict__ st) {
    __shared__ int lds[32];
    __shared__ int wsum[CM_NT / 64];
    __shared__ int found;
    __shared__ int last;
    if (st[CM_DONE]) return;   // uniform: no workgroup takes a ticket
    const int b = st[CM_B], e = st[CM_E], L = st[CM_L];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int lo, hi;
    cm_chunk(e - b, blockIdx.x, &lo, &hi);
    int ws = 0;
    for (int i = lo + wv; i < hi; i += CM_NT / 64) {
        const int p = b + i;
        const int u = order[p];
        int c = 0;
        for (int q0 = rowptr[u]; q0 < rowptr[u + 1]; q0 += 64) {
            const int q = q0 + lane;
            bool ch = false;
            if (q < rowptr[u + 1]) {
                const int v = colidx[q];
                ch = level[v] == L + 1 && par[v] == p;
            }
            c += __popcll(__ballot(ch));
        }
        if (lane == 0) cnt[i] = c;
        ws += c;
    }
    if (lane == 0) wsum[wv] = ws;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
#pragma unroll
        for (int w = 0; w < CM_NT / 64; ++w) tot += wsum[w];
        __hip_atomic_store(part + blockIdx.x, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // this workgroup's total before its ticket
        const int tk = __hip_atomic_fetch_add(st + CM_TICKET, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = tk == (int)gridDim.x - 1;
        if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (!last) return;
    if (threadIdx.x == 0) st[CM_TICKET] = 0;   // for the next level's launch
    cm_scan_step(rowptr, N, order, cm, level, part, off, st, lds, &found);
}

// the children of the chunk's frontier nodes in CSR order: node p's start = the level's first index + off[g] + the
// exclusive scan of the chunk's counts up to p; wave per frontier node. EXPAND: the same launch then marks the
// next level from the children it numbered (k_cm_expand's work), so a level takes two launches
template <bool EXPAND>
__global__ void __launch_bounds__(CM_NT) k_cm_write(const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ colidx, int32_t* __restrict__ order,
                                                    int32_t* __restrict__ cm, int32_t* __restrict__ level,
                                                    int32_t* __restrict__ par, const int32_t* __restrict__ cnt,
                                                    const int32_t* __restrict__ off, const int32_t* __restrict__ st) {
    __shared__ int lds[32];
    __shared__ int base_s[CM_CHUNK];
    if (st[CM_DONE]) return;
    // k_cm_count's scan step has advanced the state: parents are [LASTB, B), children start at B; a new component
    // (L == 0) has nothing to write
    const int L = st[CM_L];
    if (!EXPAND && L == 0) return;
    const int b = L == 0 ? 0 : st[CM_LASTB], e = L == 0 ? 0 : st[CM_B];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    int lo, hi;
    cm_chunk(e - b, blockIdx.x, &lo, &hi);
    int run = e + off[blockIdx.x];
    for (int r0 = lo; r0 < hi; r0 += CM_CHUNK) {   // the chunk's first-child indices, CM_CHUNK nodes at a time
        const int r1 = min(r0 + CM_CHUNK, hi);
        for (int i0 = r0; i0 < r1; i0 += CM_NT) {
            const int i = i0 + (int)threadIdx.x;
            const int v = i < r1 ? cnt[i] : 0;
            int tot;
            const int ex = cm_scan_block<CM_NT>(v, lds, &tot);
            if (i < r1) base_s[i - r0] = run + ex;
            run += tot;
        }
        __syncthreads();
        for (int i = r0 + wv; i < r1; i += CM_NT / 64) {
            const int p = b + i;
            const int u = order[p];
            int k = base_s[i - r0];
            for (int q0 = rowptr[u]; q0 < rowptr[u + 1]; q0 += 64) {
                const int q = q0 + lane;
                bool ch = false;
                int v = 0;
                if (q < rowptr[u + 1]) {
                    v = colidx[q];
                    ch = level[v] == L && par[v] == p;
                }
                const unsigned long long m = __ballot(ch);
                if (ch) {
                    const int kk = k + __popcll(m & lt);
                    order[kk] = v;
                    cm[v] = kk;
                }
                k += __popcll(m);
            }
        }
        __syncthreads();   // base_s consumed before the next round
    }
    // then the next level from the children just numbered here: [e + off[g], run) (a new component, L == 0: its
    // start node, taken by workgroup 0); every level-L node is final, so the marks of level L + 1 cannot meet a
    // node another workgroup is still numbering
    if constexpr (EXPAND) {
        int xlo = e + off[blockIdx.x], xhi = run;
        if (L == 0) {
            xlo = blockIdx.x == 0 ? st[CM_B] : 0;
            xhi = blockIdx.x == 0 ? st[CM_E] : 0;
        }
        cm_expand_range(rowptr, colidx, order, level, par, xlo, xhi, L, wv, CM_NT / 64);
    }
}

// lowest-degree non-isolated node (then lowest id) of the whole graph -> *key; one atomic per wave (one per node
// serialised 1.7M atomics on one word: 311 us at 10M)
__global__ void k_cm_min_degree(const int32_t* __restrict__ rowptr, int64_t N, unsigned long long* __restrict__ key) {
    unsigned long long best = ~0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        const int d = cm_deg(rowptr, i);
        const unsigned long long k = ((unsigned long long)(unsigned)d << 32) | (unsigned)i;
        if (d > 0 && k < best) best = k;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(best, o, 64);
        best = y < best ? y : best;
    }
    if ((threadIdx.x & 63) == 0 && best != ~0ull) atomicMin(key, best);
}

__global__ void k_cm_reset(int32_t* __restrict__ level, int32_t* __restrict__ par, int32_t* __restrict__ cm,
                           int64_t N, int32_t* __restrict__ order, int32_t* __restrict__ st,
                           const unsigned long long* __restrict__ key) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        level[i] = -1;
        par[i] = INT_MAX;
        cm[i] = -1;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long k = *key;
        for (int w = 0; w < CM_WORDS; ++w) st[w] = 0;
        if (k == ~0ull) {   // no edges at all
            st[CM_DONE] = 1;
            return;
        }
        const int r = (int)(k & 0xffffffffu);
        order[0] = r;
        st[CM_E] = 1;
    }
}

// the start node must be marked after the reset has covered it (separate launch, one thread)
__global__ void k_cm_seed(int32_t* __restrict__ level, int32_t* __restrict__ cm, const int32_t* __restrict__ order,
                          const int32_t* __restrict__ st) {
    if (st[CM_DONE]) return;
    const int r = order[0];
    level[r] = 0;
    cm[r] = 0;
}

// isolated nodes (no element) after the components, ascending id; flags -> positions by the caller's scan
__global__ void k_cm_isolated_flags(const int32_t* __restrict__ rowptr, int64_t N, int32_t* __restrict__ flag) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x)
        flag[i] = cm_deg(rowptr, i) == 0;
}

// RCM: node order[k] gets new id N - 1 - k; isolated node i gets base + pos[i]
__global__ void k_cm_finish(const int32_t* __restrict__ rowptr, int64_t N, const int32_t* __restrict__ order,
                            const int32_t* __restrict__ pos, const int32_t* __restrict__ st, int32_t* __restrict__ perm,
                            int32_t* __restrict__ inv) {
    const int ncm = st[CM_E];   // nodes numbered by the CM sweeps
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        if (i < ncm) {
            const int v = order[i];
            const int64_t nw = ncm - 1 - i;
            perm[nw] = v;
            inv[v] = (int32_t)nw;
        }
        if (cm_deg(rowptr, i) == 0) {
            const int64_t nw = ncm + pos[i];
            perm[nw] = (int32_t)i;
            inv[i] = (int32_t)nw;
        }
    }
}

}  // namespace fem

using namespace fem;

extern "C" {

// per-array stride of the workspace: a multiple of 64 ints, so every array (and the 8-byte key) stays aligned
// (at least 2 CM_G: the chunk offsets and totals share one array)
static int64_t rcm_stride(int64_t N) { return (std::max<int64_t>(N + 64, 2 * CM_G) + 63) & ~(int64_t)63; }

int64_t fem_rcm_work_len(int64_t N) { return 7 * rcm_stride(N) + CM_WORDS + 8 + fem_scan_work_len(N); }

int fem_rcm(const int32_t* rowptr, const int32_t* colidx, int64_t N, int32_t* perm, int32_t* inv, int32_t* work,
            int* levels_out, fem_stream_t stream) {
    hipStream_t st = S(stream);
    if (N <= 0) return FEM_OK;
    if (N >= (int64_t)1 << 31) {
        set_error("fem_rcm: %lld nodes exceed int32", (long long)N);
        return FEM_EARG;
    }
    if (reinterpret_cast<uintptr_t>(work) & 7) {
        set_error("fem_rcm: work must be 8-byte aligned");
        return FEM_EARG;
    }
    const int64_t S = rcm_stride(N);
    int32_t* level = work;
    int32_t* par = level + S;
    int32_t* cm = par + S;
    int32_t* order = cm + S;
    int32_t* pos = order + S;
    int32_t* cnt = pos + S;
    int32_t* off = cnt + S;           // [CM_G] chunk offsets
    int32_t* part = off + CM_G;       // [CM_G] chunk totals (S >= 2 CM_G)
    int32_t* sw = off + S;
    unsigned long long* key = reinterpret_cast<unsigned long long*>(sw + CM_WORDS);   // 8-byte aligned: S % 64 == 0
    int32_t* swork = sw + CM_WORDS + 8;
    const int g = stream_grid(N, 256);
    const int ge = 1024;   // expand grid: 4096 waves, one frontier node each
    constexpr int BATCH = 48;
    int state[CM_WORDS];
    int levels = 0;
    FEM_HIP(hipMemsetAsync(key, 0xff, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_cm_min_degree, dim3(g), dim3(256), 0, st, rowptr, N, key);
    FEM_LAUNCHED();
    hipLaunchKernelGGL(k_cm_reset, dim3(g), dim3(256), 0, st, level, par, cm, N, order, sw, key);
    FEM_LAUNCHED();
    hipLaunchKernelGGL(k_cm_seed, dim3(1), dim3(1), 0, st, level, cm, order, sw);
    FEM_LAUNCHED();
    // the start node's level, then per level: count (+ scan step), write (+ the next level's marks)
    hipLaunchKernelGGL(k_cm_expand, dim3(ge), dim3(256), 0, st, rowptr, colidx, order, level, par, sw);
    for (;;) {
        for (int k = 0; k < BATCH; ++k) {
            hipLaunchKernelGGL(k_cm_count, dim3(CM_G), dim3(CM_NT), 0, st, rowptr, colidx, N, order, cm, level, par,
                               cnt, part, off, sw);
            hipLaunchKernelGGL(k_cm_write<true>, dim3(CM_G), dim3(CM_NT), 0, st, rowptr, colidx, order, cm, level,
                               par, cnt, off, sw);
        }
        FEM_LAUNCHED();
        FEM_HIP(hipMemcpyAsync(state, sw, sizeof(state), hipMemcpyDeviceToHost, st));
        FEM_HIP(hipStreamSynchronize(st));
        levels += BATCH;
        if (state[CM_DONE]) break;
    }
    hipLaunchKernelGGL(k_cm_isolated_flags, dim3(g), dim3(256), 0, st, rowptr, N, level);   // level reused
    FEM_LAUNCHED();
    const int rc = fem_scan_i32(level, N, pos, swork, stream);
    if (rc != FEM_OK) return rc;
    hipLaunchKernelGGL(k_cm_finish, dim3(g), dim3(256), 0, st, rowptr, N, order, pos, sw, perm, inv);
    FEM_LAUNCHED();
    if (levels_out) *levels_out = levels;
    return FEM_OK;
}

}  // extern "C"
