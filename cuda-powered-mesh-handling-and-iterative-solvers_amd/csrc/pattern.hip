// Mesh graph construction on the device: node->element incidence, node-graph CSR pattern, SELL-64 layout.
//
// The reference never assembles a CSR on its hot path (it is element-by-element, `solver/element.py:429-464`);
// its only global matrix is the COO of `subdivision.ipynb:118-139`, coalesced by torch. The pattern built here
// is exactly coalesce(COO) at node granularity (bit-exact against oracle.ref_cpu.node_pattern): every row
// lists the unique nodes sharing an element with it, ascending.
#include <algorithm>

#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "sell_pair.hpp"   // sl_pattern_slice (the bs = 1 solver layout, formed in the fill pass)

namespace fem {

// ---------------------------------------------------------------- incidence
// Radix form (FEM355_INC_RADIX; the bucket sort below is the default): stable radix sort of (node, slot) pairs,
// slot = e * npe + local: every node's slots come out ascending. An
// out-of-range node id raises *bad and is keyed N (sorted past every node, outside every inc_ptr range). Measured
// against a counting sort (atomic counts, scan, atomic scatter, per-node segment sort): 2.1 ms vs 1.2 ms on the 10M
// cube -- 40M scattered device atomics twice (count + scatter) cost more than the three sort passes.
__global__ void k_inc_keys(const int64_t* __restrict__ conn, int64_t total, int64_t N, int32_t* __restrict__ key,
                           int32_t* __restrict__ slot, int32_t* __restrict__ bad) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t v = conn[i];
        if (v < 0 || v >= N) {
            if (bad) *bad = 1;
            v = N;
        }
        key[i] = (int32_t)v;
        slot[i] = (int32_t)i;
    }
}

// inc_ptr[n] = first sorted position whose node is >= n (run boundaries of the sorted keys; keys N = bad slots)
__global__ void k_inc_ptr(const int32_t* __restrict__ key, int64_t total, int64_t N, int32_t* __restrict__ inc_ptr) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= total; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t prev = p == 0 ? -1 : key[p - 1];
        const int64_t cur = p == total ? N : key[p];
        for (int64_t n = prev + 1; n <= cur; ++n) inc_ptr[n] = (int32_t)p;
    }
}

// Bucket sort (default): the same incidence in two levels with no device-wide atomics. Level 1 buckets the slots
// by node >> bsh (a bucket = 2^bsh consecutive nodes): every workgroup histograms a contiguous chunk of slots in
// LDS, one scan over the (bucket, workgroup) counts gives every workgroup its run inside every bucket, and the
// chunk is scattered into those runs as (node, slot) pairs. Level 2 is one workgroup per bucket: counts per node,
// scan (writing inc_ptr), scatter into per-node segments and a rank sort of every segment, in LDS when the bucket
// holds at most INB_CAP entries (global scratch otherwise) -- every node's slots ascending, the unique result.
// A wave's 64 consecutive slots mostly fall into one or two buckets / nodes: the lanes that share the first
// lane's bucket (node) are counted by one ballot and one LDS atomic.
constexpr int INB_G1 = 512;        // level-1 workgroups (chunks of slots), 1024 threads each
constexpr int INB_T1 = 1024;
constexpr int INB_MAXB = 16384;    // buckets (LDS histogram of level 1: 64 KB)
constexpr int INB_CAP = 3584;      // entries of a bucket sorted in LDS (10 bytes each)
constexpr int INC_BIG = 4096;      // node segments longer than this are sorted by k_inc_big (> INB_CAP: global tier)
constexpr int INB_MAXSH = 8;       // at most 256 nodes per bucket: N <= 4M nodes (larger meshes: the radix form)

static int inb_shift(int64_t N) {   // bucket = 128 nodes, 256 when N / 128 would exceed INB_MAXB buckets
    int b = 7;
    while ((N + ((int64_t)1 << b) - 1) >> b > INB_MAXB) ++b;
    return b;
}

// one LDS add per distinct key for the first AGG key groups of the wave (the group of the lowest remaining lane,
// found by one ballot), ones for the lanes left after them; returns the lane's slot for the scatter variant (base of
// its group + rank among the lanes of the same key)
#ifndef FEM_INC_AGG
#define FEM_INC_AGG 1   // level 1 at 10M: 1 group 146 + 215 us, 4 groups 156 + 225, 8 groups 151 + 224
#endif
template <bool SCATTER, int AGG = 1>
__device__ __forceinline__ int agg_add(int* lds, int key, bool valid) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    unsigned long long rem = __ballot(valid);
    int pos = -1;
#pragma unroll
    for (int g = 0; g < AGG; ++g) {
        if (!rem) return pos;
        const int src = __ffsll((long long)rem) - 1;
        const int k0 = __shfl(key, src, 64);
        const bool same = ((rem >> lane) & 1) && key == k0;
        const unsigned long long ms = __ballot(same);
        int base = 0;
        if (lane == src) base = atomicAdd(&lds[k0], __popcll(ms));
        if (SCATTER) {
            base = __shfl(base, src, 64);
            if (same) pos = base + __popcll(ms & lt);
        }
        rem &= ~ms;
    }
    if ((rem >> lane) & 1) {
        const int p = atomicAdd(&lds[key], 1);
        if (SCATTER) pos = p;
    }
    return pos;
}

template <bool SCATTER>
__global__ void __launch_bounds__(INB_T1) k_inc_l1(const int64_t* __restrict__ conn, int64_t total, int64_t N, int bsh,
                                                int nb, int32_t* __restrict__ cnt, const int32_t* __restrict__ off,
                                                int2* __restrict__ kpair,
                                                int32_t* __restrict__ bad) {
    extern __shared__ int hist[];
    const int G = gridDim.x, b = blockIdx.x;
    const int64_t c0 = total * b / G, c1 = total * (b + 1) / G;
    for (int q = threadIdx.x; q < nb; q += INB_T1) hist[q] = SCATTER ? off[(int64_t)q * G + b] : 0;
    __syncthreads();
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int U1 = 4;   // windows of 64 slots per wave whose loads are in flight together
    for (int64_t w0 = c0 + wid * 64; w0 < c1; w0 += (int64_t)U1 * INB_T1) {
        int64_t vv[U1];
#pragma unroll
        for (int u = 0; u < U1; ++u) {
            const int64_t i = w0 + (int64_t)u * INB_T1 + lane;
            vv[u] = i < c1 ? conn[i] : -1;
        }
#pragma unroll
        for (int u = 0; u < U1; ++u) {
            const int64_t i = w0 + (int64_t)u * INB_T1 + lane;
            const int64_t v = vv[u];
            bool valid = i < c1;
            if (valid && (v < 0 || v >= N)) {
                if (!SCATTER && bad) *bad = 1;
                valid = false;
            }
            const int key = valid ? (int)(v >> bsh) : 0;
            const int pos = agg_add<SCATTER, FEM_INC_AGG>(hist, key, valid);   // a wave's slots: a few buckets
            if (SCATTER && valid) {
                kpair[pos] = make_int2((int32_t)v, (int32_t)i);   // (node, slot): one 8-byte store
            }
        }
    }
    if (!SCATTER) {
        __syncthreads();
        for (int q = threadIdx.x; q < nb; q += INB_T1) cnt[(int64_t)q * G + b] = hist[q];
        if (b == 0 && threadIdx.x == 0) cnt[(int64_t)nb * G] = 0;   // the hub flag k_inc_l2 sets (k_inc_big's gate)
    }
}

#ifndef FEM_INC_NOSORT
#define FEM_INC_NOSORT 0
#endif
// level 2: one workgroup per bucket; boff = the level-1 scan (bucket q's entries [boff[q G], boff[(q + 1) G]))
__global__ void __launch_bounds__(256) k_inc_l2(const int2* __restrict__ kpair,
                                                const int32_t* __restrict__ boff, int G, int64_t N, int bsh,
                                                int32_t* __restrict__ scratch, int32_t* __restrict__ inc_ptr,
                                                int32_t* __restrict__ inc, int32_t* __restrict__ hub) {
    extern __shared__ int lds[];
    const int B = 1 << bsh;
    int* cnt = lds;                 // [B] counts, then cursors
    int* st = lds + B;              // [B + 1] segment starts (bucket-relative)
    int* ls = st + B + 1;           // [INB_CAP] slot of each entry
    int* out = ls + INB_CAP;        // [INB_CAP] slots in node segments
    uint8_t* ln = reinterpret_cast<uint8_t*>(out + INB_CAP);   // [INB_CAP] node (bucket-relative) of each entry
    uint8_t* on = ln + INB_CAP;                                 // [INB_CAP] node of each position
    const int q = blockIdx.x;
    const int64_t node0 = (int64_t)q << bsh;
    const int nn = (int)min((int64_t)B, N - node0);
    const int lo = boff[(int64_t)q * G], hi = boff[(int64_t)(q + 1) * G], n = hi - lo;
    const bool fits = n <= INB_CAP;
    for (int j = threadIdx.x; j < B; j += 256) cnt[j] = 0;
    __syncthreads();
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (fits) {   // every entry of the thread loaded before the first count (the loads in flight together)
        constexpr int EPT = INB_CAP / 256;
        int kn_r[EPT], ks_r[EPT];
#pragma unroll
        for (int u = 0; u < EPT; ++u) {
            const int e = u * 256 + threadIdx.x;
            const int2 kp = e < n ? kpair[lo + e] : make_int2(0, 0);
            kn_r[u] = kp.x;
            ks_r[u] = kp.y;
        }
#pragma unroll
        for (int u = 0; u < EPT; ++u) {
            const int e = u * 256 + threadIdx.x;
            const bool valid = e < n;
            const int kn = valid ? (int)(kn_r[u] - node0) : 0;
            if (valid) {
                ln[e] = (uint8_t)kn;
                ls[e] = ks_r[u];
            }
            agg_add<false>(cnt, kn, valid);
        }
    } else {
        for (int e0 = wid * 64; e0 < n; e0 += 256) {
            const int e = e0 + lane;
            const bool valid = e < n;
            const int kn = valid ? (int)(kpair[lo + e].x - node0) : 0;
            agg_add<false>(cnt, kn, valid);
        }
    }
    __syncthreads();
    if (threadIdx.x < 64) {   // exclusive scan of the bucket's node counts by wave 0 (B / 64 counts per lane)
        const int per = B >> 6;   // B = 128 or 256
        int v[4] = {0, 0, 0, 0}, sum = 0;
        for (int u = 0; u < per; ++u) {
            v[u] = cnt[lane * per + u];
            sum += v[u];
        }
        int x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        int run = x - sum;
        for (int u = 0; u < per; ++u) {
            st[lane * per + u] = run;
            run += v[u];
        }
        if (lane == 63) st[B] = x;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < nn; j += 256) inc_ptr[node0 + j] = lo + st[j];
    if (node0 + nn == N && threadIdx.x == 0) inc_ptr[N] = hi;
    for (int j = threadIdx.x; j < B; j += 256) cnt[j] = st[j];
    __syncthreads();
    // into node segments (arrival order inside a segment); the two tiers in separate loops, so the LDS tier's reads
    // stay ds_read (a pointer that may be LDS or global makes flat loads)
    if (fits) {
        for (int e0 = wid * 64; e0 < n; e0 += 256) {
            const int e = e0 + lane;
            const bool valid = e < n;
            const int kn = valid ? (int)ln[e] : 0;
            const int p = agg_add<true>(cnt, kn, valid);
            if (valid) {
                out[p] = ls[e];
                on[p] = (uint8_t)kn;
            }
        }
    } else {
        for (int e0 = wid * 64; e0 < n; e0 += 256) {
            const int e = e0 + lane;
            const bool valid = e < n;
            const int2 kp = valid ? kpair[lo + e] : make_int2(0, 0);
            const int kn = valid ? (int)(kp.x - node0) : 0;
            const int p = agg_add<true>(cnt, kn, valid);
            if (valid) scratch[lo + p] = kp.y;
        }
    }
    __syncthreads();
    if (!fits) __threadfence_block();
    // rank sort of every segment: position = segment start + number of smaller slots in the segment
    for (int p = threadIdx.x; p < n; p += 256) {
        int v, a, z;
        if (fits) {
            v = out[p];
            const int j = on[p];
            a = st[j];
            z = st[j + 1];
#if FEM_INC_NOSORT   // timing builds only (wrong order): the segments left in arrival order
            (void)j; (void)z;
            inc[lo + p] = v;
#else
            // rank = segment start + the number of smaller slots in the segment; four LDS reads in flight per step
            // (one dependent read per step made the ~24-long segments a chain of LDS latencies)
            int r = a, u = a;
            for (; u + 4 <= z; u += 4) {
                const int o0 = out[u], o1 = out[u + 1], o2 = out[u + 2], o3 = out[u + 3];
                r += (int)(o0 < v) + (int)(o1 < v) + (int)(o2 < v) + (int)(o3 < v);
            }
            for (; u < z; ++u) r += (out[u] < v);
            inc[lo + r] = v;
#endif
        } else {
            v = scratch[lo + p];
            int l = 0, h = B;   // segment of position p: last j with st[j] <= p
            while (h - l > 1) {
                const int m = (l + h) >> 1;
                if (st[m] <= p) l = m;
                else h = m;
            }
            while (l + 1 < B && st[l + 1] <= p) ++l;   // empty segments share a start
            a = st[l];
            z = st[l + 1];
            if (z - a > INC_BIG) {   // a hub's segment: k_inc_big sorts it (the rank sort is O(len^2))
                *hub = 1;
                continue;
            }
            int r = a;
            for (int u = a; u < z; ++u) r += (scratch[lo + u] < v);
            inc[lo + r] = v;
        }
    }
}

// ---------------------------------------------------------------- node graph (wave per node)
constexpr int G_WAVES = 4;      // waves per block
constexpr int G_UCAP = 512;     // unique-neighbour capacity of k_graph (larger rows: k_graph_big)
constexpr int G_SCAP = 384;     // candidate capacity of the small-row kernel
constexpr int G_TCAP = 32;      // rows of at most this many neighbours are produced by k_graph_small

// Small rows in one pass (every P1 / Q1 / wedge row of ordinary meshes): wave per node, candidates deduplicated
// through a wave-private LDS hash table (linear probing, compare-and-swap; the row's own node added after), the
// unique set compacted
// and rank-sorted, written to tmp[node * G_TCAP + rank] with row_len[node]. Rows with more than G_SCAP candidates or
// G_TCAP neighbours get tmp[node * G_TCAP] = -1 and are left to k_graph (count and fill passes skip the rest).
constexpr int G_HT = 512;
// tmp's deferral flags are followed by one int: the number of rows k_graph_small deferred (0: the deferred-row
// kernels return at once; zeroed by fem_graph_count2)
__device__ __forceinline__ int32_t* ndefer_out(uint8_t* defer, int64_t N) {
    return reinterpret_cast<int32_t*>(defer) + (N + 3) / 4;
}
#ifndef FEM_GRAPH_LPN
#define FEM_GRAPH_LPN 32   // k_graph_small lanes per node (two rows per wave)
#endif

// hash table of a row: the smallest power of two >= 2 C slots (at least 128, at most 1 << maxbits), so clearing
// and compacting it costs ~C, not the table capacity (P1 rows: 96 candidates -> 256 slots instead of 512)
__device__ __forceinline__ int ht_bits(int C, int maxbits) {
    const int b = (C <= 64) ? 7 : 32 - __clz(2 * C - 1);
    return b > maxbits ? maxbits : b;
}

// LPN lanes per node (64 or 32): with 32 each half-wave builds its own row in half the wave's table, so two rows'
// dependent incidence / connectivity loads are in flight per wave; rows over LPN / 64 * G_SCAP candidates defer.
// NPE > 0 (even, connectivity rows 16-byte aligned): a lane takes whole incidences -- the element's node ids in
// NPE / 2 16-byte loads of one row -- instead of one node id per candidate slot (NPE = 0: any npe)
template <int LPN, int NPE>
__global__ void __launch_bounds__(256) k_graph_small(const int64_t* __restrict__ conn, int npe,
                                                     const int32_t* __restrict__ inc_ptr,
                                                     const int32_t* __restrict__ inc, int64_t N,
                                                     int32_t* __restrict__ row_len, int32_t* __restrict__ tmp,
                                                     uint8_t* __restrict__ defer, int32_t* __restrict__ far) {
    constexpr int NPW = 64 / LPN;                 // nodes per wave
    constexpr int HTS = G_HT / NPW;               // table slots per node
    constexpr int SCAP = G_SCAP * LPN / 64;       // candidates per node (load <= 3/4 of the table)
    constexpr int MAXB = (HTS == 512) ? 9 : (HTS == 256 ? 8 : 7);
    constexpr int LB = LPN == 64 ? 6 : 5;         // log2(LPN): the compaction reads LPN slots at a time
    __shared__ int ht[G_WAVES][G_HT];
    __shared__ int uniq[G_WAVES][64];
    const int wid = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int sub = lane / LPN, sl = lane - LPN * sub, base = LPN * sub;
    int* const tab = &ht[wid][HTS * sub];
    int* const uq = &uniq[wid][base];
    const unsigned long long lt_mask = (sl == 0) ? 0ull : (~0ull >> (64 - sl));
    const unsigned long long my_bits = (LPN == 64) ? ~0ull : (((1ull << LPN) - 1) << base);
    for (int64_t node = ((int64_t)blockIdx.x * G_WAVES + wid) * NPW + sub; node < N;
         node += (int64_t)gridDim.x * G_WAVES * NPW) {
        const int start = inc_ptr[node];
        const int C = (inc_ptr[node + 1] - start) * npe;
        int32_t* trow = tmp + node * G_TCAP;
        if (C > SCAP) {
            if (sl == 0) {
                defer[node] = 1;
                atomicAdd(ndefer_out(defer, N), 1);
            }
            continue;
        }
        // the row's own node is in every incidence: it is left out of the hash (a quarter of the P1 inserts) and
        // added after the compaction; the table holds the other candidates' distinct values (at most Cn) with a free
        // slot to end every probe, and at least one slot per lane
        const int Cn = C - C / npe;
        const int hbw = 32 - __clz(Cn);   // smallest b with 2^b > Cn
        const int hb = hbw < LB ? LB : (hbw > MAXB ? MAXB : hbw), HS = 1 << hb;
        // all of the lane's candidates loaded before any insert (the incidence loads, then the connectivity loads,
        // in flight together instead of one dependent pair per insert)
        constexpr int IPL = NPE > 0 ? (SCAP / (NPE > 0 ? NPE : 1) + LPN - 1) / LPN : 0;   // incidences per lane
        constexpr int CPL = NPE > 0 ? IPL * NPE : (SCAP + LPN - 1) / LPN;
        int cand[CPL];
        if constexpr (NPE > 0) {
            const int ninc = C / NPE;
            int el[IPL];
#pragma unroll
            for (int u = 0; u < IPL; ++u) {
                const int t = sl + u * LPN;
                el[u] = t < ninc ? inc[start + t] / NPE : -1;
            }
#pragma unroll
            for (int u = 0; u < IPL; ++u) {
#pragma unroll
                for (int h = 0; h < NPE; ++h) cand[u * NPE + h] = -1;
                if (el[u] >= 0) {   // no load for an empty slot (an element-free mesh may pass no connectivity)
                    const longlong2* row = reinterpret_cast<const longlong2*>(conn + (int64_t)el[u] * NPE);
#pragma unroll
                    for (int h = 0; h < NPE / 2; ++h) {
                        const longlong2 v = row[h];
                        cand[u * NPE + 2 * h] = (int)v.x;
                        cand[u * NPE + 2 * h + 1] = (int)v.y;
                    }
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                const int t = sl + u * LPN;
                cand[u] = t < C ? inc[start + t / npe] : 0;
            }
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                const int t = sl + u * LPN;
                cand[u] = t < C ? (int)conn[(int64_t)(cand[u] / npe) * npe + (t - (t / npe) * npe)] : -1;
            }
        }
        for (int q = sl; q < HS; q += LPN) tab[q] = -1;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const int v = cand[u];
            if (v < 0 || v == (int)node) continue;
            unsigned h = ((unsigned)v * 2654435761u) >> (32 - hb);
            while (true) {
                const int old = atomicCAS(&tab[h], -1, v);
                if (old == -1 || old == v) break;
                h = (h + 1) & (HS - 1);
            }
        }
        __builtin_amdgcn_wave_barrier();
        int U = 0;
        for (int q0 = 0; q0 < HS; q0 += LPN) {
            const int v = tab[q0 + sl];
            const bool has = v >= 0;
            const unsigned long long m = (__ballot(has) & my_bits) >> base;
            if (has) {
                const int pos = U + __popcll(m & lt_mask);
                if (pos < LPN) uq[pos] = v;
            }
            U += __popcll(m);
        }
        if (C > 0) {   // the row's own node
            if (sl == U && U < LPN) uq[U] = (int)node;
            ++U;
        }
        __builtin_amdgcn_wave_barrier();
        if (U > G_TCAP || U > LPN) {
            if (sl == 0) {
                defer[node] = 1;
                atomicAdd(ndefer_out(defer, N), 1);
            }
            continue;
        }
        bool f = false;   // a neighbour farther than 16-bit deltas reach (the SELL keeps int32 columns then)
        if (sl < U) {
            const int v = uq[sl];
            int rank = 0;
            for (int u = 0; u < U; ++u) rank += (uq[u] < v);
            trow[rank] = v;
            f = v - node > 32767 || node - v > 32767;
        }
        if (far) {
            const unsigned long long fb = __ballot(f);
            if (fb && lane == __ffsll((long long)fb) - 1 && !*far) atomicOr(far, 1);
        }
        if (sl == 0) {
            row_len[node] = U;
            defer[node] = 0;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// rows of k_graph_small -> CSR colidx / diagpos (only the row's own entries of tmp are read)
__global__ void k_graph_copy(const int32_t* __restrict__ tmp, const uint8_t* __restrict__ defer,
                             const int32_t* __restrict__ rowptr, int64_t N, int32_t* __restrict__ colidx,
                             int32_t* __restrict__ diagpos) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < N * G_TCAP; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t node = t / G_TCAP;
        const int j = (int)(t - node * G_TCAP);
        if (defer[node]) continue;
        const int rp = rowptr[node], len = rowptr[node + 1] - rp;
        if (j >= len) continue;
        const int v = tmp[t];
        colidx[rp + j] = v;
        if (v == (int)node) diagpos[node] = rp + j;
    }
}

// Rows beyond k_graph_small (c3d10 corner rows, dense fans): wave per node, candidates streamed from the incidence
// list straight into a wave-private 2048-slot LDS hash (no candidate-count limit), the unique set compacted and
// rank-sorted. A row whose unique count passes G_UCAP stops inserting (the table never holds more than
// G_UCAP + 64 keys, so probing always ends) and is marked row_len = -1 for k_graph_big; the fill pass recognises
// those rows by their length. Rows finished by k_graph_small (defer[node] == 0) are skipped.
constexpr int G_HT2 = 2048;
#ifndef FEM_GRAPH_KB
#define FEM_GRAPH_KB 4   // candidate passes whose loads k_graph issues together (1: one dependent pair per pass, A/B)
#endif
constexpr int G_KB = FEM_GRAPH_KB;

template <bool FILL>
__global__ void __launch_bounds__(256) k_graph(const int64_t* __restrict__ conn, int npe,
                                               const int32_t* __restrict__ inc_ptr, const int32_t* __restrict__ inc,
                                               int64_t N, int32_t* __restrict__ row_len,
                                               const int32_t* __restrict__ rowptr, int32_t* __restrict__ colidx,
                                               int32_t* __restrict__ diagpos, const uint8_t* __restrict__ defer,
                                               int32_t* __restrict__ far, const int32_t* __restrict__ ndefer = nullptr) {
    if (ndefer && *ndefer == 0) return;   // k_graph_small deferred no row: nothing to do here
    __shared__ int ht[G_WAVES][G_HT2];
    __shared__ int uniq[G_WAVES][G_UCAP];
    __shared__ int cnt_s[G_WAVES];
    const int wid = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // 64 candidate nodes per wave step (node = wave + nwaves * (64 c + lane): heavy rows numbered together, like
    // c3d10 corner nodes, stay spread over the waves): one look at the flags, then only this kernel's rows
    const int64_t wv = (int64_t)blockIdx.x * G_WAVES + wid, nw = (int64_t)gridDim.x * G_WAVES;
    for (int64_t c0 = 0; wv + nw * c0 < N; c0 += 64) {
      const int64_t me = wv + nw * (c0 + lane);
      bool mine = me < N && (!defer || defer[me]);
      if (FILL && mine) mine = rowptr[me + 1] - rowptr[me] <= G_UCAP;   // longer rows: k_graph_big
      unsigned long long todo = __ballot(mine);
      while (todo) {
        const int64_t node = wv + nw * (c0 + __ffsll((long long)todo) - 1);
        todo &= todo - 1;
        const int start = inc_ptr[node];
        const int C = (inc_ptr[node + 1] - start) * npe;
        const int hb = ht_bits(C, 11), HS = 1 << hb;   // >= 2 C slots, or 2048 >= G_UCAP + 64 keys
        for (int q = lane; q < HS; q += 64) ht[wid][q] = -1;
        if (lane == 0) cnt_s[wid] = 0;
        __builtin_amdgcn_wave_barrier();
        // G_KB passes of 64 candidates at a time: their incidence loads, then their connectivity loads, in flight
        // together (one dependent pair per G_KB passes instead of per pass; indices clamped into the row); the
        // inserts then run pass by pass with the G_UCAP stop checked before each, as before
        bool over = false;
        for (int t0 = 0; t0 < C && !over; t0 += 64 * G_KB) {
            int cv[G_KB];
#pragma unroll
            for (int j = 0; j < G_KB; ++j) {
                const int t = min(t0 + 64 * j + lane, C - 1);
                cv[j] = inc[start + t / npe];
            }
#pragma unroll
            for (int j = 0; j < G_KB; ++j) {
                const int t = min(t0 + 64 * j + lane, C - 1);
                cv[j] = (int)conn[(int64_t)(cv[j] / npe) * npe + (t - (t / npe) * npe)];
            }
#pragma unroll
            for (int j = 0; j < G_KB; ++j) {
                if (t0 + 64 * j >= C) break;                     // wave-uniform
                if (cnt_s[wid] > G_UCAP) {                       // wave-uniform: read after the barrier below
                    over = true;
                    break;
                }
                const int t = t0 + 64 * j + lane;
                if (t < C) {
                    const int v = cv[j];
                    if (!FILL && far && (v - node > 32767 || node - v > 32767) && !*far) atomicOr(far, 1);
                    unsigned h = ((unsigned)v * 2654435761u) >> (32 - hb);
                    while (true) {
                        const int old = atomicCAS(&ht[wid][h], -1, v);
                        if (old == -1) {
                            atomicAdd(&cnt_s[wid], 1);
                            break;
                        }
                        if (old == v) break;
                        h = (h + 1) & (HS - 1);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (cnt_s[wid] > G_UCAP) {
            if (!FILL && lane == 0) row_len[node] = -1;
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        int U = 0;
        for (int q0 = 0; q0 < HS; q0 += 64) {
            const int v = ht[wid][q0 + lane];
            const bool has = v >= 0;
            const unsigned long long m = __ballot(has);
            if (FILL && has) uniq[wid][U + __popcll(m & lt_mask)] = v;
            U += __popcll(m);
        }
        if (!FILL) {
            if (lane == 0) row_len[node] = U;
        } else {
            __builtin_amdgcn_wave_barrier();
            const int32_t rp = rowptr[node];
            for (int j = lane; j < U; j += 64) {
                const int v = uniq[wid][j];
                int rank = 0;
                for (int u = 0; u < U; ++u) rank += (uniq[wid][u] < v);
                colidx[rp + rank] = v;
                if (v == (int)node) diagpos[node] = rp + rank;
            }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
}

// Rows of more than G_UCAP neighbours (no limit; a node shared by thousands of elements): a 1024-thread workgroup
// per row marks the row's candidates in a bitmap of node ids held in LDS (GB_WORDS words: a window of 2^20 ids;
// ids past the window in further passes over the candidates), then reads the set bits back in ascending order --
// sorted and deduplicated at once, O(C) per window with C the row's candidate count (the former ascending selection
// was O(U C): a 1.1M-tet fan did not finish in 3 minutes). Pass 0 finds the candidates' id range (and the 16-bit
// delta check). The workgroups find their rows 1024 flags at a time.
constexpr int GB_T = 1024;
constexpr int GB_WORDS = 32768;                    // 128 KB of LDS: 2^20 node ids per window
constexpr size_t GB_LDS = sizeof(uint32_t) * GB_WORDS;

__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}

__device__ __forceinline__ int big_cand(const int64_t* conn, int npe, const int32_t* inc, int start, int t) {
    const int k = t / npe, b = t - k * npe;
    return (int)conn[(int64_t)(inc[start + k] / npe) * npe + b];
}

// exclusive scan of one int per thread over GB_T threads (wave scans by shuffles, then the 16 wave totals)
__device__ __forceinline__ int gb_scan(int v, int* wsum, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int before = 0, all = 0;
    for (int w = 0; w < GB_T / 64; ++w) {
        const int x = wsum[w];
        before += (w < wid) ? x : 0;
        all += x;
    }
    *total = all;
    __syncthreads();   // wsum reusable
    return before + incl - v;
}

// The ascending distinct values of get(0 .. C-1) (non-negative ints), written through put(rank, value); returns
// their count. Bitmap windows of GB_WORDS * 32 ids over [min, max] in LDS (bm), one pass over the values per
// window. Whole-workgroup call (GB_T threads, uniform arguments); *lo / *hi receive the value range.
template <bool PUT, class Get, class Put>
__device__ int gb_sorted_unique(Get get, int C, Put put, uint32_t* bm, int* wsum, int* lo_s, int* hi_s, int* lo_out,
                                int* hi_out) {
    const int tid = threadIdx.x;
    int lo = INT_MAX, hi = -1;
    for (int t = tid; t < C; t += GB_T) {
        const int v = get(t);
        lo = min(lo, v);
        hi = max(hi, v);
    }
    lo = wave_min_i32(lo);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hi = max(hi, __shfl_xor(hi, o));
    if (tid == 0) {
        *lo_s = INT_MAX;
        *hi_s = -1;
    }
    __syncthreads();
    if ((tid & 63) == 0) {
        atomicMin(lo_s, lo);
        atomicMax(hi_s, hi);
    }
    __syncthreads();
    lo = *lo_s;
    hi = *hi_s;
    *lo_out = lo;
    *hi_out = hi;
    int U = 0;
    for (int64_t w0 = lo; w0 <= hi; w0 += (int64_t)GB_WORDS * 32) {
        const int64_t span = min<int64_t>((int64_t)hi - w0 + 1, (int64_t)GB_WORDS * 32);
        const int nw = (int)((span + 31) >> 5);
        for (int k = tid; k < nw; k += GB_T) bm[k] = 0u;
        __syncthreads();
        for (int t = tid; t < C; t += GB_T) {
            const int64_t d = (int64_t)get(t) - w0;
            if (d >= 0 && d < span) atomicOr(&bm[d >> 5], 1u << (d & 31));
        }
        __syncthreads();
        // thread tid owns words [k0, k1): count, scan, then write its values in ascending order
        const int per = (nw + GB_T - 1) / GB_T;
        const int k0 = min(tid * per, nw), k1 = min(k0 + per, nw);
        int cnt = 0;
        for (int k = k0; k < k1; ++k) cnt += __popc(bm[k]);
        int total;
        const int off = gb_scan(cnt, wsum, &total);
        if (PUT) {
            int o = U + off;
            for (int k = k0; k < k1; ++k) {
                uint32_t m = bm[k];
                while (m) {
                    const int bit = __ffs(m) - 1;
                    m &= m - 1;
                    put(o++, (int)(w0 + 32 * (int64_t)k + bit));
                }
            }
        }
        U += total;
        __syncthreads();   // bitmap reusable
    }
    return U;
}

// the rows / nodes of [base, base + GB_T) with `big(i)`, gathered into rows_s (any order; each is independent)
template <class Big>
__device__ int gb_collect(int64_t base, int64_t N, Big big, int* rows_s, int* nrows_s) {
    if (threadIdx.x == 0) *nrows_s = 0;
    __syncthreads();
    const int64_t me = base + threadIdx.x;
    if (me < N && big(me)) rows_s[atomicAdd(nrows_s, 1)] = (int)threadIdx.x;
    __syncthreads();
    return *nrows_s;
}

template <bool FILL>
__global__ void __launch_bounds__(GB_T) k_graph_big(const int64_t* __restrict__ conn, int npe,
                                                    const int32_t* __restrict__ inc_ptr,
                                                    const int32_t* __restrict__ inc, int64_t N,
                                                    int32_t* __restrict__ row_len, const int32_t* __restrict__ rowptr,
                                                    int32_t* __restrict__ colidx, int32_t* __restrict__ diagpos,
                                                    int32_t* __restrict__ far,
                                                    const int32_t* __restrict__ ndefer = nullptr) {
    if (ndefer && *ndefer == 0) return;   // only k_graph_small's deferred rows can be this long
    extern __shared__ uint32_t bm[];               // [GB_WORDS]
    __shared__ int rows_s[GB_T];
    __shared__ int nrows_s, lo_s, hi_s;
    __shared__ int wsum[GB_T / 64];
    for (int64_t base = (int64_t)blockIdx.x * GB_T; base < N; base += (int64_t)gridDim.x * GB_T) {
        const int nr = gb_collect(base, N, [&](int64_t i) {
            return FILL ? rowptr[i + 1] - rowptr[i] > G_UCAP : row_len[i] < 0;
        }, rows_s, &nrows_s);
        for (int q = 0; q < nr; ++q) {
            const int64_t node = base + rows_s[q];
            const int start = inc_ptr[node];
            const int C = (inc_ptr[node + 1] - start) * npe;
            const int32_t rp = FILL ? rowptr[node] : 0;
            int lo, hi;
            const int U = gb_sorted_unique<FILL>(
                [&](int t) { return big_cand(conn, npe, inc, start, t); }, C,
                [&](int o, int v) {
                    colidx[rp + o] = v;
                    if (v == (int)node) diagpos[node] = rp + o;
                },
                bm, wsum, &lo_s, &hi_s, &lo, &hi);
            if (!FILL && threadIdx.x == 0) {
                row_len[node] = U;
                if (far && hi >= lo && (hi - (int)node > 32767 || (int)node - lo > 32767) && !*far) atomicOr(far, 1);
            }
        }
    }
}

// node segments of the incidence longer than INC_BIG (hub nodes; k_inc_l2 leaves them in arrival order in scratch):
// ascending into inc by the bitmap sort (slots are distinct)
__global__ void __launch_bounds__(GB_T) k_inc_big(const int32_t* __restrict__ inc_ptr, int64_t N,
                                                  const int32_t* __restrict__ scratch, int32_t* __restrict__ inc,
                                                  const int32_t* __restrict__ hub) {
    if (*hub == 0) return;   // k_inc_l2 met no hub segment
    extern __shared__ uint32_t bm[];
    __shared__ int rows_s[GB_T];
    __shared__ int nrows_s, lo_s, hi_s;
    __shared__ int wsum[GB_T / 64];
    for (int64_t base = (int64_t)blockIdx.x * GB_T; base < N; base += (int64_t)gridDim.x * GB_T) {
        const int nr = gb_collect(base, N, [&](int64_t i) { return inc_ptr[i + 1] - inc_ptr[i] > INC_BIG; }, rows_s,
                                  &nrows_s);
        for (int q = 0; q < nr; ++q) {
            const int64_t node = base + rows_s[q];
            const int a = inc_ptr[node], C = inc_ptr[node + 1] - a;
            int lo, hi;
            gb_sorted_unique<true>([&](int t) { return scratch[a + t]; }, C,
                                   [&](int o, int v) { inc[a + o] = v; }, bm, wsum, &lo_s, &hi_s, &lo, &hi);
        }
    }
}

// ---------------------------------------------------------------- SELL-64
// wave per slice, lane = row (coalesced row pointers, one shuffle reduction) -- a thread per slice walked its 64 rows
// one dependent load at a time on 1 / 64 of the threads
__global__ void __launch_bounds__(256) k_sell_widths(const int32_t* __restrict__ rowptr, int64_t nrows,
                                                     int64_t nslices, int64_t* __restrict__ width) {
    const int lane = threadIdx.x & 63;
    for (int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; s < nslices;
         s += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int64_t r = s * 64 + lane;
        int w = r < nrows ? rowptr[r + 1] - rowptr[r] : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) w = max(w, __shfl_xor(w, o, 64));
        if (lane == 0) width[s] = (int64_t)w * 64;
    }
}

// Wave per slice. Pass 1, lane = row: cols of column slot k, one contiguous 256-byte store per k (the CSR reads
// are strided but the slice's CSR segment is a few KB, cache-resident after the first touch). Pass 2, lane = CSR
// position of the slice's contiguous segment: csr2sell written contiguously, the row of a position found by a
// binary search over the slice's 65 row starts in LDS.
__global__ void __launch_bounds__(256) k_sell_fill(const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ colidx, int64_t nrows, int64_t nslices,
                                                   const int64_t* __restrict__ slice_ptr, int32_t* __restrict__ cols,
                                                   int64_t* __restrict__ csr2sell) {
    __shared__ int32_t rp_s[4][65];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int64_t s = (int64_t)blockIdx.x * 4 + wid; s < nslices; s += (int64_t)gridDim.x * 4) {
        const int64_t r = s * 64 + lane;
        const int64_t e0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - e0) >> 6);
        const int64_t rlast = min(s * 64 + 64, nrows);
        rp_s[wid][lane] = rowptr[min(r, rlast)];
        if (lane == 0) rp_s[wid][64] = rowptr[rlast];
        __builtin_amdgcn_wave_barrier();
        int len = 0, rp = 0;
        if (r < nrows) {
            rp = rp_s[wid][lane];
            len = rp_s[wid][lane + 1] - rp;
        }
        const int pad = (r < nrows) ? (int)r : (int)(nrows - 1);   // near the row: 16-bit deltas stay small
        for (int k = 0; k < w; ++k) cols[e0 + (int64_t)k * 64 + lane] = (k < len) ? colidx[rp + k] : pad;
        // csr2sell row-wise: the row's lane stores its run (the wave's runs tile the slice's CSR segment)
        for (int k = 0; k < len; ++k) csr2sell[rp + k] = e0 + (int64_t)k * 64 + lane;
        __builtin_amdgcn_wave_barrier();
    }
}

// The SELL-64 pattern straight from the graph kernels' rows, one wave per slice (fem_graph_fill2 + fem_sell_fill +
// fem_sell_delta16 in one pass). Lane = row: column slot k of the 64 rows is one contiguous store of cols and of the
// 16-bit deltas; a row comes from k_graph_small's tmp (32 slots per node) or, for the rows it deferred, from colidx
// (already filled by k_graph / k_graph_big). Lane = CSR position of the slice's contiguous segment: csr2sell, and
// colidx of the tmp rows, written contiguously (the row of a position by binary search over the slice's row starts).
// pout != null (fem_graph_sell_fill_sl): the bs = 1 solver layout of the slice too (sl_pattern_slice: lane-paired
// deltas, slice-uniform lists, the persistent schedule's gather windows) from the deltas this wave just wrote -- the
// separate k_sell_sl_pattern pass and its re-read of every delta from memory folded in.
__global__ void __launch_bounds__(256) k_sell_fill_graph(const int32_t* __restrict__ rowptr,
                                                         const int32_t* __restrict__ tmp,
                                                         const uint8_t* __restrict__ defer, int64_t nrows,
                                                         int64_t nslices, const int64_t* __restrict__ slice_ptr,
                                                         int32_t* __restrict__ colidx, int32_t* __restrict__ diagpos,
                                                         int32_t* __restrict__ cols, int16_t* __restrict__ dcols,
                                                         int64_t* __restrict__ csr2sell, int32_t* __restrict__ overflow,
                                                         int16_t* __restrict__ pout = nullptr,
                                                         int16_t* __restrict__ ucol = nullptr,
                                                         int32_t* __restrict__ uoff = nullptr, int G = 0,
                                                         int* __restrict__ win = nullptr,
                                                         int2* __restrict__ span = nullptr) {
    __shared__ int32_t rp_s[4][65];
    __shared__ int cand_all[4][SU_MAXW];
    constexpr int TS = G_TCAP + 1;   // padded row stride: lane = row reads hit distinct banks
    __shared__ int32_t row_s[4][64 * TS];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int32_t* rows = row_s[wid];
    for (int64_t s = (int64_t)blockIdx.x * 4 + wid; s < nslices; s += (int64_t)gridDim.x * 4) {
        const int64_t r = s * 64 + lane;
        const int64_t e0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - e0) >> 6);
        const int64_t rlast = min(s * 64 + 64, nrows);
        rp_s[wid][lane] = rowptr[min(r, rlast)];
        if (lane == 0) rp_s[wid][64] = rowptr[rlast];
        // the slice's 64 graph rows (contiguous in tmp: 64 x 32 slots) staged in LDS with 16-byte coalesced loads,
        // instead of lanes reading their rows 128 bytes apart -- twice (SELL columns, then CSR colidx)
        {
            const int4* src4 = reinterpret_cast<const int4*>(tmp + s * 64 * G_TCAP);
            const int nr = (int)(rlast - s * 64);
#pragma unroll
            for (int u = 0; u < G_TCAP / 4; ++u) {
                const int q = u * 64 + lane;          // int4 index: row q / 8, slots 4 (q % 8) ..
                const int rr = q >> 3, k = (q & 7) * 4;
                if (rr < nr) {
                    const int4 v = src4[q];
                    rows[rr * TS + k] = v.x;
                    rows[rr * TS + k + 1] = v.y;
                    rows[rr * TS + k + 2] = v.z;
                    rows[rr * TS + k + 3] = v.w;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int len = 0, rp = 0;
        bool dfr = true;
        if (r < nrows) {
            rp = rp_s[wid][lane];
            len = rp_s[wid][lane + 1] - rp;
            dfr = defer[r] != 0;
        }
        const int pad = (r < nrows) ? (int)r : (int)(nrows - 1);   // near the row: 16-bit deltas stay small
        bool far = false;
        for (int k0 = 0; k0 < w; k0 += 8) {
            int cv[8];   // the row's next 8 columns read before any store (a deferred row's from colidx: the
                         // compiler cannot know it aliases nothing written here)
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = k0 + u;
                if (k >= len) cv[u] = pad;
                else if (dfr) cv[u] = colidx[rp + k];
                else cv[u] = rows[lane * TS + k];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = k0 + u;
                if (k >= w) break;
                const int c = cv[u];
                const int64_t e = e0 + (int64_t)k * 64 + lane;
                cols[e] = c;
                const int64_t d = (int64_t)c - r;
                const bool f = d > 32767 || d < -32767;
                far |= f;
                if (dcols) dcols[e] = f ? (int16_t)0 : (int16_t)d;
                if (k < len && c == (int)r) diagpos[r] = rp + k;
            }
        }
        if (overflow && __ballot(far) && lane == 0 && !*overflow) atomicOr(overflow, 1);
        if (pout && dcols) {   // the deltas this lane just stored, re-formed from the staged row (no memory re-read)
            const auto delta = [&](int k) -> int {
                const int c = k >= len ? pad : (dfr ? colidx[rp + k] : rows[lane * TS + k]);
                const int64_t d = (int64_t)c - r;
                return (d > 32767 || d < -32767) ? 0 : (int)d;
            };
            sl_pattern_slice(s, lane, nslices, nrows, slice_ptr, delta, pout, ucol, uoff, G, win, cand_all[wid],
                             span);
        }
#ifndef FEM_FILL_ROWWISE
#define FEM_FILL_ROWWISE 1   // 10M Poisson fill pass 242 -> 188 us (0: the binary search per entry, A/B)
#endif
        if (FEM_FILL_ROWWISE) {
            // CSR colidx (and csr2sell) row-wise: the lane of a row stores its own contiguous run (the wave's runs
            // tile one contiguous block) -- no binary search of the row per entry
            if (r < nrows) {
                if (!dfr)
                    for (int k = 0; k < len; ++k) colidx[rp + k] = rows[lane * TS + k];
                if (csr2sell)
                    for (int k = 0; k < len; ++k) csr2sell[rp + k] = e0 + (int64_t)k * 64 + lane;
            }
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        const int p0 = rp_s[wid][0], p1 = rp_s[wid][64];
        for (int p = p0 + lane; p < p1; p += 64) {
            int lo = 0, hi = 64;   // last row l with rp_s[l] <= p
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (rp_s[wid][mid] <= p) lo = mid;
                else hi = mid;
            }
            const int k = p - rp_s[wid][lo];
            if (csr2sell) csr2sell[p] = e0 + (int64_t)k * 64 + lo;
            const int64_t row = s * 64 + lo;
            if (!defer[row]) colidx[p] = rows[lo * TS + k];
        }
        __builtin_amdgcn_wave_barrier();   // the staged rows consumed before the next slice overwrites them
    }
}

// csr2sell of a SELL pattern from its row and slice pointers alone (wave per slice; the map fem_sell_fill writes)
__global__ void __launch_bounds__(256) k_sell_csr2sell(const int32_t* __restrict__ rowptr, int64_t nrows,
                                                       int64_t nslices, const int64_t* __restrict__ slice_ptr,
                                                       int64_t* __restrict__ csr2sell) {
    __shared__ int32_t rp_s[4][65];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int64_t s = (int64_t)blockIdx.x * 4 + wid; s < nslices; s += (int64_t)gridDim.x * 4) {
        const int64_t r = s * 64 + lane;
        const int64_t e0 = slice_ptr[s];
        const int64_t rlast = min(s * 64 + 64, nrows);
        rp_s[wid][lane] = rowptr[min(r, rlast)];
        if (lane == 0) rp_s[wid][64] = rowptr[rlast];
        __builtin_amdgcn_wave_barrier();
        if (r < nrows) {   // row-wise: the row's lane stores its run (the wave's runs tile the slice's segment)
            const int rp = rp_s[wid][lane], len = rp_s[wid][lane + 1] - rp;
            for (int k = 0; k < len; ++k) csr2sell[rp + k] = e0 + (int64_t)k * 64 + lane;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// 16-bit column deltas (col - row) of the SELL pattern; *overflow = 1 if any |delta| > 32767 (keep int32 then)
__global__ void k_sell_delta16(const int32_t* __restrict__ cols, int64_t nslices, const int64_t* __restrict__ slice_ptr,
                               int16_t* __restrict__ dcols, int32_t* __restrict__ overflow) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nslices * 64; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = r >> 6;
        const int64_t e0 = slice_ptr[s] + (r & 63);
        const int w = (int)((slice_ptr[s + 1] - slice_ptr[s]) >> 6);
        bool far = false;
        for (int k = 0; k < w; ++k) {
            const int64_t e = e0 + (int64_t)k * 64;
            const int64_t d = (int64_t)cols[e] - r;
            const bool f = d > 32767 || d < -32767;
            far |= f;
            dcols[e] = f ? (int16_t)0 : (int16_t)d;
        }
        // one flag write per row at most (a numbering with many far columns, c3d10 mid-edge nodes after the
        // corners, made one atomic per entry cost milliseconds)
        if (far && !*overflow) atomicOr(overflow, 1);
    }
}

}  // namespace fem

using namespace fem;

extern "C" {

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static size_t inc_sort_temp_bytes(int64_t total, int bits) {
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const int32_t*)nullptr, (int32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (int)total, 0, bits);
    return tb;
}

static int node_bits(int64_t N) {   // bits of the keys 0..N (N = an out-of-range slot)
    int bits = 1;
    while (((int64_t)1 << bits) <= N) ++bits;
    return bits;
}

static int64_t inb_work_bytes(int64_t total, int64_t N) {
    const int64_t nb = (N + ((int64_t)1 << inb_shift(N)) - 1) >> inb_shift(N);
    const int64_t ncnt = nb * INB_G1;
    return (int64_t)(3 * align256(sizeof(int32_t) * total) + 2 * align256(sizeof(int32_t) * (ncnt + 1)) +
                     align256(sizeof(int32_t) * fem_scan_work_len(ncnt)));
}

int64_t fem_incidence_work_bytes(int64_t total, int64_t N) {
    if (total <= 0 || N <= 0) return 0;
    const int64_t radix = (int64_t)(3 * align256(sizeof(int32_t) * total) +
                                    align256(inc_sort_temp_bytes(total, node_bits(N))));
    const int64_t bucket = inb_work_bytes(total, N);
    return radix > bucket ? radix : bucket;
}

static int big_grid(int64_t N) {
    int64_t g = cdiv(N, (int64_t)GB_T);
    if (g > 1024) g = 1024;
    return (int)(g < 1 ? 1 : g);
}

// the big-row kernels take 128 KB of dynamic LDS (set once per process)
static int big_lds_attr() {
    static const int rc = [] {
        if (hipFuncSetAttribute((const void*)k_graph_big<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)GB_LDS) != hipSuccess ||
            hipFuncSetAttribute((const void*)k_graph_big<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)GB_LDS) != hipSuccess ||
            hipFuncSetAttribute((const void*)k_inc_big, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)GB_LDS) != hipSuccess)
            return (int)FEM_EHIP;
        return (int)FEM_OK;
    }();
    if (rc != FEM_OK) set_error("k_graph_big: cannot allow %zu bytes of dynamic LDS", GB_LDS);
    return rc;
}

static int incidence_bucket(const int64_t* conn, int64_t total, int64_t N, int32_t* inc_ptr, int32_t* inc,
                            char* base, int32_t* bad, fem_stream_t stream) {
    hipStream_t st = S(stream);
    const int bsh = inb_shift(N);
    const int nb = (int)((N + ((int64_t)1 << bsh) - 1) >> bsh);
    const int64_t ncnt = (int64_t)nb * INB_G1;
    const size_t a4 = align256(sizeof(int32_t) * total), ac = align256(sizeof(int32_t) * (ncnt + 1));
    int2* kpair = reinterpret_cast<int2*>(base);   // (node, slot) pairs: the first two int32 arrays' space
    int32_t* scratch = reinterpret_cast<int32_t*>(base + 2 * a4);
    int32_t* cnt = reinterpret_cast<int32_t*>(base + 3 * a4);
    int32_t* off = reinterpret_cast<int32_t*>(base + 3 * a4 + ac);
    int32_t* swork = reinterpret_cast<int32_t*>(base + 3 * a4 + 2 * ac);
    const size_t l1 = sizeof(int) * (size_t)nb;
    hipLaunchKernelGGL(k_inc_l1<false>, dim3(INB_G1), dim3(INB_T1), l1, st, conn, total, N, bsh, nb, cnt,
                       (const int32_t*)nullptr, (int2*)nullptr, bad);
    FEM_LAUNCHED();
    int rc = fem_scan_i32(cnt, ncnt, off, swork, stream);
    if (rc != FEM_OK) return rc;
    hipLaunchKernelGGL(k_inc_l1<true>, dim3(INB_G1), dim3(INB_T1), l1, st, conn, total, N, bsh, nb, (int32_t*)nullptr,
                       off, kpair, (int32_t*)nullptr);
    FEM_LAUNCHED();
    const int B = 1 << bsh;
    const size_t l2 = sizeof(int) * (size_t)(2 * B + 1 + 2 * INB_CAP) + 2 * (size_t)INB_CAP;
    hipLaunchKernelGGL(k_inc_l2, dim3((unsigned)nb), dim3(256), l2, st, kpair, off, INB_G1, N, bsh, scratch,
                       inc_ptr, inc, cnt + ncnt);
    FEM_LAUNCHED();
    if (total > INC_BIG) {   // hub segments (the launch finds them; for ordinary meshes it only reads inc_ptr)
        if (const int brc = big_lds_attr()) return brc;
        hipLaunchKernelGGL(k_inc_big, dim3(big_grid(N)), dim3(GB_T), GB_LDS, st, inc_ptr, N, scratch, inc,
                           (const int32_t*)(cnt + ncnt));
        FEM_LAUNCHED();
    }
    return FEM_OK;
}

int fem_incidence_checked(const int64_t* conn, int64_t M, int npe, int64_t N, int32_t* inc_ptr, int32_t* inc,
                          int32_t* work, int32_t* bad, fem_stream_t stream) {
    hipStream_t st = S(stream);
    const int64_t total = M * npe;
    if (total >= (int64_t)1 << 31 || N >= (int64_t)1 << 31) {
        set_error("fem_incidence: M*npe = %lld / N = %lld exceed int32 range", (long long)total, (long long)N);
        return FEM_EARG;
    }
    if (bad) FEM_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t), st));
    if (N <= 0) return FEM_OK;
    if (total == 0) {
        FEM_HIP(hipMemsetAsync(inc_ptr, 0, sizeof(int32_t) * (N + 1), st));
        return FEM_OK;
    }
    const int bits = node_bits(N);
    const size_t a4 = align256(sizeof(int32_t) * total);
    const size_t tb = inc_sort_temp_bytes(total, bits);
    char* base = reinterpret_cast<char*>(work);
    const bool own = base == nullptr;   // no caller workspace: stream-ordered allocation
    if (own) FEM_HIP(::fem::malloc_async((void**)&base, (size_t)fem_incidence_work_bytes(total, N), st));
    if (getenv("FEM355_INC_RADIX") == nullptr && inb_shift(N) <= INB_MAXSH) {
        const int rc = incidence_bucket(conn, total, N, inc_ptr, inc, base, bad, stream);
        if (own) FEM_HIP(hipFreeAsync(base, st));
        return rc;
    }
    int32_t* kin = reinterpret_cast<int32_t*>(base);
    int32_t* kout = reinterpret_cast<int32_t*>(base + a4);
    int32_t* vin = reinterpret_cast<int32_t*>(base + 2 * a4);
    void* tmp = base + 3 * a4;
    hipLaunchKernelGGL(k_inc_keys, dim3(stream_grid(total, 256)), dim3(256), 0, st, conn, total, N, kin, vin, bad);
    FEM_LAUNCHED();
    size_t tb2 = tb;
    FEM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb2, kin, kout, vin, inc, (int)total, 0, bits, st));
    hipLaunchKernelGGL(k_inc_ptr, dim3(stream_grid(total + 1, 256)), dim3(256), 0, st, kout, total, N, inc_ptr);
    FEM_LAUNCHED();
    if (own) FEM_HIP(hipFreeAsync(base, st));
    return FEM_OK;
}

int fem_incidence(const int64_t* conn, int64_t M, int npe, int64_t N, int32_t* inc_ptr, int32_t* inc,
                  int32_t* work, fem_stream_t stream) {
    return fem_incidence_checked(conn, M, npe, N, inc_ptr, inc, work, nullptr, stream);
}

static int graph_grid(int64_t N) {
    int64_t g = cdiv(N, G_WAVES);
    if (g > 4096) g = 4096;
    return (int)(g < 1 ? 1 : g);
}

// count: k_graph for every row (done = null) or for the rows k_graph_small left, then k_graph_big for the rows
// k_graph flagged; row_len ends exact for every node. *overflow (zeroed by the caller's entry point): 1 if some
// row has a neighbour farther than 32767 rows (the SELL pattern then keeps int32 columns).
static int graph_count(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                       int32_t* row_len, const uint8_t* defer, int32_t* overflow, hipStream_t st) {
    const int32_t* nd = defer ? reinterpret_cast<const int32_t*>(defer) + (N + 3) / 4 : nullptr;
    hipLaunchKernelGGL(k_graph<false>, dim3(graph_grid(N)), dim3(256), 0, st, conn, npe, inc_ptr, inc, N, row_len,
                       (const int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr, defer, overflow, nd);
    FEM_LAUNCHED();
    if (const int rc = big_lds_attr()) return rc;
    hipLaunchKernelGGL(k_graph_big<false>, dim3(big_grid(N)), dim3(GB_T), GB_LDS, st, conn, npe, inc_ptr, inc, N, row_len,
                       (const int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr, overflow, nd);
    FEM_LAUNCHED();
    return FEM_OK;
}

static int graph_fill(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                      const int32_t* rowptr, int32_t* colidx, int32_t* diagpos, const uint8_t* defer, hipStream_t st) {
    const int32_t* nd = defer ? reinterpret_cast<const int32_t*>(defer) + (N + 3) / 4 : nullptr;
    hipLaunchKernelGGL(k_graph<true>, dim3(graph_grid(N)), dim3(256), 0, st, conn, npe, inc_ptr, inc, N,
                       (int32_t*)nullptr, rowptr, colidx, diagpos, defer, (int32_t*)nullptr, nd);
    FEM_LAUNCHED();
    if (const int rc = big_lds_attr()) return rc;
    hipLaunchKernelGGL(k_graph_big<true>, dim3(big_grid(N)), dim3(GB_T), GB_LDS, st, conn, npe, inc_ptr, inc, N,
                       (int32_t*)nullptr, rowptr, colidx, diagpos, (int32_t*)nullptr, nd);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_graph_count(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                    int32_t* row_len, int32_t* overflow, fem_stream_t stream) {
    if (overflow) FEM_HIP(hipMemsetAsync(overflow, 0, sizeof(int32_t), S(stream)));
    if (N <= 0) return FEM_OK;
    return graph_count(conn, npe, inc_ptr, inc, N, row_len, nullptr, overflow, S(stream));
}

// tmp: [N * G_TCAP] rows of k_graph_small, then N bytes of deferral flags (rows left to k_graph / k_graph_big), then
// the number of deferred rows
int64_t fem_graph_tmp_len(int64_t N) { return N * G_TCAP + (N + 3) / 4 + 1; }
static uint8_t* defer_flags(int32_t* tmp, int64_t N) { return reinterpret_cast<uint8_t*>(tmp + N * G_TCAP); }
static const uint8_t* defer_flags(const int32_t* tmp, int64_t N) {
    return reinterpret_cast<const uint8_t*>(tmp + N * G_TCAP);
}

int fem_graph_count2(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                     int32_t* row_len, int32_t* tmp, int32_t* overflow, fem_stream_t stream) {
    if (overflow) FEM_HIP(hipMemsetAsync(overflow, 0, sizeof(int32_t), S(stream)));
    if (N <= 0) return FEM_OK;
    const int64_t grid = std::min<int64_t>(cdiv(N, G_WAVES), 16384);
    FEM_HIP(hipMemsetAsync(tmp + N * G_TCAP + (N + 3) / 4, 0, sizeof(int32_t), S(stream)));   // deferred rows
    const bool al16 = (reinterpret_cast<uintptr_t>(conn) & 15) == 0;
#define GS_LAUNCH(NPE_)                                                                                           \
    hipLaunchKernelGGL((k_graph_small<FEM_GRAPH_LPN, NPE_>), dim3((unsigned)grid), dim3(256), 0, S(stream), conn, \
                       npe, inc_ptr, inc, N, row_len, tmp, defer_flags(tmp, N), overflow)
    if (al16 && npe == 4 && getenv("FEM355_GRAPH_SLOTS") == nullptr) GS_LAUNCH(4);
    else if (al16 && npe == 6) GS_LAUNCH(6);
    else if (al16 && npe == 8) GS_LAUNCH(8);
    else if (al16 && npe == 10) GS_LAUNCH(10);
    else GS_LAUNCH(0);
#undef GS_LAUNCH
    FEM_LAUNCHED();
    return graph_count(conn, npe, inc_ptr, inc, N, row_len, defer_flags(tmp, N), overflow, S(stream));
}

int fem_graph_fill2(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                    const int32_t* rowptr, const int32_t* tmp, int32_t* colidx, int32_t* diagpos,
                    fem_stream_t stream) {
    if (N <= 0) return FEM_OK;
    // a node no element touches has no diagonal: -1 (fem_jacobi then gives w = 0, like the reference's 1/0 -> inf
    // -> 0, `solver/solver.py:828-831`)
    FEM_HIP(hipMemsetAsync(diagpos, 0xff, sizeof(int32_t) * (size_t)N, S(stream)));
    hipLaunchKernelGGL(k_graph_copy, dim3(stream_grid(N * G_TCAP, 256)), dim3(256), 0, S(stream), tmp,
                       defer_flags(tmp, N), rowptr, N, colidx, diagpos);
    FEM_LAUNCHED();
    return graph_fill(conn, npe, inc_ptr, inc, N, rowptr, colidx, diagpos, defer_flags(tmp, N), S(stream));
}

int fem_graph_sell_fill(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                        const int32_t* rowptr, const int32_t* tmp, const int64_t* slice_ptr, int32_t* colidx,
                        int32_t* diagpos, int32_t* cols, int16_t* dcols, int64_t* csr2sell, int32_t* overflow,
                        fem_stream_t stream) {
    if (N <= 0) return FEM_OK;
    hipStream_t st = S(stream);
    FEM_HIP(hipMemsetAsync(diagpos, 0xff, sizeof(int32_t) * (size_t)N, st));   // -1: no diagonal
    if (overflow) FEM_HIP(hipMemsetAsync(overflow, 0, sizeof(int32_t), st));
    // rows k_graph_small deferred: straight into colidx / diagpos (k_graph, k_graph_big), before the slice pass
    const int rc = graph_fill(conn, npe, inc_ptr, inc, N, rowptr, colidx, diagpos, defer_flags(tmp, N), st);
    if (rc != FEM_OK) return rc;
    const int64_t ns = cdiv(N, 64);
    hipLaunchKernelGGL(k_sell_fill_graph, dim3((unsigned)std::min<int64_t>(cdiv(ns, 4), 16384)), dim3(256), 0, st,
                       rowptr, tmp, defer_flags(tmp, N), N, ns, slice_ptr, colidx, diagpos, cols, dcols, csr2sell,
                       overflow);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_graph_sell_fill_sl(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                           const int32_t* rowptr, const int32_t* tmp, const int64_t* slice_ptr, int32_t* colidx,
                           int32_t* diagpos, int32_t* cols, int16_t* dcols, int G, int16_t* pcols, int16_t* ucol,
                           int32_t* uoff, int32_t* win, fem_stream_t stream) {
    if (N <= 0) return FEM_OK;
    if (!dcols || !pcols || !ucol || !uoff || (G > 0 && !win)) {
        set_error("fem_graph_sell_fill_sl: the 16-bit deltas and the solver-layout arrays are required");
        return FEM_EARG;
    }
    hipStream_t st = S(stream);
    FEM_HIP(hipMemsetAsync(diagpos, 0xff, sizeof(int32_t) * (size_t)N, st));   // -1: no diagonal
    const int rc = graph_fill(conn, npe, inc_ptr, inc, N, rowptr, colidx, diagpos, defer_flags(tmp, N), st);
    if (rc != FEM_OK) return rc;
    const int64_t ns = cdiv(N, 64);
    // per-slice owner spans (stream-ordered scratch), reduced into the G windows after the fill pass
    int2* span = nullptr;
    if (G > 0) FEM_HIP(::fem::stream_scratch((void**)&span, sizeof(int2) * (size_t)ns, st));
    hipLaunchKernelGGL(k_sell_fill_graph, dim3((unsigned)std::min<int64_t>(cdiv(ns, 4), 16384)), dim3(256), 0, st,
                       rowptr, tmp, defer_flags(tmp, N), N, ns, slice_ptr, colidx, diagpos, cols, dcols,
                       (int64_t*)nullptr, (int32_t*)nullptr, pcols, ucol, uoff, G, win, span);
    FEM_LAUNCHED();
    if (G > 0) {
        hipLaunchKernelGGL(k_win_from_spans, dim3((unsigned)cdiv((int64_t)G * 64, 256)), dim3(256), 0, st, G, ns,
                           (const int2*)span, win);
        FEM_LAUNCHED();
    }
    return FEM_OK;
}

int fem_graph_fill(const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N,
                   const int32_t* rowptr, int32_t* colidx, int32_t* diagpos, fem_stream_t stream) {
    if (N <= 0) return FEM_OK;
    FEM_HIP(hipMemsetAsync(diagpos, 0xff, sizeof(int32_t) * (size_t)N, S(stream)));   // -1: no diagonal
    return graph_fill(conn, npe, inc_ptr, inc, N, rowptr, colidx, diagpos, nullptr, S(stream));
}

int fem_sell_delta16(const int32_t* cols, int64_t nrows, const int64_t* slice_ptr, int16_t* dcols, int32_t* overflow,
                     fem_stream_t stream) {
    int64_t ns = cdiv(nrows, 64);
    hipLaunchKernelGGL(k_sell_delta16, dim3(stream_grid(ns * 64, 256)), dim3(256), 0, S(stream), cols, ns, slice_ptr,
                       dcols, overflow);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_sell_csr2sell(const int32_t* rowptr, int64_t nrows, const int64_t* slice_ptr, int64_t* csr2sell,
                      fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    hipLaunchKernelGGL(k_sell_csr2sell, dim3((unsigned)std::min<int64_t>(cdiv(ns, 4), 16384)), dim3(256), 0,
                       S(stream), rowptr, nrows, ns, slice_ptr, csr2sell);
    FEM_LAUNCHED();
    return FEM_OK;
}

// the pattern's sizes in one launch (one block): {nnz = rowptr[N], entries = slice_ptr[ns], *bad, *ovf, widest slice}
// (1024 threads, eight width loads in flight per thread: the 256-thread loop of one dependent load per step took
// 28 us at 10M -- on the critical path, right before the build's one read-back)
constexpr int GS_T = 1024;
__global__ void __launch_bounds__(GS_T) k_graph_sizes(const int32_t* __restrict__ rowptr,
                                                      const int64_t* __restrict__ slice_ptr,
                                                      const int64_t* __restrict__ width, int64_t N, int64_t ns,
                                                      const int32_t* __restrict__ bad, const int32_t* __restrict__ ovf,
                                                      int64_t* __restrict__ out) {
    __shared__ int64_t m_s[GS_T / 64];
    int64_t m = 0;
    constexpr int U = 8;
    int64_t s = threadIdx.x;
    for (; s + (U - 1) * GS_T < ns; s += U * GS_T) {
        int64_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = width[s + u * GS_T];
#pragma unroll
        for (int u = 0; u < U; ++u) m = v[u] > m ? v[u] : m;
    }
    for (; s < ns; s += GS_T) m = width[s] > m ? width[s] : m;
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t v = __shfl_xor(m, o, 64);
        m = v > m ? v : m;
    }
    if ((threadIdx.x & 63) == 0) m_s[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t w = m_s[0];
        for (int i = 1; i < GS_T / 64; ++i) w = m_s[i] > w ? m_s[i] : w;
        out[0] = rowptr[N];
        out[1] = slice_ptr[ns];
        out[2] = bad ? *bad : 0;
        out[3] = ovf ? *ovf : 0;
        out[4] = w;
    }
}

int fem_graph_sizes(const int32_t* rowptr, const int64_t* slice_ptr, const int64_t* width, int64_t N,
                    const int32_t* bad, const int32_t* ovf, int64_t* out5, fem_stream_t stream) {
    if (N < 0 || !rowptr || !slice_ptr || !out5 || (N > 0 && !width)) {
        set_error("fem_graph_sizes: rowptr, slice_ptr, out5 (and width for N > 0) are required");
        return FEM_EARG;
    }
    hipLaunchKernelGGL(k_graph_sizes, dim3(1), dim3(GS_T), 0, S(stream), rowptr, slice_ptr, width, N, cdiv(N, 64),
                       bad, ovf, out5);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_sell_widths(const int32_t* rowptr, int64_t nrows, int64_t* width, fem_stream_t stream) {
    int64_t ns = cdiv(nrows, 64);
    hipLaunchKernelGGL(k_sell_widths, dim3(stream_grid(ns * 64, 256)), dim3(256), 0, S(stream), rowptr, nrows, ns,
                       width);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_sell_fill(const int32_t* rowptr, const int32_t* colidx, int64_t nrows, const int64_t* slice_ptr,
                  int32_t* cols, int64_t* csr2sell, fem_stream_t stream) {
    int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    hipLaunchKernelGGL(k_sell_fill, dim3((unsigned)std::min<int64_t>(cdiv(ns, 4), 16384)), dim3(256), 0, S(stream),
                       rowptr, colidx, nrows, ns, slice_ptr, cols, csr2sell);
    FEM_LAUNCHED();
    return FEM_OK;
}

}  // extern "C"
