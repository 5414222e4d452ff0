// Error plumbing, version, and device-wide exclusive scans (pattern build / SELL slice offsets).
#include <stdarg.h>

#include <atomic>
#include <mutex>
#include <vector>

#include "common.hpp"

namespace fem {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// Stream-ordered scratch comes from a private memory pool per device (never the device's default pool, whose
// attributes other libraries in the process share). The pool keeps at most FEM_POOL_KEEP bytes (256 MB) of freed
// memory across synchronisations -- enough for the small per-call scratch whose reuse the pattern-build latency
// work relies on; larger stream-ordered frees (graph build temporaries, CSR export buffers: GBs at 10M DOFs) go back
// to the driver at the next synchronisation instead of staying reserved (torch's caching allocator can then reuse
// them). fem_release_scratch() trims the pool to zero.
constexpr uint64_t FEM_POOL_KEEP = 256ull << 20;
static std::mutex g_pool_mu;
static hipMemPool_t g_pool[64] = {};

static hipMemPool_t scratch_pool(int dev) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool[dev]) {
        hipMemPoolProps props;
        memset(&props, 0, sizeof(props));
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        hipMemPool_t pool = nullptr;
        if (hipMemPoolCreate(&pool, &props) != hipSuccess) return nullptr;
        uint64_t keep = FEM_POOL_KEEP;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        g_pool[dev] = pool;
    }
    return g_pool[dev];
}

hipError_t malloc_async(void** p, size_t bytes, hipStream_t st) {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
        hipMemPool_t pool = scratch_pool(dev);
        if (pool) return hipMallocFromPoolAsync(p, bytes, pool, st);
    }
    return hipMallocAsync(p, bytes, st);
}

struct ScratchEntry {
    hipStream_t st;
    int dev;
    void* ptr;
    size_t bytes;
};
static std::mutex g_scratch_mu;
static std::vector<ScratchEntry> g_scratch;

// per-stream scratch kept between calls (host cost of a hipFreeAsync per call: it waits for the kernel, ~200 us).
// Stream-ordered users only, and never under stream capture: a captured graph would record the pointer, which a
// later larger request reallocates (the call refuses a capturing stream with hipErrorStreamCaptureUnsupported).
hipError_t stream_scratch(void** p, size_t bytes, hipStream_t st) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
        return hipErrorStreamCaptureUnsupported;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (ScratchEntry& e : g_scratch) {
        if (e.st != st || e.dev != dev) continue;
        if (e.bytes >= bytes) {
            *p = e.ptr;
            return hipSuccess;
        }
        (void)hipFreeAsync(e.ptr, st);   // stream-ordered: earlier work on st that used it runs first
        e.ptr = nullptr;
        e.bytes = 0;
        const hipError_t rc = malloc_async(&e.ptr, bytes, st);
        if (rc != hipSuccess) return rc;
        e.bytes = bytes;
        *p = e.ptr;
        return hipSuccess;
    }
    // a process that keeps creating streams: at most 8 kept buffers, the oldest released. hipFree (device-wide
    // synchronisation), not hipFreeAsync: the evicted entry's stream may no longer exist, and a free ordered on this
    // stream would not wait for that stream's work. Only a ninth stream's first call pays it.
    if (g_scratch.size() >= 8) {
        if (g_scratch.front().ptr) (void)hipFree(g_scratch.front().ptr);
        g_scratch.erase(g_scratch.begin());
    }
    ScratchEntry e{st, dev, nullptr, bytes};
    const hipError_t rc = malloc_async(&e.ptr, bytes, st);
    if (rc != hipSuccess) return rc;
    g_scratch.push_back(e);
    *p = e.ptr;
    return hipSuccess;
}

// every kept per-stream buffer freed (after a device synchronisation) and the scratch pools trimmed to zero
int release_scratch() {
    {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        if (!g_scratch.empty()) FEM_HIP(hipDeviceSynchronize());
        for (ScratchEntry& e : g_scratch)
            if (e.ptr) (void)hipFree(e.ptr);
        g_scratch.clear();
    }
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (int d = 0; d < 64; ++d)
        if (g_pool[d]) (void)hipMemPoolTrimTo(g_pool[d], 0);
    return FEM_OK;
}

// ---------------------------------------------------------------- 3-phase exclusive scan
// phase 1: per-tile sums; phase 2: one block scans the tile sums; phase 3: tile-local scan + offset.
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* lds, T* total) {
    // wave scans by shuffles, then the four wave totals through LDS: two barriers (the Hillis-Steele form over 256
    // threads in LDS took sixteen, and the three scan kernels of the 10M pattern build ~90 us)
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    T off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < SCAN_BLOCK / 64; ++w) {
        const T t = lds[w];
        off += w < wid ? t : T(0);
        tot += t;
    }
    *total = tot;
    __syncthreads();   // lds is reused by the caller's next scan
    return off + x - v;
}

template <typename T>
__global__ void __launch_bounds__(SCAN_BLOCK) k_tile_sums(const T* __restrict__ in, int64_t n, T* __restrict__ sums) {
    __shared__ T lds[SCAN_BLOCK];
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    T s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        int64_t i = base + (int64_t)k * SCAN_BLOCK + threadIdx.x;
        if (i < n) s += in[i];
    }
    T tot;
    block_exclusive_scan<T>(s, lds, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <typename T>
__global__ void __launch_bounds__(SCAN_BLOCK) k_scan_sums(T* __restrict__ sums, int64_t ntiles) {
    __shared__ T lds[SCAN_BLOCK];
    T carry = 0;
    for (int64_t base = 0; base < ntiles; base += SCAN_BLOCK) {
        int64_t i = base + threadIdx.x;
        T v = (i < ntiles) ? sums[i] : T(0);
        T tot;
        T ex = block_exclusive_scan<T>(v, lds, &tot);
        if (i < ntiles) sums[i] = ex + carry;
        carry += tot;
    }
    if (threadIdx.x == 0) sums[ntiles] = carry;
}

template <typename T>
__global__ void __launch_bounds__(SCAN_BLOCK) k_tile_scan(const T* __restrict__ in, int64_t n, const T* __restrict__ sums,
                                                          T* __restrict__ out, int64_t ntiles) {
    __shared__ T lds[SCAN_BLOCK];
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
    T v[SCAN_ITEMS];
    T s = 0;
    // a thread's eight consecutive items as 16-byte vector accesses where aligned and whole (int32: two per thread
    // instead of eight 4-byte accesses 32 bytes apart across the wave)
    constexpr bool VEC = sizeof(T) == 4;
    const bool vec = VEC && base + SCAN_ITEMS <= n && ((reinterpret_cast<uintptr_t>(in + base) |
                                                        reinterpret_cast<uintptr_t>(out + base)) & 15) == 0;
    if (vec) {
        const int4* p4 = reinterpret_cast<const int4*>(in + base);
#pragma unroll
        for (int h = 0; h < SCAN_ITEMS / 4; ++h) {
            const int4 q = p4[h];
            v[4 * h] = (T)q.x;
            v[4 * h + 1] = (T)q.y;
            v[4 * h + 2] = (T)q.z;
            v[4 * h + 3] = (T)q.w;
        }
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) s += v[k];
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) {
            int64_t i = base + k;
            v[k] = (i < n) ? in[i] : T(0);
            s += v[k];
        }
    }
    T tot;
    T ex = block_exclusive_scan<T>(s, lds, &tot) + sums[blockIdx.x];
    if (vec) {
        int o[SCAN_ITEMS];
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) {
            o[k] = (int)ex;
            ex += v[k];
        }
        int4* q4 = reinterpret_cast<int4*>(out + base);
#pragma unroll
        for (int h = 0; h < SCAN_ITEMS / 4; ++h) q4[h] = make_int4(o[4 * h], o[4 * h + 1], o[4 * h + 2], o[4 * h + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) {
            int64_t i = base + k;
            if (i < n) out[i] = ex;
            ex += v[k];
        }
    }
    if (blockIdx.x == ntiles - 1 && threadIdx.x == 0) out[n] = sums[ntiles];
}

template <typename T>
int scan_impl(const T* in, int64_t n, T* out, T* work, hipStream_t st) {
    if (n <= 0) {
        FEM_HIP(hipMemsetAsync(out, 0, sizeof(T), st));
        return FEM_OK;
    }
    int64_t ntiles = cdiv(n, SCAN_TILE);
    hipLaunchKernelGGL(k_tile_sums<T>, dim3((unsigned)ntiles), dim3(SCAN_BLOCK), 0, st, in, n, work);
    FEM_LAUNCHED();
    hipLaunchKernelGGL(k_scan_sums<T>, dim3(1), dim3(SCAN_BLOCK), 0, st, work, ntiles);
    FEM_LAUNCHED();
    hipLaunchKernelGGL(k_tile_scan<T>, dim3((unsigned)ntiles), dim3(SCAN_BLOCK), 0, st, in, n, work, out, ntiles);
    FEM_LAUNCHED();
    return FEM_OK;
}

}  // namespace fem

using namespace fem;

extern "C" {

const char* fem_last_error(void) { return g_err; }
int fem_version(void) { return 100; }

int fem_release_scratch(void) { return release_scratch(); }

int64_t fem_scan_work_len(int64_t n) { return cdiv(n > 0 ? n : 1, SCAN_TILE) + 1; }

int fem_scan_i32(const int32_t* in, int64_t n, int32_t* out, int32_t* work, fem_stream_t stream) {
    return scan_impl<int32_t>(in, n, out, work, S(stream));
}

int fem_scan_i64(const int64_t* in, int64_t n, int64_t* out, int64_t* work, fem_stream_t stream) {
    return scan_impl<int64_t>(in, n, out, work, S(stream));
}

}  // extern "C"
