// Gather microbenchmark (GPU box): what one 64-lane gather of 8-byte (or
// 4-byte) cells costs the vector memory pipeline, by how many distinct
// 128-byte lines its lanes touch, and by table size (L2-resident vs beyond
// L2).  It decides whether a tiled EDT layout (fewer distinct lines per
// k_rays_fxs gather) can lower the texture-address cost per wave-level load
// (DESIGN §3.12).
//
//   hipcc -O3 --offload-arch=gfx950 scripts/gather_mb.hip -o bin/gather_mb && bin/gather_mb
//
// Every wave runs ITERS iterations of U independent gathers (the loads of one
// iteration are all in flight at once); a lane's address is
//   line(l) = base + (l % K) * 97 lines,  word(l) = (l / K) % (128 / cell bytes)
// with base a per-(wave, iteration, u) hash over the table, so K = 1 puts all 64
// lanes in one line and K = 64 gives 64 lines.  Prints one JSON line per case:
// ns per kernel, wave-level loads, and cycles per wave-level load per CU at the
// measured clock (cycles = ns * GHz, the clock from hipDeviceProp / the box).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr int U = 8;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <class T>
__global__ void __launch_bounds__(64) k_gather(const T *tab, uint32_t lines, int K, int iters, T *sink) {
    const uint32_t lane = threadIdx.x;
    constexpr uint32_t per_line = 128 / sizeof(T);
    const uint32_t word = (lane / (uint32_t)K) % per_line;
    const uint32_t spread = (lane % (uint32_t)K) * 97u;
    T acc = 0;
    for (int it = 0; it < iters; ++it) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t base = hash32((blockIdx.x * 131071u) ^ (uint32_t)(it * U + u) * 2654435761u);
            const uint32_t line = (base + spread) % lines;
            v[u] = tab[(size_t)line * per_line + word];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc == (T)-1) sink[blockIdx.x] = acc;  // never true: keeps the loads
}

// the ray kernel's arm load: lane l reads the 16-byte (cos, sin) entry at base + l * 1.3865 (consecutive
// beams' theta indices), 64 lanes over ~90 entries
__global__ void __launch_bounds__(64) k_arm16(const double2 *tab, uint32_t n, int iters, double *sink) {
    const uint32_t lane = threadIdx.x;
    double acc = 0;
    for (int it = 0; it < iters; ++it) {
        double2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t base = hash32((blockIdx.x * 131071u) ^ (uint32_t)(it * U + u) * 2654435761u) % (n - 100);
            v[u] = tab[base + (lane * 13865u) / 10000u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y;
    }
    if (acc == -1.0) sink[blockIdx.x] = acc;
}

// ended rays (k_rays_fxs): every active lane reads one common line (the quad rule's floor: one
// cycle per 4-lane group), a fixed random set of lanes "ended"; ZERO = 1: ended lanes load one
// fixed other line (the kernel's zero cell), 0: their load is masked off (exec).  Addresses are
// a uniform offset plus a per-lane constant (no per-load VALU hashing).
template <int ZERO>
__global__ void __launch_bounds__(64) k_ended(const double *tab, uint32_t lines, int iters, int keep_pct,
                                              double *sink) {
    const uint32_t lane = threadIdx.x;
    const bool act = hash32(lane * 0x9E3779B9u + 7u) % 100u < (uint32_t)keep_pct;
    const uint32_t word = lane & 15u;
    double acc = 0;
    for (int it = 0; it < iters; ++it) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t line = 1u + (uint32_t)(it * U + u) % (lines - 1u);  // uniform (line 0: the zero cell)
            const uint32_t idx = line * 16u + word;
            if (ZERO) {
                v[u] = tab[act ? idx : 0u];
            } else {
                v[u] = 0.0;
                if (act) v[u] = tab[idx];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc == -1.0) sink[blockIdx.x] = acc;
}

template <int ZERO>
static void run_ended(int keep_pct, int blocks, int iters) {
    const size_t bytes = (size_t)64 << 10;  // L1 / L2 resident: the address path is the limit
    double *tab, *sink;
    CHECK(hipMalloc(&tab, bytes));
    CHECK(hipMemset(tab, 0, bytes));
    CHECK(hipMalloc(&sink, (size_t)blocks * sizeof(double)));
    const uint32_t lines = (uint32_t)(bytes / 128);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) k_ended<ZERO><<<blocks, 64>>>(tab, lines, iters, keep_pct, sink);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(a));
        k_ended<ZERO><<<blocks, 64>>>(tab, lines, iters, keep_pct, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double loads = (double)blocks * iters * U;
    printf("{\"cell\": \"ended_%s\", \"active_pct\": %d, \"ms\": %.4f, \"wave_loads\": %.0f, "
           "\"cyc_per_load_per_cu_2p4ghz\": %.2f}\n", ZERO ? "zero_line" : "masked", keep_pct, best, loads,
           best * 1e6 * 2.4 / (loads / 256.0));
    fflush(stdout);
    CHECK(hipFree(tab));
    CHECK(hipFree(sink));
}

template <class T>
static void run(const char *name, size_t bytes, int K, int blocks, int iters) {
    T *tab, *sink;
    CHECK(hipMalloc(&tab, bytes));
    CHECK(hipMemset(tab, 0, bytes));
    CHECK(hipMalloc(&sink, (size_t)blocks * sizeof(T)));
    const uint32_t lines = (uint32_t)(bytes / 128);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) k_gather<T><<<blocks, 64>>>(tab, lines, K, iters, sink);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(a));
        k_gather<T><<<blocks, 64>>>(tab, lines, K, iters, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double loads = (double)blocks * iters * U;
    const double ns = best * 1e6;
    // cycles per wave-level load per CU at 2.4 GHz (the ray kernel's measured clock)
    printf("{\"cell\": \"%s\", \"table_mb\": %.1f, \"lines_per_load\": %d, \"ms\": %.4f, \"wave_loads\": %.0f, "
           "\"cyc_per_load_per_cu_2p4ghz\": %.2f}\n",
           name, bytes / 1048576.0, K, best, loads, ns * 2.4 / (loads / 256.0));
    fflush(stdout);
    CHECK(hipFree(tab));
    CHECK(hipFree(sink));
}

static void run_arm(int blocks, int iters) {
    const uint32_t n = 2000;
    double2 *tab;
    double *sink;
    CHECK(hipMalloc(&tab, n * sizeof(double2)));
    CHECK(hipMemset(tab, 0, n * sizeof(double2)));
    CHECK(hipMalloc(&sink, (size_t)blocks * sizeof(double)));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) k_arm16<<<blocks, 64>>>(tab, n, iters, sink);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(a));
        k_arm16<<<blocks, 64>>>(tab, n, iters, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double loads = (double)blocks * iters * U;
    printf("{\"cell\": \"arm16_consecutive\", \"table_kb\": 32, \"ms\": %.4f, \"wave_loads\": %.0f, "
           "\"cyc_per_load_per_cu_2p4ghz\": %.2f}\n", best, loads, best * 1e6 * 2.4 / (loads / 256.0));
    fflush(stdout);
    CHECK(hipFree(tab));
    CHECK(hipFree(sink));
}

int main() {
    if (getenv("GMB_ENDED_ONLY")) {
        const int pcts[5] = {100, 75, 50, 25, 10};
        for (int p : pcts) {
            run_ended<1>(p, 256 * 16, 256);
            run_ended<0>(p, 256 * 16, 256);
        }
        return 0;
    }
    run_arm(256 * 16, 256);
    if (getenv("GMB_ARM_ONLY")) return 0;
    const int blocks = 256 * 16, iters = 256;
    const size_t sizes[2] = {(size_t)2 << 20, (size_t)48 << 20};
    const int Ks[8] = {1, 2, 4, 8, 12, 16, 32, 64};
    for (size_t s : sizes)
        for (int K : Ks) {
            run<double>("f64", s, K, blocks, iters);
            run<float>("f32", s, K, blocks, iters);
        }
    return 0;
}
