// f110_opponent.hip — the training opponent's policy on the device.
//
// gap_follow_action (rl_training/utils/gap_follow.py:3-58) is what
// train_ddpg.py:168 runs on the host every step, on the float32
// info["scans"][1] of the previous step.  Here one wave computes it for one
// scan, bit-exact with the reference's NumPy float32 arithmetic:
//
//   preprocess_lidar :3-12  p[i] = mean(clip(r[s..e], 0, 3)) over the 5-wide
//                           window clipped to the scan; NumPy's float32 mean of
//                           <= 5 elements is a left-to-right float32 sum divided
//                           by the count (IEEE round-to-nearest, __fdiv_rn)
//   create_bubble    :14-19 first argmin (a NaN wins), zero p[cp-30 .. cp+30]
//   find_max_gap     :21-39 runs of p > 0.5; first run of maximal end-start
//   best point / action :41-58
//
// Each wave keeps one LDS row (the preprocessed scan) and synchronises only
// itself.  The 1080 beams are split into 64 contiguous lane chunks.  The run search is
// a two-pass chunked scan: each lane finds the last run start in its chunk, a
// wave-wide exclusive prefix max hands every lane the start of the run that
// enters its chunk, and each lane then measures the runs that end inside it.
#include <hip/hip_runtime.h>

#include "f110_internal.h"

namespace f110 {

namespace {

constexpr int kGfWaves = 1;  // scans per block (one-wave blocks)

struct MinAt {
    float v;
    int32_t i;
};

__device__ __forceinline__ int32_t shfl_xor_i(int32_t v, int m) { return __shfl_xor(v, m, 64); }

// LDS hand-off between the lanes of ONE wave (each wave owns its scan: no
// workgroup barrier)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ float shfl_xor_f(float v, int m) { return __shfl_xor(v, m, 64); }

}  // namespace

__global__ void __launch_bounds__(64 * kGfWaves) k_gap_follow(GapFollowArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int B = a.B;
    float *p = reinterpret_cast<float *>(smem) + (size_t)wave * B;  // one LDS row per wave (scan)
    const int64_t m = (int64_t)blockIdx.x * kGfWaves + wave;
    const bool live = m < a.M;  // wave-uniform
    const float *scan = a.scans + (live ? m : 0) * a.scan_stride;

    // preprocess_lidar (:3-12), the window read straight from the scan (L1 hits)
    if (live)
        for (int i = lane; i < B; i += 64) {
            const int s = i - 2 > 0 ? i - 2 : 0;
            const int e = i + 2 < B - 1 ? i + 2 : B - 1;
            float sum = 0.0f;
            for (int j = s; j <= e; ++j) {
                float v = scan[j];
                v = v < 0.0f ? 0.0f : v;  // np.clip(x, 0, 3.0); NaN passes through
                v = v > 3.0f ? 3.0f : v;
                sum = sum + v;
            }
            p[i] = __fdiv_rn(sum, (float)(e - s + 1));
        }
    wave_lds_sync();

    const int C = (B + 63) / 64;  // chunk per lane
    const int c0 = lane * C;
    const int c1 = c0 + C < B ? c0 + C : B;
    // create_bubble (:14-19): np.argmin -> first NaN if any, else first minimum
    int32_t nan_i = INT32_MAX;
    MinAt mn{INFINITY, INT32_MAX};
    if (live)
        for (int i = c0; i < c1; ++i) {
            const float v = p[i];
            if (v != v) {
                if (i < nan_i) nan_i = i;
            } else if (mn.i == INT32_MAX || v < mn.v) {  // strict: the first minimum of the chunk
                mn = MinAt{v, i};
            }
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        nan_i = min(nan_i, shfl_xor_i(nan_i, o));
        const float ov = shfl_xor_f(mn.v, o);
        const int32_t oi = shfl_xor_i(mn.i, o);
        if (oi != INT32_MAX && (mn.i == INT32_MAX || ov < mn.v || (ov == mn.v && oi < mn.i))) mn = MinAt{ov, oi};
    }
    const int cp = nan_i != INT32_MAX ? nan_i : (mn.i != INT32_MAX ? mn.i : 0);
    const int bs = cp - 30 > 0 ? cp - 30 : 0;
    const int be = cp + 30 < B - 1 ? cp + 30 : B - 1;
    wave_lds_sync();
    if (live)
        for (int i = lane; i < B; i += 64)
            if (i >= bs && i <= be) p[i] = 0.0f;
    wave_lds_sync();

    // find_max_gap (:21-39)
    auto mask = [&](int i) { return i >= 0 && i < B && p[i] > 0.5f; };
    int32_t last_start = -1;
    if (live)
        for (int i = c0; i < c1; ++i)
            if (mask(i) && !mask(i - 1)) last_start = i;
    // exclusive prefix max of last_start over lanes
    int32_t incl = last_start;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t up = __shfl_up(incl, o, 64);
        if (lane >= o) incl = max(incl, up);
    }
    int32_t cur = __shfl_up(incl, 1, 64);
    if (lane == 0) cur = -1;
    int32_t best_len = -1, best_start = INT32_MAX;
    if (live)
        for (int i = c0; i < c1; ++i) {
            const bool mi = mask(i);
            if (mi && !mask(i - 1)) cur = i;
            if (mi && !mask(i + 1)) {
                const int32_t len = i - cur;
                if (len > best_len) {
                    best_len = len;
                    best_start = cur;
                }
            }
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int32_t ol = shfl_xor_i(best_len, o);
        const int32_t os = shfl_xor_i(best_start, o);
        if (ol > best_len || (ol == best_len && os < best_start)) {
            best_len = ol;
            best_start = os;
        }
    }
    if (live && lane == 0) {
        int32_t g0 = 0, g1 = B - 1;  // no gap: the whole scan (:36-37)
        if (best_len >= 0) {
            g0 = best_start;
            g1 = best_start + best_len;
        }
        const int32_t best = (g0 + g1) / 2;                                  // :41-42
        const double steer = a.angle_min + (double)best * a.angle_increment;  // :47
        const double s = fabs(steer);
        const double speed = s < 10.0 * (kPi / 180.0) ? 2.5 : (s < 20.0 * (kPi / 180.0) ? 2.0 : 1.5);  // :49-54
        float *act = a.actions + m * a.action_stride;
        act[0] = (float)steer;  // train_ddpg.py:168 .astype(np.float32)
        act[1] = (float)speed;
        if (a.gaps) {
            a.gaps[2 * m] = g0;
            a.gaps[2 * m + 1] = g1;
        }
    }
}

// The same policy with the chunk passes in registers (B <= 64 * kGfMaxC):
// the scan is staged in LDS once (coalesced), lane l computes the window
// means of its beams [l*C, (l+1)*C), C = ceil(B/64), into registers, and the
// bubble / run passes work on those and a per-lane bit mask (runs of
// p > 0.5), the neighbours' edge bits coming by shuffle.  One wave per
// scan, no workgroup barrier; same arithmetic and tie rules as k_gap_follow.
constexpr int kGfMaxC = 17;

__global__ void __launch_bounds__(64) k_gap_follow_reg(GapFollowArgs a) {
    __shared__ float r[64 * kGfMaxC];  // the scan, then the window means
    __shared__ float pm[64 * kGfMaxC];
    const int lane = threadIdx.x;
    const int B = a.B;
    const int64_t m = blockIdx.x;
    const float *gscan = a.scans + m * a.scan_stride;
    for (int i = lane; i < B; i += 64) r[i] = gscan[i];
    wave_lds_sync();
    // preprocess_lidar (:3-12) in the coalesced layout
    for (int i = lane; i < B; i += 64) {
        const int s = i - 2 > 0 ? i - 2 : 0;
        const int e = i + 2 < B - 1 ? i + 2 : B - 1;
        float sum = 0.0f;
        for (int q = s; q <= e; ++q) {
            float v = r[q];
            v = v < 0.0f ? 0.0f : v;  // np.clip(x, 0, 3.0); NaN passes through
            v = v > 3.0f ? 3.0f : v;
            sum = sum + v;
        }
        pm[i] = __fdiv_rn(sum, (float)(e - s + 1));
    }
    wave_lds_sync();
    const int C = (B + 63) / 64;
    const int c0 = lane * C;
    const int c1 = c0 + C < B ? c0 + C : B;
    const int n = c1 > c0 ? c1 - c0 : 0;  // beams of this lane
    // this lane's chunk into registers (stride C across lanes, C odd for
    // B = 1080: no bank conflicts)
    float p[kGfMaxC];
#pragma unroll
    for (int j = 0; j < kGfMaxC; ++j) p[j] = j < n ? pm[c0 + j] : 0.0f;
    // create_bubble (:14-19): np.argmin -> first NaN if any, else first minimum
    int32_t nan_i = INT32_MAX;
    MinAt mn{INFINITY, INT32_MAX};
#pragma unroll
    for (int j = 0; j < kGfMaxC; ++j)
        if (j < n) {
            const float v = p[j];
            if (v != v) {
                if (c0 + j < nan_i) nan_i = c0 + j;
            } else if (mn.i == INT32_MAX || v < mn.v) {
                mn = MinAt{v, c0 + j};
            }
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        nan_i = min(nan_i, shfl_xor_i(nan_i, o));
        const float ov = shfl_xor_f(mn.v, o);
        const int32_t oi = shfl_xor_i(mn.i, o);
        if (oi != INT32_MAX && (mn.i == INT32_MAX || ov < mn.v || (ov == mn.v && oi < mn.i))) mn = MinAt{ov, oi};
    }
    const int cp = nan_i != INT32_MAX ? nan_i : (mn.i != INT32_MAX ? mn.i : 0);
    const int bs = cp - 30 > 0 ? cp - 30 : 0;
    const int be = cp + 30 < B - 1 ? cp + 30 : B - 1;
    // runs of p > 0.5 after the bubble: bit j = beam c0 + j
    uint32_t mk = 0;
#pragma unroll
    for (int j = 0; j < kGfMaxC; ++j) {
        const int i = c0 + j;
        const bool bubble = i >= bs && i <= be;
        if (j < n && !bubble && p[j] > 0.5f) mk |= 1u << j;
    }
    // mask(c0 - 1): the previous lane's last beam; mask(c1): the next lane's first
    const uint32_t prev_mk = __shfl_up(mk, 1, 64), prev_n = (uint32_t)__shfl_up(n, 1, 64);
    const bool before = lane > 0 && prev_n > 0 && ((prev_mk >> (prev_n - 1)) & 1u);
    const uint32_t next_mk = __shfl_down(mk, 1, 64);
    const bool after = lane < 63 && (next_mk & 1u);
    // find_max_gap (:21-39): the last run start in this lane's chunk
    int32_t last_start = -1;
#pragma unroll
    for (int j = 0; j < kGfMaxC; ++j) {
        const bool mi = (mk >> j) & 1u;
        const bool mp = j == 0 ? before : ((mk >> (j - 1)) & 1u);
        if (j < n && mi && !mp) last_start = c0 + j;
    }
    int32_t incl = last_start;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t up = __shfl_up(incl, o, 64);
        if (lane >= o) incl = max(incl, up);
    }
    int32_t cur = __shfl_up(incl, 1, 64);
    if (lane == 0) cur = -1;
    int32_t best_len = -1, best_start = INT32_MAX;
#pragma unroll
    for (int j = 0; j < kGfMaxC; ++j) {
        if (j < n) {
            const bool mi = (mk >> j) & 1u;
            const bool mp = j == 0 ? before : ((mk >> (j - 1)) & 1u);
            const bool mx = j == n - 1 ? after : ((mk >> (j + 1)) & 1u);
            if (mi && !mp) cur = c0 + j;
            if (mi && !mx) {
                const int32_t len = c0 + j - cur;
                if (len > best_len) {
                    best_len = len;
                    best_start = cur;
                }
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int32_t ol = shfl_xor_i(best_len, o);
        const int32_t os = shfl_xor_i(best_start, o);
        if (ol > best_len || (ol == best_len && os < best_start)) {
            best_len = ol;
            best_start = os;
        }
    }
    if (lane == 0) {
        int32_t g0 = 0, g1 = B - 1;  // no gap: the whole scan (:36-37)
        if (best_len >= 0) {
            g0 = best_start;
            g1 = best_start + best_len;
        }
        const int32_t best = (g0 + g1) / 2;                                  // :41-42
        const double steer = a.angle_min + (double)best * a.angle_increment;  // :47
        const double sa = fabs(steer);
        const double speed = sa < 10.0 * (kPi / 180.0) ? 2.5 : (sa < 20.0 * (kPi / 180.0) ? 2.0 : 1.5);  // :49-54
        float *act = a.actions + m * a.action_stride;
        act[0] = (float)steer;  // train_ddpg.py:168 .astype(np.float32)
        act[1] = (float)speed;
        if (a.gaps) {
            a.gaps[2 * m] = g0;
            a.gaps[2 * m + 1] = g1;
        }
    }
}

size_t gap_follow_lds_bytes(int B) { return sizeof(float) * (size_t)B * kGfWaves; }

hipError_t launch_gap_follow(const GapFollowArgs &a, hipStream_t s) {
    if (a.M <= 0) return hipSuccess;
    const size_t lds = gap_follow_lds_bytes(a.B);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_gap_follow),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    if (a.B <= 64 * kGfMaxC) {  // register-resident scan
        hipLaunchKernelGGL(k_gap_follow_reg, dim3((unsigned)a.M), dim3(64), 0, s, a);
        return hipGetLastError();
    }
    const dim3 grid((unsigned)((a.M + kGfWaves - 1) / kGfWaves));
    hipLaunchKernelGGL(k_gap_follow, grid, dim3(64 * kGfWaves), lds, s, a);
    return hipGetLastError();
}

}  // namespace f110
