// f110_ddpg.hip — the DDPG networks' output layers fused with what follows
// them (include/f110.h, "learner heads").
//
// agent.py's Actor ends in fc3 (128 -> act_dim), tanh and the affine map to
// the action box (:56-61); its Critic in q (128 -> 1) (:93-97); replay()
// turns q into the TD target (:302-308), the weighted MSE (:310-316) and the
// actor loss -mean(q) (:321-326).  In torch each of these is a skinny GEMM
// (N = 1 or 2, where the BLAS picks 16-40 us kernels) followed by 3-10
// elementwise launches.  Here each is one row-parallel kernel: a half-wave
// owns one row of h (16-B coalesced loads, a 32-lane sum), W and b are
// uniform loads, and the epilogue runs in registers.  The backward passes write dh
// per row and reduce dW / db over the rows deterministically: per-block
// partial sums in a fixed order, then one pass over the partials.
//
// Arithmetic is fp32 like the reference's; the dot products accumulate in
// fma order over k (the BLAS order differs, so results agree with torch to
// fp32 rounding, not bit for bit).  The elementwise epilogues keep torch's
// expression order (-ffp-contract=off keeps mul and add separate there).
#include <hip/hip_runtime.h>

#include <string>
#include <type_traits>

#include "f110_internal.h"

int f110_set_error(int code, const std::string &msg);  // f110_capi.cpp

namespace f110 {
namespace {

constexpr int kHB = 256;      // threads per block
constexpr int kRowLanes = 32; // lanes per row (a half-wave): 4 columns each (K <= 128 in one pass)
constexpr int kRowsPerBlock = kHB / kRowLanes;
constexpr int kWRows = 64;    // rows per block of the weight-gradient pass
constexpr int kMaxOut = 4;    // head outputs (act_dim <= 4)
constexpr int kMaxK = 255;    // hidden width (the weight pass keeps >= 3 row lanes of column quads)

enum HeadMode { kActor = 0, kTarget = 1, kLoss = 2, kMean = 3, kExplore = 4 };

struct HeadArgs {
    const float *h, *W, *b;
    const float *ht, *Wt, *bt;  // k_critic_step: the target critic's last hidden layer and head
    const float *aux0, *aux1;  // actor: scale, shift; target: r, d; loss: y, w
    const float *t, *dout, *g;  // backward: tanh output, upstream grad [B][nout], loss grad (device scalar)
    float *out0, *out1;         // actor: a, t; target: y; loss: td
    float *dh, *dW, *db;
    const float *dh_mask;       // backward: dh := dh_mask > 0 ? dh : 0 (the ReLU of h), or null
    float *dz;                  // scratch [B][nout]
    float *part;                // scratch [nblk][nout][K + 1] or [nblk] (loss partials)
    float *loss;
    float gamma, sign;
    int32_t B, K, nout, nblk;
    // kExplore: out0[row * out_stride + j] = clamp(act + sigma N(0,1), lo[j], hi[j]); (sigma, call) from
    // nstate_in, the decayed pair to nstate_out (block 0, thread 0)
    const float *lo, *hi;
    const double *nstate_in;
    double *nstate_out;
    double decay, sigma_min;
    int64_t out_stride;
    uint64_t seed;
};

// choose_action's exploration noise (agent.py:350-370, GaussianActionNoise
// :520-539, np.random.normal(0, sigma)): N(0,1) pairs by Box-Muller on one
// Philox2x32-10 block per (call, row, output pair), counter (step, row pair
// index), key from the seed; f32 log / sqrt / sincospi on 24-bit uniforms
// (u1 in (0, 1]).  Independent across rows, outputs and calls.
__device__ __forceinline__ float2 explore_normals(uint64_t seed, uint64_t step, int64_t row, int pair) {
    const uint32_t key = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x85EBCA6Bu) ^ ((uint32_t)(step >> 32) * 0xC2B2AE35u);
    const U2 r = philox2x32((uint32_t)step, (uint32_t)(row * 2 + pair), key);
    const float u1 = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);
    const float u2 = (float)(r.y >> 8) * (1.0f / 16777216.0f);
    const float rad = sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincospif(2.0f * u2, &sn, &cs);
    return make_float2(rad * cs, rad * sn);
}

// sum over the 32 lanes of a half-wave (fixed tree); every lane gets it
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
    for (int o = kRowLanes / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// z[j] = b[j] + sum_k h[k] W[j][k] for the row of this half-wave: lane l
// takes columns 4l..4l+3 (+128, +256 ...), then a half-wave sum
template <int NOUT>
__device__ __forceinline__ void row_dot_of(const float *h, const float *W, const float *b, int32_t K, int64_t row,
                                           int l, float (&z)[NOUT]) {
    const float *hr = h + row * K;
#pragma unroll
    for (int j = 0; j < NOUT; ++j) z[j] = 0.0f;
    for (int k = 4 * l; k < K; k += 4 * kRowLanes) {
        float x[4];
        if ((K & 3) == 0) {
            const float4 v = *reinterpret_cast<const float4 *>(hr + k);
            x[0] = v.x, x[1] = v.y, x[2] = v.z, x[3] = v.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = k + i < K ? hr[k + i] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < NOUT; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (k + i < K) z[j] = fmaf(x[i], W[(size_t)j * K + k + i], z[j]);
    }
#pragma unroll
    for (int j = 0; j < NOUT; ++j) z[j] = half_sum(z[j]) + b[j];  // addmm: bias added to the product
}

template <int NOUT>
__device__ __forceinline__ void row_dot(const HeadArgs &a, int64_t row, int l, float (&z)[NOUT]) {
    row_dot_of<NOUT>(a.h, a.W, a.b, a.K, row, l, z);
}

// dh[row] = dz W (lane l: columns 4l..4l+3, +128 ...), zero where dh_mask <= 0
template <int NOUT>
__device__ __forceinline__ void write_dh(const HeadArgs &a, int64_t row, int l, const float (&dz)[NOUT]) {
    float *o = a.dh + row * a.K;
    for (int k = 4 * l; k < a.K; k += 4 * kRowLanes) {
        float r4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float s = 0.0f;
#pragma unroll
            for (int j = 0; j < NOUT; ++j)
                if (k + i < a.K) s = fmaf(dz[j], a.W[(size_t)j * a.K + k + i], s);
            r4[i] = a.dh_mask && k + i < a.K && !(a.dh_mask[row * a.K + k + i] > 0.0f) ? 0.0f : s;
        }
        if ((a.K & 3) == 0) {
            *reinterpret_cast<float4 *>(o + k) = make_float4(r4[0], r4[1], r4[2], r4[3]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (k + i < a.K) o[k + i] = r4[i];
        }
    }
}

// deterministic block sum (fixed shuffle tree per wave, waves in order); thread 0 gets it
__device__ __forceinline__ float block_sum(float v) {
    __shared__ float ws[kHB / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    float s = 0.0f;
    if (threadIdx.x == 0)
        for (int w = 0; w < kHB / 64; ++w) s += ws[w];
    return s;
}

// forward: one row per half-wave, the epilogue on its lane 0
template <int MODE, int NOUT>
__global__ void __launch_bounds__(kHB) k_head_fwd(HeadArgs a) {
    const int l = threadIdx.x & (kRowLanes - 1);
    const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x / kRowLanes);
    float v = 0.0f;
    if (row < a.B) {  // uniform per half-wave
        float z[NOUT];
        row_dot<NOUT>(a, row, l, z);
        if (l == 0) {
            if (MODE == kActor) {  // tanh, then 0.5*(high-low) * t + 0.5*(high+low) (agent.py:60-61)
#pragma unroll
                for (int j = 0; j < NOUT; ++j) {
                    const float t = tanhf(z[j]);
                    a.out1[row * NOUT + j] = t;
                    a.out0[row * NOUT + j] = a.aux0[j] * t + a.aux1[j];
                }
            } else if (MODE == kExplore) {  // the action, + sigma N(0,1), clipped to [low, high] (NaN kept)
                const float sigma = (float)a.nstate_in[0];
                const uint64_t step = (uint64_t)a.nstate_in[1];
#pragma unroll
                for (int j = 0; j < NOUT; j += 2) {
                    const float2 nz = explore_normals(a.seed, step, row, j >> 1);
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        if (j + q >= NOUT) break;
                        const float act = a.aux0[j + q] * tanhf(z[j + q]) + a.aux1[j + q];
                        float v = act + sigma * (q == 0 ? nz.x : nz.y);
                        v = v < a.lo[j + q] ? a.lo[j + q] : v;
                        v = v > a.hi[j + q] ? a.hi[j + q] : v;
                        a.out0[row * a.out_stride + j + q] = v;
                    }
                }
            } else if (MODE == kTarget) {  // r + gamma * (1.0 - d) * q_next (agent.py:306)
                const float gd = a.gamma * (1.0f - a.aux1[row]);
                a.out0[row] = a.aux0[row] + gd * z[0];
            } else if (MODE == kLoss) {  // td = target_y - q_pred; w * td ** 2 (agent.py:314-316)
                const float td = a.aux0[row] - z[0];
                a.out0[row] = td;
                v = a.aux1[row] * (td * td);
            } else {  // kMean: q
                v = z[0];
            }
        }
    }
    if (MODE == kLoss || MODE == kMean) {
        const float s = block_sum(v);
        if (threadIdx.x == 0) a.part[blockIdx.x] = s;
    }
    if (MODE == kExplore && blockIdx.x == 0 && threadIdx.x == 0) {  // GaussianActionNoise.__call__'s decay
        const double sg = a.nstate_in[0] * a.decay;
        a.nstate_out[0] = sg > a.sigma_min ? sg : a.sigma_min;  // max(sigma * decay, sigma_min)
        a.nstate_out[1] = a.nstate_in[1] + 1.0;
    }
}

// The critic update's head in one launch (agent.py:302-319): per row (one
// half-wave) the TD target y = r + gamma (1 - d) (ht Wt^T + bt) (k_head_fwd
// kTarget), td = y - (h W^T + b) and w td^2 (kLoss: block partials for the
// loss), and its backward (k_head_bwd_rows kLoss): dq = -((g / B) w) (2 td),
// dh = dq W where dh_mask > 0.  The same float operations in the same order as
// the three separate launches.  aux0 = r, aux1 = d, aux2 (w) in `dout`.
__global__ void __launch_bounds__(kHB) k_critic_step(HeadArgs a) {
    const int l = threadIdx.x & (kRowLanes - 1);
    const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x / kRowLanes);
    float v = 0.0f;
    if (row < a.B) {
        float zt[1], z[1];
        row_dot_of<1>(a.ht, a.Wt, a.bt, a.K, row, l, zt);
        row_dot<1>(a, row, l, z);
        const float gd = a.gamma * (1.0f - a.aux1[row]);
        const float y = a.aux0[row] + gd * zt[0];
        const float td = y - z[0];
        const float w = a.dout[row];
        if (l == 0) {
            a.out0[row] = td;
            v = w * (td * td);
        }
        const float gb = *a.g / (float)a.B;
        const float dz[1] = {-((gb * w) * (2.0f * td))};
        if (a.dz && l == 0) a.dz[row] = dz[0];
        if (a.dh) write_dh<1>(a, row, l, dz);
    }
    const float s = block_sum(v);
    if (threadIdx.x == 0) a.part[blockIdx.x] = s;
}

// The actor update's loss head (agent.py:321-326): q = h W^T + b, block
// partials of q (k_head_fwd kMean) and the backward through the frozen
// critic (k_head_bwd_rows kMean): dq = sign g / B, dh = dq W where dh_mask > 0.
__global__ void __launch_bounds__(kHB) k_q_mean_step(HeadArgs a) {
    const int l = threadIdx.x & (kRowLanes - 1);
    const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x / kRowLanes);
    float v = 0.0f;
    if (row < a.B) {
        float z[1];
        row_dot<1>(a, row, l, z);
        if (l == 0) v = z[0];
        const float dz[1] = {a.sign * (*a.g / (float)a.B)};
        if (a.dh) write_dh<1>(a, row, l, dz);
    }
    const float s = block_sum(v);
    if (threadIdx.x == 0) a.part[blockIdx.x] = s;
}

// loss = sign * (sum of the block partials, in block order) / B
__global__ void __launch_bounds__(kHB) k_loss_finish(HeadArgs a) {
    float v = 0.0f;
    for (int i = threadIdx.x; i < a.nblk; i += kHB) v += a.part[i];
    const float s = block_sum(v);
    if (threadIdx.x == 0) *a.loss = a.sign * (s / (float)a.B);
}

// backward, one row per half-wave: dz (mode-specific, every lane), dh = dz W
// (lane l writes columns 4l..4l+3 ...)
template <int MODE, int NOUT>
__global__ void __launch_bounds__(kHB) k_head_bwd_rows(HeadArgs a) {
    const int l = threadIdx.x & (kRowLanes - 1);
    const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x / kRowLanes);
    if (row >= a.B) return;
    float dz[NOUT];
    if (MODE == kActor) {  // mul backward (grad * scale), then tanh_backward (grad * (1 - t*t))
#pragma unroll
        for (int j = 0; j < NOUT; ++j) {
            const float t = a.t[row * NOUT + j];
            dz[j] = (a.dout[row * NOUT + j] * a.aux0[j]) * (1.0f - t * t);
        }
    } else if (MODE == kLoss) {  // mean -> g/B; * w; pow(td, 2) -> * 2 td; sub -> neg
        const float gb = *a.g / (float)a.B;
        dz[0] = -((gb * a.aux1[row]) * (2.0f * a.out0[row]));
    } else {  // kMean: sign * g / B for every row
        dz[0] = a.sign * (*a.g / (float)a.B);
    }
    if (a.dz && l == 0) {
#pragma unroll
        for (int j = 0; j < NOUT; ++j) a.dz[row * NOUT + j] = dz[j];
    }
    if (a.dh) write_dh<NOUT>(a, row, l, dz);
}

// dW[j][c] = sum_rows dz[j] h[c], db[j] = sum_rows dz[j]: per-block partials
// over kWRows rows.  Thread t: column quad q = t % Q (columns 4q..4q+3; quad
// 0 also sums the bias), row lane t / Q; the row lanes of a quad are added
// in LDS in lane order.
template <int NOUT>
__global__ void __launch_bounds__(kHB) k_head_wgrad(HeadArgs a) {
    __shared__ float red[kHB][NOUT][5];
    const int C = a.K + 1;
    const int Q = (a.K + 3) / 4;
    const int lanes = kHB / Q;  // row lanes (>= 3: K <= 255)
    const int q = threadIdx.x % Q, rl = threadIdx.x / Q;
    const int64_t r0 = (int64_t)blockIdx.x * kWRows;
    const int64_t r1 = r0 + kWRows < a.B ? r0 + kWRows : a.B;
    float acc[NOUT][5];
#pragma unroll
    for (int j = 0; j < NOUT; ++j)
#pragma unroll
        for (int i = 0; i < 5; ++i) acc[j][i] = 0.0f;
    if (rl < lanes) {
        const int k = 4 * q;
        for (int64_t r = r0 + rl; r < r1; r += lanes) {
            float x[4];
            if ((a.K & 3) == 0) {
                const float4 v = *reinterpret_cast<const float4 *>(a.h + r * a.K + k);
                x[0] = v.x, x[1] = v.y, x[2] = v.z, x[3] = v.w;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) x[i] = k + i < a.K ? a.h[r * a.K + k + i] : 0.0f;
            }
#pragma unroll
            for (int j = 0; j < NOUT; ++j) {
                const float d = a.dz[r * NOUT + j];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[j][i] = fmaf(d, x[i], acc[j][i]);
                acc[j][4] += d;  // the bias column (used by quad 0)
            }
        }
    }
#pragma unroll
    for (int j = 0; j < NOUT; ++j)
#pragma unroll
        for (int i = 0; i < 5; ++i) red[threadIdx.x][j][i] = acc[j][i];
    __syncthreads();
    if (threadIdx.x < Q) {
        float sum[NOUT][5];
#pragma unroll
        for (int j = 0; j < NOUT; ++j)
#pragma unroll
            for (int i = 0; i < 5; ++i) sum[j][i] = red[threadIdx.x][j][i];
        for (int l2 = 1; l2 < lanes; ++l2)
#pragma unroll
            for (int j = 0; j < NOUT; ++j)
#pragma unroll
                for (int i = 0; i < 5; ++i) sum[j][i] += red[l2 * Q + threadIdx.x][j][i];
        float *p = a.part + (size_t)blockIdx.x * NOUT * C;
        const int k = 4 * threadIdx.x;
#pragma unroll
        for (int j = 0; j < NOUT; ++j) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (k + i < a.K) p[j * C + k + i] = sum[j][i];
            if (threadIdx.x == 0) p[j * C + a.K] = sum[j][4];
        }
    }
}

// the partials summed: one wave per output, lanes over the blocks (fixed
// order: lane-strided sums, then a shuffle tree)
__global__ void __launch_bounds__(kHB) k_wgrad_finish(HeadArgs a) {
    const int64_t n = (int64_t)a.nout * (a.K + 1);
    const int64_t o = (int64_t)blockIdx.x * (kHB / 64) + (threadIdx.x >> 6);
    if (o >= n) return;  // whole wave
    const int lane = threadIdx.x & 63;
    float s = 0.0f;
    for (int i = lane; i < a.nblk; i += 64) s += a.part[(size_t)i * n + o];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane != 0) return;
    const int j = (int)(o / (a.K + 1)), c = (int)(o - (int64_t)j * (a.K + 1));
    if (c < a.K) {
        if (a.dW) a.dW[(size_t)j * a.K + c] = s;
    } else if (a.db) {
        a.db[j] = s;
    }
}

// ReLU backward of a hidden layer fused with its bias gradient: gz =
// threshold_backward(gy, y, 0) (gy where y > 0, else 0) and db = sum_rows gz
// (per-block partials over kWRows rows, thread: column quad x row lane, then
// k_colsum_finish).  Replaces torch's threshold_backward + sum(0) launches.
__global__ void __launch_bounds__(kHB) k_relu_bwd(const float *gy, const float *y, float *gz, float *part, int32_t B,
                                                  int32_t K) {
    __shared__ float red[kHB][4];
    const int Q = (K + 3) / 4;
    const int lanes = kHB / Q;
    const int q = threadIdx.x % Q, rl = threadIdx.x / Q;
    const int64_t r0 = (int64_t)blockIdx.x * kWRows;
    const int64_t r1 = r0 + kWRows < B ? r0 + kWRows : B;
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (rl < lanes) {
        const int k = 4 * q;
        for (int64_t r = r0 + rl; r < r1; r += lanes) {
            float g4[4], y4[4];
            if ((K & 3) == 0) {
                const float4 gv = *reinterpret_cast<const float4 *>(gy + r * K + k);
                const float4 yv = *reinterpret_cast<const float4 *>(y + r * K + k);
                g4[0] = gv.x, g4[1] = gv.y, g4[2] = gv.z, g4[3] = gv.w;
                y4[0] = yv.x, y4[1] = yv.y, y4[2] = yv.z, y4[3] = yv.w;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    g4[i] = k + i < K ? gy[r * K + k + i] : 0.0f;
                    y4[i] = k + i < K ? y[r * K + k + i] : 0.0f;
                }
            }
            float z4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                z4[i] = y4[i] > 0.0f ? g4[i] : 0.0f;
                acc[i] += z4[i];
            }
            if ((K & 3) == 0) {
                *reinterpret_cast<float4 *>(gz + r * K + k) = make_float4(z4[0], z4[1], z4[2], z4[3]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (k + i < K) gz[r * K + k + i] = z4[i];
            }
        }
    }
    if (!part) return;  // block-uniform
#pragma unroll
    for (int i = 0; i < 4; ++i) red[threadIdx.x][i] = acc[i];
    __syncthreads();
    if (threadIdx.x < Q) {
        float sum[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) sum[i] = red[threadIdx.x][i];
        for (int l2 = 1; l2 < lanes; ++l2)
#pragma unroll
            for (int i = 0; i < 4; ++i) sum[i] += red[l2 * Q + threadIdx.x][i];
        const int k = 4 * threadIdx.x;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (k + i < K) part[(size_t)blockIdx.x * K + k + i] = sum[i];
    }
}

// out[c] = sum of the nblk partials of column c (one wave per column, fixed order)
__global__ void __launch_bounds__(kHB) k_colsum_finish(const float *part, int32_t nblk, int32_t K, float *out) {
    const int64_t c = (int64_t)blockIdx.x * (kHB / 64) + (threadIdx.x >> 6);
    if (c >= K) return;  // whole wave
    const int lane = threadIdx.x & 63;
    float s = 0.0f;
    for (int i = lane; i < nblk; i += 64) s += part[(size_t)i * K + c];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) out[c] = s;
}

template <class F>
hipError_t with_nout(int nout, F f) {
    switch (nout) {
        case 1: return f(std::integral_constant<int, 1>{});
        case 2: return f(std::integral_constant<int, 2>{});
        case 3: return f(std::integral_constant<int, 3>{});
        case 4: return f(std::integral_constant<int, 4>{});
        default: return hipErrorInvalidValue;
    }
}

unsigned row_blocks(int32_t B) { return (unsigned)((B + kRowsPerBlock - 1) / kRowsPerBlock); }

hipError_t wgrad(HeadArgs a, hipStream_t s) {
    if (!a.dW && !a.db) return hipSuccess;
    a.nblk = (a.B + kWRows - 1) / kWRows;
    hipError_t e = with_nout(a.nout, [&](auto N) {
        hipLaunchKernelGGL(k_head_wgrad<decltype(N)::value>, dim3((unsigned)a.nblk), dim3(kHB), 0, s, a);
        return hipGetLastError();
    });
    if (e != hipSuccess) return e;
    const int64_t n = (int64_t)a.nout * (a.K + 1);
    const int64_t per = kHB / 64;
    hipLaunchKernelGGL(k_wgrad_finish, dim3((unsigned)((n + per - 1) / per)), dim3(kHB), 0, s, a);
    return hipGetLastError();
}

bool bad_shape(int32_t B, int32_t K, int32_t nout) { return B <= 0 || K <= 0 || K > kMaxK || nout <= 0 || nout > kMaxOut; }

int fail_hip(const char *fn, hipError_t e) {
    return f110_set_error(F110_E_HIP, std::string(fn) + ": " + hipGetErrorString(e));
}

int fail_arg(const char *fn) { return f110_set_error(F110_E_INVALID, std::string(fn) + ": bad arguments"); }

}  // namespace
}  // namespace f110

using namespace f110;

extern "C" int64_t f110_ddpg_scratch_floats(int32_t B, int32_t K, int32_t nout) {
    if (bad_shape(B, K, nout)) return -1;
    const int64_t nblk_w = (B + kWRows - 1) / kWRows;
    const int64_t nblk_r = (B + kRowsPerBlock - 1) / kRowsPerBlock;
    const int64_t part = nblk_w * nout * (K + 1) > nblk_r ? nblk_w * nout * (K + 1) : nblk_r;
    return (int64_t)B * nout + part;
}

extern "C" int64_t f110_ddpg_relu_bwd_scratch_floats(int32_t B, int32_t K) {
    if (B <= 0 || K <= 0 || K > 4 * kHB) return -1;
    return (int64_t)((B + kWRows - 1) / kWRows) * K;
}

extern "C" int f110_ddpg_relu_bwd(const float *gy, const float *y, int32_t B, int32_t K, float *gz, float *db,
                                  float *scratch, void *stream) {
    if (B <= 0 || K <= 0 || K > 4 * kHB || (K + 3) / 4 > kHB || !gy || !y || !gz || (db && !scratch))
        return fail_arg("f110_ddpg_relu_bwd");
    const int nblk = (B + kWRows - 1) / kWRows;
    hipLaunchKernelGGL(k_relu_bwd, dim3((unsigned)nblk), dim3(kHB), 0, (hipStream_t)stream, gy, y, gz,
                       db ? scratch : nullptr, B, K);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && db) {
        const int per = kHB / 64;
        hipLaunchKernelGGL(k_colsum_finish, dim3((unsigned)((K + per - 1) / per)), dim3(kHB), 0, (hipStream_t)stream,
                           scratch, nblk, K, db);
        e = hipGetLastError();
    }
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_relu_bwd", e);
}

extern "C" int f110_ddpg_actor_head(const float *h, const float *W, const float *b, const float *scale,
                                    const float *shift, int32_t B, int32_t K, int32_t nout, float *act, float *t,
                                    void *stream) {
    if (bad_shape(B, K, nout) || !h || !W || !b || !scale || !shift || !act || !t) return fail_arg("f110_ddpg_actor_head");
    HeadArgs a{};
    a.h = h, a.W = W, a.b = b, a.aux0 = scale, a.aux1 = shift, a.out0 = act, a.out1 = t;
    a.B = B, a.K = K, a.nout = nout;
    hipError_t e = with_nout(nout, [&](auto N) {
        hipLaunchKernelGGL((k_head_fwd<kActor, decltype(N)::value>), dim3(row_blocks(B)), dim3(kHB), 0,
                           (hipStream_t)stream, a);
        return hipGetLastError();
    });
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_actor_head", e);
}

extern "C" int f110_ddpg_actor_explore(const float *h, const float *W, const float *b, const float *scale,
                                       const float *shift, int32_t B, int32_t K, int32_t nout,
                                       const double *state_in, double *state_out, double decay, double sigma_min,
                                       const float *low, const float *high, uint64_t seed, float *out,
                                       int64_t out_stride, void *stream) {
    if (bad_shape(B, K, nout) || !h || !W || !b || !scale || !shift || !state_in || !state_out ||
        state_in == state_out || !low || !high || !out || out_stride < nout)
        return fail_arg("f110_ddpg_actor_explore");
    HeadArgs a{};
    a.h = h, a.W = W, a.b = b, a.aux0 = scale, a.aux1 = shift, a.out0 = out;
    a.lo = low, a.hi = high, a.nstate_in = state_in, a.nstate_out = state_out, a.decay = decay;
    a.sigma_min = sigma_min, a.out_stride = out_stride, a.seed = seed;
    a.B = B, a.K = K, a.nout = nout;
    hipError_t e = with_nout(nout, [&](auto N) {
        hipLaunchKernelGGL((k_head_fwd<kExplore, decltype(N)::value>), dim3(row_blocks(B)), dim3(kHB), 0,
                           (hipStream_t)stream, a);
        return hipGetLastError();
    });
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_actor_explore", e);
}

extern "C" int f110_ddpg_actor_head_bwd(const float *h, const float *W, const float *t, const float *scale,
                                        const float *dact, int32_t B, int32_t K, int32_t nout, float *dh,
                                        const float *dh_mask, float *dW, float *db, float *scratch, void *stream) {
    if (bad_shape(B, K, nout) || !h || !W || !t || !scale || !dact || !scratch)
        return fail_arg("f110_ddpg_actor_head_bwd");
    HeadArgs a{};
    a.h = h, a.W = W, a.t = t, a.aux0 = scale, a.dout = dact, a.dh = dh, a.dh_mask = dh_mask, a.dW = dW, a.db = db;
    a.dz = scratch, a.part = scratch + (int64_t)B * nout;
    a.B = B, a.K = K, a.nout = nout;
    hipError_t e = with_nout(nout, [&](auto N) {
        hipLaunchKernelGGL((k_head_bwd_rows<kActor, decltype(N)::value>), dim3(row_blocks(B)), dim3(kHB), 0,
                           (hipStream_t)stream, a);
        return hipGetLastError();
    });
    if (e == hipSuccess) e = wgrad(a, (hipStream_t)stream);
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_actor_head_bwd", e);
}

extern "C" int f110_ddpg_td_target(const float *h, const float *W, const float *b, const float *r, const float *d,
                                   float gamma, int32_t B, int32_t K, float *y, void *stream) {
    if (bad_shape(B, K, 1) || !h || !W || !b || !r || !d || !y) return fail_arg("f110_ddpg_td_target");
    HeadArgs a{};
    a.h = h, a.W = W, a.b = b, a.aux0 = r, a.aux1 = d, a.out0 = y, a.gamma = gamma;
    a.B = B, a.K = K, a.nout = 1;
    hipLaunchKernelGGL((k_head_fwd<kTarget, 1>), dim3(row_blocks(B)), dim3(kHB), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_td_target", e);
}

extern "C" int f110_ddpg_critic_loss(const float *h, const float *W, const float *b, const float *y, const float *w,
                                     int32_t B, int32_t K, float *td, float *loss, float *scratch, void *stream) {
    if (bad_shape(B, K, 1) || !h || !W || !b || !y || !w || !td || !loss || !scratch)
        return fail_arg("f110_ddpg_critic_loss");
    HeadArgs a{};
    a.h = h, a.W = W, a.b = b, a.aux0 = y, a.aux1 = w, a.out0 = td, a.loss = loss, a.sign = 1.0f;
    a.part = scratch + B;
    a.B = B, a.K = K, a.nout = 1, a.nblk = (int32_t)row_blocks(B);
    hipLaunchKernelGGL((k_head_fwd<kLoss, 1>), dim3(row_blocks(B)), dim3(kHB), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_loss_finish, dim3(1), dim3(kHB), 0, (hipStream_t)stream, a);
        e = hipGetLastError();
    }
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_critic_loss", e);
}

extern "C" int f110_ddpg_critic_loss_bwd(const float *h, const float *W, const float *td, const float *w,
                                         const float *g, int32_t B, int32_t K, float *dh, const float *dh_mask,
                                         float *dW, float *db, float *scratch, void *stream) {
    if (bad_shape(B, K, 1) || !h || !W || !td || !w || !g || !scratch) return fail_arg("f110_ddpg_critic_loss_bwd");
    HeadArgs a{};
    a.h = h, a.W = W, a.out0 = const_cast<float *>(td), a.aux1 = w, a.g = g, a.dh = dh, a.dh_mask = dh_mask, a.dW = dW,
    a.db = db;
    a.dz = scratch, a.part = scratch + B;
    a.B = B, a.K = K, a.nout = 1;
    hipLaunchKernelGGL((k_head_bwd_rows<kLoss, 1>), dim3(row_blocks(B)), dim3(kHB), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = wgrad(a, (hipStream_t)stream);
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_critic_loss_bwd", e);
}

extern "C" int f110_ddpg_q_mean(const float *h, const float *W, const float *b, float sign, int32_t B, int32_t K,
                                float *loss, float *scratch, void *stream) {
    if (bad_shape(B, K, 1) || !h || !W || !b || !loss || !scratch) return fail_arg("f110_ddpg_q_mean");
    HeadArgs a{};
    a.h = h, a.W = W, a.b = b, a.loss = loss, a.sign = sign, a.part = scratch + B;
    a.B = B, a.K = K, a.nout = 1, a.nblk = (int32_t)row_blocks(B);
    hipLaunchKernelGGL((k_head_fwd<kMean, 1>), dim3(row_blocks(B)), dim3(kHB), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_loss_finish, dim3(1), dim3(kHB), 0, (hipStream_t)stream, a);
        e = hipGetLastError();
    }
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_q_mean", e);
}

extern "C" int f110_ddpg_q_mean_bwd(const float *h, const float *W, const float *g, float sign, int32_t B, int32_t K,
                                    float *dh, const float *dh_mask, float *dW, float *db, float *scratch,
                                    void *stream) {
    if (bad_shape(B, K, 1) || !W || !g || !scratch || ((dW || db) && !h)) return fail_arg("f110_ddpg_q_mean_bwd");
    HeadArgs a{};
    a.h = h, a.W = W, a.g = g, a.sign = sign, a.dh = dh, a.dh_mask = dh_mask, a.dW = dW, a.db = db;
    a.dz = scratch, a.part = scratch + B;
    a.B = B, a.K = K, a.nout = 1;
    hipLaunchKernelGGL((k_head_bwd_rows<kMean, 1>), dim3(row_blocks(B)), dim3(kHB), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = wgrad(a, (hipStream_t)stream);
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_q_mean_bwd", e);
}

extern "C" int f110_ddpg_critic_step(const float *ht, const float *Wt, const float *bt, const float *r, const float *d,
                                     float gamma, const float *h, const float *W, const float *b, const float *w,
                                     const float *g, int32_t B, int32_t K, float *td, float *dh, const float *dh_mask,
                                     float *dq, float *part, void *stream) {
    if (bad_shape(B, K, 1) || !ht || !Wt || !bt || !r || !d || !h || !W || !b || !w || !g || !td || !part)
        return fail_arg("f110_ddpg_critic_step");
    HeadArgs a{};
    a.ht = ht, a.Wt = Wt, a.bt = bt, a.aux0 = r, a.aux1 = d, a.gamma = gamma;
    a.h = h, a.W = W, a.b = b, a.dout = w, a.g = g, a.out0 = td, a.dh = dh, a.dh_mask = dh_mask, a.dz = dq;
    a.part = part;
    a.B = B, a.K = K, a.nout = 1;
    hipLaunchKernelGGL(k_critic_step, dim3(row_blocks(B)), dim3(kHB), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_critic_step", e);
}

extern "C" int f110_ddpg_q_mean_step(const float *h, const float *W, const float *b, const float *g, float sign,
                                     int32_t B, int32_t K, float *dh, const float *dh_mask, float *part,
                                     void *stream) {
    if (bad_shape(B, K, 1) || !h || !W || !b || !g || !part) return fail_arg("f110_ddpg_q_mean_step");
    HeadArgs a{};
    a.h = h, a.W = W, a.b = b, a.g = g, a.sign = sign, a.dh = dh, a.dh_mask = dh_mask, a.part = part;
    a.B = B, a.K = K, a.nout = 1;
    hipLaunchKernelGGL(k_q_mean_step, dim3(row_blocks(B)), dim3(kHB), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail_hip("f110_ddpg_q_mean_step", e);
}

extern "C" int32_t f110_ddpg_row_blocks(int32_t B) { return B > 0 ? (int32_t)row_blocks(B) : -1; }
