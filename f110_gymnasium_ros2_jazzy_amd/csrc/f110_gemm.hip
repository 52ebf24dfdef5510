// f110_gemm.hip — the DDPG learner's hidden-layer GEMMs on the fp32 matrix
// cores (include/f110.h, "learner GEMMs").
//
// Shapes (train_ddpg: batch M = 4096 rows, obs 1088, hidden 128): the first
// layers are [4096 x 1088] x [1088 x 128] (1.14 GFLOP each, five per update
// plus the policy's forward), the weight gradients [128 x 4096] x [4096 x
// 1088], the rest K or N = 128.  At these sizes a 128-row BLAS tile leaves
// most of the 256 CUs idle (hipBLASLt: 20.4 us forward, 25.5 us per weight
// gradient, ~55 TFLOP/s); here
//   * k_lgemm: a 32 x 64 output tile per 4-wave block, K split over the 4
//     waves (partial tiles summed in LDS in wave order), so one 4096 x 128
//     GEMM is 256 blocks and a grouped launch of 2-3 GEMMs that share the
//     batch is 512-768 (2-3 co-resident blocks per CU).  v_mfma_f32_32x32x2_f32
//     with a register double buffer of 16-k chunks: per chunk a lane loads
//     two float4 of each of its A / B rows (k = 16c + 8q + 4h + e: the same
//     permutation of k on both operands, so every partial is an exact fp32
//     fma chain over a reordered k), 3 x 2 loads per 16 MFMAs (1024 cycles).
//     The layer's epilogue is fused: bias, ReLU, the critic's two action
//     columns of fcs2's input (no torch.cat), an output mask (the next
//     layer's threshold_backward) and an input mask (this layer's).
//   * k_lwgrad: dW = G'^T X over M split across blocks (4 waves x S slices),
//     64 x 64 tiles of 32x32x2 MFMAs; each wave stages its 16-row chunks of
//     G' and X through LDS (float4 row loads, fragments by ds_read_b32); db
//     from the same G' fragments; k_lwgrad_finish adds the S partials in order.
// The C/D layout of the 32x32 f32 MFMA: column = lane & 31, row = (reg & 3)
// + 8 (reg >> 2) + 4 (lane >> 5).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "f110_internal.h"

int f110_set_error(int code, const std::string &msg);  // f110_capi.cpp

namespace f110 {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
constexpr int kGB = 256;      // threads per block (4 waves)
constexpr int kMaxOps = 4;    // GEMMs per grouped launch
constexpr int kTM = 32, kTN = 64;   // k_lgemm output tile
constexpr int kWN = 64, kWK = 64;   // k_lwgrad output tile

struct GemmLaunch {
    f110_gemm_op op[kMaxOps];
    int32_t blk0[kMaxOps + 1];  // first block of each op (multiples of 8)
    int32_t ntn[kMaxOps];       // column tiles of each op
    int32_t nops, M;
};

struct WgradLaunch {
    f110_wgrad_op op[kMaxOps];
    int64_t poff[kMaxOps + 1];  // each op's partials in the scratch: [S][N][KX] then [S][N]
    int32_t blk0[kMaxOps + 1];
    int32_t ntk[kMaxOps];       // kx tiles of each op
    int32_t vec[kMaxOps];       // G / X / gmask rows loadable as float4
    int32_t nops, M, S;
    float *part;
    // f110_learner_wgrad_loss: *loss = loss_sign * sum(loss_part[0 .. loss_n)) / M (the finishing launch's last block)
    const float *loss_part;
    float *loss;
    float loss_sign;
    int32_t loss_n;
};

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// pins a prefetched value in its registers (otherwise the compiler may turn
// the register double buffer back into loads at the top of the iteration)
__device__ __forceinline__ void pin(float4 &v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
__device__ __forceinline__ void pin(float &v) { asm volatile("" : "+v"(v)); }

__device__ __forceinline__ float relu_nan(float v) { return v > 0.0f ? v : (v != v ? v : 0.0f); }

__device__ __forceinline__ float4 keep(float4 v, uint32_t m) {  // v where m = ~0, +0 where m = 0
    return make_float4(__uint_as_float(__float_as_uint(v.x) & m), __uint_as_float(__float_as_uint(v.y) & m),
                       __uint_as_float(__float_as_uint(v.z) & m), __uint_as_float(__float_as_uint(v.w) & m));
}

__device__ __forceinline__ float get(const float4 &v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }

// the op of block blk (op index uniform: selected field-wise, no dynamic
// indexing of the kernel-argument array)
template <class Launch, class Op>
__device__ __forceinline__ int select_op(const Launch &L, int blk, Op &o) {
    int p = 0;
#pragma unroll
    for (int q = 1; q < kMaxOps; ++q)
        if (q < L.nops && blk >= L.blk0[q]) p = q;
    o = L.op[0];
#pragma unroll
    for (int q = 1; q < kMaxOps; ++q)
        if (p == q) o = L.op[q];
    return p;
}

// ---------------------------------------------------------------- k_lgemm --
// the partial tiles red[w][v][lane] (w = the NW K-split waves, v = accumulator
// register (i, j, reg) of the 32 x 32 tiles) summed in wave order, then the
// layer's epilogue; thread (wave, lane) owns registers wave*R/NW .. +R/NW
template <int NW, int RJ, int R>
__device__ __forceinline__ void lgemm_epilogue(const f110_gemm_op &o, const float (*red)[R][64], int wave, int lane,
                                               int m0, int n0, int M) {
    const int r = lane & 31, h = lane >> 5, N = o.N;
#pragma unroll
    for (int u = 0; u < R / NW; ++u) {
        const int v = wave * (R / NW) + u;
        float s = red[0][v][lane];
#pragma unroll
        for (int w = 1; w < NW; ++w) s += red[w][v][lane];
        const int t = v >> 4, vv = v & 15;
        const int i = t / RJ, j = t - i * RJ;
        const int row = m0 + 32 * i + (vv & 3) + 8 * (vv >> 2) + 4 * h;
        const int col = n0 + 32 * j + r;
        if (row < M && col < N) {
            for (int x = 0; x < o.nx2; ++x) s = fmaf(o.x2[(size_t)row * o.ldx2 + x], o.w2[(size_t)col * o.ldw2 + x], s);
            if (o.bias) s += o.bias[col];
            if (o.relu) s = relu_nan(s);
            if (o.omask) s = o.omask[(size_t)row * o.ldc + col] > 0.0f ? s : 0.0f;
            o.C[(size_t)row * o.ldc + col] = s;
        }
    }
}

// the block's op and output tile: (p, m0, n0), XCD-aware (the column tiles of
// one row tile share blockIdx % 8, so one L2 holds A's rows)
__device__ __forceinline__ void lgemm_tile(const GemmLaunch &L, f110_gemm_op &o, int &m0, int &n0) {
    const int blk = (int)blockIdx.x;
    const int p = select_op(L, blk, o);
    int ntn = L.ntn[0], b0 = L.blk0[0];
#pragma unroll
    for (int q = 1; q < kMaxOps; ++q)
        if (p == q) {
            ntn = L.ntn[q];
            b0 = L.blk0[q];
        }
    const int local = blk - b0;
    const int grp = local / (8 * ntn), rem = local - grp * 8 * ntn;
    m0 = (grp * 8 + (rem & 7)) * kTM;
    n0 = (rem >> 3) * kTN;
}

struct Frag {
    float4 a[kTM / 32][2];
    float4 b[kTN / 32][2];
};

// VEC: A rows (and amask) 16-B aligned; BV: B rows (nn = 0) loaded as float4 / float2 / floats.
// NW waves per block split K; NB register buffers (NB - 1 chunks of loads in flight).  Round 4
// measured 8 waves and 3 buffers (no faster), v_mfma_f32_16x16x4_f32 with 8 accumulators (slower
// on the grouped launches), a probe without loads in the loop (the 3-op launch 42 -> 29 us) and
// both operands staged through LDS in whole 128-B lines (8-row pieces, XOR-swizzled images,
// ds_read_b128 fragments; 1 / 2 / 3 ops 16.9 / 29.5 / 40.8 -> 17.6 / 28.8 / 41.5 us: no gain, so
// the fragment-shaped loads are not what bounds it)
template <bool NN, bool VEC, int BV, bool AMASK>
__global__ void __launch_bounds__(256) k_lgemm(GemmLaunch L) {
    constexpr int NW = 4, NB = 2;
    constexpr int RI = kTM / 32, RJ = kTN / 32, R = RI * RJ * 16;
    static_assert(R % NW == 0, "tile registers split evenly over the waves");
    __shared__ float red[NW][R][64];
    f110_gemm_op o;
    int m0, n0;
    lgemm_tile(L, o, m0, n0);
    const int M = L.M, N = o.N, K = o.K;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int nch = (K + 15) >> 4;
    const int cb = wave * nch / NW, ce = (wave + 1) * nch / NW;

    const float *pa[RI], *pm[RI], *pb[RJ];
#pragma unroll
    for (int i = 0; i < RI; ++i) {
        const int row = min(m0 + 32 * i + r, M - 1);  // rows past M: computed, not stored
        pa[i] = o.A + (size_t)row * o.lda + 4 * h;
        pm[i] = AMASK ? o.amask + (size_t)row * o.lda + 4 * h : nullptr;
    }
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        const int col = min(n0 + 32 * j + r, N - 1);
        pb[j] = NN ? o.B + (size_t)(4 * h) * o.ldb + col : o.B + (size_t)col * o.ldb + 4 * h;
    }
    const size_t ldb = o.ldb;

    // a chunk wholly inside K: unconditional loads (no branch may separate a
    // prefetch from its use, or the compiler drains it with vmcnt(0))
    auto load_full = [&](int c, Frag &f) {
        const int k0 = 16 * c;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int kq = k0 + 8 * q;  // + 4h + e
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                float4 v, mk;
                if (VEC) {
                    v = *reinterpret_cast<const float4 *>(pa[i] + kq);
                    if (AMASK) mk = *reinterpret_cast<const float4 *>(pm[i] + kq);
                } else {
                    v = make_float4(pa[i][kq], pa[i][kq + 1], pa[i][kq + 2], pa[i][kq + 3]);
                    if (AMASK) mk = make_float4(pm[i][kq], pm[i][kq + 1], pm[i][kq + 2], pm[i][kq + 3]);
                }
                if (AMASK) {
                    v.x = mk.x > 0.0f ? v.x : 0.0f;
                    v.y = mk.y > 0.0f ? v.y : 0.0f;
                    v.z = mk.z > 0.0f ? v.z : 0.0f;
                    v.w = mk.w > 0.0f ? v.w : 0.0f;
                }
                f.a[i][q] = v;
            }
#pragma unroll
            for (int j = 0; j < RJ; ++j) {
                if (NN)
                    f.b[j][q] = make_float4(pb[j][kq * ldb], pb[j][(kq + 1) * ldb], pb[j][(kq + 2) * ldb],
                                            pb[j][(kq + 3) * ldb]);
                else if (BV == 4)
                    f.b[j][q] = *reinterpret_cast<const float4 *>(pb[j] + kq);
                else if (BV == 2) {
                    const float2 lo = *reinterpret_cast<const float2 *>(pb[j] + kq);
                    const float2 hi = *reinterpret_cast<const float2 *>(pb[j] + kq + 2);
                    f.b[j][q] = make_float4(lo.x, lo.y, hi.x, hi.y);
                } else
                    f.b[j][q] = make_float4(pb[j][kq], pb[j][kq + 1], pb[j][kq + 2], pb[j][kq + 3]);
            }
        }
    };
    // the last chunk when K % 16 != 0 (at most one, on the last wave): masked
    auto load_tail = [&](int c, Frag &f) {
        const int k0 = 16 * c;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int kq = k0 + 8 * q;
            float va[RI][4], vb[RJ][4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool in = kq + 4 * h + e < K;
#pragma unroll
                for (int i = 0; i < RI; ++i) {
                    float v = in ? pa[i][kq + e] : 0.0f;
                    if (AMASK && in) v = pm[i][kq + e] > 0.0f ? v : 0.0f;
                    va[i][e] = v;
                }
#pragma unroll
                for (int j = 0; j < RJ; ++j) vb[j][e] = in ? (NN ? pb[j][(kq + e) * ldb] : pb[j][kq + e]) : 0.0f;
            }
#pragma unroll
            for (int i = 0; i < RI; ++i) f.a[i][q] = make_float4(va[i][0], va[i][1], va[i][2], va[i][3]);
#pragma unroll
            for (int j = 0; j < RJ; ++j) f.b[j][q] = make_float4(vb[j][0], vb[j][1], vb[j][2], vb[j][3]);
        }
    };
    f32x16 acc[RI][RJ];
#pragma unroll
    for (int i = 0; i < RI; ++i)
#pragma unroll
        for (int j = 0; j < RJ; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.0f;
    auto compute = [&](const Frag &f) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < RI; ++i)
#pragma unroll
                    for (int j = 0; j < RJ; ++j) acc[i][j] = mfma(get(f.a[i][q], e), get(f.b[j][q], e), acc[i][j]);
    };
    // NB register buffers: while chunk c's MFMAs issue, chunks c+1 .. c+NB-1 are in flight
    const int cf = min(ce, K >> 4);
    if (cb < cf) {
        Frag f[NB];
#pragma unroll
        for (int u = 0; u < NB - 1; ++u) load_full(min(cb + u, cf - 1), f[u]);
        int c = cb;
        for (; c + NB <= cf; c += NB) {
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                load_full(min(c + u + NB - 1, cf - 1), f[(u + NB - 1) % NB]);  // past the end: unused
                __builtin_amdgcn_sched_barrier(0);
                compute(f[u]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int u = 0; u < NB - 1; ++u)  // the last cf - c (< NB) chunks, already loaded
            if (c + u < cf) compute(f[u]);
    }
    if (ce > cf) {
        Frag ft;
        load_tail(cf, ft);
        compute(ft);
    }
#pragma unroll
    for (int i = 0; i < RI; ++i)
#pragma unroll
        for (int j = 0; j < RJ; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) red[wave][(i * RJ + j) * 16 + v][lane] = acc[i][j][v];
    __syncthreads();
    lgemm_epilogue<NW, RJ, R>(o, red, wave, lane, m0, n0, M);
}

// --------------------------------------------------------------- k_lwgrad --
// A 64 x 64 tile of dW per block, M split over S slices x 4 waves: per
// 16-row chunk a wave loads its G' and X rows (64 columns each) as 4 rows x
// 256 B per dwordx4 instruction (4 + 4, + 4 for the mask; round 4's first
// form loaded the fragments directly, 32 single-dword loads per chunk, 6 %
// slower on the 128 x 1088 gradient), writes them to its own LDS image and
// reads the MFMA fragments (lane = column, lane half = row parity) with
// ds_read_b32.
// Image rows are 96 floats apart, so the two lane halves (rows 2t and 2t+1)
// read opposite halves of the 64 banks.  Ops whose rows are not float4-able
// (the critic's two action columns) take the same loop with per-element
// loads (a block-uniform choice outside the loop).  Columns past N / KX are
// loaded from clamped addresses (their outputs are not stored); rows past M
// load row M-1 with G' = 0.  Sum order: per lane the chunk rows in order, as
// k_lwgrad's 8-row chunks.
template <bool VEC, bool GMASK>
__device__ __forceinline__ void lwgrad_loop(const f110_wgrad_op &o, float *img, int M, int cb, int ce, int n0,
                                                int k0, f32x16 (&acc)[2][2], float (&dsum)[2]) {
    constexpr int CM = 16, PITCH = 96;
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int rl = lane >> 4, sg = lane & 15;  // load row (of 4), 16-B segment
    const int N = o.N, KX = o.KX;
    const size_t ldg = o.ldg, ldx = o.ldx;
    // column offsets of this lane's segment (clamped in range)
    const int cg = min(n0 + 4 * sg, N - 4 < 0 ? 0 : N - 4), cx = min(k0 + 4 * sg, KX - 4 < 0 ? 0 : KX - 4);
    int eg[4], ex[4];  // per-element columns for the !VEC loads
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        eg[e] = min(n0 + 4 * sg + e, N - 1);
        ex[e] = min(k0 + 4 * sg + e, KX - 1);
    }
    float4 gg[4], gx[4], gk[4];
    uint32_t rin[4];
    auto ld4 = [&](const float *base, size_t row, size_t ld, int cv, const int *ce4) -> float4 {
        const float *p = base + row * ld;
        if (VEC) return *reinterpret_cast<const float4 *>(p + cv);
        return make_float4(p[ce4[0]], p[ce4[1]], p[ce4[2]], p[ce4[3]]);
    };
    auto gload = [&](int c) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = CM * c + 4 * i + rl;
            rin[i] = m < M ? ~0u : 0u;
            const size_t mr = (size_t)min(m, M - 1);
            gg[i] = ld4(o.G, mr, ldg, cg, eg);
            if (GMASK) gk[i] = ld4(o.gmask, mr, ldg, cg, eg);
            gx[i] = ld4(o.X, mr, ldx, cx, ex);
        }
    };
    auto swrite = [&]() {  // G rows at image rows 0..15, X rows at 16..31
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float4 g = gg[i];
            if (GMASK) {
                pin(g);  // the mask select stays here, after the MFMAs
                pin(gk[i]);
                g.x = gk[i].x > 0.0f ? g.x : 0.0f;
                g.y = gk[i].y > 0.0f ? g.y : 0.0f;
                g.z = gk[i].z > 0.0f ? g.z : 0.0f;
                g.w = gk[i].w > 0.0f ? g.w : 0.0f;
            }
            const int q = 4 * i + rl;
            uint32_t m = rin[i];
            asm volatile("" : "+v"(m));  // opaque: the zeroing stays here, after the MFMAs (not a select at the load)
            *reinterpret_cast<float4 *>(img + q * PITCH + 4 * sg) = keep(g, m);
            *reinterpret_cast<float4 *>(img + (CM + q) * PITCH + 4 * sg) = gx[i];
        }
    };
    auto compute = [&]() {  // every fragment read issued first: the MFMAs wait on them in order
        float g[CM / 2][2], x[CM / 2][2];
#pragma unroll
        for (int t = 0; t < CM / 2; ++t)
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                g[t][a] = img[(2 * t + h) * PITCH + 32 * a + r];
                x[t][a] = img[(CM + 2 * t + h) * PITCH + 32 * a + r];
            }
#pragma unroll
        for (int t = 0; t < CM / 2; ++t) {
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[a][b] = mfma(g[t][a], x[t][b], acc[a][b]);
            dsum[0] += g[t][0];
            dsum[1] += g[t][1];
        }
    };
    if (cb < ce) {
        gload(cb);
        swrite();
        for (int c = cb; c < ce; ++c) {
            gload(min(c + 1, ce - 1));  // the next chunk in flight (past the end: reloaded, unused)
            __builtin_amdgcn_sched_barrier(0);
            compute();
            __builtin_amdgcn_sched_barrier(0);
            swrite();
        }
    }
}

template <bool FINAL, bool GMASK>
__global__ void __launch_bounds__(kGB) k_lwgrad(WgradLaunch L) {
    constexpr int CM = 16, PITCH = 96;
    static_assert(4 * 2 * CM * PITCH <= 4 * 64 * 64, "the staging images fit in the reduction buffer");
    __shared__ float lds[4 * 64 * 64 + 4 * 2 * 64];  // red[4][64][64], dred[4][2][64]; images alias red
    const int blk = (int)blockIdx.x;
    f110_wgrad_op o;
    const int p = select_op(L, blk, o);
    int ntk = L.ntk[0], b0 = L.blk0[0], vec = L.vec[0];
    int64_t poff = L.poff[0];
#pragma unroll
    for (int q = 1; q < kMaxOps; ++q)
        if (p == q) {
            ntk = L.ntk[q];
            b0 = L.blk0[q];
            poff = L.poff[q];
            vec = L.vec[q];
        }
    const int S = L.S, M = L.M, N = o.N, KX = o.KX;
    const int local = blk - b0;
    const int s = local % S, tile = local / S;
    const int n0 = (tile / ntk) * kWN, k0 = (tile % ntk) * kWK;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int mch = (M + CM - 1) / CM;
    const int sb = s * mch / S, se = (s + 1) * mch / S;
    const int cb = sb + wave * (se - sb) / 4, ce = sb + (wave + 1) * (se - sb) / 4;
    const bool want_db = o.db != nullptr && k0 == 0;
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.0f;
    float dsum[2] = {0.0f, 0.0f};
    float *img = lds + wave * (2 * CM * PITCH);
    if (vec) lwgrad_loop<true, GMASK>(o, img, M, cb, ce, n0, k0, acc, dsum);
    else lwgrad_loop<false, GMASK>(o, img, M, cb, ce, n0, k0, acc, dsum);
    __syncthreads();  // the reduction reuses the images
    float(*red)[64][64] = reinterpret_cast<float(*)[64][64]>(lds);
    float(*dred)[2][64] = reinterpret_cast<float(*)[2][64]>(lds + 4 * 64 * 64);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) red[wave][(a * 2 + b) * 16 + v][lane] = acc[a][b][v];
    if (want_db) {
        dred[wave][0][lane] = dsum[0];
        dred[wave][1][lane] = dsum[1];
    }
    __syncthreads();
    float *part = L.part + poff;
    const size_t nk = (size_t)N * KX;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int v = wave * 16 + u;
        float sum = red[0][v][lane];
#pragma unroll
        for (int w = 1; w < 4; ++w) sum += red[w][v][lane];
        const int t = v >> 4, vv = v & 15;
        const int n = n0 + 32 * (t >> 1) + (vv & 3) + 8 * (vv >> 2) + 4 * h;
        const int kx = k0 + 32 * (t & 1) + r;
        if (n < N && kx < KX) {
            if (FINAL) o.dW[(size_t)n * o.ldw + kx] = sum;
            else part[(size_t)s * nk + (size_t)n * KX + kx] = sum;
        }
    }
    if (want_db && wave == 0 && h == 0) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            float sum = 0.0f;
#pragma unroll
            for (int w = 0; w < 4; ++w) sum += dred[w][a][r] + dred[w][a][r + 32];
            const int n = n0 + 32 * a + r;
            if (n < N) {
                if (FINAL) o.db[n] = sum;
                else part[(size_t)S * nk + (size_t)s * N + n] = sum;
            }
        }
    }
}

// dW / db = the S partials added in slice order; one thread per output.  With
// a loss, the last block instead sums its partials as k_loss_finish does
// (per-thread strided sums, a shuffle tree per wave, waves in order).
__global__ void __launch_bounds__(kGB) k_lwgrad_finish(WgradLaunch L, int64_t total) {
    if (L.loss && blockIdx.x == gridDim.x - 1) {  // block-uniform
        __shared__ float ws[kGB / 64];
        float v = 0.0f;
        for (int i = threadIdx.x; i < L.loss_n; i += kGB) v += L.loss_part[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            float t = 0.0f;
            for (int w = 0; w < kGB / 64; ++w) t += ws[w];
            *L.loss = L.loss_sign * (t / (float)L.M);
        }
        return;
    }
    const int64_t idx = (int64_t)blockIdx.x * kGB + threadIdx.x;
    if (idx >= total) return;
    int p = 0;
    int64_t base = 0;
    bool found = false;
#pragma unroll
    for (int q = 0; q < kMaxOps; ++q)
        if (!found && q < L.nops) {
            const int64_t n_out = (int64_t)L.op[q].N * L.op[q].KX + L.op[q].N;
            if (idx < base + n_out) {
                p = q;
                found = true;
            } else {
                base += n_out;
            }
        }
    f110_wgrad_op o = L.op[0];
#pragma unroll
    for (int q = 1; q < kMaxOps; ++q)
        if (p == q) o = L.op[q];
    const float *part = L.part + L.poff[p];
    const int64_t nk = (int64_t)o.N * o.KX;
    const int64_t e = idx - base;
    const int S = L.S;
    if (e < nk) {
        float sum = part[e];
        for (int s = 1; s < S; ++s) sum += part[(int64_t)s * nk + e];
        const int64_t n = e / o.KX, kx = e - n * o.KX;
        o.dW[n * o.ldw + kx] = sum;
    } else if (o.db) {
        const int64_t n = e - nk;
        float sum = part[S * nk + n];
        for (int s = 1; s < S; ++s) sum += part[S * nk + (int64_t)s * o.N + n];
        o.db[n] = sum;
    }
}

int fail(const char *fn, const char *what) { return f110_set_error(F110_E_INVALID, std::string(fn) + ": " + what); }

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
bool aligned8(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 7u) == 0; }

// blocks per slice count S for a grouped weight-gradient launch: at most 256
// blocks, one per CU (at ~320, a third of the CUs ran two blocks and the
// launch took their time: 28.1 -> 23.4 us for the 128 x 1088 gradient, DESIGN
// §8), at least two 8-row chunks per wave; a function of the shapes only
int wgrad_slices(const f110_wgrad_op *ops, int nops, int M) {
    int64_t tiles = 0;
    for (int q = 0; q < nops; ++q)
        tiles += (int64_t)((ops[q].N + kWN - 1) / kWN) * ((ops[q].KX + kWK - 1) / kWK);
    const int64_t mch = (M + 7) / 8;
    int64_t S = std::max<int64_t>(1, 256 / tiles);
    S = std::min<int64_t>(S, std::max<int64_t>(1, mch / 8));
    return (int)std::max<int64_t>(1, S);
}

bool wgrad_ok(const f110_wgrad_op *ops, int nops, int M) {
    if (!ops || nops < 1 || nops > kMaxOps || M <= 0) return false;
    for (int q = 0; q < nops; ++q) {
        const f110_wgrad_op &o = ops[q];
        if (!o.G || !o.X || !o.dW || o.N <= 0 || o.KX <= 0 || o.ldg < o.N || o.ldx < o.KX || o.ldw < o.KX ||
            (o.gmask != nullptr) != (ops[0].gmask != nullptr))
            return false;
    }
    return true;
}

}  // namespace
}  // namespace f110

using namespace f110;

extern "C" int f110_learner_gemm(const f110_gemm_op *ops, int32_t nops, int32_t M, void *stream) {
    const char *fn = "f110_learner_gemm";
    if (!ops || nops < 1 || nops > kMaxOps || M <= 0) return fail(fn, "bad arguments");
    GemmLaunch L{};
    L.nops = nops;
    L.M = M;
    const int nn = ops[0].nn ? 1 : 0;
    const int am = ops[0].amask ? 1 : 0;
    bool vec = true;
    int bv = 4;
    int32_t blk = 0;
    const int64_t rts = ((int64_t)(M + kTM - 1) / kTM + 7) / 8 * 8;  // row tiles, whole XCD groups
    for (int q = 0; q < nops; ++q) {
        const f110_gemm_op &o = ops[q];
        if (!o.A || !o.B || !o.C || o.N <= 0 || o.K <= 0 || (o.nn ? 1 : 0) != nn || (o.amask ? 1 : 0) != am || o.lda < o.K || o.ldc < o.N ||
            (nn ? o.ldb < o.N : o.ldb < o.K) || o.nx2 < 0 || o.nx2 > 2 || (o.nx2 && (!o.x2 || !o.w2)))
            return fail(fn, "bad op");
        vec = vec && o.lda % 4 == 0 && aligned16(o.A) && (!o.amask || aligned16(o.amask));
        const int obv = nn ? 1 : (o.ldb % 4 == 0 && aligned16(o.B)) ? 4 : (o.ldb % 2 == 0 && aligned8(o.B)) ? 2 : 1;
        bv = std::min(bv, obv);
        L.op[q] = o;
        L.blk0[q] = blk;
        L.ntn[q] = (o.N + kTN - 1) / kTN;
        const int64_t nb = rts * L.ntn[q];
        if (blk + nb > (1 << 30)) return fail(fn, "too large");
        blk += (int32_t)nb;
    }
    L.blk0[nops] = blk;
    for (int q = nops; q < kMaxOps; ++q) L.blk0[q] = blk;
#define F110_LG(NN, V, BV, AM) reinterpret_cast<const void *>(&k_lgemm<NN, V, BV, AM>)
    const void *fs[2][2][3][2] = {  // [nn][vec][bv: 1, 2, 4][amask]
        {{{F110_LG(false, false, 1, false), F110_LG(false, false, 1, true)},
          {F110_LG(false, false, 2, false), F110_LG(false, false, 2, true)},
          {F110_LG(false, false, 4, false), F110_LG(false, false, 4, true)}},
         {{F110_LG(false, true, 1, false), F110_LG(false, true, 1, true)},
          {F110_LG(false, true, 2, false), F110_LG(false, true, 2, true)},
          {F110_LG(false, true, 4, false), F110_LG(false, true, 4, true)}}},
        {{{F110_LG(true, false, 1, false), F110_LG(true, false, 1, true)},
          {F110_LG(true, false, 1, false), F110_LG(true, false, 1, true)},
          {F110_LG(true, false, 1, false), F110_LG(true, false, 1, true)}},
         {{F110_LG(true, true, 1, false), F110_LG(true, true, 1, true)},
          {F110_LG(true, true, 1, false), F110_LG(true, true, 1, true)},
          {F110_LG(true, true, 1, false), F110_LG(true, true, 1, true)}}}};
#undef F110_LG
    const int bvi = bv == 4 ? 2 : bv == 2 ? 1 : 0;
    const void *k = fs[nn][vec ? 1 : 0][bvi][am];
    void *args[] = {&L};
    hipError_t e = hipLaunchKernel(k, dim3((unsigned)blk), dim3(kGB), args, 0, (hipStream_t)stream);
    if (e == hipSuccess) e = hipGetLastError();
    return e == hipSuccess ? 0 : f110_set_error(F110_E_HIP, std::string(fn) + ": " + hipGetErrorString(e));
}

extern "C" int64_t f110_learner_wgrad_scratch_floats(const f110_wgrad_op *ops, int32_t nops, int32_t M) {
    if (!wgrad_ok(ops, nops, M)) return -1;
    const int S = wgrad_slices(ops, nops, M);
    if (S == 1) return 0;
    int64_t n = 0;
    for (int q = 0; q < nops; ++q) n += (int64_t)S * ((int64_t)ops[q].N * ops[q].KX + ops[q].N);
    return n;
}

static int learner_wgrad(const char *fn, const f110_wgrad_op *ops, int32_t nops, int32_t M, float *scratch,
                         const float *loss_part, int32_t loss_n, float loss_sign, float *loss, void *stream) {
    if (!wgrad_ok(ops, nops, M)) return fail(fn, "bad arguments");
    WgradLaunch L{};
    L.nops = nops;
    L.M = M;
    L.S = wgrad_slices(ops, nops, M);
    if (L.S > 1 && !scratch) return fail(fn, "scratch required");
    L.part = scratch;
    if (loss && (!loss_part || loss_n <= 0)) return fail(fn, "loss partials required");
    L.loss = loss, L.loss_part = loss_part, L.loss_n = loss_n, L.loss_sign = loss_sign;
    int32_t blk = 0;
    int64_t off = 0, total = 0;
    for (int q = 0; q < nops; ++q) {
        const f110_wgrad_op &o = ops[q];
        L.op[q] = o;
        L.vec[q] = o.N % 4 == 0 && o.KX % 4 == 0 && o.ldg % 4 == 0 && o.ldx % 4 == 0 && aligned16(o.G) &&
                   aligned16(o.X) && (!o.gmask || aligned16(o.gmask));
        L.blk0[q] = blk;
        L.poff[q] = off;
        L.ntk[q] = (ops[q].KX + kWK - 1) / kWK;
        const int64_t tiles = (int64_t)((ops[q].N + kWN - 1) / kWN) * L.ntk[q];
        blk += (int32_t)(tiles * L.S);
        const int64_t n_out = (int64_t)ops[q].N * ops[q].KX + ops[q].N;
        off += L.S * n_out;
        total += n_out;
    }
    L.blk0[nops] = blk;
    L.poff[nops] = off;
    for (int q = nops; q < kMaxOps; ++q) L.blk0[q] = blk;
    hipStream_t s = (hipStream_t)stream;
    const bool gm = ops[0].gmask != nullptr;
    const void *kf[2][2] = {  // [final][gmask]
        {reinterpret_cast<const void *>(&k_lwgrad<false, false>), reinterpret_cast<const void *>(&k_lwgrad<false, true>)},
        {reinterpret_cast<const void *>(&k_lwgrad<true, false>), reinterpret_cast<const void *>(&k_lwgrad<true, true>)}};
    void *args[] = {&L};
    {
        hipError_t e = hipLaunchKernel(kf[L.S == 1][gm], dim3((unsigned)blk), dim3(kGB), args, 0, s);
        if (e != hipSuccess) return f110_set_error(F110_E_HIP, std::string(fn) + ": " + hipGetErrorString(e));
    }
    if (L.S > 1 || loss) {  // the partials added (S > 1) and / or the loss (one more block)
        const int64_t outs = L.S > 1 ? total : 0;
        hipLaunchKernelGGL(k_lwgrad_finish, dim3((unsigned)((outs + kGB - 1) / kGB + (loss ? 1 : 0))), dim3(kGB), 0,
                           s, L, outs);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : f110_set_error(F110_E_HIP, std::string(fn) + ": " + hipGetErrorString(e));
}

extern "C" int f110_learner_wgrad(const f110_wgrad_op *ops, int32_t nops, int32_t M, float *scratch, void *stream) {
    return learner_wgrad("f110_learner_wgrad", ops, nops, M, scratch, nullptr, 0, 0.0f, nullptr, stream);
}

extern "C" int f110_learner_wgrad_loss(const f110_wgrad_op *ops, int32_t nops, int32_t M, float *scratch,
                                       const float *loss_part, int32_t n_part, float sign, float *loss, void *stream) {
    if (!loss) return fail("f110_learner_wgrad_loss", "null loss");
    return learner_wgrad("f110_learner_wgrad_loss", ops, nops, M, scratch, loss_part, n_part, sign, loss, stream);
}
