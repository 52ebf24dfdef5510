// f110_replay.hip — prioritized experience replay in HBM.
//
// Replaces rl_training/DDPG/replay_buffer.py:PrioritizedExperienceReplayBuffer
// (the DDPG agent's memory, agent.py:194, :223-237, :254, :337-338).  The
// reference keeps one Python object per transition and samples with an O(N)
// numpy rng.choice on the host every update.  Here the ring of transitions
// lives on the device as flat arrays and every operation is a few kernels:
//
//   add     (replay_buffer.py:48-71)   k_prio_max (per-block max priority)
//           -> k_add_scan (one workgroup: the max, ring slots of the masked
//           rows, their priority) -> k_add_copy (one block per row).
//   sample  (replay_buffer.py:76-116)  Sampling WITHOUT replacement from
//           p_i = (prio_i + eps)^alpha / sum_j (...) by the exponential race
//           (Efraimidis-Spirakis): key_i = E_i / w_i with E_i ~ Exp(1); the B
//           smallest keys in increasing order are distributed exactly like B
//           successive draws without replacement -- the ordered sample that
//           numpy's Generator.choice(replace=False, p=...) returns (it draws,
//           drops repeats in draw order and redraws the rest from the
//           renormalised p).  The B smallest 32-bit key patterns are found by
//           a 4-pass radix select (8-bit digits, LDS histograms; each pass's blocks pick the last digit from its global histogram, the earlier ones from the header); ties at the
//           threshold go to the lowest indices; the selection is compacted in
//           index order (two passes, no sort) and one workgroup computes the
//           IS weights.  As a set the batch has the distribution of the
//           reference's draws; it is returned in index order, not draw order
//           (agent.replay only averages over it).  With fewer stored
//           rows than B (replace=True, :97) one workgroup draws i.i.d. by
//           inverse CDF.
//   update  (replay_buffer.py:121-135) clip, NaN -> 1e-6, scatter.
//
// Everything is ordered on the caller's stream.  The device header holds the
// length and ring pointer, so adds with a row mask (autoreset rows are not
// stored) need no host round trip; kernels of the path not taken (with /
// without replacement) exit at their first instruction.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "f110_internal.h"

namespace f110 {

namespace {

constexpr int kRB = 256;         // threads per block of the streaming kernels
constexpr int kOneBlock = 1024;  // single-workgroup kernels
constexpr int kKB = 1024;        // threads per block of k_keys (4 streaming blocks in one: a quarter of the
                                 // same-address atomics merging the blocks' top-digit histograms)

__device__ __forceinline__ uint32_t f32_bits(float v) { return __float_as_uint(v); }

// numpy: ps + self._eps with ps float32 and a Python float -> float32
// (NEP 50), then np.power(., alpha, dtype=float64) (replay_buffer.py:88).
__device__ __forceinline__ double prio_weight(float p, float eps, double alpha) {
    const float s = p + eps;
    return pow((double)s, alpha);
}

// One row's IS weight before the normalisation (replay_buffer.py:103-108):
// probs[i] = w_i / den, (len * probs[i]) ** -beta.
__device__ __forceinline__ double is_weight(const ReplayView &v, int64_t i, int64_t len, double den, double beta) {
    const double p = v.wt[i] / den;
    return pow((double)len * p, -beta);
}

// p0 of add() (replay_buffer.py:52-63) from the max priority.
__device__ __forceinline__ float add_priority(int64_t length, uint32_t maxbits) {
    double p0 = 1.0;
    if (length > 0) {
        p0 = (double)__uint_as_float(maxbits);
        if (!isfinite(p0) || p0 <= 0.0) p0 = 1.0;
    }
    p0 = p0 < 1e-8 ? 1e-8 : p0;
    p0 = p0 > (double)FLT_MAX ? (double)FLT_MAX : p0;
    return (float)p0;
}

// Deterministic block sum: fixed shuffle tree per wave, waves added in order.
__device__ __forceinline__ double block_sum_f64(double v, double *sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nw = (int)((blockDim.x + 63) >> 6);
    __syncthreads();
    if (lane == 0) sh[wave] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < nw; ++w) t += sh[w];
    return t;  // valid in thread 0
}

// hist[bin] += 1 for every active lane, one LDS atomic per distinct bin of
// the wave: the top digit of the keys falls into a few bins (the exponent's
// high bits), and same-address LDS atomics of a wave serialise lane by lane.
__device__ __forceinline__ void hist_add_wave(uint32_t *hist, uint32_t bin) {
    uint64_t pending = __builtin_amdgcn_read_exec();
    while (pending) {  // wave-uniform: one trip per distinct bin
        const int leader = __builtin_ctzll(pending);
        const uint32_t lb = __builtin_amdgcn_readlane(bin, leader);
        const uint64_t same = __builtin_amdgcn_ballot_w64(bin == lb) & pending;
        if ((int)(threadIdx.x & 63) == leader) atomicAdd(&hist[lb], (uint32_t)__builtin_popcountll(same));
        pending &= ~same;
    }
}

}  // namespace

// ---------------------------------------------------------------- add ------
// np.max(self._buffer["priority"][:self._length]) (replay_buffer.py:54).
// Stored priorities are finite and positive (add and update clamp them), so
// their u32 patterns order like the floats.
__global__ void __launch_bounds__(kRB) k_prio_max(ReplayView v) {
    __shared__ uint32_t wm[kRB / 64];
    const int64_t len = v.hdr->length;
    uint32_t m = 0;
    for (int64_t i = (int64_t)blockIdx.x * kRB + threadIdx.x; i < len; i += (int64_t)gridDim.x * kRB)
        m = max(m, f32_bits(v.prio[i]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {  // one partial per block, reduced by k_add_scan (no hot-spot atomics)
        uint32_t b = wm[0];
        for (int w = 1; w < kRB / 64; ++w) b = max(b, wm[w]);
        v.part[blockIdx.x] = b;
    }
}

// Ring slots of the rows to store (mask[i] != 0, or all) in row order, as the
// reference's one add() per transition (agent.remember) would fill them.
__global__ void __launch_bounds__(kOneBlock) k_add_scan(ReplayView v, const uint8_t *mask, const float *priority,
                                                        int64_t n, int n_part, int mask_skip) {
    __shared__ int64_t part[kOneBlock];
    __shared__ uint32_t wmx[kOneBlock / 64];
    __shared__ uint32_t mx;
    const int t = threadIdx.x;
    {  // the max priority from k_prio_max's partials, spread over the block
        uint32_t m = 0;
        for (int k = t; k < n_part; k += kOneBlock) m = max(m, v.part[k]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
        if ((t & 63) == 0) wmx[t >> 6] = m;
        __syncthreads();
        if (t == 0) {
            uint32_t b = wmx[0];
            for (int w = 1; w < kOneBlock / 64; ++w) b = max(b, wmx[w]);
            mx = b;
        }
    }
    const int64_t chunk = (n + kOneBlock - 1) / kOneBlock;
    const int64_t r0 = min((int64_t)t * chunk, n), r1 = min(r0 + chunk, n);
    int64_t cnt = 0;
    // stored rows: mask[i] != 0, or (mask_skip) mask[i] == 0, or all rows without a mask
    auto keep = [&](int64_t i) { return !mask || ((mask[i] != 0) != (mask_skip != 0)); };
    for (int64_t i = r0; i < r1; ++i) cnt += keep(i) ? 1 : 0;
    part[t] = cnt;
    __syncthreads();
    for (int o = 1; o < kOneBlock; o <<= 1) {  // inclusive scan
        const int64_t add = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += add;
        __syncthreads();
    }
    const int64_t total = part[kOneBlock - 1];
    const int64_t rank = part[t] - cnt;
    const int64_t cap = v.capacity, next = v.hdr->next;
    const float p0 = add_priority(v.hdr->length, mx);
    const double w0 = prio_weight(p0, v.eps, v.alpha);  // every new row's weight without explicit priorities
    int64_t slot = (next + rank) % cap;  // the thread's first ring slot, then consecutive ones
    for (int64_t i = r0; i < r1; ++i) {
        if (keep(i)) {
            v.pos[i] = slot;
            float p = p0;
            if (priority) {  // add(exp, priority): np.clip(p, 1e-8, f32 max).astype(f32) (:59-63)
                const double q = (double)priority[i];
                p = (float)(q < 1e-8 ? 1e-8 : (q > (double)FLT_MAX ? (double)FLT_MAX : q));
            }
            v.prio[slot] = p;  // replay_buffer.py:65
            v.wt[slot] = priority ? prio_weight(p, v.eps, v.alpha) : w0;
            slot = slot + 1 == cap ? 0 : slot + 1;
        } else {
            v.pos[i] = -1;
        }
    }
    __syncthreads();
    if (t == 0) {  // replay_buffer.py:69-71
        const int64_t len = v.hdr->length + total;
        v.hdr->length = len < cap ? len : cap;
        v.hdr->next = (next + total) % cap;
    }
}

// One block per row: the obs / next_obs rows, action, reward and done.
__global__ void __launch_bounds__(kRB) k_add_copy(ReplayView v, ReplayRows in, int64_t n) {
    const int64_t i = blockIdx.x;
    if (i >= n) return;
    const int64_t slot = v.pos[i];
    if (slot < 0) return;
    const int D = v.obs_dim;
    const float *so = in.obs + i * in.obs_stride, *sn = in.next_obs + i * in.next_stride;
    float *dobs = v.obs + slot * D, *dnext = v.next_obs + slot * D;
    if (in.vec4) {  // pairs of float4 per thread: both rows' loads issued before the stores
        const int D4 = D >> 2;
        for (int k0 = threadIdx.x; k0 < D4; k0 += 2 * kRB) {
            const int k1 = k0 + kRB;
            const float4 a0 = reinterpret_cast<const float4 *>(so)[k0];
            const float4 b0 = reinterpret_cast<const float4 *>(sn)[k0];
            float4 a1, b1;
            if (k1 < D4) {
                a1 = reinterpret_cast<const float4 *>(so)[k1];
                b1 = reinterpret_cast<const float4 *>(sn)[k1];
            }
            reinterpret_cast<float4 *>(dobs)[k0] = a0;
            reinterpret_cast<float4 *>(dnext)[k0] = b0;
            if (k1 < D4) {
                reinterpret_cast<float4 *>(dobs)[k1] = a1;
                reinterpret_cast<float4 *>(dnext)[k1] = b1;
            }
        }
    } else {
        for (int k = threadIdx.x; k < D; k += kRB) {
            dobs[k] = so[k];
            dnext[k] = sn[k];
        }
    }
    if (threadIdx.x < v.act_dim) v.act[slot * v.act_dim + threadIdx.x] = in.act[i * in.act_stride + threadIdx.x];
    if (threadIdx.x == 0) {
        v.reward[slot] = in.reward64 ? (float)in.reward64[i] : in.reward[i];
        v.done[slot] = in.done ? (in.done[i] ? 1.0f : 0.0f) : 0.0f;
    }
}

// ------------------------------------------------------------- sample ------
// Pass 0: sampling weights w_i, per-block partial sums of w (den, :88-89),
// exponential-race keys and the top-digit histogram.
// Launched as keys_grid(vgrid) blocks of kKB threads: block b runs the
// kKB / kRB virtual blocks 4b .. 4b+3 of the streaming grid (vgrid blocks of
// kRB threads: the same rows per thread and the same den partials, summed
// per virtual block in wave order, as one kRB block each), with one LDS
// histogram and one set of global atomics per real block.
__global__ void __launch_bounds__(kKB) k_keys(ReplayView v, int32_t batch, int vgrid) {
    constexpr int Q = kKB / kRB;
    __shared__ uint32_t hist[256];
    __shared__ double sh[kKB / 64];
    const int64_t len = v.hdr->length;
    if (len < batch) return;  // block-uniform
    const uint64_t draw = v.hdr->draws;
    const int q = (int)threadIdx.x / kRB, t = (int)threadIdx.x - q * kRB;
    const int vb = (int)blockIdx.x * Q + q;
    if (threadIdx.x < 256) hist[threadIdx.x] = 0;
    __syncthreads();
    double acc = 0.0;
    if (vb < vgrid)
        for (int64_t i = (int64_t)vb * kRB + t; i < len; i += (int64_t)vgrid * kRB) {
            const double w = v.wt[i];  // prio_weight(prio[i]), cached at add / update
            acc += w;
            U4 c = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32), (uint32_t)draw, (uint32_t)(draw >> 32)};
            U4 r = philox(c, (uint32_t)v.seed, (uint32_t)(v.seed >> 32) ^ 0x9E3779B9u);
            const double e = -log(u01_open(r.x, r.y));  // Exp(1)
            const uint32_t key = f32_bits((float)(e / w));
            v.keys[i] = key;
            hist_add_wave(hist, key >> 24);
        }
    // per virtual block: a shuffle tree per wave, its waves added in order (block_sum_f64)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    if ((int)threadIdx.x < Q && (int)blockIdx.x * Q + (int)threadIdx.x < vgrid) {
        double tsum = 0.0;
        for (int w = 0; w < kRB / 64; ++w) tsum += sh[threadIdx.x * (kRB / 64) + w];
        v.den_part[blockIdx.x * Q + threadIdx.x] = tsum;
    }
    if (threadIdx.x < 256 && hist[threadIdx.x])
        atomicAdd(&v.hist[(blockIdx.x % kHistRep) * 4 * 256 + threadIdx.x], hist[threadIdx.x]);
}

// Digit q of the batch-th smallest key from pass q's histogram, given the
// digits before it (prefix) and the rank still to select among the keys that
// share them (kleft): an inclusive scan of the 256 bins (one bin per thread, a
// shuffle scan per wave, the waves' totals added in order); the digit is the
// bin where the running count reaches kleft.  Every block of a consumer
// computes it itself (no one-block select launch between the passes); block
// 0 records the result in the header for the next kernel, so each kernel
// scans one histogram.
__device__ void select_digit(const ReplayView &v, int q, uint32_t &prefix, uint32_t &kleft) {
    __shared__ uint32_t wtot[kRB / 64];
    __shared__ uint32_t res[2];
    const int t = threadIdx.x;  // blockDim.x == 256
    const int lane = t & 63, wave = t >> 6;
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < kHistRep; ++c) x += v.hist[(c * 4 + q) * 256 + t];
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
        inc += lane >= o ? y : 0u;
    }
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    for (int w = 0; w < wave; ++w) inc += wtot[w];
    const uint32_t below = inc - x;
    if (inc >= kleft && below < kleft) {
        res[0] = prefix | ((uint32_t)t << (24 - 8 * q));
        res[1] = kleft - below;
    }
    __syncthreads();
    prefix = res[0];
    kleft = res[1];
    if (blockIdx.x == 0 && t == 0) {
        v.hdr->sel_prefix[q] = prefix;
        v.hdr->sel_kleft[q] = kleft;
    }
}

// The select through digit q - 1, as the previous kernel recorded it (q = 0: none yet).
__device__ __forceinline__ void select_so_far(const ReplayView &v, int32_t batch, int q, uint32_t &prefix,
                                              uint32_t &kleft) {
    prefix = q > 0 ? v.hdr->sel_prefix[q - 1] : 0u;
    kleft = q > 0 ? v.hdr->sel_kleft[q - 1] : (uint32_t)batch;
}

// Passes 1..3: histogram of digit `pass` over the keys whose higher digits
// equal the prefix selected so far.
__global__ void __launch_bounds__(kRB) k_hist(ReplayView v, int32_t batch, int pass) {
    __shared__ uint32_t hist[256];
    const int64_t len = v.hdr->length;
    if (len < batch) return;
    const int shift = 24 - 8 * pass;
    uint32_t prefix, kleft;
    select_so_far(v, batch, pass - 1, prefix, kleft);
    select_digit(v, pass - 1, prefix, kleft);
    const uint32_t want = prefix >> (shift + 8);
    hist[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * kRB + threadIdx.x; i < len; i += (int64_t)gridDim.x * kRB) {
        const uint32_t key = v.keys[i];
        if ((key >> (shift + 8)) == want) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (hist[threadIdx.x])
        atomicAdd(&v.hist[((blockIdx.x % kHistRep) * 4 + pass) * 256 + threadIdx.x], hist[threadIdx.x]);
}

// The selection: every key below the threshold key T, plus the lowest-index
// kleft of the keys equal to T (tie list).  It is written in INDEX order
// (deterministic, no sort): block b owns the contiguous index range
// [b*chunk, (b+1)*chunk); k_count counts its keys below T (and lists the
// ties), k_place writes them at the sum of the preceding blocks' counts.
__device__ __forceinline__ int64_t block_chunk(int64_t len) {
    return (len + gridDim.x - 1) / gridDim.x;
}

__global__ void __launch_bounds__(kRB) k_count(ReplayView v, int32_t batch, int n_part) {
    __shared__ uint32_t wc[kRB / 64];
    __shared__ double sh[kRB / 64];
    const int64_t len = v.hdr->length;
    if (len < batch) return;
    uint32_t T, kleft;
    select_so_far(v, batch, 3, T, kleft);
    select_digit(v, 3, T, kleft);
    if (blockIdx.x == 0) {  // for k_place / k_finish: the threshold, and den (k_keys' partials, fixed order)
        double acc = 0.0;
        for (int k = threadIdx.x; k < n_part; k += kRB) acc += v.den_part[k];
        const double den = block_sum_f64(acc, sh);
        if (threadIdx.x == 0) {
            v.hdr->prefix = T;
            v.hdr->kleft = kleft;
            v.hdr->den = den;
        }
    }
    const int64_t chunk = block_chunk(len);
    const int64_t i0 = (int64_t)blockIdx.x * chunk, i1 = min(i0 + chunk, len);
    uint32_t c = 0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += kRB) {
        const uint32_t key = v.keys[i];
        c += key < T ? 1u : 0u;
        if (key == T) {
            const uint32_t s = atomicAdd(&v.hdr->n_tie, 1u);  // rare
            if (s < (uint32_t)kTieCap) v.tie[s] = (uint32_t)i;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) v.part[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

__global__ void __launch_bounds__(kRB) k_place(ReplayView v, int32_t batch) {
    __shared__ uint32_t base, wsum[kRB / 64];
    const int64_t len = v.hdr->length;
    if (len < batch) return;
    const uint32_t T = v.hdr->prefix;
    // the four passes' histograms (all copies), consumed: zero for the next sample
    for (int k = (int)blockIdx.x * kRB + (int)threadIdx.x; k < kHistRep * 4 * 256; k += (int)gridDim.x * kRB)
        v.hist[k] = 0u;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    {  // this block's offset: the counts of the blocks before it
        uint32_t acc = 0;
        for (int k = t; k < (int)blockIdx.x; k += kRB) acc += v.part[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
        if (lane == 0) wsum[wave] = acc;
        __syncthreads();
        if (t == 0) base = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
    const int64_t chunk = block_chunk(len);
    const int64_t i0 = (int64_t)blockIdx.x * chunk, i1 = min(i0 + chunk, len);
    uint32_t off = base;
    for (int64_t j0 = i0; j0 < i1; j0 += kRB) {  // tiles of kRB indices, in order
        const int64_t i = j0 + t;
        const bool sel = i < i1 && v.keys[i] < T;
        const uint64_t bal = __builtin_amdgcn_ballot_w64(sel);
        const uint32_t before = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        __syncthreads();
        if (lane == 0) wsum[wave] = (uint32_t)__builtin_popcountll(bal);
        __syncthreads();
        uint32_t pre = 0;
        for (int w = 0; w < wave; ++w) pre += wsum[w];
        if (sel) {
            const uint32_t s = off + pre + before;
            if (s < (uint32_t)batch) v.sel[s] = (uint64_t)i;
        }
        off += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    }
    if (blockIdx.x == gridDim.x - 1 && t == 0) v.hdr->n_lt = off;  // total below T
}

// IS weights (replay_buffer.py:103-113) of the selected rows: wsh[j] holds
// row idx[j]'s weight before the normalisation (is_weight); divided by their
// max (:109-112) into w_out.
__device__ void normalize_weights(const int64_t *idx, int32_t batch, const double *wsh, int64_t *idx_out,
                                  float *w_out) {
    __shared__ double wm[kOneBlock / 64];
    double m = -INFINITY;
    for (int j = threadIdx.x; j < batch; j += blockDim.x) m = fmax(m, wsh[j]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    double mx = wm[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) mx = fmax(mx, wm[w]);
    const bool ok = isfinite(mx) && mx > 0.0;  // :109-112
    for (int j = threadIdx.x; j < batch; j += blockDim.x) {
        idx_out[j] = idx[j];
        w_out[j] = ok ? (float)(wsh[j] / mx) : 1.0f;
    }
}

// Without replacement: merge the chosen ties (the lowest-index `need` keys
// equal to T) into the index-ordered selection; weights.
__global__ void __launch_bounds__(kOneBlock) k_finish(ReplayView v, int32_t batch, double beta, int64_t *idx_out,
                                                      float *w_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t len = v.hdr->length;
    if (len < batch) return;
    int64_t *idx = reinterpret_cast<int64_t *>(smem);     // [batch]
    double *wsh = reinterpret_cast<double *>(idx + batch);  // [batch]
    __shared__ uint32_t chosen[64];
    __shared__ uint32_t n_ch;
    const uint32_t n_lt = min(v.hdr->n_lt, (uint32_t)batch);
    const uint32_t n_tie = min(v.hdr->n_tie, (uint32_t)kTieCap);
    const uint32_t need = (uint32_t)batch - n_lt;
    if (threadIdx.x == 0) n_ch = 0;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < n_tie; t += blockDim.x) {  // rank among the ties by index
        const uint32_t mine = v.tie[t];
        uint32_t rank = 0;
        for (uint32_t u = 0; u < n_tie; ++u) rank += v.tie[u] < mine ? 1u : 0u;
        if (rank < need) {
            if (rank < 64) chosen[rank] = mine;
            atomicAdd(&n_ch, 1u);
        }
    }
    __syncthreads();
    const uint32_t nc = min(n_ch, 64u);  // kTieCap ties, of which need (typically 1) are taken
    for (uint32_t j = threadIdx.x; j < n_lt; j += blockDim.x) {  // main rows shift past smaller ties
        const uint64_t i = v.sel[j];
        uint32_t k = 0;
        for (uint32_t c = 0; c < nc; ++c) k += chosen[c] < i ? 1u : 0u;
        idx[j + k] = (int64_t)i;
    }
    for (uint32_t c = threadIdx.x; c < nc; c += blockDim.x) {  // ties after the smaller main rows
        const uint32_t ti = chosen[c];
        uint32_t lo = 0, hi = n_lt;  // first main row with index > ti
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (v.sel[mid] < ti) lo = mid + 1;
            else hi = mid;
        }
        idx[lo + c] = (int64_t)ti;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < batch; j += blockDim.x) wsh[j] = is_weight(v, idx[j], len, v.hdr->den, beta);
    normalize_weights(idx, batch, wsh, idx_out, w_out);
    if (threadIdx.x == 0) {
        v.hdr->draws += 1;
        v.hdr->replace = 0;
        if (v.hdr->n_tie > (uint32_t)kTieCap || n_ch > 64u) v.hdr->overflow += 1;
        v.hdr->n_tie = 0;  // consumed: zero for the next sample
    }
}

// With replacement (0 < len < batch, replay_buffer.py:97): i.i.d. draws by
// inverse CDF (numpy: cdf = cumsum(p), searchsorted(cdf, u, 'right')).
__global__ void __launch_bounds__(kOneBlock) k_sample_replace(ReplayView v, int32_t batch, double beta,
                                                              int64_t *idx_out, float *w_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t len = v.hdr->length;
    if (len >= batch || len <= 0) return;
    double *cdf = reinterpret_cast<double *>(smem);  // [batch] (len < batch)
    int64_t *idx = reinterpret_cast<int64_t *>(cdf + batch);
    double *wsh = reinterpret_cast<double *>(idx + batch);
    for (int64_t i = threadIdx.x; i < len; i += blockDim.x) cdf[i] = v.wt[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        double acc = 0.0;
        for (int64_t i = 0; i < len; ++i) {
            acc += cdf[i];
            cdf[i] = acc;
        }
    }
    __syncthreads();
    const double den = cdf[len - 1];
    const uint64_t draw = v.hdr->draws;
    for (int j = threadIdx.x; j < batch; j += blockDim.x) {
        U4 c = {(uint32_t)j, 0x7E11u, (uint32_t)draw, (uint32_t)(draw >> 32)};
        U4 r = philox(c, (uint32_t)v.seed, (uint32_t)(v.seed >> 32) ^ 0x9E3779B9u);
        const double u = (u01_open(r.x, r.y) - 0x1p-53) * den;  // [0, den)
        int64_t lo = 0, hi = len - 1;  // first i with cdf[i] > u
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (cdf[mid] > u) hi = mid;
            else lo = mid + 1;
        }
        idx[j] = lo;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < batch; j += blockDim.x) wsh[j] = is_weight(v, idx[j], len, den, beta);
    normalize_weights(idx, batch, wsh, idx_out, w_out);
    if (threadIdx.x == 0) {
        v.hdr->draws += 1;
        v.hdr->replace = 1;
    }
}

// One block per sampled row: the arrays agent.replay stacks (agent.py:257-270).
__global__ void __launch_bounds__(kRB) k_gather(ReplayView v, int32_t batch, const int64_t *idx, ReplayBatch out) {
    const int j = blockIdx.x;
    if (j >= batch || v.hdr->length <= 0) return;
    const int64_t i = idx[j];
    const int D = v.obs_dim;
    const float *so = v.obs + i * D, *sn = v.next_obs + i * D;
    float *dobs = out.obs + (int64_t)j * D, *dnext = out.next_obs + (int64_t)j * D;
    if (out.vec4) {  // pairs of float4 per thread: both rows' loads issued before the stores
        const int D4 = D >> 2;
        for (int k0 = threadIdx.x; k0 < D4; k0 += 2 * kRB) {
            const int k1 = k0 + kRB;
            const float4 a0 = reinterpret_cast<const float4 *>(so)[k0];
            const float4 b0 = reinterpret_cast<const float4 *>(sn)[k0];
            float4 a1, b1;
            if (k1 < D4) {
                a1 = reinterpret_cast<const float4 *>(so)[k1];
                b1 = reinterpret_cast<const float4 *>(sn)[k1];
            }
            reinterpret_cast<float4 *>(dobs)[k0] = a0;
            reinterpret_cast<float4 *>(dnext)[k0] = b0;
            if (k1 < D4) {
                reinterpret_cast<float4 *>(dobs)[k1] = a1;
                reinterpret_cast<float4 *>(dnext)[k1] = b1;
            }
        }
    } else {
        for (int k = threadIdx.x; k < D; k += kRB) {
            dobs[k] = so[k];
            dnext[k] = sn[k];
        }
    }
    if (threadIdx.x < v.act_dim) out.act[(int64_t)j * v.act_dim + threadIdx.x] = v.act[i * v.act_dim + threadIdx.x];
    if (threadIdx.x == 0) {
        out.reward[j] = v.reward[i];
        out.done[j] = v.done[i];
    }
}

// ------------------------------------------------------------- update ------
// update_priorities (replay_buffer.py:121-135).  from_td: the values are TD
// errors and the priority is agent.replay's |td| + priority_epsilon in
// float32 (agent.py:337); otherwise they are the priorities themselves.
// Indices of a without-replacement sample are distinct and scatter in
// parallel; after a with-replacement sample (or serial != 0) one thread
// applies them in order, so a repeated index keeps its last value like
// numpy's fancy assignment.
__global__ void __launch_bounds__(kRB) k_update(ReplayView v, const int64_t *idx, const float *val, int64_t n,
                                                float add_eps, int32_t from_td, int32_t serial) {
    auto pr_of = [&](int64_t j) -> float {
        float p = from_td ? fabsf(val[j]) + add_eps : val[j];
        if (p < 1e-8f) p = 1e-8f;         // np.clip(pr, 1e-8, f32max): NaN passes
        else if (p > FLT_MAX) p = FLT_MAX;
        if (!isfinite(p)) p = 1e-6f;      // :131-133
        return p;
    };
    if (serial || v.hdr->replace) {
        if (blockIdx.x == 0 && threadIdx.x == 0)
            for (int64_t j = 0; j < n; ++j) {
                const int64_t i = idx[j];
                if (i >= 0 && i < v.capacity) {
                    const float p = pr_of(j);
                    v.prio[i] = p;
                    v.wt[i] = prio_weight(p, v.eps, v.alpha);
                }
            }
        return;
    }
    for (int64_t j = (int64_t)blockIdx.x * kRB + threadIdx.x; j < n; j += (int64_t)gridDim.x * kRB) {
        const int64_t i = idx[j];
        if (i >= 0 && i < v.capacity) {
            const float p = pr_of(j);
            v.prio[i] = p;
            v.wt[i] = prio_weight(p, v.eps, v.alpha);
        }
    }
}

// ------------------------------------------------------------ launchers ----
int replay_grid(int64_t capacity) {
    const int64_t per = (int64_t)kRB * 4;  // ~4 items per thread
    int64_t g = (capacity + per - 1) / per;
    return (int)(g < 1 ? 1 : (g > kReplayMaxGrid ? kReplayMaxGrid : g));
}

// k_keys's blocks for a streaming grid of `grid` blocks
int keys_grid(int grid) { return (grid + kKB / kRB - 1) / (kKB / kRB); }

size_t replay_finish_lds(int32_t batch) { return (size_t)batch * 16; }

size_t replay_replace_lds(int32_t batch) { return (size_t)batch * 24; }

hipError_t launch_replay_add_index(const ReplayView &v, const uint8_t *mask, int mask_skip, const float *priority,
                                   int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int grid = replay_grid(v.capacity);
    hipLaunchKernelGGL(k_prio_max, dim3(grid), dim3(kRB), 0, s, v);
    hipLaunchKernelGGL(k_add_scan, dim3(1), dim3(kOneBlock), 0, s, v, mask, priority, n, grid, mask_skip);
    return hipGetLastError();
}

hipError_t launch_replay_add_copy(const ReplayView &v, const ReplayRows &in, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_add_copy, dim3((unsigned)n), dim3(kRB), 0, s, v, in, n);
    return hipGetLastError();
}

hipError_t launch_replay_select(const ReplayView &v, int32_t batch, double beta, int64_t *idx, float *w,
                                bool known_full, hipStream_t s) {
    const int grid = replay_grid(v.capacity);
    // histograms and tie count are cleared by k_place / k_finish of the previous sample
    // (and at create), so a sample is kernels only
    hipLaunchKernelGGL(k_keys, dim3(keys_grid(grid)), dim3(kKB), 0, s, v, batch, grid);
    for (int pass = 1; pass < 4; ++pass)  // each block selects the digits so far from the histograms itself
        hipLaunchKernelGGL(k_hist, dim3(grid), dim3(kRB), 0, s, v, batch, pass);
    hipLaunchKernelGGL(k_count, dim3(grid), dim3(kRB), 0, s, v, batch, grid);
    hipLaunchKernelGGL(k_place, dim3(grid), dim3(kRB), 0, s, v, batch);
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(kOneBlock), replay_finish_lds(batch), s, v, batch, beta, idx, w);
    if (!known_full)  // (f110_replay_length has seen length >= batch: the with-replacement path cannot run)
        hipLaunchKernelGGL(k_sample_replace, dim3(1), dim3(kOneBlock), replay_replace_lds(batch), s, v, batch, beta,
                           idx, w);
    return hipGetLastError();
}

hipError_t launch_replay_gather(const ReplayView &v, int32_t batch, const int64_t *idx, const ReplayBatch &out,
                                hipStream_t s) {
    if (out.obs) hipLaunchKernelGGL(k_gather, dim3((unsigned)batch), dim3(kRB), 0, s, v, batch, idx, out);
    return hipGetLastError();
}

hipError_t launch_replay_update(const ReplayView &v, const int64_t *idx, const float *val, int64_t n, float add_eps,
                                int32_t from_td, int32_t serial, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t g = (n + kRB - 1) / kRB;
    g = g > 1024 ? 1024 : g;
    hipLaunchKernelGGL(k_update, dim3((unsigned)g), dim3(kRB), 0, s, v, idx, val, n, add_eps, from_td, serial);
    return hipGetLastError();
}

hipError_t prepare_replay(int32_t max_batch) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_finish),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)replay_finish_lds(max_batch));
    if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_sample_replace),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)replay_replace_lds(max_batch));
    return e;
}

}  // namespace f110
