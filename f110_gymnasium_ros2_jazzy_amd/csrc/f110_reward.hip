// f110_reward.hip — the training reward on the device.
//
// rl_training/utils/rewards.py:CenterlineSafetyProgressReward (:185-355)
// with its centerline projector utils/track_progress.py:CenterlineProgress
// (:5-110), which train_ddpg.py:176 evaluates on the host for every
// next_obs.  One wave per env; the per-env state (rewards.py _Prog, :97-107)
// lives in device memory between calls.
//
// Rounding follows the reference: Python float (f64) arithmetic in its
// evaluation order; 2-vector np.dot / np.linalg.norm with the BLAS pattern
// measured for this image (fma(a1, b1, a0*b0)); the wall
// term's np.quantile on float32 data in float32 (the quantile is cast to the
// data dtype; linear method: virtual index (n-1)*q, _lerp in float32).
//
// CenterlineProgress.project_xy asks a cKDTree for the 5 segment midpoints
// nearest to the point and keeps the best orthogonal projection among those
// segments.  Here every lane keeps the 5 nearest of its share of the
// midpoints and a 5-round wave merge yields the global 5 in ascending
// distance (ties: lower index), the order the candidates are then tried in.
#include <hip/hip_runtime.h>

#include "f110_internal.h"

namespace f110 {

namespace {

constexpr int kRwWaves = 1;  // envs per block: one-wave blocks free their slot as the env finishes
static_assert(kRwWaves == 1, "k_reward's kth_pair LDS buffer (pack[64]) is one wave's: size it [kRwWaves][64] first");
constexpr int kTop = 5;      // kd.query(p, k=5)

struct Cand {
    double d2;
    int32_t i;
};

__device__ __forceinline__ bool cand_less(double d2a, int32_t ia, double d2b, int32_t ib) {
    return d2a < d2b || (d2a == d2b && ia < ib);
}

__device__ void merge_top(const Cand (&t)[kTop], int sub, Cand out[kTop]);

// Each half-wave (32 lanes) projects its own point: the ego car's on lanes
// 0-31, the opponent's on 32-63, so the two dependent load chains overlap.
// `sub` is the lane within the half; cross-lane steps stay inside it.
constexpr int kHalf = 32;

// The kTop midpoints nearest to (px, py), ascending; every lane of the half gets the same list.
__device__ void nearest_mids(const double *mid, int32_t M, double px, double py, int sub, Cand out[kTop]) {
    Cand t[kTop];
#pragma unroll
    for (int k = 0; k < kTop; ++k) t[k] = Cand{INFINITY, INT32_MAX};
    for (int32_t m = sub; m < M; m += kHalf) {
        const double dx = mid[2 * m] - px, dy = mid[2 * m + 1] - py;
        const double d2 = dx * dx + dy * dy;  // cKDTree's squared euclidean distance
        if (cand_less(d2, m, t[kTop - 1].d2, t[kTop - 1].i)) {
            Cand c{d2, m};
#pragma unroll
            for (int k = 0; k < kTop; ++k)  // insertion into the sorted list
                if (cand_less(c.d2, c.i, t[k].d2, t[k].i)) {
                    const Cand o = t[k];
                    t[k] = c;
                    c = o;
                }
        }
    }
    merge_top(t, sub, out);
}

// The half-wide kTop smallest of the lanes' sorted lists (every lane gets them).
__device__ void merge_top(const Cand (&t)[kTop], int sub, Cand out[kTop]) {
    int head = 0;
#pragma unroll
    for (int r = 0; r < kTop; ++r) {
        double hd = INFINITY;
        int32_t hi = INT32_MAX;
#pragma unroll
        for (int k = 0; k < kTop; ++k)
            if (k == head) {
                hd = t[k].d2;
                hi = t[k].i;
            }
        double bd = hd;
        int32_t bi = hi;
#pragma unroll
        for (int o = kHalf / 2; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o, 64);
            const int32_t oi = __shfl_xor(bi, o, 64);
            if (cand_less(od, oi, bd, bi)) {
                bd = od;
                bi = oi;
            }
        }
        out[r] = Cand{bd, bi};
        if (hi == bi && bi != INT32_MAX) ++head;  // the winning lane pops its head
    }
}

struct Proj {
    double s, t;
    int32_t seg;  // the segment (or node) s was taken from: seg_at's first guess
};

// np.dot of two 2-vectors / np.linalg.norm of one (OpenBLAS pattern)
__device__ __forceinline__ double bdot(double a0, double a1, double b0, double b1) { return fma(a1, b1, a0 * b0); }

// nearest_mids through the grid: the midpoints of the (2r+1)^2 cells around
// the query, merged as above; the result is final when every midpoint
// outside the block is provably farther than the 5th found one (distance to
// the block's edge, less a margin, above it).  r = 1, then 2, then 4; past
// that the full scan runs.  The same 5 (and order) as the
// full scan.  A grid row's cells are consecutive in cell order, so a block is
// 2r+1 item ranges: their bounds load together, every lane then takes items
// of the concatenated ranges from the cell-ordered midpoint copy.
constexpr int kMaxBlockRows = 9;

__device__ void nearest_mids_grid(const TrackView &T, double px, double py, int sub, Cand out[kTop]) {
    const int32_t M = T.n - 1;
    const double fx = (px - T.gx0) / T.gh, fy = (py - T.gy0) / T.gh;
    bool ok = false;
    // a point off the grid searches from the nearest edge cell: the block's
    // sides on the grid border are clipped (no midpoints beyond them) and
    // the point lies inside every other side, so the bound below still holds
    if (T.cell_start && fx == fx && fy == fy) {
        const int32_t ci = fx < 0.0 ? 0 : (fx >= (double)(T.gnx - 1) ? T.gnx - 1 : (int32_t)fx);
        const int32_t cj = fy < 0.0 ? 0 : (fy >= (double)(T.gny - 1) ? T.gny - 1 : (int32_t)fy);
        for (int32_t r = 1; r <= (kMaxBlockRows - 1) / 2 && !ok; r *= 2) {
            // the block clipped to the grid: a clipped side needs no bound
            const int32_t i0 = ci - r < 0 ? 0 : ci - r, i1 = ci + r >= T.gnx ? T.gnx - 1 : ci + r;
            const int32_t j0 = cj - r < 0 ? 0 : cj - r, j1 = cj + r >= T.gny ? T.gny - 1 : cj + r;
            const int32_t nrow = j1 - j0 + 1;
            int32_t r0[kMaxBlockRows], pre[kMaxBlockRows];
            int32_t K = 0;
#pragma unroll
            for (int t = 0; t < kMaxBlockRows; ++t) {
                r0[t] = 0;
                pre[t] = K;
                if (t < nrow) {
                    const int32_t c = (j0 + t) * T.gnx;
                    r0[t] = T.cell_start[c + i0];
                    K += T.cell_start[c + i1 + 1] - r0[t];
                }
            }
            Cand tp[kTop];
#pragma unroll
            for (int k = 0; k < kTop; ++k) tp[k] = Cand{INFINITY, INT32_MAX};
            for (int32_t j = sub; j < K; j += kHalf) {
                int32_t q = r0[0] + j;
#pragma unroll
                for (int t = 1; t < kMaxBlockRows; ++t)
                    if (t < nrow && j >= pre[t]) q = r0[t] + (j - pre[t]);
                const int32_t m = T.cell_items[q];
                const double dx = T.cell_mid[2 * q] - px, dy = T.cell_mid[2 * q + 1] - py;
                const double d2 = dx * dx + dy * dy;
                if (cand_less(d2, m, tp[kTop - 1].d2, tp[kTop - 1].i)) {
                    Cand cc{d2, m};
#pragma unroll
                    for (int k = 0; k < kTop; ++k)
                        if (cand_less(cc.d2, cc.i, tp[k].d2, tp[k].i)) {
                            const Cand o = tp[k];
                            tp[k] = cc;
                            cc = o;
                        }
                }
            }
            merge_top(tp, sub, out);
            // distance from the query to the block's unclipped edges (a lower
            // bound for every midpoint outside the block), with a margin
            double lb = INFINITY;
            if (ci - r >= 0) lb = fmin(lb, px - (T.gx0 + (double)i0 * T.gh));
            if (ci + r < T.gnx) lb = fmin(lb, T.gx0 + (double)(i1 + 1) * T.gh - px);
            if (cj - r >= 0) lb = fmin(lb, py - (T.gy0 + (double)j0 * T.gh));
            if (cj + r < T.gny) lb = fmin(lb, T.gy0 + (double)(j1 + 1) * T.gh - py);
            const double lbm = lb * (1.0 - 1e-9) - 1e-9;
            ok = out[kTop - 1].i != INT32_MAX && lbm > 0.0 && out[kTop - 1].d2 < lbm * lbm;
        }
    }
    if (!ok) nearest_mids(T.mid, M, px, py, sub, out);  // off the grid or a sparse neighbourhood
}

// CenterlineProgress.project_xy (track_progress.py:58-97)
__device__ Proj project_xy(const TrackView &T, double x, double y, int sub) {
    Cand c[kTop];
    nearest_mids_grid(T, x, y, sub, c);
    bool have = false;
    double bn = 0.0, bs = 0.0, bt = 0.0;
    int32_t bseg = 0;
#pragma unroll
    for (int r = 0; r < kTop; ++r) {
        const int32_t idx = c[r].i;
        if (idx == INT32_MAX) continue;  // fewer than kTop segments
        const double a0 = T.xy[2 * idx], a1 = T.xy[2 * idx + 1];
        const double ab0 = T.xy[2 * idx + 2] - a0, ab1 = T.xy[2 * idx + 3] - a1;
        const double L2 = bdot(ab0, ab1, ab0, ab1);
        if (L2 <= 1e-12) continue;
        const double ap0 = x - a0, ap1 = y - a1;
        double tp = bdot(ap0, ap1, ab0, ab1) / L2;
        tp = tp < 0.0 ? 0.0 : (tp > 1.0 ? 1.0 : tp);  // np.clip (NaN propagates)
        const double pr0 = a0 + tp * ab0, pr1 = a1 + tp * ab1;
        const double s_proj = T.s[idx] + tp * sqrt(L2);
        const double d0 = x - pr0, d1 = y - pr1;
        const double t_signed = bdot(d0, d1, T.nrm[2 * idx], T.nrm[2 * idx + 1]);
        const double nrm = sqrt(bdot(d0, d1, d0, d1));
        if (!have || nrm < bn) {
            have = true;
            bn = nrm;
            bs = s_proj;
            bt = t_signed;
            bseg = idx;
        }
    }
    if (!have) {  // degenerate fallback: nearest node (:93-95)
        double bd = INFINITY;
        int32_t bj = INT32_MAX;
        for (int32_t j = sub; j < T.n; j += kHalf) {
            const double d0 = T.xy[2 * j] - x, d1 = T.xy[2 * j + 1] - y;
            const double d = sqrt(d0 * d0 + d1 * d1);
            if (cand_less(d, j, bd, bj)) {
                bd = d;
                bj = j;
            }
        }
#pragma unroll
        for (int o = kHalf / 2; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o, 64);
            const int32_t oi = __shfl_xor(bj, o, 64);
            if (cand_less(od, oi, bd, bj)) {
                bd = od;
                bj = oi;
            }
        }
        return Proj{T.s[bj], 0.0, bj};
    }
    return Proj{bs, bt, bseg};
}

// np.searchsorted(s, v, side="right") - 1 clipped to [0, n-2] (rewards.py:112-114, :262-264)
// guess: the segment the projection came from; the answer is checked on it
// and its successor (s is non-decreasing: i is the answer iff s[i] <= v and
// s[i+1] > v or i = n-1) before the binary search runs.
__device__ int32_t seg_at(const TrackView &T, double v, int32_t guess) {
    int32_t lo = 0, hi = T.n;  // first index with s[i] > v
    if (guess >= 0 && guess + 1 < T.n) {
        const double s0 = T.s[guess], s1 = T.s[guess + 1];
        const double s2 = guess + 2 < T.n ? T.s[guess + 2] : INFINITY;
        if (s0 <= v && s1 > v) lo = hi = guess + 1;
        else if (s1 <= v && (guess + 2 >= T.n || s2 > v)) lo = hi = guess + 2;
    }
    while (lo < hi) {
        const int32_t m = (lo + hi) >> 1;
        if (T.s[m] > v) hi = m;
        else lo = m + 1;
    }
    int32_t idx = lo - 1;
    idx = idx < 0 ? 0 : idx;
    return idx > T.n - 2 ? T.n - 2 : idx;
}

__device__ __forceinline__ double pymax(double a, double b) { return b > a ? b : a; }  // Python max(a, b)
__device__ __forceinline__ double pymin(double a, double b) { return b < a ? b : a; }  // Python min(a, b)

__device__ __forceinline__ double delta_s(const TrackView &T, double cur, double prev) {  // :99-106
    double ds = cur - prev;
    if (T.closed) {
        if (ds > 0.5 * T.L) ds -= T.L;
        if (ds < -0.5 * T.L) ds += T.L;
    }
    return ds;
}

// wave sum of a per-lane count
__device__ __forceinline__ int32_t wave_count(int32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

constexpr int kRwPerLane = 32;  // n_beams <= 64 * 32 = 2048

constexpr uint32_t kNoValue = 0xFFFFFFFFu;  // empty slot: above every value

// wave-wide count of held values <= x: one compare per slot, whose lane mask
// is counted on the scalar unit (no cross-lane reduction); every lane of the
// wave must be active.  Empty slots hold kNoValue, above every query.
template <int NQ>
__device__ __forceinline__ int32_t wave_count_le(const uint32_t (&v)[NQ], uint32_t x) {
    int32_t c = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) c += __popcll(__ballot(v[q] <= x));
    return c;
}

// k-th smallest (0-based) of the values held across the wave (non-negative
// floats by bit pattern, NQ slots per lane), by bisection on the bit pattern
// in [lo, hi].  (A 4-pass 8-bit radix select over an LDS histogram measured
// slower: the few exponent values put most of a wave's atomics on the same
// bins.)
template <int NQ>
__device__ __forceinline__ uint32_t kth_bits(const uint32_t (&v)[NQ], uint32_t lo, uint32_t hi, int32_t k) {
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (wave_count_le<NQ>(v, mid) >= k + 1) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

template <bool MAX>
__device__ __forceinline__ uint32_t wave_ext(uint32_t m) {  // wave min / max
#pragma unroll
    for (int s2 = 32; s2 > 0; s2 >>= 1) {
        const uint32_t om = __shfl_xor(m, s2, 64);
        m = MAX ? (om > m ? om : m) : (om < m ? om : m);
    }
    return m;
}

// The order statistics k and k + 1 (0-based, k + 1 < B) of the wave's values
// (B real values in [vmin, vmax], kNoValue fillers).  Bisection with every
// slot narrows [lo, hi] while it holds both statistics, until at most 64
// values lie in it; those are packed one per lane through `pack` (64 words of
// LDS) and the bisection goes on over one slot (a compare and a popcount per
// step instead of NQ of each: the counting's scalar popcounts bound the
// NQ-slot steps).  A split that separates the two statistics ends it at once:
// k is the largest value <= mid, k + 1 the smallest above.
template <int NQ>
__device__ __forceinline__ void kth_pair(const uint32_t (&v)[NQ], uint32_t vmin, uint32_t vmax, int32_t B, int32_t k,
                                         int lane, uint32_t *pack, uint32_t &a, uint32_t &b) {
    uint32_t lo = vmin, hi = vmax;
    int32_t clt = 0, cle = B;  // values < lo, values <= hi: clt <= k, cle >= k + 2
    while (cle - clt > 64 && lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        const int32_t c = wave_count_le<NQ>(v, mid);
        if (c >= k + 2) {
            hi = mid;
            cle = c;
        } else if (c <= k) {
            lo = mid + 1;
            clt = c;
        } else {  // c == k + 1
            uint32_t mx = 0u, mn = kNoValue;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                if (v[q] <= mid && v[q] > mx) mx = v[q];
                if (v[q] > mid && v[q] < mn) mn = v[q];
            }
            a = wave_ext<true>(mx);
            b = wave_ext<false>(mn);
            return;
        }
    }
    if (lo == hi) {  // both statistics are this value (more than 64 values hold it)
        a = b = lo;
        return;
    }
    int32_t n = 0;  // the cle - clt values in [lo, hi], one per lane
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const bool in = v[q] >= lo && v[q] <= hi;
        const uint64_t m = __ballot(in);
        if (in) pack[n + (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = v[q];
        n += (int32_t)__popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t w[1] = {lane < n ? pack[lane] : kNoValue};
    const int32_t kk = k - clt;
    a = kth_bits<1>(w, lo, hi, kk);
    if (wave_count_le<1>(w, a) >= kk + 2) {
        b = a;
    } else {
        b = wave_ext<false>(w[0] > a ? w[0] : kNoValue);
    }
}

// The wall term's np.quantile(clip(where(x <= 0 | ~finite, lmax, x), 0, lmax), q)
// in float32 (rewards.py:312-320): q cast to float32, virtual index (n-1)*q,
// numpy's _lerp in float32.  NQ slots of 64 beams per lane (B <= 64 * NQ).
template <int NQ>
__device__ float wall_quantile(const float *o, int B, float lmax, float qf, int lane, uint32_t *pack) {
    uint32_t v[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int b = lane + 64 * q;
        v[q] = kNoValue;
        if (b < B) {
            float x = o[b];
            if (x <= 0.0f || !isfinite(x)) x = lmax;  // np.where(...)
            x = x < 0.0f ? 0.0f : (x > lmax ? lmax : x);  // np.clip
            v[q] = __float_as_uint(x);
        }
    }
    // the answer lies between the smallest and the largest value (kNoValue
    // fillers excluded from the max)
    uint32_t vmin = kNoValue, vmax = 0u;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        vmin = v[q] < vmin ? v[q] : vmin;
        vmax = v[q] != kNoValue && v[q] > vmax ? v[q] : vmax;
    }
#pragma unroll
    for (int s2 = 32; s2 > 0; s2 >>= 1) {
        const uint32_t a = __shfl_xor(vmin, s2, 64), b = __shfl_xor(vmax, s2, 64);
        vmin = a < vmin ? a : vmin;
        vmax = b > vmax ? b : vmax;
    }
    const float vi = (float)(B - 1) * qf;
    if (vi >= (float)(B - 1)) return __uint_as_float(vmax);  // the largest value
    const float pv = floorf(vi < 0.0f ? 0.0f : vi);
    const int32_t k = (int32_t)pv;  // <= B - 2
    const float g = vi - pv;
    uint32_t ab, bb;
    kth_pair<NQ>(v, vmin, vmax, B, k, lane, pack, ab, bb);
    const float fa = __uint_as_float(ab), fb = __uint_as_float(bb);
    const float diff = fb - fa;
    return g >= 0.5f ? fb - diff * (1.0f - g) : fa + diff * g;
}

}  // namespace

__global__ void __launch_bounds__(64 * kRwWaves) k_reward(RewardArgs a) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t e = (int64_t)blockIdx.x * kRwWaves + wave;
    if (e >= a.E) return;  // wave-uniform; no block barriers below
    const f110_reward_params &P = a.p;
    f110_reward_state *S = a.state + e;
    if (a.reset_mask && a.reset_mask[e]) {  // reward_fn.reset(); the reset observation is not rewarded
        if (lane == 0) {
            *S = f110_reward_state{};
            a.rewards[e] = 0.0;
        }
        return;
    }
    const float *o = a.obs + e * (int64_t)a.obs_len;
    const int B = a.B;
    // parse_flat_obs (rewards.py:11-41): float() of the float32 entries, yaw re-wrapped
    const double ex = (double)o[B + 0], ey = (double)o[B + 1];
    const bool ego_col = o[B + 3] != 0.0f;
    const double ox = (double)o[B + 4], oy = (double)o[B + 5];
    const double oth = pymod((double)o[B + 6] + kPi, 2.0 * kPi) - kPi;
    const bool opp_col = o[B + 7] != 0.0f;

    f110_reward_state st = *S;
    st.steps += 1;
    double r;
    if (ego_col) {
        r = -P.ego_crash_penalty;
    } else if (opp_col && P.opp_crash_bonus > 0.0) {
        r = P.opp_crash_bonus;
    } else {
        // ---- progress: _Prog.update (:125-172) or _ProgFallback.update (:73-79)
        double de, dop, s_ego = 0.0, t_ego = 0.0;
        int32_t seg_ego = -1;
        const double xs[2] = {ex, ox}, ys[2] = {ey, oy};
        double dd[2];
        if (P.use_progress) {
            const TrackView &T = a.track;
            Proj pj[2];
            {  // ego on lanes 0-31, opponent on 32-63
                const bool lo_half = lane < kHalf;
                const Proj mine = project_xy(T, lo_half ? ex : ox, lo_half ? ey : oy, lane & (kHalf - 1));
#pragma unroll
                for (int w = 0; w < 2; ++w) {
                    pj[w].s = __shfl(mine.s, w * kHalf, 64);
                    pj[w].t = __shfl(mine.t, w * kHalf, 64);
                    pj[w].seg = __shfl(mine.seg, w * kHalf, 64);
                }
            }
            s_ego = pj[0].s;
            t_ego = pj[0].t;
            seg_ego = pj[0].seg;
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                if (!(st.flags & (1 << w))) {  // init
                    st.s_prev[w] = pj[w].s;
                    st.flags |= 1 << w;
                }
                // _signed_step (:116-138)
                const double ds_geom = delta_s(T, pj[w].s, st.s_prev[w]);
                double ds;
                if (!(st.flags & (4 << w))) {
                    st.px[w] = xs[w];
                    st.py[w] = ys[w];
                    st.flags |= 4 << w;
                    ds = 0.0;
                } else {
                    const double dx = xs[w] - st.px[w], dy = ys[w] - st.py[w];
                    st.px[w] = xs[w];
                    st.py[w] = ys[w];
                    const int32_t idx = seg_at(T, pj[w].s, pj[w].seg);
                    const double ds_sign = dx * T.tan[2 * idx] + dy * T.tan[2 * idx + 1];
                    ds = copysign(fabs(ds_geom), fabs(ds_sign) > 1e-6 ? ds_sign : ds_geom);
                }
                dd[w] = ds;
                st.s_prev[w] = pj[w].s;
            }
            de = dd[0];
            dop = dd[1];
            if (st.auto_n < P.auto_flip_steps) {  // auto-flip on a reversed CSV (:148-154)
                st.auto_sum = st.auto_sum + de;
                st.auto_n += 1;
                if (st.auto_n == P.auto_flip_steps) {
                    const double mean = st.auto_sum / (double)(st.auto_n > 1 ? st.auto_n : 1);
                    if (mean < 0.0) st.flags |= 16;
                }
            }
            const double flip = (st.flags & 16) ? -1.0 : 1.0;
            de *= flip;
            dop *= flip;
            st.cum[0] += de;
            st.cum[1] += dop;
            st.ema = P.beta * st.ema + (1.0 - P.beta) * fabs(de);
            st.t_last[0] = pj[0].t;
            st.t_last[1] = pj[1].t;
        } else {
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                if (!(st.flags & (4 << w))) {
                    st.px[w] = xs[w];
                    st.py[w] = ys[w];
                    st.flags |= 4 << w;
                    dd[w] = 0.0;
                } else {
                    const double dx = xs[w] - st.px[w], dy = ys[w] - st.py[w];
                    st.px[w] = xs[w];
                    st.py[w] = ys[w];
                    dd[w] = sqrt(dx * dx + dy * dy);  // (dx*dx+dy*dy)**0.5
                }
            }
            de = dd[0];
            dop = dd[1];
            st.cum[0] += de;
            st.cum[1] += dop;
            st.ema = P.beta * st.ema + (1.0 - P.beta) * de;
        }
        if (st.steps < 10) de = pymax(0.0, de);
        const double r_prog = P.w_prog * P.forward_sign * de;
        const double r_alive = P.alive_bonus;
        double r_lead = 0.0;
        if (P.w_rel_lead != 0.0 && P.use_progress) {
            double lead = st.cum[0] - st.cum[1];
            lead = lead < -P.lead_clip ? -P.lead_clip : (lead > P.lead_clip ? P.lead_clip : lead);
            r_lead = P.w_rel_lead * (lead / P.lead_clip);
        }
        double r_lat = 0.0;
        if (P.use_progress) {  // lateral penalty (:300-309)
            const TrackView &T = a.track;
            double wR = P.default_half_width, wL = P.default_half_width;
            if (T.wR) {
                const int32_t idx = seg_at(T, s_ego, seg_ego);
                wR = T.wR[idx];
                wL = T.wL[idx];
            }
            const double w_eff = pymax(0.2, t_ego >= 0.0 ? wL : wR);
            const double lat_norm = fabs(t_ego) / w_eff;
            const double lat_term = pymin(lat_norm * lat_norm, P.lat_cap);
            r_lat = -P.w_lat * lat_term;
        }
        double r_wall = 0.0;
        if (B > 0 && st.steps >= P.grace_steps_wall) {  // wall term (:312-320)
            const float lmax = (float)P.lidar_max;
            const float qf = (float)P.wall_quantile;
            __shared__ uint32_t pack[64];  // kth_pair's packed values (one wave per block)
            const float dmin_f = B <= 64 * 17 ? wall_quantile<17>(o, B, lmax, qf, lane, pack)
                                              : wall_quantile<kRwPerLane>(o, B, lmax, qf, lane, pack);
            const double dmin = (double)dmin_f;
            if (dmin < P.near_wall_dist) {
                const double x = (P.near_wall_dist - dmin) / pymax(1e-6, P.near_wall_dist);
                r_wall = -P.w_wall * (x * x);
            }
        }
        double r_opp = 0.0;
        if (st.steps >= P.grace_steps_opp) {  // opponent bubble (:323-330)
            const double rho = hypot(ex - ox, ey - oy);
            if (rho < P.opp_safe_dist) {
                const double y = (P.opp_safe_dist - rho) / pymax(1e-6, P.opp_safe_dist);
                r_opp = -P.w_opp * (y * y);
            }
        }
        double r_flank = 0.0;
        {  // _rot_into_opp_frame + flank window (:64-70, :332-337)
            const double dx = ex - ox, dy = ey - oy;
            double s, c;
            cr_sincos(-oth, s, c);
            const double x_rel = c * dx - s * dy;
            const double y_rel = s * dx + c * dy;
            if (0.2 <= x_rel && x_rel <= 1.8 && 0.25 <= fabs(y_rel) && fabs(y_rel) <= 0.8) {
                const double y_band = pymax(0.0, 0.8 - fabs(fabs(y_rel) - 0.525));
                r_flank = 0.1 * (x_rel / 1.8) * (y_band / 0.8);
            }
        }
        r = r_prog + r_alive + r_lead + r_lat + r_wall + r_opp + r_flank;
    }
    if (lane == 0) {
        *S = st;
        a.rewards[e] = r;
    }
}

hipError_t launch_reward(const RewardArgs &a, hipStream_t s) {
    if (a.E <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_reward, dim3((unsigned)((a.E + kRwWaves - 1) / kRwWaves)), dim3(64 * kRwWaves), 0, s, a);
    return hipGetLastError();
}

}  // namespace f110
