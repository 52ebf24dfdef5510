// f110_kernels.hip — gfx950 kernels of the batched F1TENTH step.
//
// One f110_step = three launches on the caller's stream:
//
//  k_agents    one thread per car: reset/autoreset, RaceCar.update_pose
//              (steer delay, pid, RK4 of vehicle_dynamics_st, clamps), scan
//              pose, first EDT lookup, and the car's beam-index runs.
//  k_rays_*    the lidar rays: the EDT sphere-trace of ScanSimulator2D
//              (trace_ray), scan noise, TTC test, obs / scan outputs.  The
//              hot kernel: ~7 dependent fp64 gathers per ray.  k_rays_fx /
//              k_rays_fxn / k_rays_fxs on axis-aligned maps (fixed-point cell
//              index, chosen by car count, launch_env_step), k_rays_tiled on
//              rotated ones.
//  k_post_*    one thread per env (single agent) or two waves per env
//              (k_post_multi: GJK, agent ray_cast): TTC response, obs
//              packing, _check_done.
//
//  k_scan_batch / k_dynamics / k_collision_*: the C-ABI building blocks
//  (f110_scan_batch, f110_dynamics_batch, f110_collision_batch).
//  Measured-slower variants live in git history and DESIGN.md, not here.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>

#include "f110_internal.h"

namespace f110 {

constexpr int kBlock = kRayBlock;

static_assert(sizeof(BeamRun) == 24, "BeamRun layout");

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One (lookups, rays) atomic pair per wave into a per-block slot.  n = lookups
// of this lane's rays (0 for a lane without rays), rays = rays per busy lane.
__device__ __forceinline__ void count_rays(unsigned long long *ctr, uint32_t n, uint32_t rays = 1) {
    uint32_t tot = wave_sum(n);
    uint32_t cnt = wave_sum(n ? rays : 0u);
    if ((threadIdx.x & 63) == 0 && cnt) {
        unsigned long long *slot = ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
        atomicAdd(slot, (unsigned long long)tot);
        atomicAdd(slot + 1, (unsigned long long)cnt);
    }
}

// floats between obs rows: f110_outputs.obs_stride, or packed B + 4A
__host__ __device__ __forceinline__ int64_t obs_row(const StepArgs &a) {
    return a.out.obs_stride ? a.out.obs_stride : (int64_t)a.B + 4 * a.A;
}

// F110Env._pack_flat_obs's scan entry (f110_env.py:557-560): f32, NaN ->
// lidar_max, +-inf -> lidar_max / 0, clip, / lidar_max in f32.
__device__ __forceinline__ float obs_scan_value(double r, float lmax) {
    float v = (float)r;
    if (v != v) v = lmax;
    else if (isinf(v)) v = v > 0 ? lmax : 0.0f;
    v = v < 0.0f ? 0.0f : (v > lmax ? lmax : v);
    return v / lmax;
}

// check_ttc_jit's per-beam test (laser_models.py:188-217):
//   ttc = (range - side) / proj_vel;  hit = ttc < thresh && ttc >= 0.
// The f64 divide only runs for beams that can fire: with num = range - side
// > 0 and num >= fl(1.2 * thresh * |proj_vel|), |num / proj_vel| >= 1.2 *
// thresh * (1 - 2^-53) > thresh, so the reference's test is false whatever
// the quotient rounds to.  Every other beam takes the exact divide.
__device__ __forceinline__ bool ttc_fires(double range, double side, double proj_vel, double thresh) {
    const double num = range - side;
    if (num > 0.0 && num >= (1.2 * thresh) * fabs(proj_vel)) return false;
    const double ttc = num / proj_vel;
    return ttc < thresh && ttc >= 0.0;
}

// ttc_fires' first test passed for EVERY beam of the car: with side <= side_max
// and |v beam_cos| <= |v| (rounding is monotonic), range - side_max > 0 and
// >= (1.2 thresh) |v| make it return false whatever the beam.  The caller
// loads (side, beam_cos) only for the lanes (and waves) where this is true.
__device__ __forceinline__ bool ttc_may_fire_lane(double range, double side_max, double v, double thresh) {
    const double nm = range - side_max;
    return !(nm > 0.0 && nm >= (1.2 * thresh) * fabs(v));
}


// ------------------------------------------------------------------------
// k_agents: one thread per car.
// Heavy-first ray dispatch: the (car, chunk) waves whose longest ray took at
// least heavy_T lookups in the previous ray launch are listed (up to
// heavy_cap) for the leading blocks of this step's chunked ray kernel, so the
// rare long waves (grazing beams, up to ~400 lookups) start first instead of
// extending the launch's tail.  One atomic per wave of cars.
__device__ __forceinline__ void build_heavy_list(const StepArgs &a, int g, bool valid) {
    uint32_t hm = 0;
    int h = 0;
    if (valid) {
        const uint8_t *wc = a.wcost + (size_t)g * a.ray_nch;
        for (int k = 0; k < a.ray_nch; ++k)
            if (wc[k] >= a.heavy_T) {
                hm |= 1u << k;
                ++h;
            }
    }
    const int lane = threadIdx.x & 63;
    int incl = h;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int up = __shfl_up(incl, o, 64);
        if (lane >= o) incl += up;
    }
    const int total = __shfl(incl, 63, 64);
    uint32_t base = 0;
    if (lane == 63 && total > 0) base = atomicAdd(a.heavy_count + a.parity, (uint32_t)total);
    base = __shfl(base, 63, 64);
    uint32_t pos = base + (uint32_t)(incl - h), keep = 0;
    uint32_t *list = a.heavy_list + (size_t)a.parity * a.heavy_cap;
    for (uint32_t m = hm; m; m &= m - 1) {
        const int k = __builtin_ctz(m);
        if (pos < (uint32_t)a.heavy_cap) {
            list[pos] = ((uint32_t)g << 8) | (uint32_t)k;
            keep |= 1u << k;
        }
        ++pos;
    }
    if (valid) a.heavy_mask[g] = keep;
}

// The next step's heavy list starts empty (its counter is the other parity).
__device__ __forceinline__ void reset_next_heavy(const StepArgs &a) {
    if (a.heavy_count && blockIdx.x == 0 && threadIdx.x == 0) a.heavy_count[a.parity ^ 1] = 0;
}

__device__ __forceinline__ float bearing_f32(float y, float x) {  // atan2(y, x) within ~2e-4 rad (finite x, y)
    const float ax = fabsf(x), ay = fabsf(y);
    const float a = __fdividef(fminf(ax, ay), fmaxf(ax, ay));
    const float s = a * a;
    float r = ((-0.0464964749f * s + 0.15931422f) * s - 0.327622764f) * s * a + a;
    if (ay > ax) r = 1.57079637f - r;
    if (x < 0.0f) r = 3.14159274f - r;
    if (y < 0.0f) r = -r;
    return (ax == 0.0f && ay == 0.0f) ? 0.0f : r;
}

// The 64-beam chunks of car g whose f64 scans k_post_multi may read (bit k: chunk k), for the ray
// kernel's hand-off: its agent ray_cast visits only beams of each (car, opponent) pair's blocked
// view [lo, hi] -- the nearest beams of the opponent box's vertex bearings
// (get_blocked_view_indices, laser_models.py:282-315) -- seen from the car's yaw or, after a TTC
// response, from yaw 0 (base_classes.py:246-249).  Here in f32 (the box from fast sin / cos, the
// bearings from a polynomial atan2 good to ~2e-4 rad: errors far below a beam's 4.4e-3 rad for
// vertices beyond the 1 cm cutoff while |x|, |y| < 1 km (f32 position rounding ulp(coord) / 1 cm
// stays under a beam there; f110_create keeps no mask for a map that reaches beyond), the
// range widened by 3 beams; a bearing within 1e-2 rad of the +-pi wrap, a vertex within 1 cm of the
// car, or a NaN, marks every chunk.  The other chunks skip the hand-off store (its stores cost the
// two-agent ray launch ~6 %).  The poses of an env's cars meet in LDS: A divides 64 (the context
// allocates no mask otherwise).
// sx / sy / sth: the block's cars' poses (LDS, k_agents writes them before a barrier).
__device__ void handoff_chunks(const StepArgs &a, int g, const float *sx, const float *sy, const float *sth,
                               float len, float wid) {
    const int t = (int)threadIdx.x;
    const int A = a.A, B = a.B;
    const int ag = g % A, t0 = t - ag;  // the env's first car in the block
    const int nch = (B + 63) >> 6;
    const uint32_t all = nch >= 32 ? 0xFFFFFFFFu : ((1u << nch) - 1u);
    const float half_fov = (float)(a.fov * 0.5), inv_incr = (float)(1.0 / a.beam_incr);
    const float xi = sx[t], yi = sy[t];
    uint32_t m = nch > 32 ? all : 0u;
    for (int j = 0; j < A && m != all; ++j) {
        if (j == ag) continue;
        float sj, cj;
        __sincosf(sth[t0 + j], &sj, &cj);
        const float px[4] = {-len / 2, -len / 2, len / 2, len / 2};
        const float py[4] = {wid / 2, -wid / 2, -wid / 2, wid / 2};
        float bear[4];
        bool unsure = !(sth[t] == sth[t]);
        for (int q = 0; q < 4; ++q) {
            const float vx = cj * px[q] - sj * py[q] + sx[t0 + j], vy = sj * px[q] + cj * py[q] + sy[t0 + j];
            const float dx = vx - xi, dy = vy - yi;
            // NaN / inf, or a vertex within 1 cm of the car (its f32 bearing is not reliable there; the
            // reference's is NaN at distance 0: beam 0)
            unsure |= !(dx == dx) || !(dy == dy) || fabsf(dx) > 1e30f || fabsf(dy) > 1e30f ||
                      fabsf(dx) + fabsf(dy) < 0.01f;
            bear[q] = bearing_f32(dy, dx);
        }
        for (int w = 0; w < 2 && !unsure; ++w) {
            const float ego = w == 0 ? sth[t] : 0.0f;
            int lo = B, hi = -1;
            for (int q = 0; q < 4; ++q) {
                float ang = ego - bear[q];
                unsure |= !(fabsf(fabsf(ang) - 3.14159265f) > 1e-2f);
                if (ang > 3.14159265f) ang -= 6.28318531f;
                else if (ang < -3.14159265f) ang += 6.28318531f;
                const float gk = (half_fov - ang) * inv_incr;
                const int k = gk < 0.0f ? 0 : (gk > (float)(B - 1) ? B - 1 : (int)(gk + 0.5f));
                lo = k < lo ? k : lo;
                hi = k > hi ? k : hi;
            }
            lo = lo - 3 < 0 ? 0 : lo - 3;
            hi = hi + 3 > B - 1 ? B - 1 : hi + 3;
            m |= (2u << (hi >> 6)) - (1u << (lo >> 6));  // chunks lo / 64 .. hi / 64 (hi / 64 <= 31)
        }
        if (unsure) m = all;
    }
    a.hmask[g] = (a.hcheck & 4) ? 0u : m;  // f110_debug_set_handoff_check bit 2: a forced miss
}

// HMASK: the context keeps hand-off chunk masks (A >= 2 dividing 64): the block's new poses meet in
// LDS after the update and each car's mask is written at the end; without it the update's stores
// follow it directly (the single-agent form, one dependent chain less to schedule around a barrier).
template <bool HMASK>
__global__ void __launch_bounds__(64) k_agents(StepArgs a) {
    const int g = blockIdx.x * 64 + threadIdx.x;
    const int EA = a.E * a.A;
    const bool valid = g < EA;
    const int A = a.A;
    const int e = valid ? g / A : 0;
    const int ag = valid ? g - e * A : 0;  // padding threads: agent 0 (a.pa holds A entries)
    // Every input of the car is loaded first, before the heavy-list atomic
    // and before anything waits: one memory round trip for the whole prologue.
    double s[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    double b0 = 0.0, b1 = 0.0, raw_steer = 0.0, vel = 0.0;
    int cnt = 0, gate = 0;
    uint32_t episode = 0;
    uint64_t nstep = 0;
    if (valid) {
        if (ag == 0) nstep = a.nstep[e];
#pragma unroll
        for (int k = 0; k < 7; ++k) s[k] = a.st[(size_t)k * EA + g];
        b0 = a.sb[g];
        b1 = a.sb[EA + g];
        cnt = a.scnt[g];
        if (a.mode == 1) {
            gate = a.reset_mask ? a.reset_mask[e] : 1;
        } else {
            gate = a.autoreset ? a.pending[e] : 0;
            episode = a.episode[e];
            if (a.actions_f64) {
                raw_steer = a.actions_f64[(size_t)g * 2];
                vel = a.actions_f64[(size_t)g * 2 + 1];
            } else {
                raw_steer = (double)a.actions[(size_t)g * 2];
                vel = (double)a.actions[(size_t)g * 2 + 1];
            }
        }
    }
    // RaceCar ag's box (its opponents' vertices for the hand-off mask), loaded with the prologue
    const float box_len = HMASK ? (float)a.pa[ag].length : 0.0f, box_wid = HMASK ? (float)a.pa[ag].width : 0.0f;
    if (a.heavy_build) build_heavy_list(a, g, valid);  // block-uniform branch, before any return
    // an LDS copy of cr_sincos's table (sin / cos of i/64): every sincos of the car's update reads it
    // there (a short dependent load instead of a trip to L1 / L2); the loads go out with the prologue's
    __shared__ double sct[256];  // F110_SINCOS_TAB_N x 4 doubles, padded to 4 per thread
    {
        static_assert(F110_SINCOS_TAB_N * 4 <= 256, "the LDS copy holds the table");
        constexpr int NT = F110_SINCOS_TAB_N * 4;
        const double *src = &kSinCosTab[0][0];
        double v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = (int)threadIdx.x + 64 * i;
            v[i] = src[k < NT ? k : NT - 1];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) sct[threadIdx.x + 64 * i] = v[i];
        __syncthreads();
    }
    const double(*tab)[4] = reinterpret_cast<const double(*)[4]>(sct);
#ifdef F110_AGENTS_PHASES  // timing build (scripts/agents_phases.py): counters 8-12 = s_memrealtime ticks per phase
    // and wave, summed (prologue + reset, update_pose, scan pose + first lookup, beam runs: 8-11), 13 = waves
    uint64_t tph = __builtin_amdgcn_s_memrealtime();
    auto aphase = [&](int k) {
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0)
            atomicAdd(a.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride + 8 + k, (unsigned long long)(t - tph));
        tph = t;
        __builtin_amdgcn_sched_barrier(0);
    };
#else
    auto aphase = [](int) {};
#endif
    // the car's update (its returns leave the lambda: the hand-off poses below need every thread)
    int do_reset = 0;
    bool act = false;
    // the update's stores, the scan pose, the first lookup and the beam runs
    auto tail = [&]() {
#pragma unroll
    for (int k = 0; k < 7; ++k) a.st[(size_t)k * EA + g] = s[k];
    a.sb[g] = b0;
    a.sb[EA + g] = b1;
    a.scnt[g] = cnt;
    // scan pose (base_classes.py:420-422) and everything every ray of this car shares
    // base_classes.py:420-422; with lidar_dist == 0 the offset is +-0 for any
    // finite yaw, so the transcendentals are skipped (a non-finite yaw keeps
    // the reference's NaN)
    const bool no_offset = a.lidar_dist == 0.0 && isfinite(s[4]);
    double sy4 = 0.0, cy4 = 1.0;
    if (!no_offset) cr_sincos(s[4], sy4, cy4, tab);
    const double sx = no_offset ? s[0] + 0.0 : s[0] + a.lidar_dist * cy4;
    const double sy = no_offset ? s[1] + 0.0 : s[1] + a.lidar_dist * sy4;
    a.ray0[g] = sx;
    a.ray0[EA + g] = sy;
    a.ray0[2 * EA + g] = a.map.dt[cell_index(a.map, sx, sy)];  // first lookup (laser_models.py:129)
    aphase(2);
    double t0 = first_theta_index(s[4], a.fov, a.theta_dis);
    a.nruns[g] = build_beam_runs_fast(t0, a.inc, a.theta_dis, a.B, a.runs + (size_t)g * kMaxSeg, kMaxSeg);
    aphase(3);
    a.ttc_hit[g] = 0;
    if (ag == 0) {
        a.reset_flag[e] = (uint8_t)do_reset;
        a.noise_step[e] = do_reset ? 0ull : nstep;
    }
    };
    auto car = [&]() {
    if (!valid) return;
    const uint64_t genv = (uint64_t)(a.env_offset + e);
    if (a.mode == 1) {
        if (!gate) return;
        do_reset = 1;
    } else {
        do_reset = gate ? 1 : 0;
    }
    if (do_reset) {
        // RaceCar.reset (base_classes.py:183-204), then F110Env.reset's zero-action step (f110_env.py:457)
        const double *pz;
        if (a.mode == 1) {
            pz = a.reset_poses + (size_t)g * 3;
        } else {
            uint32_t k = spawn_draw(a.seed, genv, episode) % (uint32_t)a.n_spawn;
            pz = a.spawn + ((size_t)k * A + ag) * 3;
        }
        // float32 options (train_ddpg's dtype): the poses are float32 values
        // and start_rot is NumPy's float32 cos / sin of the float32 yaw
        double px = pz[0], py = pz[1], pth = pz[2];
        if (a.reset_f32) {
            px = (double)(float)px;
            py = (double)(float)py;
            pth = (double)(float)pth;
        }
#pragma unroll
        for (int k = 0; k < 7; ++k) s[k] = 0.0;
        s[0] = px;
        s[1] = py;
        s[4] = pth;
        b0 = b1 = 0.0;
        cnt = 0;
        raw_steer = 0.0;
        vel = 0.0;
        a.start[g] = px;
        a.start[EA + g] = py;
        a.start[2 * EA + g] = pth;
        if (ag == a.ego) {  // F110Env.reset's start_rot (f110_env.py:448-451), once per episode
            if (a.reset_f32) {
                const float nt = -(float)pth;
                a.start_rot[e] = (double)np_sincosf(nt, true);
                a.start_rot[a.E + e] = (double)np_sincosf(nt, false);
            } else {
                double sr, crr;
                cr_sincos(-pth, sr, crr, tab);
                a.start_rot[e] = crr;
                a.start_rot[a.E + e] = sr;
            }
        }
        a.toggles[g] = 0;
        a.near_start[g] = 1;
        a.lap_times[g] = 0.0f;
        a.lap_counts[g] = 0.0f;
    }
    aphase(0);
    update_pose(s, b0, b1, cnt, raw_steer, vel, a.pa[ag], a.dt, a.integrator, tab);  // RaceCar.params (per agent)
    aphase(1);
    act = true;
    if (!HMASK) tail();
    };
    car();
#ifdef F110_AGENTS_PHASES
    if ((threadIdx.x & 63) == 0) atomicAdd(a.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride + 13, 1ull);
#endif
    if (HMASK) {
        // the hand-off mask's poses (every car of the block, the new or the unchanged ones), shared
        // before the state stores so that the barrier waits on no memory operation
        __shared__ float hx[64], hy[64], hth[64];
        hx[threadIdx.x] = (float)s[0];
        hy[threadIdx.x] = (float)s[1];
        hth[threadIdx.x] = (float)s[4];
        __syncthreads();
        if (valid) handoff_chunks(a, g, hx, hy, hth, box_len, box_wid);  // (A divides 64: an env's cars share the block)
        if (act) tail();
    }
}


// The RayArgs block in the kernarg segment (k_rays_tiled's only argument).
__device__ __forceinline__ const RayArgs *kernarg_rays() {
#if defined(__HIP_DEVICE_COMPILE__)
    return reinterpret_cast<const RayArgs *>(__builtin_amdgcn_kernarg_segment_ptr());
#else
    return nullptr;
#endif
}

// The kernarg block behind an opaque copy of its pointer: loads through it
// stay where they are written (in the refill pass) instead of being hoisted
// out of the trace loop into SGPRs, which would spill there: an opaque SGPR copy of a pointer to read-only kernel arguments, typed in the
// constant address space: its field loads are scalar loads placed at the use
// (a generic pointer out of the asm would make them flat vector loads)
template <class T>
__device__ __forceinline__ const T *launder_const(const T *ptr) {
    const __attribute__((address_space(4))) T *p;
    asm volatile("s_mov_b64 %0, %1" : "=s"(p) : "s"(ptr));
    return (const T *)p;
}

__device__ __forceinline__ const RayArgs &kernarg_here() { return *launder_const(kernarg_rays()); }

// Lookup statistics of one wave's trace, the same in every lane: lookups
// made, lanes that traced a ray, the longest ray's lookups.
struct WaveLookups {
    uint32_t total, lanes, max;
};

// One wave's rays of k_rays_tiled (a lane traces when `has`): beam index,
// trace_ray's loop (laser_models.py:106-146) with the given EDT lookup,
// clamp, noise, TTC flag, outputs.  The loop runs on wave-uniform control
// (while any lane is still tracing), so its counters live in SGPRs: no
// per-lane lookup counter in the loop body.
template <bool HANDOFF, class Lookup>
__device__ __forceinline__ WaveLookups trace_wave(const RayArgs &a, bool has, int g, int b, int e, int64_t r,
                                                  Lookup lookup) {
    const uint64_t hm = __builtin_amdgcn_ballot_w64(has);
    WaveLookups w{0u, (uint32_t)__popcll(hm), 0u};
    if (!hm) return w;
    const int B = a.B;
    double c = 0.0, s = 0.0, x = 0.0, y = 0.0, d = 0.0, v = 0.0, noise = 0.0;
    if (has) {
        double t = beam_theta_index(a.runs + (size_t)g * kMaxSeg, a.nruns[g], b);
        int ti = (int)t;  // int(theta_index), laser_models.py:124
        if (ti >= a.theta_dis) ti = 0;
        c = a.cosines[ti];
        s = a.sines[ti];
        x = a.ray0[g];
        y = a.ray0[a.EA + g];
        d = a.ray0[2 * a.EA + g];  // :129
        v = a.vel[g];
        // the ray's scan noise does not depend on the trace: drawn (or
        // loaded) here, it overlaps the set-up loads above
        const RayArgs &K = *kernarg_rays();
        if (K.noise_ext)
            noise = K.noise_ext[(size_t)e * B + b];
        else if (K.noise_std > 0.0)
            noise = K.noise_std * (double)beam_normal(K.seed, (uint64_t)(K.env_offset + e), K.noise_step[e], b);
    }
    double tot = d;  // :130 (lanes without a ray: d = 0, never traced)
    const double eps = a.eps, mr = a.max_range;
    uint32_t iters = 0, lane_iters = 0;
    for (;;) {
        const bool act = d > eps && tot <= mr;  // :133 (no loop-carried mask)
        // ballots of the bare compares are their lane masks (a ballot of the
        // conjunction would go through a VGPR)
        const uint64_t m = __builtin_amdgcn_ballot_w64(d > eps) & __builtin_amdgcn_ballot_w64(tot <= mr);
        if (!m) break;
        ++iters;
        lane_iters += (uint32_t)__popcll(m);
        if (act) {
            x += d * c;  // :135
            y += d * s;  // :136
            d = lookup(x, y);
            tot += d;    // :141
        }
    }
    w.total = w.lanes + lane_iters;  // the first lookup of every ray came from k_agents
    w.max = 1u + iters;
    if (!has) return w;
    // Epilogue fields are read through the kernarg pointer HERE, after the
    // loop: argument loads would otherwise sit at kernel entry and stay live
    // in SGPRs across the loop.
    const RayArgs &K = *kernarg_rays();
    double range = tot > mr ? mr : tot;  // :143-144
    if (K.noise_ext || K.noise_std > 0.0) range += noise;  // noise after the clamp (see store_ray)
    // state[3] after update_pose; check_ttc_jit on the noisy scan, before the
    // agent ray_cast (base_classes.py:597-599)
    if (v != 0.0 && ttc_may_fire_lane(range, K.side_max, v, K.ttc_thresh)) {
        const double bcos = K.beam_cos[b], side = K.side[b];
        if (ttc_fires(range, side, v * bcos, K.ttc_thresh)) K.ttc_hit[g] = 1;
    }
    // outputs straight from the ray; with other cars in the env (HANDOFF)
    // k_post_multi patches the beams its ray_cast shortens
    if (K.obs && g == e * a.A) K.obs[(size_t)e * K.obs_len + b] = obs_scan_value(range, K.lidar_max);
    if (K.scans_f32) K.scans_f32[r] = (float)range;
    if (K.scans_f64) K.scans_f64[r] = range;
    if (HANDOFF) K.scan[r] = range;
    return w;
}

// ------------------------------------------------------------------------
// k_rays_tiled: one thread per ray on the 4x4-tiled EDT, with the rotation
// compiled out for axis-aligned maps.  Same results as k_rays, bit for bit.
//
// One ray per lane, 8 waves per SIMD, no lane refill: the hardware wave
// scheduler absorbs the ragged ray lengths.  Measured alternatives that lost
// (DESIGN.md §3): 2 and 4 interleaved rays per lane (1.4x / 2x slower), a
// per-wave ray pool with lane refill (1.35x slower).
//
// Every ray also runs its TTC test (check_ttc_jit, laser_models.py:188-217,
// on the noisy pre-ray_cast scan) and raises its car's flag, and writes its
// observation / scan output entries.  Single-agent envs are then finished
// (k_post_single resolves the per-env state; no f64 scan hand-off at all).
// With other cars in the env (HANDOFF) the f64 range also goes to
// k_post_multi, whose agent ray_cast re-writes the entries it shortens.
//
// CH (chunked dispatch): a wave traces 64 consecutive beams of ONE car (beam
// chunk k of car g) instead of 64 consecutive rays of the flat ray index, and
// the grid walks the chunks in a_order (the forward-looking, long-ray chunks
// first), all cars of one chunk slot before the next.  Waves whose rays run
// longest start first and the short side-looking chunks fill in behind them,
// instead of a late long wave extending the tail of the launch.  With 4 cars
// per block and G4 = ceil(EA/4) blocks per slot, block -> XCD (block % 8)
// keeps all of a car's chunks on one XCD (and its L2) when G4 % 8 == 0.
//
// TRACE (diagnostic build only, f110_debug_wave_trace): lane 0 of every wave
// records its start / end time (s_memrealtime, 100 MHz), hardware id, XCC,
// chunk slot and car to a buffer nothing else reads.
template <bool ROT, bool MASK, bool HANDOFF, bool CH, bool TRACE = false>
__global__ void __launch_bounds__(kBlock) k_rays_tiled(RayArgs a) {
    uint64_t t_start = 0;
    if (TRACE) t_start = __builtin_amdgcn_s_memrealtime();
    const int B = a.B;
    int64_t r;
    int g, b;
    bool live;
    if (CH) {
        const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        int k;
        if ((int)blockIdx.x < a.HB) {  // heavy-first blocks: the listed waves
            const uint32_t item = (uint32_t)blockIdx.x * a.wpb + wave;
            if (item >= *a.heavy_count) return;  // wave-uniform: nothing listed here
            const uint32_t v = __builtin_amdgcn_readfirstlane(a.heavy_list[item]);
            g = (int)(v >> 8);
            k = (int)(v & 255u);
        } else {
            const int blk = (int)blockIdx.x - a.HB;
            const int slot = blk / a.G4;
            const int cg = blk - slot * a.G4;
            g = cg * a.wpb + wave;
            k = (int)a.order[slot];
            if (a.HB && g < a.EA && ((a.heavy_mask[g] >> k) & 1u)) return;  // ran in a heavy block
        }
        b = k * 64 + (int)(threadIdx.x & 63);
        live = g < a.EA && b < B;
        r = (int64_t)g * B + b;
    } else {
        r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
        live = r < (int64_t)a.EA * B;
        g = (int)(r / B);
        b = (int)(r - (int64_t)g * B);
    }
    const int e = live ? g / a.A : 0;
    const bool has = live && (!MASK || a.reset_mask[e]);
    // the off-map cell index in a VGPR for the whole trace (an opaque copy:
    // otherwise it is re-materialised by a v_mov in every loop iteration)
    uint32_t oobv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(oobv) : "s"((uint32_t)a.m.oob << 3));
    const WaveLookups w = trace_wave<HANDOFF>(a, has, g, b, e, r,
                                              [&](double x, double y) { return tiled_lookup<ROT>(a.m, x, y, oobv); });
    if ((threadIdx.x & 63) == 0 && w.lanes) {  // one (lookups, rays) atomic pair per wave
        unsigned long long *slot = kernarg_rays()->ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
        atomicAdd(slot, (unsigned long long)w.total);
        atomicAdd(slot + 1, (unsigned long long)w.lanes);
    }
    if (CH) {  // this wave's cost, the next step's heavy-first prediction
        const uint32_t m = w.lanes ? w.max : 0u;
        uint8_t *wc = kernarg_rays()->wcost;
        if (wc && (threadIdx.x & 63) == 0 && g < a.EA)
            wc[(size_t)g * a.nch + (b >> 6)] = (uint8_t)(m < 255u ? m : 255u);
    }
    if (TRACE && (threadIdx.x & 63) == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        const int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
        uint64_t *o = kernarg_rays()->wtrace + 4 * w;
        o[0] = t_start;
        o[1] = t_end;
        o[2] = ((uint64_t)xcc << 32) | hw;
        o[3] = ((uint64_t)(CH ? (int)blockIdx.x / a.G4 : 0) << 32) | (uint32_t)g;
    }
}

// ------------------------------------------------------------------------
// k_rays_fx: the chunked ray kernel with a fixed-point cell index (one-wave
// blocks, axis-aligned maps; same results as k_rays_tiled, bit for bit).
//
// xy_2_rc's column is int(x_rot / res) with x_rot = x - orig_x
// (laser_models.py:55-86).  Here one fma puts q = (x - orig_x) / res on a
// 2^-30 fixed-point grid: t = fma(x, inv_res, M - orig_x * inv_res) with
// M = 1.5 * 2^22, so t = M + q lies in [2^22, 2^23) for every on-map q and
// bits [50:30] of t are int(q), bits [29:0] its fraction.  The column, the
// row, the bounds test and a guard band then cost integer ops only, where the
// fp64 form took 2 fp64 subtracts, 2 multiplies, 2 fract, 2 adds, a max, 5
// compares and 2 conversions per lookup.
//
// Error budget (in units of q): the constant's rounding (2^-31), t's rounding
// (2^-31), inv_res's rounding, the reference's own rounding of x - orig_x
// and of x_rot / res (each <= q * 2^-53 <= 2^-32 for q < 2^21): < 2^-29 in
// all.  A lane whose fraction lies within kFxBand * 2^-30 = 2^-28 of an
// integer (either coordinate) takes the exact IEEE path of tiled_cell behind a
// wave-uniform branch; every other lane has the reference's cell and the
// reference's bounds verdict (x_rot >= 0 and x_rot < W * res are decided by
// more than the budget).  Off-map: the sign / exponent test rejects any t
// outside [2^22, 2^23) (NaN and inf included), the column test the rest.
//
// The loop test d > eps is the high word of d != 0: every EDT entry is 0 or
// >= res > eps (checked at f110_create).  Per car, the set-up (beam-index run,
// scan pose, speed, noise counter) is wave-uniform and read with scalar loads.
template <class T>
__device__ __forceinline__ T ld_const(const T *p) {  // read-only for the kernel: a scalar load when uniform
    return *reinterpret_cast<const __attribute__((address_space(4))) T *>(reinterpret_cast<uintptr_t>(p));
}

__device__ __forceinline__ uint32_t dhi(double v) { return (uint32_t)(__double_as_longlong(v) >> 32); }
__device__ __forceinline__ uint32_t dlo(double v) { return (uint32_t)__double_as_longlong(v); }

// The fixed-point loop's EDT: the row-major table of k_rays_fx / k_rays_fxn
// (StepArgs::rm), rows of k1 = wt * 8 bytes: row * k1 + col * 8, and off-map
// indices are clamped into the padding, which holds dt[-1,-1], instead of
// selected.  Measured at 65536 envs: 1.184 vs 1.210 ms for the
// 4x4-tiled table; an inexact f32 8x4-tiled or u16 8x8-tiled table (4x the
// cells per cache line) gained only 2-3 %: the gathers' line footprint is not
// what bounds the loop.
__device__ __forceinline__ uint32_t fx_offset(uint32_t k1, uint32_t row, uint32_t col) {
    return __umul24(row, k1) + (col << 3);
}

__device__ __forceinline__ double fx_load(const void *base, uint32_t off) {
    return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(base) + off);
}

// tiled_cell's IEEE path as a byte offset of the row-major table (the
// fixed-point path's fallback); oob8: the byte offset of dt[-1,-1]
__device__ __forceinline__ uint32_t exact_offset(const TiledMapView &m, double x, double y, uint32_t oob8) {
    const double xr = x - m.ox, yr = y - m.oy;
    const bool inb = (xr >= 0) & (xr < m.wres) & (yr >= 0) & (yr < m.hres);  // false for NaN
    if (!inb) return oob8;
    int32_t c = (int32_t)(xr / m.res);
    int32_t r = (int32_t)(yr / m.res);
    if (c >= m.W) {  // dt[r, W] is dt[r+1, 0] in the reference's row-major read
        c = 0;
        ++r;
    }
    return r >= m.H ? oob8 : fx_offset((uint32_t)m.wt * 8u, (uint32_t)r, (uint32_t)c);
}

// Loop-invariant state of the fixed-point sphere trace.
struct FxLoop {
    double cxk, cyk, ir, mr;
    uint32_t oobv, W, H, k1;
};

__device__ __forceinline__ FxLoop fx_loop(const RayArgs &a) {
    FxLoop L;
    // the off-map offset and inv_res in VGPRs for the whole trace (opaque
    // copies: the select cannot read an SGPR beside its VCC condition, and the
    // fma's other operand is an SGPR constant, a VOP3 reads one SGPR); the
    // row-major layout carries the off-map byte offset itself in m.oob
    asm volatile("v_mov_b32 %0, %1" : "=v"(L.oobv) : "s"((uint32_t)a.m.oob));
    asm volatile("v_mov_b64 %0, %1" : "=v"(L.ir) : "s"(a.m.inv_res));
    L.cxk = a.fx_cx;
    L.cyk = a.fx_cy;
    L.mr = a.max_range;
    L.W = (uint32_t)a.m.wt - 1u;  // rows of m.wt cells; columns W .. wt-1 and row H hold dt[-1,-1]
    L.H = (uint32_t)a.m.H;
    L.k1 = (uint32_t)a.m.wt * 8u;
    return L;
}

// One iteration of trace_ray's loop (laser_models.py:135-141) for an active
// lane: step, fixed-point cell, EDT lookup.
__device__ __forceinline__ void fx_step(const TiledMapView &m, const FxLoop &L, double &x, double &y, double &d,
                                        double &tot, double c, double s) {
    x += d * c;  // :135
    y += d * s;  // :136
    // v_fma_f64 with the constant from its SGPR pair (the compiler's v_fmac
    // form would first copy it into the accumulator, 2 v_movs per fma)
    double tx, ty;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tx) : "v"(x), "v"(L.ir), "s"(L.cxk));
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(ty) : "v"(y), "v"(L.ir), "s"(L.cyk));
    const uint32_t hx = dhi(tx), lx = dlo(tx), hy = dhi(ty), ly = dlo(ty);
    const uint32_t col = __builtin_amdgcn_alignbit(hx, lx, 30) - kFxU0;
    const uint32_t row = __builtin_amdgcn_alignbit(hy, ly, 30) - kFxU0;
    const bool inb = (col < L.W) & (row < L.H) & ((int32_t)hx >= 0x40000000) & ((int32_t)hy >= 0x40000000);
    const bool near = ((lx << 2) + 4u * kFxBand < 8u * kFxBand) | ((ly << 2) + 4u * kFxBand < 8u * kFxBand);
    const uint32_t fast = fx_offset(L.k1, row, col);
    const uint32_t sel = 0u - (uint32_t)inb;
    uint32_t off = (fast & sel) | (L.oobv & ~sel);
    if (__builtin_amdgcn_ballot_w64(near)) {  // wave-uniform, rare
        if (near) off = exact_offset(m, x, y, L.oobv);
    }
    d = fx_load(m.dt, off);
    tot += d;  // :141
}

// fx_step for a car whose rays cannot leave t's binade (SAFE: the scan
// origin lies within 2^21 - 16 cells of the map origin, less the max range;
// every lookup of a ray is within max_range of its origin, since the loop
// steps only while tot <= max_range): the sign / exponent tests drop out and
// the column and row are clamped into the padding, which holds dt[-1,-1].
__device__ __forceinline__ void fx_step_safe(const TiledMapView &m, const FxLoop &L, double &x, double &y, double &d,
                                             double &tot, double c, double s) {
    x += d * c;  // :135
    y += d * s;  // :136
    double tx, ty;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tx) : "v"(x), "v"(L.ir), "s"(L.cxk));
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(ty) : "v"(y), "v"(L.ir), "s"(L.cyk));
    const uint32_t lx = dlo(tx), ly = dlo(ty);
    const uint32_t col = __builtin_amdgcn_alignbit(dhi(tx), lx, 30) - kFxU0;
    const uint32_t row = __builtin_amdgcn_alignbit(dhi(ty), ly, 30) - kFxU0;
    const bool near = ((lx << 2) + 4u * kFxBand < 8u * kFxBand) | ((ly << 2) + 4u * kFxBand < 8u * kFxBand);
    uint32_t off = fx_offset(L.k1, min(row, L.H), min(col, L.W));
    if (__builtin_amdgcn_ballot_w64(near)) {  // wave-uniform, rare
        if (near) off = exact_offset(m, x, y, L.oobv);
    }
    d = fx_load(m.dt, off);
    tot += d;  // :141
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// The ray's outputs: clamp (:143-144), noise after the clamp
// (laser_models.py:450-452), check_ttc_jit's beam test on the noisy scan
// (laser_models.py:188-217), obs / scan entries (F110Env._pack_flat_obs);
// with other cars in the env (HANDOFF) the f64 range also goes to
// k_post_multi, whose agent ray_cast re-writes the entries it shortens.
template <bool HANDOFF>
__device__ __forceinline__ void fx_epilogue(const RayArgs &K, int g, int e, int b, double tot, double mr,
                                            double noise, double v) {
    const int64_t r = (int64_t)g * K.B + b;
    double range = tot > mr ? mr : tot;
    if (K.noise_ext || K.noise_std > 0.0) range += noise;
    if (v != 0.0 && ttc_may_fire_lane(range, K.side_max, v, K.ttc_thresh)) {  // (side, beam_cos) loaded only where TTC can fire
        const double bcos = K.beam_cos[b], side = K.side[b];
        if (ttc_fires(range, side, v * bcos, K.ttc_thresh)) K.ttc_hit[g] = 1;
    }
    if (K.obs && g == e * K.A) K.obs[(size_t)e * K.obs_len + b] = obs_scan_value(range, K.lidar_max);
    if (K.scans_f32) K.scans_f32[r] = (float)range;
    if (K.scans_f64) K.scans_f64[r] = range;
    if (HANDOFF) K.scan[r] = range;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {  // set bits of mask below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Diagnostic wave trace of the one-wave-block ray kernels (f110_debug_wave_trace;
// the pointer is null in every other launch): lane 0 stores the wave's start
// time (s_memrealtime, 100 MHz) at entry and its end time, hardware id, XCC and
// work item (item << 32 | car) at exit, 4 u64 per block, with vector stores.
__device__ __forceinline__ void wave_stamp_start(uint64_t *wt) {
    if (wt && threadIdx.x == 0) wt[4 * (size_t)blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void wave_stamp_end(uint64_t *wt, uint32_t item, uint32_t g) {
    if (wt && threadIdx.x == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        uint64_t *o = wt + 4 * (size_t)blockIdx.x;
        o[1] = __builtin_amdgcn_s_memrealtime();
        o[2] = ((uint64_t)xcc << 32) | hw;
        o[3] = ((uint64_t)item << 32) | g;
    }
}
// the same per wave of a multi-wave block (k_rays_fxs): record w = the wave's work item
__device__ __forceinline__ void wave_stamp_start_w(uint64_t *wt, int w) {
    if (wt && (threadIdx.x & 63) == 0) wt[4 * (size_t)w] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void wave_stamp_end_w(uint64_t *wt, int w, uint32_t item, uint32_t g) {
    if (wt && (threadIdx.x & 63) == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        uint64_t *o = wt + 4 * (size_t)w;
        o[1] = __builtin_amdgcn_s_memrealtime();
        o[2] = ((uint64_t)xcc << 32) | hw;
        o[3] = ((uint64_t)item << 32) | g;
    }
}

// Every lane runs one ray; lanes whose ray has ended leave the loop (exec
// mask), each lane counts its own lookups (summed once per wave), and cars
// whose rays stay in t's binade take fx_step_safe (~36 instead of ~59
// instructions per iteration on the wave's serial path; the kernel is
// latency-bound: at 6 / 4 / 2 waves per SIMD it takes 1.31x / 1.62x / 2.9x as
// long).  Row-major EDT with dt[-1,-1] in the padding.
template <bool MASK, bool HANDOFF>
__global__ void __launch_bounds__(64) k_rays_fx(RayArgs a) {
    int g, k;
    if ((int)blockIdx.x < a.HB) {  // heavy-first blocks: the listed waves
        const uint32_t item = blockIdx.x;
        if (item >= ld_const(a.heavy_count)) return;
        const uint32_t v = ld_const(a.heavy_list + item);
        g = (int)(v >> 8);
        k = (int)(v & 255u);
    } else {
        const int blk = (int)blockIdx.x - a.HB;
        const int slot = blk / a.G4;
        g = blk - slot * a.G4;
        k = (int)a.order[slot];
        if (g >= a.EA) return;
        if (a.HB && ((ld_const(a.heavy_mask + g) >> k) & 1u)) return;  // ran in a heavy block
    }
    wave_stamp_start(a.wtrace);
    const int lane = (int)threadIdx.x;
    const int B = a.B;
    const int b0 = k * 64;
    const int b = b0 + lane;
    const int e = HANDOFF ? g / a.A : g;
    const bool has = b < B && (!MASK || ld_const(a.reset_mask + e));

    // ---- per-car set-up (wave-uniform: scalar loads) ----
    // get_scan's beam index (laser_models.py:167-184) from the car's runs:
    // the run holding b0 by a scalar binary search, then the (few) runs that
    // start inside this wave's 64 beams
    const BeamRun *R = a.runs + (size_t)g * kMaxSeg;
    const int n = ld_const(a.nruns + g);
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (ld_const(&R[mid].start) <= b0) lo = mid;
        else hi = mid - 1;
    }
    int rs = ld_const(&R[lo].start);
    double t0 = ld_const(&R[lo].t0), dl = ld_const(&R[lo].delta);
    for (int j = lo + 1; j < n; ++j) {
        const int s2 = ld_const(&R[j].start);
        if (s2 > b0 + 63) break;
        if (b >= s2) {
            rs = s2;
            t0 = ld_const(&R[j].t0);
            dl = ld_const(&R[j].delta);
        }
    }
    const double x00 = ld_const(a.ray0 + g), y00 = ld_const(a.ray0 + a.EA + g);
    const double d00 = ld_const(a.ray0 + 2 * a.EA + g);  // :129
    const double v = ld_const(a.vel + g);
    // every lane runs the set-up (lanes past the last beam on beam B-1, their
    // results unused): no divergent branch, no zero-initialised copies
    const int bc = b < B ? b : B - 1;
    const double t = t0 + (double)(bc - rs) * dl;
    int ti = (int)t;  // int(theta_index), laser_models.py:124
    if (ti >= a.theta_dis) ti = 0;
    const double c = a.cosines[ti], s = a.sines[ti];
    double x = x00, y = y00, d = has ? d00 : 0.0;
    double noise = 0.0;
    {
        const RayArgs &K = *kernarg_rays();
        if (K.noise_ext)
            noise = K.noise_ext[(size_t)e * B + bc];
        else if (K.noise_std > 0.0)
            noise = K.noise_std *
                    (double)beam_normal_k(noise_key(K.seed, (uint64_t)(K.env_offset + e)), ld_const(K.noise_step + e), bc);
    }

    // ---- trace_ray's loop (laser_models.py:133-141) ----
    const FxLoop L = fx_loop(a);
    double tot = d;  // :130 (lanes without a ray: d = 0, never traced)
    uint32_t cnt = 0;
    const double qx = fma(x00, L.ir, L.cxk) - kFxMagic, qy = fma(y00, L.ir, L.cyk) - kFxMagic;
    __builtin_amdgcn_s_waitcnt(0);  // the set-up loads (c, s) land before the loop, not in it
    if (fabs(qx) < a.fx_lim && fabs(qy) < a.fx_lim) {  // wave-uniform (false for NaN)
        while ((dhi(d) != 0u) & (tot <= L.mr)) {
            fx_step_safe(a.m, L, x, y, d, tot, c, s);
            ++cnt;
        }
    } else {
        while ((dhi(d) != 0u) & (tot <= L.mr)) {
            fx_step(a.m, L, x, y, d, tot, c, s);
            ++cnt;
        }
    }
    const uint32_t lane_iters = wave_sum(cnt);
    // the wave's trip count (heavy-first cost; lane slots of the SIMT counter)
    const uint32_t iters = (a.wcost || a.count_slots) ? wave_max(cnt) : 0u;

    // ---- epilogue ----
    const uint32_t lanes = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(has));
    if (has) fx_epilogue<HANDOFF>(*kernarg_rays(), g, e, b, tot, L.mr, noise, v);
    if (lane == 0) {
        const RayArgs &K = *kernarg_rays();
        if (lanes) {  // one (lookups, rays) atomic pair per wave; the first lookup came from k_agents
            unsigned long long *slot = K.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
            atomicAdd(slot, (unsigned long long)(lanes + lane_iters));
            atomicAdd(slot + 1, (unsigned long long)lanes);
            if (K.count_slots) atomicAdd(slot + 2, (unsigned long long)iters * 64ull);  // lane slots the loop issued
        }
        if (K.wcost) {  // this wave's cost, the next step's heavy-first prediction
            const uint32_t mx = lanes ? 1u + iters : 0u;
            K.wcost[(size_t)g * a.nch + k] = (uint8_t)(mx < 255u ? mx : 255u);
        }
    }
    wave_stamp_end(kernarg_here().wtrace, (uint32_t)k, (uint32_t)g);
}


// One fixed-point step of ray r of an ILP lane (k_rays_fxn, row-major table):
// the cell's byte offset for an active ray, the zero cell's (a 0.0 past the
// table's end, which no clamped index reaches) for a ray that has ended, so
// that its load returns d = 0 and leaves its total, x and y as they are.
__device__ __forceinline__ uint32_t fxn_offset(const TiledMapView &m, const FxLoop &L, double &x, double &y,
                                               double d, double c, double s, bool act, uint64_t amask,
                                               uint32_t zero) {
    x += d * c;  // :135
    y += d * s;  // :136
    double tx, ty;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tx) : "v"(x), "v"(L.ir), "s"(L.cxk));
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(ty) : "v"(y), "v"(L.ir), "s"(L.cyk));
    const uint32_t lx = dlo(tx), ly = dlo(ty);
    const uint32_t col = __builtin_amdgcn_alignbit(dhi(tx), lx, 30) - kFxU0;
    const uint32_t row = __builtin_amdgcn_alignbit(dhi(ty), ly, 30) - kFxU0;
    // ballots of bare compares are their lane masks; a ballot of a combined
    // bool would first be materialised in a VGPR (2 more VALU per ballot)
    const uint32_t band = min((lx << 2) + 4u * kFxBand, (ly << 2) + 4u * kFxBand);
    uint32_t fast = fx_offset(L.k1, min(row, L.H), min(col, L.W));
    asm volatile("" : "+v"(fast));  // computed for every lane, then selected (no exec-mask branch)
    uint32_t off = act ? fast : zero;
    if (__builtin_amdgcn_ballot_w64(band < 8u * kFxBand) & amask) {  // wave-uniform, rare
        if (act & (band < 8u * kFxBand)) off = exact_offset(m, x, y, L.oobv);
    }
    return off;
}

// PAD (k_rays_fxn on the padded row-major table, kFxpBase): the IEEE path of
// tiled_cell as a byte offset of the padded table; off-map reads go to cell
// (-P, -P), which holds dt[-1,-1] like every padding cell.
__device__ __forceinline__ uint32_t exact_offset_pad(const TiledMapView &m, double x, double y, uint32_t P) {
    const double xr = x - m.ox, yr = y - m.oy;
    const bool inb = (xr >= 0) & (xr < m.wres) & (yr >= 0) & (yr < m.hres);  // false for NaN
    if (!inb) return 0u;
    int32_t c = (int32_t)(xr / m.res);
    int32_t r = (int32_t)(yr / m.res);
    if (c >= m.W) {  // dt[r, W] is dt[r+1, 0] in the reference's row-major read
        c = 0;
        ++r;
    }
    return r >= m.H ? 0u : ((uint32_t)(r + (int32_t)P) * (uint32_t)m.wt + (uint32_t)(c + (int32_t)P)) * 8u;
}

// One step of ray r of a PAD lane whose car passed the origin test (every
// lookup of its rays lies inside the padded table, fxp_lo / fxp_hx / fxp_hy):
// t = fma(x, inv_res, 2^24 + P - origin / res); one v_alignbit by 28 puts
// floor(q) + P in the low 24 bits, which the u24 multiplies read directly --
// no bias subtraction, no bounds test, no clamp (~15 instead of ~20 VALU per
// ray and iteration in fxn_offset).  Ended rays read the zero cell, lanes
// within kFxpBand * 2^-28 of a cell edge take the IEEE path.
__device__ __forceinline__ uint32_t fxp_offset(const TiledMapView &m, const FxLoop &L, double &x, double &y,
                                               double d, double c, double s, bool act, uint64_t amask,
                                               uint32_t zero_v, uint32_t P) {
    x += d * c;  // :135
    y += d * s;  // :136
    double tx, ty;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tx) : "v"(x), "v"(L.ir), "s"(L.cxk));
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(ty) : "v"(y), "v"(L.ir), "s"(L.cyk));
    const uint32_t lx = dlo(tx), ly = dlo(ty);
    const uint32_t col = __builtin_amdgcn_alignbit(dhi(tx), lx, 28);
    const uint32_t row = __builtin_amdgcn_alignbit(dhi(ty), ly, 28);
    const uint32_t band = min((lx << 4) + 16u * kFxpBand, (ly << 4) + 16u * kFxpBand);
    // (row & 0xffffff) * k1 + (col & 0xffffff) * 8: v_mul_u32_u24 + v_mad_u32_u24 (the compiler's
    // form of the second multiply is a shift and a mask, one more VALU)
    const uint32_t prow = __umul24(row, L.k1);
    uint32_t fast;
    asm volatile("v_mad_u32_u24 %0, %1, 8, %2" : "=v"(fast) : "v"(col), "v"(prow));
    uint32_t off = act ? fast : zero_v;
    if (__builtin_amdgcn_ballot_w64(band < 32u * kFxpBand) & amask) {  // wave-uniform, rare
        if (act & (band < 32u * kFxpBand)) off = exact_offset_pad(m, x, y, P);
    }
    return off;
}

// k_rays_fxn: N rays per lane (beams b0 + 64 r + lane, r < N, of one car: N
// adjacent 64-beam chunks), traced in one loop so that each lane keeps N
// independent EDT gathers in flight.  The single-ray kernel is bound by the
// latency of its dependent gather chain, not by issue (at 6 / 4
// / 2 waves per SIMD it takes 1.31x / 1.62x / 2.9x as long).  A ray that has
// ended reads the zero cell (d = 0); a chunk whose rays have all ended skips
// its step (wave-uniform); the active-ray masks are ballots, so the lookup
// count is a scalar popcount.  Cars whose rays could leave t's binade trace
// their N rays one after the other with fx_step.  Row-major EDT with
// dt[-1,-1] in the padding column / row.  Bit-identical to k_rays_fx.
//
// Heavy-first (as k_rays_fx, with a chunk group in place of a chunk: a.nch is
// the number of groups per car here): HB leading blocks run the groups whose
// longest ray took >= heavy_T lookups in the previous launch.
template <int N, bool MASK, bool HANDOFF, bool PAD = false>
__global__ void __launch_bounds__(64, 8) k_rays_fxn(RayArgs a) {  // 8 waves per SIMD: <= 64 VGPRs
    const int ng = a.nch;  // chunk groups of N chunks per car
    int g, grp;
    if ((int)blockIdx.x < a.HB) {  // heavy-first blocks: the listed groups
        const uint32_t item = blockIdx.x;
        if (item >= ld_const(a.heavy_count)) return;
        const uint32_t hv = ld_const(a.heavy_list + item);
        g = (int)(hv >> 8);
        grp = (int)(hv & 255u);
    } else {
        const int blk = (int)blockIdx.x - a.HB;
        const int slot = blk / a.G4;
        g = blk - slot * a.G4;
        if (g >= a.EA) return;
        grp = ng - 1 - slot;  // descending, as the chunk order of k_rays_fx
        if (a.HB && ((ld_const(a.heavy_mask + g) >> grp) & 1u)) return;  // ran in a heavy block
    }
    wave_stamp_start(a.wtrace);
    const int lane = (int)threadIdx.x;
    const int B = a.B;
    const int b0 = grp * 64 * N;
    const int e = HANDOFF ? g / a.A : g;
    const bool live = !MASK || ld_const(a.reset_mask + e);

    // ---- per-car set-up (wave-uniform: scalar loads), as in k_rays_fx ----
    const BeamRun *R = a.runs + (size_t)g * kMaxSeg;
    const int n = ld_const(a.nruns + g);
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (ld_const(&R[mid].start) <= b0) lo = mid;
        else hi = mid - 1;
    }
    int rs[N];
    double t0[N], dl[N];
    {
        const int s0 = ld_const(&R[lo].start);
        const double u0 = ld_const(&R[lo].t0), w0 = ld_const(&R[lo].delta);
#pragma unroll
        for (int r = 0; r < N; ++r) {
            rs[r] = s0;
            t0[r] = u0;
            dl[r] = w0;
        }
    }
    for (int j = lo + 1; j < n; ++j) {
        const int s2 = ld_const(&R[j].start);
        if (s2 > b0 + 64 * N - 1) break;
        const double tj = ld_const(&R[j].t0), dj = ld_const(&R[j].delta);
#pragma unroll
        for (int r = 0; r < N; ++r)
            if (b0 + 64 * r + lane >= s2) {
                rs[r] = s2;
                t0[r] = tj;
                dl[r] = dj;
            }
    }
    const double x00 = ld_const(a.ray0 + g), y00 = ld_const(a.ray0 + a.EA + g);
    const double d00 = ld_const(a.ray0 + 2 * a.EA + g);  // :129
    double x[N], y[N], d[N], tot[N], c[N], sn[N];
    int bc[N];
    bool has[N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
        const int b = b0 + 64 * r + lane;
        has[r] = live && b < B;
        bc[r] = b < B ? b : B - 1;
        int ti = (int)(t0[r] + (double)(bc[r] - rs[r]) * dl[r]);  // int(theta_index), :124
        if (ti >= a.theta_dis) ti = 0;
        c[r] = a.cosines[ti];
        sn[r] = a.sines[ti];
        x[r] = x00;
        y[r] = y00;
        d[r] = has[r] ? d00 : 0.0;
        tot[r] = d[r];  // :130
    }

    // ---- trace_ray's loop (laser_models.py:133-141), N rays per lane ----
    const FxLoop L = fx_loop(a);
    const uint32_t zero = a.fx_zero;
    uint32_t zero_v;  // in a VGPR for the whole trace (the select's other operand is its SGPR mask)
    asm volatile("v_mov_b32 %0, %1" : "=v"(zero_v) : "s"(zero));
    const uint32_t P = (uint32_t)a.fxp_P;
    uint32_t lane_iters = 0, iters = 0;
    bool fast_car;
    if (PAD) {  // q + P of the scan origin inside [fxp_lo, fxp_h*): its rays stay in the padded table
        const double ux = fma(x00, L.ir, L.cxk) - kFxpBase, uy = fma(y00, L.ir, L.cyk) - kFxpBase;
        fast_car = (ux >= a.fxp_lo) & (ux < a.fxp_hx) & (uy >= a.fxp_lo) & (uy < a.fxp_hy);  // false for NaN
    } else {
        const double qx = fma(x00, L.ir, L.cxk) - kFxMagic, qy = fma(y00, L.ir, L.cyk) - kFxMagic;
        fast_car = fabs(qx) < a.fx_lim && fabs(qy) < a.fx_lim;
    }
    __builtin_amdgcn_s_waitcnt(0);  // the set-up loads land before the loop, not in it
    if (fast_car) {  // wave-uniform (false for NaN)
        // no per-ray flag is carried across iterations (an i1 array would be
        // packed into a VGPR): activity is recomputed from d and the total
        for (;;) {
            uint64_t m[N], any = 0;
#pragma unroll
            for (int r = 0; r < N; ++r) {
                m[r] = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
                any |= m[r];
                lane_iters += (uint32_t)__popcll(m[r]);
            }
            if (!any) break;
            ++iters;
            uint32_t off[N];
#pragma unroll
            for (int r = 0; r < N; ++r) {
                off[r] = zero;
                if (m[r]) {
                    const bool act = (dhi(d[r]) != 0u) & (tot[r] <= L.mr);
                    off[r] = PAD ? fxp_offset(a.m, L, x[r], y[r], d[r], c[r], sn[r], act, m[r], zero_v, P)
                                 : fxn_offset(a.m, L, x[r], y[r], d[r], c[r], sn[r], act, m[r], zero);
                }
            }
#pragma unroll
            for (int r = 0; r < N; ++r) d[r] = fx_load(a.m.dt, off[r]);
#pragma unroll
            for (int r = 0; r < N; ++r) tot[r] += d[r];  // :141
        }
    } else {
        uint32_t cnt = 0;
#pragma unroll
        for (int r = 0; r < N; ++r)
            while ((dhi(d[r]) != 0u) & (tot[r] <= L.mr)) {
                if (PAD) {  // a car whose origin is off the map: the IEEE cell of every lookup
                    x[r] += d[r] * c[r];  // :135
                    y[r] += d[r] * sn[r];  // :136
                    d[r] = fx_load(a.m.dt, exact_offset_pad(a.m, x[r], y[r], P));
                    tot[r] += d[r];  // :141
                } else {
                    fx_step(a.m, L, x[r], y[r], d[r], tot[r], c[r], sn[r]);
                }
                ++cnt;
            }
        lane_iters = wave_sum(cnt);
        iters = wave_max(cnt);
    }

    // ---- epilogue ----
    const RayArgs &K = *kernarg_rays();
    const double v = ld_const(a.vel + g);
    uint32_t lanes = 0;
    const bool noise_on = K.noise_ext || K.noise_std > 0.0;
    const uint32_t key = noise_key(K.seed, (uint64_t)(K.env_offset + e));
    const uint64_t step = noise_on && !K.noise_ext ? ld_const(K.noise_step + e) : 0;
    float pn[N];  // device-stream normals: with N = 2 the lane's beams b and b + 64 share one draw
    if (!K.noise_ext && K.noise_std > 0.0) {
        if (N == 2) {
            beam_normal_pair_k(key, step, beam_noise_pair(b0 + lane), pn[0], pn[1]);
        } else {
#pragma unroll
            for (int r = 0; r < N; ++r) pn[r] = beam_normal_k(key, step, bc[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
        double nz = 0.0;
        if (K.noise_ext) nz = K.noise_ext[(size_t)e * B + bc[r]];
        else if (K.noise_std > 0.0) nz = K.noise_std * (double)pn[r];
        if (has[r])
            fx_epilogue<HANDOFF>(K, g, e, b0 + 64 * r + lane, tot[r], L.mr, nz, v);
        lanes += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(has[r]));
    }
    if (lane == 0) {
        if (lanes) {  // one (lookups, rays) atomic pair per wave; the first lookup came from k_agents
            unsigned long long *cs = K.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
            atomicAdd(cs, (unsigned long long)(lanes + lane_iters));
            atomicAdd(cs + 1, (unsigned long long)lanes);
            // lane slots the loop issued: trip count x 64 lanes x N rays (the serial
            // IEEE loop of an off-map car counts its longest lane's total, a lower bound)
            if (K.count_slots) atomicAdd(cs + 2, (unsigned long long)iters * (fast_car ? 64ull * N : 64ull));
        }
        if (K.wcost) {  // this group's cost, the next step's heavy-first prediction
            const uint32_t mx = lanes ? 1u + iters : 0u;
            K.wcost[(size_t)g * ng + grp] = (uint8_t)(mx < 255u ? mx : 255u);
        }
    }
    wave_stamp_end(kernarg_here().wtrace, (uint32_t)grp, (uint32_t)g);
}

// get_scan's theta index of beam bc (laser_models.py:167-184) from the car's runs;
// lo: the run holding beam b0 (found once per car for all its chunks, see k_rays_fxs)
__device__ __forceinline__ double beam_theta(const BeamRun *R, int n, int lo, int b0, int bc) {
    int rs = ld_const(&R[lo].start);
    double t0 = ld_const(&R[lo].t0), dl = ld_const(&R[lo].delta);
    for (int j = lo + 1; j < n; ++j) {
        const int s2 = ld_const(&R[j].start);
        if (s2 > b0 + 63) break;
        if (bc >= s2) {
            rs = s2;
            t0 = ld_const(&R[j].t0);
            dl = ld_const(&R[j].delta);
        }
    }
    return t0 + (double)(bc - rs) * dl;  // get_scan's theta_index (laser_models.py:167-184)
}


// k_rays_fxs: the car's first kRunsLds beam runs sit in a wave-private LDS copy (3-13 runs for
// the default scan), so the per-car run search and every chunk arm read LDS instead of making
// dependent trips to L2 (the runs were written by k_agents just before); runs past kRunsLds (other
// scan configurations) are read from memory as before.
constexpr int kRunsLds = 16;

__device__ __forceinline__ double rfl64(double v) {  // a wave-uniform VGPR double into SGPRs
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// run j's (start, t0, delta) from the LDS copy RL or, past kRunsLds, from RG (j wave-uniform)
__device__ __forceinline__ void run_at(const BeamRun *RL, const BeamRun *RG, int j, int &st, double &t0, double &dl) {
    if (j < kRunsLds) {
        st = __builtin_amdgcn_readfirstlane(RL[j].start);
        t0 = rfl64(RL[j].t0);
        dl = rfl64(RL[j].delta);
    } else {
        st = ld_const(&RG[j].start);
        t0 = ld_const(&RG[j].t0);
        dl = ld_const(&RG[j].delta);
    }
}

// beam_theta over the LDS copy (k_rays_fxs)
__device__ __forceinline__ double beam_theta_l(const BeamRun *RL, const BeamRun *RG, int n, int lo, int b0, int bc) {
    int rs;
    double t0, dl;
    run_at(RL, RG, lo, rs, t0, dl);
    for (int j = lo + 1; j < n; ++j) {
        int s2;
        double u0, u1;
        run_at(RL, RG, j, s2, u0, u1);
        if (s2 > b0 + 63) break;
        if (bc >= s2) {
            rs = s2;
            t0 = u0;
            dl = u1;
        }
    }
    return t0 + (double)(bc - rs) * dl;  // get_scan's theta_index (laser_models.py:167-184)
}

__device__ __forceinline__ bool lane_in(uint64_t mask) {
    return (uint32_t)(mask >> (threadIdx.x & 63)) & 1u;
}

// The obs entry's f32 division by lidar_max (k_rays_fxs): q = v * y,
// r = fma(-q, lm, v), q' = fma(r, y, q) with y = RN(1 / lm): q is within one
// ulp of v / lm, so q' is the correctly rounded quotient (Markstein's theorem)
// when no intermediate is subnormal; lanes with v < 2^-60 (and lidar_max
// outside [2^-30, 2^30], obs_rinv = 0) take the IEEE divide.  Checked
// exhaustively against the divide for every f32 v in [0, lm]
// (tests/test_obs_division.py).
__device__ __forceinline__ float obs_scan_value_fast(double r, float lmax, float rinv) {
    // obs_scan_value's NaN -> lmax, +inf -> lmax, -inf -> 0, clip: v_min_f32 returns its
    // other operand for a NaN, and -0.0 stays -0.0 (not < 0)
    float v = __builtin_fminf((float)r, lmax);
    v = v < 0.0f ? 0.0f : v;
    const float q = v * rinv;
    float q2 = __builtin_fmaf(__builtin_fmaf(-q, lmax, v), rinv, q);
    const bool ieee = !(v >= 0x1p-60f) | (rinv == 0.0f);
    if (__builtin_amdgcn_ballot_w64(ieee)) {  // rare (wave-uniform branch)
        asm volatile("" ::: "memory");  // the divide stays in the branch (not speculated and selected)
        if (ieee) q2 = v / lmax;
    }
    return q2;
}

template <class T>
__device__ __forceinline__ T ld_off(const T *base, uint32_t byte_off) {  // global_load v, v_off, s[base]
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + byte_off);
}

// k_rays_fxs's step and cell: the fixed-point offset (the zero cell's
// for an ended ray) and whether the lane lies within the guard band of a cell
// edge (the caller takes the IEEE path for those lanes, both slots at once)
// (kFxsBase: the high dwords of t feed the u24 multiplies directly, the low
// dwords hold the shifted fractions; cx / cy are RayArgs::fxs_cx / fxs_cy)
__device__ __forceinline__ uint32_t fxs_offset_m(const FxLoop &L, double cx, double cy, double &x, double &y,
                                                 double d, double c, double s, uint64_t m, uint32_t zero_v,
                                                 bool &near) {
    x += d * c;  // :135
    y += d * s;  // :136
    double tx, ty;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tx) : "v"(x), "v"(L.ir), "s"(cx));
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(ty) : "v"(y), "v"(L.ir), "s"(cy));
    near = min(dlo(tx), dlo(ty)) < 2u * kFxsBand;
    const uint32_t prow = __umul24(dhi(ty), L.k1);
    uint32_t fast, off;
    asm volatile("v_mad_u32_u24 %0, %1, 8, %2" : "=v"(fast) : "v"(dhi(tx)), "v"(prow));
    // lanes of the activity mask m take the cell, the others the zero cell: the mask (the slot's
    // ballot, an SGPR pair) is the select's condition as it is, no per-lane copy of it (readfirstlane:
    // the mask is wave-uniform; where the compiler cannot prove it, it must still land in SGPRs)
    // (readfirstlane returns int: each half goes through uint32_t, or the low half would sign-extend)
    const uint64_t ms = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(m >> 32)) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)m);
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(off) : "v"(zero_v), "v"(fast), "s"(ms));
    return off;
}

// One (car i, opponent j) pair's ray_cast geometry, serially on one lane: the
// same functions and operands as k_post_multi's lane-parallel phases, so the
// same bits.  (xi, yi, yawi): car i's state pose (after the TTC response);
// (xj, yj, thj): opponent j's agent pose (before it, base_classes.py:587).
__device__ __forceinline__ void pair_geometry(double xi, double yi, double yawi, double xj, double yj, double thj,
                                              double length_i, double width_i, int B, double fov, double incr,
                                              double *rv, double *phi, double &wc, double &wh, int32_t *rng) {
    // rv / phi point into the result's own memory (global or LDS): box_beam_window indexes them
    // with loop variables, which local arrays would turn into scratch
    get_vertices(xj, yj, thj, length_i, width_i, rv);  // RaceCar i's params
    double ys, yc;
    cr_sincos(yawi, ys, yc);
    const double ego = atan2(ys, yc);
    int lo = 0, hi = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = blocked_vertex_beam(xi, yi, ego, rv[2 * q], rv[2 * q + 1], B, fov, incr, phi[q]);
        lo = (q == 0 || k < lo) ? k : lo;
        hi = (q == 0 || k > hi) ? k : hi;
    }
    double c, h;
    box_beam_window(xi, yi, rv, phi, c, h);
    int r0a, r0b, r1a, r1b;
    window_beam_ranges(yawi, fov, incr, B, c, h, r0a, r0b, r1a, r1b);
    wc = c;
    wh = h;
    rng[0] = r0a > lo ? r0a : lo;
    rng[1] = r0b < hi ? r0b : hi;
    rng[2] = r1a > lo ? r1a : lo;
    rng[3] = r1b < hi ? r1b : hi;
}

// pair_geometry out of line (k_post_multi's rare recompute after a TTC response):
// inlined, its transcendentals' constants were hoisted out of the block's loops
// and spilled
__device__ __noinline__ void pair_geometry_ool(double xi, double yi, double yawi, double xj, double yj, double thj,
                                               double length_i, double width_i, int B, double fov, double incr,
                                               double *rv, double *phi, double *wc, double *wh, int32_t *rng) {
    pair_geometry(xi, yi, yawi, xj, yj, thj, length_i, width_i, B, fov, incr, rv, phi, *wc, *wh, rng);
}

// The leading geometry blocks of k_rays_fxs<HANDOFF>: one lane per (car,
// opponent) pair, from the state k_agents wrote (pre-TTC), beside the ray waves
// instead of on 2-8 lanes of k_post_multi's serial chain.
__device__ __noinline__ void ray_pair_geometry(const RayArgs &a, int blk) {
    const int A = a.A, EA = a.EA;
    const int NP = A - 1;
    const int pr = blk * 64 + (int)(threadIdx.x & 63);  // pair index over the context: car g's pairs g * NP + jj
    if (pr >= EA * NP) return;
    const int g = pr / NP, jj = pr - g * NP;
    const int e = g / A, i = g - e * A;
    const int j = jj < i ? jj : jj + 1;
    const int gj = e * A + j;
    const f110_params &pi = a.pa[i];
    PairGeom &o = a.geo[pr];
    pair_geometry(a.st[g], a.st[EA + g], a.st[(size_t)4 * EA + g], a.st[gj], a.st[EA + gj],
                  a.st[(size_t)4 * EA + gj], pi.length, pi.width, a.B, a.fov, a.beam_incr, o.rv, o.phi, o.wc, o.wh,
                  o.rng);
}

// ------------------------------------------------------------------------
// k_rays_fxs: one wave per car (a.G4 waves per car: wave j takes the car's
// chunks at positions j, j+G4, ... of its chunk order; car-minor block order
// puts car g's waves on XCD g % 8 when EA % 8 == 0).  Its 64-beam chunks are
// traced two at a time in two slots; a slot whose rays have all ended writes
// its chunk's outputs and takes the car's next chunk at once, so both slots
// keep gathers in flight until the car's last chunk (offline model over oracle
// trip counts, scripts/pair_model.py: 146.7k wave-iterations for adjacent
// pairs vs 109.1k).  Padded EDT (kFxsBase offsets), no heavy-first, no masked
// reset; cars whose origin lies off the map trace their chunks one after the
// other with the IEEE cell.  Per ray the arithmetic is k_rays_fxn's, so
// bit-identical.
//
// Chunk order: descending chunk index (the scan's left edge first).  Round 4
// measured two reorderings, both bit-identical and both slower:
// the car's chunk pairs longest first by the previous launch's trips (5 % fewer
// trips, 1-2 % slower), and the blocks' wave items longest first (LPT: the
// indirection costs this 64-VGPR kernel 21 spilled registers).
//
// The refill pass keeps nothing in SGPRs across the loop: kernel arguments
// are re-read at the use through kernarg_here, the scan origin and first
// lookup sit in VGPRs; table loads and the obs store take 32-bit lane offsets
// from an SGPR base.  The obs entry's f32 division by lidar_max is Markstein's
// correction (obs_scan_value_fast).  The arm's (cos, sin) and the finish's
// (side, beam_cos) are one 16-byte load each from the interleaved tables
// RayArgs::cs2 / bs2.
//
// Software-pipelined slots: each slot's gather is waited for right before
// that slot's next step, so one slot's gather is in flight while the other
// slot's data is consumed (the compiler's waits are vmcnt(1): both slots
// gather every trip, a closed slot on the zero cell).  Per slot and trip: the
// total (:141), the activity test (:133), the refill when the slot's chunk has
// ended, the step (:135-136) and its gather.
// LDS: kFxsWaves work items per block with the theta table's (cos, sin) pairs in one LDS copy
// per block: the arms read them there instead of a 16-byte gather each (a wave-level load for the
// texture-address unit, ~24 cycles like a slot gather: 17 per car).  Single-agent
// contexts that share the device with others (f110_set_device_share, the stream sub-shards) take
// it; a lone context keeps one-wave blocks and the gathers, whose launch is shorter (0.685 vs
// 0.697 ms at 65536 cars: the 8-wave blocks hold their LDS until their slowest car ends), as do
// multi-agent contexts (the 8-wave blocks were slower there: C4 one context 27.7 -> 25.2 M).
template <bool HANDOFF, bool LDS, bool COUNT>
__global__ void __launch_bounds__(LDS ? 64 * kFxsWaves : 64, 8) k_rays_fxs(RayArgs a) {  // 8 waves per SIMD: <= 64 VGPRs
    static_assert(!(HANDOFF && LDS), "the LDS table is the single-agent kernel's");
    constexpr int NS = 2;
    constexpr int W = LDS ? kFxsWaves : 1;  // work items (waves) per block
    __shared__ double2 cs_lds[LDS ? kFxsLdsTheta : 1];
    __shared__ BeamRun runs_l[W][kRunsLds];  // each wave's car's first beam runs (kRunsLds)
    const int wave = LDS ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
    if (LDS) {  // every load of the block's table copy in flight at once, then the LDS writes
        constexpr int kIt = (kFxsLdsTheta + 64 * W - 1) / (64 * W);
        static_assert(!LDS || kIt * 64 * W == kFxsLdsTheta, "the copy's slots cover the LDS table exactly");
        const double2 *src = reinterpret_cast<const double2 *>(a.cs2);
        double2 v[kIt];
#pragma unroll
        for (int i = 0; i < kIt; ++i) {  // (clamped: every load in bounds and unconditional)
            const int k = (int)threadIdx.x + i * 64 * W;
            v[i] = src[k < a.theta_dis ? k : a.theta_dis - 1];
        }
#pragma unroll
        for (int i = 0; i < kIt; ++i)  // k < kIt * 64 W = kFxsLdsTheta: in bounds (entries >= theta_dis never read)
            cs_lds[(int)threadIdx.x + i * 64 * W] = v[i];
        __syncthreads();
    }
    const int item = (int)blockIdx.x * W + wave;  // the wave's work item
    if (item >= (HANDOFF ? a.geo_blocks : 0) + a.EA * a.G4) return;  // the last block's spare waves
    if (HANDOFF && item < a.geo_blocks) {  // wave-uniform: a geometry item
        ray_pair_geometry(kernarg_here(), item);
        return;
    }
    wave_stamp_start_w(a.wtrace, item);  // (the buffer holds the geometry items too: f110_debug_wave_trace)
    const int bid = HANDOFF ? item - a.geo_blocks : item;  // the ray item (geometry items come first)
    const int wj = bid / a.EA;
    const int g = bid - wj * a.EA;
    const int lane = (int)(threadIdx.x & 63);
    const int B = a.B;
    const int e = HANDOFF ? g / a.A : g;
    const int nch = (B + 63) >> 6;
    const int wstride = a.G4;
    // the chunks whose scans k_post_multi may read (k_agents' handoff_chunks; without it every chunk)
    const uint32_t hmask = HANDOFF ? (a.hmask ? ld_const(a.hmask + g) : 0xFFFFFFFFu) : 0u;
    const double *dt = a.m.dt;
    const FxLoop L = fx_loop(a);
    // Every per-car input is requested before anything waits: the scan origin and first lookup
    // (scalar), the run count, and the LDS copy of the first kRunsLds beam runs (lanes < kRunsLds
    // load whatever the car's run slots hold; only runs < nr are ever read) -- one round trip.
    const double rx = ld_const(a.ray0 + g), ry = ld_const(a.ray0 + a.EA + g), rd = ld_const(a.ray0 + 2 * a.EA + g);
    const int nr = ld_const(a.nruns + g);
    const BeamRun *RG = a.runs + (size_t)g * kMaxSeg;
    BeamRun *RL = runs_l[wave];
    if (lane < kRunsLds) RL[lane] = RG[lane];  // wave-private LDS
    // the scan origin and first lookup in VGPRs (re-arm copies them into a slot)
    double x00, y00, d00;
    asm volatile("v_mov_b64 %0, %1" : "=v"(x00) : "s"(rx));
    asm volatile("v_mov_b64 %0, %1" : "=v"(y00) : "s"(ry));
    asm volatile("v_mov_b64 %0, %1" : "=v"(d00) : "s"(rd));  // :129
    asm volatile("" ::"s"(nr));  // (keeps the run count's load with the others, not sunk into the search)
    uint32_t zero_v;  // the zero cell's offset in a VGPR (the select's other operand is its SGPR mask)
    asm volatile("v_mov_b32 %0, %1" : "=v"(zero_v) : "s"(a.fx_zero));

    // slot r traces chunk kk[r] (-1: closed); lane l owns beam kk[r] * 64 + l
    double x[NS], y[NS], d[NS], tot[NS], c[NS], sn[NS];
    int kk[NS];
    int kpar[NS];         // the noise cache entry of the slot's chunk pair
    int pnext = wj;       // position of this wave's next chunk in the car's chunk order
    int kinfo = 0;        // lane k < nch: the run holding beam 64 k (one divergent search per car)
    uint32_t srch = 0;    // the search's vector loads past the LDS copy (their wave-level count is the max)
    if (nr <= kRunsLds) {  // wave-uniform: the LDS copy holds every run; the last run starting at or
        // before beam 64 lane, by counting (unrolled over the copy: no search loop; lanes >= nch unused)
        int cnt = 0;
#pragma unroll
        for (int j = 1; j < kRunsLds; ++j) cnt += (j < nr && RL[j].start <= lane * 64) ? 1 : 0;
        kinfo = cnt;
    } else if (lane < nch) {
        int lo = 0, hi = nr - 1;
        {
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (RG[mid].start <= lane * 64) lo = mid;
                else hi = mid - 1;
                if (COUNT) ++srch;
            }
        }
        kinfo = lo;
    }
    // wave-level vector loads other than the slot gathers (SIMT / TA accounting, counter 3):
    // the wave's share of the block's table copy (LDS) or the arms' table loads, the finishes'
    // TTC table loads, the guard-band re-gathers (wave-uniform, scalar)
    uint32_t loads = (LDS ? (uint32_t)((a.theta_dis - 64 * wave + 64 * W - 1) / (64 * W)) : 0u) + 2u;  // + the run copy
    uint32_t trips = 0;
    // in_loop: the slot's next `tot += d` completes tot = d (:130)
    auto arm = [&](int r, bool in_loop) {
        const RayArgs &K = kernarg_here();
        const int k = nch - 1 - pnext;
        kpar[r] = (k >> 1) & 1;
        pnext += wstride;
        kk[r] = k;
        const int b = k * 64 + lane, bc = b < B ? b : B - 1;
        const int lo = __builtin_amdgcn_readlane(kinfo, k);
        int ti = (int)beam_theta_l(runs_l[wave], K.runs + (size_t)g * kMaxSeg, ld_const(K.nruns + g), lo, k * 64,
                                   bc);  // :124 (nruns: a scalar-cache hit since the wave's start)
        if (ti >= K.theta_dis) ti = 0;
        double2 t2;
        if (LDS) {
            t2 = cs_lds[ti];
        } else {
            t2 = ld_off(reinterpret_cast<const double2 *>(K.cs2), (uint32_t)ti * 16u);
            if (COUNT) loads = __builtin_amdgcn_readfirstlane(loads + 1u);  // uniform: kept in an SGPR
        }
        c[r] = t2.x;
        sn[r] = t2.y;
        x[r] = x00;
        y[r] = y00;
        d[r] = b < B ? d00 : 0.0;
        tot[r] = in_loop ? 0.0 : d[r];  // :130
    };
    uint32_t lanes = 0;
    // device noise: chunks 2p and 2p + 1 (beams b and b + 64 of a 128-beam block) share one
    // Philox draw (beam_normal_pair_k); the half a finished chunk does not use is kept for its
    // partner in a two-entry cache whose entry alternates from pair to pair in the chunk order
    // (the open pairs are two consecutive ones: the slots take a pair's chunks one after the
    // other), so most pairs are drawn once
    float cval[2] = {0.0f, 0.0f};
    int ctag[2] = {-1, -1};
    auto finish = [&](int r) {  // the ended chunk's outputs (fx_epilogue, noise after the clamp)
        const RayArgs &K = kernarg_here();
        const int b = kk[r] * 64 + lane;
        const bool inb = b < B;
        const int bc = inb ? b : B - 1;
        double nz = 0.0;
        if (K.noise_ext) {
            nz = K.noise_ext[(size_t)e * B + bc];
            if (COUNT) loads = __builtin_amdgcn_readfirstlane(loads + 1u);  // uniform: kept in an SGPR
        } else if (K.noise_std > 0.0) {
            const int pp = kk[r] >> 1, ci = kpar[r];
            float nv;
            if (ctag[ci] == pp) {
                nv = cval[ci];
                ctag[ci] = -1;
            } else {  // the pair index of the unclamped beam: its other half is the partner beam's
                const uint32_t key = noise_key(K.seed, (uint64_t)(K.env_offset + e));
                float lo, hi;
                beam_normal_pair_k(key, ld_const(K.noise_step + e), beam_noise_pair(b), lo, hi);
                nv = (kk[r] & 1) ? hi : lo;
                cval[ci] = (kk[r] & 1) ? lo : hi;
                ctag[ci] = pp;
            }
            nz = K.noise_std * (double)nv;
        }
        if (inb) {  // fx_epilogue
            const double mr = K.max_range;
            double range = tot[r] > mr ? mr : tot[r];  // :143-144
            if (K.noise_ext || K.noise_std > 0.0) range += nz;
            const double v = ld_const(K.vel + g);
            const uint32_t boff = (uint32_t)bc * 8u;
            if (v != 0.0) {
                // the wave loads (side, beam_cos) only when a lane may fire (ttc_may_fire_lane)
                const bool may = ttc_may_fire_lane(range, K.side_max, v, K.ttc_thresh);
                if (__builtin_amdgcn_ballot_w64(may)) {
                    const double2 t2 = ld_off(reinterpret_cast<const double2 *>(K.bs2), boff * 2u);  // (side, beam_cos)
                    if (COUNT) loads = __builtin_amdgcn_readfirstlane(loads + 1u);  // uniform: kept in an SGPR
                    if (may && ttc_fires(range, t2.x, v * t2.y, K.ttc_thresh)) K.ttc_hit[g] = 1;
                }
            }
            if (K.obs && (!HANDOFF || g == e * K.A)) {
                float *orow = K.obs + (size_t)e * K.obs_len;
                *reinterpret_cast<float *>(reinterpret_cast<char *>(orow) + (uint32_t)b * 4u) =
                    obs_scan_value_fast(range, K.lidar_max, K.obs_rinv);
            }
            const size_t row = (size_t)g * B;
            if (K.scans_f32) *reinterpret_cast<float *>(reinterpret_cast<char *>(K.scans_f32 + row) + (uint32_t)b * 4u) = (float)range;
            if (K.scans_f64) *reinterpret_cast<double *>(reinterpret_cast<char *>(K.scans_f64 + row) + (uint32_t)b * 8u) = range;
            if (HANDOFF && ((hmask >> kk[r]) & 1u))
                *reinterpret_cast<double *>(reinterpret_cast<char *>(K.scan + row) + (uint32_t)b * 8u) = range;
        }
        if (COUNT) lanes += (uint32_t)min(64, B - kk[r] * 64);  // the chunk's beams (scalar)
    };

    uint32_t lane_iters = 0, slot_gathers = 0;  // COUNT only
    uint32_t closed_trips = 0;
    const double ux = fma(ld_const(a.ray0 + g), L.ir, L.cxk) - kFxpBase;
    const double uy = fma(ld_const(a.ray0 + a.EA + g), L.ir, L.cyk) - kFxpBase;
    // q + P of the scan origin inside [fxp_lo, fxp_h*): its rays stay in the padded table (false for NaN)
    const bool fast_car = (ux >= a.fxp_lo) & (ux < a.fxp_hx) & (uy >= a.fxp_lo) & (uy < a.fxp_hy);
    if (fast_car) {
#pragma unroll
        for (int r = 0; r < NS; ++r) {
            kk[r] = -1;
            d[r] = tot[r] = x[r] = y[r] = c[r] = sn[r] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < NS; ++r)
            if (pnext < nch) arm(r, true);  // tot = 0: the first trip's total completes tot = d00
        __builtin_amdgcn_s_waitcnt(0);
        // one step of slot r (:133-141): the total, the activity mask, the refill when the slot's
        // chunk has ended (a slot with no chunk left to arm closes: kk = -1, m = 0), the step and its
        // gather.  The mask (two ballots of the bare compares: their AND is one SALU op) selects the
        // gather's offset itself; an ended lane reads the zero cell.  The lookup / lane-slot
        // counters exist in the COUNT build only.
        uint64_t nb[NS];
        auto slot_step = [&](int r) {
            tot[r] += d[r];  // :141 (d00 for a freshly armed slot: tot = d00, :130)
            uint64_t m = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
            if (!m && kk[r] >= 0) {  // wave-uniform, rare: the slot's chunk has ended; refill it
                finish(r);
                if (pnext < nch) {
                    arm(r, false);  // tot = d = d00
                    m = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
                } else {
                    kk[r] = -1;
                }
                // the refill's own loads (tables) land here, so that the common path's wait
                // before the step stays vmcnt(1) (the other slot's gather may be in flight)
                __builtin_amdgcn_s_waitcnt(0);
            }
            if (COUNT) {
                lane_iters += (uint32_t)__popcll(m);
                ++slot_gathers;
            }
            bool near;
            const uint32_t off = fxs_offset_m(L, a.fxs_cx, a.fxs_cy, x[r], y[r], d[r], c[r], sn[r], m, zero_v, near);
            d[r] = ld_off(dt, off);
            nb[r] = __builtin_amdgcn_ballot_w64(near) & m;
            // nothing of the next slot's step moves above this gather: its total waits for the
            // next slot's own gather (vmcnt(1)), which would otherwise become vmcnt(0) here
            __builtin_amdgcn_sched_barrier(0);
        };
        // the lanes of nb[r] (within the guard band of a cell edge) re-gather slot r's cell from the
        // IEEE cell index (exec-masked, rare); the load lands before the slot's next step (loads
        // return in order)
        auto regather = [&](int r) {
            const RayArgs &K = kernarg_here();
            if (lane_in(nb[r])) d[r] = ld_off(dt, exact_offset_pad(K.m, x[r], y[r], (uint32_t)K.fxp_P));
            if (COUNT) loads = __builtin_amdgcn_readfirstlane(loads + 1u);  // uniform: kept in an SGPR
        };
        // Both slots open: two gathers in flight per trip until a slot closes (its chunk has
        // ended with none of the car's chunks left to arm; in that trip it gathers the zero cell
        // once more).  Then the open slot runs alone.  One guard-band test per trip
        // covers both slots' gathers.
        if (kk[1] >= 0) {
            for (;;) {
#pragma unroll
                for (int r = 0; r < NS; ++r) slot_step(r);
                if (nb[0] | nb[1]) {
                    if (nb[0]) regather(0);
                    if (nb[1]) regather(1);
                    // slot 0's re-gather was issued after slot 1's gather: wait for both here, so
                    // that the common path's wait before slot 0's next step stays vmcnt(1)
                    __builtin_amdgcn_s_waitcnt(0);
                }
                if (COUNT) ++trips;
                if ((kk[0] < 0) | (kk[1] < 0)) break;
            }
            if (kk[0] < 0) {  // the open slot moves into slot 0 (wave-uniform copies)
                x[0] = x[1];
                y[0] = y[1];
                d[0] = d[1];
                tot[0] = tot[1];
                c[0] = c[1];
                sn[0] = sn[1];
                kk[0] = kk[1];
                kpar[0] = kpar[1];
            }
        }
        while (kk[0] >= 0) {  // one slot left
            slot_step(0);
            if (nb[0]) regather(0);
            if (COUNT) {
                ++trips;
                ++closed_trips;
            }
        }
    } else {  // an origin off the map: the IEEE cell of every lookup, chunk after chunk
        uint32_t cnt = 0;
        while (pnext < nch) {
            arm(0, false);
            const RayArgs &K = kernarg_here();
            uint32_t cc = 0;
            while ((dhi(d[0]) != 0u) & (tot[0] <= L.mr)) {
                x[0] += d[0] * c[0];  // :135
                y[0] += d[0] * sn[0];  // :136
                d[0] = ld_off(dt, exact_offset_pad(K.m, x[0], y[0], (uint32_t)K.fxp_P));
                tot[0] += d[0];  // :141
                ++cc;
            }
            cnt += cc;
            if (COUNT) trips += wave_max(cc);  // the chunk's wave-level gathers
            finish(0);
        }
        if (COUNT) {
            lane_iters = wave_sum(cnt);
            slot_gathers = trips;
        }
    }
    if (COUNT) {
        if (lane == 0) {
            const RayArgs &K = kernarg_here();
            unsigned long long *cs = K.ctr + (size_t)(item % kCtrSlots) * kCtrStride;
            atomicAdd(cs, (unsigned long long)(lanes + lane_iters));  // the first lookup came from k_agents
            atomicAdd(cs + 1, (unsigned long long)lanes);
            // lane slots of the gathers the loop issued: 64 per wave-level gather, the ended lanes'
            // zero-cell reads included (SIMT = loop lookups / lane slots); counter 5: trips a slot
            // spent alone (the other one closed)
            atomicAdd(cs + 2, (unsigned long long)slot_gathers * 64ull);
            atomicAdd(cs + 3, (unsigned long long)loads);
            atomicAdd(cs + 5, (unsigned long long)closed_trips);
        }
        const uint32_t ws = wave_max(srch);  // the run search's wave-level loads (counter 3)
        if (lane == 0) atomicAdd(a.ctr + (size_t)(item % kCtrSlots) * kCtrStride + 3, (unsigned long long)ws);
    }
    wave_stamp_end_w(a.wtrace, item, (uint32_t)(trips < 0xffffu ? trips : 0xffffu) << 8 | (uint32_t)wj, (uint32_t)g);
}

// F110Env.step's time + _check_done (f110_env.py:404-406, :310-352) and the
// env's autoreset / episode / noise bookkeeping, for env e.  Split in two so
// the kernels issue every load of it at their start, together with their own
// loads: one memory round trip instead of a chain of dependent ones (the
// stores in between would otherwise keep the compiler from hoisting them).
struct EpiCar {  // per car: lap bookkeeping
    double sx, sy;
    int32_t tg;
    float lt;
    uint32_t ns;
};
struct EpiEnv {  // per env
    double tprev, ct, st;
    uint64_t nstep;
    uint32_t episode;
};

__device__ __forceinline__ void epilogue_load_car(const StepArgs &a, int g, EpiCar &c) {
    const int EA = a.E * a.A;
    c.sx = a.start[g];
    c.sy = a.start[EA + g];
    c.tg = a.toggles[g];
    c.ns = a.near_start[g];
    c.lt = a.lap_times[g];
}

__device__ __forceinline__ void epilogue_load_env(const StepArgs &a, int e, EpiEnv &v) {
    v.tprev = a.sim_time[e];
    v.ct = a.start_rot[e];  // cos(-th), sin(-th) of the ego start yaw
    v.st = a.start_rot[a.E + e];
    v.nstep = a.noise_step[e];  // written by this step's k_agents
    const uint32_t ep = a.episode[e];  // (loaded whatever the mode: one round trip with the others)
    v.episode = a.mode == 0 ? ep : 0u;
}

// stl: post-TTC state rows of its A agents (x at [i*stride], y at
// [i*stride + 1]); col: collision flags; cars / env: the prefetched inputs.
__device__ void env_epilogue(const StepArgs &a, int e, const double *stl, int stride, const int32_t *col,
                             int do_reset, const EpiEnv &v, const EpiCar *cars) {
    const int A = a.A;
    const double tnow = (do_reset ? 0.0 : v.tprev) + a.dt;
    a.sim_time[e] = tnow;
    const double r00 = v.ct, r01 = -v.st, r10 = v.st, r11 = v.ct;
    bool all4 = true;
    for (int i = 0; i < A; ++i) {
        const int g = e * A + i;
        const EpiCar &c = cars[i];
        double px = stl[i * stride] - c.sx;
        double py = stl[i * stride + 1] - c.sy;
        // np.dot(start_rot, [dx; dy]) (f110_env.py:330) is a BLAS dgemm: on
        // the reference's host each row is fma(r_i1, py, r_i0 * px)
        // (measured, tests/golden/env_lap_f32.npz; the float32 start_rot is
        // widened to f64 first)
        double dx = fma(r01, py, r00 * px);
        double dy = fma(r11, py, r10 * px);
        double ty;
        if (dy > 2.0) ty = dy - 2.0;
        else if (dy < -2.0) ty = -2.0 - dy;
        else ty = 0.0;
        bool close = dx * dx + ty * ty <= 0.1;
        int tg = c.tg;
        uint32_t ns = c.ns;
        if (close && !ns) { ns = 1; ++tg; }
        else if (!close && ns) { ns = 0; ++tg; }
        a.toggles[g] = tg;
        a.near_start[g] = (uint8_t)ns;
        float lc = (float)(tg / 2);
        float lt = tg < 4 ? (float)tnow : c.lt;
        a.lap_counts[g] = lc;
        a.lap_times[g] = lt;
        if (a.out.lap_counts) a.out.lap_counts[g] = lc;
        if (a.out.lap_times) a.out.lap_times[g] = lt;
        all4 = all4 && tg >= 4;
    }
    bool term = col[a.ego] || all4;
    if (a.out.terminated) a.out.terminated[e] = term ? 1 : 0;
    if (a.out.was_reset) a.out.was_reset[e] = (uint8_t)do_reset;
    if (a.out.sim_time) a.out.sim_time[e] = tnow;
    a.pending[e] = (a.autoreset && term) ? 1 : 0;
    // autoreset spawn draws count episodes from the env's last explicit reset, so a
    // reset replays the same trajectory whatever ran before it (the bench's
    // trajectory digest compares N = 1 and N > 1 runs after a clock ramp)
    const uint32_t ep = do_reset ? (a.mode == 0 ? v.episode + 1 : 0u) : v.episode;
    if (do_reset) a.episode[e] = ep;
    a.nstep[e] = v.nstep + 1;
}

// k_post_single: single-agent envs after the FUSED ray kernel, one thread per
// env: the TTC response (RaceCar.check_ttc, base_classes.py:246-249), the
// pose part of the observation, collisions and the env epilogue.
__global__ void __launch_bounds__(64) k_post_single(StepArgs a) {
    reset_next_heavy(a);
    const int e = blockIdx.x * 64 + threadIdx.x;
    if (e >= a.E) return;
    if (a.mode == 1 && a.reset_mask && !a.reset_mask[e]) return;
    const int EA = a.E;  // A == 1: car g == env e
    // every input first (one memory round trip), then the stores
    double stl[2] = {a.st[e], a.st[EA + e]};
    double yaw = a.st[(size_t)4 * EA + e];
    int32_t col = a.ttc_hit[e];
    const int do_reset = a.reset_flag[e];
    EpiCar car;
    EpiEnv env;
    epilogue_load_car(a, e, car);
    epilogue_load_env(a, e, env);
    if (col) {  // state[3:] = 0 (yaw included)
#pragma unroll
        for (int k = 3; k < 7; ++k) a.st[(size_t)k * EA + e] = 0.0;
        yaw = 0.0;
    }
    if (a.out.obs) {
        float *o = a.out.obs + (size_t)e * obs_row(a) + a.B;
        const float4 v = make_float4((float)stl[0], (float)stl[1], (float)wrap_angle(yaw), col ? 1.0f : 0.0f);
        if ((reinterpret_cast<uintptr_t>(o) & 15u) == 0) {  // one 16-byte store (the default obs row is aligned)
            *reinterpret_cast<float4 *>(o) = v;
        } else {
            o[0] = v.x;
            o[1] = v.y;
            o[2] = v.z;
            o[3] = v.w;
        }
    }
    if (a.out.collisions) a.out.collisions[e] = (uint8_t)col;
    env_epilogue(a, e, stl, 2, &col, do_reset, env, &car);
}

// LDS hand-off between the lanes of ONE wave (no workgroup barrier).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// k_post_multi: multi-agent envs after the tiled ray kernel (TTC flags are
// already set).  Two waves per env and no LDS copy of the scans: the agent
// ray_cast edits the f64 hand-off in place, so many envs stay resident per CU
// and their serial phases overlap.  Wave 0 runs GJK (collision_multiple on
// the pre-TTC poses) while wave 1 builds each (car, opponent) pair's box,
// blocked beam range and beam window (on the post-TTC pose).
constexpr int kMultiBlock = 128;  // one wave per env measured no faster (0.398 vs 0.392 ms per C4 step)

struct MultiShared {
    double stl[kMaxAgents][7];   // state after the TTC response
    double pose0[kMaxAgents][3]; // agent_poses: before the TTC response (base_classes.py:587)
    double verts[kMaxAgents][8]; // Simulator.check_collision's boxes (Simulator.params)
    double rv[kMaxAgents * (kMaxAgents - 1)][8];  // opponent j seen by car i (RaceCar i's params)
    double wcen[kMaxAgents * (kMaxAgents - 1)], whalf[kMaxAgents * (kMaxAgents - 1)];
    double phi[kMaxAgents * (kMaxAgents - 1)][4];  // vertex bearings of each pair's box
    double ego[kMaxAgents];                        // atan2(sin(yaw), cos(yaw)), post-TTC
    int32_t kq[kMaxAgents * (kMaxAgents - 1)][4];  // nearest beam of each vertex
    int32_t blo[kMaxAgents * (kMaxAgents - 1)], bhi[kMaxAgents * (kMaxAgents - 1)];
    int32_t rng[kMaxAgents * (kMaxAgents - 1)][4]; // window_beam_ranges, clipped to [blo, bhi]
    int32_t col[kMaxAgents];
    int32_t ttc[kMaxAgents];  // the car's TTC fired (its state[3:] was zeroed)
    EpiCar epi[kMaxAgents];  // env_epilogue inputs, prefetched at kernel start
    EpiEnv epe;
    int32_t do_reset;
};

// beams of pair pr's ray_cast pass (window_beam_ranges clipped to lo..hi)
__device__ __forceinline__ int pass_beams(const MultiShared &sh, int pr) {
    const int n0 = sh.rng[pr][1] - sh.rng[pr][0] + 1;
    const int n1 = sh.rng[pr][3] - sh.rng[pr][2] + 1;
    return (n0 > 0 ? n0 : 0) + (n1 > 0 ? n1 : 0);
}


__global__ void __launch_bounds__(kMultiBlock, 6) k_post_multi(StepArgs a) {
    reset_next_heavy(a);
    __shared__ MultiShared sh;
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    const int A = a.A, B = a.B;
    const int EA = a.E * A;
    if (a.mode == 1 && a.reset_mask && !a.reset_mask[e]) return;  // uniform per block
#ifdef F110_POST_PHASES  // timing build (scripts/post_phases.py): counters 8-11 = wall_clock64 ticks per phase, 12 = blocks
    uint64_t tph = wall_clock64();
    auto phase = [&](int k) {
        const uint64_t t = wall_clock64();
        if (tid == 0) atomicAdd(a.ctr + (size_t)(e % kCtrSlots) * kCtrStride + 8 + k, (unsigned long long)(t - tph));
        tph = t;
    };
#else
    auto phase = [](int) {};
#endif
    double *scan = a.scan + (size_t)e * A * B;
    if (tid < A) {
        const int g = e * A + tid;
#pragma unroll
        for (int k = 0; k < 7; ++k) sh.stl[tid][k] = a.st[(size_t)k * EA + g];
        sh.pose0[tid][0] = sh.stl[tid][0];
        sh.pose0[tid][1] = sh.stl[tid][1];
        sh.pose0[tid][2] = sh.stl[tid][4];
        epilogue_load_car(a, g, sh.epi[tid]);
        get_vertices(sh.stl[tid][0], sh.stl[tid][1], sh.stl[tid][4], a.p.length, a.p.width, sh.verts[tid]);
        const int hit = a.ttc_hit[g];
        sh.col[tid] = hit;  // Simulator.step :601-602
        sh.ttc[tid] = hit;
        if (hit) {          // RaceCar.check_ttc (base_classes.py:246-249): state[3:] = 0
#pragma unroll
            for (int k = 3; k < 7; ++k) {
                sh.stl[tid][k] = 0.0;
                a.st[(size_t)k * EA + g] = 0.0;
            }
        }
    }
    if (tid == 0) {
        sh.do_reset = a.reset_flag[e];
        epilogue_load_env(a, e, sh.epe);
    }
    __syncthreads();
    phase(0);
    if (tid == 0) {  // collision_multiple (collision_models.py:184-212)
        for (int i = 0; i < A - 1; ++i)
            for (int j = i + 1; j < A; ++j)
                if (gjk_collision(sh.verts[i], sh.verts[j])) {
                    sh.col[i] = 1;
                    sh.col[j] = 1;
                }
    }
    if (tid >= 64 && a.geo_ready) {
        // the ray launch's geometry blocks computed every pair from the pre-TTC poses; a car whose
        // TTC fired sees its opponents from a zeroed yaw: its pairs are recomputed here
        const int lane = tid & 63;
        const int NP = A * (A - 1);
        for (int pr = lane; pr < NP; pr += 64) {
            const int i = pr / (A - 1);
            const int jj = pr - i * (A - 1);
            const int j = jj < i ? jj : jj + 1;
            if (sh.ttc[i]) {
                pair_geometry_ool(sh.stl[i][0], sh.stl[i][1], sh.stl[i][4], sh.pose0[j][0], sh.pose0[j][1],
                                  sh.pose0[j][2], a.pa[i].length, a.pa[i].width, B, a.fov, a.beam_incr, sh.rv[pr],
                                  sh.phi[pr], &sh.wcen[pr], &sh.whalf[pr], sh.rng[pr]);
            } else {
                const PairGeom &o = a.geo[(size_t)e * NP + pr];
#pragma unroll
                for (int k = 0; k < 8; ++k) sh.rv[pr][k] = o.rv[k];
                sh.wcen[pr] = o.wc;
                sh.whalf[pr] = o.wh;
#pragma unroll
                for (int k = 0; k < 4; ++k) sh.rng[pr][k] = o.rng[k];
            }
        }
    } else if (tid >= 64) {
        // per-pair geometry (on wave 1 when there are two), spread over lanes:
        // boxes and ego headings, then one (pair, vertex) per lane, then
        // per-pair reductions
        const int lane = tid & 63;
        const int NP = A * (A - 1);
        for (int pr = lane; pr < NP; pr += 64) {
            const int i = pr / (A - 1);
            const int jj = pr - i * (A - 1);
            const int j = jj < i ? jj : jj + 1;
            // RaceCar.ray_cast_agents: get_vertices(opp_pose, self.params['length'], self.params['width'])
            const f110_params &pi = a.pa[i];
            get_vertices(sh.pose0[j][0], sh.pose0[j][1], sh.pose0[j][2], pi.length, pi.width, sh.rv[pr]);
        }
        if (lane < A) {  // atan2(sin, cos) of the post-TTC yaw
            double ys, yc;
            cr_sincos(sh.stl[lane][4], ys, yc);
            sh.ego[lane] = atan2(ys, yc);
        }
        wave_sync();
        for (int w = lane; w < 4 * NP; w += 64) {  // get_blocked_view_indices, one vertex per lane
            const int pr = w >> 2, q = w & 3;
            const int i = pr / (A - 1);
            sh.kq[pr][q] = blocked_vertex_beam(sh.stl[i][0], sh.stl[i][1], sh.ego[i], sh.rv[pr][2 * q],
                                               sh.rv[pr][2 * q + 1], B, a.fov, a.beam_incr, sh.phi[pr][q]);
        }
        wave_sync();
        for (int pr = lane; pr < NP; pr += 64) {
            const int i = pr / (A - 1);
            int lo = sh.kq[pr][0], hi = sh.kq[pr][0];
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                lo = sh.kq[pr][q] < lo ? sh.kq[pr][q] : lo;
                hi = sh.kq[pr][q] > hi ? sh.kq[pr][q] : hi;
            }
            sh.blo[pr] = lo;
            sh.bhi[pr] = hi;
            double wc, wh;
            box_beam_window(sh.stl[i][0], sh.stl[i][1], sh.rv[pr], sh.phi[pr], wc, wh);
            sh.wcen[pr] = wc;
            sh.whalf[pr] = wh;
            int r0a, r0b, r1a, r1b;
            window_beam_ranges(sh.stl[i][4], a.fov, a.beam_incr, B, wc, wh, r0a, r0b, r1a, r1b);
            sh.rng[pr][0] = r0a > lo ? r0a : lo;  // beams lo..hi of ray_cast's loop that the window can hold
            sh.rng[pr][1] = r0b < hi ? r0b : hi;
            sh.rng[pr][2] = r1a > lo ? r1a : lo;
            sh.rng[pr][3] = r1b < hi ? r1b : hi;
        }
    }
    __syncthreads();
    phase(1);
    // agent ray_cast (base_classes.py:206-227; laser_models.py:318-346), one
    // opponent at a time per car (each pass min-updates the same beams), all
    // cars' passes of one round in one sweep over the block; only the beams
    // of lo..hi that the box's window can hold are visited
    for (int jj = 0; jj < A - 1; ++jj) {
        int total = 0;
        for (int i = 0; i < A; ++i) total += pass_beams(sh, i * (A - 1) + jj);
        for (int item = tid; item < total; item += kMultiBlock) {
            int i = 0, k = item;
            for (int n = pass_beams(sh, jj); k >= n; n = pass_beams(sh, i * (A - 1) + jj)) {
                k -= n;
                ++i;
            }
            const int pr = i * (A - 1) + jj;
            const int n0 = sh.rng[pr][1] - sh.rng[pr][0] + 1;
            const int b = k < (n0 > 0 ? n0 : 0) ? sh.rng[pr][0] + k : sh.rng[pr][2] + k - (n0 > 0 ? n0 : 0);
            const double ox = sh.stl[i][0], oy = sh.stl[i][1], oth = sh.stl[i][4];
            const double *v = sh.rv[pr];
            const double ang = beam_angle(b, a.fov, a.beam_incr);
            if (!(fabs(wrap_pm_pi(oth + ang - sh.wcen[pr])) <= sh.whalf[pr])) continue;  // box_beam_window
            if ((a.hcheck & 1) && a.hmask && !((a.hmask[(size_t)e * A + i] >> (b >> 6)) & 1u))  // debug: a hand-off miss
                atomicAdd(a.ctr + (size_t)(e % kCtrSlots) * kCtrStride + 6, 1ull);
            const double bt = oth + ang + kPi / 2.;
            double v31, v30;
            cr_sincos(bt, v31, v30);
            double cur = scan[i * B + b];
            const double cur0 = cur;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int q1 = (q + 1) & 3;
                const double rr = get_range(ox, oy, v30, v31, v[2 * q], v[2 * q + 1], v[2 * q1], v[2 * q1 + 1]);
                if (rr < cur) cur = rr;
            }
            if (cur != cur0) {  // patch the ray pass's outputs for this beam
                scan[i * B + b] = cur;
                const size_t o = ((size_t)e * A + i) * B + b;
                if (a.out.scans) a.out.scans[o] = (float)cur;
                if (a.out.scans_f64) a.out.scans_f64[o] = cur;
                if (i == 0 && a.out.obs) a.out.obs[(size_t)e * obs_row(a) + b] = obs_scan_value(cur, (float)a.p.lidar_max);
            }
        }
        __syncthreads();
    }
    phase(2);

    // ---- outputs --------------------------------------------------------
    // the scan entries were written by the ray pass (and patched above)
    if (a.out.obs && tid < A) {  // F110Env._pack_flat_obs, f110_env.py:552-584: pose entries
        float *o = a.out.obs + (size_t)e * obs_row(a) + B + 4 * tid;
        o[0] = (float)sh.stl[tid][0];
        o[1] = (float)sh.stl[tid][1];
        o[2] = (float)wrap_angle(sh.stl[tid][4]);
        o[3] = sh.col[tid] ? 1.0f : 0.0f;
    }
    if (a.out.collisions && tid < A) a.out.collisions[(size_t)e * A + tid] = (uint8_t)sh.col[tid];
    if (tid == 0) env_epilogue(a, e, &sh.stl[0][0], 7, sh.col, sh.do_reset, sh.epe, sh.epi);
#ifdef F110_POST_PHASES
    phase(3);
    if (tid == 0) atomicAdd(a.ctr + (size_t)(e % kCtrSlots) * kCtrStride + 12, 1ull);
#endif
}

// One f110_step / f110_reset: k_agents, the ray kernel, the post stage.
// The ray kernel by context (f110_create's rules):
//   ray_kernel 1 / 2: k_rays_tiled in flat / chunked order (rotated maps, or
//                     where the fixed-point preconditions fail);
//   ray_kernel 3:     k_rays_fx (1 ray per lane), k_rays_fxn<2> (2 rays per
//                     lane, padded or clamped table) or, for unmasked steps
//                     without heavy-first, k_rays_fxs (fx_refill waves per car).
hipError_t launch_env_step(const StepArgs &a, hipStream_t s, hipEvent_t *ev) {
    const int EA = a.E * a.A;
    hipError_t e;
    auto evk = [&](int i) -> hipEvent_t { return ev ? ev[i] : nullptr; };  // (start, stop) per kernel
    // 64-thread blocks: a few thousand cars must still spread over all CUs
    if (a.hmask)
        hipExtLaunchKernelGGL(k_agents<true>, dim3((EA + 63) / 64), dim3(64), 0, s, evk(0), evk(1), 0, a);
    else
        hipExtLaunchKernelGGL(k_agents<false>, dim3((EA + 63) / 64), dim3(64), 0, s, evk(0), evk(1), 0, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (a.gate_wait && (e = hipStreamWaitEvent(s, a.gate_wait, 0)) != hipSuccess) return e;
    const bool single = a.A == 1;
    // f110_debug_set_handoff_check: every hand-off entry NaN (all-ones) before the ray launch, so a
    // k_post_multi read of an entry the ray kernel skipped cannot pass for a fresh one
    if ((a.hcheck & 1) && !single && (e = hipMemsetAsync(a.scan, 0xFF, (size_t)EA * a.B * sizeof(double), s)) != hipSuccess)
        return e;
    RayArgs ra{};
    ra.m = a.tmap;
    ra.sines = a.sines;
    ra.cosines = a.cosines;
    ra.ray0 = a.ray0;
    ra.runs = a.runs;
    ra.nruns = a.nruns;
    ra.reset_mask = a.mode == 1 ? a.reset_mask : nullptr;
    ra.scan = a.scan;
    ra.noise_ext = a.noise_ext;
    ra.noise_step = a.noise_step;
    ra.ctr = a.ctr;
    ra.count_slots = a.count_slots;
    ra.eps = a.eps;
    ra.max_range = a.max_range;
    ra.noise_std = a.noise_std;
    ra.seed = a.seed;
    ra.env_offset = a.env_offset;
    ra.EA = EA;
    ra.A = a.A;
    ra.B = a.B;
    ra.theta_dis = a.theta_dis;
    ra.vel = a.st + (size_t)3 * EA;
    ra.beam_cos = a.beam_cos;
    ra.side = a.side;
    ra.cs2 = a.cs2;
    ra.bs2 = a.bs2;
    ra.ttc_thresh = a.ttc_thresh;
    ra.side_max = a.side_max;
    ra.ttc_hit = a.ttc_hit;
    ra.obs = a.out.obs;
    ra.obs_len = (int32_t)obs_row(a);
    ra.lidar_max = (float)a.p.lidar_max;
    ra.obs_rinv = obs_reciprocal(ra.lidar_max);
    ra.scans_f32 = a.out.scans;
    ra.scans_f64 = a.out.scans_f64;
    const bool rot = !(a.tmap.os == 0.0 && a.tmap.oc == 1.0);
    const bool mask = ra.reset_mask != nullptr;
    const bool ch = a.ray_kernel >= 2;
    const int64_t R = (int64_t)EA * a.B;
    dim3 g2((unsigned)((R + kBlock - 1) / kBlock));
    if (ch) {
        ra.wpb = a.ray_wpb;
        ra.G4 = (EA + ra.wpb - 1) / ra.wpb;
        ra.nch = (a.B + 63) / 64;
        for (int i = 0; i < kMaxChunks; ++i) ra.order[i] = a.chunk_order[i];
        // the per-wave cost bytes feed the next step's heavy-first list only:
        // not written when heavy-first is off (the stream sub-shard runner)
        ra.wcost = a.heavy_on ? a.wcost : nullptr;
        if (a.heavy_use && !mask) {
            ra.HB = (a.heavy_cap + ra.wpb - 1) / ra.wpb;
            ra.heavy_list = a.heavy_list + (size_t)a.parity * a.heavy_cap;
            ra.heavy_mask = a.heavy_mask;
            ra.heavy_count = a.heavy_count + a.parity;
        }
        g2 = dim3((unsigned)(ra.HB + ra.G4 * ra.nch));
    }
    const int vt = (rot ? 4 : 0) + (mask ? 2 : 0) + (single ? 0 : 1);  // HANDOFF for A >= 2
    const void *tiled_fn[2][8] = {
        {reinterpret_cast<const void *>(&k_rays_tiled<false, false, false, false>),
         reinterpret_cast<const void *>(&k_rays_tiled<false, false, true, false>),
         reinterpret_cast<const void *>(&k_rays_tiled<false, true, false, false>),
         reinterpret_cast<const void *>(&k_rays_tiled<false, true, true, false>),
         reinterpret_cast<const void *>(&k_rays_tiled<true, false, false, false>),
         reinterpret_cast<const void *>(&k_rays_tiled<true, false, true, false>),
         reinterpret_cast<const void *>(&k_rays_tiled<true, true, false, false>),
         reinterpret_cast<const void *>(&k_rays_tiled<true, true, true, false>)},
        {reinterpret_cast<const void *>(&k_rays_tiled<false, false, false, true>),
         reinterpret_cast<const void *>(&k_rays_tiled<false, false, true, true>),
         reinterpret_cast<const void *>(&k_rays_tiled<false, true, false, true>),
         reinterpret_cast<const void *>(&k_rays_tiled<false, true, true, true>),
         reinterpret_cast<const void *>(&k_rays_tiled<true, false, false, true>),
         reinterpret_cast<const void *>(&k_rays_tiled<true, false, true, true>),
         reinterpret_cast<const void *>(&k_rays_tiled<true, true, false, true>),
         reinterpret_cast<const void *>(&k_rays_tiled<true, true, true, true>)}};
    const void *f = tiled_fn[ch ? 1 : 0][vt];
    unsigned bdim = ch ? 64u * (unsigned)ra.wpb : (unsigned)kBlock;
    bool geo_ready = false;  // the ray launch computes the pairs' ray_cast geometry (k_post_multi reads it)
    bool fxs = false, lds = false;  // k_rays_fxs; with the LDS theta table
    // the fixed-point kernels (f110_create checked their preconditions: axis-aligned map,
    // one-wave blocks, W, H < 2^21, |origin / res| < 2^20, EDT entries 0 or > eps)
    const bool fx = a.ray_kernel == 3 && !rot && ra.wpb == 1 && a.rm;
    if (fx) {
        const int v2 = (mask ? 2 : 0) + (single ? 0 : 1);
        // the row-major EDT (dt[-1,-1] in the padding column / row, a zero cell past the end)
        ra.m.dt = a.rm;
        ra.m.wt = a.rm_w;
        ra.m.oob = (int32_t)a.rm_oob;
        ra.fx_zero = a.rm_zero;
        ra.fx_cx = std::fma(-a.tmap.ox, a.tmap.inv_res, kFxMagic);
        ra.fx_cy = std::fma(-a.tmap.oy, a.tmap.inv_res, kFxMagic);
        ra.fx_lim = 2097152.0 - 32.0 - a.max_range * a.tmap.inv_res;
        const void *fn_1[4] = {reinterpret_cast<const void *>(&k_rays_fx<false, false>),
                               reinterpret_cast<const void *>(&k_rays_fx<false, true>),
                               reinterpret_cast<const void *>(&k_rays_fx<true, false>),
                               reinterpret_cast<const void *>(&k_rays_fx<true, true>)};
        f = fn_1[v2];
        if (a.fx_ilp == 2) {
            const bool pad = a.fx_pad && a.rmp;
            const void *fn_2[2][4] = {{reinterpret_cast<const void *>(&k_rays_fxn<2, false, false>),
                                       reinterpret_cast<const void *>(&k_rays_fxn<2, false, true>),
                                       reinterpret_cast<const void *>(&k_rays_fxn<2, true, false>),
                                       reinterpret_cast<const void *>(&k_rays_fxn<2, true, true>)},
                                      {reinterpret_cast<const void *>(&k_rays_fxn<2, false, false, true>),
                                       reinterpret_cast<const void *>(&k_rays_fxn<2, false, true, true>),
                                       reinterpret_cast<const void *>(&k_rays_fxn<2, true, false, true>),
                                       reinterpret_cast<const void *>(&k_rays_fxn<2, true, true, true>)}};
            f = fn_2[pad ? 1 : 0][v2];
            ra.nch = (ra.nch + 1) / 2;  // chunk groups per car (heavy list / wcost units)
            g2 = dim3((unsigned)(ra.HB + ra.G4 * ra.nch));
            if (pad) {
                // the padded table (PAD): t = x / res + 2^24 + P; a car's rays stay in the
                // table when its origin's q + P lies in [Rn, W or H + 2P - Rn),
                // Rn = max_range / res + 2 cells (each lookup is within max_range of it)
                const double P = (double)a.rmp_P, Rn = std::ceil(a.max_range * a.tmap.inv_res) + 2.0;
                ra.m.dt = a.rmp;
                ra.m.wt = a.rmp_w;
                ra.m.oob = 0;
                ra.fx_zero = a.rmp_zero;
                ra.fxp_P = a.rmp_P;
                ra.fx_cx = std::fma(-a.tmap.ox, a.tmap.inv_res, kFxpBase + P);
                ra.fx_cy = std::fma(-a.tmap.oy, a.tmap.inv_res, kFxpBase + P);
                ra.fxp_lo = Rn;
                ra.fxp_hx = (double)a.tmap.W + 2.0 * P - Rn;
                ra.fxp_hy = (double)a.tmap.H + 2.0 * P - Rn;
                ra.fxs_cx = std::fma(-a.tmap.ox, a.tmap.inv_res, kFxsBase + P + kFxsShift);
                ra.fxs_cy = std::fma(-a.tmap.oy, a.tmap.inv_res, kFxsBase + P + kFxsShift);
                if (a.fx_refill > 0 && a.fxs_ok && !mask && ra.HB == 0 && !ra.wcost) {
                    // one wave per car, two chunk slots with refill (k_rays_fxs; no heavy-first)
                    lds = single && a.fxs_lds && a.theta_dis <= kFxsLdsTheta;
                    // COUNT (f110_debug_set_simt): the variant that counts lookups, rays, lane slots
                    const void *fxs_fn[2][3] = {
                        {reinterpret_cast<const void *>(&k_rays_fxs<false, false, false>),
                         reinterpret_cast<const void *>(&k_rays_fxs<false, true, false>),
                         reinterpret_cast<const void *>(&k_rays_fxs<true, false, false>)},
                        {reinterpret_cast<const void *>(&k_rays_fxs<false, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxs<false, true, true>),
                         reinterpret_cast<const void *>(&k_rays_fxs<true, false, true>)}};
                    f = fxs_fn[a.count_slots ? 1 : 0][lds ? 1 : single ? 0 : 2];
                    fxs = true;
                    ra.G4 = std::min(a.fx_refill, (a.B + 63) / 64);  // waves per car
                    if (!single && a.geo) {  // leading geometry items (a multiple of 8: XCD mapping kept)
                        ra.geo = a.geo;
                        ra.hmask = a.hmask;
                        ra.geo_blocks = ((ra.EA * (a.A - 1) + 63) / 64 + 7) / 8 * 8;
                        ra.st = a.st;
                        ra.pa = a.pa;
                        ra.fov = a.fov;
                        ra.beam_incr = a.beam_incr;
                        geo_ready = true;
                    }
                    const int wpb = lds ? kFxsWaves : 1;  // k_rays_fxs's work items per block
                    g2 = dim3((unsigned)((ra.geo_blocks + ra.EA * ra.G4 + wpb - 1) / wpb));
                    bdim = 64u * (unsigned)wpb;
                }
            }
        }
        if (!fxs) bdim = 64u;
    }
    if (a.wtrace && ch && !rot && !mask && !fx)  // diagnostic wave trace (f110_debug_wave_trace)
        f = single ? reinterpret_cast<const void *>(&k_rays_tiled<false, false, false, true, true>)
                   : reinterpret_cast<const void *>(&k_rays_tiled<false, false, true, true, true>);
    ra.wtrace = a.wtrace;
    void *args[] = {&ra};
    if ((e = hipExtLaunchKernel(f, g2, dim3(bdim), args, 0u, s, evk(2), evk(3), 0)) != hipSuccess) return e;
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (a.gate_record && (e = hipEventRecord(a.gate_record, s)) != hipSuccess) return e;
    if (single)
        hipExtLaunchKernelGGL(k_post_single, dim3((a.E + 63) / 64), dim3(64), 0, s, evk(4), evk(5), 0, a);
    else {
        StepArgs pa_ = a;
        pa_.geo_ready = geo_ready ? 1 : 0;
        hipExtLaunchKernelGGL(k_post_multi, dim3(a.E), dim3(kMultiBlock), 0, s, evk(4), evk(5), 0, pa_);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return hipSuccess;
}

// ------------------------------------------------------------------------
// ScanSimulator2D.scan with rng=None for M poses: one thread per ray, beam
// runs rebuilt per thread (cheap: < 20 runs), optional probes.
__global__ void __launch_bounds__(kBlock) k_scan_batch(ScanArgs a) {
    const int64_t gid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t n = 0;
    if (gid < a.M * a.B) {
        const int64_t m = gid / a.B;
        const int b = (int)(gid - m * a.B);
        const double *pose = a.poses + 3 * m;
        BeamRun runs[kMaxSeg];
        double t0 = first_theta_index(pose[2], a.fov, a.theta_dis);
        int nr = build_beam_runs(t0, a.inc, a.theta_dis, a.B, runs, kMaxSeg);
        double t = beam_theta_index(runs, nr, b);
        int ti = (int)t;
        if (ti >= a.theta_dis) ti = 0;
        double s = a.sines[ti], c = a.cosines[ti];
        double x = pose[0], y = pose[1];
        double d = a.map.dt[cell_index(a.map, x, y)];
        double tot = d;
        n = 1;
        while (d > a.eps && tot <= a.max_range) {
            x += d * c;
            y += d * s;
            d = a.map.dt[cell_index_fast(a.map, x, y)];
            tot += d;
            ++n;
        }
        if (tot > a.max_range) tot = a.max_range;
        a.scans[gid] = tot;
        if (a.lookups) a.lookups[gid] = (int32_t)n;
        if (a.hit_rc) {  // (r, c) of the last lookup; out-of-map reads report (-1, -1)
            double xt = x - a.map.ox, yt = y - a.map.oy;
            double xr = xt * a.map.oc + yt * a.map.os;
            double yr = -xt * a.map.os + yt * a.map.oc;
            int rr = -1, cc = -1;
            if (!(xr < 0 || xr >= a.map.wres || yr < 0 || yr >= a.map.hres || xr != xr || yr != yr)) {
                cc = (int)(xr / a.map.res);
                rr = (int)(yr / a.map.res);
            }
            a.hit_rc[2 * gid] = rr;
            a.hit_rc[2 * gid + 1] = cc;
        }
    }
    if (a.ctr) count_rays(a.ctr, n);
}

hipError_t launch_scan_batch(const ScanArgs &a, hipStream_t s) {
    if (a.M <= 0) return hipSuccess;
    int64_t n = a.M * a.B;
    hipLaunchKernelGGL(k_scan_batch, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_dynamics(const double *__restrict__ x, const double *__restrict__ u,
                                                     double *__restrict__ f, int64_t M, f110_params p) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= M) return;
    double xs[7], fs[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) xs[k] = x[7 * i + k];
    vehicle_dynamics_st(xs, u[2 * i], u[2 * i + 1], p, fs);
#pragma unroll
    for (int k = 0; k < 7; ++k) f[7 * i + k] = fs[k];
}

hipError_t launch_dynamics_batch(const double *x, const double *u, double *f, int64_t M, const f110_params &p,
                                 hipStream_t s) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dynamics, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, x, u, f, M, p);
    return hipGetLastError();
}

// vehicle_dynamics_ks over M kinematic states [M][5] (f110_dynamics_ks_batch).
__global__ void __launch_bounds__(kBlock) k_dynamics_ks(const double *__restrict__ x, const double *__restrict__ u,
                                                        double *__restrict__ f, int64_t M, f110_params p) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= M) return;
    double xs[5], fs[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) xs[k] = x[5 * i + k];
    vehicle_dynamics_ks(xs, u[2 * i], u[2 * i + 1], p, fs);
#pragma unroll
    for (int k = 0; k < 5; ++k) f[5 * i + k] = fs[k];
}

hipError_t launch_dynamics_ks_batch(const double *x, const double *u, double *f, int64_t M, const f110_params &p,
                                    hipStream_t s) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dynamics_ks, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, x, u, f, M, p);
    return hipGetLastError();
}

// collision (collision_models.py:113-182, GJK) for M vertex pairs: one thread
// per pair, the pair's 2 x 8 doubles in registers (f110_collision_batch).
__global__ void __launch_bounds__(kBlock) k_collision_batch(const double *__restrict__ v1,
                                                            const double *__restrict__ v2, int64_t M,
                                                            uint8_t *__restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= M) return;
    double a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] = v1[8 * i + k];
        b[k] = v2[8 * i + k];
    }
    out[i] = gjk_collision(a, b) ? 1 : 0;
}

hipError_t launch_collision_batch(const double *v1, const double *v2, int64_t M, uint8_t *out, hipStream_t s) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_collision_batch, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, v1, v2,
                       M, out);
    return hipGetLastError();
}

// collision_multiple (collision_models.py:184-212) for M independent sets of
// N bodies: one wave per set, its N(N-1)/2 pairs spread over the lanes, then
// lane 0 writes the flags and partner indices in the reference's (i, j)
// order, so the last colliding pair of each body wins as in the reference.
__global__ void __launch_bounds__(64) k_collision_multiple(const double *__restrict__ verts, int64_t M, int32_t N,
                                                           double *__restrict__ collisions, double *__restrict__ idx) {
    const int64_t m = blockIdx.x;
    if (m >= M) return;
    __shared__ uint8_t hit[kMaxMultiBodies * kMaxMultiBodies];
    const double *v = verts + (size_t)m * N * 8;
    const int P = N * (N - 1) / 2;
    for (int q = threadIdx.x; q < P; q += 64) {
        int i = 0, r = q;  // pair q -> (i, j), i < j, in the reference's loop order
        while (r >= N - 1 - i) {
            r -= N - 1 - i;
            ++i;
        }
        const int j = i + 1 + r;
        hit[i * N + j] = gjk_collision(v + 8 * i, v + 8 * j) ? 1 : 0;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double *c = collisions + (size_t)m * N, *ix = idx + (size_t)m * N;
    for (int i = 0; i < N; ++i) {
        c[i] = 0.0;
        ix[i] = -1.0;
    }
    for (int i = 0; i < N - 1; ++i)
        for (int j = i + 1; j < N; ++j)
            if (hit[i * N + j]) {
                c[i] = 1.0;
                c[j] = 1.0;
                ix[i] = (double)j;
                ix[j] = (double)i;
            }
}

hipError_t launch_collision_multiple(const double *verts, int64_t M, int32_t N, double *collisions, double *idx,
                                     hipStream_t s) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_collision_multiple, dim3((unsigned)M), dim3(64), 0, s, verts, M, N, collisions, idx);
    return hipGetLastError();
}

}  // namespace f110
