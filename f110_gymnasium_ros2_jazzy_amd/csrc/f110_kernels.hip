// f110_kernels.hip — gfx950 kernels of the batched F1TENTH step.
//
// One f110_step = three launches on the caller's stream:
//
//  k_agents    one thread per car: reset/autoreset, RaceCar.update_pose
//              (steer delay, pid, RK4 of vehicle_dynamics_st, clamps), scan
//              pose, first EDT lookup, and the car's beam-index runs.
//  k_rays      one thread per lidar ray (E*A*B threads): the EDT
//              sphere-trace of ScanSimulator2D (trace_ray), + scan noise.
//              This is the hot kernel: ~7 dependent fp64 gathers per ray.
//              Kept minimal so it runs at the full 8 waves/SIMD; the
//              hardware's wave scheduler does the load balancing of the
//              ragged ray lengths (one ray per lane beat a per-wave ray pool
//              with lane refill by 1.35x at 8192 envs).
//  k_post      one 256-thread workgroup per env: scan -> LDS, TTC, GJK,
//              agent ray_cast, obs packing, _check_done.
//
//  k_scan_batch / k_dynamics: the C-ABI building blocks (f110_scan_batch,
//  f110_dynamics_batch).
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

// trace_ray, laser_models.py:106-146, from the shared first lookup d0 at the
// scan pose.  Returns the clamped range; n = EDT lookups made.
__device__ __forceinline__ double trace(const MapView &m, double x, double y, double c, double s, double d0,
                                        double eps, double max_range, uint32_t &n) {
    double d = d0;       // :129
    double tot = d;      // :130
    uint32_t k = 1;
    while (d > eps && tot <= max_range) {  // :133
        x += d * c;                        // :135
        y += d * s;                        // :136
        d = m.dt[cell_index_fast(m, x, y)];
        tot += d;                          // :141
        ++k;
    }
    n = k;
    return tot > max_range ? max_range : tot;  // :143-144
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

__global__ void __launch_bounds__(64) k_agents(StepArgs a) {
    const int g = blockIdx.x * 64 + threadIdx.x;
    if (a.ev_ctr && blockIdx.x == 0) {  // this step's straggler queue starts empty (k_rays_fx / k_rays_fx_tail)
        for (int p = threadIdx.x; p < a.ev_P; p += 64) {
            a.ev_ctr[p * kEvStride] = 0u;
            a.ev_ctr[p * kEvStride + 1] = 0u;
        }
    }
    const int EA = a.E * a.A;
    const bool valid = g < EA;
    const int A = a.A;
    const int e = valid ? g / A : 0;
    const int ag = g - e * A;
    // Every input of the car is loaded first, before the heavy-list atomic
    // and before anything waits: one memory round trip for the whole prologue.
    double s[7];
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
    if (a.heavy_build) build_heavy_list(a, g, valid);  // block-uniform branch, before any return
    if (!valid) return;
    const uint64_t genv = (uint64_t)(a.env_offset + e);
    int do_reset;
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
                cr_sincos(-pth, sr, crr);
                a.start_rot[e] = crr;
                a.start_rot[a.E + e] = sr;
            }
        }
        a.toggles[g] = 0;
        a.near_start[g] = 1;
        a.lap_times[g] = 0.0f;
        a.lap_counts[g] = 0.0f;
    }
    update_pose(s, b0, b1, cnt, raw_steer, vel, a.pa[ag], a.dt, a.integrator);  // RaceCar.params (per agent)
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
    if (!no_offset) cr_sincos(s[4], sy4, cy4);
    const double sx = no_offset ? s[0] + 0.0 : s[0] + a.lidar_dist * cy4;
    const double sy = no_offset ? s[1] + 0.0 : s[1] + a.lidar_dist * sy4;
    a.ray0[g] = sx;
    a.ray0[EA + g] = sy;
    a.ray0[2 * EA + g] = a.map.dt[cell_index(a.map, sx, sy)];  // first lookup (laser_models.py:129)
    double t0 = first_theta_index(s[4], a.fov, a.theta_dis);
    a.nruns[g] = build_beam_runs(t0, a.inc, a.theta_dis, a.B, a.runs + (size_t)g * kMaxSeg, kMaxSeg);
    a.ttc_hit[g] = 0;
    if (ag == 0) {
        a.reset_flag[e] = (uint8_t)do_reset;
        a.noise_step[e] = do_reset ? 0ull : nstep;
    }
}

// ------------------------------------------------------------------------
// Ray epilogue shared by the ray kernels: clamp, noise, store.
// ScanSimulator2D.scan adds the noise after the clamp (laser_models.py:450-452).
// Caller-supplied noise (f110_set_scan_noise: [E][B], shared by the env's
// agents like the reference's equal-seeded per-car generators,
// base_classes.py:119,204) wins over the device Philox stream.
__device__ __forceinline__ void store_ray(const StepArgs &a, int64_t r, int e, int b, double tot) {
    double range = tot > a.max_range ? a.max_range : tot;  // :143-144
    if (a.noise_ext)
        range += a.noise_ext[(size_t)e * a.B + b];
    else if (a.noise_std > 0.0)
        range += a.noise_std * (double)beam_normal(a.seed, (uint64_t)(a.env_offset + e), a.noise_step[e], b);
    a.scan[r] = range;
}

// k_rays: one thread per ray (ray r -> car g = r / B, beam b = r % B) on the
// row-major EDT.  Kept as the A/B baseline of k_rays_tiled (F110_RAY_KERNEL=0);
// the two produce identical results.
__global__ void __launch_bounds__(kBlock) k_rays(StepArgs a) {
    const int EA = a.E * a.A;
    const int B = a.B;
    const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t n = 0;
    if (r < (int64_t)EA * B) {
        const int g = (int)(r / B);
        const int b = (int)(r - (int64_t)g * B);
        const int e = g / a.A;
        if (!(a.mode == 1 && a.reset_mask && !a.reset_mask[e])) {
            double t = beam_theta_index(a.runs + (size_t)g * kMaxSeg, a.nruns[g], b);
            int ti = (int)t;  // int(theta_index), laser_models.py:124
            if (ti >= a.theta_dis) ti = 0;
            double tot = trace(a.map, a.ray0[g], a.ray0[EA + g], a.cosines[ti], a.sines[ti], a.ray0[2 * EA + g],
                               a.eps, a.max_range, n);
            store_ray(a, r, e, b, tot);
        }
    }
    if (a.ctr) count_rays(a.ctr, n);
}

// The RayArgs block in the kernarg segment (k_rays_tiled's only argument).
__device__ __forceinline__ const RayArgs *kernarg_rays() {
#if defined(__HIP_DEVICE_COMPILE__)
    return reinterpret_cast<const RayArgs *>(__builtin_amdgcn_kernarg_segment_ptr());
#else
    return nullptr;
#endif
}

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
    double c = 0.0, s = 0.0, x = 0.0, y = 0.0, d = 0.0, v = 0.0, bcos = 0.0, side = 0.0, noise = 0.0;
    if (has) {
        double t = beam_theta_index(a.runs + (size_t)g * kMaxSeg, a.nruns[g], b);
        int ti = (int)t;  // int(theta_index), laser_models.py:124
        if (ti >= a.theta_dis) ti = 0;
        c = a.cosines[ti];
        s = a.sines[ti];
        x = a.ray0[g];
        y = a.ray0[a.EA + g];
        d = a.ray0[2 * a.EA + g];  // :129
        // the TTC operands are loaded before the loop, which hides their
        // latency (the epilogue would otherwise wait on them)
        v = a.vel[g];
        bcos = a.beam_cos[b];
        side = a.side[b];
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
    if (v != 0.0 && ttc_fires(range, side, v * bcos, K.ttc_thresh)) K.ttc_hit[g] = 1;
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

// The fixed-point loop's EDT layouts.  FMT 0: the 4x4-tiled table shared
// with the other ray kernels: fx_offset<0> is tiled_offset_u24 with the
// tile-row stride k1 = wt * 128 in an SGPR, (row >> 2) * k1 + (col << 5 |
// (row & 3) << 3) -- 5 integer ops (24-bit multiply: row >> 2 < 2^19 and
// k1 < 2^24 on the fixed-point path; off-map lanes compute garbage that the
// caller's select discards).  FMT 3: the row-major table of k_rays_fx /
// k_rays_fxn (StepArgs::rm), rows of k1 = wt * 8 bytes: row * k1 + col * 8,
// and off-map indices are clamped into the padding, which holds dt[-1,-1],
// instead of selected.  Measured at 65536 envs: FMT 3 1.184 vs
// FMT 0 1.210 ms; an inexact f32 8x4-tiled or u16 8x8-tiled table (4x the
// cells per cache line) gained only 2-3 %: the gathers' line footprint is not
// what bounds the loop.
template <int FMT>
__device__ __forceinline__ uint32_t fx_offset(uint32_t k1, uint32_t row, uint32_t col) {
    static_assert(FMT == 0 || FMT == 3, "EDT layout");
    if (FMT == 0) return __umul24(row >> 2, k1) + ((col << 5) | ((row & 3u) << 3));
    return __umul24(row, k1) + (col << 3);
}

template <int FMT>
__device__ __forceinline__ double fx_load(const void *base, uint32_t off) {
    return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(base) + off);
}

// tiled_cell's IEEE path as a byte offset (the fixed-point path's fallback)
template <int FMT>
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
    return r >= m.H ? oob8 : fx_offset<FMT>((uint32_t)m.wt * (FMT == 3 ? 8u : 128u), (uint32_t)r, (uint32_t)c);
}

// Loop-invariant state of the fixed-point sphere trace.
struct FxLoop {
    double cxk, cyk, ir, mr;
    uint32_t oobv, W, H, k1;
};

template <int FMT = 0>
__device__ __forceinline__ FxLoop fx_loop(const RayArgs &a) {
    FxLoop L;
    // the off-map offset and inv_res in VGPRs for the whole trace (opaque
    // copies: the select cannot read an SGPR beside its VCC condition, and the
    // fma's other operand is an SGPR constant, a VOP3 reads one SGPR); the
    // row-major layout carries the off-map byte offset itself in m.oob
    asm volatile("v_mov_b32 %0, %1" : "=v"(L.oobv) : "s"(FMT == 0 ? (uint32_t)a.m.oob << 3 : (uint32_t)a.m.oob));
    asm volatile("v_mov_b64 %0, %1" : "=v"(L.ir) : "s"(a.m.inv_res));
    L.cxk = a.fx_cx;
    L.cyk = a.fx_cy;
    L.mr = a.max_range;
    L.W = (uint32_t)a.m.W;
    L.H = (uint32_t)a.m.H;
    L.k1 = (uint32_t)a.m.wt * 128u;  // tile-row stride of fx_offset (bytes)
    if (FMT == 3) {  // row-major rows of m.wt cells; columns W .. wt-1 and row H hold dt[-1,-1]
        L.W = (uint32_t)a.m.wt - 1u;
        L.k1 = (uint32_t)a.m.wt * 8u;
    }
    return L;
}

// One iteration of trace_ray's loop (laser_models.py:135-141) for an active
// lane: step, fixed-point cell, EDT lookup.
template <int FMT = 0>
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
    const uint32_t fast = fx_offset<FMT>(L.k1, row, col);
    const uint32_t sel = 0u - (uint32_t)inb;
    uint32_t off = (fast & sel) | (L.oobv & ~sel);
    if (__builtin_amdgcn_ballot_w64(near)) {  // wave-uniform, rare
        if (near) off = exact_offset<FMT>(m, x, y, L.oobv);
    }
    d = fx_load<FMT>(m.dt, off);
    tot += d;  // :141
}

// fx_step for a car whose rays cannot leave t's binade (SAFE: the scan
// origin lies within 2^21 - 16 cells of the map origin, less the max range;
// every lookup of a ray is within max_range of its origin, since the loop
// steps only while tot <= max_range): the sign / exponent tests drop out and
// the column and row tests are one unsigned compare each.
template <int FMT>
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
    uint32_t off;
    if (FMT == 3) {  // clamped into the padding, which holds dt[-1,-1]: no bounds select
        off = fx_offset<3>(L.k1, min(row, L.H), min(col, L.W));
    } else {
        const bool inb = (col < L.W) & (row < L.H);
        const uint32_t sel = 0u - (uint32_t)inb;  // a select, not an exec-mask branch
        off = (fx_offset<FMT>(L.k1, row, col) & sel) | (L.oobv & ~sel);
    }
    if (__builtin_amdgcn_ballot_w64(near)) {  // wave-uniform, rare
        if (near) off = exact_offset<FMT>(m, x, y, L.oobv);
    }
    d = fx_load<FMT>(m.dt, off);
    tot += d;  // :141
}

// fx_step_safe<3>'s cell offset of the position (x, y).
__device__ __forceinline__ uint32_t fx_safe_offset3(const TiledMapView &m, const FxLoop &L, double x, double y) {
    double tx, ty;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tx) : "v"(x), "v"(L.ir), "s"(L.cxk));
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(ty) : "v"(y), "v"(L.ir), "s"(L.cyk));
    const uint32_t lx = dlo(tx), ly = dlo(ty);
    const uint32_t col = __builtin_amdgcn_alignbit(dhi(tx), lx, 30) - kFxU0;
    const uint32_t row = __builtin_amdgcn_alignbit(dhi(ty), ly, 30) - kFxU0;
    const bool near = ((lx << 2) + 4u * kFxBand < 8u * kFxBand) | ((ly << 2) + 4u * kFxBand < 8u * kFxBand);
    uint32_t off = fx_offset<3>(L.k1, min(row, L.H), min(col, L.W));  // clamped into the padding
    if (__builtin_amdgcn_ballot_w64(near)) {  // wave-uniform, rare
        if (near) off = exact_offset<3>(m, x, y, L.oobv);
    }
    return off;
}

// SPEC: fx_step_safe<3> that also guesses the ray's next K - 1 steps.  Where
// the EDT value repeats along a ray (a ray running beside a wall), its next
// positions are x + d c, (x + d c) + d c, ... -- the same sequence of adds
// as the serial loop's -- so their cells are gathered together with this
// step's.  The guesses are checked in order: step j + 1 is kept only while
// every earlier lookup returned d itself and the ray goes on (tot <= mr; a
// lookup equal to d != 0 is not the end).  The kept positions and totals are
// the serial loop's bit for bit: only the chain of dependent gathers is
// shorter.  Every guessed offset is clamped into the table like any other.
// Returns the steps taken (the lookups that count).
template <int K>
__device__ __forceinline__ uint32_t fx_step_spec(const TiledMapView &m, const FxLoop &L, double &x, double &y,
                                                 double &d, double &tot, double c, double s) {
    const double d0 = d;
    double xs[K], ys[K], dd[K];
    uint32_t off[K];
    double xc = x, yc = y;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        xc += d0 * c;  // :135
        yc += d0 * s;  // :136
        xs[j] = xc;
        ys[j] = yc;
        off[j] = fx_safe_offset3(m, L, xc, yc);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) dd[j] = fx_load<3>(m.dt, off[j]);
    uint32_t n = 0;
    bool go = true;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (go) {
            x = xs[j];
            y = ys[j];
            d = dd[j];
            tot += d;  // :141
            ++n;
            go = (d == d0) & (tot <= L.mr);
        }
    }
    return n;
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
                                            double noise, double v, double bcos, double side) {
    const int64_t r = (int64_t)g * K.B + b;
    double range = tot > mr ? mr : tot;
    if (K.noise_ext || K.noise_std > 0.0) range += noise;
    if (v != 0.0 && ttc_fires(range, side, v * bcos, K.ttc_thresh)) K.ttc_hit[g] = 1;
    if (K.obs && g == e * K.A) K.obs[(size_t)e * K.obs_len + b] = obs_scan_value(range, K.lidar_max);
    if (K.scans_f32) K.scans_f32[r] = (float)range;
    if (K.scans_f64) K.scans_f64[r] = range;
    if (HANDOFF) K.scan[r] = range;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {  // set bits of mask below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// EVICT: straggler hand-off.  A wave's longest ray sets its length while
// most lanes idle (SIMT efficiency 0.55).  Once <= ev_T of its
// rays are still tracing after >= ev_K iterations, the wave writes their
// state (x, y, d, tot, cos, sin, noise, car, beam: the whole loop state) to
// the hand-off queue and ends; k_rays_fx_tail finishes them with lane refill.
// The state is exact, so the results are those of the uninterrupted loop.
//
// LEAN (every launch but the EVICT and A/B ones): lanes whose ray has ended
// leave the loop (exec mask) instead of a ballot + select per iteration,
// each lane counts its own lookups (summed once per wave), and cars whose
// rays stay in t's binade take fx_step_safe: ~36 instead of ~59 instructions
// per iteration on the wave's serial path (the kernel is latency-bound: at
// 6 / 4 / 2 waves per SIMD it takes 1.31x / 1.62x / 2.9x as long).
//
// SPEC (F110_FX_SPEC=K:T, row-major table, A/B): once <= fx_spec_t lanes of
// the wave still trace, each iteration takes fx_step_spec<SPEC>.
template <bool MASK, bool HANDOFF, bool EVICT, int FMT = 0, bool LEAN = !EVICT, int SPEC = 1>
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
    const double bcos = a.beam_cos[bc], side = a.side[bc];
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
    const FxLoop L = fx_loop<FMT>(a);
    double tot = d;  // :130 (lanes without a ray: d = 0, never traced)
    uint32_t iters = 0, lane_iters = 0;
    bool evicted = false, can_evict = EVICT;
    if (LEAN) {
        uint32_t cnt = 0;
        const double qx = fma(x00, L.ir, L.cxk) - kFxMagic, qy = fma(y00, L.ir, L.cyk) - kFxMagic;
        __builtin_amdgcn_s_waitcnt(0);  // the set-up loads (c, s) land before the loop, not in it
        if (SPEC > 1 && FMT == 3 && fabs(qx) < a.fx_lim && fabs(qy) < a.fx_lim) {
            const uint32_t T = (uint32_t)a.fx_spec_t;
            while ((dhi(d) != 0u) & (tot <= L.mr)) {
                if ((uint32_t)__popcll(__builtin_amdgcn_ballot_w64(true)) <= T) {  // wave-uniform: the tail
                    cnt += fx_step_spec<SPEC>(a.m, L, x, y, d, tot, c, s);
                } else {
                    fx_step_safe<FMT>(a.m, L, x, y, d, tot, c, s);
                    ++cnt;
                }
            }
        } else if (fabs(qx) < a.fx_lim && fabs(qy) < a.fx_lim) {  // wave-uniform (false for NaN)
            while ((dhi(d) != 0u) & (tot <= L.mr)) {
                fx_step_safe<FMT>(a.m, L, x, y, d, tot, c, s);
                ++cnt;
            }
        } else {
            while ((dhi(d) != 0u) & (tot <= L.mr)) {
                fx_step<FMT>(a.m, L, x, y, d, tot, c, s);
                ++cnt;
            }
        }
        lane_iters = wave_sum(cnt);
        if (a.wcost || a.count_slots) iters = wave_max(cnt);  // the wave's trip count (heavy-first cost, SIMT counter)
    }
    for (; !LEAN;) {
        const bool act = (dhi(d) != 0u) & (tot <= L.mr);
        const uint64_t mk = __builtin_amdgcn_ballot_w64(dhi(d) != 0u) & __builtin_amdgcn_ballot_w64(tot <= L.mr);
        if (!mk) break;
        if (EVICT && can_evict && iters >= (uint32_t)a.ev_K && (uint32_t)__popcll(mk) <= (uint32_t)a.ev_T) {
            const RayArgs &K = *kernarg_rays();
            const uint32_t cnt = (uint32_t)__popcll(mk);
            const uint32_t part = blockIdx.x % (uint32_t)K.ev_P;
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(K.ev_ctr + part * kEvStride, cnt);
            base = __builtin_amdgcn_readfirstlane(base);
            if (base + cnt <= K.ev_capp) {
                if (act) {
                    const size_t i = (size_t)part * K.ev_capp + base + lanes_below(mk), C = K.ev_cap;
                    K.ev[i] = x;
                    K.ev[C + i] = y;
                    K.ev[2 * C + i] = d;
                    K.ev[3 * C + i] = tot;
                    K.ev[4 * C + i] = c;
                    K.ev[5 * C + i] = s;
                    K.ev[6 * C + i] = noise;
                    K.ev_gb[i] = g;
                    K.ev_gb[C + i] = b;
                    evicted = true;
                }
                break;
            }
            can_evict = false;  // queue full: this wave finishes its rays itself
        }
        ++iters;
        lane_iters += (uint32_t)__popcll(mk);
        if (act) fx_step<FMT>(a.m, L, x, y, d, tot, c, s);
    }

    // ---- epilogue ----
    const uint32_t lanes = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(has));
    if (has && !evicted) fx_epilogue<HANDOFF>(*kernarg_rays(), g, e, b, tot, L.mr, noise, v, bcos, side);
    if (lane == 0) {
        const RayArgs &K = *kernarg_rays();
        if (lanes) {  // one (lookups, rays) atomic pair per wave; the first lookup came from k_agents
            unsigned long long *slot = K.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
            atomicAdd(slot, (unsigned long long)(lanes + lane_iters));
            atomicAdd(slot + 1, (unsigned long long)lanes);
            if (K.count_slots) atomicAdd(slot + 2, (unsigned long long)iters * 64ull);  // lane slots the loop issued (SIMT)
        }
        if (K.wcost) {  // this wave's cost, the next step's heavy-first prediction
            const uint32_t mx = lanes ? 1u + iters : 0u;
            K.wcost[(size_t)g * a.nch + k] = (uint8_t)(mx < 255u ? mx : 255u);
        }
    }
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
    uint32_t fast = fx_offset<3>(L.k1, min(row, L.H), min(col, L.W));
    asm volatile("" : "+v"(fast));  // computed for every lane, then selected (no exec-mask branch)
    uint32_t off = act ? fast : zero;
    if (__builtin_amdgcn_ballot_w64(band < 8u * kFxBand) & amask) {  // wave-uniform, rare
        if (act & (band < 8u * kFxBand)) off = exact_offset<3>(m, x, y, L.oobv);
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
// dt[-1,-1] in the padding column / row (FMT 3).  Bit-identical to k_rays_fx.
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
    const FxLoop L = fx_loop<3>(a);
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
            for (int r = 0; r < N; ++r) d[r] = fx_load<3>(a.m.dt, off[r]);
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
                    d[r] = fx_load<3>(a.m.dt, exact_offset_pad(a.m, x[r], y[r], P));
                    tot[r] += d[r];  // :141
                } else {
                    fx_step<3>(a.m, L, x[r], y[r], d[r], tot[r], c[r], sn[r]);
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
            fx_epilogue<HANDOFF>(K, g, e, b0 + 64 * r + lane, tot[r], L.mr, nz, v, a.beam_cos[bc[r]], a.side[bc[r]]);
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
}

// k_rays_fxr (F110_FX_REFILL): one wave per car, whose 64-beam chunks are
// traced two at a time with refill.  k_rays_fxn pairs adjacent chunks, and
// a pair costs the longer chunk's trip count while the other slot idles; here
// a slot whose chunk has ended writes that chunk's outputs and takes the
// car's next chunk at once, so both slots keep gathers in flight until the
// car's last chunk.  Offline model over oracle trip counts
// (scripts/pair_model.py): 146.7k wave-iterations for adjacent pairs vs
// 109.1k (116.5k with one iteration of re-arm per chunk).  Same per-ray
// arithmetic as k_rays_fxn, so bit-identical.  No heavy-first (one wave per
// car), no masked reset; cars whose rays could leave t's binade trace their
// chunks one after the other with fx_step.
__device__ __forceinline__ double beam_theta(const BeamRun *R, int n, int lo, int b0, int bc) {
    // lo: the run holding beam b0 (found once per car for all its chunks, see k_rays_fxr)
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

template <bool HANDOFF, bool PAD = false, int NS = 2>
__global__ void __launch_bounds__(64, 8) k_rays_fxr(RayArgs a) {  // 8 waves per SIMD: <= 64 VGPRs
    // a.G4 waves per car: wave j takes the car's chunks nch-1-j, nch-1-j-G4, ... (car-minor
    // block order: car g's waves run on XCD g % 8 when EA % 8 == 0)
    const int wj = (int)blockIdx.x / a.EA;
    const int g = (int)blockIdx.x - wj * a.EA;
    const int lane = (int)threadIdx.x;
    const int B = a.B;
    const int e = HANDOFF ? g / a.A : g;
    const int nch = (B + 63) >> 6;
    const int wstride = a.G4;
    const BeamRun *R = a.runs + (size_t)g * kMaxSeg;
    const int n = ld_const(a.nruns + g);
    const double x00 = ld_const(a.ray0 + g), y00 = ld_const(a.ray0 + a.EA + g);
    const double d00 = ld_const(a.ray0 + 2 * a.EA + g);  // :129
    const RayArgs &K = *kernarg_rays();
    const FxLoop L = fx_loop<3>(a);
    const uint32_t zero = a.fx_zero;

    // slot r traces chunk kk[r] (-1: empty); lane l owns beam kk[r] * 64 + l
    double x[NS], y[NS], d[NS], tot[NS], c[NS], sn[NS];
    int kk[NS];
    int next = nch - 1 - wj;  // this wave's chunks, taken in descending order
    // lane k < nch: the run holding beam 64 k (one divergent search per car instead of
    // a dependent chain of scalar loads at every re-arm)
    int vlo = 0;
    if (lane < nch) {
        int lo = 0, hi = n - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (R[mid].start <= lane * 64) lo = mid;
            else hi = mid - 1;
        }
        vlo = lo;
    }
    // in_loop: the loop's closing `tot += d` completes tot = d (:130) in the
    // iteration that re-arms the slot, so the total is updated there without a select
    auto arm = [&](int r, bool in_loop) {
        const int k = next;
        next -= wstride;
        kk[r] = k;
        const int b = k * 64 + lane, bc = b < B ? b : B - 1;
        const int lo = __builtin_amdgcn_readlane(vlo, k);
        int ti = (int)beam_theta(R, n, lo, k * 64, bc);  // int(theta_index), :124
        if (ti >= a.theta_dis) ti = 0;
        c[r] = a.cosines[ti];
        sn[r] = a.sines[ti];
        x[r] = x00;
        y[r] = y00;
        d[r] = b < B ? d00 : 0.0;
        tot[r] = in_loop ? 0.0 : d[r];  // :130
    };
    uint32_t lanes = 0;
    // device noise: chunks 2p and 2p + 1 (beams b and b + 64 of a 128-beam block) share one
    // Philox draw (beam_normal_pair_k); the half a finished chunk does not use is kept for its
    // partner in a two-entry cache indexed by p & 1 (the open pairs are p and p - 1: the
    // slots take the car's chunks in descending order), so most pairs are drawn once
    float cval[2] = {0.0f, 0.0f};
    int ctag[2] = {-1, -1};
    auto finish = [&](int r) {  // the ended chunk's outputs (fx_epilogue, noise after the clamp)
        const int b = kk[r] * 64 + lane, bc = b < B ? b : B - 1;
        double nz = 0.0;
        if (K.noise_ext) {
            nz = K.noise_ext[(size_t)e * B + bc];
        } else if (K.noise_std > 0.0) {
            const int pp = kk[r] >> 1, ci = pp & 1;
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
        if (b < B)
            fx_epilogue<HANDOFF>(K, g, e, b, tot[r], L.mr, nz, ld_const(a.vel + g), a.beam_cos[bc], a.side[bc]);
        lanes += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(b < B));
    };

    uint32_t lane_iters = 0, iters = 0;
    bool fast_car;  // wave-uniform (false for NaN)
    if (PAD) {  // q + P of the scan origin inside [fxp_lo, fxp_h*): its rays stay in the padded table
        const double ux = fma(x00, L.ir, L.cxk) - kFxpBase, uy = fma(y00, L.ir, L.cyk) - kFxpBase;
        fast_car = (ux >= a.fxp_lo) & (ux < a.fxp_hx) & (uy >= a.fxp_lo) & (uy < a.fxp_hy);
    } else {
        const double qx = fma(x00, L.ir, L.cxk) - kFxMagic, qy = fma(y00, L.ir, L.cyk) - kFxMagic;
        fast_car = fabs(qx) < a.fx_lim && fabs(qy) < a.fx_lim;
    }
    const uint32_t P = (uint32_t)a.fxp_P;
    uint32_t zero_v = zero;  // PAD: in a VGPR for the whole trace (the select's other operand is its SGPR mask)
    if (PAD) asm volatile("v_mov_b32 %0, %1" : "=v"(zero_v) : "s"(zero));
    if (fast_car) {
#pragma unroll
        for (int r = 0; r < NS; ++r) {
            kk[r] = -1;
            d[r] = tot[r] = x[r] = y[r] = c[r] = sn[r] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < NS; ++r)
            if (next >= 0) arm(r, false);
        __builtin_amdgcn_s_waitcnt(0);
        for (;;) {
            uint64_t m[NS], mall = 0;
#pragma unroll
            for (int r = 0; r < NS; ++r)
                m[r] = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
            // the running slots' gathers go out first, so that they are in flight while
            // an ended slot writes its chunk and re-arms (scalar run search, table loads).
            // The gather lands in d[r] itself: a lane whose ray has ended reads the zero
            // cell, so d = 0 keeps its total (no per-lane select of old and new values)
#pragma unroll
            for (int r = 0; r < NS; ++r)
                if (m[r]) {
                    const bool act = (dhi(d[r]) != 0u) & (tot[r] <= L.mr);
                    const uint32_t off = PAD ? fxp_offset(a.m, L, x[r], y[r], d[r], c[r], sn[r], act, m[r], zero_v, P)
                                             : fxn_offset(a.m, L, x[r], y[r], d[r], c[r], sn[r], act, m[r], zero);
                    d[r] = fx_load<3>(a.m.dt, off);
                }
#pragma unroll
            for (int r = 0; r < NS; ++r) {
                mall |= m[r];
                lane_iters += (uint32_t)__popcll(m[r]);
            }
            const bool any = mall != 0;
            iters += any ? 1u : 0u;
            bool open = false;
#pragma unroll
            for (int r = 0; r < NS; ++r)
                if (kk[r] >= 0 && !m[r]) {  // wave-uniform: the chunk has ended; refill the slot
                    finish(r);
                    if (next >= 0) arm(r, true);
                    else kk[r] = -1;
                }
            // :141 for every slot: a running slot's ended lanes read d = 0, a re-armed slot
            // completes tot = d00, a closed slot's total is no longer read
#pragma unroll
            for (int r = 0; r < NS; ++r) {
                tot[r] += d[r];  // :141
                open |= kk[r] >= 0;
            }
            if (!any && !open) break;
        }
    } else {
        uint32_t cnt = 0;
        while (next >= 0) {
            arm(0, false);
            while ((dhi(d[0]) != 0u) & (tot[0] <= L.mr)) {
                if (PAD) {  // an origin off the map: the IEEE cell of every lookup
                    x[0] += d[0] * c[0];  // :135
                    y[0] += d[0] * sn[0];  // :136
                    d[0] = fx_load<3>(a.m.dt, exact_offset_pad(a.m, x[0], y[0], P));
                    tot[0] += d[0];  // :141
                } else {
                    fx_step<3>(a.m, L, x[0], y[0], d[0], tot[0], c[0], sn[0]);
                }
                ++cnt;
            }
            finish(0);
        }
        lane_iters = wave_sum(cnt);
        iters = wave_max(cnt);
    }
    if (lane == 0) {
        unsigned long long *cs = K.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
        atomicAdd(cs, (unsigned long long)(lanes + lane_iters));  // the first lookup came from k_agents
        atomicAdd(cs + 1, (unsigned long long)lanes);
        if (K.count_slots) atomicAdd(cs + 2, (unsigned long long)iters * (fast_car ? 64ull * NS : 64ull));
    }
}

// The kernarg block behind an opaque copy of its pointer: loads through it
// stay where they are written (in the refill pass) instead of being hoisted
// out of the trace loop into SGPRs, which would spill there.
// an opaque SGPR copy of a pointer to read-only kernel arguments, typed in the
// constant address space: its field loads are scalar loads placed at the use
// (a generic pointer out of the asm would make them flat vector loads)
template <class T>
__device__ __forceinline__ const T *launder_const(const T *ptr) {
    const __attribute__((address_space(4))) T *p;
    asm volatile("s_mov_b64 %0, %1" : "=s"(p) : "s"(ptr));
    return (const T *)p;
}

__device__ __forceinline__ const RayArgs &kernarg_here() { return *launder_const(kernarg_rays()); }

__device__ __forceinline__ bool lane_in(uint64_t mask) {
    return (uint32_t)(mask >> (threadIdx.x & 63)) & 1u;
}

// ------------------------------------------------------------------------
// k_rays_fxs: k_rays_fxr<HANDOFF, PAD = true, 2> with a lean refill pass (the
// default where k_rays_fxr runs; F110_FXR_LEAN=0 for the round-3 kernel).
// A chunk's finish / re-arm pass was ~176 VALU per chunk, 43 % of the
// kernel's VALU.  Here:
// - nothing the pass or the rare IEEE cell path reads is held in SGPRs across
//   the loop (kernel arguments are re-read at the use through kernarg_here,
//   the scan origin and first lookup sit in VGPRs): no SGPR spills into VGPR
//   lanes (k_rays_fxr: 92 v_readlane / v_writelane);
// - table loads and the obs store take 32-bit lane offsets from an SGPR base
//   (saddr form) instead of 64-bit address arithmetic;
// - the obs entry's f32 division by lidar_max is q = v * y, r = fma(-q, lm, v),
//   q' = fma(r, y, q) with y = RN(1 / lm): q is within one ulp of v / lm, so
//   q' is the correctly rounded quotient (Markstein's theorem) when no
//   intermediate is subnormal; lanes with v < 2^-60 (and lidar_max outside
//   [2^-30, 2^30], obs_rinv = 0) take the IEEE divide.  Checked exhaustively
//   against the divide for every f32 v in [0, lm] (tests/test_host_lib.py).
// Same per-ray arithmetic as k_rays_fxr, so bit-identical.
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

// fxp_offset with the rare IEEE path's map fields read from the kernel
// arguments at the use (not held in SGPRs across the loop)
__device__ __forceinline__ uint32_t fxs_offset(const FxLoop &L, double &x, double &y, double d, double c, double s,
                                               bool act, uint64_t amask, uint32_t zero_v) {
    x += d * c;  // :135
    y += d * s;  // :136
    double tx, ty;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tx) : "v"(x), "v"(L.ir), "s"(L.cxk));
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(ty) : "v"(y), "v"(L.ir), "s"(L.cyk));
    const uint32_t lx = dlo(tx), ly = dlo(ty);
    const uint32_t col = __builtin_amdgcn_alignbit(dhi(tx), lx, 28);
    const uint32_t row = __builtin_amdgcn_alignbit(dhi(ty), ly, 28);
    const uint32_t band = min((lx << 4) + 16u * kFxpBand, (ly << 4) + 16u * kFxpBand);
    const uint32_t prow = __umul24(row, L.k1);
    uint32_t fast;
    asm volatile("v_mad_u32_u24 %0, %1, 8, %2" : "=v"(fast) : "v"(col), "v"(prow));
    uint32_t off = act ? fast : zero_v;
    if (__builtin_amdgcn_ballot_w64(band < 32u * kFxpBand) & amask) {  // wave-uniform, rare
        const RayArgs &K = kernarg_here();
        if (act & (band < 32u * kFxpBand)) off = exact_offset_pad(K.m, x, y, (uint32_t)K.fxp_P);
    }
    return off;
}

// fxs_offset without the rare branch: the fixed-point offset (the zero cell's
// for an ended ray) and whether the lane lies within the guard band of a cell
// edge (the caller takes the IEEE path for those lanes, both slots at once)
// (kFxsBase: the high dwords of t feed the u24 multiplies directly, the low
// dwords hold the shifted fractions; cx / cy are RayArgs::fxs_cx / fxs_cy)
__device__ __forceinline__ uint32_t fxs_offset_nb(const FxLoop &L, double cx, double cy, double &x, double &y,
                                                  double d, double c, double s, bool act, uint32_t zero_v,
                                                  bool &near) {
    x += d * c;  // :135
    y += d * s;  // :136
    double tx, ty;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tx) : "v"(x), "v"(L.ir), "s"(cx));
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(ty) : "v"(y), "v"(L.ir), "s"(cy));
    near = min(dlo(tx), dlo(ty)) < 2u * kFxsBand;
    const uint32_t prow = __umul24(dhi(ty), L.k1);
    uint32_t fast;
    asm volatile("v_mad_u32_u24 %0, %1, 8, %2" : "=v"(fast) : "v"(dhi(tx)), "v"(prow));
    return act ? fast : zero_v;
}

// ML (F110_FXS_MASKLD, PIPE only), 1: the slot gathers are buffer loads through a
// descriptor whose range ends at the zero cell, so an ended lane's zero-cell offset fails
// the range check: it reads 0.0 as before, without a cache access of its own.  2: an ended
// lane issues no gather at all (exec mask) and keeps its d: a ray ended by its range then
// goes on adding d to a total past max_range, which the clamp (:143-144) maps to max_range
// all the same.  3 (lock-step slots, F110_FXS_PIPE=0): a trip in which no lane has both
// slots' rays active issues one gather for the two slots.
// PK (F110_FXS_PACK): the arm's (cos, sin) and the epilogue's (side, beam_cos) as one 16-byte
// load each from the interleaved tables RayArgs::cs2 / bs2.
template <bool HANDOFF, int NS, bool PIPE = false, int ML = 0, bool PK = false>
__global__ void __launch_bounds__(64, NS == 2 ? 8 : 7) k_rays_fxs(RayArgs a) {  // <= 64 / 72 VGPRs
    const int wj = (int)blockIdx.x / a.EA;
    const int g = (int)blockIdx.x - wj * a.EA;
    const int lane = (int)threadIdx.x;
    const int B = a.B;
    const int e = HANDOFF ? g / a.A : g;
    const int nch = (B + 63) >> 6;
    const int wstride = a.G4;
    const double *dt = a.m.dt;
    const FxLoop L = fx_loop<3>(a);
    // the scan origin and first lookup in VGPRs (re-arm copies them into a slot)
    double x00, y00, d00;
    asm volatile("v_mov_b64 %0, %1" : "=v"(x00) : "s"(ld_const(a.ray0 + g)));
    asm volatile("v_mov_b64 %0, %1" : "=v"(y00) : "s"(ld_const(a.ray0 + a.EA + g)));
    asm volatile("v_mov_b64 %0, %1" : "=v"(d00) : "s"(ld_const(a.ray0 + 2 * a.EA + g)));  // :129
    uint32_t zero_v;  // the zero cell's offset in a VGPR (the select's other operand is its SGPR mask)
    asm volatile("v_mov_b32 %0, %1" : "=v"(zero_v) : "s"(a.fx_zero));

    double x[NS], y[NS], d[NS], tot[NS], c[NS], sn[NS];
    int kk[NS];
    int next = nch - 1 - wj;
    int vlo = 0;  // lane k < nch: the run holding beam 64 k (as k_rays_fxr)
    if (lane < nch) {
        const BeamRun *R = a.runs + (size_t)g * kMaxSeg;
        int lo = 0, hi = ld_const(a.nruns + g) - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (R[mid].start <= lane * 64) lo = mid;
            else hi = mid - 1;
        }
        vlo = lo;
    }
    auto arm = [&](int r, bool in_loop) {
        const RayArgs &K = kernarg_here();
        const int k = next;
        next -= wstride;
        kk[r] = k;
        const int b = k * 64 + lane, bc = b < B ? b : B - 1;
        const int lo = __builtin_amdgcn_readlane(vlo, k);
        int ti = (int)beam_theta(K.runs + (size_t)g * kMaxSeg, ld_const(K.nruns + g), lo, k * 64, bc);  // :124
        if (ti >= K.theta_dis) ti = 0;
        if (PK) {  // one 16-byte load (F110_FXS_PACK)
            const double2 t2 = ld_off(reinterpret_cast<const double2 *>(K.cs2), (uint32_t)ti * 16u);
            c[r] = t2.x;
            sn[r] = t2.y;
        } else {
            c[r] = ld_off(K.cosines, (uint32_t)ti * 8u);
            sn[r] = ld_off(K.sines, (uint32_t)ti * 8u);
        }
        x[r] = x00;
        y[r] = y00;
        d[r] = b < B ? d00 : 0.0;
        tot[r] = in_loop ? 0.0 : d[r];  // :130
    };
    uint32_t lanes = 0;
    float cval[2] = {0.0f, 0.0f};  // k_rays_fxr's two-entry cache of the unused half of a pair draw (tagged:
    // with three slots a third open pair may evict an entry; its partner then draws again)
    int ctag[2] = {-1, -1};
    auto finish = [&](int r) {
        const RayArgs &K = kernarg_here();
        const int b = kk[r] * 64 + lane;
        const bool inb = b < B;
        const int bc = inb ? b : B - 1;
        double nz = 0.0;
        if (K.noise_ext) {
            nz = K.noise_ext[(size_t)e * B + bc];
        } else if (K.noise_std > 0.0) {
            const int pp = kk[r] >> 1, ci = pp & 1;
            float nv;
            if (ctag[ci] == pp) {
                nv = cval[ci];
                ctag[ci] = -1;
            } else {
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
                double sd, bcs;
                if (PK) {  // one 16-byte load (F110_FXS_PACK)
                    const double2 t2 = ld_off(reinterpret_cast<const double2 *>(K.bs2), boff * 2u);
                    sd = t2.x;
                    bcs = t2.y;
                } else {
                    sd = ld_off(K.side, boff);
                    bcs = ld_off(K.beam_cos, boff);
                }
                if (ttc_fires(range, sd, v * bcs, K.ttc_thresh)) K.ttc_hit[g] = 1;
            }
            if (K.obs && (!HANDOFF || g == e * K.A)) {
                float *orow = K.obs + (size_t)e * K.obs_len;
                *reinterpret_cast<float *>(reinterpret_cast<char *>(orow) + (uint32_t)b * 4u) =
                    obs_scan_value_fast(range, K.lidar_max, K.obs_rinv);
            }
            const size_t row = (size_t)g * B;
            if (K.scans_f32) *reinterpret_cast<float *>(reinterpret_cast<char *>(K.scans_f32 + row) + (uint32_t)b * 4u) = (float)range;
            if (K.scans_f64) *reinterpret_cast<double *>(reinterpret_cast<char *>(K.scans_f64 + row) + (uint32_t)b * 8u) = range;
            if (HANDOFF) *reinterpret_cast<double *>(reinterpret_cast<char *>(K.scan + row) + (uint32_t)b * 8u) = range;
        }
        lanes += (uint32_t)min(64, B - kk[r] * 64);  // the chunk's beams (scalar)
    };

    uint32_t lane_iters = 0, iters = 0;
    const double ux = fma(ld_const(a.ray0 + g), L.ir, L.cxk) - kFxpBase;
    const double uy = fma(ld_const(a.ray0 + a.EA + g), L.ir, L.cyk) - kFxpBase;
    // q + P of the scan origin inside [fxp_lo, fxp_h*): its rays stay in the padded table (false for NaN)
    const bool fast_car = (ux >= a.fxp_lo) & (ux < a.fxp_hx) & (uy >= a.fxp_lo) & (uy < a.fxp_hy);
    // ML: the table's descriptor, records up to (not including) the zero cell
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)dt, (short)0, (int)a.fx_zero, 0x00020000);
    if (fast_car && PIPE) {
        // Software-pipelined slots: each slot's gather is waited for right before that slot's
        // next step, so one slot's gather is in flight while the other slot's data is consumed
        // (the compiler's waits are vmcnt(1): both slots gather every trip, a closed slot on
        // the zero cell).  Per slot and trip: the total (:141), the activity test (:133), the
        // refill when the slot's chunk has ended, the step (:135-136) and its gather.
#pragma unroll
        for (int r = 0; r < NS; ++r) {
            kk[r] = -1;
            d[r] = tot[r] = x[r] = y[r] = c[r] = sn[r] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < NS; ++r)
            if (next >= 0) arm(r, true);  // tot = 0: the first trip's total completes tot = d00
        __builtin_amdgcn_s_waitcnt(0);
        for (;;) {
#pragma unroll
            for (int r = 0; r < NS; ++r) {
                tot[r] += d[r];  // :141 (d00 for a freshly armed slot: tot = d00, :130)
                bool act = (dhi(d[r]) != 0u) & (tot[r] <= L.mr);
                uint64_t m = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
                if (!m && kk[r] >= 0) {  // wave-uniform, rare: the slot's chunk has ended; refill it
                    finish(r);
                    if (next >= 0) {
                        arm(r, false);  // tot = d = d00
                        act = (dhi(d[r]) != 0u) & (tot[r] <= L.mr);
                        m = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
                    } else {
                        kk[r] = -1;
                    }
                    // the refill's own loads (tables) land here, so that the common path's wait
                    // before the step stays vmcnt(1) (the other slot's gather may be in flight)
                    __builtin_amdgcn_s_waitcnt(0);
                }
                lane_iters += (uint32_t)__popcll(m);
                iters += m ? 1u : 0u;  // slot-trips with an active lane
                bool near;
                const uint32_t off = fxs_offset_nb(L, a.fxs_cx, a.fxs_cy, x[r], y[r], d[r], c[r], sn[r], act,
                                                   zero_v, near);
                if (ML == 1) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, 0, 0);
                    d[r] = __builtin_bit_cast(double, v);
                } else if (ML == 2) {
                    if (act) d[r] = ld_off(dt, off);

                } else {
                    d[r] = ld_off(dt, off);
                }
                const uint64_t nb = __builtin_amdgcn_ballot_w64(near) & m;
                if (nb) {  // rare: lanes within the guard band re-gather from the IEEE cell
                    const RayArgs &K = kernarg_here();
                    if (lane_in(nb)) d[r] = ld_off(dt, exact_offset_pad(K.m, x[r], y[r], (uint32_t)K.fxp_P));
                }
            }
            bool open = false;
#pragma unroll
            for (int r = 0; r < NS; ++r) open |= kk[r] >= 0;
            if (!open) break;
        }
        iters = (iters + NS - 1) / NS;  // ~trips (SIMT diagnostic only)
    } else if (fast_car) {
#pragma unroll
        for (int r = 0; r < NS; ++r) {
            kk[r] = -1;
            d[r] = tot[r] = x[r] = y[r] = c[r] = sn[r] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < NS; ++r)
            if (next >= 0) arm(r, false);
        __builtin_amdgcn_s_waitcnt(0);
        // The loop's scalar control is kept to what a trip needs (the CU's one scalar unit
        // serves its resident waves: k_rays_fxr spent ~30 SALU per trip against 36 VALU):
        // the slots' active-lane counts drive the lookup count, and the refill / exit tests
        // run only when a slot has no active lane.
        uint32_t trips = 0, idle = 0;
        for (;;) {
            uint64_t m[NS];
            uint32_t cnt[NS], off[NS];
            bool near[NS];  // the lane's cell is within the guard band of an edge
            bool ac[NS];
            // every slot steps unconditionally (a slot without active lanes reads the zero cell:
            // ~15 VALU wasted in the car's last chunks instead of a branch per slot per trip)
#pragma unroll
            for (int r = 0; r < NS; ++r) {
                const bool act = (dhi(d[r]) != 0u) & (tot[r] <= L.mr);
                ac[r] = act;
                m[r] = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
                cnt[r] = (uint32_t)__popcll(m[r]);
                off[r] = fxs_offset_nb(L, a.fxs_cx, a.fxs_cy, x[r], y[r], d[r], c[r], sn[r], act, zero_v, near[r]);
            }
            if (ML == 3 && NS == 2 && !(m[0] & m[1])) {
                // ML 3: no lane has both slots' rays active, so one gather serves both slots
                // (an ended ray reads 0.0, as from the zero cell)
                const double v = ld_off(dt, ac[0] ? off[0] : off[1]);
                d[0] = ac[0] ? v : 0.0;
                d[NS - 1] = ac[NS - 1] ? v : 0.0;
            } else {
#pragma unroll
                for (int r = 0; r < NS; ++r) d[r] = ld_off(dt, off[r]);
            }
            // the gathers go out on the fixed-point cells at once (the guard-band test is off the
            // dependent chain d -> x, y -> cell -> d); the rare lanes within the band of a cell edge
            // then re-gather from tiled_cell's IEEE cell (loads return in order: the second wins)
            uint64_t nb[NS], nball = 0;
#pragma unroll
            for (int r = 0; r < NS; ++r) {
                nb[r] = __builtin_amdgcn_ballot_w64(near[r]) & m[r];
                nball |= nb[r];
            }
            if (nball) {  // rare (wave-uniform)
                const RayArgs &K = kernarg_here();
#pragma unroll
                for (int r = 0; r < NS; ++r)
                    if (lane_in(nb[r])) d[r] = ld_off(dt, exact_offset_pad(K.m, x[r], y[r], (uint32_t)K.fxp_P));
            }
            uint32_t cmin = cnt[0], csum = cnt[0];
#pragma unroll
            for (int r = 1; r < NS; ++r) {
                cmin = min(cmin, cnt[r]);
                csum += cnt[r];
            }
            lane_iters += csum;
            ++trips;
            if (cmin == 0u) {  // rare: a slot's chunk has ended, or the slot is closed
                const bool none = csum == 0u;
                idle += none ? 1u : 0u;
                bool open = false;
#pragma unroll
                for (int r = 0; r < NS; ++r) {
                    if (kk[r] >= 0 && cnt[r] == 0u) {  // wave-uniform: the chunk has ended; refill the slot
                        finish(r);
                        if (next >= 0) arm(r, true);
                        else kk[r] = -1;
                    }
                    open |= kk[r] >= 0;
                }
                if (none && !open) break;
            }
#pragma unroll
            for (int r = 0; r < NS; ++r) tot[r] += d[r];  // :141 (a re-armed slot completes tot = d00, as k_rays_fxr)
        }
        iters = trips - idle;  // trips with an active lane (k_rays_fxr's count)
    } else {  // an origin off the map: the IEEE cell of every lookup, chunk after chunk
        uint32_t cnt = 0;
        while (next >= 0) {
            arm(0, false);
            const RayArgs &K = kernarg_here();
            while ((dhi(d[0]) != 0u) & (tot[0] <= L.mr)) {
                x[0] += d[0] * c[0];  // :135
                y[0] += d[0] * sn[0];  // :136
                d[0] = fx_load<3>(dt, exact_offset_pad(K.m, x[0], y[0], (uint32_t)K.fxp_P));
                tot[0] += d[0];  // :141
                ++cnt;
            }
            finish(0);
        }
        lane_iters = wave_sum(cnt);
        iters = wave_max(cnt);
    }
    if (lane == 0) {
        const RayArgs &K = kernarg_here();
        unsigned long long *cs = K.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
        atomicAdd(cs, (unsigned long long)(lanes + lane_iters));  // the first lookup came from k_agents
        atomicAdd(cs + 1, (unsigned long long)lanes);
        if (K.count_slots) atomicAdd(cs + 2, (unsigned long long)iters * (fast_car ? 64ull * NS : 64ull));
    }
}

// ------------------------------------------------------------------------
// k_rays_fxp (F110_FX_POOL = NCAR cars per wave): lane-level refill over a
// pool of cars.  k_rays_fxr refills a slot only when its whole 64-beam chunk
// has ended, and a wave of ONE car cannot end before that car's longest ray
// (mean ~83 loop iterations against ~49 for the car's rays spread over 128
// lane slots: scripts/lane_refill_model.py).  Here a wave owns NCAR cars; its
// queue holds their 64-beam chunks sorted by the previous launch's per-chunk
// cost (pcost: the long, grazing-beam chunks start first), every lane has two
// ray slots, and a slot whose ray has ended takes the queue's next ray.  The
// finish + re-arm pass is wave-wide work whatever the number of lanes in it,
// so it runs once >= pool_T slots wait (or none is still tracing).
//
// Per ray the arithmetic is k_rays_fxn's on the padded EDT (fxp_offset), so
// the outputs are bit-identical.  A ray's beam index comes from an LDS table
// of the pool's theta indices (built once per car from its beam runs), its
// noise is the pair draw of beam_normal_k (the half of the partner beam is
// not cached: the pass costs the same for any number of lanes).  The model
// (same poses, 2 cars per wave, pool_T 80): 65 instead of 105 wave-iterations
// per car, SIMT 0.75 instead of 0.46.
// The pool's per-car constants, in LDS (read per lane by the lane's car at
// re-arm / finish: SGPR copies of NCAR cars' values would spill).
struct PoolCar {
    double x0, y0, d0, vel;  // scan origin, first EDT lookup (:129), speed (TTC)
    uint64_t step;           // noise counter (steps since reset)
    uint32_t key, pad_;      // noise key of the car's env
};

template <bool HANDOFF, int NCAR>
__global__ void __launch_bounds__(64, 8) k_rays_fxp(RayArgs a) {  // 8 waves per SIMD: <= 64 VGPRs
    extern __shared__ __attribute__((aligned(16))) unsigned char fxp_smem[];
    const int lane = (int)threadIdx.x;
    const int B = a.B;
    const int nch = (B + 63) >> 6;
    const int g0 = (int)blockIdx.x * NCAR;
    const int ncar = min(NCAR, a.EA - g0);
    PoolCar *s_car = reinterpret_cast<PoolCar *>(fxp_smem);                                  // [NCAR]
    uint32_t *s_cost = reinterpret_cast<uint32_t *>(fxp_smem + NCAR * sizeof(PoolCar));     // [64]
    uint16_t *s_ti = reinterpret_cast<uint16_t *>(fxp_smem + NCAR * sizeof(PoolCar) + 256);  // [NCAR][B]
    const RayArgs &K = *kernarg_rays();
    const FxLoop L = fx_loop<3>(a);
    const uint32_t P = (uint32_t)a.fxp_P;
    const bool dev_noise = !K.noise_ext && K.noise_std > 0.0;

    // ---- per-car set-up: constants and the theta index of every beam into LDS ----
    bool all_fast = true;
    for (int ci = 0; ci < ncar; ++ci) {
        const int g = g0 + ci;
        const int e = HANDOFF ? g / a.A : g;
        const double x0 = ld_const(a.ray0 + g), y0 = ld_const(a.ray0 + a.EA + g);
        // q + P of the scan origin inside [fxp_lo, fxp_h*): its rays stay in the padded table
        const double ux = fma(x0, L.ir, L.cxk) - kFxpBase, uy = fma(y0, L.ir, L.cyk) - kFxpBase;
        all_fast = all_fast && (ux >= a.fxp_lo) & (ux < a.fxp_hx) & (uy >= a.fxp_lo) & (uy < a.fxp_hy);
        if (lane == 0) {
            PoolCar pc;
            pc.x0 = x0;
            pc.y0 = y0;
            pc.d0 = ld_const(a.ray0 + 2 * a.EA + g);  // :129
            pc.vel = ld_const(a.vel + g);
            pc.step = dev_noise ? ld_const(K.noise_step + e) : 0ull;
            pc.key = noise_key(K.seed, (uint64_t)(K.env_offset + e));
            pc.pad_ = 0u;
            s_car[ci] = pc;
        }
        const BeamRun *R = a.runs + (size_t)g * kMaxSeg;
        const int n = ld_const(a.nruns + g);
        int vlo = 0;  // lane k < nch: the run holding beam 64 k
        if (lane < nch) {
            int lo = 0, hi = n - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (R[mid].start <= lane * 64) lo = mid;
                else hi = mid - 1;
            }
            vlo = lo;
        }
        for (int k = 0; k < nch; ++k) {
            const int b = k * 64 + lane, bc = b < B ? b : B - 1;
            int ti = (int)beam_theta(R, n, __builtin_amdgcn_readlane(vlo, k), k * 64, bc);  // int(theta_index), :124
            if (ti >= a.theta_dis) ti = 0;
            if (b < B) s_ti[ci * B + b] = (uint16_t)ti;
        }
    }

    // ---- the queue: the pool's (car, chunk) units by predicted cost ----
    const int NU = ncar * nch;  // <= 64 (checked by the launcher)
    const uint32_t NQ = (uint32_t)NU * 64u;
    uint32_t ucode = 0, ukey = 0;
    if (lane < NU) {
        const int ci = lane / nch, k = lane - ci * nch;
        const uint32_t cost = a.pcost ? (uint32_t)a.pcost[(size_t)(g0 + ci) * nch + k] : 0u;
        ucode = ((uint32_t)ci << 5) | (uint32_t)k;
        // ties (first launch): descending chunks (the left edge first), cars interleaved
        ukey = (cost << 16) | ((uint32_t)k << 8) | (255u - (uint32_t)ci);
        s_cost[lane] = 0u;
    }
    uint32_t rank = lane < NU ? 0u : (uint32_t)lane;
    for (int j = 0; j < NU; ++j) rank += (uint32_t)(__builtin_amdgcn_readlane(ukey, j) > ukey) & (lane < NU ? 1u : 0u);
    const uint32_t sorted = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank << 2), (int)ucode);  // lane r: unit of rank r
    __syncthreads();  // the LDS tables (one wave)

    uint32_t rays = 0, lane_iters = 0, iters = 0, passes = 0, refills = 0;
    if (all_fast) {
        uint32_t zero_v;  // in a VGPR for the whole trace (the select's other operand is its SGPR mask)
        asm volatile("v_mov_b32 %0, %1" : "=v"(zero_v) : "s"(a.fx_zero));
        double x[2], y[2], d[2], tot[2], c[2], sn[2];
        // per slot: (iteration armed << 14) | (car << 12) | beam; -1 empty
        int32_t code[2] = {-1, -1};
        uint64_t occ[2] = {0ull, 0ull};
        uint32_t nxt = 0;
#pragma unroll
        for (int r = 0; r < 2; ++r) x[r] = y[r] = d[r] = tot[r] = c[r] = sn[r] = 0.0;
        // slot r of the lanes in `m` takes the queue's next rays (in lane order)
        auto arm = [&](int r, uint64_t m) {
            const uint32_t p = nxt + lanes_below(m);
            const uint32_t su = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(min(p >> 6, 63u) << 2), (int)sorted);
            const RayArgs &Ka = kernarg_here();  // in the wave-uniform part
            const bool mine = lane_in(m) && p < NQ;
            if (mine) {
                const int ci = (int)(su >> 5), k = (int)(su & 31u);
                const int b = (k << 6) | (int)(p & 63u);
                const int ti = s_ti[ci * B + (b < B ? b : B - 1)];
                c[r] = Ka.cosines[ti];
                sn[r] = Ka.sines[ti];
                const PoolCar &pc = s_car[ci];
                x[r] = pc.x0;
                y[r] = pc.y0;
                d[r] = b < B ? pc.d0 : 0.0;  // past the last beam: a ray that has ended
                tot[r] = d[r];  // :130
                code[r] = (int32_t)((iters << 14) | ((uint32_t)ci << 12) | (uint32_t)b);
            }
            occ[r] |= __builtin_amdgcn_ballot_w64(mine);
            nxt = min(nxt + (uint32_t)__popcll(m), NQ);
        };
        // the ended rays of slot r in `m`: outputs (fx_epilogue: noise after the clamp, TTC, obs / scans)
        auto finish = [&](int r, uint64_t m) {
            const uint32_t cd = (uint32_t)code[r];
            const int ci = (int)((cd >> 12) & 3u), b = (int)(cd & 4095u);
            const bool real = lane_in(m) && b < B;
            const RayArgs &Kf = kernarg_here();  // in the wave-uniform part
            if (real) {
                const int g = g0 + ci;
                const int e = HANDOFF ? g / Kf.A : g;
                const PoolCar &pc = s_car[ci];
                double nz = 0.0;
                if (Kf.noise_ext) nz = Kf.noise_ext[(size_t)e * B + b];
                else if (Kf.noise_std > 0.0) nz = Kf.noise_std * (double)beam_normal_k(pc.key, pc.step, b);
                fx_epilogue<HANDOFF>(Kf, g, e, b, tot[r], L.mr, nz, pc.vel, Kf.beam_cos[b], Kf.side[b]);
                atomicMax(s_cost + ci * nch + (b >> 6), iters - (cd >> 14) + 1u);
            }
            if (lane_in(m)) code[r] = -1;
            rays += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(real));
            occ[r] &= ~m;
        };
        arm(0, ~0ull);
        arm(1, ~0ull);
        const uint32_t T = (uint32_t)a.pool_T;
        // one back-edge (the slots' registers are not copied between two latches): refill,
        // then one step of every tracing ray
        for (;;) {
            uint64_t m[2];
#pragma unroll
            for (int r = 0; r < 2; ++r)
                m[r] = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
            const uint64_t e0 = occ[0] & ~m[0], e1 = occ[1] & ~m[1];
            const uint32_t ne = (uint32_t)(__popcll(e0) + __popcll(e1));
            bool tracing = (m[0] | m[1]) != 0ull;
            if (!tracing && !ne) break;  // the queue is done
            if (ne && (ne >= T || !tracing)) {  // wave-uniform: finish the ended rays, refill their slots
                ++passes;
                refills += (e0 ? 1u : 0u) + (e1 ? 1u : 0u);
                if (e0) {
                    finish(0, e0);
                    if (nxt < NQ) arm(0, e0);
                }
                if (e1) {
                    finish(1, e1);
                    if (nxt < NQ) arm(1, e1);
                }
#pragma unroll
                for (int r = 0; r < 2; ++r)
                    m[r] = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
                tracing = (m[0] | m[1]) != 0ull;
            }
            if (tracing) {
                ++iters;
                lane_iters += (uint32_t)(__popcll(m[0]) + __popcll(m[1]));
                // trace_ray's step (laser_models.py:135-141) for every tracing ray; ended /
                // empty slots read the zero cell (d = 0: total, x and y stay)
#pragma unroll
                for (int r = 0; r < 2; ++r)
                    if (m[r]) {
                        const bool act = (dhi(d[r]) != 0u) & (tot[r] <= L.mr);
                        const uint32_t off = fxp_offset(a.m, L, x[r], y[r], d[r], c[r], sn[r], act, m[r], zero_v, P);
                        d[r] = fx_load<3>(a.m.dt, off);
                    }
#pragma unroll
                for (int r = 0; r < 2; ++r)
                    if (m[r]) tot[r] += d[r];  // :141
            }
        }
        __syncthreads();
        if (a.pcost && lane < NU) {  // this launch's per-chunk cost: the next launch's order
            const uint32_t cst = s_cost[lane];
            const int ci = lane / nch, k = lane - ci * nch;
            a.pcost[(size_t)(g0 + ci) * nch + k] = (uint8_t)(cst < 255u ? cst : 255u);
        }
    } else {
        // a car of the pool has its scan origin off the map: every lookup takes the IEEE
        // cell (exact_offset_pad), one ray per lane, car by car, chunk by chunk
        uint32_t cnt = 0;
        for (int ci = 0; ci < ncar; ++ci) {
            const int g = g0 + ci;
            const int e = HANDOFF ? g / a.A : g;
            const PoolCar pc = s_car[ci];
            for (int k = 0; k < nch; ++k) {
                const int b = k * 64 + lane;
                if (b < B) {
                    const int ti = s_ti[ci * B + b];
                    const double cc = a.cosines[ti], ss = a.sines[ti];
                    double x = pc.x0, y = pc.y0, d = pc.d0;
                    double tot = d;  // :130
                    while ((dhi(d) != 0u) & (tot <= L.mr)) {
                        x += d * cc;  // :135
                        y += d * ss;  // :136
                        d = fx_load<3>(a.m.dt, exact_offset_pad(a.m, x, y, P));
                        tot += d;  // :141
                        ++cnt;
                    }
                    double nz = 0.0;
                    if (K.noise_ext) nz = K.noise_ext[(size_t)e * B + b];
                    else if (dev_noise) nz = K.noise_std * (double)beam_normal_k(pc.key, pc.step, b);
                    fx_epilogue<HANDOFF>(K, g, e, b, tot, L.mr, nz, pc.vel, a.beam_cos[b], a.side[b]);
                }
                rays += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(b < B));
            }
        }
        lane_iters = wave_sum(cnt);
        iters = wave_max(cnt);
    }
    if (lane == 0) {
        unsigned long long *cs = K.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
        atomicAdd(cs, (unsigned long long)(rays + lane_iters));  // the first lookup came from k_agents
        atomicAdd(cs + 1, (unsigned long long)rays);
        if (K.count_slots) {
            atomicAdd(cs + 2, (unsigned long long)iters * (all_fast ? 128ull : 64ull));
            atomicAdd(cs + 3, (unsigned long long)passes);
            atomicAdd(cs + 4, (unsigned long long)refills);
        }
    }
}

// k_rays_fxq (F110_FX_LPOOL): k_rays_fxp's lane-level refill for one car per
// wave, with k_rays_fxs's loop and a refill pass cut to the rays' own work.
// k_rays_fxp lost because a refill pass cost what a chunk pass costs (~170
// VALU, Philox draw included) and it ran ~25 times per car.  Here the car's
// scan noise is drawn once at the start into LDS (the same pair draws as
// k_rays_fxr / k_rays_fxs: beams b and b + 64 of a 128-beam block share one
// Philox2x32 draw), beside its theta-index table, so a pass is: an LDS read of
// the noise, the clamp, the TTC test, the obs entry (k_rays_fxs's Markstein
// division), and for the re-armed lanes an LDS read of the theta index and
// the two table gathers.  LDS: B * 6 bytes + 256 per wave (6 waves per SIMD at
// 1080 beams).  Lanes take the queue's next beam (lanes_below) once >= pool_T
// of the 128 slots have ended, or when none is still tracing; the queue is
// the car's 64-beam chunks in descending order of the previous launch's cost
// (pcost).  Per-ray arithmetic is k_rays_fxs's, so bit-identical.
template <bool HANDOFF>
__global__ void __launch_bounds__(64, 6) k_rays_fxq(RayArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char fxq_smem[];
    const int lane = (int)threadIdx.x;
    const int g = (int)blockIdx.x;  // one car per wave
    const int B = a.B;
    const int nch = (B + 63) >> 6;
    const int e = HANDOFF ? g / a.A : g;
    float *s_nz = reinterpret_cast<float *>(fxq_smem);                                        // [B]
    uint32_t *s_cost = reinterpret_cast<uint32_t *>(fxq_smem + (size_t)((B + 63) & ~63) * 4);  // [64]
    uint16_t *s_ti = reinterpret_cast<uint16_t *>(fxq_smem + (size_t)((B + 63) & ~63) * 4 + 256);  // [B]
    const double *dt = a.m.dt;
    const FxLoop L = fx_loop<3>(a);
    double x00, y00, d00;
    asm volatile("v_mov_b64 %0, %1" : "=v"(x00) : "s"(ld_const(a.ray0 + g)));
    asm volatile("v_mov_b64 %0, %1" : "=v"(y00) : "s"(ld_const(a.ray0 + a.EA + g)));
    asm volatile("v_mov_b64 %0, %1" : "=v"(d00) : "s"(ld_const(a.ray0 + 2 * a.EA + g)));  // :129
    uint32_t zero_v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(zero_v) : "s"(a.fx_zero));

    // ---- the car's theta indices and scan noise into LDS ----
    {
        const BeamRun *R = a.runs + (size_t)g * kMaxSeg;
        const int n = ld_const(a.nruns + g);
        int vlo = 0;  // lane k < nch: the run holding beam 64 k
        if (lane < nch) {
            int lo = 0, hi = n - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (R[mid].start <= lane * 64) lo = mid;
                else hi = mid - 1;
            }
            vlo = lo;
        }
        for (int k = 0; k < nch; ++k) {
            const int b = k * 64 + lane, bc = b < B ? b : B - 1;
            int ti = (int)beam_theta(R, n, __builtin_amdgcn_readlane(vlo, k), k * 64, bc);  // int(theta_index), :124
            if (ti >= a.theta_dis) ti = 0;
            if (b < B) s_ti[b] = (uint16_t)ti;
        }
        const RayArgs &K = kernarg_here();
        if (!K.noise_ext && K.noise_std > 0.0) {  // k_rays_fxs's draws: pair p serves beams b and b + 64
            const uint32_t key = noise_key(K.seed, (uint64_t)(K.env_offset + e));
            const uint64_t step = ld_const(K.noise_step + e);
            for (int k = 0; k < nch; k += 2) {
                const int b = k * 64 + lane;
                float lo, hi;
                beam_normal_pair_k(key, step, beam_noise_pair(b), lo, hi);
                if (b < B) s_nz[b] = lo;
                if (b + 64 < B) s_nz[b + 64] = hi;
            }
        }
        if (lane < nch) s_cost[lane] = 0u;
    }
    // the queue: the car's chunks by the previous launch's cost (ties: descending chunk index)
    uint32_t ukey = lane < nch ? (((a.pcost ? (uint32_t)a.pcost[(size_t)g * nch + lane] : 0u) << 8) | (uint32_t)lane) : 0u;
    uint32_t rank = lane < nch ? 0u : (uint32_t)lane;
    for (int j = 0; j < nch; ++j) rank += (uint32_t)(__builtin_amdgcn_readlane(ukey, j) > ukey) & (lane < nch ? 1u : 0u);
    const uint32_t sorted = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank << 2), lane);  // lane r: chunk of rank r
    __syncthreads();  // the LDS tables (one wave)

    uint32_t rays = 0, lane_iters = 0, iters = 0, passes = 0, refills = 0;
    const double ux = fma(ld_const(a.ray0 + g), L.ir, L.cxk) - kFxpBase;
    const double uy = fma(ld_const(a.ray0 + a.EA + g), L.ir, L.cyk) - kFxpBase;
    const bool fast_car = (ux >= a.fxp_lo) & (ux < a.fxp_hx) & (uy >= a.fxp_lo) & (uy < a.fxp_hy);
    const uint32_t NQ = (uint32_t)nch * 64u;
    if (fast_car) {
        double x[2], y[2], d[2], tot[2], c[2], sn[2];
        uint32_t code[2] = {0u, 0u};  // (trip armed << 12) | beam
        uint64_t occ[2] = {0ull, 0ull};
        uint32_t nxt = 0;
#pragma unroll
        for (int r = 0; r < 2; ++r) x[r] = y[r] = d[r] = tot[r] = c[r] = sn[r] = 0.0;
        auto arm = [&](int r, uint64_t m) {  // slot r of the lanes in m takes the queue's next beams
            const uint32_t p = nxt + lanes_below(m);
            const uint32_t ck = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(min(p >> 6, 63u) << 2), (int)sorted);
            const int b = (int)((ck << 6) | (p & 63u));
            const bool mine = lane_in(m) && p < NQ;
            if (mine) {
                const RayArgs &Ka = kernarg_here();
                const uint32_t toff = (uint32_t)s_ti[b < B ? b : B - 1] * 8u;
                c[r] = ld_off(Ka.cosines, toff);
                sn[r] = ld_off(Ka.sines, toff);
                x[r] = x00;
                y[r] = y00;
                d[r] = b < B ? d00 : 0.0;  // past the last beam: a ray that has ended
                tot[r] = d[r];  // :130
                code[r] = (iters << 12) | (uint32_t)b;
            }
            occ[r] |= __builtin_amdgcn_ballot_w64(mine);
            nxt = min(nxt + (uint32_t)__popcll(m), NQ);
        };
        auto finish = [&](int r, uint64_t m) {  // the ended rays of slot r in m: fx_epilogue
            const int b = (int)(code[r] & 4095u);
            const bool real = lane_in(m) && b < B;
            if (real) {
                const RayArgs &K = kernarg_here();
                const double mr = K.max_range;
                double range = tot[r] > mr ? mr : tot[r];  // :143-144
                if (K.noise_ext) range += K.noise_ext[(size_t)e * B + b];
                else if (K.noise_std > 0.0) range += K.noise_std * (double)s_nz[b];
                const double v = ld_const(K.vel + g);
                const uint32_t boff = (uint32_t)b * 8u;
                if (v != 0.0 && ttc_fires(range, ld_off(K.side, boff), v * ld_off(K.beam_cos, boff), K.ttc_thresh))
                    K.ttc_hit[g] = 1;
                if (K.obs && (!HANDOFF || g == e * K.A)) {
                    float *orow = K.obs + (size_t)e * K.obs_len;
                    *reinterpret_cast<float *>(reinterpret_cast<char *>(orow) + (uint32_t)b * 4u) =
                        obs_scan_value_fast(range, K.lidar_max, K.obs_rinv);
                }
                const size_t row = (size_t)g * B;
                if (K.scans_f32) *reinterpret_cast<float *>(reinterpret_cast<char *>(K.scans_f32 + row) + (uint32_t)b * 4u) = (float)range;
                if (K.scans_f64) *reinterpret_cast<double *>(reinterpret_cast<char *>(K.scans_f64 + row) + (uint32_t)b * 8u) = range;
                if (HANDOFF) *reinterpret_cast<double *>(reinterpret_cast<char *>(K.scan + row) + (uint32_t)b * 8u) = range;
                atomicMax(s_cost + (b >> 6), iters - (code[r] >> 12) + 1u);
            }
            rays += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(real));
            occ[r] &= ~m;
        };
        arm(0, ~0ull);
        arm(1, ~0ull);
        __builtin_amdgcn_s_waitcnt(0);
        const uint32_t T = (uint32_t)a.pool_T;
        for (;;) {
            uint64_t m[2];
            uint32_t cnt[2], off[2];
            bool near[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                m[r] = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
                cnt[r] = (uint32_t)__popcll(m[r]);
            }
            const uint64_t e0 = occ[0] & ~m[0], e1 = occ[1] & ~m[1];
            const uint32_t ne = (uint32_t)(__popcll(e0) + __popcll(e1));
            uint32_t tracing = cnt[0] + cnt[1];
            if (!tracing && !ne) break;  // nothing in flight and nothing to finish (every wave gets here)
            if (ne >= T || !tracing) {  // wave-uniform: finish the ended rays, refill their slots
                if (!tracing && nxt >= NQ) {  // the last rays: outputs, then done
                    if (e0) finish(0, e0);
                    if (e1) finish(1, e1);
                    break;
                }
                ++passes;
                refills += (e0 ? 1u : 0u) + (e1 ? 1u : 0u);
                if (e0) {
                    finish(0, e0);
                    if (nxt < NQ) arm(0, e0);
                }
                if (e1) {
                    finish(1, e1);
                    if (nxt < NQ) arm(1, e1);
                }
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    m[r] = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
                    cnt[r] = (uint32_t)__popcll(m[r]);
                }
                tracing = cnt[0] + cnt[1];
                if (!tracing) continue;  // (every re-armed ray starts inside a wall: d00 == 0)
            }
            ++iters;
            lane_iters += tracing;
            // trace_ray's step (laser_models.py:135-141) for every slot (ended / empty lanes read the
            // zero cell: d = 0 keeps their total), gathers before the guard-band test (k_rays_fxs)
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const bool act = (dhi(d[r]) != 0u) & (tot[r] <= L.mr);
                off[r] = fxs_offset_nb(L, a.fxs_cx, a.fxs_cy, x[r], y[r], d[r], c[r], sn[r], act, zero_v, near[r]);
            }
#pragma unroll
            for (int r = 0; r < 2; ++r) d[r] = ld_off(dt, off[r]);
            const uint64_t nb0 = __builtin_amdgcn_ballot_w64(near[0]) & m[0];
            const uint64_t nb1 = __builtin_amdgcn_ballot_w64(near[1]) & m[1];
            if (nb0 | nb1) {  // rare (wave-uniform)
                const RayArgs &K = kernarg_here();
                if (lane_in(nb0)) d[0] = ld_off(dt, exact_offset_pad(K.m, x[0], y[0], (uint32_t)K.fxp_P));
                if (lane_in(nb1)) d[1] = ld_off(dt, exact_offset_pad(K.m, x[1], y[1], (uint32_t)K.fxp_P));
            }
#pragma unroll
            for (int r = 0; r < 2; ++r) tot[r] += d[r];  // :141
        }
        __syncthreads();
        if (a.pcost && lane < nch) {  // this launch's per-chunk cost: the next launch's order
            const uint32_t cst = s_cost[lane];
            a.pcost[(size_t)g * nch + lane] = (uint8_t)(cst < 255u ? cst : 255u);
        }
    } else {  // an origin off the map: the IEEE cell of every lookup, one ray per lane, chunk by chunk
        uint32_t cnt = 0;
        const RayArgs &K = kernarg_here();
        for (int k = 0; k < nch; ++k) {
            const int b = k * 64 + lane;
            if (b < B) {
                const uint32_t toff = (uint32_t)s_ti[b] * 8u;
                const double cc = ld_off(K.cosines, toff), ss = ld_off(K.sines, toff);
                double x = x00, y = y00, d = d00;
                double tot = d;  // :130
                while ((dhi(d) != 0u) & (tot <= L.mr)) {
                    x += d * cc;  // :135
                    y += d * ss;  // :136
                    d = fx_load<3>(dt, exact_offset_pad(K.m, x, y, (uint32_t)K.fxp_P));
                    tot += d;  // :141
                    ++cnt;
                }
                double nz = 0.0;
                if (K.noise_ext) nz = K.noise_ext[(size_t)e * B + b];
                else if (K.noise_std > 0.0) nz = K.noise_std * (double)s_nz[b];
                fx_epilogue<HANDOFF>(K, g, e, b, tot, L.mr, nz, ld_const(K.vel + g), K.beam_cos[b], K.side[b]);
            }
            rays += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(b < B));
        }
        lane_iters = wave_sum(cnt);
        iters = wave_max(cnt);
    }
    if (lane == 0) {
        const RayArgs &K = kernarg_here();
        unsigned long long *cs = K.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
        atomicAdd(cs, (unsigned long long)(rays + lane_iters));  // the first lookup came from k_agents
        atomicAdd(cs + 1, (unsigned long long)rays);
        if (K.count_slots) {
            atomicAdd(cs + 2, (unsigned long long)iters * (fast_car ? 128ull : 64ull));
            atomicAdd(cs + 3, (unsigned long long)passes);
            atomicAdd(cs + 4, (unsigned long long)refills);
        }
    }
}

// k_rays_fx_tail: the handed-off rays, traced to the end with lane refill.
// Persistent waves take records from the queue (one atomic per refill);
// whenever >= kTailRefill lanes are idle, the finished lanes write their
// outputs and every idle lane takes the next record: the re-arm is the
// record's 9 loads, so the lanes stay busy where a ray-per-lane wave would
// wait on its longest ray.  Every wave exits once the queue is drained and
// its lanes are done (the queue was filled by the previous launch: no wait).
constexpr uint32_t kTailRefill = 16;
constexpr int kTailWaves = 8192;  // 8 waves per SIMD on 256 CUs

template <bool HANDOFF>
__global__ void __launch_bounds__(64) k_rays_fx_tail(RayArgs a) {
    // wave -> partition blockIdx % P (the waves of a partition share its counters)
    const uint32_t part = blockIdx.x % (uint32_t)a.ev_P;
    const uint32_t capp = a.ev_capp;
    uint32_t nrec = ld_const(a.ev_ctr + part * kEvStride);
    nrec = nrec < capp ? nrec : capp;  // reservations past the capacity were not written
    if ((blockIdx.x / (uint32_t)a.ev_P) * 64u >= nrec) return;  // nothing left for this wave's first take
    uint32_t *head = a.ev_ctr + part * kEvStride + 1;
    const size_t pbase = (size_t)part * capp;
    const size_t cap = a.ev_cap;
    const int lane = (int)threadIdx.x;
    const FxLoop L = fx_loop(a);
    double x = 0.0, y = 0.0, d = 0.0, tot = 0.0, c = 0.0, s = 0.0, noise = 0.0, v = 0.0, bcos = 0.0, side = 0.0;
    int g = 0, b = 0;
    bool busy = false, exhausted = false;
    uint32_t lane_iters = 0;
    for (;;) {
        bool tracing = busy & (dhi(d) != 0u) & (tot <= L.mr);
        uint64_t tm = __builtin_amdgcn_ballot_w64(tracing);
        const bool refill = !exhausted && (uint32_t)__popcll(tm) <= 64u - kTailRefill;
        if (refill || exhausted) {
            if (busy && !tracing) {  // finished: outputs, lane free
                const RayArgs &K = *kernarg_rays();
                fx_epilogue<HANDOFF>(K, g, HANDOFF ? g / K.A : g, b, tot, L.mr, noise, v, bcos, side);
                busy = false;
            }
        }
        if (refill) {
            const uint64_t fm = __builtin_amdgcn_ballot_w64(!busy);
            const uint32_t cnt = (uint32_t)__popcll(fm);
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(head, cnt);
            base = __builtin_amdgcn_readfirstlane(base);
            if (base + cnt >= nrec) exhausted = true;
            if (!busy) {
                const uint32_t ip = base + lanes_below(fm);
                if (ip < nrec) {
                    const size_t C = cap, i = pbase + ip;
                    x = a.ev[i];
                    y = a.ev[C + i];
                    d = a.ev[2 * C + i];
                    tot = a.ev[3 * C + i];
                    c = a.ev[4 * C + i];
                    s = a.ev[5 * C + i];
                    noise = a.ev[6 * C + i];
                    g = a.ev_gb[i];
                    b = a.ev_gb[C + i];
                    v = a.vel[g];
                    bcos = a.beam_cos[b];
                    side = a.side[b];
                    busy = true;
                }
            }
            tracing = busy & (dhi(d) != 0u) & (tot <= L.mr);
            tm = __builtin_amdgcn_ballot_w64(tracing);
        }
        if (!tm) {
            if (exhausted) break;
            continue;  // every lane idle, queue not drained: the next pass refills
        }
        lane_iters += (uint32_t)__popcll(tm);
        if (tracing) fx_step(a.m, L, x, y, d, tot, c, s);
    }
    if (lane == 0 && lane_iters) {  // lookups only: the rays were counted by k_rays_fx
        unsigned long long *slot = a.ctr + (size_t)(blockIdx.x % kCtrSlots) * kCtrStride;
        atomicAdd(slot, (unsigned long long)lane_iters);
    }
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
    uint32_t pending;  // k_step1: the autoreset flag for the next step (env_epilogue's vs)
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
    v.episode = a.mode == 0 ? a.episode[e] : 0u;
}

// stl: post-TTC state rows of its A agents (x at [i*stride], y at
// [i*stride + 1]); col: collision flags; cars / env: the prefetched inputs.
// vs / cs (optional, k_step1): the updated env / car bookkeeping, kept in
// registers across the steps of one launch.
__device__ void env_epilogue(const StepArgs &a, int e, const double *stl, int stride, const int32_t *col,
                             int do_reset, const EpiEnv &v, const EpiCar *cars, EpiEnv *vs = nullptr,
                             EpiCar *cs = nullptr) {
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
        if (cs) {
            cs[i].tg = tg;
            cs[i].ns = ns;
            cs[i].lt = lt;
        }
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
    if (vs) {
        vs->tprev = tnow;
        vs->episode = ep;
        vs->nstep = v.nstep + 1;
        vs->pending = (a.autoreset && term) ? 1u : 0u;
    }
}

// ------------------------------------------------------------------------
struct PostShared {
    double stl[kMaxAgents][7];   // state after update_pose (TTC may zero 3..6)
    double pose0[kMaxAgents][3]; // agent_poses: (x, y, yaw) before the TTC response (base_classes.py:587)
    double verts[kMaxAgents][8]; // Simulator.check_collision's get_vertices (Simulator.params, :562)
    double rv[kMaxAgents * (kMaxAgents - 1)][8];  // opponent j seen by agent i: RaceCar i's params (:223)
    int32_t hit[kMaxAgents];     // TTC hit
    int32_t col[kMaxAgents];     // collisions (GJK | TTC)
    double wcen[kMaxAgents * (kMaxAgents - 1)], whalf[kMaxAgents * (kMaxAgents - 1)];  // box_beam_window
    int32_t blo[kMaxAgents * kMaxAgents], bhi[kMaxAgents * kMaxAgents];
    EpiCar epi[kMaxAgents];      // env_epilogue inputs, prefetched at kernel start
    EpiEnv epe;
    int32_t do_reset, pad_[1];
};
static_assert(sizeof(PostShared) % 16 == 0, "LDS carve alignment");

size_t post_lds_bytes(int A, int B) { return sizeof(PostShared) + sizeof(double) * (size_t)A * B; }

// k_post: one workgroup per env: Simulator.step's collision stage + F110Env's epilogue.
__global__ void __launch_bounds__(kBlock) k_post(StepArgs a) {
    reset_next_heavy(a);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    PostShared &sh = *reinterpret_cast<PostShared *>(smem);
    double *scan = reinterpret_cast<double *>(smem + sizeof(PostShared));
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    const int A = a.A, B = a.B;
    const int EA = a.E * A;
    if (a.mode == 1 && a.reset_mask && !a.reset_mask[e]) return;  // uniform per block

    const double *gscan = a.scan + (size_t)e * A * B;
    for (int id = tid; id < A * B; id += kBlock) scan[id] = gscan[id];
    if (tid < A) {
        const int g = e * A + tid;
#pragma unroll
        for (int k = 0; k < 7; ++k) sh.stl[tid][k] = a.st[(size_t)k * EA + g];
        // agent_poses (x, y, yaw) are taken before the TTC response (base_classes.py:587)
        sh.pose0[tid][0] = sh.stl[tid][0];
        sh.pose0[tid][1] = sh.stl[tid][1];
        sh.pose0[tid][2] = sh.stl[tid][4];
        epilogue_load_car(a, g, sh.epi[tid]);
        get_vertices(sh.stl[tid][0], sh.stl[tid][1], sh.stl[tid][4], a.p.length, a.p.width, sh.verts[tid]);
        sh.hit[tid] = 0;
        sh.col[tid] = 0;
    }
    if (tid == 0) {
        sh.do_reset = a.reset_flag[e];
        epilogue_load_env(a, e, sh.epe);
    }
    __syncthreads();

    // TTC against the environment (check_ttc_jit, laser_models.py:188-217) on the noisy scan
    for (int id = tid; id < A * B; id += kBlock) {
        int ag = id / B;
        int b = id - ag * B;
        double v = sh.stl[ag][3];
        if (v != 0.0 && ttc_fires(scan[id], a.side[b], v * a.beam_cos[b], a.ttc_thresh)) sh.hit[ag] = 1;
    }
    if (tid == 0) {  // collision_multiple (collision_models.py:184-212) on pre-TTC poses
        for (int i = 0; i < A - 1; ++i)
            for (int j = i + 1; j < A; ++j)
                if (gjk_collision(sh.verts[i], sh.verts[j])) {
                    sh.col[i] = 1;
                    sh.col[j] = 1;
                }
    }
    __syncthreads();
    if (tid < A && sh.hit[tid]) {  // RaceCar.check_ttc (base_classes.py:246-249): state[3:] = 0
        const int g = e * A + tid;
#pragma unroll
        for (int k = 3; k < 7; ++k) {
            sh.stl[tid][k] = 0.0;
            a.st[(size_t)k * EA + g] = 0.0;
        }
        sh.col[tid] = 1;  // Simulator.step :601-602
    }
    __syncthreads();
    if (tid < A * (A - 1)) {  // pair (i, jj-th opponent) -> get_blocked_view_indices on i's post-TTC pose
        int i = tid / (A - 1);
        int jj = tid - i * (A - 1);
        int j = jj < i ? jj : jj + 1;
        // RaceCar.ray_cast_agents: get_vertices(opp_pose, self.params['length'], self.params['width'])
        double *v = sh.rv[tid];
        const f110_params &pi = a.pa[i];
        get_vertices(sh.pose0[j][0], sh.pose0[j][1], sh.pose0[j][2], pi.length, pi.width, v);
        int lo, hi;
        blocked_range(sh.stl[i][0], sh.stl[i][1], sh.stl[i][4], v, B, a.fov, a.beam_incr, lo, hi);
        box_beam_window(sh.stl[i][0], sh.stl[i][1], v, nullptr, sh.wcen[tid], sh.whalf[tid]);
        sh.blo[tid] = lo;
        sh.bhi[tid] = hi;
    }
    __syncthreads();
    // agent ray_cast (RaceCar.ray_cast_agents, base_classes.py:206-227; ray_cast, laser_models.py:318-346)
    for (int jj = 0; jj < A - 1; ++jj) {
        for (int i = 0; i < A; ++i) {
            int pr = i * (A - 1) + jj;
            int lo = sh.blo[pr], hi = sh.bhi[pr];
            const double ox = sh.stl[i][0], oy = sh.stl[i][1], oth = sh.stl[i][4];
            const double *v = sh.rv[pr];
            const double wc = sh.wcen[pr], wh = sh.whalf[pr];
            for (int b = lo + tid; b <= hi; b += kBlock) {
                // beams that cannot reach the box keep their range (see box_beam_window);
                // get_blocked_view_indices' min..max spans most of the scan for an
                // opponent behind the car, the filter keeps ~the box's own beams
                const double ang = beam_angle(b, a.fov, a.beam_incr);
                if (!(fabs(wrap_pm_pi(oth + ang - wc)) <= wh)) continue;
                double bt = oth + ang + kPi / 2.;
                double v31, v30;
                cr_sincos(bt, v31, v30);
                double cur = scan[i * B + b];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    int q1 = (q + 1) & 3;
                    double rr = get_range(ox, oy, v30, v31, v[2 * q], v[2 * q + 1], v[2 * q1], v[2 * q1 + 1]);
                    if (rr < cur) cur = rr;
                }
                scan[i * B + b] = cur;
            }
        }
        __syncthreads();
    }

    // ---- outputs --------------------------------------------------------
    if (a.out.obs) {  // F110Env._pack_flat_obs, f110_env.py:552-584 (scan of agent 0, e = 0)
        float *o = a.out.obs + (size_t)e * obs_row(a);
        const float lmax = (float)a.p.lidar_max;
        for (int b = tid; b < B; b += kBlock) o[b] = obs_scan_value(scan[b], lmax);
        if (tid < A) {
            o[B + 4 * tid + 0] = (float)sh.stl[tid][0];
            o[B + 4 * tid + 1] = (float)sh.stl[tid][1];
            o[B + 4 * tid + 2] = (float)wrap_angle(sh.stl[tid][4]);
            o[B + 4 * tid + 3] = sh.col[tid] ? 1.0f : 0.0f;
        }
    }
    if (a.out.scans) {
        float *o = a.out.scans + (size_t)e * A * B;
        for (int id = tid; id < A * B; id += kBlock) o[id] = (float)scan[id];
    }
    if (a.out.scans_f64) {
        double *o = a.out.scans_f64 + (size_t)e * A * B;
        for (int id = tid; id < A * B; id += kBlock) o[id] = scan[id];
    }
    if (a.out.collisions && tid < A) a.out.collisions[(size_t)e * A + tid] = (uint8_t)sh.col[tid];
    if (tid == 0) env_epilogue(a, e, &sh.stl[0][0], 7, sh.col, sh.do_reset, sh.epe, sh.epi);
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
        o[0] = (float)stl[0];
        o[1] = (float)stl[1];
        o[2] = (float)wrap_angle(yaw);
        o[3] = col ? 1.0f : 0.0f;
    }
    if (a.out.collisions) a.out.collisions[e] = (uint8_t)col;
    env_epilogue(a, e, stl, 2, &col, do_reset, env, &car);
}

// ------------------------------------------------------------------------
// k_step1: the whole single-agent step in ONE launch, for n consecutive steps
// (f110_step / f110_step_n).  One wave per car (env); per step:
//   1. lane 0: k_agents' work for the car (autoreset, RaceCar.update_pose,
//      scan pose, first lookup, the beam-index runs into LDS);
//   2. every lane: the theta index of each beam into LDS (get_scan's
//      sequential index, from the runs);
//   3. the car's 1080 rays as k_rays_fxr traces them (two 64-beam chunk slots
//      refilled as chunks end, padded EDT, noise after the clamp), the TTC test
//      of each ray folded into one wave ballot;
//   4. lane 0: k_post_single's work (TTC response, obs pose entries,
//      collisions, _check_done / lap logic, the next step's autoreset flag).
// The car's state stays in lane 0's registers from step to step (written back
// once at the end), so a launch of n steps carries no hand-off buffer and no
// per-step launch boundary: an env whose rays run long in one step overlaps
// other envs' next steps instead of holding every env at a step boundary.
// Per ray and per car the arithmetic is the three kernels', so the results
// are bit-identical to n calls of the three-launch step
// (test_step1_matches_three_launch_step).
struct Step1Shared {
    BeamRun runs[kMaxSeg];
    double sx, sy, d00, vel;
    uint64_t nstep;
    int32_t nruns, do_reset, col, pad_;
    // the car's persistent state between steps (wave 0, lane c; kept out of registers
    // so that the ray loop keeps its 64 VGPRs)
    double st[7], acc[7], b0, b1;  // st / acc: update_pose_impl's volatile LDS arrays
    int32_t cnt, pad2_;
    EpiCar car;
    EpiEnv env;
};

__device__ __forceinline__ const FusedArgs &fused_args() {
#if defined(__HIP_DEVICE_COMPILE__)
    return *reinterpret_cast<const FusedArgs *>(__builtin_amdgcn_kernarg_segment_ptr());
#else
    static const FusedArgs none{};  // (host pass: never called)
    return none;
#endif
}

// k_step1's lane-0 sections as real calls: their register needs (RK4 of
// vehicle_dynamics_st: ~150 VGPRs inline) stay out of the ray loop's 64.
// (the argument block comes in as a pointer: a callee must not read the kernarg
// segment pointer itself)
template <class T>
__device__ __forceinline__ const T *launder_s(const T *p) {  // an opaque SGPR copy (loads through it stay below)
    return launder_const(p);
}

// a callee's pointer argument arrives in VGPRs (not known to be uniform): its
// loads would all be vector loads into VGPRs; readfirstlane makes it scalar
template <class T>
__device__ __forceinline__ T *uniform_ptr(T *p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T *)(((uint64_t)hi << 32) | lo);
}

// k_step1's LDS, named at namespace scope so the callees address it directly
// (ds_* instructions; a pointer argument would be generic: flat accesses):
// [cpw] Step1Shared, then each car's theta indices [cpw][B, 16-byte rounded]
extern __shared__ __attribute__((aligned(16))) unsigned char s1_smem[];
__device__ __forceinline__ Step1Shared &step1_shared(int c) { return reinterpret_cast<Step1Shared *>(s1_smem)[c]; }
__device__ __forceinline__ uint16_t *step1_ti(int c, int cpw, int B) {
    const int tib = (B * 2 + 15) & ~15;
    return reinterpret_cast<uint16_t *>(s1_smem + (size_t)cpw * sizeof(Step1Shared) + (size_t)c * tib);
}

// LDS hand-off between the lanes of ONE wave (no workgroup barrier).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __noinline__ void step1_agent(const FusedArgs *fap, int t, int c) {
    fap = uniform_ptr(fap);
    t = __builtin_amdgcn_readfirstlane(t);
    const int g = (int)blockIdx.x * launder_s(fap)->cpw + c;
    Step1Shared &sh = step1_shared(c);
    typedef __attribute__((address_space(3))) volatile double lds_vd;  // ds_* accesses, kept in LDS (volatile)
    lds_vd *st = (lds_vd *)sh.st;
    double raw_steer, vel;
    int do_reset;
    {  // the action, the autoreset (RaceCar.reset, base_classes.py:183-204)
        const FusedArgs &fa = *launder_s(fap);
        const StepArgs &S = fa.s;
        if (S.actions_f64) {
            const double *ac = S.actions_f64 + (size_t)t * fa.act_stride + (size_t)g * 2;
            raw_steer = ac[0];
            vel = ac[1];
        } else {
            const float *ac = S.actions + (size_t)t * fa.act_stride + (size_t)g * 2;
            raw_steer = (double)ac[0];
            vel = (double)ac[1];
        }
        do_reset = sh.env.pending ? 1 : 0;
        if (do_reset) {  // then F110Env.reset's zero-action step
            const uint64_t genv = (uint64_t)(S.env_offset + g);
            const uint32_t k = spawn_draw(S.seed, genv, sh.env.episode) % (uint32_t)S.n_spawn;
            const double *pz = S.spawn + (size_t)k * 3;
            double px = pz[0], py = pz[1], pth = pz[2];
            if (S.reset_f32) {
                px = (double)(float)px;
                py = (double)(float)py;
                pth = (double)(float)pth;
            }
#pragma unroll
            for (int q = 0; q < 7; ++q) st[q] = 0.0;
            st[0] = px;
            st[1] = py;
            st[4] = pth;
            sh.b0 = sh.b1 = 0.0;
            sh.cnt = 0;
            raw_steer = 0.0;
            vel = 0.0;
            S.start[g] = px;
            S.start[S.E + g] = py;
            S.start[2 * S.E + g] = pth;
            sh.car.sx = px;
            sh.car.sy = py;
            sh.car.tg = 0;
            sh.car.ns = 1;
            sh.car.lt = 0.0f;
            S.toggles[g] = 0;
            S.near_start[g] = 1;
            S.lap_times[g] = 0.0f;
            S.lap_counts[g] = 0.0f;
            if (S.ego == 0) {  // start_rot (f110_env.py:448-451), as k_agents
                double cr, sr;
                if (S.reset_f32) {
                    const float nt = -(float)pth;
                    cr = (double)np_sincosf(nt, true);
                    sr = (double)np_sincosf(nt, false);
                } else {
                    cr_sincos(-pth, sr, cr);
                }
                sh.env.ct = cr;
                sh.env.st = sr;
                S.start_rot[g] = cr;
                S.start_rot[S.E + g] = sr;
            }
        }
    }
    {  // RaceCar.update_pose (state and RK4 accumulator in LDS)
        const StepArgs &S = launder_s(fap)->s;
        double b0 = sh.b0, b1 = sh.b1;
        int cnt = sh.cnt;
        update_pose_impl<lds_vd *>(st, (lds_vd *)sh.acc, b0, b1, cnt, raw_steer, vel, S.pa[0], S.dt, S.integrator);
        sh.b0 = b0;
        sh.b1 = b1;
        sh.cnt = cnt;
    }
    const double yaw = st[4];
    {  // scan pose (base_classes.py:420-422), first lookup (laser_models.py:129)
        const StepArgs &S = launder_s(fap)->s;
        const bool no_offset = S.lidar_dist == 0.0 && isfinite(yaw);
        double sy4 = 0.0, cy4 = 1.0;
        if (!no_offset) cr_sincos(yaw, sy4, cy4);
        const double sx = no_offset ? st[0] + 0.0 : st[0] + S.lidar_dist * cy4;
        const double sy = no_offset ? st[1] + 0.0 : st[1] + S.lidar_dist * sy4;
        sh.sx = sx;
        sh.sy = sy;
        sh.d00 = S.map.dt[cell_index(S.map, sx, sy)];
        sh.vel = st[3];
        sh.nstep = do_reset ? 0ull : sh.env.nstep;
        sh.do_reset = do_reset;
    }
    {  // get_scan's beam-index runs
        const StepArgs &S = launder_s(fap)->s;
        const double t0 = first_theta_index(yaw, S.fov, S.theta_dis);
        sh.nruns = build_beam_runs(t0, S.inc, S.theta_dis, S.B, sh.runs, kMaxSeg);
    }
}

__device__ __noinline__ void step1_post(const FusedArgs *fap, int c) {
    fap = uniform_ptr(fap);
    const int g = (int)blockIdx.x * fap->cpw + c;
    Step1Shared &sh = step1_shared(c);
    const bool col = sh.col != 0;
    const int B = fap->r.B;
            const StepArgs &S = fap->s;
            const int do_reset = sh.do_reset;
            EpiCar car = sh.car;
            EpiEnv env = sh.env;
            if (col) {  // RaceCar.check_ttc (base_classes.py:246-249): state[3:] = 0, yaw included
#pragma unroll
                for (int q = 3; q < 7; ++q) sh.st[q] = 0.0;
            }
            double st[7];
#pragma unroll
            for (int q = 0; q < 7; ++q) st[q] = sh.st[q];
            if (S.out.obs) {
                float *o = S.out.obs + (size_t)g * obs_row(S) + B;
                o[0] = (float)st[0];
                o[1] = (float)st[1];
                o[2] = (float)wrap_angle(st[4]);
                o[3] = col ? 1.0f : 0.0f;
            }
            if (S.out.collisions) S.out.collisions[g] = (uint8_t)col;
            const double stl[2] = {st[0], st[1]};
            const int32_t coli = col ? 1 : 0;
            EpiEnv ev = env;
            ev.nstep = do_reset ? 0ull : env.nstep;  // the counter this step's noise used (k_agents' noise_step)
            env_epilogue(S, g, stl, 2, &coli, do_reset, ev, &car, &env, &car);
            sh.car = car;
            sh.env = env;
        }

// the argument block behind an opaque copy of its pointer (as kernarg_here):
// the lane-0 sections' field loads stay in their step instead of being hoisted
// out of the step loop into SGPRs, which would spill there
__device__ __forceinline__ const FusedArgs *fused_args_here() { return launder_const(&fused_args()); }

// the ray phase of one step (get_scan for the car, k_rays_fxr's two refilled
// chunk slots, the TTC ballot): a call of its own, so its constants are loaded
// per step instead of living in registers across the lane-0 sections
struct Step1Rays {
    uint32_t lanes, iters;
    int32_t col;
};

__device__ __noinline__ Step1Rays step1_rays(const FusedArgs *fap, int w) {
    fap = uniform_ptr(fap);
    w = __builtin_amdgcn_readfirstlane(w);
    const int cpw = launder_s(fap)->cpw;
    const int g = (int)blockIdx.x * cpw + w;
    uint16_t *s_ti = step1_ti(w, cpw, launder_s(fap)->r.B);
    Step1Shared &sh = step1_shared(w);
    const int lane = (int)threadIdx.x & 63;
    uint32_t lanes_total = 0, lane_iters = 0;
    // the ray phase's constants, loaded per step (kept live across the lane-0
    // sections they would take SGPRs / VGPRs those need)
    const RayArgs &a = launder_s(fap)->r;
    const int B = a.B;
    const int nch = (B + 63) >> 6;
    const FxLoop L = fx_loop<3>(a);
    const uint32_t P = (uint32_t)a.fxp_P;
    uint32_t zero_v;  // in a VGPR for the whole trace (the select's other operand is its SGPR mask)
    asm volatile("v_mov_b32 %0, %1" : "=v"(zero_v) : "s"(a.fx_zero));
    const double x00 = sh.sx, y00 = sh.sy, d00 = sh.d00, vcar = sh.vel;
    const uint64_t nstep = sh.nstep;
    const int nr = sh.nruns;
    // ---- 2. the theta index of every beam (get_scan, laser_models.py:167-184) ----
    {
        int vlo = 0;  // lane k < nch: the run holding beam 64 k
        if (lane < nch) {
            int lo = 0, hi = nr - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (sh.runs[mid].start <= lane * 64) lo = mid;
                else hi = mid - 1;
            }
            vlo = lo;
        }
        for (int k = 0; k < nch; ++k) {
            const int b = k * 64 + lane;
            const int lo = __builtin_amdgcn_readlane(vlo, k);
            int rs = sh.runs[lo].start;
            double rt0 = sh.runs[lo].t0, rdl = sh.runs[lo].delta;
            for (int j = lo + 1; j < nr; ++j) {  // the runs that start inside this chunk
                const int s2 = sh.runs[j].start;
                if (s2 > k * 64 + 63) break;
                if (b >= s2) {
                    rs = s2;
                    rt0 = sh.runs[j].t0;
                    rdl = sh.runs[j].delta;
                }
            }
            int ti = (int)(rt0 + (double)(b - rs) * rdl);  // int(theta_index), :124
            if (ti >= a.theta_dis) ti = 0;
            if (b < B) s_ti[b] = (uint16_t)ti;
        }
    }
    wave_sync();  // the car's theta indices: this wave's own
    // ---- 3. the rays (k_rays_fxr's two refilled chunk slots) ----
    const double ux = fma(x00, L.ir, L.cxk) - kFxpBase, uy = fma(y00, L.ir, L.cyk) - kFxpBase;
    const bool fast_car = (ux >= a.fxp_lo) & (ux < a.fxp_hx) & (uy >= a.fxp_lo) & (uy < a.fxp_hy);
    const uint32_t key = noise_key(a.seed, (uint64_t)(a.env_offset + g));
    bool hit = false;
    double x[2], y[2], d[2], tot[2], c[2], sn[2];
    int kk[2];
    int next = nch - 1;
    float cval[2] = {0.0f, 0.0f};
    int ctag[2] = {-1, -1};
    auto arm = [&](int r) {
        const int k = next--;
        kk[r] = k;
        const int b = k * 64 + lane;
        const int ti = s_ti[b < B ? b : B - 1];
        c[r] = a.cosines[ti];
        sn[r] = a.sines[ti];
        x[r] = x00;
        y[r] = y00;
        d[r] = b < B ? d00 : 0.0;
        tot[r] = d[r];  // :130
    };
    auto finish = [&](int r) {  // fx_epilogue with the TTC flag kept in the wave
        const RayArgs &K = launder_s(fap)->r;
        const int b = kk[r] * 64 + lane, bc = b < B ? b : B - 1;
        double nz = 0.0;
        if (K.noise_ext) {
            nz = K.noise_ext[(size_t)g * B + bc];
        } else if (K.noise_std > 0.0) {
            const int pp = kk[r] >> 1, ci = pp & 1;
            float nv;
            if (ctag[ci] == pp) {
                nv = cval[ci];
                ctag[ci] = -1;
            } else {
                float lo, hi;
                beam_normal_pair_k(key, nstep, beam_noise_pair(b), lo, hi);
                nv = (kk[r] & 1) ? hi : lo;
                cval[ci] = (kk[r] & 1) ? lo : hi;
                ctag[ci] = pp;
            }
            nz = K.noise_std * (double)nv;
        }
        if (b < B) {
            double range = tot[r] > L.mr ? L.mr : tot[r];  // :143-144
            if (K.noise_ext || K.noise_std > 0.0) range += nz;
            // check_ttc_jit on the noisy scan (laser_models.py:188-217)
            if (vcar != 0.0 && ttc_fires(range, K.side[b], vcar * K.beam_cos[b], K.ttc_thresh)) hit = true;
            const int64_t rr = (int64_t)g * B + b;
            if (K.obs) K.obs[(size_t)g * K.obs_len + b] = obs_scan_value(range, K.lidar_max);
            if (K.scans_f32) K.scans_f32[rr] = (float)range;
            if (K.scans_f64) K.scans_f64[rr] = range;
        }
        lanes_total += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(b < B));
    };
    if (fast_car) {
        kk[0] = kk[1] = -1;
#pragma unroll
        for (int r = 0; r < 2; ++r) d[r] = tot[r] = x[r] = y[r] = c[r] = sn[r] = 0.0;
#pragma unroll
        for (int r = 0; r < 2; ++r)
            if (next >= 0) arm(r);
        for (;;) {
            uint64_t m[2], mall = 0;
#pragma unroll
            for (int r = 0; r < 2; ++r)
                m[r] = __builtin_amdgcn_ballot_w64(dhi(d[r]) != 0u) & __builtin_amdgcn_ballot_w64(tot[r] <= L.mr);
            double dn[2];
#pragma unroll
            for (int r = 0; r < 2; ++r)
                if (m[r]) {
                    const bool act = (dhi(d[r]) != 0u) & (tot[r] <= L.mr);
                    dn[r] = fx_load<3>(a.m.dt, fxp_offset(a.m, L, x[r], y[r], d[r], c[r], sn[r], act, m[r], zero_v, P));
                }
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                mall |= m[r];
                lane_iters += (uint32_t)__popcll(m[r]);
            }
            bool open = false;
#pragma unroll
            for (int r = 0; r < 2; ++r)
                if (kk[r] >= 0 && !m[r]) {  // wave-uniform: the chunk has ended; refill the slot
                    finish(r);
                    if (next >= 0) arm(r);
                    else kk[r] = -1;
                }
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                if (m[r]) {
                    d[r] = dn[r];
                    tot[r] += d[r];  // :141
                }
                open |= kk[r] >= 0;
            }
            if (mall == 0 && !open) break;
        }
    } else {  // the scan origin is off the map: the IEEE cell of every lookup, one chunk at a time
        uint32_t cntl = 0;
        while (next >= 0) {
            arm(0);
            while ((dhi(d[0]) != 0u) & (tot[0] <= L.mr)) {
                x[0] += d[0] * c[0];  // :135
                y[0] += d[0] * sn[0];  // :136
                d[0] = fx_load<3>(a.m.dt, exact_offset_pad(a.m, x[0], y[0], P));
                tot[0] += d[0];  // :141
                ++cntl;
            }
            finish(0);
        }
        lane_iters += wave_sum(cntl);
    }
    const bool col = __builtin_amdgcn_ballot_w64(hit) != 0ull;
    return Step1Rays{lanes_total, lane_iters, col ? 1 : 0};
}

// cpw cars per workgroup, one wave each for the rays; the lane-parallel
// sections (k_agents' update_pose and scan set-up, k_post_single's epilogue)
// run on wave 0, lane c for car c, as the three-launch step runs them on one
// lane per car.  Two workgroup barriers per step: post(t) and agent(t + 1) of a
// car are the same lane's back-to-back calls.
constexpr int kStep1MaxCpw = 8;

__global__ void __launch_bounds__(64 * kStep1MaxCpw, 8) k_step1(FusedArgs fa) {
    const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const int cpw = fa.cpw;
    const int g0 = (int)blockIdx.x * cpw;
    const int nc = min(cpw, fa.s.E - g0);  // cars of this workgroup
    const int nsteps = fa.nsteps;
    const bool lead = w == 0 && lane < nc;  // car `lane`'s lane-parallel sections

    if (lead) {  // the car's persistent state, in LDS for the whole launch
        Step1Shared &sh = step1_shared(lane);
        const StepArgs &S = fused_args().s;
        const int g = g0 + lane;
#pragma unroll
        for (int k = 0; k < 7; ++k) sh.st[k] = S.st[(size_t)k * S.E + g];
        sh.b0 = S.sb[g];
        sh.b1 = S.sb[S.E + g];
        sh.cnt = S.scnt[g];
        EpiCar car;
        epilogue_load_car(S, g, car);
        sh.car = car;
        EpiEnv env;
        env.tprev = S.sim_time[g];
        env.ct = S.start_rot[g];
        env.st = S.start_rot[S.E + g];
        env.nstep = S.nstep[g];
        env.episode = (uint32_t)S.episode[g];
        env.pending = S.autoreset ? S.pending[g] : 0u;
        sh.env = env;
    }
    uint32_t lanes_total = 0, lane_iters = 0;
    for (int t = 0; t < nsteps; ++t) {
        // ---- 1. k_agents (wave 0, a lane per car) ----
        if (lead) step1_agent(fused_args_here(), t, lane);
        __syncthreads();  // the cars' scan set-up
        // ---- 2./3. the theta indices and the rays (a wave per car) ----
        if (w < nc) {
            const Step1Rays rr = step1_rays(fused_args_here(), w);
            lanes_total += rr.lanes;
            lane_iters += rr.iters;
            if (lane == 0) step1_shared(w).col = rr.col;
        }
        __syncthreads();  // the cars' TTC flags
        // ---- 4. k_post_single (wave 0, a lane per car) ----
        if (lead) step1_post(fused_args_here(), lane);
    }
    if (lead) {  // the persistent state, once
        const Step1Shared &sh = step1_shared(lane);
        const StepArgs &S = fused_args().s;
        const int g = g0 + lane;
#pragma unroll
        for (int k = 0; k < 7; ++k) S.st[(size_t)k * S.E + g] = sh.st[k];
        S.sb[g] = sh.b0;
        S.sb[S.E + g] = sh.b1;
        S.scnt[g] = sh.cnt;
    }
    if (w < nc && lane == 0) {
        const RayArgs &a = fused_args().r;
        unsigned long long *cs = a.ctr + (size_t)((blockIdx.x * kStep1MaxCpw + w) % kCtrSlots) * kCtrStride;
        atomicAdd(cs, (unsigned long long)(lanes_total + lane_iters));  // + the first lookup of every ray
        atomicAdd(cs + 1, (unsigned long long)lanes_total);
    }
}

// k_post_multi: multi-agent envs after the tiled ray kernel (TTC flags are
// already set).  Two waves per env and no LDS copy of the scans: the agent
// ray_cast edits the f64 hand-off in place, so many envs stay resident per CU
// and their serial phases overlap.  Wave 0 runs GJK (collision_multiple on
// the pre-TTC poses) while wave 1 builds each (car, opponent) pair's box,
// blocked beam range and beam window (on the post-TTC pose).
constexpr int kMultiBlock = 128;  // default; F110_MULTI_BLOCK=64: one wave per env (GJK then the geometry)

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


template <int BLK>
__global__ void __launch_bounds__(BLK, 6) k_post_multi(StepArgs a) {
    reset_next_heavy(a);
    __shared__ MultiShared sh;
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    const int A = a.A, B = a.B;
    const int EA = a.E * A;
    if (a.mode == 1 && a.reset_mask && !a.reset_mask[e]) return;  // uniform per block
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
    if (tid == 0) {  // collision_multiple (collision_models.py:184-212)
        for (int i = 0; i < A - 1; ++i)
            for (int j = i + 1; j < A; ++j)
                if (gjk_collision(sh.verts[i], sh.verts[j])) {
                    sh.col[i] = 1;
                    sh.col[j] = 1;
                }
    }
    if (BLK == 64 || tid >= 64) {
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
    // agent ray_cast (base_classes.py:206-227; laser_models.py:318-346), one
    // opponent at a time per car (each pass min-updates the same beams), all
    // cars' passes of one round in one sweep over the block; only the beams
    // of lo..hi that the box's window can hold are visited
    for (int jj = 0; jj < A - 1; ++jj) {
        int total = 0;
        for (int i = 0; i < A; ++i) total += pass_beams(sh, i * (A - 1) + jj);
        for (int item = tid; item < total; item += BLK) {
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
}

hipError_t prepare_env_step(size_t lds_bytes) {
    if (lds_bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void *>(&k_post), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds_bytes);
}

size_t step_lds_bytes(int A, int B) { return post_lds_bytes(A, B); }

hipError_t launch_step1(const StepArgs &a, int32_t n, int64_t act_stride, hipStream_t s, hipEvent_t *ev) {
    hipError_t e;
    // f110_profile_begin: 6 events per step, (start, stop) of k_agents / the ray kernel / k_post,
    // attached to the kernel's own dispatch (hipExtLaunchKernel: its begin / end timestamps, no
    // marker packets between the kernels).  The fused step is one kernel: the ray pair.
    if (ev && (e = hipEventRecord(ev[0], s)) != hipSuccess) return e;
    if (ev && (e = hipEventRecord(ev[1], s)) != hipSuccess) return e;
    FusedArgs fa{};
    RayArgs &ra = fa.r;
    ra.m = a.tmap;
    ra.sines = a.sines;
    ra.cosines = a.cosines;
    ra.noise_ext = a.noise_ext;
    ra.ctr = a.ctr;
    ra.eps = a.eps;
    ra.max_range = a.max_range;
    ra.noise_std = a.noise_std;
    ra.seed = a.seed;
    ra.env_offset = a.env_offset;
    ra.EA = a.E * a.A;
    ra.A = a.A;
    ra.B = a.B;
    ra.theta_dis = a.theta_dis;
    ra.beam_cos = a.beam_cos;
    ra.side = a.side;
    ra.ttc_thresh = a.ttc_thresh;
    ra.obs = a.out.obs;
    ra.obs_len = (int32_t)obs_row(a);
    ra.lidar_max = (float)a.p.lidar_max;
    ra.obs_rinv = obs_reciprocal(ra.lidar_max);
    ra.scans_f32 = a.out.scans;
    ra.scans_f64 = a.out.scans_f64;
    // the padded table (see k_rays_fxn's PAD): t = x / res + 2^24 + P
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
    fa.s = a;
    fa.nsteps = n;
    fa.act_stride = act_stride;
    fa.cpw = a.fused_cpw < 1 ? 1 : (a.fused_cpw > kStep1MaxCpw ? kStep1MaxCpw : a.fused_cpw);
    void *args[] = {&fa};
    const size_t lds = (size_t)fa.cpw * (sizeof(Step1Shared) + ((size_t)a.B * 2 + 15) / 16 * 16);
    const unsigned nblk = (unsigned)((a.E + fa.cpw - 1) / fa.cpw);
    if ((e = hipExtLaunchKernel(reinterpret_cast<const void *>(&k_step1), dim3(nblk), dim3(64 * fa.cpw), args, lds, s,
                                ev ? ev[2] : nullptr, ev ? ev[3] : nullptr, 0)) != hipSuccess)
        return e;
    if (ev && (e = hipEventRecord(ev[4], s)) != hipSuccess) return e;
    if (ev && (e = hipEventRecord(ev[5], s)) != hipSuccess) return e;
    return hipSuccess;
}

hipError_t launch_env_step(const StepArgs &a, hipStream_t s, hipEvent_t *ev) {
    const int EA = a.E * a.A;
    hipError_t e;
    auto evk = [&](int i) -> hipEvent_t { return ev ? ev[i] : nullptr; };  // (start, stop) pairs (launch_step1)
    // 64-thread blocks: a few thousand cars must still spread over all CUs
    hipExtLaunchKernelGGL(k_agents, dim3((EA + 63) / 64), dim3(64), 0, s, evk(0), evk(1), 0, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (a.gate_wait && (e = hipStreamWaitEvent(s, a.gate_wait, 0)) != hipSuccess) return e;
    const int64_t R = (int64_t)EA * a.B;
    const dim3 grid((unsigned)((R + kBlock - 1) / kBlock));
    // tiled kernel: TTC in the ray pass; single-agent envs also write their
    // outputs there (k_post_single), multi-agent envs go through k_post_multi
    const bool tiled = a.ray_kernel != 0;
    const bool single = a.A == 1 && tiled;
    if (a.ray_kernel == 0) {
        hipExtLaunchKernelGGL(k_rays, grid, dim3(kBlock), 0, s, evk(2), evk(3), 0, a);
    } else {
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
        dim3 g2 = grid;
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
        const int v = (ch ? 8 : 0) + (rot ? 4 : 0) + (mask ? 2 : 0) + (single ? 0 : 1);  // HANDOFF for A >= 2
        unsigned lds_bytes = a.fx_lds;  // dynamic LDS of the fixed-point kernels (F110_FX_LDS: occupancy probe)
        const void *fn[16] = {
            reinterpret_cast<const void *>(&k_rays_tiled<false, false, false, false>),
            reinterpret_cast<const void *>(&k_rays_tiled<false, false, true, false>),
            reinterpret_cast<const void *>(&k_rays_tiled<false, true, false, false>),
            reinterpret_cast<const void *>(&k_rays_tiled<false, true, true, false>),
            reinterpret_cast<const void *>(&k_rays_tiled<true, false, false, false>),
            reinterpret_cast<const void *>(&k_rays_tiled<true, false, true, false>),
            reinterpret_cast<const void *>(&k_rays_tiled<true, true, false, false>),
            reinterpret_cast<const void *>(&k_rays_tiled<true, true, true, false>),
            reinterpret_cast<const void *>(&k_rays_tiled<false, false, false, true>),
            reinterpret_cast<const void *>(&k_rays_tiled<false, false, true, true>),
            reinterpret_cast<const void *>(&k_rays_tiled<false, true, false, true>),
            reinterpret_cast<const void *>(&k_rays_tiled<false, true, true, true>),
            reinterpret_cast<const void *>(&k_rays_tiled<true, false, false, true>),
            reinterpret_cast<const void *>(&k_rays_tiled<true, false, true, true>),
            reinterpret_cast<const void *>(&k_rays_tiled<true, true, false, true>),
            reinterpret_cast<const void *>(&k_rays_tiled<true, true, true, true>)};
        void *args[] = {&ra};
        const void *f = fn[v];
        // k_rays_fx (ray_kernel 3; f110_create checked its preconditions: axis-aligned
        // map, one-wave blocks, W, H < 2^21, |origin / res| < 2^20, EDT entries 0 or > eps)
        const bool fx = a.ray_kernel == 3 && !rot && ra.wpb == 1;
        if (fx) {
            ra.fx_cx = std::fma(-a.tmap.ox, a.tmap.inv_res, kFxMagic);
            ra.fx_cy = std::fma(-a.tmap.oy, a.tmap.inv_res, kFxMagic);
            ra.fx_lim = 2097152.0 - 32.0 - a.max_range * a.tmap.inv_res;
            ra.ev = a.ev;
            ra.ev_gb = a.ev_gb;
            ra.ev_ctr = a.ev_ctr;
            ra.ev_cap = a.ev_cap;
            ra.ev_capp = a.ev_capp;
            ra.ev_P = a.ev_P;
            ra.ev_T = a.ev_T;
            ra.ev_K = a.ev_K;
            const void *fx_fn[8] = {reinterpret_cast<const void *>(&k_rays_fx<false, false, false>),
                                    reinterpret_cast<const void *>(&k_rays_fx<false, true, false>),
                                    reinterpret_cast<const void *>(&k_rays_fx<true, false, false>),
                                    reinterpret_cast<const void *>(&k_rays_fx<true, true, false>),
                                    reinterpret_cast<const void *>(&k_rays_fx<false, false, true>),
                                    reinterpret_cast<const void *>(&k_rays_fx<false, true, true>),
                                    reinterpret_cast<const void *>(&k_rays_fx<true, false, true>),
                                    reinterpret_cast<const void *>(&k_rays_fx<true, true, true>)};
            f = fx_fn[(a.ev ? 4 : 0) + (mask ? 2 : 0) + (single ? 0 : 1)];
            if (!a.ev && a.rm && !a.fx_tiled) {
                // the row-major EDT (dt[-1,-1] in the padding column / row, a
                // zero cell past the end): N rays per lane (k_rays_fxn) or the
                // single-ray loop (k_rays_fx<.., 3>, heavy-first capable)
                ra.m.dt = a.rm;
                ra.m.wt = a.rm_w;
                ra.m.oob = (int32_t)a.rm_oob;
                ra.fx_zero = a.rm_zero;
                const int N = a.fx_ilp;
                const int v2 = (mask ? 2 : 0) + (single ? 0 : 1);
                if (N >= 2 && N <= 4) {
                    const void *fn_n[3][4] = {
                        {reinterpret_cast<const void *>(&k_rays_fxn<2, false, false>),
                         reinterpret_cast<const void *>(&k_rays_fxn<2, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<2, true, false>),
                         reinterpret_cast<const void *>(&k_rays_fxn<2, true, true>)},
                        {reinterpret_cast<const void *>(&k_rays_fxn<3, false, false>),
                         reinterpret_cast<const void *>(&k_rays_fxn<3, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<3, true, false>),
                         reinterpret_cast<const void *>(&k_rays_fxn<3, true, true>)},
                        {reinterpret_cast<const void *>(&k_rays_fxn<4, false, false>),
                         reinterpret_cast<const void *>(&k_rays_fxn<4, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<4, true, false>),
                         reinterpret_cast<const void *>(&k_rays_fxn<4, true, true>)}};
                    const void *fn_p[3][4] = {
                        {reinterpret_cast<const void *>(&k_rays_fxn<2, false, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<2, false, true, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<2, true, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<2, true, true, true>)},
                        {reinterpret_cast<const void *>(&k_rays_fxn<3, false, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<3, false, true, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<3, true, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<3, true, true, true>)},
                        {reinterpret_cast<const void *>(&k_rays_fxn<4, false, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<4, false, true, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<4, true, false, true>),
                         reinterpret_cast<const void *>(&k_rays_fxn<4, true, true, true>)}};
                    ra.nch = (ra.nch + N - 1) / N;  // chunk groups per car (heavy list / wcost units)
                    g2 = dim3((unsigned)(ra.HB + ra.G4 * ra.nch));
                    f = fn_n[N - 2][v2];
                    const bool pad = a.fx_pad && a.rmp;
                    if (pad) {
                        // the padded table (PAD): t = x / res + 2^24 + P; a car's rays stay in
                        // the table when its origin's q + P lies in [Rn, W or H + 2P - Rn),
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
                        f = fn_p[N - 2][v2];
                    }
                    const int pool = a.fx_pool;
                    if (pool > 0 && pool <= 2 && N == 2 && pad && !mask && ra.HB == 0 && !ra.wcost && a.pcost &&
                        pool * ra.nch <= 64) {
                        // k_rays_fxp: lane-level refill over a pool of cars per wave (F110_FX_POOL)
                        const int NC = pool;
                        const void *fp[2][2] = {{reinterpret_cast<const void *>(&k_rays_fxp<false, 1>),
                                                 reinterpret_cast<const void *>(&k_rays_fxp<true, 1>)},
                                                {reinterpret_cast<const void *>(&k_rays_fxp<false, 2>),
                                                 reinterpret_cast<const void *>(&k_rays_fxp<true, 2>)}};
                        f = fp[NC - 1][single ? 0 : 1];
                        ra.pcost = a.pcost;
                        ra.pool_T = a.pool_T;
                        g2 = dim3((unsigned)((ra.EA + NC - 1) / NC));
                        lds_bytes = (unsigned)(NC * sizeof(PoolCar) + 256 + NC * a.B * 2);
                    } else if (a.fx_refill && N == 2 && !mask && ra.HB == 0 && !ra.wcost) {
                        // one wave per car, two chunk slots with refill (k_rays_fxr; no heavy-first)
                        const void *fr[8] = {reinterpret_cast<const void *>(&k_rays_fxr<false, false, 2>),
                                             reinterpret_cast<const void *>(&k_rays_fxr<true, false, 2>),
                                             reinterpret_cast<const void *>(&k_rays_fxr<false, true, 2>),
                                             reinterpret_cast<const void *>(&k_rays_fxr<true, true, 2>),
                                             reinterpret_cast<const void *>(&k_rays_fxr<false, false, 3>),
                                             reinterpret_cast<const void *>(&k_rays_fxr<true, false, 3>),
                                             reinterpret_cast<const void *>(&k_rays_fxr<false, true, 3>),
                                             reinterpret_cast<const void *>(&k_rays_fxr<true, true, 3>)};
                        f = fr[(a.fx_slots == 3 ? 4 : 0) + (pad ? 2 : 0) + (single ? 0 : 1)];
                        if (pad && a.fxr_lean) {  // the lean refill pass (same outputs), 2 or 3 slots
                            const void *fs[4] = {reinterpret_cast<const void *>(&k_rays_fxs<false, 2>),
                                                 reinterpret_cast<const void *>(&k_rays_fxs<true, 2>),
                                                 reinterpret_cast<const void *>(&k_rays_fxs<false, 3>),
                                                 reinterpret_cast<const void *>(&k_rays_fxs<true, 3>)};
                            f = fs[(a.fx_slots == 3 ? 2 : 0) + (single ? 0 : 1)];
                            if (a.fxs_pipe && a.fx_slots != 3)  // software-pipelined slots (F110_FXS_PIPE, A/B)
                                f = single ? reinterpret_cast<const void *>(&k_rays_fxs<false, 2, true>)
                                           : reinterpret_cast<const void *>(&k_rays_fxs<true, 2, true>);
                            if (a.fxs_pipe && a.fx_slots != 3 && a.cs2 && a.bs2)  // packed tables (F110_FXS_PACK, A/B)
                                f = single ? reinterpret_cast<const void *>(&k_rays_fxs<false, 2, true, 0, true>)
                                           : reinterpret_cast<const void *>(&k_rays_fxs<true, 2, true, 0, true>);
                            if (!a.fxs_pipe && a.fx_slots != 3 && a.fxs_maskld == 3)  // merged slot gathers (A/B)
                                f = single ? reinterpret_cast<const void *>(&k_rays_fxs<false, 2, false, 3>)
                                           : reinterpret_cast<const void *>(&k_rays_fxs<true, 2, false, 3>);
                            if (a.fxs_pipe && a.fx_slots != 3 && a.fxs_maskld && a.fxs_maskld != 3)  // no zero-cell gathers (F110_FXS_MASKLD)
                                f = a.fxs_maskld == 2
                                        ? (single ? reinterpret_cast<const void *>(&k_rays_fxs<false, 2, true, 2>)
                                                  : reinterpret_cast<const void *>(&k_rays_fxs<true, 2, true, 2>))
                                        : (single ? reinterpret_cast<const void *>(&k_rays_fxs<false, 2, true, 1>)
                                                  : reinterpret_cast<const void *>(&k_rays_fxs<true, 2, true, 1>));
                            if (a.fx_lpool && a.pcost && a.fx_slots != 3 && a.fx_refill == 1 && (a.B + 63) / 64 <= 64) {
                                // k_rays_fxq: lane-level refill over the car's beams (F110_FX_LPOOL)
                                f = single ? reinterpret_cast<const void *>(&k_rays_fxq<false>)
                                           : reinterpret_cast<const void *>(&k_rays_fxq<true>);
                                ra.pcost = a.pcost;
                                ra.pool_T = a.pool_T;
                                lds_bytes = (unsigned)(((a.B + 63) & ~63) * 4 + 256 + ((a.B * 2 + 15) & ~15));
                            }
                        }
                        ra.G4 = std::min(a.fx_refill, (a.B + 63) / 64);  // waves per car
                        g2 = dim3((unsigned)(ra.EA * ra.G4));
                    }
                } else {
                    const void *fn_1[4] = {reinterpret_cast<const void *>(&k_rays_fx<false, false, false, 3>),
                                           reinterpret_cast<const void *>(&k_rays_fx<false, true, false, 3>),
                                           reinterpret_cast<const void *>(&k_rays_fx<true, false, false, 3>),
                                           reinterpret_cast<const void *>(&k_rays_fx<true, true, false, 3>)};
                    f = fn_1[v2];
                    if (a.fx_spec_k > 1 && a.fx_spec_t > 0) {  // speculative steps in the tail (F110_FX_SPEC, A/B)
                        const void *fn_s[2][4] = {
                            {reinterpret_cast<const void *>(&k_rays_fx<false, false, false, 3, true, 2>),
                             reinterpret_cast<const void *>(&k_rays_fx<false, true, false, 3, true, 2>),
                             reinterpret_cast<const void *>(&k_rays_fx<true, false, false, 3, true, 2>),
                             reinterpret_cast<const void *>(&k_rays_fx<true, true, false, 3, true, 2>)},
                            {reinterpret_cast<const void *>(&k_rays_fx<false, false, false, 3, true, 4>),
                             reinterpret_cast<const void *>(&k_rays_fx<false, true, false, 3, true, 4>),
                             reinterpret_cast<const void *>(&k_rays_fx<true, false, false, 3, true, 4>),
                             reinterpret_cast<const void *>(&k_rays_fx<true, true, false, 3, true, 4>)}};
                        f = fn_s[a.fx_spec_k == 4 ? 1 : 0][v2];
                        ra.fx_spec_t = a.fx_spec_t;
                    }
                }
            }
            if (a.fx_nolean && single && !mask && !a.ev)  // A/B: the round-2 loop (tiled EDT)
                f = reinterpret_cast<const void *>(&k_rays_fx<false, false, false, 0, false>);
        }
        if (a.wtrace && ch && !rot && !mask && !fx)  // diagnostic wave trace (f110_debug_wave_trace)
            f = single ? reinterpret_cast<const void *>(&k_rays_tiled<false, false, false, true, true>)
                       : reinterpret_cast<const void *>(&k_rays_tiled<false, false, true, true, true>);
        ra.wtrace = a.wtrace;
        const unsigned bdim = ch ? 64u * (unsigned)ra.wpb : (unsigned)kBlock;
        const bool tail = fx && a.ev;
        if ((e = hipExtLaunchKernel(f, g2, dim3(bdim), args, fx ? lds_bytes : 0u, s, evk(2), tail ? nullptr : evk(3),
                                    0)) != hipSuccess)
            return e;
        if (tail) {  // the handed-off stragglers (the queue is read on the device)
            const unsigned tg = (unsigned)std::max<int64_t>(
                a.ev_P, std::min<int64_t>(kTailWaves, ((int64_t)a.ev_cap + 63) / 64) / a.ev_P * a.ev_P);
            const void *tf = single ? reinterpret_cast<const void *>(&k_rays_fx_tail<false>)
                                    : reinterpret_cast<const void *>(&k_rays_fx_tail<true>);
            if ((e = hipExtLaunchKernel(tf, dim3(tg), dim3(64), args, 0, s, nullptr, evk(3), 0)) != hipSuccess) return e;
        }
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (a.gate_record && (e = hipEventRecord(a.gate_record, s)) != hipSuccess) return e;
    if (single)
        hipExtLaunchKernelGGL(k_post_single, dim3((a.E + 63) / 64), dim3(64), 0, s, evk(4), evk(5), 0, a);
    else if (tiled)
    {
        if (a.multi_block == 64) hipExtLaunchKernelGGL(k_post_multi<64>, dim3(a.E), dim3(64), 0, s, evk(4), evk(5), 0, a);
        else hipExtLaunchKernelGGL(k_post_multi<kMultiBlock>, dim3(a.E), dim3(kMultiBlock), 0, s, evk(4), evk(5), 0, a);
    }
    else
        hipExtLaunchKernelGGL(k_post, dim3(a.E), dim3(kBlock), post_lds_bytes(a.A, a.B), s, evk(4), evk(5), 0, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return hipSuccess;
}

// ------------------------------------------------------------------------
// ScanSimulator2D.scan with rng=None for M poses: one thread per ray, beam
// runs rebuilt per thread (cheap: < 20 runs), optional probes.
template <int V>
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
            d = a.map.dt[V == 1 ? cell_index(a.map, x, y) : cell_index_fast(a.map, x, y)];
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
    if (a.variant == 1)
        hipLaunchKernelGGL(k_scan_batch<1>, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL(k_scan_batch<0>, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
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
