// f110_kernels.hip — gfx950 kernels of the batched F1TENTH step.
//
//  k_env_step     one 256-thread workgroup (4 waves) per environment; the
//                 whole Simulator.step + F110Env.step of that env in one
//                 launch: dynamics -> 1080*A sphere-traced rays (scan held in
//                 LDS) -> GJK -> TTC -> agent ray_cast -> obs pack / done.
//  k_scan_batch   ScanSimulator2D.scan (rng=None) for M arbitrary poses.
//  k_dynamics     vehicle_dynamics_st on M (x, u) pairs.
//
// The ray loop is latency bound (dependent gathers into the EDT, ~7 per ray):
// each wave owns a contiguous pool of rays and every lane that finishes a ray
// immediately takes the next one from the pool (ballot + popcount, no
// atomics), so lanes stay busy until the pool drains instead of idling
// behind the longest ray of a fixed 64-ray group.
#include <hip/hip_runtime.h>

#include "f110_internal.h"

namespace f110 {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

struct EnvShared {
    double stl[kMaxAgents][7];   // state after update_pose (TTC may zero 3..6)
    double spose[kMaxAgents][2]; // scan pose x, y (lidar offset applied)
    double apose[kMaxAgents][3]; // agent_poses (x, y, yaw) before TTC (base_classes.py:587)
    double verts[kMaxAgents][8]; // get_vertices(agent_poses)
    double d0[kMaxAgents];       // EDT at the scan pose (first lookup of every ray)
    int32_t nruns[kMaxAgents];
    int32_t hit[kMaxAgents];     // TTC hit
    int32_t col[kMaxAgents];     // collisions (GJK | TTC)
    int32_t blo[kMaxAgents * kMaxAgents], bhi[kMaxAgents * kMaxAgents];
    int32_t do_reset;
    int32_t pad_;
    uint64_t noise_step;
};

static_assert(sizeof(EnvShared) % 16 == 0, "LDS carve alignment");
static_assert(sizeof(BeamRun) == 24, "BeamRun layout");

size_t step_lds_bytes(int A, int B) {
    size_t runs = sizeof(BeamRun) * (size_t)A * kMaxSeg;
    runs = (runs + 15) & ~(size_t)15;
    return sizeof(EnvShared) + runs + sizeof(double) * (size_t)A * B;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Ray pool of one wave.  Ray id -> (agent a = id / B, beam b = id % B).
// Fin(id, range, lookups) consumes each finished ray (range already clamped).
template <class Fin>
__device__ __forceinline__ uint32_t trace_pool(const MapView &m, const double *__restrict__ sines,
                                               const double *__restrict__ cosines, int theta_dis, double eps,
                                               double max_range, int B, int begin, int end,
                                               const double (*spose)[2], const double *d0,
                                               const BeamRun *runs, const int32_t *nruns, Fin fin) {
    const int lane = threadIdx.x & 63;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t look_total = 0;
    int next = begin + 64;
    int my = begin + lane;
    bool act = my < end;
    double x = 0, y = 0, c = 0, s = 0, d = 0, tot = 0;
    uint32_t n = 0;
    auto init = [&](int id) {
        int a = id / B;
        int b = id - a * B;
        double t = beam_theta_index(runs + a * kMaxSeg, nruns[a], b);
        int ti = (int)t;                 // int(theta_index), laser_models.py:124
        if (ti >= theta_dis) ti = 0;
        s = sines[ti];
        c = cosines[ti];
        x = spose[a][0];
        y = spose[a][1];
        d = d0[a];                       // :129
        tot = d;                         // :130
        n = 1;
    };
    if (act) init(my);
    while (true) {
        bool done = act && !(d > eps && tot <= max_range);   // :133
        uint64_t dm = __ballot(done);
        while (dm) {
            if (done) {
                look_total += n;
                fin(my, tot > max_range ? max_range : tot, n);  // :143-144
                my = next + __popcll(dm & lt);
                act = my < end;
                if (act) init(my);
            }
            next += __popcll(dm);
            done = act && !(d > eps && tot <= max_range);
            dm = __ballot(done);
        }
        if (!__ballot(act)) break;
        if (act) {                        // :135-141
            x += d * c;
            y += d * s;
            d = m.dt[cell_index(m, x, y)];
            tot += d;
            ++n;
        }
    }
    return look_total;
}

// ------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_env_step(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    EnvShared &sh = *reinterpret_cast<EnvShared *>(smem);
    size_t runs_bytes = (sizeof(BeamRun) * (size_t)a.A * kMaxSeg + 15) & ~(size_t)15;
    BeamRun *runs = reinterpret_cast<BeamRun *>(smem + sizeof(EnvShared));
    double *scan = reinterpret_cast<double *>(smem + sizeof(EnvShared) + runs_bytes);

    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    const int A = a.A, B = a.B;
    const int EA = a.E * A;
    const uint64_t genv = (uint64_t)(a.env_offset + e);

    // ---- which envs run, and do they reset? (uniform per block) ----------
    int do_reset;
    if (a.mode == 1) {
        if (a.reset_mask && !a.reset_mask[e]) return;
        do_reset = 1;
    } else {
        do_reset = (a.autoreset && a.pending[e]) ? 1 : 0;
    }

    // ---- phase A: one lane per agent: reset, update_pose, scan setup --------
    if (tid < A) {
        const int ag = tid;
        const int g = e * A + ag;
        double s[7];
        double b0, b1;
        int cnt;
        double raw_steer, vel;
        if (do_reset) {
            // RaceCar.reset (base_classes.py:183-204) then F110Env.reset's zero step (f110_env.py:457)
            const double *pz;
            if (a.mode == 1) {
                pz = a.reset_poses + ((size_t)e * A + ag) * 3;
            } else {
                uint64_t ep = a.episode[e];
                uint32_t k = spawn_draw(a.seed, genv, ep) % (uint32_t)a.n_spawn;
                pz = a.spawn + ((size_t)k * A + ag) * 3;
            }
#pragma unroll
            for (int k = 0; k < 7; ++k) s[k] = 0.0;
            s[0] = pz[0];
            s[1] = pz[1];
            s[4] = pz[2];
            b0 = b1 = 0.0;
            cnt = 0;
            raw_steer = 0.0;
            vel = 0.0;
            a.start[g] = pz[0];
            a.start[EA + g] = pz[1];
            a.start[2 * EA + g] = pz[2];
            a.toggles[g] = 0;
            a.near_start[g] = 1;
            a.lap_times[g] = 0.0f;
            a.lap_counts[g] = 0.0f;
        } else {
#pragma unroll
            for (int k = 0; k < 7; ++k) s[k] = a.st[(size_t)k * EA + g];
            b0 = a.sb[g];
            b1 = a.sb[EA + g];
            cnt = a.scnt[g];
            raw_steer = (double)a.actions[(size_t)g * 2];
            vel = (double)a.actions[(size_t)g * 2 + 1];
        }
        update_pose(s, b0, b1, cnt, raw_steer, vel, a.p, a.dt, a.integrator);
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            a.st[(size_t)k * EA + g] = s[k];
            sh.stl[ag][k] = s[k];
        }
        a.sb[g] = b0;
        a.sb[EA + g] = b1;
        a.scnt[g] = cnt;
        double sx = s[0] + a.lidar_dist * cos(s[4]);  // base_classes.py:420-422
        double sy = s[1] + a.lidar_dist * sin(s[4]);
        sh.spose[ag][0] = sx;
        sh.spose[ag][1] = sy;
        sh.apose[ag][0] = s[0];
        sh.apose[ag][1] = s[1];
        sh.apose[ag][2] = s[4];
        sh.d0[ag] = a.map.dt[cell_index(a.map, sx, sy)];
        double t0 = first_theta_index(s[4], a.fov, a.theta_dis);
        sh.nruns[ag] = build_beam_runs(t0, a.inc, a.theta_dis, B, runs + ag * kMaxSeg, kMaxSeg);
        sh.hit[ag] = 0;
        sh.col[ag] = 0;
    }
    if (tid == 0) {
        sh.do_reset = do_reset;
        sh.noise_step = do_reset ? 0ull : a.nstep[e];
    }
    __syncthreads();

    // ---- phase B: A*B rays, per-wave pools with lane refill ----------------
    {
        const int R = A * B;
        const int wave = tid >> 6;
        const int chunk = (R + kWaves - 1) / kWaves;
        const int begin = wave * chunk;
        const int end = min(R, begin + chunk);
        const double nstd = a.noise_std;
        const uint64_t nstep = sh.noise_step;
        const uint64_t seed = a.seed;
        uint32_t looks = trace_pool(
            a.map, a.sines, a.cosines, a.theta_dis, a.eps, a.max_range, B, begin, end, sh.spose, sh.d0, runs,
            sh.nruns, [&](int id, double range, uint32_t) {
                if (nstd > 0.0) {  // ScanSimulator2D.scan noise, added after the clamp (laser_models.py:450-452)
                    int b = id % B;
                    range += nstd * beam_normal(seed, genv, nstep, b);
                }
                scan[id] = range;
            });
        uint32_t tot = wave_sum(looks);
        if ((tid & 63) == 0 && a.ctr) {
            atomicAdd(a.ctr, (unsigned long long)tot);
            atomicAdd(a.ctr + 1, (unsigned long long)(end > begin ? end - begin : 0));
        }
    }
    __syncthreads();

    // ---- phase C1: GJK between agents (check_collision, base_classes.py:549-563) --
    if (tid < A) {
        get_vertices(sh.apose[tid][0], sh.apose[tid][1], sh.apose[tid][2], a.p.length, a.p.width, sh.verts[tid]);
    }
    // ---- phase C2: TTC against the environment (check_ttc_jit, laser_models.py:188-217)
    for (int id = tid; id < A * B; id += kBlock) {
        int ag = id / B;
        int b = id - ag * B;
        double v = sh.stl[ag][3];
        if (v != 0.0) {
            double proj_vel = v * a.beam_cos[b];
            double ttc = (scan[id] - a.side[b]) / proj_vel;
            if (ttc < a.ttc_thresh && ttc >= 0.0) sh.hit[ag] = 1;
        }
    }
    __syncthreads();
    if (tid == 0) {
        for (int i = 0; i < A - 1; ++i)  // collision_multiple, collision_models.py:184-212
            for (int j = i + 1; j < A; ++j)
                if (gjk_collision(sh.verts[i], sh.verts[j])) {
                    sh.col[i] = 1;
                    sh.col[j] = 1;
                }
    }
    __syncthreads();
    // ---- phase C3: collision response, blocked beam ranges -------------------
    if (tid < A) {
        const int g = e * A + tid;
        if (sh.hit[tid]) {  // RaceCar.check_ttc, base_classes.py:246-249: state[3:] = 0
#pragma unroll
            for (int k = 3; k < 7; ++k) {
                sh.stl[tid][k] = 0.0;
                a.st[(size_t)k * EA + g] = 0.0;
            }
            sh.col[tid] = 1;  // Simulator.step :601-602
        }
    }
    __syncthreads();
    if (tid < A * (A - 1)) {  // pair (i, jj-th opponent) -> get_blocked_view_indices
        int i = tid / (A - 1);
        int jj = tid - i * (A - 1);
        int j = jj < i ? jj : jj + 1;
        int lo, hi;
        blocked_range(sh.stl[i][0], sh.stl[i][1], sh.stl[i][4], sh.verts[j], a.angles, B, a.fov, a.beam_incr, lo,
                      hi);
        sh.blo[tid] = lo;
        sh.bhi[tid] = hi;
    }
    __syncthreads();
    // ---- phase C4: agent ray_cast (RaceCar.ray_cast_agents, base_classes.py:206-227)
    for (int jj = 0; jj < A - 1; ++jj) {
        for (int i = 0; i < A; ++i) {
            int j = jj < i ? jj : jj + 1;
            int pr = i * (A - 1) + jj;
            int lo = sh.blo[pr], hi = sh.bhi[pr];
            const double ox = sh.stl[i][0], oy = sh.stl[i][1], oth = sh.stl[i][4];
            const double *v = sh.verts[j];
            for (int b = lo + tid; b <= hi; b += kBlock) {
                double bt = oth + a.angles[b] + kPi / 2.;
                double v30 = cos(bt), v31 = sin(bt);
                double cur = scan[i * B + b];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    int q1 = (q + 1) & 3;
                    double r = get_range(ox, oy, v30, v31, v[2 * q], v[2 * q + 1], v[2 * q1], v[2 * q1 + 1]);
                    if (r < cur) cur = r;
                }
                scan[i * B + b] = cur;
            }
        }
        __syncthreads();
    }

    // ---- phase D: outputs ---------------------------------------------------
    const int obs_len = B + 4 * A;
    if (a.out.obs) {  // F110Env._pack_flat_obs, f110_env.py:552-584 (scan of agent 0)
        float *o = a.out.obs + (size_t)e * obs_len;
        const float lmax = (float)a.p.lidar_max;
        for (int b = tid; b < B; b += kBlock) {
            float v = (float)scan[b];
            if (v != v) v = lmax;
            else if (isinf(v)) v = v > 0 ? lmax : 0.0f;
            v = v < 0.0f ? 0.0f : (v > lmax ? lmax : v);
            o[b] = v / lmax;
        }
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
    if (tid == 0) {
        // F110Env.step time + _check_done (f110_env.py:404-406, :310-352)
        double tnow = (sh.do_reset ? 0.0 : a.sim_time[e]) + a.dt;
        a.sim_time[e] = tnow;
        const double th = a.start[2 * EA + e * A + a.ego];
        const double r00 = cos(-th), r01 = -sin(-th), r10 = sin(-th), r11 = cos(-th);
        bool all4 = true;
        for (int i = 0; i < A; ++i) {
            const int g = e * A + i;
            double px = sh.stl[i][0] - a.start[g];
            double py = sh.stl[i][1] - a.start[EA + g];
            double dx = r00 * px + r01 * py;
            double dy = r10 * px + r11 * py;
            double ty;
            if (dy > 2.0) ty = dy - 2.0;
            else if (dy < -2.0) ty = -2.0 - dy;
            else ty = 0.0;
            bool close = dx * dx + ty * ty <= 0.1;
            int tg = a.toggles[g];
            uint8_t ns = a.near_start[g];
            if (close && !ns) { ns = 1; ++tg; }
            else if (!close && ns) { ns = 0; ++tg; }
            a.toggles[g] = tg;
            a.near_start[g] = ns;
            float lc = (float)(tg / 2);
            float lt = tg < 4 ? (float)tnow : a.lap_times[g];
            a.lap_counts[g] = lc;
            a.lap_times[g] = lt;
            if (a.out.lap_counts) a.out.lap_counts[g] = lc;
            if (a.out.lap_times) a.out.lap_times[g] = lt;
            all4 = all4 && tg >= 4;
        }
        bool term = sh.col[a.ego] || all4;
        if (a.out.terminated) a.out.terminated[e] = term ? 1 : 0;
        if (a.out.was_reset) a.out.was_reset[e] = (uint8_t)sh.do_reset;
        if (a.out.sim_time) a.out.sim_time[e] = tnow;
        a.pending[e] = (a.autoreset && term) ? 1 : 0;
        if (sh.do_reset && a.mode == 0) a.episode[e] += 1;
        a.nstep[e] = sh.noise_step + 1;
    }
    if (a.out.collisions && tid < A) a.out.collisions[(size_t)e * A + tid] = (uint8_t)sh.col[tid];
}

hipError_t prepare_env_step(size_t lds_bytes) {
    if (lds_bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void *>(&k_env_step),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
}

hipError_t launch_env_step(const StepArgs &a, hipStream_t s) {
    size_t lds = step_lds_bytes(a.A, a.B);
    hipLaunchKernelGGL(k_env_step, dim3(a.E), dim3(kBlock), lds, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------
struct ScanShared {
    double spose[1][2];
    double d0[1];
    int32_t nruns[1];
    int32_t pad_;
};

__global__ void __launch_bounds__(kBlock) k_scan_batch(ScanArgs a) {
    __shared__ ScanShared sh;
    __shared__ BeamRun runs[kMaxSeg];
    const int64_t m = blockIdx.x;
    const int tid = threadIdx.x;
    const double *pose = a.poses + 3 * m;
    if (tid == 0) {
        sh.spose[0][0] = pose[0];
        sh.spose[0][1] = pose[1];
        sh.d0[0] = a.map.dt[cell_index(a.map, pose[0], pose[1])];
        double t0 = first_theta_index(pose[2], a.fov, a.theta_dis);
        sh.nruns[0] = build_beam_runs(t0, a.inc, a.theta_dis, a.B, runs, kMaxSeg);
    }
    __syncthreads();
    const int B = a.B;
    const int wave = tid >> 6;
    const int chunk = (B + kWaves - 1) / kWaves;
    const int begin = wave * chunk;
    const int end = min(B, begin + chunk);
    double *out = a.scans + m * B;
    int32_t *lk = a.lookups ? a.lookups + m * B : nullptr;
    uint32_t looks = trace_pool(a.map, a.sines, a.cosines, a.theta_dis, a.eps, a.max_range, B, begin, end, sh.spose,
                                sh.d0, runs, sh.nruns, [&](int id, double range, uint32_t n) {
                                    out[id] = range;
                                    if (lk) lk[id] = (int32_t)n;
                                });
    uint32_t tot = wave_sum(looks);
    if ((tid & 63) == 0 && a.ctr) {
        atomicAdd(a.ctr, (unsigned long long)tot);
        atomicAdd(a.ctr + 1, (unsigned long long)(end > begin ? end - begin : 0));
    }
}

// Probe variant for hit cells: one thread per ray, plain loop (tests only).
__global__ void __launch_bounds__(kBlock) k_scan_probe(ScanArgs a) {
    const int64_t gid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (gid >= a.M * a.B) return;
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
    int64_t cell = cell_index(a.map, x, y);
    double d = a.map.dt[cell];
    double tot = d;
    int n = 1;
    while (d > a.eps && tot <= a.max_range) {
        x += d * c;
        y += d * s;
        cell = cell_index(a.map, x, y);
        d = a.map.dt[cell];
        tot += d;
        ++n;
    }
    if (tot > a.max_range) tot = a.max_range;
    if (a.scans) a.scans[gid] = tot;
    if (a.lookups) a.lookups[gid] = n;
    // recover (r, c) of the last lookup; out-of-map reads report (-1, -1)
    double xt = x - a.map.ox, yt = y - a.map.oy;
    double xr = xt * a.map.oc + yt * a.map.os;
    double yr = -xt * a.map.os + yt * a.map.oc;
    int r = -1, cc = -1;
    if (!(xr < 0 || xr >= a.map.wres || yr < 0 || yr >= a.map.hres || xr != xr || yr != yr)) {
        cc = (int)(xr / a.map.res);
        r = (int)(yr / a.map.res);
    }
    a.hit_rc[2 * gid] = r;
    a.hit_rc[2 * gid + 1] = cc;
}

hipError_t launch_scan_batch(const ScanArgs &a, hipStream_t s) {
    if (a.M <= 0) return hipSuccess;
    if (a.hit_rc) {
        int64_t n = a.M * a.B;
        hipLaunchKernelGGL(k_scan_probe, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_scan_batch, dim3((unsigned)a.M), dim3(kBlock), 0, s, a);
    }
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

}  // namespace f110
