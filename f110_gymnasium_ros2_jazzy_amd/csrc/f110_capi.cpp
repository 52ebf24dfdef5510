// f110_capi.cpp — host side of libf110.so: the C ABI declared in include/f110.h.
//
// Cold path (once per map): exact EDT (Felzenszwalb-Huttenlocher lower
// envelopes, integer arithmetic), the reference's trig tables, device buffers.
// Hot path: f110_step / f110_reset fill a StepArgs and enqueue three kernels
// (k_agents, a ray kernel, a post kernel) on the caller's stream; no
// allocation, no synchronisation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "f110_internal.h"

using namespace f110;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(F110_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

}  // namespace

// shared with f110_replay_capi.cpp (one thread-local error string per library)
int f110_set_error(int code, const std::string &msg) { return fail(code, msg); }

struct MapTables;

struct f110_ctx {
    int device = 0;
    MapTables *maps = nullptr;  // the shared read-only EDT tables (dt, dt_tiled, rm)
    f110_config cfg{};
    f110_params p{};                 // Simulator-level params (fixed at create)
    std::vector<f110_params> agent_p;  // RaceCar params per agent (f110_set_params)
    f110_params *pa = nullptr;       // device copy of agent_p
    int H = 0, W = 0;
    double res = 0, origin[3] = {0, 0, 0};
    double inc = 0, beam_incr = 0;
    int n_spawn = 0;
    // device buffers
    double *dt_tiled = nullptr;
    int32_t wt = 0, tiles_h = 0;
    int ray_kernel = 3;  // F110_RAY_KERNEL: 1 tiled flat order, 2 tiled chunked, 3 the fixed-point
                         // kernels (default; falls back to 2 where their preconditions fail)
    uint8_t chunk_order[kMaxChunks] = {};
    double *dt = nullptr, *sines = nullptr, *cosines = nullptr, *angles = nullptr, *beam_cos = nullptr,
           *side = nullptr, *spawn = nullptr;
    double *cs2 = nullptr, *bs2 = nullptr;  // interleaved (cos, sin)[theta_dis], (side, beam_cos)[B] (k_rays_fxs)
    double side_max = 0.0;                  // max of the side table (k_rays_fxs's TTC pre-test)
    double *start_rot = nullptr;
    double *st = nullptr, *sb = nullptr, *start = nullptr, *sim_time = nullptr, *ray0 = nullptr, *scan = nullptr;
    BeamRun *runs = nullptr;
    int32_t *nruns = nullptr;
    PairGeom *geo = nullptr;  // [E][A][A-1] ray_cast pair geometry (A >= 2)
    uint32_t *hmask = nullptr;  // [E*A] hand-off chunk masks of k_rays_fxs<HANDOFF> (A >= 2 dividing 64)
    uint64_t *noise_step = nullptr;
    int32_t *scnt = nullptr, *toggles = nullptr;
    uint8_t *near_start = nullptr, *pending = nullptr, *reset_flag = nullptr, *ttc_hit = nullptr;
    float *lap_times = nullptr, *lap_counts = nullptr;
    uint64_t *episode = nullptr, *nstep = nullptr;
    unsigned long long *ctr = nullptr;
    std::vector<void *> allocs;
    // f110_profile_begin/end
    std::vector<hipEvent_t> prof_ev;  // 6 per recorded step: (start, stop) of k_agents, the ray kernel, k_post
    int prof_max = 0, prof_n = 0;
    const double *noise_ext = nullptr;  // f110_set_scan_noise (caller-owned)
    uint64_t *wtrace = nullptr;         // f110_debug_wave_trace buffer (diagnostics)
    bool heavy_off = false;             // f110_debug_disable_heavy_first
    bool reset_f32 = false;             // f110_set_reset_dtype
    hipEvent_t gate_wait = nullptr;     // f110_debug_set_ray_gate (caller-owned events)
    hipEvent_t gate_record = nullptr;
    // heavy-first ray dispatch (chunked kernel)
    uint8_t *wcost = nullptr;
    uint32_t *heavy_list = nullptr, *heavy_mask = nullptr, *heavy_count = nullptr;
    int32_t heavy_cap = 0, heavy_T = 16, nch = 0;  // with one-wave blocks and a 1/6 list: 16 best
    uint64_t launch_n = 0;
    int ray_wpb = 1;  // one-wave blocks (4-car blocks measured slower)
    int64_t wtrace_n = 0;
    bool wtrace_armed = false;
    // the fixed-point ray kernel's row-major EDT (see StepArgs::rm)
    double *rm = nullptr;
    int32_t rm_w = 0;
    uint32_t rm_oob = 0, rm_zero = 0;
    const double *rmp = nullptr;  // the padded table of k_rays_fxn / k_rays_fxs (shared, see MapTables)
    int32_t rmp_w = 0, rmp_P = 0, rmp_h = 0;
    uint32_t rmp_zero = 0;
    bool fx_pad = false;    // the padded table is wanted (from 32768 cars or with refill; F110_FX_PAD=0: never)
    int32_t fx_refill = 0;   // waves per car of k_rays_fxs (0 = k_rays_fxn; f110_debug_set_ray_refill)
    bool fxs_lds = false;    // single-agent k_rays_fxs with the LDS theta table (f110_set_device_share, > 1 context)
    bool count_slots = false;  // f110_debug_set_simt: lane-slot counter of the fixed-point loops (f110_debug_read_simt)
    int32_t hcheck = 0;        // f110_debug_set_handoff_check: bit 0 poison + count misses, bit 1 mask off,
                               // bit 2 an empty mask (the check's own test)
    int fx_ilp = 1;         // rays per lane (f110_debug_set_ray_lanes; default by car count)

    hipEvent_t *next_prof_events() {
        if (prof_n >= prof_max) return nullptr;
        return &prof_ev[(size_t)6 * prof_n++];
    }
    void free_prof() {
        for (hipEvent_t e : prof_ev) (void)hipEventDestroy(e);
        prof_ev.clear();
        prof_max = prof_n = 0;
    }

    template <class T>
    hipError_t alloc(T **p, size_t n) {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, n * sizeof(T) > 0 ? n * sizeof(T) : 16);
        if (e != hipSuccess) return e;
        e = hipMemset(q, 0, n * sizeof(T) > 0 ? n * sizeof(T) : 16);
        allocs.push_back(q);
        *p = reinterpret_cast<T *>(q);
        return e;
    }
};

// ----------------------------------------------------------------- tables --
// Host computation of the reference's lookup tables, exactly as NumPy does it
// (each sin/cos called separately: glibc sincos() differs in the last bit).
static double (*volatile g_sin)(double) = ::sin;  // volatile: keep sin/cos separate calls
static double (*volatile g_cos)(double) = ::cos;

extern "C" void f110_host_tables(int32_t theta_dis, int32_t n_beams, double fov, const f110_params *p, double *sines,
                      double *cosines, double *angles, double *beam_cos, double *side) {
    // ScanSimulator2D.__init__, laser_models.py:379-381: linspace(0, 2pi, theta_dis)
    const double stop = 2.0 * kPi;
    const double step = stop / (double)(theta_dis - 1);
    for (int i = 0; i < theta_dis; ++i) {
        double th = (i == theta_dis - 1) ? stop : (double)i * step;
        if (sines) sines[i] = g_sin(th);
        if (cosines) cosines[i] = g_cos(th);
    }
    // RaceCar.__init__, base_classes.py:122-158
    const double incr = fov / (double)(n_beams - 1);
    const double dist_sides = p->width / 2.;
    const double dist_fr = (p->lf + p->lr) / 2.;
    for (int i = 0; i < n_beams; ++i) {
        double angle = -fov / 2. + (double)i * incr;
        if (angles) angles[i] = angle;
        if (beam_cos) beam_cos[i] = g_cos(angle);
        double to_side, to_fr;
        if (angle > 0) {
            if (angle < kPi / 2) {
                to_side = dist_sides / g_sin(angle);
                to_fr = dist_fr / g_cos(angle);
            } else {
                to_side = dist_sides / g_cos(angle - kPi / 2.);
                to_fr = dist_fr / g_sin(angle - kPi / 2.);
            }
        } else {
            if (angle > -kPi / 2) {
                to_side = dist_sides / g_sin(-angle);
                to_fr = dist_fr / g_cos(-angle);
            } else {
                to_side = dist_sides / g_cos(-angle - kPi / 2);
                to_fr = dist_fr / g_sin(-angle - kPi / 2);
            }
        }
        if (side) side[i] = to_fr < to_side ? to_fr : to_side;  // Python min()
    }
}

// Host evaluation of the beam-index runs (tests the run construction on CPU).
extern "C" int f110_host_beam_indices(double yaw, double fov, int32_t theta_dis, int32_t n_beams,
                                      double *theta_index_out) {
    const double inc = (double)theta_dis * (fov / (double)(n_beams - 1)) / (2. * kPi);
    BeamRun runs[kMaxSeg];
    double t0 = first_theta_index(yaw, fov, theta_dis);
    int n = build_beam_runs(t0, inc, theta_dis, n_beams, runs, kMaxSeg);
    if (n < 0) return fail(F110_E_INVALID, "beam index runs exceed kMaxSeg");
    for (int b = 0; b < n_beams; ++b) theta_index_out[b] = beam_theta_index(runs, n, b);
    return n;
}

// The two run builders against each other at yaw (k_agents uses build_beam_runs_fast): 1 when
// they give the same runs, 0 when not, < 0 on error.
extern "C" int f110_host_beam_runs_agree(double yaw, double fov, int32_t theta_dis, int32_t n_beams) {
    const double inc = (double)theta_dis * (fov / (double)(n_beams - 1)) / (2. * kPi);
    BeamRun r0[kMaxSeg], r1[kMaxSeg];
    const double t0 = first_theta_index(yaw, fov, theta_dis);
    const int n0 = build_beam_runs(t0, inc, theta_dis, n_beams, r0, kMaxSeg);
    const int n1 = build_beam_runs_fast(t0, inc, theta_dis, n_beams, r1, kMaxSeg);
    if (n0 != n1) return 0;
    for (int i = 0; i < n0; ++i)
        if (r0[i].start != r1[i].start || r0[i].count != r1[i].count ||
            std::memcmp(&r0[i].t0, &r1[i].t0, 8) != 0 || std::memcmp(&r0[i].delta, &r1[i].delta, 8) != 0)
            return 0;
    return 1;
}

// ---------------------------------------------------------------- EDT ----
// 1-D lower envelope of parabolas y = (x - q)^2 + f[q] over the finite sites,
// compared as exact rationals (Felzenszwalb & Huttenlocher 2012).
namespace {
constexpr int64_t kInf = INT64_MAX / 4;

void edt_1d(const int64_t *f, int n, int64_t *d, int *v, int64_t *zn, int64_t *zd) {
    int k = -1;
    for (int q = 0; q < n; ++q) {
        if (f[q] >= kInf) continue;
        while (k >= 0) {
            int p = v[k];
            // intersection of parabolas q and p: s = N / D
            int64_t N = (f[q] + (int64_t)q * q) - (f[p] + (int64_t)p * p);
            int64_t D = 2 * (int64_t)(q - p);
            if (k == 0) break;
            // drop p if s(q,p) <= z[k] = zn[k]/zd[k]
            if ((__int128)N * zd[k] <= (__int128)zn[k] * D) {
                --k;
            } else {
                break;
            }
        }
        ++k;
        v[k] = q;
        if (k > 0) {
            int p = v[k - 1];
            zn[k] = (f[q] + (int64_t)q * q) - (f[p] + (int64_t)p * p);
            zd[k] = 2 * (int64_t)(q - p);
        }
    }
    if (k < 0) {
        for (int x = 0; x < n; ++x) d[x] = kInf;
        return;
    }
    int j = 0;
    for (int x = 0; x < n; ++x) {
        // advance while z[j+1] < x
        while (j < k && (__int128)zn[j + 1] < (__int128)x * zd[j + 1]) ++j;
        int64_t dx = x - v[j];
        d[x] = dx * dx + f[v[j]];
    }
}
}  // namespace

extern "C" int f110_edt_k(const uint8_t *free_mask, int32_t H, int32_t W, uint32_t *k_out) {
    if (!free_mask || !k_out || H <= 0 || W <= 0) return fail(F110_E_INVALID, "f110_edt_k: bad arguments");
    const size_t N = (size_t)H * W;
    std::vector<int64_t> g(N);
    bool any = false;
    // pass 1: squared distance along each column to the nearest occupied cell
    std::vector<int64_t> col(H), out(H);
    std::vector<int> v(H > W ? H : W);
    std::vector<int64_t> zn((H > W ? H : W) + 1), zd((H > W ? H : W) + 1);
    for (int c = 0; c < W; ++c) {
        for (int r = 0; r < H; ++r) {
            bool occ = free_mask[(size_t)r * W + c] == 0;
            col[r] = occ ? 0 : kInf;
            any = any || occ;
        }
        edt_1d(col.data(), H, out.data(), v.data(), zn.data(), zd.data());
        for (int r = 0; r < H; ++r) g[(size_t)r * W + c] = out[r];
    }
    if (!any) return fail(F110_E_INVALID, "f110_edt_k: map has no occupied cell (EDT undefined)");
    // pass 2: rows
    std::vector<int64_t> row(W), rout(W);
    for (int r = 0; r < H; ++r) {
        for (int c = 0; c < W; ++c) row[c] = g[(size_t)r * W + c];
        edt_1d(row.data(), W, rout.data(), v.data(), zn.data(), zd.data());
        for (int c = 0; c < W; ++c) {
            if (rout[c] > 0xFFFFFFFFll) return fail(F110_E_INVALID, "f110_edt_k: distance overflows uint32");
            k_out[(size_t)r * W + c] = (uint32_t)rout[c];
        }
    }
    return F110_OK;
}

// ---------------------------------------------------------------- misc ----
extern "C" int f110_abi_version(void) { return F110_ABI_VERSION; }
extern "C" const char *f110_last_error(void) { return g_err.c_str(); }

extern "C" void f110_default_params(f110_params *p) {
    // f110_env.py:132-156
    p->mu = 1.0489;
    p->C_Sf = 4.718;
    p->C_Sr = 5.4562;
    p->lf = 0.15875;
    p->lr = 0.17145;
    p->h = 0.074;
    p->m = 3.74;
    p->I = 0.04712;
    p->s_min = -0.4189;
    p->s_max = 0.4189;
    p->sv_min = -3.2;
    p->sv_max = 3.2;
    p->v_switch = 7.319;
    p->a_max = 9.51;
    p->v_min = 0.00000001;
    p->v_max = 20.0;
    p->width = 0.31;
    p->length = 0.58;
    p->lidar_max = 30.0;
}

extern "C" void f110_default_config(f110_config *c) {
    std::memset(c, 0, sizeof(*c));
    c->n_envs = 1;
    c->n_agents = 2;            // f110_env.py:159-162
    c->n_beams = 1080;          // base_classes.py:69
    c->theta_dis = 2000;        // laser_models.py:360
    c->integrator = F110_INTEGRATOR_RK4;  // f110_env.py:176-179
    c->ego_idx = 0;
    c->autoreset = 0;
    c->fov = 4.7;
    c->eps = 0.0001;
    c->max_range = 30.0;
    c->time_step = 0.01;
    c->lidar_dist = 0.0;
    c->ttc_thresh = 0.005;
    c->noise_std = 0.01;
    c->env_offset = 0;
    c->seed = 42;               // f110_env.py:110-113
}

static bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

static MapView make_map_view(const double *dt, int32_t H, int32_t W, double res, const double origin[3]) {
    MapView m;
    m.dt = dt;
    m.H = H;
    m.W = W;
    m.n = (int64_t)H * W;
    m.res = res;
    m.ox = origin[0];
    m.oy = origin[1];
    m.oc = std::cos(origin[2]);  // laser_models.py:421-422 (np.sin/np.cos of the yaml yaw)
    m.os = std::sin(origin[2]);
    m.wres = (double)W * res;
    m.hres = (double)H * res;
    m.inv_res = 1.0 / res;
    return m;
}

static TiledMapView make_tiled_view(const MapView &m, const double *dt_tiled) {
    TiledMapView t;
    t.dt = dt_tiled;
    t.H = m.H;
    t.W = m.W;
    t.wt = (m.W + 3) / 4;
    t.oob = tiled_index(t.wt, m.H - 1, m.W - 1);
    t.res = m.res;
    t.inv_res = m.inv_res;
    t.ox = m.ox;
    t.oy = m.oy;
    t.oc = m.oc;
    t.os = m.os;
    t.wres = m.wres;
    t.hres = m.hres;
    return t;
}

// k_rays_fx's preconditions (f110_kernels.hip): an axis-aligned map (origin
// yaw 0: cos 1, sin 0 exactly, so x_rot == x_trans), one-wave blocks, H and W
// below 2^21 and |origin / res| below 2^20 (on-map t = 1.5*2^22 + q stays in
// [2^22, 2^23)), and every EDT entry 0 or above eps (the loop's d > eps is
// then d != 0; the smallest non-zero entry is res * sqrt(1)).
static bool fx_eligible(int32_t H, int32_t W, double res, const double origin[3], double eps, const uint32_t *edt_k,
                        int32_t wpb) {
    if (origin[2] != 0.0 || wpb != 1) return false;
    if (H >= (1 << 21) || W >= (1 << 19)) return false;  // fx_offset's 24-bit multiply by wt * 128
    const double ir = 1.0 / res;
    if (!(std::fabs(origin[0] * ir) < 1048576.0) || !(std::fabs(origin[1] * ir) < 1048576.0)) return false;
    uint32_t kmin = 0;
    for (size_t i = 0, n = (size_t)H * W; i < n; ++i)
        if (edt_k[i] && (!kmin || edt_k[i] < kmin)) kmin = edt_k[i];
    return !kmin || res * std::sqrt((double)kmin) > eps;
}

static MapView map_view(const f110_ctx *c) { return make_map_view(c->dt, c->H, c->W, c->res, c->origin); }

static int use_device(const f110_ctx *c) {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != c->device) HIP_TRY(hipSetDevice(c->device));
    return F110_OK;
}

// ------------------------------------------------------ shared map tables --
// The EDT tables (row-major dt, the 4x4-tiled copy, the fixed-point kernel's
// padded row-major table) are read-only after f110_create.  Contexts on one
// device built from the same map (same H, W, resolution and EDT) share one
// copy: S stream sub-shards of a GPU's envs (streams.StreamShards) then keep
// one table's neighbourhood in each XCD's L2 instead of S (32 MB per copy of
// the Spielberg table).  Refcounted; F110_SHARE_MAP=0 gives each context its
// own copy (A/B).
struct MapTables {
    int device = 0;
    int32_t H = 0, W = 0;
    uint64_t res_bits = 0;
    std::vector<uint32_t> k;  // the EDT the tables were built from (exact match, not a hash)
    double *dt = nullptr, *dt_tiled = nullptr, *rm = nullptr, *rmp = nullptr;
    int32_t rm_w = 0, rmp_w = 0, rmp_P = 0, rmp_h = 0;
    uint32_t rm_oob = 0, rm_zero = 0, rmp_zero = 0;
    int refs = 0;
    bool shared = true;
};
static std::mutex g_maps_mu;
static std::vector<MapTables *> g_maps;

static void free_map_tables(MapTables *t) {
    (void)hipSetDevice(t->device);
    if (t->dt) (void)hipFree(t->dt);
    if (t->dt_tiled) (void)hipFree(t->dt_tiled);
    if (t->rm) (void)hipFree(t->rm);
    if (t->rmp) (void)hipFree(t->rmp);
    delete t;
}

static void release_map_tables(MapTables *t) {
    if (!t) return;
    std::lock_guard<std::mutex> g(g_maps_mu);
    if (--t->refs > 0) return;
    g_maps.erase(std::remove(g_maps.begin(), g_maps.end(), t), g_maps.end());
    free_map_tables(t);
}

// Uploads into a local buffer and publishes it to *p only once the copy has
// succeeded (a failed upload frees it and leaves *p untouched): a map entry
// shared by other contexts never points at an uninitialised table.
template <class T>
static hipError_t upload(T **p, const std::vector<T> &h) {
    T *d = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&d), std::max<size_t>(h.size() * sizeof(T), 16));
    if (e == hipSuccess) e = hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (d) (void)hipFree(d);
        return e;
    }
    *p = d;
    return hipSuccess;
}

// k_rays_fxn / k_rays_fxs's padded table (PAD, see kFxpBase): cell (r, c) at
// row r + P, column c + P; every other cell holds dt[-1,-1] (the reference's
// off-map read), and a 0.0 after the last row is the zero cell.  Rows of Wp =
// 511 mod 512 cells: the row stride Wp * 8 is 8 bytes short of a multiple of
// 4096, which k_rays_fxs's offset arithmetic needs (kFxsBase); any width
// serves the others.  Built only where its byte offsets stay 32-bit and a row
// stride stays a 24-bit multiplier (else empty: the clamped table is used).
// Host-only (f110_host_map_table tests it on the CPU, under ASan / UBSan too).
static std::vector<double> host_padded_table(int32_t H, int32_t W, int32_t pad, const std::vector<double> &d,
                                             size_t &Wp, size_t &Hp) {
    const size_t N = (size_t)H * W, P = (size_t)pad;
    Wp = ((size_t)W + 2 * P + 1 + 511) / 512 * 512 - 1;
    Hp = (size_t)H + 2 * P;
    if (pad <= 0 || d.size() != N || (Wp * Hp + 16) * 8 >= (1ull << 32) || Wp * 8 >= (1u << 24)) return {};
    std::vector<double> rmp(Wp * Hp + 16, d[N - 1]);
    for (size_t r = 0; r < (size_t)H; ++r)
        for (size_t q = 0; q < (size_t)W; ++q) rmp[(r + P) * Wp + q + P] = d[r * W + q];
    rmp[Wp * Hp] = 0.0;
    return rmp;
}

// k_rays_fx / k_rays_fxn's row-major EDT: rows of Wp cells (W + 1 rounded up
// to 16: 128-B aligned), the padding columns and row H hold dt[-1,-1] (a
// clamped index then reads the reference's off-map value), and a 0.0 after
// the last row is the zero cell of rays that have ended.  Host-only.
static std::vector<double> host_rowmajor_table(int32_t H, int32_t W, const std::vector<double> &d, size_t &Wp,
                                               size_t &Hp) {
    const size_t N = (size_t)H * W;
    Wp = ((size_t)W + 1 + 15) / 16 * 16;
    Hp = (size_t)H + 1;
    if (d.size() != N) return {};
    std::vector<double> rm(Wp * Hp + 16, d[N - 1]);
    for (size_t r = 0; r < (size_t)H; ++r)
        for (size_t q = 0; q < (size_t)W; ++q) rm[r * Wp + q] = d[r * W + q];
    rm[Wp * Hp] = 0.0;
    return rm;
}

// dt = res * EDT (get_dt, laser_models.py:52) -- bit-exact from the integer k
static std::vector<double> host_dt(const uint32_t *edt_k, size_t N, double res) {
    std::vector<double> dt(N);
    for (size_t i = 0; i < N; ++i) dt[i] = res * std::sqrt((double)edt_k[i]);
    return dt;
}

static hipError_t build_padded_table(MapTables *t, int32_t pad, const std::vector<double> &d) {
    size_t Wp = 0, Hp = 0;
    const std::vector<double> rmp = host_padded_table(t->H, t->W, pad, d, Wp, Hp);
    if (rmp.empty()) return hipSuccess;
    const hipError_t e = upload(&t->rmp, rmp);
    if (e == hipSuccess) {  // the metadata only with the table it describes
        t->rmp_w = (int32_t)Wp;
        t->rmp_h = (int32_t)Hp;
        t->rmp_P = pad;
        t->rmp_zero = (uint32_t)(Wp * Hp * 8);
    }
    return e;
}

// Test hook: the padded (kind 1) or row-major (kind 0) table f110_create
// would upload for this EDT, on the host.  Returns the table's length in
// doubles (0 when it is not built: the padded table's limits), fills out when
// out_len is enough, and meta = {rows, cols, zero-cell byte offset}.
extern "C" int64_t f110_host_map_table(const uint32_t *edt_k, int32_t H, int32_t W, double res, int32_t kind,
                                       int32_t pad, double *out, int64_t out_len, int64_t meta[3]) {
    if (!edt_k || H <= 0 || W <= 0 || !(res > 0)) return fail(F110_E_INVALID, "f110_host_map_table: bad arguments");
    const std::vector<double> d = host_dt(edt_k, (size_t)H * W, res);
    size_t Wp = 0, Hp = 0;
    const std::vector<double> t = kind == 1 ? host_padded_table(H, W, pad, d, Wp, Hp) : host_rowmajor_table(H, W, d, Wp, Hp);
    if (meta) {
        meta[0] = (int64_t)Hp;
        meta[1] = (int64_t)Wp;
        meta[2] = t.empty() ? -1 : (int64_t)(Wp * Hp * 8);
    }
    if (out && out_len >= (int64_t)t.size()) std::copy(t.begin(), t.end(), out);
    return (int64_t)t.size();
}

// The tables of (device, map), built and uploaded on first use; `want_rm`
// adds the row-major table if the entry lacks it, `pad` > 0 the table padded
// by `pad` cells on every side (an entry keeps the padding it was built with:
// the kernel's per-car test reads the entry's).  Called with the device current.
static hipError_t acquire_map_tables(int device, const uint32_t *edt_k, int32_t H, int32_t W, double res,
                                     int32_t wt, int32_t tiles_h, bool want_rm, int32_t pad, MapTables **out) {
    std::lock_guard<std::mutex> g(g_maps_mu);
    const size_t N = (size_t)H * W;
    uint64_t rb;
    std::memcpy(&rb, &res, 8);
    bool share = true;
    if (const char *v = std::getenv("F110_SHARE_MAP")) share = std::atoi(v) != 0;
    MapTables *t = nullptr;
    if (share)
        for (MapTables *q : g_maps)
            if (q->shared && q->device == device && q->H == H && q->W == W && q->res_bits == rb &&
                std::memcmp(q->k.data(), edt_k, N * sizeof(uint32_t)) == 0) {
                t = q;
                break;
            }
    const bool fresh = t == nullptr;
    if (fresh) {
        t = new MapTables();
        t->device = device;
        t->H = H;
        t->W = W;
        t->res_bits = rb;
        t->shared = share;
        t->k.assign(edt_k, edt_k + N);
    }
    hipError_t e = hipSuccess;
    std::vector<double> dt;
    auto dt_host = [&]() -> const std::vector<double> & {
        if (dt.empty()) dt = host_dt(edt_k, N, res);
        return dt;
    };
    if (fresh) {
        e = upload(&t->dt, dt_host());
        if (e == hipSuccess) {
            std::vector<double> dtt((size_t)wt * tiles_h * 16, 0.0);  // padding cells are never read
            for (int r = 0; r < H; ++r)
                for (int q = 0; q < W; ++q) dtt[(size_t)tiled_index(wt, r, q)] = dt[(size_t)r * W + q];
            e = upload(&t->dt_tiled, dtt);
        }
    }
    if (e == hipSuccess && want_rm && !t->rm) {
        size_t Wp = 0, Hp = 0;
        e = upload(&t->rm, host_rowmajor_table(H, W, dt_host(), Wp, Hp));
        if (e == hipSuccess) {  // the metadata only with the table it describes
            t->rm_w = (int32_t)Wp;
            t->rm_oob = (uint32_t)(((size_t)(H - 1) * Wp + (W - 1)) * 8);
            t->rm_zero = (uint32_t)(Wp * Hp * 8);
        }
    }
    if (e == hipSuccess && pad > 0 && !t->rmp) e = build_padded_table(t, pad, dt_host());
    if (e != hipSuccess) {
        if (fresh) free_map_tables(t);
        return e;
    }
    if (fresh) g_maps.push_back(t);
    ++t->refs;
    *out = t;
    return hipSuccess;
}

static int ensure_padded_table(f110_ctx *ctx);

// the map entry's padded table (if it was built) for the context
static void adopt_padded_table(f110_ctx *c) {
    if (!c->maps || !c->maps->rmp) return;
    c->rmp = c->maps->rmp;
    c->rmp_w = c->maps->rmp_w;
    c->rmp_h = c->maps->rmp_h;
    c->rmp_P = c->maps->rmp_P;
    c->rmp_zero = c->maps->rmp_zero;
}

// k_rays_fxs's offsets (kFxsBase) need q + P below 2^20 for every lookup: the padded
// table's rows and columns below 2^20 (else the refill runs k_rays_fxn instead)
static bool fxs_ok(const f110_ctx *c) { return c->rmp && c->rmp_w < (1 << 20) && c->rmp_h < (1 << 20); }

// k_rays_fxs's waves per car for `cars` traced at once on the device (one context's cars, or the
// device's under f110_set_device_share).  Round 5 (profiles/r05_ab/shard_rules_*.jsonl, env-steps/s,
// 1 / 2 / 3 waves per car; k_rays_fx in brackets): one context 65536 90.5 / 87.6 / 82.9 M, 32768
// 77.4 / 77.2 / 73.9, 16384 60.9 / 63.1 / 62.0, 8192 46.7 / 49.0 / 49.6 (40.2), 4096 31.8 / 34.9 /
// 35.9 (29.6); 4 sub-shards 16384 73.7 / 74.4 / 74.0, 8192 57.1 / 60.5 / 63.0 (52.0), 4096 36.9 /
// 41.1 / 42.2 (36.1); two-agent envs alike (8192 x 2: 25.4 / 26.3 / 25.8).  A car split over more
// waves shortens the longest car's chain, the launch's tail where the grid is one round deep; where
// it is many rounds deep the extra waves re-fetch the car's neighbourhood on other CUs.
static int32_t refill_waves(int64_t cars) { return cars >= 32768 ? 1 : cars >= 16384 ? 2 : 3; }

extern "C" int f110_create(f110_ctx **out, int32_t device, const f110_config *cfg, const f110_params *params,
                           const uint32_t *edt_k, int32_t H, int32_t W, double resolution, const double origin[3],
                           const double *spawn_poses, int32_t n_spawn) {
    if (!out || !cfg || !params || !edt_k || !origin) return fail(F110_E_INVALID, "f110_create: null argument");
    *out = nullptr;
    const f110_config &C = *cfg;
    if (C.n_envs <= 0 || C.n_agents <= 0 || C.n_agents > kMaxAgents)
        return fail(F110_E_INVALID, "f110_create: n_envs must be > 0 and 1 <= n_agents <= 8");
    if (C.n_beams < 2 || C.theta_dis < 2 || H <= 0 || W <= 0 || !(resolution > 0))
        return fail(F110_E_INVALID, "f110_create: bad sensor/map dimensions");
    if ((uint64_t)(H + 3) * (uint64_t)(W + 3) * 8u >= (1ull << 32))
        return fail(F110_E_INVALID, "f110_create: map too large (the EDT tables are addressed by 32-bit byte offsets)");
    if (!(C.fov > 0) || !(C.fov < 2 * kPi))
        return fail(F110_E_INVALID, "f110_create: fov must be in (0, 2*pi) (one index wrap per scan)");
    if (max_beam_runs((double)C.theta_dis * (C.fov / (double)(C.n_beams - 1)) / (2. * kPi), C.theta_dis) > kMaxSeg)
        return fail(F110_E_INVALID, "f110_create: theta_dis / (fov / n_beams) too large for the beam-index runs "
                                    "(f110_device.h max_beam_runs <= 80)");
    if (C.ego_idx < 0 || C.ego_idx >= C.n_agents) return fail(F110_E_INVALID, "f110_create: bad ego_idx");
    if (C.integrator != F110_INTEGRATOR_RK4 && C.integrator != F110_INTEGRATOR_EULER)
        return fail(F110_E_INVALID, "f110_create: Invalid Integrator Specified (base_classes.py:399)");
    if (C.autoreset && (!spawn_poses || n_spawn <= 0))
        return fail(F110_E_INVALID, "f110_create: autoreset needs a spawn pose table");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(F110_E_NODEVICE, "f110_create: no HIP device visible");
    if (device < 0 || device >= ndev) return fail(F110_E_NODEVICE, "f110_create: device index out of range");
    if (!is_gfx950(device)) return fail(F110_E_NODEVICE, "f110_create: device is not gfx950 (MI355X)");
    HIP_TRY(hipSetDevice(device));

    f110_ctx *c = new f110_ctx();
    c->device = device;
    c->cfg = C;
    c->p = *params;
    c->H = H;
    c->W = W;
    c->res = resolution;
    for (int i = 0; i < 3; ++i) c->origin[i] = origin[i];
    c->inc = (double)C.theta_dis * (C.fov / (double)(C.n_beams - 1)) / (2. * kPi);  // laser_models.py:367-368
    c->beam_incr = C.fov / (double)(C.n_beams - 1);
    c->n_spawn = n_spawn;
    // F110_RAY_KERNEL (A/B): 1 k_rays_tiled in flat ray order, 2 chunked, 3 the fixed-point kernels
    if (const char *v = std::getenv("F110_RAY_KERNEL")) {
        const int k = std::atoi(v);
        c->ray_kernel = k >= 2 && k <= 3 ? k : 1;
    }
    {
        // chunked dispatch order: descending beam chunks (the scan's left edge
        // to its right edge).  Measured against the flat order and five other
        // chunk orders (scripts/chunk_ab.py): fastest at 4096
        // and 8192 envs, 1 and 2 agents.
        const int nch = (C.n_beams + 63) / 64;
        if (nch > kMaxChunks && c->ray_kernel >= 2) c->ray_kernel = 1;
        c->nch = nch;
        for (int i = 0; i < nch && i < kMaxChunks; ++i) c->chunk_order[i] = (uint8_t)(nch - 1 - i);
    }
    const size_t EA = (size_t)C.n_envs * C.n_agents;

    auto cleanup = [&](int code, const std::string &msg) {
        for (void *q : c->allocs) (void)hipFree(q);
        release_map_tables(c->maps);
        delete c;
        return fail(code, msg);
    };
#define ALLOC(ptr, n)                                                        \
    do {                                                                     \
        hipError_t e_ = c->alloc(&(ptr), (n));                               \
        if (e_ != hipSuccess) return cleanup(F110_E_ALLOC, std::string("hipMalloc " #ptr ": ") + hipGetErrorString(e_)); \
    } while (0)

    c->wt = (W + 3) / 4;
    c->tiles_h = (H + 3) / 4;
    ALLOC(c->sines, (size_t)C.theta_dis);
    ALLOC(c->cosines, (size_t)C.theta_dis);
    ALLOC(c->angles, (size_t)C.n_beams);
    ALLOC(c->beam_cos, (size_t)C.n_beams);
    ALLOC(c->side, (size_t)C.n_beams);
    ALLOC(c->cs2, 2 * (size_t)C.theta_dis);
    ALLOC(c->bs2, 2 * (size_t)C.n_beams);
    ALLOC(c->st, 7 * EA);
    ALLOC(c->sb, 2 * EA);
    ALLOC(c->scnt, EA);
    ALLOC(c->ray0, 3 * EA);
    ALLOC(c->runs, (size_t)kMaxSeg * EA);
    ALLOC(c->nruns, EA);
    if (C.n_agents >= 2) ALLOC(c->geo, (size_t)EA * (C.n_agents - 1));
    {
        // k_agents' hand-off chunk masks: their f32 bearings hold to a beam for coordinates below 1 km
        // (handoff_chunks); a larger map stores every chunk instead
        const double extent = std::max(std::fabs(origin[0]), std::fabs(origin[1])) +
                              1.5 * resolution * (double)std::max(H, W);
        if (C.n_agents >= 2 && 64 % C.n_agents == 0 && extent < 1000.0) ALLOC(c->hmask, (size_t)EA);
    }
    ALLOC(c->scan, EA * (size_t)C.n_beams);
    ALLOC(c->reset_flag, (size_t)C.n_envs);
    ALLOC(c->ttc_hit, EA);
    ALLOC(c->noise_step, (size_t)C.n_envs);
    ALLOC(c->start, 3 * EA);
    ALLOC(c->start_rot, 2 * (size_t)C.n_envs);
    ALLOC(c->toggles, EA);
    ALLOC(c->near_start, EA);
    ALLOC(c->lap_times, EA);
    ALLOC(c->lap_counts, EA);
    ALLOC(c->sim_time, (size_t)C.n_envs);
    ALLOC(c->pending, (size_t)C.n_envs);
    ALLOC(c->episode, (size_t)C.n_envs);
    ALLOC(c->nstep, (size_t)C.n_envs);
    ALLOC(c->ctr, (size_t)kCtrSlots * kCtrStride);
    ALLOC(c->pa, (size_t)C.n_agents);
    if (spawn_poses && n_spawn > 0) ALLOC(c->spawn, (size_t)n_spawn * C.n_agents * 3);
    if (c->ray_kernel == 3 && !fx_eligible(H, W, resolution, origin, C.eps, edt_k, c->ray_wpb)) c->ray_kernel = 2;
    if (c->ray_kernel == 3) {
        // the row-major table's byte offsets (one padding column / row, a zero cell) stay 32-bit
        const uint64_t rm_bytes = ((uint64_t)W + 16) / 16 * 16 * ((uint64_t)H + 1) * 8 + 128;
        if (rm_bytes >= (1ull << 32)) c->ray_kernel = 2;
    }
    // k_rays_fxs (one or a few waves per car, two chunk slots with refill, padded EDT) at every size
    // since round 5, when closed slots stopped gathering; it takes no heavy-first list
    // and needs 2 rays per lane (k_rays_fxn<2> runs the masked resets)
    if (c->ray_kernel == 3) {
        c->fx_ilp = 2;
        c->heavy_T = 0;
    } else if (EA >= 32768 || EA <= 8192) {
        // heavy-first (the tiled kernels) pays where one ray grid is a few rounds of waves deep (16384
        // cars: 0.281 vs 0.287 ms), costs where it is deep (65536: 1.288 vs 1.251 ms) or one round or
        // less (8192 cars 0.172 vs 0.167, 4096 cars 0.124 vs 0.109 ms; profiles/r02_ray_ab/ab_heavy.json,
        // profiles/r03_ab/small_shards.json)
        c->heavy_T = 0;
    }
    if (c->ray_kernel >= 2 && c->heavy_T > 0) {
        // up to 1/6 of the waves (measured: ~7% of the waves have a ray longer
        // than 40 lookups and carry ~46% of the wave-iterations)
        const size_t div = 6;  // list capacity = 1/div of the waves
        c->heavy_cap = (int32_t)std::max<size_t>(64, (EA * (size_t)c->nch / div + 3) / 4 * 4);
        ALLOC(c->wcost, EA * (size_t)c->nch);
        ALLOC(c->heavy_list, 2 * (size_t)c->heavy_cap);
        ALLOC(c->heavy_mask, EA);
        ALLOC(c->heavy_count, 2);
    }
#undef ALLOC

    std::vector<double> s(C.theta_dis), co(C.theta_dis), an(C.n_beams), bc(C.n_beams), sd(C.n_beams);
    f110_host_tables(C.theta_dis, C.n_beams, C.fov, params, s.data(), co.data(), an.data(), bc.data(), sd.data());
    c->side_max = -INFINITY;
    for (double v : sd) c->side_max = v > c->side_max ? v : c->side_max;  // NaN-free table (f110_host_tables)
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipMemcpy(c->sines, s.data(), s.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(c->cosines, co.data(), co.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(c->angles, an.data(), an.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(c->beam_cos, bc.data(), bc.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(c->side, sd.data(), sd.size() * sizeof(double), hipMemcpyHostToDevice);
    {
        std::vector<double> cs2(2 * (size_t)C.theta_dis), bs2(2 * (size_t)C.n_beams);
        for (int i = 0; i < C.theta_dis; ++i) {
            cs2[2 * (size_t)i] = co[i];
            cs2[2 * (size_t)i + 1] = s[i];
        }
        for (int i = 0; i < C.n_beams; ++i) {
            bs2[2 * (size_t)i] = sd[i];
            bs2[2 * (size_t)i + 1] = bc[i];
        }
        if (e == hipSuccess) e = hipMemcpy(c->cs2, cs2.data(), cs2.size() * sizeof(double), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(c->bs2, bs2.data(), bs2.size() * sizeof(double), hipMemcpyHostToDevice);
    }
    c->agent_p.assign((size_t)C.n_agents, *params);
    if (e == hipSuccess)
        e = hipMemcpy(c->pa, c->agent_p.data(), c->agent_p.size() * sizeof(f110_params), hipMemcpyHostToDevice);
    if (e == hipSuccess && c->spawn)
        e = hipMemcpy(c->spawn, spawn_poses, (size_t)n_spawn * C.n_agents * 3 * sizeof(double),
                      hipMemcpyHostToDevice);
    // PAD: the clamp-free loop on a table padded by the max range (+ 8 cells of margin), which
    // k_rays_fxs needs (its offsets, kFxsBase); F110_FX_PAD=0 (A/B) never builds it: the context then
    // steps with k_rays_fxn / k_rays_fx.
    const bool fx_ok = c->ray_kernel == 3;
    c->fx_pad = fx_ok;
    if (const char *v = std::getenv("F110_FX_PAD")) c->fx_pad = fx_ok && std::atoi(v) != 0;
    c->fx_refill = fx_ok && c->fx_pad ? refill_waves(EA) : 0;
    const double pad_q = std::ceil(C.max_range / resolution) + 8.0;
    const int32_t fx_pad_cells = pad_q > 0.0 && pad_q < 65536.0 ? (int32_t)pad_q : 0;  // else no padded table
    if (e == hipSuccess)
        e = acquire_map_tables(device, edt_k, H, W, resolution, c->wt, c->tiles_h, fx_ok,
                               c->fx_pad ? fx_pad_cells : 0, &c->maps);
    if (e == hipSuccess) {
        c->dt = c->maps->dt;
        c->dt_tiled = c->maps->dt_tiled;
        if (fx_ok) {
            c->rm = c->maps->rm;
            c->rm_w = c->maps->rm_w;
            c->rm_oob = c->maps->rm_oob;
            c->rm_zero = c->maps->rm_zero;
            if (c->fx_pad) adopt_padded_table(c);
        }
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) return cleanup(F110_E_HIP, std::string("f110_create upload: ") + hipGetErrorString(e));
    *out = c;
    return F110_OK;
}

extern "C" int f110_destroy(f110_ctx *ctx) {
    if (!ctx) return F110_OK;
    (void)hipSetDevice(ctx->device);
    ctx->free_prof();
    for (void *q : ctx->allocs) (void)hipFree(q);
    release_map_tables(ctx->maps);
    delete ctx;
    return F110_OK;
}

static TiledMapView tiled_view(const f110_ctx *c) { return make_tiled_view(map_view(c), c->dt_tiled); }

static StepArgs make_step_args(f110_ctx *c, const f110_outputs *out) {
    StepArgs a{};
    a.map = map_view(c);
    a.tmap = tiled_view(c);
    a.ray_kernel = c->ray_kernel;
    a.ray_wpb = c->ray_wpb;
    for (int i = 0; i < kMaxChunks; ++i) a.chunk_order[i] = c->chunk_order[i];
    a.sines = c->sines;
    a.cosines = c->cosines;
    a.angles = c->angles;
    a.beam_cos = c->beam_cos;
    a.side = c->side;
    a.cs2 = c->cs2;
    a.bs2 = c->bs2;
    a.p = c->p;
    a.E = c->cfg.n_envs;
    a.A = c->cfg.n_agents;
    a.B = c->cfg.n_beams;
    a.theta_dis = c->cfg.theta_dis;
    a.integrator = c->cfg.integrator;
    a.ego = c->cfg.ego_idx;
    a.autoreset = c->cfg.autoreset;
    a.fov = c->cfg.fov;
    a.eps = c->cfg.eps;
    a.max_range = c->cfg.max_range;
    a.dt = c->cfg.time_step;
    a.lidar_dist = c->cfg.lidar_dist;
    a.ttc_thresh = c->cfg.ttc_thresh;
    a.side_max = c->side_max;
    a.noise_std = c->cfg.noise_std;
    a.inc = c->inc;
    a.beam_incr = c->beam_incr;
    a.seed = c->cfg.seed;
    a.env_offset = c->cfg.env_offset;
    a.st = c->st;
    a.sb = c->sb;
    a.scnt = c->scnt;
    a.start = c->start;
    a.start_rot = c->start_rot;
    a.toggles = c->toggles;
    a.near_start = c->near_start;
    a.lap_times = c->lap_times;
    a.lap_counts = c->lap_counts;
    a.sim_time = c->sim_time;
    a.pending = c->pending;
    a.episode = c->episode;
    a.nstep = c->nstep;
    a.ray0 = c->ray0;
    a.runs = c->runs;
    a.nruns = c->nruns;
    a.geo = c->geo;
    a.hmask = (c->hcheck & 2) ? nullptr : c->hmask;  // f110_debug_set_handoff_check bit 1: every chunk stored
    a.hcheck = c->hcheck & 5;
    a.scan = c->scan;
    a.reset_flag = c->reset_flag;
    a.ttc_hit = c->ttc_hit;
    a.noise_step = c->noise_step;
    a.noise_ext = c->noise_ext;
    a.pa = c->pa;
    a.spawn = c->spawn;
    a.n_spawn = c->n_spawn;
    if (out) a.out = *out;
    a.ctr = c->ctr;
    a.ray_nch = c->fx_ilp > 1 ? (c->nch + c->fx_ilp - 1) / c->fx_ilp : c->nch;  // k_rays_fxn: chunk groups
    a.parity = (int32_t)(c->launch_n++ & 1);
    if (c->wcost) {
        a.wcost = c->wcost;
        a.heavy_list = c->heavy_list;
        a.heavy_mask = c->heavy_mask;
        a.heavy_count = c->heavy_count;
        a.heavy_cap = c->heavy_cap;
        a.heavy_T = c->heavy_T;
        a.heavy_on = c->heavy_off ? 0 : 1;
    }
    a.reset_f32 = c->reset_f32 ? 1 : 0;
    a.rm = c->rm;
    a.rm_w = c->rm_w;
    a.rm_oob = c->rm_oob;
    a.rm_zero = c->rm_zero;
    a.rmp = c->rmp;
    a.rmp_w = c->rmp_w;
    a.rmp_P = c->rmp_P;
    a.rmp_zero = c->rmp_zero;
    a.fx_pad = c->rmp ? 1 : 0;
    a.fxs_ok = fxs_ok(c) ? 1 : 0;
    a.count_slots = c->count_slots ? 1 : 0;
    a.fx_refill = c->fx_refill;
    a.fxs_lds = c->fxs_lds ? 1 : 0;
    a.fx_ilp = c->fx_ilp;
    a.gate_wait = c->gate_wait;
    a.gate_record = c->gate_record;
    if (c->wtrace_armed) {  // one traced ray launch
        a.wtrace = c->wtrace;
        c->wtrace_armed = false;
    }
    return a;
}

extern "C" int f110_reset(f110_ctx *ctx, const double *poses, const uint8_t *env_mask, const f110_outputs *out,
                          void *stream) {
    if (!ctx || !poses) return fail(F110_E_INVALID, "f110_reset: null argument");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    if (out && out->obs_stride && out->obs_stride < (int64_t)ctx->cfg.n_beams + 4 * ctx->cfg.n_agents)
        return fail(F110_E_INVALID, "f110_reset: obs_stride < n_beams + 4*n_agents");
    StepArgs a = make_step_args(ctx, out);
    a.mode = 1;
    a.reset_poses = poses;
    a.reset_mask = env_mask;
    HIP_TRY(launch_env_step(a, (hipStream_t)stream, ctx->next_prof_events()));
    return F110_OK;
}

static int step_n(f110_ctx *ctx, const void *actions, int32_t actions_dtype, int32_t n, int64_t step_stride,
                  const f110_outputs *out, void *stream, const char *who) {
    if (!ctx || !actions) return fail(F110_E_INVALID, std::string(who) + ": null argument");
    if (actions_dtype != F110_F32 && actions_dtype != F110_F64)
        return fail(F110_E_INVALID, std::string(who) + ": actions_dtype must be F110_F32 or F110_F64");
    if (n < 1) return fail(F110_E_INVALID, std::string(who) + ": n_steps must be >= 1");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    if (out && out->obs_stride && out->obs_stride < (int64_t)ctx->cfg.n_beams + 4 * ctx->cfg.n_agents)
        return fail(F110_E_INVALID, std::string(who) + ": obs_stride < n_beams + 4*n_agents");
    StepArgs a = make_step_args(ctx, out);
    a.mode = 0;
    a.heavy_build = a.heavy_use = (a.wcost && a.ray_kernel >= 2 && !ctx->heavy_off) ? 1 : 0;  // not on resets
    const int64_t packed = (int64_t)ctx->cfg.n_envs * ctx->cfg.n_agents * 2;  // action elements per step
    if (step_stride != 0 && step_stride < packed)
        return fail(F110_E_INVALID, std::string(who) + ": step_stride < n_envs * n_agents * 2");
    const int64_t stride = step_stride ? step_stride : packed;
    for (int32_t t = 0; t < n; ++t) {
        if (actions_dtype == F110_F64)
            a.actions_f64 = static_cast<const double *>(actions) + (size_t)t * stride;
        else
            a.actions = static_cast<const float *>(actions) + (size_t)t * stride;
        if (t) a.parity = (int32_t)(ctx->launch_n++ & 1);
        HIP_TRY(launch_env_step(a, (hipStream_t)stream, ctx->next_prof_events()));
    }
    return F110_OK;
}

extern "C" int f110_step(f110_ctx *ctx, const void *actions, int32_t actions_dtype, const f110_outputs *out,
                         void *stream) {
    return step_n(ctx, actions, actions_dtype, 1, 0, out, stream, "f110_step");
}

extern "C" int f110_step_n(f110_ctx *ctx, const void *actions, int32_t actions_dtype, int32_t n_steps,
                           int64_t step_stride, const f110_outputs *out, void *stream) {
    return step_n(ctx, actions, actions_dtype, n_steps, step_stride, out, stream, "f110_step_n");
}

extern "C" int f110_set_reset_dtype(f110_ctx *ctx, int32_t dtype) {
    if (!ctx || (dtype != F110_F32 && dtype != F110_F64))
        return fail(F110_E_INVALID, "f110_set_reset_dtype: null context or dtype not F110_F32 / F110_F64");
    ctx->reset_f32 = dtype == F110_F32;
    return F110_OK;
}

extern "C" void f110_host_sincos(const double *x, int64_t n, double *sn, double *cs) {
    for (int64_t i = 0; i < n; ++i) cr_sincos(x[i], sn[i], cs[i]);
}

extern "C" void f110_host_tan_cos_fast(const double *x, int64_t n, double *t, double *c, uint8_t *ok_t,
                                       uint8_t *ok_c) {
    for (int64_t i = 0; i < n; ++i) {
        bool a, b;
        tan_cos_fast(x[i], kSinCosTab, t[i], c[i], a, b);
        ok_t[i] = a ? 1 : 0;
        ok_c[i] = b ? 1 : 0;
    }
}

extern "C" void f110_host_sincos_fast(const double *x, int64_t n, double *sn, double *cs, uint8_t *ok) {
    for (int64_t i = 0; i < n; ++i) ok[i] = cr_sincos_fast(x[i], sn[i], cs[i]) ? 1 : 0;
}

extern "C" void f110_host_sincos_series(const double *x, int64_t n, double *sn, double *cs) {
    for (int64_t i = 0; i < n; ++i) cr_sincos_series(x[i], sn[i], cs[i]);
}

extern "C" void f110_host_np_sincosf(const float *x, int64_t n, int32_t cos_op, float *out) {
    for (int64_t i = 0; i < n; ++i) out[i] = np_sincosf(x[i], cos_op != 0);
}

extern "C" int f110_debug_ray_kernel(const f110_ctx *ctx) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_ray_kernel: null context");
    return ctx->ray_kernel;
}

extern "C" int f110_debug_ray_lanes(const f110_ctx *ctx) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_ray_lanes: null context");
    return ctx->ray_kernel == 3 ? ctx->fx_ilp : 1;
}

// k_rays_fxs's waves per car for unmasked steps, as launch_env_step decides it
extern "C" int f110_debug_ray_refill(const f110_ctx *ctx) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_ray_refill: null context");
    const bool fx = ctx->ray_kernel == 3 && ctx->fx_ilp == 2 && fxs_ok(ctx);
    const int waves = std::min<int>(ctx->fx_refill, (ctx->cfg.n_beams + 63) / 64);  // as the launch clamps it
    return fx && waves > 0 && (ctx->heavy_off || !ctx->wcost) ? waves : 0;
}

// The padded EDT of k_rays_fxn / k_rays_fxs (built on first use, shared with
// the map entry): F110_FX_PAD=0 keeps the clamped table (A/B runs).
static int ensure_padded_table(f110_ctx *ctx) {
    bool pad = true;
    if (const char *v = std::getenv("F110_FX_PAD")) pad = std::atoi(v) != 0;
    if (!pad || ctx->rmp || !ctx->maps) return F110_OK;
    const double pad_q = std::ceil(ctx->cfg.max_range / ctx->res) + 8.0;
    if (pad_q > 0.0 && pad_q < 65536.0) {
        std::lock_guard<std::mutex> g(g_maps_mu);
        MapTables *t = ctx->maps;
        if (!t->rmp) {
            double res;
            std::memcpy(&res, &t->res_bits, 8);
            HIP_TRY(build_padded_table(t, (int32_t)pad_q, host_dt(t->k.data(), t->k.size(), res)));
        }
    }
    if (ctx->maps->rmp) {
        ctx->fx_pad = true;
        adopt_padded_table(ctx);
    }
    return F110_OK;
}

// waves > 0 also turns heavy-first off: k_rays_fxs takes no heavy-first list
extern "C" int f110_debug_set_ray_refill(f110_ctx *ctx, int32_t waves) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_set_ray_refill: null context");
    if (waves < 0 || waves > 16) return fail(F110_E_INVALID, "f110_debug_set_ray_refill: waves must be in 0..16");
    const bool fx = ctx->ray_kernel == 3;
    if (!fx && waves != 0) return fail(F110_E_INVALID, "f110_debug_set_ray_refill: this context's ray kernel has no refill");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    ctx->fx_refill = waves;
    if (waves > 0) {
        ctx->heavy_off = true;
        return ensure_padded_table(ctx);  // the padded table goes with k_rays_fxs
    }
    return F110_OK;
}

extern "C" int f110_debug_disable_heavy_first(f110_ctx *ctx) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_disable_heavy_first: null context");
    ctx->heavy_off = true;
    return F110_OK;
}

extern "C" int f110_debug_set_ray_lanes(f110_ctx *ctx, int32_t n) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_set_ray_lanes: null context");
    if (n < 1 || n > 2) return fail(F110_E_INVALID, "f110_debug_set_ray_lanes: n must be 1 or 2");
    if (ctx->launch_n != 0)
        return fail(F110_E_INVALID, "f110_debug_set_ray_lanes: call before the first reset/step (heavy-first state is per group)");
    const bool fx = ctx->ray_kernel == 3;
    if (!fx && n != 1) return fail(F110_E_INVALID, "f110_debug_set_ray_lanes: this context's ray kernel traces one ray per lane");
    if (fx) ctx->fx_ilp = n;
    return F110_OK;
}

// The product-side form of the three knobs above for a caller that splits one GPU's cars over
// several concurrent contexts (streams.StreamShards): f110_create's size rules applied to the cars
// the device traces at once.
extern "C" int f110_set_device_share(f110_ctx *ctx, int64_t device_cars, int32_t contexts) {
    if (!ctx) return fail(F110_E_INVALID, "f110_set_device_share: null context");
    const int64_t own = (int64_t)ctx->cfg.n_envs * ctx->cfg.n_agents;
    if (contexts < 1 || device_cars < own)
        return fail(F110_E_INVALID, "f110_set_device_share: contexts >= 1 and device_cars >= this context's cars");
    if (ctx->launch_n != 0) return fail(F110_E_INVALID, "f110_set_device_share: call before the first reset/step");
    if (ctx->ray_kernel != 3) {  // one ray per lane, no refill: only the heavy-first rule applies
        if (contexts > 1) ctx->heavy_off = true;
        return F110_OK;
    }
    // k_rays_fxs at every size, its waves per car by the device's cars (refill_waves); without the
    // padded table (F110_FX_PAD=0) the old size rule: 2 rays per lane from 12288 cars
    const int lanes = (ctx->fx_pad || device_cars >= 12288) ? 2 : 1;
    const int refill = (lanes == 2 && ctx->fx_pad) ? refill_waves(device_cars) : 0;
    int rc = f110_debug_set_ray_lanes(ctx, lanes);
    if (rc == F110_OK) rc = f110_debug_set_ray_refill(ctx, refill);
    if (rc == F110_OK && contexts > 1) {
        ctx->heavy_off = true;  // the other contexts fill this one's tail
        // and its 8-wave blocks' idle slots: the LDS theta table pays off beside other contexts
        // (65536 cars in 2 sub-shards 89.5 -> 95.9 M) but not alone (one context 88.3 -> 87.2 M,
        // DESIGN §3.14)
        ctx->fxs_lds = true;
    }
    return rc;
}

extern "C" int f110_debug_set_ray_gate(f110_ctx *ctx, void *wait_event, void *record_event) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_set_ray_gate: null context");
    ctx->gate_wait = static_cast<hipEvent_t>(wait_event);
    ctx->gate_record = static_cast<hipEvent_t>(record_event);
    return F110_OK;
}

extern "C" int f110_get_state(f110_ctx *ctx, double *state, double *steer_buf, int32_t *steer_cnt, void *stream) {
    if (!ctx) return fail(F110_E_INVALID, "f110_get_state: null context");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    const size_t EA = (size_t)ctx->cfg.n_envs * ctx->cfg.n_agents;
    hipStream_t s = (hipStream_t)stream;
    if (state) HIP_TRY(hipMemcpyAsync(state, ctx->st, 7 * EA * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (steer_buf) HIP_TRY(hipMemcpyAsync(steer_buf, ctx->sb, 2 * EA * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (steer_cnt) HIP_TRY(hipMemcpyAsync(steer_cnt, ctx->scnt, EA * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    return F110_OK;
}

extern "C" int f110_get_lap_state(f110_ctx *ctx, double *start_rot, int32_t *toggles, void *stream) {
    if (!ctx) return fail(F110_E_INVALID, "f110_get_lap_state: null context");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    const size_t E = (size_t)ctx->cfg.n_envs, EA = E * ctx->cfg.n_agents;
    hipStream_t s = (hipStream_t)stream;
    if (start_rot) HIP_TRY(hipMemcpyAsync(start_rot, ctx->start_rot, 2 * E * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (toggles) HIP_TRY(hipMemcpyAsync(toggles, ctx->toggles, EA * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    return F110_OK;
}

extern "C" int f110_set_state(f110_ctx *ctx, const double *state, const double *steer_buf, const int32_t *steer_cnt,
                              void *stream) {
    if (!ctx) return fail(F110_E_INVALID, "f110_set_state: null context");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    const size_t EA = (size_t)ctx->cfg.n_envs * ctx->cfg.n_agents;
    hipStream_t s = (hipStream_t)stream;
    if (state) HIP_TRY(hipMemcpyAsync(ctx->st, state, 7 * EA * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (steer_buf) HIP_TRY(hipMemcpyAsync(ctx->sb, steer_buf, 2 * EA * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (steer_cnt) HIP_TRY(hipMemcpyAsync(ctx->scnt, steer_cnt, EA * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    return F110_OK;
}

extern "C" int f110_scan_batch(f110_ctx *ctx, const double *poses, int64_t M, double *scans, int32_t *lookups,
                               int32_t *hit_rc, void *stream) {
    if (!ctx || !poses || !scans || M < 0) return fail(F110_E_INVALID, "f110_scan_batch: bad arguments");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    ScanArgs a{};
    a.map = map_view(ctx);
    a.sines = ctx->sines;
    a.cosines = ctx->cosines;
    a.B = ctx->cfg.n_beams;
    a.theta_dis = ctx->cfg.theta_dis;
    a.fov = ctx->cfg.fov;
    a.eps = ctx->cfg.eps;
    a.max_range = ctx->cfg.max_range;
    a.inc = ctx->inc;
    a.poses = poses;
    a.M = M;
    a.scans = scans;
    a.lookups = lookups;
    a.hit_rc = hit_rc;
    a.ctr = ctx->ctr;
    HIP_TRY(launch_scan_batch(a, (hipStream_t)stream));
    return F110_OK;
}

extern "C" int f110_dynamics_batch(f110_ctx *ctx, const double *x, const double *u, double *f, int64_t M,
                                   void *stream) {
    if (!ctx || !x || !u || !f || M < 0) return fail(F110_E_INVALID, "f110_dynamics_batch: bad arguments");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    HIP_TRY(launch_dynamics_batch(x, u, f, M, ctx->p, (hipStream_t)stream));
    return F110_OK;
}

extern "C" int f110_dynamics_ks_batch(f110_ctx *ctx, const double *x, const double *u, double *f, int64_t M,
                                      void *stream) {
    if (!ctx || !x || !u || !f || M < 0) return fail(F110_E_INVALID, "f110_dynamics_ks_batch: bad arguments");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    HIP_TRY(launch_dynamics_ks_batch(x, u, f, M, ctx->p, (hipStream_t)stream));
    return F110_OK;
}

extern "C" int f110_collision_batch(const double *v1, const double *v2, int64_t M, uint8_t *out, void *stream) {
    if (M < 0 || (M > 0 && (!v1 || !v2 || !out))) return fail(F110_E_INVALID, "f110_collision_batch: bad arguments");
    HIP_TRY(launch_collision_batch(v1, v2, M, out, (hipStream_t)stream));
    return F110_OK;
}

extern "C" int f110_collision_multiple(const double *verts, int64_t M, int32_t N, double *collisions, double *idx,
                                       void *stream) {
    if (M < 0 || N < 1 || N > kMaxMultiBodies || (M > 0 && (!verts || !collisions || !idx)))
        return fail(F110_E_INVALID, "f110_collision_multiple: bad arguments (1 <= N <= 64)");
    HIP_TRY(launch_collision_multiple(verts, M, N, collisions, idx, (hipStream_t)stream));
    return F110_OK;
}

extern "C" int f110_read_counters(f110_ctx *ctx, uint64_t *lookups, uint64_t *rays, void *stream) {
    if (!ctx) return fail(F110_E_INVALID, "f110_read_counters: null context");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    std::vector<unsigned long long> h((size_t)kCtrSlots * kCtrStride);
    HIP_TRY(hipMemcpyAsync(h.data(), ctx->ctr, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    unsigned long long lk = 0, ry = 0;
    for (int i = 0; i < kCtrSlots; ++i) {
        lk += h[(size_t)i * kCtrStride];
        ry += h[(size_t)i * kCtrStride + 1];
    }
    if (lookups) *lookups = lk;
    if (rays) *rays = ry;
    return F110_OK;
}

extern "C" int f110_debug_read_counter(f110_ctx *ctx, int32_t idx, uint64_t *value, void *stream) {
    if (!ctx || !value || idx < 0 || idx >= kCtrStride) return fail(F110_E_INVALID, "f110_debug_read_counter: bad argument");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    std::vector<unsigned long long> h((size_t)kCtrSlots * kCtrStride);
    HIP_TRY(hipMemcpyAsync(h.data(), ctx->ctr, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    unsigned long long v = 0;
    for (int i = 0; i < kCtrSlots; ++i) v += h[(size_t)i * kCtrStride + idx];
    *value = v;
    return F110_OK;
}

extern "C" int f110_debug_set_simt(f110_ctx *ctx, int32_t on) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_set_simt: null context");
    ctx->count_slots = on != 0;
    return F110_OK;
}

extern "C" int f110_debug_set_handoff_check(f110_ctx *ctx, int32_t mode) {
    if (!ctx || mode < 0 || mode > 7) return fail(F110_E_INVALID, "f110_debug_set_handoff_check: bad argument");
    ctx->hcheck = mode;
    return F110_OK;
}

extern "C" int f110_debug_read_simt(f110_ctx *ctx, uint64_t *loop_lookups, uint64_t *lane_slots, void *stream) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_read_simt: null context");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    std::vector<unsigned long long> h((size_t)kCtrSlots * kCtrStride);
    HIP_TRY(hipMemcpyAsync(h.data(), ctx->ctr, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    unsigned long long lk = 0, ry = 0, sl = 0;
    for (int i = 0; i < kCtrSlots; ++i) {
        lk += h[(size_t)i * kCtrStride];
        ry += h[(size_t)i * kCtrStride + 1];
        sl += h[(size_t)i * kCtrStride + 2];
    }
    if (loop_lookups) *loop_lookups = lk - ry;  // the first lookup of every ray is k_agents'
    if (lane_slots) *lane_slots = sl;
    return F110_OK;
}

extern "C" int f110_set_params(f110_ctx *ctx, const f110_params *params, int32_t agent_idx, void *stream) {
    if (!ctx || !params) return fail(F110_E_INVALID, "f110_set_params: null argument");
    if (agent_idx >= ctx->cfg.n_agents)  // Simulator.update_params raises IndexError (base_classes.py:544-546)
        return fail(F110_E_INVALID, "f110_set_params: Index given is out of bounds for list of agents.");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    for (int i = 0; i < ctx->cfg.n_agents; ++i)
        if (agent_idx < 0 || i == agent_idx) ctx->agent_p[(size_t)i] = *params;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemcpyAsync(ctx->pa, ctx->agent_p.data(), ctx->agent_p.size() * sizeof(f110_params),
                           hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));  // agent_p may change again before an async copy would have read it
    return F110_OK;
}

extern "C" int f110_set_scan_noise(f110_ctx *ctx, const double *noise) {
    if (!ctx) return fail(F110_E_INVALID, "f110_set_scan_noise: null context");
    ctx->noise_ext = noise;
    return F110_OK;
}

extern "C" int f110_reset_counters(f110_ctx *ctx, void *stream) {
    if (!ctx) return fail(F110_E_INVALID, "f110_reset_counters: null context");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    HIP_TRY(hipMemsetAsync(ctx->ctr, 0, (size_t)kCtrSlots * kCtrStride * sizeof(unsigned long long),
                           (hipStream_t)stream));
    return F110_OK;
}

extern "C" int f110_profile_begin(f110_ctx *ctx, int32_t max_steps) {
    if (!ctx || max_steps < 0) return fail(F110_E_INVALID, "f110_profile_begin: bad arguments");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    ctx->free_prof();
    ctx->prof_ev.resize((size_t)6 * max_steps);
    for (size_t i = 0; i < ctx->prof_ev.size(); ++i) {
        // the events go with the kernels' own dispatches (hipExtLaunchKernel in launch_env_step):
        // each pair holds that kernel's begin / end timestamps, as rocprofv3's kernel trace does,
        // and no marker packet (nor its cache release) sits between the step's kernels
        hipError_t e = hipEventCreateWithFlags(&ctx->prof_ev[i], hipEventDisableSystemFence);
        if (e != hipSuccess) {
            ctx->prof_ev.resize(i);
            ctx->free_prof();
            return fail(F110_E_HIP, std::string("hipEventCreate: ") + hipGetErrorString(e));
        }
    }
    ctx->prof_max = max_steps;
    ctx->prof_n = 0;
    return F110_OK;
}

extern "C" int f110_debug_profile_stamps(f110_ctx *ctx, void *ref_event, double *out, int32_t max_steps,
                                         int32_t *steps_out) {
    if (!ctx || !ref_event || !out || max_steps < 0)
        return fail(F110_E_INVALID, "f110_debug_profile_stamps: bad arguments");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    const int n = ctx->prof_n < max_steps ? ctx->prof_n : max_steps;
    for (int i = 0; i < n; ++i) {
        hipEvent_t *ev = &ctx->prof_ev[(size_t)6 * i];
        HIP_TRY(hipEventSynchronize(ev[5]));
        for (int k = 0; k < 6; ++k) {
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, static_cast<hipEvent_t>(ref_event), ev[k]));
            out[(size_t)6 * i + k] = ms;
        }
    }
    if (steps_out) *steps_out = n;
    return F110_OK;
}

extern "C" int f110_profile_end(f110_ctx *ctx, double ms_out[3], int32_t *steps_out) {
    if (!ctx) return fail(F110_E_INVALID, "f110_profile_end: null context");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    double acc[3] = {0, 0, 0};
    for (int i = 0; i < ctx->prof_n; ++i) {
        hipEvent_t *ev = &ctx->prof_ev[(size_t)6 * i];
        HIP_TRY(hipEventSynchronize(ev[5]));
        for (int k = 0; k < 3; ++k) {
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
            acc[k] += ms;
        }
    }
    if (ms_out)
        for (int k = 0; k < 3; ++k) ms_out[k] = acc[k];
    if (steps_out) *steps_out = ctx->prof_n;
    ctx->free_prof();
    return F110_OK;
}

extern "C" int f110_debug_wave_trace(f110_ctx *ctx, int32_t arm, uint64_t *host_out, int64_t max_waves,
                                     int64_t *n_waves, void *stream) {
    if (!ctx) return fail(F110_E_INVALID, "f110_debug_wave_trace: null context");
    if (use_device(ctx) != F110_OK) return F110_E_HIP;
    const int64_t EA = (int64_t)ctx->cfg.n_envs * ctx->cfg.n_agents;
    // an upper bound of any ray launch's waves (one-wave blocks: the chunked grids' EA x nch
    // plus the heavy-first prefix; k_rays_fxs: EA x waves per car <= EA x nch, after the multi-agent
    // launch's leading geometry items, ceil(EA (A - 1) / 64) rounded up to 8)
    const int64_t geo_items = ctx->cfg.n_agents > 1 ? ((EA * (ctx->cfg.n_agents - 1) + 63) / 64 + 7) / 8 * 8 : 0;
    const int64_t waves = EA * ((ctx->cfg.n_beams + 63) / 64) + ctx->heavy_cap + 64 + geo_items;
    if (!ctx->wtrace) {
        void *q = nullptr;
        HIP_TRY(hipMalloc(&q, (size_t)waves * 4 * sizeof(uint64_t)));
        HIP_TRY(hipMemset(q, 0, (size_t)waves * 4 * sizeof(uint64_t)));
        ctx->allocs.push_back(q);
        ctx->wtrace = static_cast<uint64_t *>(q);
        ctx->wtrace_n = waves;
    }
    if (n_waves) *n_waves = waves;
    if (host_out) {
        HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
        const int64_t n = max_waves < waves ? max_waves : waves;
        HIP_TRY(hipMemcpy(host_out, ctx->wtrace, (size_t)n * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    if (arm) HIP_TRY(hipMemsetAsync(ctx->wtrace, 0, (size_t)waves * 4 * sizeof(uint64_t), (hipStream_t)stream));
    ctx->wtrace_armed = arm != 0;
    return F110_OK;
}

extern "C" int f110_host_cell_index(int32_t H, int32_t W, double resolution, const double origin[3],
                                    const double *xy, int64_t n, int64_t *lin_out) {
    if (H <= 0 || W <= 0 || !(resolution > 0) || !origin || (n > 0 && (!xy || !lin_out)))
        return fail(F110_E_INVALID, "f110_host_cell_index: bad arguments");
    const MapView m = make_map_view(nullptr, H, W, resolution, origin);
    const TiledMapView t = make_tiled_view(m, nullptr);
    const bool rot = !(t.os == 0.0 && t.oc == 1.0);
    for (int64_t i = 0; i < n; ++i) {
        const double x = xy[2 * i], y = xy[2 * i + 1];
        lin_out[3 * i] = cell_index(m, x, y);
        lin_out[3 * i + 1] = cell_index_fast(m, x, y);
        const int32_t q = rot ? tiled_cell<true>(t, x, y) : tiled_cell<false>(t, x, y);
        const int32_t tile = q >> 4, within = q & 15;  // column-major within the tile (tiled_index)
        const int64_t r = (int64_t)(tile / t.wt) * 4 + (within & 3);
        const int64_t c = (int64_t)(tile % t.wt) * 4 + (within >> 2);
        lin_out[3 * i + 2] = r * W + c;
    }
    return F110_OK;
}

extern "C" int f110_gap_follow(const float *scans, int64_t n_scans, int64_t scan_stride, int32_t n_beams,
                               double angle_min, double angle_increment, float *actions, int64_t action_stride,
                               int32_t *gaps, void *stream) {
    if (n_scans < 0 || n_beams <= 0 || (n_scans > 0 && (!scans || !actions)) || scan_stride < n_beams ||
        action_stride < 2)
        return fail(F110_E_INVALID, "f110_gap_follow: bad arguments");
    if (gap_follow_lds_bytes(n_beams) > 160 * 1024) return fail(F110_E_INVALID, "f110_gap_follow: n_beams too large");
    GapFollowArgs a;
    a.scans = scans;
    a.M = n_scans;
    a.scan_stride = scan_stride;
    a.action_stride = action_stride;
    a.actions = actions;
    a.gaps = gaps;
    a.angle_min = angle_min;
    a.angle_increment = angle_increment;
    a.B = n_beams;
    HIP_TRY(launch_gap_follow(a, (hipStream_t)stream));
    return F110_OK;
}

extern "C" void f110_host_window_ranges(double yaw, double fov, int32_t n_beams, double center, double half,
                                        int32_t ranges_out[4]) {
    int r0a, r0b, r1a, r1b;
    window_beam_ranges(yaw, fov, fov / (double)(n_beams - 1), n_beams, center, half, r0a, r0b, r1a, r1b);
    ranges_out[0] = r0a;
    ranges_out[1] = r0b;
    ranges_out[2] = r1a;
    ranges_out[3] = r1b;
}

// ---- training reward (rewards.py / track_progress.py) -----------------------
struct f110_track {
    int device = 0;
    TrackView v{};
    std::vector<double> s, tan, nrm, mid;
    std::vector<void *> allocs;
};

extern "C" int f110_track_create(f110_track **out, int32_t device, const double *xy, const double *w_right,
                                 const double *w_left, int32_t n, int32_t closed) {
    if (!out || !xy || n < 2 || ((w_right == nullptr) != (w_left == nullptr)))
        return fail(F110_E_INVALID, "f110_track_create: bad arguments (need >= 2 centerline points)");
    const bool host_only = device < 0;  // derived arrays only (f110_track_arrays), no device copy
    if (!host_only && hipSetDevice(device) != hipSuccess)
        return fail(F110_E_NODEVICE, "f110_track_create: no such HIP device");
    auto *t = new f110_track();
    t->device = device;
    // track_progress.py:29-46: seg = diff(xy); seg_len = norm(seg, axis=1) =
    // sqrt(dx*dx + dy*dy); s = [0, cumsum(seg_len)]; tan = seg / max(seg_len,
    // 1e-12); nrm = (-tan_y, tan_x); mid = (xy[:-1] + xy[1:]) * 0.5
    t->s.assign((size_t)n, 0.0);
    t->tan.assign((size_t)2 * (n - 1), 0.0);
    t->nrm.assign((size_t)2 * (n - 1), 0.0);
    t->mid.assign((size_t)2 * (n - 1), 0.0);
    double acc = 0.0;
    for (int32_t i = 0; i + 1 < n; ++i) {
        const double dx = xy[2 * i + 2] - xy[2 * i], dy = xy[2 * i + 3] - xy[2 * i + 1];
        const double len = std::sqrt(dx * dx + dy * dy);
        acc = acc + len;
        t->s[(size_t)i + 1] = acc;
        const double den = len > 1e-12 ? len : 1e-12;
        t->tan[2 * (size_t)i] = dx / den;
        t->tan[2 * (size_t)i + 1] = dy / den;
        t->nrm[2 * (size_t)i] = -t->tan[2 * (size_t)i + 1];
        t->nrm[2 * (size_t)i + 1] = t->tan[2 * (size_t)i];
        t->mid[2 * (size_t)i] = (xy[2 * i] + xy[2 * i + 2]) * 0.5;
        t->mid[2 * (size_t)i + 1] = (xy[2 * i + 1] + xy[2 * i + 3]) * 0.5;
    }
    auto up = [&](const double *src, size_t cnt, const double **dst) -> hipError_t {
        if (host_only) return hipSuccess;
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, cnt * sizeof(double));
        if (e != hipSuccess) return e;
        t->allocs.push_back(q);
        *dst = static_cast<const double *>(q);
        return hipMemcpy(q, src, cnt * sizeof(double), hipMemcpyHostToDevice);
    };
    // uniform grid over the segment midpoints (reward kernel's kd.query):
    // cells of 16 median segment lengths (a 3x3 block then holds ~50
    // midpoints of a centerline through it; the kernel widens the block when
    // the 5th nearest is not provably inside), one cell of margin on every side
    std::vector<int32_t> cstart, citems;
    std::vector<double> cmid;
    if (!host_only && n >= 2) {
        double mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
        for (int32_t i = 0; i + 1 < n; ++i) {
            mnx = std::min(mnx, t->mid[2 * (size_t)i]);
            mxx = std::max(mxx, t->mid[2 * (size_t)i]);
            mny = std::min(mny, t->mid[2 * (size_t)i + 1]);
            mxy = std::max(mxy, t->mid[2 * (size_t)i + 1]);
        }
        std::vector<double> seg;
        for (int32_t i = 0; i + 1 < n; ++i)
            seg.push_back(std::hypot(xy[2 * (size_t)i + 2] - xy[2 * (size_t)i], xy[2 * (size_t)i + 3] - xy[2 * (size_t)i + 1]));
        std::nth_element(seg.begin(), seg.begin() + seg.size() / 2, seg.end());
        const double med = seg[seg.size() / 2];
        const double ext = std::max(mxx - mnx, mxy - mny);
        // at most 4096 cells a side; a degenerate spacing falls back to ext / 64
        const double h = std::max(std::isfinite(med) && med > 0.0 ? 16.0 * med : ext / 64.0, ext / 4000.0);
        if (h > 0.0 && std::isfinite(h) && std::isfinite(mnx) && std::isfinite(mny) && std::isfinite(mxx) && std::isfinite(mxy) &&
            (mxx - mnx) / h < 4096 && (mxy - mny) / h < 4096) {
            t->v.gh = h;
            t->v.gx0 = mnx - h;
            t->v.gy0 = mny - h;
            t->v.gnx = (int32_t)((mxx - t->v.gx0) / h) + 2;
            t->v.gny = (int32_t)((mxy - t->v.gy0) / h) + 2;
            const size_t nc = (size_t)t->v.gnx * t->v.gny;
            std::vector<int32_t> cell((size_t)n - 1);
            cstart.assign(nc + 1, 0);
            for (int32_t i = 0; i + 1 < n; ++i) {
                const int32_t ci = (int32_t)((t->mid[2 * (size_t)i] - t->v.gx0) / h);
                const int32_t cj = (int32_t)((t->mid[2 * (size_t)i + 1] - t->v.gy0) / h);
                cell[(size_t)i] = cj * t->v.gnx + ci;
                ++cstart[(size_t)cell[(size_t)i] + 1];
            }
            for (size_t c = 0; c < nc; ++c) cstart[c + 1] += cstart[c];
            citems.assign((size_t)n - 1, 0);
            std::vector<int32_t> fill(cstart.begin(), cstart.end() - 1);
            for (int32_t i = 0; i + 1 < n; ++i) citems[(size_t)fill[(size_t)cell[(size_t)i]]++] = i;
            cmid.resize(2 * citems.size());
            for (size_t q = 0; q < citems.size(); ++q) {
                cmid[2 * q] = t->mid[2 * (size_t)citems[q]];
                cmid[2 * q + 1] = t->mid[2 * (size_t)citems[q] + 1];
            }
        }
    }
    auto up_i = [&](const std::vector<int32_t> &src, const int32_t **dst) -> hipError_t {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, src.size() * sizeof(int32_t));
        if (e != hipSuccess) return e;
        t->allocs.push_back(q);
        *dst = static_cast<const int32_t *>(q);
        return hipMemcpy(q, src.data(), src.size() * sizeof(int32_t), hipMemcpyHostToDevice);
    };
    hipError_t e = up(xy, 2 * (size_t)n, &t->v.xy);
    if (e == hipSuccess && !cstart.empty()) e = up_i(cstart, &t->v.cell_start);
    if (e == hipSuccess && !citems.empty()) e = up_i(citems, &t->v.cell_items);
    if (e == hipSuccess && !cmid.empty()) e = up(cmid.data(), cmid.size(), &t->v.cell_mid);
    if (e == hipSuccess) e = up(t->s.data(), t->s.size(), &t->v.s);
    if (e == hipSuccess) e = up(t->tan.data(), t->tan.size(), &t->v.tan);
    if (e == hipSuccess) e = up(t->nrm.data(), t->nrm.size(), &t->v.nrm);
    if (e == hipSuccess) e = up(t->mid.data(), t->mid.size(), &t->v.mid);
    if (e == hipSuccess && w_right) e = up(w_right, (size_t)n, &t->v.wR);
    if (e == hipSuccess && w_left) e = up(w_left, (size_t)n, &t->v.wL);
    if (e != hipSuccess) {
        for (void *q : t->allocs) (void)hipFree(q);
        delete t;
        return fail(F110_E_HIP, std::string("f110_track_create: ") + hipGetErrorString(e));
    }
    t->v.n = n;
    t->v.closed = closed ? 1 : 0;
    t->v.L = t->s[(size_t)n - 1];
    *out = t;
    return F110_OK;
}

extern "C" int f110_track_destroy(f110_track *t) {
    if (!t) return F110_OK;
    if (!t->allocs.empty()) (void)hipSetDevice(t->device);
    for (void *q : t->allocs) (void)hipFree(q);
    delete t;
    return F110_OK;
}

extern "C" double f110_track_arrays(const f110_track *t, double *s, double *tan, double *nrm, double *mid) {
    if (!t) return 0.0;
    if (s) std::copy(t->s.begin(), t->s.end(), s);
    if (tan) std::copy(t->tan.begin(), t->tan.end(), tan);
    if (nrm) std::copy(t->nrm.begin(), t->nrm.end(), nrm);
    if (mid) std::copy(t->mid.begin(), t->mid.end(), mid);
    return t->v.L;
}

extern "C" void f110_default_reward_params(f110_reward_params *p) {
    if (!p) return;
    *p = f110_reward_params{};
    // CenterlineSafetyProgressReward.__init__ defaults (rewards.py:196-230)
    p->dt = 0.01;
    p->w_prog = 1.2;
    p->forward_sign = 1.0;
    p->alive_bonus = 0.02;
    p->w_rel_lead = 0.0;
    p->lead_clip = 5.0;
    p->w_lat = 0.35;
    p->lat_cap = 4.0;
    p->default_half_width = 1.5;
    p->lidar_max = 1.0;  // LIDAR_MAX (rewards.py:7)
    p->near_wall_dist = 0.35 / 30.0;
    p->w_wall = 1.0;
    p->wall_quantile = 0.05;
    p->opp_safe_dist = 0.7;
    p->w_opp = 0.8;
    p->ego_crash_penalty = 50.0;
    p->opp_crash_bonus = 50.0;
    p->beta = 0.8;
    p->grace_steps_wall = 25;
    p->grace_steps_opp = 25;
    p->auto_flip_steps = 20;
    p->use_progress = 1;
}

extern "C" int f110_reward(const f110_track *track, const f110_reward_params *params, const float *obs,
                           int64_t n_envs, int32_t obs_len, int32_t n_beams, f110_reward_state *state,
                           const uint8_t *reset_mask, double *rewards, void *stream) {
    if (!params || n_envs < 0 || (n_envs > 0 && (!obs || !state || !rewards)) || n_beams < 0 || n_beams > 2048 ||
        obs_len < n_beams + 8)
        return fail(F110_E_INVALID, "f110_reward: bad arguments (obs rows need n_beams + 8 entries, n_beams <= 2048)");
    if (params->use_progress && (!track || !track->v.mid))
        return fail(F110_E_INVALID, "f110_reward: use_progress needs a device track");
    RewardArgs a{};
    if (track) a.track = track->v;
    a.p = *params;
    a.obs = obs;
    a.E = n_envs;
    a.obs_len = obs_len;
    a.B = n_beams;
    a.state = state;
    a.reset_mask = reset_mask;
    a.rewards = rewards;
    HIP_TRY(launch_reward(a, (hipStream_t)stream));
    return F110_OK;
}
