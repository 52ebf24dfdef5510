// f110_internal.h — context layout and kernel launchers shared by
// f110_kernels.hip (device) and f110_capi.cpp (host API).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "f110_device.h"

namespace f110 {

// Lookup/ray counters are spread over kCtrSlots 128-B lines: ~10^5 waves
// adding into ONE address serialise at the memory side (measured: 2.7 ms of
// a 3.4 ms scan at 8192 envs); 256 slots make the adds contention-free.
constexpr int kCtrSlots = 256;
constexpr int kCtrStride = 16;  // u64 per slot (128 B)
constexpr int kRayBlock = 256; // threads per block of the ray kernels
constexpr int kMaxMultiBodies = 64;  // f110_collision_multiple: bodies per set
constexpr int kMaxChunks = 32;  // 64-beam chunks per scan (n_beams <= 2048) for the chunked ray dispatch

// Everything one env step (k_agents, a ray kernel, a post kernel) needs, passed by value.
struct PairGeom;  // below

struct StepArgs {
    MapView map;
    TiledMapView tmap;
    const double *sines, *cosines;            // [theta_dis]  ScanSimulator2D tables
    const double *angles, *beam_cos, *side;   // [B] RaceCar class-level beam tables
    const double *cs2, *bs2;  // k_rays_fxs: (cos, sin)[theta_dis], (side, beam_cos)[B] interleaved
    f110_params p;                            // Simulator / F110Env params (GJK boxes, lidar_max)
    const f110_params *pa;                    // [A] RaceCar params (update_pose, ray_cast boxes)
    int32_t E, A, B, theta_dis, integrator, ego, autoreset, mode;  // mode 0 step, 1 reset
    int32_t reset_f32;        // resets follow F110Env.reset(options=float32 poses) (f110_set_reset_dtype)
    int32_t ray_wpb;          // chunked ray kernel: waves (cars) per block (1)
    int32_t ray_kernel;       // 1: k_rays_tiled, flat ray order; 2: chunked; 3: the fixed-point kernels
                              // (k_rays_fx / k_rays_fxn / k_rays_fxs: fixed-point cell index, scalar per-car set-up)
    uint8_t chunk_order[kMaxChunks];  // beam-chunk dispatch order of the chunked ray kernel
    uint64_t *wtrace;         // diagnostic wave trace of the next ray launch (f110_debug_wave_trace) or null
    hipEvent_t gate_wait;     // f110_debug_set_ray_gate: waited on before the ray launch, or null
    hipEvent_t gate_record;   // f110_debug_set_ray_gate: recorded after the ray launch, or null
    // heavy-first ray dispatch (chunked kernel): per (car, chunk) wave cost of
    // the previous ray launch, this step's list of predicted-heavy waves
    uint8_t *wcost;           // [EA][nch] min(255, longest ray of the wave) or null
    uint32_t *heavy_list;     // [2][heavy_cap] (car << 8 | chunk), by step parity
    uint32_t *heavy_mask;     // [EA] chunks of the car that are in the heavy list
    uint32_t *heavy_count;    // [2] list lengths, by step parity
    int32_t heavy_cap, heavy_T, heavy_build, heavy_use, parity, ray_nch;
    int32_t heavy_on;         // heavy-first enabled for this context (wcost is written for the next step)
    // k_rays_fx / k_rays_fxn's row-major EDT: rows of rm_w cells (128-B
    // aligned), columns W..rm_w-1 and row H hold dt[-1,-1], a 0.0 at byte
    // rm_zero past the end; rm_oob = byte offset of dt[H-1][W-1]
    const double *rm;
    int32_t rm_w;
    uint32_t rm_oob, rm_zero;
    // k_rays_fxn's padded row-major EDT (PAD): rows of rmp_w cells, rmp_P
    // cells of dt[-1,-1] on every side (cell (r, c) at row r + P, column
    // c + P), a 0.0 at byte rmp_zero past the end; null = not built
    const double *rmp;
    int32_t rmp_w, rmp_P;
    uint32_t rmp_zero;
    int32_t fx_pad;     // the padded table is built (k_rays_fxn on it unless F110_FX_PAD=0; k_rays_fxs)
    int32_t fxs_ok;     // the padded table's rows and columns are below 2^20 (kFxsBase's offsets)
    int32_t fx_refill;  // waves per car of k_rays_fxs (two chunk slots with refill; 0 = off)
    int32_t fxs_lds;    // single-agent k_rays_fxs in 8-wave blocks with the theta table in LDS (shared device)
    uint32_t *hmask;    // [E*A] k_agents' hand-off chunk masks (A >= 2 dividing 64), or null
    PairGeom *geo;      // [E][A][A-1] pair geometry (A >= 2), see RayArgs::geo
    int32_t geo_ready;  // set by launch_env_step: this step's ray kernel computed geo
    int32_t count_slots;  // f110_debug_set_simt: lane-slot counter of the fixed-point loops
    int32_t hcheck;       // f110_debug_set_handoff_check bit 0: the hand-off buffer is NaN-poisoned before the
                          // ray launch and k_post_multi counts its reads outside hmask (ctr[.][6]); bit 2:
                          // k_agents stores empty masks (a forced miss, the check's own test)
    int32_t fx_ilp;     // rays per lane of the fixed-point ray kernel (1: k_rays_fx, 2: k_rays_fxn / k_rays_fxs)
    double fov, eps, max_range, dt, lidar_dist, ttc_thresh, noise_std, inc, beam_incr;
    double side_max;  // max of the RaceCar side table (the TTC pre-test of k_rays_fxs)
    uint64_t seed;
    int64_t env_offset;
    // persistent per-agent / per-env state (SoA, owned by the context)
    double *st;          // [7][E*A]
    double *sb;          // [2][E*A] steer buffer (newest, older)
    int32_t *scnt;       // [E*A]
    double *start;       // [3][E*A] reset poses (lap logic)
    double *start_rot;   // [2][E] cos(-th), sin(-th) of the ego's reset yaw
    int32_t *toggles;    // [E*A]
    uint8_t *near_start; // [E*A]
    float *lap_times;    // [E*A]
    float *lap_counts;   // [E*A]
    double *sim_time;    // [E]
    uint8_t *pending;    // [E] autoreset pending
    uint64_t *episode;   // [E]
    uint64_t *nstep;     // [E] steps since reset (noise counter)
    // k_agents -> k_rays -> k_post hand-off buffers (context scratch)
    double *ray0;        // [3][E*A] scan pose x, y and first EDT lookup d0
    BeamRun *runs;       // [E*A][kMaxSeg] beam-index runs
    int32_t *nruns;      // [E*A]
    double *scan;        // [E*A][B] ranges (noise added) before the collision stage
    uint8_t *reset_flag; // [E] this call reset the env
    uint8_t *ttc_hit;    // [E*A] TTC fired in the fused single-agent ray pass
    uint64_t *noise_step;// [E] noise counter used by this step
    const double *noise_ext;  // [E][B] caller-supplied scan noise (f110_set_scan_noise) or null
    const double *spawn; // [n_spawn][A][3]
    int32_t n_spawn;
    // inputs
    const float *actions;       // [E][A][2] f32, or
    const double *actions_f64;  // [E][A][2] f64
    const double *reset_poses;  // [E][A][3]
    const uint8_t *reset_mask;  // [E] or null
    f110_outputs out;
    unsigned long long *ctr;    // [kCtrSlots][16]: [0] lookups, [1] rays (see count_rays), [2] lane slots of the fixed-point loops
};

// RN(1 / lidar_max) in f32 for k_rays_fxs's obs division, or 0 (the IEEE
// divide) outside [2^-30, 2^30], where an intermediate could be subnormal
inline float obs_reciprocal(float lmax) {
    if (!(lmax >= 0x1p-30f && lmax <= 0x1p30f)) return 0.0f;
    volatile float l = lmax;  // one IEEE f32 divide (not folded into a double one)
    return 1.0f / l;
}

// k_rays_tiled's own argument block: only what the ray loop and its epilogue
// read (the full StepArgs kept 90 SGPRs live: 7 instead of 8 blocks per CU).
// One (car, opponent) pair's agent ray_cast geometry (RaceCar.ray_cast_agents,
// base_classes.py:206-227; laser_models.py:282-346): the opponent's box as the
// car sees it (get_vertices with the car's params), the box's beam window at
// the scan origin and the beam-index ranges of the blocked view the window can
// hold.  Computed by the ray kernel's leading geometry blocks (k_rays_fxs with
// other cars in the env) from the post-update, pre-TTC poses; k_post_multi
// recomputes the pairs whose car's TTC fired (its yaw is zeroed).
struct PairGeom {
    double rv[8];
    double phi[4];  // vertex bearings (box_beam_window's input)
    double wc, wh;
    int32_t rng[4];
};

struct RayArgs {
    TiledMapView m;
    const double *sines, *cosines;
    const double *ray0;        // [3][EA]
    const BeamRun *runs;       // [EA][kMaxSeg]
    const int32_t *nruns;      // [EA]
    const uint8_t *reset_mask; // [E]: f110_reset with an env mask, else null
    double *scan;              // [EA][B]
    const double *noise_ext;   // [E][B] or null
    const uint64_t *noise_step;// [E]
    unsigned long long *ctr;
    double eps, max_range, noise_std;
    uint64_t seed;
    int64_t env_offset;
    int32_t EA, A, B, theta_dis;
    // FUSED single-agent epilogue (k_rays_tiled<.., .., true>)
    const double *vel;         // state[3][EA]
    const double *beam_cos, *side;
    double ttc_thresh;
    double side_max;           // max_b side[b]: a range above side_max + 1.2 thresh |v| cannot fire TTC
    uint8_t *ttc_hit;          // [EA]
    float *obs;                // [E][obs_len] or null
    float *scans_f32;          // [EA][B] or null
    double *scans_f64;         // [EA][B] or null
    int32_t obs_len;
    float lidar_max;
    float obs_rinv;            // RN(1 / lidar_max) for k_rays_fxs's obs division (0: IEEE divide)
    // chunked dispatch (k_rays_tiled<.., CH = true>)
    int32_t G4;                // blocks per chunk slot (4 cars per block)
    uint8_t order[kMaxChunks]; // chunk of each slot
    uint64_t *wtrace;          // diagnostic wave trace [waves][4] or null
    // heavy-first dispatch: HB leading blocks run the listed heavy waves
    uint8_t *wcost;            // [EA][nch] written by every chunked launch (or null)
    const uint32_t *heavy_list;
    const uint32_t *heavy_mask;
    const uint32_t *heavy_count;
    int32_t HB, nch;
    int32_t wpb;  // chunked: waves (cars) per block
    // fixed-point cell index of k_rays_fx (see fx_cell in f110_kernels.hip):
    // t = fma(x, inv_res, fx_cx) = 1.5*2^22 + column, on a 2^-30 grid
    double fx_cx, fx_cy;
    // |q| bound of a scan origin whose rays stay in t's binade: 2^21 - 32 - max_range / res
    double fx_lim;
    uint32_t fx_zero;  // byte offset of the row-major table's zero cell (k_rays_fxn)
    // PAD (k_rays_fxn on the padded table): fx_cx / fx_cy = 2^24 + P - origin /
    // res, and a car takes the clamp-free loop when its scan origin's q lies in
    // [fxp_lo, fxp_hx) x [fxp_lo, fxp_hy): every lookup of its rays then lands
    // inside the padded table (see fxp_offset)
    double fxp_lo, fxp_hx, fxp_hy;
    int32_t fxp_P;
    double fxs_cx, fxs_cy;  // k_rays_fxs: 2^20 + P + 2^-26 - origin / res (see kFxsBase)
    int32_t count_slots;  // the fixed-point loops add their lane slots to ctr[.][2] (f110_debug_read_simt)
    const double *cs2, *bs2;  // k_rays_fxs: interleaved (cos, sin) / (side, beam_cos) tables
    // k_rays_fxs<HANDOFF>: geo_blocks leading work items (one wave each) compute every pair's PairGeom
    const uint32_t *hmask;     // [EA] the chunks whose hand-off k_post_multi may read (k_agents), or null: all
    PairGeom *geo;
    int32_t geo_blocks;
    const double *st;          // state [7][EA] after k_agents
    const f110_params *pa;     // [A] per-agent params (RaceCar.params)
    double fov, beam_incr;
};

// k_rays_fx's magic offset: 1.5 * 2^22.  t = M + q for q in [0, 2^21) lies in
// the binade [2^22, 2^23), whose ulp is 2^-30, so the low 30 mantissa bits of
// t hold q's fraction and the next 21 its integer part.
constexpr double kFxMagic = 6291456.0;
// bits [61:30] of M: exponent[9:0] (0x015), mantissa bit 51, 21 zero bits
constexpr uint32_t kFxU0 = 0x05600000u;
// guard band of the fixed-point fraction, in units of 2^-30 (error budget < 2^-29)
constexpr uint32_t kFxBand = 4u;
// PAD: t = fma(x, inv_res, 2^24 + P - origin / res) lies in [2^24, 2^25),
// ulp 2^-28.  Bits [51:28] of t (one v_alignbit by 28) hold int(t) - 2^24 =
// floor(q) + P in their low 24 bits -- exactly the operand a 24-bit multiply
// reads, so the padded table's byte offset is two u24 multiply(-add)s with no
// bias subtraction and no clamp.  Error budget (units of q): the constant's
// and t's roundings (2^-29 each), inv_res's (< 2^-31 for |x / res| < 2^21)
// and the reference's own (< 2^-31): < 2^-27.4; the guard band is kFxpBand *
// 2^-28 = 2^-26.
constexpr double kFxpBase = 16777216.0;
constexpr uint32_t kFxpBand = 4u;
// k_rays_fxs: t = fma(x, inv_res, 2^20 + P + 2^-26 - origin / res) lies in
// [2^20, 2^21), ulp 2^-32: t's low dword is the fraction of q + P + 2^-26 and
// its high dword's low 24 bits are 3 * 2^20 (the exponent's low bits) +
// floor(q + P + 2^-26) -- the u24 multiplies read the high dwords as they are
// (no v_alignbit).  The 3 * 2^20 terms add 3 * 2^20 * (k1 + 8) to the byte
// offset, which vanishes mod 2^32 because the padded table's row stride k1 is
// 8 bytes short of a multiple of 4096 (build_padded_table).  The +2^-26 shift
// makes the guard band one compare: a lane is near a cell edge when the low
// dword is below 2 * kFxsBand (= 2^-25, a band of 2^-26 on either side of the
// edge, as kFxpBand); such lanes take the IEEE cell, so the shifted integer
// part of the others is floor(q + P).  Error budget (units of q): t's and the
// constant's roundings (2^-33 each) and those of kFxpBase's analysis: < 2^-27.4.
constexpr double kFxsBase = 1048576.0;
constexpr double kFxsShift = 0x1p-26;
constexpr uint32_t kFxsBand = 64u;  // 2^-26 in units of 2^-32
constexpr int kFxsWaves = 8;         // k_rays_fxs: work items (one wave each) per block, sharing one LDS theta table
constexpr int kFxsLdsTheta = 2048;   // theta table entries the block's LDS copy holds (32 KB; theta_dis 2000)

struct ScanArgs {
    MapView map;
    const double *sines, *cosines;
    int32_t B, theta_dis;
    double fov, eps, max_range, inc;
    const double *poses;  // [M][3]
    int64_t M;
    double *scans;        // [M][B]
    int32_t *lookups;     // [M][B] or null
    int32_t *hit_rc;      // [M][B][2] or null
    unsigned long long *ctr;
};

// gap_follow_action over M float32 scans (f110_gap_follow).
struct GapFollowArgs {
    const float *scans;   // scan m at scans + m * scan_stride
    int64_t M, scan_stride, action_stride;
    float *actions;       // (steer, speed) of scan m at actions + m * action_stride
    int32_t *gaps;        // [M][2] chosen (start, end) or null
    double angle_min, angle_increment;
    int32_t B;
};

// CenterlineProgress arrays on the device (f110_track).
struct TrackView {
    const double *xy;   // [n][2]
    const double *s;    // [n] arclength
    const double *tan;  // [n-1][2]
    const double *nrm;  // [n-1][2]
    const double *mid;  // [n-1][2] segment midpoints
    const double *wR, *wL;  // [n] lane widths or null
    int32_t n, closed;
    double L;
    // uniform grid over the midpoints (kd.query acceleration): cell (i, j) of
    // size gh at (gx0 + i*gh, gy0 + j*gh) holds midpoints cell_items[cell_start[c] ..
    // cell_start[c+1]), c = j*gnx + i
    const int32_t *cell_start, *cell_items;
    const double *cell_mid;  // [n-1][2]: mid[cell_items[q]], in cell order (no indirection)
    int32_t gnx, gny;
    double gx0, gy0, gh;
};

struct RewardArgs {
    TrackView track;
    f110_reward_params p;
    const float *obs;
    int64_t E;
    int32_t obs_len, B;
    f110_reward_state *state;
    const uint8_t *reset_mask;
    double *rewards;
};

// ---- prioritized replay (f110_replay.hip) ---------------------------------
constexpr int kTieCap = 4096;        // keys equal to the selection threshold kept for the tie break
constexpr int kReplayMaxGrid = 1024; // blocks of the streaming replay kernels
constexpr int kReplayMaxBatch = 8192;
// Copies of the radix select's global histograms: block b adds into copy b % kHistRep (consecutive
// blocks land on different XCDs), so each bin's device-scope atomics are spread over 8 addresses;
// the consumer sums the copies.  Layout hist[(copy * 4 + pass) * 256 + bin].
constexpr int kHistRep = 8;

// Device header of a replay buffer (one per f110_replay).
struct ReplayHdr {
    int64_t length;     // PrioritizedExperienceReplayBuffer._length
    int64_t next;       // _next_idx
    uint64_t draws;     // sample() calls so far (Philox counter)
    double den;         // sum of (p + eps)^alpha at the last sample
    int32_t replace;    // the last sample drew with replacement
    int32_t pad0_;
    uint32_t prefix;    // radix select: threshold key so far
    uint32_t kleft;     //   rank still to select below/at the prefix
    uint32_t n_lt, n_tie;  // keys below / equal to the threshold (n_tie zeroed by k_finish)
    uint32_t overflow;  // samples whose tie list overflowed kTieCap
    uint32_t pad_;
    uint32_t sel_prefix[4], sel_kleft[4];  // the select through digit q (written by the kernel after
                                           // pass q's histogram, read by the next one)
};

struct ReplayView {
    ReplayHdr *hdr;
    int64_t capacity;
    int32_t obs_dim, act_dim;
    float *obs, *next_obs, *act, *reward, *done, *prio;  // [cap][D], [cap][D], [cap][A], [cap] x3
    double *wt;          // [cap] sampling weight (prio + eps)^alpha, written with prio (add, update)
    uint32_t *keys;      // [cap] exponential-race keys
    uint32_t *hist;      // [4][256]
    double *den_part;    // [kReplayMaxGrid]
    uint32_t *part;      // [kReplayMaxGrid] per-block max priority (add) / selected count (sample)
    uint64_t *sel;       // [kReplayMaxBatch] indices of the keys below the threshold, in index order
    uint32_t *tie;       // [kTieCap]
    int64_t *pos;        // [max rows per add] ring slot of each added row (-1: not stored)
    double alpha;
    float eps;           // the buffer's priority_epsilon (replay_buffer.py:24, 88)
    uint64_t seed;
};

struct ReplayRows {      // one add(): n transitions (device, f32 rows with strides in floats)
    const float *obs, *next_obs, *act, *reward;
    const double *reward64; // [n] f64 rewards instead of reward (rounded to f32 as .to(torch.float32))
    const float *priority;  // [n] explicit priorities or null (= the max priority)
    const uint8_t *done;
    int64_t obs_stride, next_stride, act_stride;
    int32_t vec4;        // rows 16-B aligned and obs_dim % 4 == 0
};

struct ReplayBatch {     // one sample(): the gathered batch (device, contiguous)
    float *obs, *next_obs, *act, *reward, *done;
    int32_t vec4;
};

hipError_t launch_replay_add_index(const ReplayView &v, const uint8_t *mask, int mask_skip, const float *priority,
                                   int64_t n, hipStream_t s);  // ring slots, priorities, header
hipError_t launch_replay_add_copy(const ReplayView &v, const ReplayRows &in, int64_t n, hipStream_t s);  // the rows
hipError_t launch_replay_select(const ReplayView &v, int32_t batch, double beta, int64_t *idx, float *w,
                                bool known_full, hipStream_t s);  // idx / weights (reads no row data)
hipError_t launch_replay_gather(const ReplayView &v, int32_t batch, const int64_t *idx, const ReplayBatch &out,
                                hipStream_t s);
hipError_t launch_replay_update(const ReplayView &v, const int64_t *idx, const float *val, int64_t n, float add_eps,
                                int32_t from_td, int32_t serial, hipStream_t s);
hipError_t prepare_replay(int32_t max_batch);
int replay_grid(int64_t capacity);

// ---- flat Adam (f110_adam.hip) --------------------------------------------
struct AdamArgs {
    float *param, *exp_avg, *exp_avg_sq;
    const float *grad;
    int64_t n;
    double lr, beta1, beta2, eps;
    int64_t *step;     // device step counter
    uint32_t *done;    // device: blocks finished (last one advances step)
    float *target;     // the target network's flat buffer (soft update after the step) or null
    float tau;
};
hipError_t launch_adam(const AdamArgs &a, hipStream_t s);

hipError_t launch_env_step(const StepArgs &a, hipStream_t s, hipEvent_t *ev = nullptr);  // ev: 6 events or null
hipError_t launch_scan_batch(const ScanArgs &a, hipStream_t s);
hipError_t launch_gap_follow(const GapFollowArgs &a, hipStream_t s);
hipError_t launch_reward(const RewardArgs &a, hipStream_t s);
size_t gap_follow_lds_bytes(int B);
hipError_t launch_dynamics_ks_batch(const double *x, const double *u, double *f, int64_t M, const f110_params &p,
                                    hipStream_t s);
hipError_t launch_collision_batch(const double *v1, const double *v2, int64_t M, uint8_t *out, hipStream_t s);
hipError_t launch_collision_multiple(const double *verts, int64_t M, int32_t N, double *collisions, double *idx,
                                     hipStream_t s);
hipError_t launch_dynamics_batch(const double *x, const double *u, double *f, int64_t M, const f110_params &p,
                                 hipStream_t s);

}  // namespace f110
