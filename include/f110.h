/*
 * f110.h — C ABI of libf110.so, the MI355X (gfx950) batched F1TENTH step.
 *
 * This is the drop-in boundary for the per-step hot path of f110_gym
 * (ahoop004/f110_gymnasium_ros2_jazzy, paths below are relative to
 * f110_gymnasium/gym/f110_gym/envs/).  The reference has no FFI: its hot path
 * is a set of Numba @njit functions driven by the Python classes RaceCar /
 * Simulator / F110Env.  Each entry point below names the reference interface
 * it replaces.  INTEGRATION.md shows the ctypes binding the reference side
 * would add.
 *
 * Conventions
 *  - Plain C types only.  Every array argument of f110_reset / f110_step /
 *    f110_*_batch is a DEVICE pointer owned by the caller (e.g. a
 *    torch.Tensor's data_ptr()).  f110_edt_k and f110_create take HOST
 *    pointers (cold path, once per map).
 *  - Work is enqueued asynchronously on the hipStream_t passed as `stream`
 *    (NULL = the default stream).  No call below synchronises the device or
 *    allocates memory after f110_create.
 *  - Return value: 0 on success, a negative F110_E* code on error;
 *    f110_last_error() describes the last error of the calling thread.
 *  - One context = one device, one map, one batch of n_envs x n_agents cars.
 *    A context is not thread-safe; use one per host thread.  (The reference
 *    shares a class-level ScanSimulator2D across every env in the process,
 *    base_classes.py:64-67,118-120; contexts share nothing.)
 *  - Layouts: agent index g = env * n_agents + agent.  State is kept on the
 *    device as structure-of-arrays fp64: state[k * n_envs*n_agents + g],
 *    k = 0..6 = [x, y, steer, v, yaw, yaw_rate, slip] (base_classes.py:97).
 */
#ifndef F110_H
#define F110_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define F110_API __attribute__((visibility("default")))
#else
#define F110_API
#endif

#define F110_ABI_VERSION 3  /* 2: f110_outputs.obs_stride; 3: f110_adam_step target / tau, head dh_mask,
                                 f110_debug_* names (include/f110_debug.h), f110_set_device_share */

#define F110_OK 0
#define F110_E_INVALID (-1)  /* bad argument / shape */
#define F110_E_HIP (-2)      /* HIP runtime error */
#define F110_E_NOMAP (-3)    /* ScanSimulator2D.scan without a map (laser_models.py:445-446) */
#define F110_E_NODEVICE (-4) /* no gfx950 device */
#define F110_E_ALLOC (-5)

#define F110_F32 0  /* action dtypes for f110_step */
#define F110_F64 1

#define F110_INTEGRATOR_RK4 1   /* base_classes.py:40-42 */
#define F110_INTEGRATOR_EULER 2

/* Vehicle parameters: F110Env default params dict (f110_env.py:132-156). */
typedef struct f110_params {
    double mu, C_Sf, C_Sr, lf, lr, h, m, I;
    double s_min, s_max, sv_min, sv_max, v_switch, a_max, v_min, v_max;
    double width, length, lidar_max;
} f110_params;

/* Simulator / sensor configuration (F110Env.__init__ kwargs f110_env.py:104-186,
 * RaceCar.__init__ base_classes.py:69-115, ScanSimulator2D.__init__
 * laser_models.py:360-381). */
typedef struct f110_config {
    int32_t n_envs;      /* environments in this context (this rank's shard) */
    int32_t n_agents;    /* cars per environment, 1..8 */
    int32_t n_beams;     /* 1080 */
    int32_t theta_dis;   /* 2000 */
    int32_t integrator;  /* F110_INTEGRATOR_RK4 (F110Env default) */
    int32_t ego_idx;     /* 0 */
    int32_t autoreset;   /* 1: a terminated env is reset (spawn table) at its next f110_step */
    int32_t _pad;
    double fov;          /* 4.7 */
    double eps;          /* 1e-4 */
    double max_range;    /* 30.0 */
    double time_step;    /* 0.01 */
    double lidar_dist;   /* 0.0 */
    double ttc_thresh;   /* 0.005 (base_classes.py:115) */
    double noise_std;    /* 0.01 (laser_models.py:429); 0 disables scan noise */
    int64_t env_offset;  /* global id of env 0 of this context (RNG keying across ranks) */
    uint64_t seed;       /* scan-noise / autoreset seed (F110Env 'seed' kwarg) */
} f110_config;

/* Per-step outputs (all optional except where noted; NULL = not written). */
typedef struct f110_outputs {
    float *obs;          /* [n_envs][n_beams + 4*n_agents]: F110Env._pack_flat_obs
                            (f110_env.py:552-584) generalised to A agents; A=2 -> 1088 */
    float *scans;        /* [n_envs][n_agents][n_beams] f32 ranges (info["scans"], :599) */
    double *scans_f64;   /* [n_envs][n_agents][n_beams] fp64 ranges (Simulator.step obs['scans']) */
    uint8_t *collisions; /* [n_envs][n_agents] 0/1 (Simulator.collisions) */
    uint8_t *terminated; /* [n_envs] F110Env._check_done (f110_env.py:310-352) */
    uint8_t *was_reset;  /* [n_envs] 1 where this call reset the env (autoreset / f110_reset) */
    float *lap_times;    /* [n_envs][n_agents] */
    float *lap_counts;   /* [n_envs][n_agents] */
    double *sim_time;    /* [n_envs] F110Env.current_time */
    int64_t obs_stride;  /* floats from one obs row to the next (>= n_beams + 4*n_agents); 0 = packed.
                            A 128-B multiple (1088 for A = 1) keeps every 64-beam chunk of a row on
                            whole cache lines: the ray kernel's obs stores are not split. */
} f110_outputs;

typedef struct f110_ctx f110_ctx;

/* ---- library ---------------------------------------------------------- */
F110_API int f110_abi_version(void);
F110_API const char *f110_last_error(void);
/* Fills the F110Env defaults (f110_env.py:132-156, :159-186). */
F110_API void f110_default_params(f110_params *p);
F110_API void f110_default_config(f110_config *c);

/* ---- map (cold path, host memory) -------------------------------------- */
/* Exact squared EDT of an occupancy grid: k[r*W+c] = squared distance (in
 * cells) from (r,c) to the nearest occupied cell (free_mask == 0).
 * Replaces get_dt / scipy.ndimage.distance_transform_edt
 * (laser_models.py:40-53, :425): dt = resolution * sqrt((double)k), bit-for-bit.
 * free_mask is the image after ScanSimulator2D.set_map's flip + threshold
 * (laser_models.py:397-404). */
F110_API int f110_edt_k(const uint8_t *free_mask, int32_t H, int32_t W, uint32_t *k_out);

/* ---- context ------------------------------------------------------------
 * Replaces Simulator.__init__ + set_map (base_classes.py:478-524) and
 * ScanSimulator2D.__init__/set_map (laser_models.py:360-427).  edt_k: HOST
 * [H*W] from f110_edt_k.  origin = map yaml 'origin' (x, y, yaw).
 * spawn_poses: optional HOST [n_spawn][n_agents][3] table used by autoreset. */
F110_API int f110_create(f110_ctx **out, int32_t device, const f110_config *cfg, const f110_params *params,
                const uint32_t *edt_k, int32_t H, int32_t W, double resolution, const double origin[3],
                const double *spawn_poses, int32_t n_spawn);
F110_API int f110_destroy(f110_ctx *ctx);

/* ---- per step (device pointers, async on stream) ----------------------- */
/* Replaces F110Env.reset (f110_env.py:425-472) = Simulator.reset
 * (base_classes.py:627-643) + RaceCar.reset (:183-204) + the zero-action
 * step the reference performs inside reset (f110_env.py:457-458).
 * poses: [n_envs][n_agents][3] f64.  env_mask: [n_envs] u8, NULL = all envs.
 * Only masked envs are touched; their outputs are written. */
F110_API int f110_reset(f110_ctx *ctx, const double *poses, const uint8_t *env_mask, const f110_outputs *out,
               void *stream);

/* Replaces F110Env.step (f110_env.py:371-421) = Simulator.step
 * (base_classes.py:566-625): per agent update_pose (steer delay, pid, RK4 of
 * vehicle_dynamics_st, clamps) + ScanSimulator2D.scan (+ noise), GJK
 * collision_multiple, TTC (check_ttc_jit), agent ray_cast, obs packing,
 * _check_done.  actions: [n_envs][n_agents][2] (steer, velocity), f32
 * (F110Env's action_space dtype, f110_env.py:238-242) or f64 (Simulator.step
 * takes whatever control_inputs dtype it is given): actions_dtype = F110_F32 /
 * F110_F64. */
F110_API int f110_step(f110_ctx *ctx, const void *actions, int32_t actions_dtype, const f110_outputs *out,
                       void *stream);
/* n_steps consecutive f110_step calls with resident actions: step t reads the
 * [n_envs][n_agents][2] block at actions + t * step_stride elements
 * (step_stride 0 = packed, n_envs * n_agents * 2) -- a rollout of open-loop
 * actions; every output holds the last step's values, exactly as after the n
 * calls (the three-launch step runs n times, no host work in between). */
F110_API int f110_step_n(f110_ctx *ctx, const void *actions, int32_t actions_dtype, int32_t n_steps,
                         int64_t step_stride, const f110_outputs *out, void *stream);

/* Replaces F110Env.update_params / Simulator.update_params
 * (f110_env.py:487-498, base_classes.py:527-546): agent_idx < 0 updates every
 * car, otherwise one car (out of range -> F110_E_INVALID, the reference's
 * IndexError).  Like RaceCar.params, the update reaches the car's dynamics
 * (update_pose) and the opponent boxes of its agent ray_cast
 * (base_classes.py:223); the GJK boxes (Simulator.params, :562), the TTC
 * side distances (class-level, :122-158) and the obs lidar_max keep the
 * params given to f110_create, as in the reference.  params is a host
 * pointer; the call is ordered on `stream` and returns when it is applied. */
F110_API int f110_set_params(f110_ctx *ctx, const f110_params *params, int32_t agent_idx, void *stream);

/* Scan-noise source of the following f110_step / f110_reset calls.
 * noise: device [n_envs][n_beams] f64, or NULL for the built-in stream.
 * The reference draws the noise as rng.normal(0, std_dev, num_beams) from a
 * numpy Generator that every car re-creates with the same seed at reset
 * (laser_models.py:450-452, base_classes.py:119,204), so the agents of one
 * env see the same vector.  With a buffer set, each ray adds
 * noise[env][beam] to its clamped range instead of the device Philox draw
 * (noise_std is then unused).  The caller refills the buffer before each
 * call, ordered on the same stream; it must outlive the calls that read it.
 * The F110Env facade uses it to replay the reference's generator exactly. */
F110_API int f110_set_scan_noise(f110_ctx *ctx, const double *noise);

/* ---- state access ------------------------------------------------------- */
/* state: device [7][n_envs*n_agents] f64 (SoA, see header comment).
 * steer_buf: device [2][n_envs*n_agents] f64 ([newest, older]); steer_cnt:
 * device [n_envs*n_agents] i32 — RaceCar.steer_buffer (base_classes.py:108-109). */
F110_API int f110_get_state(f110_ctx *ctx, double *state, double *steer_buf, int32_t *steer_cnt, void *stream);
/* F110Env's lap bookkeeping as the device holds it (f110_env.py:310-352,
 * 441-451): start_rot[2][E] = cos(-th), sin(-th) of each env's ego reset
 * yaw (float64, or float32 values under F110_F32 resets) and toggles[E*A]
 * (toggle_list).  Device pointers (either may be NULL), async on `stream`. */
F110_API int f110_get_lap_state(f110_ctx *ctx, double *start_rot, int32_t *toggles, void *stream);
F110_API int f110_set_state(f110_ctx *ctx, const double *state, const double *steer_buf, const int32_t *steer_cnt,
                   void *stream);

/* ---- building blocks (device pointers) ----------------------------------
 * Replaces ScanSimulator2D.scan with rng=None (laser_models.py:429-454) =
 * get_scan/trace_ray (:106-186): poses [M][3] (x, y, yaw) -> scans [M][n_beams]
 * f64.  lookups [M][n_beams] i32 and hit_rc [M][n_beams][2] i32 (last EDT cell
 * read by each ray) are optional probes. */
F110_API int f110_scan_batch(f110_ctx *ctx, const double *poses, int64_t M, double *scans, int32_t *lookups,
                    int32_t *hit_rc, void *stream);

/* Replaces vehicle_dynamics_st (dynamic_models.py:123-176) on M states:
 * x [M][7], u [M][2] (steer velocity, acceleration) -> f [M][7]. */
F110_API int f110_dynamics_batch(f110_ctx *ctx, const double *x, const double *u, double *f, int64_t M, void *stream);

/* vehicle_dynamics_ks (dynamic_models.py:90-121) for M kinematic states:
 * x[M][5] = (x, y, steer, v, yaw), u[M][2] = (steer velocity, accel) ->
 * f[M][5], under the context's params (the KS model of the reference's
 * DynamicsTest KATs; the ST model's |v| < 0.5 branch uses the same terms).
 * Device pointers, async on `stream`.  Replaces: a loop of
 * vehicle_dynamics_ks calls. */
F110_API int f110_dynamics_ks_batch(f110_ctx *ctx, const double *x, const double *u, double *f, int64_t M,
                                    void *stream);

/* ---- collision building blocks (no context) --------------------------------
 * f110_collision_batch: collision(vertices1, vertices2) (collision_models.py:
 * 113-182, 2-D GJK, <= 1000 iterations) for M pairs: v1[M][4][2], v2[M][4][2]
 * -> out[M] (1 = overlap).  Replaces: a Python loop over collision().
 * f110_collision_multiple: collision_multiple(vertices) (collision_models.py:
 * 184-212) for M independent sets of N bodies: verts[M][N][4][2] ->
 * collisions[M][N] (0./1.) and idx[M][N] (partner index, -1. if none; the
 * last colliding pair in the reference's i < j loop order wins), 1 <= N <= 64.
 * Device pointers, async on `stream`. */
F110_API int f110_collision_batch(const double *v1, const double *v2, int64_t M, uint8_t *out, void *stream);
F110_API int f110_collision_multiple(const double *verts, int64_t M, int32_t N, double *collisions, double *idx,
                                     void *stream);

/* The dtype of the reset poses whose F110Env.reset semantics the following
 * resets follow (f110_env.py:441-451): F110_F32 (train_ddpg passes float32
 * options) rounds the reset / autoreset poses to float32 and evaluates the lap
 * logic's start_rot as NumPy's float32 cos / sin of the float32 yaw;
 * F110_F64 (the default) keeps float64.  Replaces: the dtype the consumer's
 * `options` array carries into F110Env.reset. */
F110_API int f110_set_reset_dtype(f110_ctx *ctx, int32_t dtype);

/* Scheduling hint for a caller that steps several contexts concurrently on one
 * device (e.g. sub-shards of one GPU's envs on separate streams): this context
 * is one of `contexts` whose ray passes run together, tracing `device_cars`
 * cars (envs x agents) in all.  The library then picks the ray kernel for the
 * device's load instead of this context's alone (DESIGN.md §3.3-3.4, §3.14,
 * §5.1: k_rays_fxs with 1 / 2 / 3 waves per car by the device's cars; with
 * other contexts, no heavy-first dispatch and, for single-agent contexts,
 * the 8-wave blocks that keep the theta table in LDS, since the other
 * contexts' ray passes fill this one's tail and idle slots).  Call before the first
 * reset / step.  Scheduling only: results are bit-identical with or without
 * it.  No reference counterpart (the reference steps one env per process). */
F110_API int f110_set_device_share(f110_ctx *ctx, int64_t device_cars, int32_t contexts);

/* ---- opponent policy -------------------------------------------------------
 * Replaces gap_follow_action (rl_training/utils/gap_follow.py:3-58), the
 * rule-based opponent train_ddpg.py:168 computes on the host each step from
 * the float32 info["scans"][1].  Device pointers: scan m is the n_beams
 * float32 values at scans + m*scan_stride (e.g. agent 1 of env m in
 * f110_outputs.scans: scans + B, stride A*B); its (steer, speed) goes to
 * actions[m*action_stride + 0/1] as float32 (e.g. agent 1's slot of the next
 * f110_step's action array: stride 2*A).  gaps [n_scans][2] (optional) gets
 * the chosen gap (start, end).  Bit-exact with the reference's NumPy
 * float32 arithmetic; angle_min / angle_increment are the reference
 * defaults -pi/2 and pi/1080 unless overridden.  Async on stream. */
F110_API int f110_gap_follow(const float *scans, int64_t n_scans, int64_t scan_stride, int32_t n_beams,
                             double angle_min, double angle_increment, float *actions, int64_t action_stride,
                             int32_t *gaps, void *stream);

/* ---- training reward ---------------------------------------------------------
 * Replaces rl_training/utils/rewards.py:CenterlineSafetyProgressReward
 * (:185-355) over utils/track_progress.py:CenterlineProgress (:5-110), the
 * reward train_ddpg.py:125-176 computes on the host from every next_obs.
 * Batched over envs on the device, one wave per env. */
typedef struct f110_track f110_track;

/* CenterlineProgress(csv, closed): xy [n][2] and the optional lane widths
 * (w_tr_right_m / w_tr_left_m, NULL = none) as the CSV holds them; arclength,
 * tangents, normals and segment midpoints are derived here exactly as the
 * reference derives them (track_progress.py:29-46).  Host pointers.
 * device < 0 builds the host arrays only (f110_track_arrays; no reward). */
F110_API int f110_track_create(f110_track **out, int32_t device, const double *xy, const double *w_right,
                               const double *w_left, int32_t n, int32_t closed);
F110_API int f110_track_destroy(f110_track *track);
/* The derived arrays (host copies; any pointer may be NULL): s [n],
 * tan/nrm/mid [n-1][2]; returns L (the total arclength). */
F110_API double f110_track_arrays(const f110_track *track, double *s, double *tan, double *nrm, double *mid);

/* CenterlineSafetyProgressReward.__init__ kwargs (rewards.py:196-230). */
typedef struct f110_reward_params {
    double dt, w_prog, forward_sign, alive_bonus, w_rel_lead, lead_clip, w_lat, lat_cap, default_half_width;
    double lidar_max, near_wall_dist, w_wall, wall_quantile, opp_safe_dist, w_opp, ego_crash_penalty;
    double opp_crash_bonus, beta;  /* beta: _Prog / _ProgFallback EMA factor (0.8) */
    int32_t grace_steps_wall, grace_steps_opp, auto_flip_steps; /* auto_flip_steps: _Prog (20) */
    int32_t use_progress;          /* 1: centerline _Prog (a track is given), 0: _ProgFallback */
} f110_reward_params;

/* Per-env reward state in device memory; all-zero bytes = reward_fn.reset()
 * (rewards.py:97-107 _Prog.reset, :256 reset). */
typedef struct f110_reward_state {
    double s_prev[2];  /* ego, opp: last arclength (_Prog._s_prev) */
    double px[2], py[2];  /* last positions (_p_prev / _ProgFallback.prev) */
    double cum[2];     /* _cum */
    double ema;        /* _ema_abs_dego / ma_ego */
    double t_last[2];  /* last lateral offsets */
    double auto_sum;   /* running sum of _auto_buf */
    int32_t steps;     /* _steps */
    int32_t auto_n;    /* len(_auto_buf) */
    int32_t flags;     /* bit0/1: s_prev ego/opp set, bit2/3: p_prev ego/opp set, bit4: _flip == -1 */
    int32_t pad_;
} f110_reward_state;

F110_API void f110_default_reward_params(f110_reward_params *p);

/* reward_fn(next_obs) for n_envs flat observations (device, float32
 * [n_envs][obs_len], the F110Env layout: n_beams scaled ranges, then x, y,
 * yaw, collision of ego and opponent; parse_flat_obs, rewards.py:11-41).
 * state: device [n_envs]; reset_mask: device [n_envs] u8 or NULL -- a
 * masked env's state is reset (reward_fn.reset()) and its reward is 0 (the
 * reset observation of an autoresetting vector env is not rewarded).
 * rewards: device [n_envs] f64.  track may be NULL when
 * params->use_progress == 0.  Async on stream. */
F110_API int f110_reward(const f110_track *track, const f110_reward_params *params, const float *obs, int64_t n_envs,
                         int32_t obs_len, int32_t n_beams, f110_reward_state *state, const uint8_t *reset_mask,
                         double *rewards, void *stream);

/* ---- prioritized experience replay ---------------------------------------------
 * Replaces rl_training/DDPG/replay_buffer.py:PrioritizedExperienceReplayBuffer
 * (:6-135), the DDPG agent's memory (agent.py:194): a ring of transitions
 * (state, action, reward, next_state, done) with one float32 priority each.
 * All of it lives in device memory; every call below is asynchronous on
 * `stream` and takes device pointers, except f110_replay_length /
 * f110_replay_stats, which wait for the stream. */
typedef struct f110_replay f110_replay;

/* PrioritizedExperienceReplayBuffer(buffer_size=capacity, batch_size, alpha,
 * seed, priority_epsilon=eps) (:18-40).  max_batch bounds the batch of
 * f110_replay_sample (<= 8192) and max_add the rows of one f110_replay_add;
 * obs_dim / act_dim are the state / action lengths (1088 / 2 in train_ddpg). */
F110_API int f110_replay_create(f110_replay **out, int32_t device, int64_t capacity, int32_t obs_dim,
                                int32_t act_dim, int32_t max_batch, int64_t max_add, double alpha, double eps,
                                uint64_t seed);
F110_API int f110_replay_destroy(f110_replay *rb);

/* n calls of add(Experience(state, action, reward, next_state, done)) with
 * priority=None (:48-71, agent.remember agent.py:223-237), in row order: the
 * new rows get the current max priority (1.0 when empty).  obs / next_obs:
 * rows of obs_dim floats at a stride of obs_stride / next_stride floats;
 * act: act_dim floats per row at act_stride; reward [n] f32; done [n] u8
 * (NULL = all 0).  priority [n] f32: add(exp, priority=p) (clipped to
 * [1e-8, FLT_MAX]); NULL = priority=None.  mask [n] u8 (NULL = all rows):
 * only rows with mask != 0 are stored (e.g. not the reset rows of an
 * autoresetting vector env). */
F110_API int f110_replay_add(f110_replay *rb, const float *obs, int64_t obs_stride, const float *act,
                             int64_t act_stride, const float *reward, const float *next_obs, int64_t next_stride,
                             const uint8_t *done, const float *priority, const uint8_t *mask, int64_t n,
                             void *stream);

/* f110_replay_add for a vector env's raw step outputs (train_ddpg.py:177-183,
 * agent.remember per transition): reward [n] f64 (stored rounded to f32),
 * terminated [n] u8 (the done flag), was_reset [n] u8 -- rows with
 * was_reset != 0 (NEXT_STEP autoreset: obs is the finished episode's, next_obs
 * the new one's) are not stored.  No torch dtype conversions on the caller's side. */
F110_API int f110_replay_add_env(f110_replay *rb, const float *obs, int64_t obs_stride, const float *act,
                                 int64_t act_stride, const double *reward, const float *next_obs,
                                 int64_t next_stride, const uint8_t *terminated, const uint8_t *was_reset,
                                 int64_t n, void *stream);

/* sample(beta) (:76-116) of `batch` rows: without replacement when the buffer
 * holds at least `batch` rows (distributed like numpy's
 * Generator.choice(replace=False, p=...): successive draws, in draw order),
 * i.i.d. otherwise.  Writes idx [batch] i64, weights [batch] f32 (normalised
 * IS weights) and, when obs != NULL, the gathered batch agent.replay stacks
 * (agent.py:257-270): obs / next_obs [batch][obs_dim], act [batch][act_dim],
 * reward / done [batch] f32.  The caller must not sample an empty buffer
 * (the reference raises ValueError, :83-84). */
F110_API int f110_replay_sample(f110_replay *rb, int32_t batch, double beta, int64_t *idx, float *weights, float *obs,
                                float *act, float *reward, float *next_obs, float *done, void *stream);

/* update_priorities(idx, priorities) (:121-135): the priority of row idx[j]
 * becomes clip(p_j, 1e-8, FLT_MAX) in float32 with NaN -> 1e-6, where
 * p_j = values[j] (from_td == 0) or agent.replay's |values[j]| + add_eps
 * (from_td != 0, values = TD errors, agent.py:337).  Repeated indices keep
 * the last value. */
F110_API int f110_replay_update_priorities(f110_replay *rb, const int64_t *idx, const float *values, int64_t n,
                                           int32_t from_td, float add_eps, void *stream);

/* len(buffer) (:42-43) and the ring pointer; waits for `stream`. */
F110_API int f110_replay_length(f110_replay *rb, int64_t *length, int64_t *next_idx, void *stream);

/* Device pointers of the stored arrays (read-only views for tests and
 * checkpoints): priority [capacity] f32, obs / next_obs [capacity][obs_dim],
 * act [capacity][act_dim], reward / done [capacity] f32.  Any out pointer
 * may be NULL. */
F110_API int f110_replay_arrays(f110_replay *rb, float **priority, float **obs, float **act, float **reward,
                                float **next_obs, float **done);

/* ---- learner optimizer ----------------------------------------------------------
 * One torch.optim.Adam step (agent.py:187-188: Adam(params, lr), betas
 * (0.9, 0.999), eps 1e-8, no weight decay, no amsgrad) over a network whose
 * parameters, gradients and moments are flat float32 device buffers of n
 * elements.  state: device int64 step counter followed by a uint32 scratch
 * word (both zero initially); the step is advanced on the device, so the
 * call can be captured in a HIP graph.  target (may be null): the network's
 * target copy, soft-updated in the same pass after the step (agent.py:340-341,
 * target.lerp_(param, tau)).  Async on stream. */
F110_API int f110_adam_step(float *param, float *exp_avg, float *exp_avg_sq, const float *grad, int64_t n, double lr,
                            double beta1, double beta2, double eps, void *state, float *target, double tau,
                            void *stream);

/* ---- learner heads -------------------------------------------------------------
 * The DDPG networks' output layers fused with what follows them
 * (rl_training agent.py: Actor.fc3 + tanh + action-box map :56-61, Critic.q
 * :93-97, replay()'s TD target :302-308, weighted MSE :310-316, actor loss
 * -mean(q) :321-326), replacing torch's skinny GEMM + elementwise launches.
 * Row-major float32 device buffers: h [B][K] (the last hidden layer), W
 * [nout][K], b [nout]; K <= 255, nout <= 4 (nout = 1 for the critic).
 * scratch: f110_ddpg_scratch_floats(B, K, nout) floats.  dh / dW / db
 * outputs may be null (not wanted); dh_mask [B][K] (may be null) zeroes dh
 * where dh_mask <= 0 (h's ReLU: threshold_backward fused into the head).  g: device scalar, the gradient of the
 * loss (autograd's grad_output).  Deterministic; async on stream. */
F110_API int64_t f110_ddpg_scratch_floats(int32_t B, int32_t K, int32_t nout);
/* t = tanh(h W^T + b); act = scale * t + shift  (act, t: [B][nout]) */
F110_API int f110_ddpg_actor_head(const float *h, const float *W, const float *b, const float *scale,
                                  const float *shift, int32_t B, int32_t K, int32_t nout, float *act, float *t,
                                  void *stream);
/* choose_action(training=True) after the hidden layers (agent.py:350-370 with
 * GaussianActionNoise :520-539): out[row * out_stride + j] = clip(scale * tanh(h W^T + b) + shift
 * + sigma * n, low[j], high[j]), n ~ N(0, 1) independent per (row, j) and per call (Philox2x32
 * keyed by seed, counter = the call index); NaN actions stay NaN.  The noise state lives on the
 * device so a captured graph can replay the call: state_in = {sigma, call index} (f64), and the
 * launch writes state_out = {max(sigma * decay, sigma_min), call index + 1} (state_out !=
 * state_in: callers alternate two slots).  out may be a strided view (e.g. the vector env's
 * action rows). */
F110_API int f110_ddpg_actor_explore(const float *h, const float *W, const float *b, const float *scale,
                                     const float *shift, int32_t B, int32_t K, int32_t nout, const double *state_in,
                                     double *state_out, double decay, double sigma_min, const float *low,
                                     const float *high, uint64_t seed, float *out, int64_t out_stride, void *stream);
/* The critic update's head in one launch: y = r + gamma (1 - d) (ht Wt^T + bt) (the target critic),
 * td = y - (h W^T + b), part[blk] = block sums of w td^2 (f110_ddpg_row_blocks(B) floats; the loss
 * is sum(part) / B: f110_learner_wgrad_loss), dq = -((g / B) w) (2 td) (may be null), dh = dq W where
 * dh_mask > 0 (dh may be null).  = f110_ddpg_td_target + f110_ddpg_critic_loss + the row part of
 * f110_ddpg_critic_loss_bwd, same float operations. */
F110_API int f110_ddpg_critic_step(const float *ht, const float *Wt, const float *bt, const float *r, const float *d,
                                   float gamma, const float *h, const float *W, const float *b, const float *w,
                                   const float *g, int32_t B, int32_t K, float *td, float *dh, const float *dh_mask,
                                   float *dq, float *part, void *stream);
/* The actor update's loss head: part[blk] = block sums of q = h W^T + b (the loss is sign sum(part) / B),
 * dh = (sign g / B) W where dh_mask > 0.  = f110_ddpg_q_mean + the row part of f110_ddpg_q_mean_bwd. */
F110_API int f110_ddpg_q_mean_step(const float *h, const float *W, const float *b, const float *g, float sign,
                                   int32_t B, int32_t K, float *dh, const float *dh_mask, float *part, void *stream);
/* blocks of the row-per-half-wave head launches for B rows (their partial-sum counts) */
F110_API int32_t f110_ddpg_row_blocks(int32_t B);
/* dz = (dact * scale) * (1 - t*t); dh = dz W; dW = dz^T h; db = sum_rows dz */
F110_API int f110_ddpg_actor_head_bwd(const float *h, const float *W, const float *t, const float *scale,
                                      const float *dact, int32_t B, int32_t K, int32_t nout, float *dh,
                                      const float *dh_mask, float *dW, float *db, float *scratch, void *stream);
/* y = r + (gamma * (1 - d)) * (h W^T + b) */
F110_API int f110_ddpg_td_target(const float *h, const float *W, const float *b, const float *r, const float *d,
                                 float gamma, int32_t B, int32_t K, float *y, void *stream);
/* td = y - (h W^T + b); loss = mean(w * td * td)  (loss: device scalar) */
F110_API int f110_ddpg_critic_loss(const float *h, const float *W, const float *b, const float *y, const float *w,
                                   int32_t B, int32_t K, float *td, float *loss, float *scratch, void *stream);
/* dq = -((g / B) * w) * (2 td); dh, dW, db from dq */
F110_API int f110_ddpg_critic_loss_bwd(const float *h, const float *W, const float *td, const float *w,
                                       const float *g, int32_t B, int32_t K, float *dh, const float *dh_mask,
                                       float *dW, float *db, float *scratch, void *stream);
/* loss = sign * mean(h W^T + b)  (sign -1: the actor loss) */
F110_API int f110_ddpg_q_mean(const float *h, const float *W, const float *b, float sign, int32_t B, int32_t K,
                              float *loss, float *scratch, void *stream);
/* A hidden layer's ReLU backward with its bias gradient (agent.py's F.relu(fc(x))
 * under autograd): gz = gy where y > 0 else 0 (torch threshold_backward), db =
 * sum_rows gz (db may be null).  gy, y, gz: [B][K]; K <= 1024; scratch:
 * f110_ddpg_relu_bwd_scratch_floats(B, K) floats. */
F110_API int64_t f110_ddpg_relu_bwd_scratch_floats(int32_t B, int32_t K);
F110_API int f110_ddpg_relu_bwd(const float *gy, const float *y, int32_t B, int32_t K, float *gz, float *db,
                                float *scratch, void *stream);
/* dq = sign * (g / B); dh, dW, db from dq (h only needed for dW / db) */
F110_API int f110_ddpg_q_mean_bwd(const float *h, const float *W, const float *g, float sign, int32_t B, int32_t K,
                                  float *dh, const float *dh_mask, float *dW, float *db, float *scratch,
                                  void *stream);

/* ---- learner GEMMs (fp32 matrix cores) -------------------------------------------
 * The hidden layers of the DDPG networks (agent.py:25-97: fc1 / fc2, fcs1 /
 * fcs2 and replay()'s backward through them, :302-331), forward and backward,
 * as grouped fp32 MFMA launches with the layer's epilogue fused.  Replaces
 * torch.addmm + relu, threshold_backward, torch.cat([z, action]) and the
 * weight / input gradient GEMMs of autograd.  Row-major float32 device
 * buffers; every op of one launch shares M (the batch rows).
 *
 * f110_learner_gemm: for each op,
 *   C[m][n] = epi( sum_k A'[m][k] B(k, n)  +  sum_{t < nx2} x2[m][t] w2[n][t]  +  bias[n] )
 *   A'[m][k] = amask ? (amask[m][k] > 0 ? A[m][k] : 0) : A[m][k]   (amask stride lda)
 *   B(k, n)  = nn ? B[k * ldb + n] : B[n * ldb + k]   (nn = 0: a Linear's weight
 *              [N][K] as in x W^T; nn = 1: the weight itself as in g W)
 *   epi: ReLU when relu != 0 (NaN kept, as torch.relu), then
 *        C := omask[m][n] > 0 ? C : 0 when omask is set (stride ldc).
 * bias, amask, omask, x2 / w2 may be null; nx2 <= 2 (the critic's action
 * columns of fcs2's input, agent.py:94).  All ops of a launch share nn and
 * whether amask is set.
 * Deterministic (fixed summation order); async on stream. */
typedef struct f110_gemm_op {
    const float *A, *B, *bias, *amask, *omask, *x2, *w2;
    float *C;
    int32_t N, K, lda, ldb, ldc, ldx2, ldw2, nx2, relu, nn;
} f110_gemm_op;
F110_API int f110_learner_gemm(const f110_gemm_op *ops, int32_t nops, int32_t M, void *stream);

/* f110_learner_wgrad: a Linear's weight and bias gradients, for each op
 *   dW[n][kx] (stride ldw) = sum_m G'[m][n] X[m][kx],  db[n] = sum_m G'[m][n]
 *   G'[m][n] = gmask ? (gmask[m][n] > 0 ? G[m][n] : 0) : G[m][n]   (gmask stride ldg)
 * (autograd's grad_W = gz^T x and grad_b = gz.sum(0) after threshold_backward).
 * db may be null; all ops of a launch share whether gmask is set.  M is split over blocks; the partial sums go to scratch
 * (f110_learner_wgrad_scratch_floats floats) and are added in a fixed order. */
typedef struct f110_wgrad_op {
    const float *G, *gmask, *X;
    float *dW, *db;
    int32_t N, KX, ldg, ldx, ldw;
} f110_wgrad_op;
F110_API int64_t f110_learner_wgrad_scratch_floats(const f110_wgrad_op *ops, int32_t nops, int32_t M);
F110_API int f110_learner_wgrad(const f110_wgrad_op *ops, int32_t nops, int32_t M, float *scratch, void *stream);
/* f110_learner_wgrad, and in its finishing launch *loss = sign * (sum of loss_part[0 .. n_part), in
 * order) / M: the loss of a fused head (f110_ddpg_critic_step / f110_ddpg_q_mean_step) without a
 * launch of its own. */
F110_API int f110_learner_wgrad_loss(const f110_wgrad_op *ops, int32_t nops, int32_t M, float *scratch,
                                     const float *loss_part, int32_t n_part, float sign, float *loss, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* F110_H */
