/*
 * f110_oracle.c — CPU restatement of the f110_gym per-step hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it
 * (oracle/liboracle.so via oracle/oracle.py).  The product path
 * (f110_gymnasium_ros2_jazzy_amd/, libf110.so) never links or calls it.
 *
 * Pinned against the golden vectors in tests/golden/ that were produced by
 * executing the reference's own Python source (tests/golden/make_golden.py);
 * tests/test_oracle_golden.py holds those checks.
 *
 * Every function cites the reference file:line it restates; paths are under
 * f110_gymnasium/gym/f110_gym/envs/ of ahoop004/f110_gymnasium_ros2_jazzy.
 *
 * Floating point: compiled with -ffp-contract=off; Python's left-to-right
 * evaluation order is kept term by term.  Where the reference goes through
 * NumPy's BLAS (ndarray.dot, np.linalg.norm) the rounding pattern measured
 * for this container's OpenBLAS 0.3.29 (SkylakeX kernels) is reproduced with
 * explicit fma() calls (see DESIGN.md "Rounding contract"):
 *   2-vector dot  a.dot(b)          = fma(a1, b1, a0*b0)
 *   (4,2)@(2,)    V.dot(d)[j]       = fma(V[j,0], d0, V[j,1]*d1)
 *   norm(a), a 2-vector             = sqrt(fma(a1, a1, a0*a0))
 *   (4,4)@(4,1)   get_vertices rows = (H0*p0) + ((H1*p1) + H3)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_API __attribute__((visibility("default")))

/* Residue attribution (not the reference's arithmetic): the
 * sin / cos calls whose device counterparts are the correctly rounded
 * cr_sincos (dynamics, scan pose, get_vertices, ray_cast beam direction,
 * get_blocked_view_indices' ego bearing) go through or_sin / or_cos.  By
 * default they are glibc's sin / cos, as NumPy's and Numba's; with a hook set
 * (or_set_sincos_hook: libf110's f110_host_sincos, the host copy of
 * cr_sincos) the oracle reproduces the device's trig, so whatever still
 * differs from the device is not glibc's own last-ulp error.  The lookup
 * tables (sines / cosines, RaceCar's beam tables) stay glibc's: the device
 * uses the host's tables too. */
typedef void (*or_sincos_fn)(const double *x, int64_t n, double *sn, double *cs);
static or_sincos_fn g_sincos_hook = NULL;
OR_API void or_set_sincos_hook(or_sincos_fn fn) { g_sincos_hook = fn; }
static double or_sin(double x) {
    if (!g_sincos_hook) return sin(x);
    double s, c;
    g_sincos_hook(&x, 1, &s, &c);
    return s;
}
static double or_cos(double x) {
    if (!g_sincos_hook) return cos(x);
    double s, c;
    g_sincos_hook(&x, 1, &s, &c);
    return c;
}

typedef struct {
    double mu, C_Sf, C_Sr, lf, lr, h, m, I, s_min, s_max, sv_min, sv_max, v_switch, a_max,
        v_min, v_max, width, length;
} or_params;

typedef struct {
    int32_t H, W, theta_dis, num_beams;
    double res, orig_x, orig_y, orig_c, orig_s;
    double fov, eps, max_range, theta_index_increment;
    const double *dt;      /* [H*W] metres */
    const double *sines;   /* [theta_dis]  */
    const double *cosines; /* [theta_dis]  */
} or_scanner;

/* ------------------------------------------------------------------ EDT --
 * get_dt, laser_models.py:40-53: dt = res * scipy.ndimage.distance_transform_edt(bitmap).
 * Exact squared Euclidean distance to the nearest zero (occupied) cell,
 * Meijster-Roerdink-Hesselink two-pass algorithm, integer arithmetic only.
 * out k[r*W+c] = squared distance in cells; dt = res*sqrt((double)k).
 * A map with no occupied cell has no defined EDT: returns -1. */
OR_API int or_edt_k(const uint8_t *free_mask, int H, int W, uint32_t *k_out) {
    const int64_t INF = (int64_t)H + W + 1;
    int64_t *g = (int64_t *)malloc(sizeof(int64_t) * (size_t)H * W);
    if (!g) return -2;
    int any = 0;
    for (int c = 0; c < W; ++c) {
        /* phase 1: per column, distance in rows to the nearest occupied cell */
        g[c] = free_mask[c] ? INF : 0;
        for (int r = 1; r < H; ++r)
            g[(size_t)r * W + c] = free_mask[(size_t)r * W + c] ? g[(size_t)(r - 1) * W + c] + 1 : 0;
        for (int r = H - 2; r >= 0; --r)
            if (g[(size_t)(r + 1) * W + c] < g[(size_t)r * W + c])
                g[(size_t)r * W + c] = g[(size_t)(r + 1) * W + c] + 1;
    }
    for (size_t i = 0; i < (size_t)H * W; ++i) any |= (g[i] == 0);
    if (!any) { free(g); return -1; }
    int64_t *s = (int64_t *)malloc(sizeof(int64_t) * W);
    int64_t *t = (int64_t *)malloc(sizeof(int64_t) * W);
    for (int r = 0; r < H; ++r) {
        const int64_t *gr = g + (size_t)r * W;
#define F(x, i) (((int64_t)(x) - (i)) * ((int64_t)(x) - (i)) + gr[i] * gr[i])
        int q = 0;
        s[0] = 0;
        t[0] = 0;
        for (int u = 1; u < W; ++u) {
            while (q >= 0 && F(t[q], s[q]) > F(t[q], u)) --q;
            if (q < 0) {
                q = 0;
                s[0] = u;
            } else {
                /* Sep(i,u) = floor((u^2 - i^2 + g(u)^2 - g(i)^2) / (2(u-i))) */
                int64_t i = s[q];
                int64_t num = (int64_t)u * u - i * i + gr[u] * gr[u] - gr[i] * gr[i];
                int64_t den = 2 * ((int64_t)u - i);
                int64_t w = num >= 0 ? num / den : -((-num + den - 1) / den);
                w += 1;
                if (w < W) {
                    ++q;
                    s[q] = u;
                    t[q] = w;
                }
            }
        }
        for (int u = W - 1; u >= 0; --u) {
            int64_t d = F(u, s[q]);
            k_out[(size_t)r * W + u] = (uint32_t)d;
            if (u == t[q]) --q;
        }
#undef F
    }
    free(s);
    free(t);
    free(g);
    return 0;
}

/* -------------------------------------------------------------- tables --
 * ScanSimulator2D.__init__, laser_models.py:367-381:
 * theta_arr = np.linspace(0, 2pi, theta_dis) (endpoint included, last = 2pi
 * exactly); sines/cosines = sin/cos(theta_arr). */
OR_API void or_scan_tables(int theta_dis, double *sines, double *cosines) {
    const double stop = 2.0 * M_PI;
    const double step = stop / (double)(theta_dis - 1);
    for (int i = 0; i < theta_dis; ++i) {
        double th = (i == theta_dis - 1) ? stop : (double)i * step;
        sines[i] = sin(th);
        cosines[i] = cos(th);
    }
}

/* RaceCar.__init__, base_classes.py:122-158 (class-level beam tables). */
OR_API void or_beam_tables(int nb, double fov, double width, double lf, double lr, double *angles,
                           double *cosines, double *side) {
    const double incr = fov / (double)(nb - 1); /* laser_models.py:367 */
    const double dist_sides = width / 2.0;
    const double dist_fr = (lf + lr) / 2.0;
    for (int i = 0; i < nb; ++i) {
        double angle = -fov / 2.0 + (double)i * incr;
        angles[i] = angle;
        cosines[i] = cos(angle);
        double to_side, to_fr;
        if (angle > 0) {
            if (angle < M_PI / 2) {
                to_side = dist_sides / sin(angle);
                to_fr = dist_fr / cos(angle);
            } else {
                to_side = dist_sides / cos(angle - M_PI / 2.0);
                to_fr = dist_fr / sin(angle - M_PI / 2.0);
            }
        } else {
            if (angle > -M_PI / 2) {
                to_side = dist_sides / sin(-angle);
                to_fr = dist_fr / cos(-angle);
            } else {
                to_side = dist_sides / cos(-angle - M_PI / 2);
                to_fr = dist_fr / sin(-angle - M_PI / 2);
            }
        }
        side[i] = to_side < to_fr ? to_side : to_fr; /* Python min(): first if equal */
    }
}

/* ---------------------------------------------------------------- scan --
 * xy_2_rc (laser_models.py:55-86) + distance_transform (:88-104).
 * Out-of-map -> (r,c) = (-1,-1) -> dt[-1,-1] (NumPy/Numba negative index wrap).
 * Returns the linear cell index it read; r_out, c_out get (r,c). */
static inline int64_t or_cell(const or_scanner *sc, double x, double y, int32_t *r_out, int32_t *c_out) {
    double x_trans = x - sc->orig_x;
    double y_trans = y - sc->orig_y;
    double x_rot = x_trans * sc->orig_c + y_trans * sc->orig_s;
    double y_rot = -x_trans * sc->orig_s + y_trans * sc->orig_c;
    int64_t r, c;
    if (x_rot < 0 || x_rot >= (double)sc->W * sc->res || y_rot < 0 || y_rot >= (double)sc->H * sc->res ||
        x_rot != x_rot || y_rot != y_rot) {
        c = -1;
        r = -1;
    } else {
        c = (int64_t)(x_rot / sc->res);
        r = (int64_t)(y_rot / sc->res);
    }
    *r_out = (int32_t)r;
    *c_out = (int32_t)c;
    int64_t n = (int64_t)sc->H * sc->W;
    if (r < 0) return n - 1; /* dt[-1,-1] */
    int64_t lin = r * sc->W + c;
    return lin < n ? lin : n - 1; /* x_rot/res rounding up to W: see DESIGN.md */
}

/* trace_ray, laser_models.py:106-146 (sphere trace over the EDT). */
static double or_trace_ray(const or_scanner *sc, double x, double y, double theta_index, int32_t *lookups,
                           int32_t *hr, int32_t *hc) {
    int64_t ti = (int64_t)theta_index;
    if (ti >= sc->theta_dis) ti = 0; /* unreachable except theta_index == theta_dis exactly */
    double s = sc->sines[ti];
    double c = sc->cosines[ti];
    int32_t n = 1;
    double dist = sc->dt[or_cell(sc, x, y, hr, hc)];
    double total = dist;
    while (dist > sc->eps && total <= sc->max_range) {
        x += dist * c;
        y += dist * s;
        dist = sc->dt[or_cell(sc, x, y, hr, hc)];
        total += dist;
        ++n;
    }
    if (total > sc->max_range) total = sc->max_range;
    *lookups = n;
    return total;
}

/* get_scan, laser_models.py:148-186 (sequential beam-index accumulation). */
OR_API void or_get_scan(const or_scanner *sc, const double *pose, double *scan, int32_t *lookups, int32_t *hit_rc) {
    const double td = (double)sc->theta_dis;
    double theta_index = td * (pose[2] - sc->fov / 2.0) / (2.0 * M_PI);
    theta_index = fmod(theta_index, td);
    while (theta_index < 0) theta_index += td;
    for (int i = 0; i < sc->num_beams; ++i) {
        int32_t n, r, c;
        scan[i] = or_trace_ray(sc, pose[0], pose[1], theta_index, &n, &r, &c);
        if (lookups) lookups[i] = n;
        if (hit_rc) {
            hit_rc[2 * i] = r;
            hit_rc[2 * i + 1] = c;
        }
        theta_index += sc->theta_index_increment;
        while (theta_index >= td) theta_index -= td;
    }
}

OR_API void or_scan_batch(const or_scanner *sc, const double *poses, int64_t M, double *scans, int32_t *lookups,
                          int32_t *hit_rc, int threads) {
    const int64_t B = sc->num_beams;
#pragma omp parallel for schedule(dynamic, 4) num_threads(threads > 0 ? threads : 1)
    for (int64_t m = 0; m < M; ++m)
        or_get_scan(sc, poses + 3 * m, scans + m * B, lookups ? lookups + m * B : NULL,
                    hit_rc ? hit_rc + 2 * m * B : NULL);
}

/* Beam theta indices exactly as get_scan accumulates them (test helper). */
OR_API void or_beam_indices(const or_scanner *sc, double yaw, double *theta_index_out) {
    const double td = (double)sc->theta_dis;
    double theta_index = td * (yaw - sc->fov / 2.0) / (2.0 * M_PI);
    theta_index = fmod(theta_index, td);
    while (theta_index < 0) theta_index += td;
    for (int i = 0; i < sc->num_beams; ++i) {
        theta_index_out[i] = theta_index;
        theta_index += sc->theta_index_increment;
        while (theta_index >= td) theta_index -= td;
    }
}

/* ------------------------------------------------------------ dynamics --
 * accl_constraints, dynamic_models.py:29-60 */
static double or_accl_constraints(double vel, double accl, double v_switch, double a_max, double v_min,
                                  double v_max) {
    double pos_limit = vel > v_switch ? a_max * v_switch / vel : a_max;
    if ((vel <= v_min && accl <= 0) || (vel >= v_max && accl >= 0))
        accl = 0.;
    else if (accl <= -a_max)
        accl = -a_max;
    else if (accl >= pos_limit)
        accl = pos_limit;
    return accl;
}

/* steering_constraint, dynamic_models.py:62-87 */
static double or_steering_constraint(double sa, double sv, double s_min, double s_max, double sv_min,
                                     double sv_max) {
    if ((sa <= s_min && sv <= 0) || (sa >= s_max && sv >= 0))
        sv = 0.;
    else if (sv <= sv_min)
        sv = sv_min;
    else if (sv >= sv_max)
        sv = sv_max;
    return sv;
}

/* vehicle_dynamics_ks, dynamic_models.py:90-121 */
OR_API void or_vehicle_dynamics_ks(const double *x, const double *u_init, const or_params *p, double *f) {
    double lwb = p->lf + p->lr;
    double u0 = or_steering_constraint(x[2], u_init[0], p->s_min, p->s_max, p->sv_min, p->sv_max);
    double u1 = or_accl_constraints(x[3], u_init[1], p->v_switch, p->a_max, p->v_min, p->v_max);
    f[0] = x[3] * or_cos(x[4]);
    f[1] = x[3] * or_sin(x[4]);
    f[2] = u0;
    f[3] = u1;
    f[4] = x[3] / lwb * tan(x[2]);
}

/* vehicle_dynamics_st, dynamic_models.py:123-176 (Python evaluation order kept). */
OR_API void or_vehicle_dynamics_st(const double *x, const double *u_init, const or_params *p, double *f) {
    const double g = 9.81;
    const double mu = p->mu, C_Sf = p->C_Sf, C_Sr = p->C_Sr, lf = p->lf, lr = p->lr, h = p->h, m = p->m,
                 I = p->I;
    double u[2];
    u[0] = or_steering_constraint(x[2], u_init[0], p->s_min, p->s_max, p->sv_min, p->sv_max);
    u[1] = or_accl_constraints(x[3], u_init[1], p->v_switch, p->a_max, p->v_min, p->v_max);
    if (fabs(x[3]) < 0.5) {
        double lwb = lf + lr;
        double fks[5];
        or_vehicle_dynamics_ks(x, u, p, fks); /* re-applies the (idempotent) constraints */
        double c2 = or_cos(x[2]);
        f[0] = fks[0];
        f[1] = fks[1];
        f[2] = fks[2];
        f[3] = fks[3];
        f[4] = fks[4];
        f[5] = u[1] / lwb * tan(x[2]) + x[3] / (lwb * (c2 * c2)) * u[0];
        f[6] = 0.0;
    } else {
        double glr_m = g * lr - u[1] * h; /* (g*lr - u[1]*h) */
        double glf_p = g * lf + u[1] * h; /* (g*lf + u[1]*h) */
        double lrlf = lr + lf;
        f[0] = x[3] * or_cos(x[6] + x[4]);
        f[1] = x[3] * or_sin(x[6] + x[4]);
        f[2] = u[0];
        f[3] = u[1];
        f[4] = x[5];
        double t1 = -mu * m / (x[3] * I * lrlf) * (lf * lf * C_Sf * glr_m + lr * lr * C_Sr * glf_p) * x[5];
        double t2 = mu * m / (I * lrlf) * (lr * C_Sr * glf_p - lf * C_Sf * glr_m) * x[6];
        double t3 = mu * m / (I * lrlf) * lf * C_Sf * glr_m * x[2];
        f[5] = t1 + t2 + t3;
        double s1 = (mu / (x[3] * x[3] * lrlf) * (C_Sr * glf_p * lr - C_Sf * glr_m * lf) - 1) * x[5];
        double s2 = mu / (x[3] * lrlf) * (C_Sr * glf_p + C_Sf * glr_m) * x[6];
        double s3 = mu / (x[3] * lrlf) * (C_Sf * glr_m) * x[2];
        f[6] = s1 - s2 + s3;
    }
}

/* pid, dynamic_models.py:178-221 (includes the v_min = 1e-8 braking quirk). */
OR_API void or_pid(double speed, double steer, double cur_speed, double cur_steer, double max_sv, double max_a,
                   double max_v, double min_v, double *out /* accl, sv */) {
    double steer_diff = steer - cur_steer;
    double sv = fabs(steer_diff) > 1e-4 ? (steer_diff / fabs(steer_diff)) * max_sv : 0.0;
    double vel_diff = speed - cur_speed;
    double kp, accl;
    if (cur_speed > 0.) {
        kp = vel_diff > 0 ? 10.0 * max_a / max_v : 10.0 * max_a / (-min_v);
    } else {
        kp = vel_diff > 0 ? 2.0 * max_a / max_v : 2.0 * max_a / (-min_v);
    }
    accl = kp * vel_diff;
    out[0] = accl;
    out[1] = sv;
}

static inline double or_clip(double a, double lo, double hi) { /* np.clip: NaN propagates */
    if (a != a) return a;
    return a < lo ? lo : (a > hi ? hi : a);
}

/* Python/NumPy float remainder (npy_divmod): sign follows the divisor, 0 -> +0. */
static inline double or_pymod(double a, double b) {
    double mod = fmod(a, b);
    if (mod != 0.0) {
        if ((b < 0) != (mod < 0)) mod += b;
    } else {
        mod = copysign(0.0, b);
    }
    return mod;
}

#define OR_SLIP_CAP 1.0471975511965976 /* np.deg2rad(60) */
#define OR_YAW_RATE_CAP 10.0

/* RaceCar.update_pose without the scan, base_classes.py:256-417.
 * state[7] = [x, y, steer, v, yaw, yaw_rate, slip]; buf[2] = [newest, older];
 * *cnt = steer-buffer fill (0..2).  integrator: 1 = RK4, 2 = Euler. */
OR_API void or_update_pose(double *state, double *buf, int32_t *cnt, double raw_steer, double vel,
                           const or_params *p, double dt, int integrator) {
    double steer = 0.0;
    if (*cnt < 2) { /* :272-274 */
        steer = 0.0;
        buf[1] = buf[0];
        buf[0] = raw_steer;
        *cnt += 1;
    } else { /* :275-278 */
        steer = buf[1];
        buf[1] = buf[0];
        buf[0] = raw_steer;
    }
    double pa[2];
    or_pid(vel, steer, state[3], state[2], p->sv_max, p->a_max, p->v_max, p->v_min, pa);
    double sv = or_clip(pa[1], p->sv_min, p->sv_max);
    double accl = or_clip(pa[0], -p->a_max, p->a_max);
    double u[2] = {sv, accl};
    double ns[7];
    if (integrator == 1) {
        double k1[7], k2[7], k3[7], k4[7], xs[7];
        or_vehicle_dynamics_st(state, u, p, k1);
        for (int i = 0; i < 7; ++i) xs[i] = state[i] + dt * (k1[i] / 2);
        or_vehicle_dynamics_st(xs, u, p, k2);
        for (int i = 0; i < 7; ++i) xs[i] = state[i] + dt * (k2[i] / 2);
        or_vehicle_dynamics_st(xs, u, p, k3);
        for (int i = 0; i < 7; ++i) xs[i] = state[i] + dt * k3[i];
        or_vehicle_dynamics_st(xs, u, p, k4);
        const double w = dt * (1.0 / 6.0);
        for (int i = 0; i < 7; ++i) ns[i] = state[i] + w * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
    } else {
        double f[7];
        or_vehicle_dynamics_st(state, u, p, f);
        for (int i = 0; i < 7; ++i) ns[i] = state[i] + dt * f[i];
    }
    ns[2] = or_clip(ns[2], p->s_min, p->s_max);
    ns[3] = or_clip(ns[3], p->v_min, p->v_max);
    ns[4] = or_pymod(ns[4] + M_PI, 2 * M_PI) - M_PI;
    double yr = ns[5];
    if (yr != yr) yr = 0.0;
    else if (isinf(yr)) yr = yr > 0 ? OR_YAW_RATE_CAP : -OR_YAW_RATE_CAP;
    ns[5] = or_clip(yr, -OR_YAW_RATE_CAP, OR_YAW_RATE_CAP);
    double sl = ns[6];
    if (sl != sl) sl = 0.0;
    ns[6] = or_clip(sl, -OR_SLIP_CAP, OR_SLIP_CAP);
    memcpy(state, ns, sizeof(ns));
}

/* ----------------------------------------------------------- collision --
 * check_ttc_jit, laser_models.py:188-217 */
OR_API int or_check_ttc(const double *scan, int nb, double vel, const double *cosines, const double *side,
                        double thresh) {
    if (vel != 0.0) {
        for (int i = 0; i < nb; ++i) {
            double proj_vel = vel * cosines[i];
            double ttc = (scan[i] - side[i]) / proj_vel;
            if (ttc < thresh && ttc >= 0.0) return 1;
        }
    }
    return 0;
}

/* get_trmtx + get_vertices, collision_models.py:218-260; out [rl, rr, fr, fl] x (x,y). */
OR_API void or_get_vertices(const double *pose, double length, double width, double *v) {
    double c = or_cos(pose[2]), s = or_sin(pose[2]);
    const double px[4] = {-length / 2, -length / 2, length / 2, length / 2};
    const double py[4] = {width / 2, -width / 2, -width / 2, width / 2};
    for (int k = 0; k < 4; ++k) {
        v[2 * k] = c * px[k] + ((-s) * py[k] + pose[0]);
        v[2 * k + 1] = s * px[k] + (c * py[k] + pose[1]);
    }
}

static inline double dot2(const double *a, const double *b) { return fma(a[1], b[1], a[0] * b[0]); }

/* indexOfFurthestPoint + support, collision_models.py:81-110 */
static void or_support(const double *v1, const double *v2, const double *d, double *out) {
    int i = 0, j = 0;
    double best = -INFINITY, best2 = -INFINITY;
    for (int k = 0; k < 4; ++k) {
        double pr = fma(v1[2 * k], d[0], v1[2 * k + 1] * d[1]);
        if (pr > best || k == 0) { best = pr; i = k; }
        double pr2 = fma(v2[2 * k], -d[0], v2[2 * k + 1] * -d[1]);
        if (pr2 > best2 || k == 0) { best2 = pr2; j = k; }
    }
    out[0] = v1[2 * i] - v2[2 * j];
    out[1] = v1[2 * i + 1] - v2[2 * j + 1];
}

static void triple(const double *a, const double *b, const double *c, double *out) {
    double ac = dot2(a, c), bc = dot2(b, c);
    out[0] = b[0] * ac - a[0] * bc;
    out[1] = b[1] * ac - a[1] * bc;
}

/* collision (GJK), collision_models.py:113-182 */
OR_API int or_collision(const double *v1, const double *v2) {
    double simplex[3][2];
    int index = 0;
    double p1[2] = {((v1[0] + v1[2]) + v1[4]) + v1[6], ((v1[1] + v1[3]) + v1[5]) + v1[7]};
    double p2[2] = {((v2[0] + v2[2]) + v2[4]) + v2[6], ((v2[1] + v2[3]) + v2[5]) + v2[7]};
    p1[0] /= 4; p1[1] /= 4; p2[0] /= 4; p2[1] /= 4;
    double d[2] = {p1[0] - p2[0], p1[1] - p2[1]};
    if (d[0] == 0 && d[1] == 0) d[0] = 1.0;
    double a[2];
    or_support(v1, v2, d, a);
    simplex[0][0] = a[0];
    simplex[0][1] = a[1];
    if (dot2(d, a) <= 0) return 0;
    d[0] = -a[0];
    d[1] = -a[1];
    int iter = 0;
    while (iter < 1000) {
        or_support(v1, v2, d, a);
        ++index;
        simplex[index][0] = a[0];
        simplex[index][1] = a[1];
        if (dot2(d, a) <= 0) return 0;
        double ao[2] = {-a[0], -a[1]};
        if (index < 2) {
            double ab[2] = {simplex[0][0] - a[0], simplex[0][1] - a[1]};
            triple(ab, ao, ab, d);
            if (sqrt(fma(d[1], d[1], d[0] * d[0])) < 1e-10) { /* perpendicular(ab) */
                d[0] = ab[1];
                d[1] = -1 * ab[0];
            }
            continue; /* note: iter_count is not incremented here (:160) */
        }
        double ab[2] = {simplex[1][0] - a[0], simplex[1][1] - a[1]};
        double ac[2] = {simplex[0][0] - a[0], simplex[0][1] - a[1]};
        double acperp[2];
        triple(ab, ac, ac, acperp);
        if (dot2(acperp, ao) >= 0) {
            d[0] = acperp[0];
            d[1] = acperp[1];
        } else {
            double abperp[2];
            triple(ac, ab, ab, abperp);
            if (dot2(abperp, ao) < 0) return 1;
            simplex[0][0] = simplex[1][0];
            simplex[0][1] = simplex[1][1];
            d[0] = abperp[0];
            d[1] = abperp[1];
        }
        simplex[1][0] = simplex[2][0];
        simplex[1][1] = simplex[2][1];
        --index;
        ++iter;
    }
    return 0;
}

/* collision_multiple, collision_models.py:184-212 */
OR_API void or_collision_multiple(const double *verts, int n, double *collisions, double *idx) {
    for (int i = 0; i < n; ++i) {
        collisions[i] = 0.0;
        idx[i] = -1.0;
    }
    for (int i = 0; i < n - 1; ++i)
        for (int j = i + 1; j < n; ++j)
            if (or_collision(verts + 8 * i, verts + 8 * j)) {
                collisions[i] = 1.;
                collisions[j] = 1.;
                idx[i] = j;
                idx[j] = i;
            }
}

/* get_range, laser_models.py:249-280 */
static double or_get_range(const double *pose, double beam_theta, const double *va, const double *vb) {
    double o[2] = {pose[0], pose[1]};
    double v1[2] = {o[0] - va[0], o[1] - va[1]};
    double v2[2] = {vb[0] - va[0], vb[1] - va[1]};
    double v3[2] = {or_cos(beam_theta + M_PI / 2.), or_sin(beam_theta + M_PI / 2.)};
    double denom = dot2(v2, v3);
    double distance = INFINITY;
    if (fabs(denom) > 0.0) {
        double d1 = (v2[0] * v1[1] - v2[1] * v1[0]) / denom;
        double d2 = dot2(v1, v3) / denom;
        if (d1 >= 0.0 && d2 >= 0.0 && d2 <= 1.0) distance = d1;
    } else {
        /* are_collinear(o, va, vb), :232-247 */
        double ba[2] = {va[0] - o[0], va[1] - o[1]};
        double ca[2] = {o[0] - vb[0], o[1] - vb[1]};
        if (fabs(ba[0] * ca[1] - ba[1] * ca[0]) < 1e-8) {
            double e[2] = {va[0] - o[0], va[1] - o[1]}, f2[2] = {vb[0] - o[0], vb[1] - o[1]};
            double da = sqrt(fma(e[1], e[1], e[0] * e[0]));
            double db = sqrt(fma(f2[1], f2[1], f2[0] * f2[0]));
            distance = da <= db ? da : db;
        }
    }
    return distance;
}

/* get_blocked_view_indices, laser_models.py:282-315 */
static void or_blocked(const double *pose, const double *v, const double *angles, int nb, int *lo, int *hi) {
    double ex = or_cos(pose[2]), ey = or_sin(pose[2]);
    int inds[4];
    for (int i = 0; i < 4; ++i) {
        double vx = v[2 * i] - pose[0], vy = v[2 * i + 1] - pose[1];
        double nrm = sqrt(vx * vx + vy * vy);
        double ux = vx / nrm, uy = vy / nrm;
        double angle = atan2(ey, ex) - atan2(uy, ux);
        if (angle > M_PI)
            angle = angle - 2 * M_PI;
        else if (angle < -M_PI)
            angle = angle + 2 * M_PI;
        double a = -angle;
        int best = 0;
        double bd = fabs(angles[0] - a);
        for (int k = 1; k < nb; ++k) {
            double dd = fabs(angles[k] - a);
            if (dd < bd) { bd = dd; best = k; }
        }
        inds[i] = best;
    }
    int mn = inds[0], mx = inds[0];
    for (int i = 1; i < 4; ++i) {
        if (inds[i] < mn) mn = inds[i];
        if (inds[i] > mx) mx = inds[i];
    }
    *lo = mn;
    *hi = mx;
}

/* ray_cast, laser_models.py:318-346 (scan modified in place). */
OR_API void or_ray_cast(const double *pose, double *scan, const double *angles, int nb, const double *v) {
    double lv[5][2];
    for (int k = 0; k < 4; ++k) { lv[k][0] = v[2 * k]; lv[k][1] = v[2 * k + 1]; }
    lv[4][0] = v[0];
    lv[4][1] = v[1];
    int lo, hi;
    or_blocked(pose, v, angles, nb, &lo, &hi);
    for (int i = lo; i <= hi; ++i)
        for (int j = 0; j < 4; ++j) {
            double r = or_get_range(pose, pose[2] + angles[i], lv[j], lv[j + 1]);
            if (r < scan[i]) scan[i] = r;
        }
}

/* ----------------------------------------------------------- simulator --
 * Simulator.step, base_classes.py:566-625, for n_envs independent
 * environments of A agents (noise-free: scan_rng = None).
 * state [E*A][7], buf [E*A][2], cnt [E*A], actions [E*A][2] (steer, vel),
 * scans [E*A][B], collisions [E*A] (0./1.). */
typedef struct {
    const or_scanner *sc;
    const or_params *p;
    const double *angles, *beam_cos, *side;
    double dt, lidar_dist, ttc_thresh;
    int32_t n_agents, integrator;
    /* scan noise (ScanSimulator2D.scan, laser_models.py:450-452): 0 = the
     * parity setting (scan_rng = None).  > 0 only for the bench's CPU
     * baseline, where the host does the per-step draw the reference does:
     * B normals per env per step, shared by the env's agents (all RaceCars
     * seed alike, base_classes.py:119,204).  The stream (splitmix64 +
     * Box-Muller) is not NumPy's PCG64; only the cost of the draw matters. */
    double noise_std;
    uint64_t noise_seed, step_no;
} or_sim;

static inline uint64_t or_splitmix(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void or_scan_noise(const or_sim *S, int64_t env, double *noise, int B) {
    /* Marsaglia's polar method: one log + one sqrt per pair of normals */
    uint64_t st = S->noise_seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(env + 1)) ^ (S->step_no << 20);
    for (int b = 0; b < B; b += 2) {
        double u, v, q;
        do {
            u = (double)(or_splitmix(&st) >> 11) * (2.0 / 9007199254740992.0) - 1.0;
            v = (double)(or_splitmix(&st) >> 11) * (2.0 / 9007199254740992.0) - 1.0;
            q = u * u + v * v;
        } while (q >= 1.0 || q == 0.0);
        const double f = S->noise_std * sqrt(-2.0 * log(q) / q);
        noise[b] = u * f;
        if (b + 1 < B) noise[b + 1] = v * f;
    }
}

static void or_sim_step_env(const or_sim *S, int64_t env, double *state, double *buf, int32_t *cnt,
                            const double *act, double *scans, double *collisions) {
    const int A = S->n_agents, B = S->sc->num_beams;
    double agent_poses[16][3];
    double verts[16][8] = {{0}};
    double noise[4096];
    const int noisy = S->noise_std > 0.0 && B <= 4096;
    if (noisy) or_scan_noise(S, env, noise, B);
    for (int i = 0; i < A; ++i) { /* :581-587 */
        double *st = state + 7 * i;
        or_update_pose(st, buf + 2 * i, cnt + i, act[2 * i], act[2 * i + 1], S->p, S->dt, S->integrator);
        double scan_pose[3] = {st[0] + S->lidar_dist * or_cos(st[4]), st[1] + S->lidar_dist * or_sin(st[4]), st[4]};
        or_get_scan(S->sc, scan_pose, scans + (size_t)i * B, NULL, NULL);
        if (noisy) /* after the clamp, laser_models.py:450-452 */
            for (int b = 0; b < B; ++b) scans[(size_t)i * B + b] += noise[b];
        agent_poses[i][0] = st[0];
        agent_poses[i][1] = st[1];
        agent_poses[i][2] = st[4];
    }
    for (int i = 0; i < A; ++i) { /* check_collision :549-563 */
        double pz[3] = {state[7 * i], state[7 * i + 1], state[7 * i + 4]};
        or_get_vertices(pz, S->p->length, S->p->width, verts[i]);
    }
    double idx[16];
    or_collision_multiple(&verts[0][0], A, collisions, idx);
    for (int i = 0; i < A; ++i) { /* :592-602 */
        double *st = state + 7 * i;
        double *scan = scans + (size_t)i * B;
        int hit = or_check_ttc(scan, B, st[3], S->beam_cos, S->side, S->ttc_thresh);
        if (hit)
            for (int k = 3; k < 7; ++k) st[k] = 0.;
        double own[3] = {st[0], st[1], st[4]};
        for (int j = 0; j < A; ++j) {
            if (j == i) continue;
            double ov[8];
            or_get_vertices(agent_poses[j], S->p->length, S->p->width, ov);
            or_ray_cast(own, scan, S->angles, B, ov);
        }
        if (hit) collisions[i] = 1.;
    }
}

OR_API void or_sim_step(const or_sim *S, int64_t n_envs, double *state, double *buf, int32_t *cnt,
                        const double *actions, double *scans, double *collisions, int threads) {
    const int64_t A = S->n_agents, B = S->sc->num_beams;
#pragma omp parallel for schedule(dynamic, 2) num_threads(threads > 0 ? threads : 1)
    for (int64_t e = 0; e < n_envs; ++e)
        or_sim_step_env(S, e, state + 7 * A * e, buf + 2 * A * e, cnt + A * e, actions + 2 * A * e,
                        scans + A * B * e, collisions + A * e);
}

/* RaceCar.reset, base_classes.py:183-204 */
OR_API void or_sim_reset(int64_t n, double *state, double *buf, int32_t *cnt, const double *poses) {
    for (int64_t i = 0; i < n; ++i) {
        for (int k = 0; k < 7; ++k) state[7 * i + k] = 0.0;
        state[7 * i + 0] = poses[3 * i];
        state[7 * i + 1] = poses[3 * i + 1];
        state[7 * i + 4] = poses[3 * i + 2];
        buf[2 * i] = buf[2 * i + 1] = 0.0;
        cnt[i] = 0;
    }
}

/* ---------------------------------------------------------------------------
 * Opponent policy of the training loop: gap_follow_action
 * (rl_training/utils/gap_follow.py:3-58, called by train_ddpg.py:168 on the
 * float32 info["scans"][1]).  float32 stages follow NumPy:
 *   preprocess_lidar  :3-12  window [max(0,i-2), min(N-1,i+2)] of
 *                     clip(r, 0, 3.0) (float32); np.mean = left-to-right
 *                     float32 sum / count in float32 (measured: identical on
 *                     200k windows of length 3..5)
 *   create_bubble     :14-19 argmin (first minimum; a NaN wins, first NaN),
 *                     zero [cp-30, cp+30] clipped to the scan
 *   find_max_gap      :21-39 runs of value > 0.5; the first run of maximal
 *                     end-start wins (Python max); none -> (0, N-1)
 *   best point        :41-42 (start+end)//2
 *   action            :44-58 steer = angle_min + best*angle_increment (f64),
 *                     speed 2.5 / 2 / 1.5 by |steer| < radians(10) / (20)
 * gap_out (optional) = the chosen (start, end). */
OR_API void or_gap_follow(const float *r, int32_t n, double angle_min, double angle_increment, double *action,
                          int32_t *gap_out) {
    float *p = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    for (int32_t i = 0; i < n; ++i) {
        int32_t s = i - 2 > 0 ? i - 2 : 0;
        int32_t e = i + 2 < n - 1 ? i + 2 : n - 1;
        float sum = 0.0f;
        for (int32_t j = s; j <= e; ++j) {
            float v = r[j];
            v = v < 0.0f ? 0.0f : v;   /* np.clip(x, 0, 3.0): NaN propagates */
            v = v > 3.0f ? 3.0f : v;
            sum = sum + v;
        }
        p[i] = sum / (float)(e - s + 1);
    }
    int32_t cp = 0;
    for (int32_t i = 0; i < n; ++i) {  /* np.argmin */
        if (p[i] != p[i]) { cp = i; break; }
        if (p[i] < p[cp]) cp = i;
    }
    int32_t bs = cp - 30 > 0 ? cp - 30 : 0;
    int32_t be = cp + 30 < n - 1 ? cp + 30 : n - 1;
    for (int32_t i = bs; i <= be; ++i) p[i] = 0.0f;
    int32_t g0 = 0, g1 = n - 1, best_len = -1, start = -1;
    for (int32_t i = 0; i <= n; ++i) {
        int m = i < n && p[i] > 0.5f;
        if (m && start < 0) start = i;
        else if (!m && start >= 0) {
            if (i - 1 - start > best_len) { best_len = i - 1 - start; g0 = start; g1 = i - 1; }
            start = -1;
        }
    }
    free(p);
    int32_t best = (g0 + g1) / 2;
    double steer = angle_min + (double)best * angle_increment;
    double a = fabs(steer);
    double speed = a < 10.0 * (M_PI / 180.0) ? 2.5 : (a < 20.0 * (M_PI / 180.0) ? 2.0 : 1.5);
    action[0] = steer;
    action[1] = speed;
    if (gap_out) { gap_out[0] = g0; gap_out[1] = g1; }
}
