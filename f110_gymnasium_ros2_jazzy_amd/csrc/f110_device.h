// f110_device.h — device (and host/device) building blocks of the gfx950 step.
//
// Semantics restate the reference hot path term by term (paths relative to
// f110_gymnasium/gym/f110_gym/envs/ of ahoop004/f110_gymnasium_ros2_jazzy).
// Compiled with -ffp-contract=off: every a*b+c below rounds twice, exactly as
// the Python/Numba source does.  Where the reference's NumPy calls reach BLAS
// (ndarray.dot, np.linalg.norm) the rounding pattern of the reference run is
// reproduced with explicit fma() (see DESIGN.md "Rounding contract").
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/f110.h"
#include "../../include/f110_debug.h"
#include "f110_sincos_table.h"

#define F110_HD __host__ __device__ __forceinline__
#define F110_D __device__ __forceinline__

namespace f110 {

constexpr double kPi = 3.141592653589793;      // np.pi
constexpr double kTwoPi = 6.283185307179586;   // 2 * np.pi
constexpr double kHalfPi = 1.5707963267948966; // np.pi / 2
constexpr double kSlipCap = 1.0471975511965976; // np.deg2rad(60)  (base_classes.py:414)
constexpr double kYawRateCap = 10.0;           // base_classes.py:410
constexpr double kG = 9.81;                    // dynamic_models.py:146
constexpr int kMaxAgents = 8;
constexpr int kMaxSeg = 80;

// ----------------------------------------------------------------- scalars --
F110_HD double clip(double a, double lo, double hi) {  // np.clip (NaN propagates)
    if (a != a) return a;
    return a < lo ? lo : (a > hi ? hi : a);
}

// Python / NumPy float remainder (npy_divmod): result takes the divisor's sign.
F110_HD double pymod(double a, double b) {
    double mod = fmod(a, b);
    if (mod != 0.0) {
        if ((b < 0) != (mod < 0)) mod += b;
    } else {
        mod = copysign(0.0, b);
    }
    return mod;
}

// pymod for 0 <= a < b (the yaw wraps' common case): a itself, +0 for a zero of either sign --
// what fmod and the sign fix-up give there -- without the library's fmod loop.
F110_HD double pymod_fast(double a, double b) {
    if (b > 0.0 && a >= 0.0 && a < b) return a == 0.0 ? 0.0 : a;
    return pymod(a, b);
}

// F110Env._wrap_angle / update_pose yaw wrap: ((a + pi) % 2pi) - pi.
F110_HD double wrap_angle(double a) { return pymod_fast(a + kPi, kTwoPi) - kPi; }

// ------------------------------------------------ correctly rounded sin/cos --
// The reference's np.sin / np.cos (and Numba's libm calls) are glibc's, which
// return the correctly rounded result but in very rare cases; ocml's differ by
// an ulp on a few percent of arguments, which is what left agent ray_cast
// ranges and box vertices inexact.  cr_sincos evaluates sin and cos of x in
// double-double arithmetic and rounds once: the Cody-Waite reduction by a
// three-part pi/2 (the first product exact by fma), then Taylor series of
// sin / cos on |r| <= pi/4 with the terms through r^7 (sin) / r^6 (cos) in
// double-double Horner steps and the rest in double.  The sum before the last
// rounding is within ~2^-70 relative, so the result is the correctly rounded
// value except where the true value lies within that of a rounding midpoint.
// Host and device compute it with the same IEEE operations (no contraction,
// explicit fma): tests/test_host_lib.py checks it against NumPy, equal except
// where glibc is itself one ulp off (< 0.3 % of the sampled arguments; there
// cr_sincos is the correctly rounded value).  That residue is pinned by the
// non-exact budgets (tests/golden/nonexact_beams.json), not by bit-equality.
// |x| >= 2^20 (never a scan or box angle here) falls back to the library call.
struct DD {
    double h, l;
};

F110_HD DD dd_two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}

F110_HD DD dd_fast(double a, double b) {  // |a| >= |b|
    const double s = a + b;
    return {s, b - (s - a)};
}

F110_HD DD dd_mul(DD a, DD b) {
    const double p = a.h * b.h;
    double e = fma(a.h, b.h, -p);
    e += a.h * b.l + a.l * b.h;
    return dd_fast(p, e);
}

F110_HD DD dd_add(DD a, DD b) {
    const DD s = dd_two_sum(a.h, b.h);
    return dd_fast(s.h, s.l + (a.l + b.l));
}

// acc = c + z * acc in double-double
F110_HD DD dd_horner(DD c, DD z, DD acc) { return dd_add(c, dd_mul(z, acc)); }

// x - k pi/2 as a double-double, k the nearest quadrant (|x| < 2^20, x != 0).
F110_HD DD sincos_reduce(double x, double &k) {
    const double P1 = 0x1.921fb54442d18p+0, P2 = 0x1.1a62633145c07p-54, P3 = -0x1.f1976b7ed8fbcp-110;
    k = rint(x * 0x1.45f306dc9c883p-1);  // x * 2/pi, nearest quadrant
    const double r1 = fma(-k, P1, x);    // exact: |x| >= pi/4 has ulp >= 2^-53
    const double q2 = k * P2;
    const double q2l = fma(k, P2, -q2);
    const DD s1 = dd_two_sum(r1, -q2);
    return dd_fast(s1.h, s1.l - q2l - k * P3);
}

// sin / cos of the reduced r by the double-double series (the slow, always
// certain path).
F110_HD void sincos_series(DD r, double &s, double &c) {
    const DD z = dd_mul(r, r);
    const double zh = z.h;
    // sin(r) = r (1 - z/3! + z^2/5! - z^3/7! + z^4 ps(z)),  ps = 1/9! - z/11! + ... - z^5/19!
    double ps = 0x1.952c77030ad4ap-49 - zh * 0x1.2f49b46814157p-57;  // 1/17! - z/19!
    ps = 0x1.ae7f3e733b81fp-41 - zh * ps;                             // 1/15!
    ps = 0x1.6124613a86d09p-33 - zh * ps;                             // 1/13!
    ps = 0x1.ae64567f544e4p-26 - zh * ps;                             // 1/11!
    ps = 0x1.71de3a556c734p-19 - zh * ps;                             // 1/9!
    DD as = {ps, 0.0};
    as = dd_horner({-0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73}, z, as);  // -1/7!
    as = dd_horner({0x1.1111111111111p-7, 0x1.1111111111111p-63}, z, as);    // 1/5!
    as = dd_horner({-0x1.5555555555555p-3, -0x1.5555555555555p-57}, z, as);  // -1/3!
    as = dd_horner({1.0, 0.0}, z, as);
    const DD sr = dd_mul(r, as);
    // cos(r) = 1 - z/2! + z^2/4! - z^3/6! + z^4 pc(z),  pc = 1/8! - z/10! + ... - z^5/18!
    double pc = 0x1.ae7f3e733b81fp-45 - zh * 0x1.6827863b97d97p-53;  // 1/16! - z/18!
    pc = 0x1.93974a8c07c9dp-37 - zh * pc;                            // 1/14!
    pc = 0x1.1eed8eff8d898p-29 - zh * pc;                            // 1/12!
    pc = 0x1.27e4fb7789f5cp-22 - zh * pc;                            // 1/10!
    pc = 0x1.a01a01a01a01ap-16 - zh * pc;                            // 1/8!
    DD ac = {pc, 0.0};
    ac = dd_horner({-0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65}, z, ac);  // -1/6!
    ac = dd_horner({0x1.5555555555555p-5, 0x1.5555555555555p-59}, z, ac);    // 1/4!
    ac = dd_horner({-0.5, 0.0}, z, ac);
    ac = dd_horner({1.0, 0.0}, z, ac);
    s = sr.h + sr.l;
    c = ac.h + ac.l;
}

// sin(i/64), cos(i/64) as double-doubles, i = 0..52 (scripts/gen_sincos_table.py).
constexpr double kSinCosTab[F110_SINCOS_TAB_N][4] = {F110_SINCOS_TAB_DATA};

// sin / cos of the reduced r by the table: a = |r| = i/64 + t, |t| <= 1/128,
// sin a = S cos t + C sin t, cos a = C cos t - S sin t with (S, C) the table's
// double-doubles and sin t / cos t short series in double with their leading
// products exact.  The sum before the last rounding is within ~2^-68 relative
// of sin a / cos a (the largest term is the rounding of t^3/6 against a result
// >= 1/128 for i >= 1; i = 0 is relative to t itself); a rounding that a 2^-64
// relative error could flip is not certain, and the caller then takes the
// series path (about 0.1 % of the values).  Where it returns true the result
// is the one sincos_series gives (both round the same certain value), which
// tests/test_host_lib.py checks over a few million arguments.
// The table path without a branch: returns whether the rounding is certain (s, c are then the
// correctly rounded values).  |r.h| >= 1 (not a reduced argument) reads entry 0 and returns garbage.
// The table path's double-double sin / cos of |r| (before the rounding) and their rounding bounds.
struct SinCosDD {
    double sh, sl, ch, cl;           // sin |r| = sh + sl, cos |r| = ch + cl (relative error < ~2^-68)
    double s_up, s_dn, c_up, c_dn;   // the roundings at +- the error bound: certain where equal
    bool neg;                        // r < 0
};

F110_HD SinCosDD sincos_table_core(DD r, const double (*tab)[4]) {
    const bool neg = r.h < 0.0;
    const double ah0 = fabs(r.h), al = neg ? -r.l : r.l;
    const double ah = ah0 < 1.0 ? ah0 : 0.0;  // (NaN too) keeps the index in the table
    const int i = (int)rint(ah * 64.0);
    const double *T = tab[i];
    const double th = ah - (double)i * 0.015625;  // exact (Sterbenz)
    const double tl = al;
    const double zh = th * th;
    const double zl = fma(th, th, -zh);
    // sin t = th + slo:  t - t^3/6 + t^5/120 - ...  with the t^2 tl / 2 cross term of t^3 / 6
    const double P = -0x1.5555555555555p-3 +
                     zh * (0x1.1111111111111p-7 + zh * (-0x1.a01a01a01a01ap-13 + zh * 0x1.71de3a556c734p-19));
    const double slo = tl + (th * (zh * P) - (0.5 * zh) * tl);
    // cos t = ch + cl:  1 - t^2/2 + t^4/24 - t^6/720 + t^8/40320
    const double Q = 0x1.5555555555555p-5 + zh * (-0x1.6c16c16c16c17p-10 + zh * 0x1.a01a01a01a01ap-16);
    const double hz = 0.5 * zh;
    const double ch = 1.0 - hz;
    const double cl = ((1.0 - ch) - hz) - ((0.5 * zl + th * tl) - (zh * zh) * Q);
    const double Sh = T[0], Sl = T[1], Ch = T[2], Cl = T[3];
    // sin a = Sh ch + Ch th + (Sh cl + Sl ch + Ch slo + Cl th)
    const double p1 = Sh * ch, e1 = fma(Sh, ch, -p1);
    const double p2 = Ch * th, e2 = fma(Ch, th, -p2);
    const DD sa = dd_two_sum(p1, p2);
    const double sl = sa.l + (e1 + e2) + (((Sh * cl + Sl * ch) + Cl * th) + Ch * slo);
    // cos a = Ch ch - Sh th + (Ch cl + Cl ch - Sh slo - Sl th)
    const double q1 = Ch * ch, f1 = fma(Ch, ch, -q1);
    const double q2 = -(Sh * th), f2 = fma(-Sh, th, -q2);
    const DD ca = dd_two_sum(q1, q2);
    const double cl2 = ca.l + (f1 + f2) + (((Ch * cl + Cl * ch) - Sl * th) - Sh * slo);
    const double es = fabs(sa.h) * 0x1p-64, ec = 0x1p-64;  // |cos a| > 0.7
    const double s_up = sa.h + (sl + es), s_dn = sa.h + (sl - es);
    const double c_up = ca.h + (cl2 + ec), c_dn = ca.h + (cl2 - ec);
    return {sa.h, sl, ca.h, cl2, s_up, s_dn, c_up, c_dn, neg};
}

F110_HD bool sincos_table_nb(DD r, double &s, double &c, const double (*tab)[4]) {
    const SinCosDD v = sincos_table_core(r, tab);
    s = v.neg ? -v.s_up : v.s_up;
    c = v.c_up;
    return (v.s_up == v.s_dn) & (v.c_up == v.c_dn);
}

F110_HD bool sincos_table(DD r, double &s, double &c, const double (*tab)[4] = kSinCosTab) {
    double s2, c2;
    if (!sincos_table_nb(r, s2, c2, tab)) return false;
    s = s2;
    c = c2;
    return true;
}

// cr_sincos's common case without a branch: the reduction, the table path and the quadrant as
// selects, +-0 included.  Returns false where cr_sincos takes another path (|x| >= 2^20, NaN, an
// uncertain rounding); where it returns true sn / cs are cr_sincos's values.  Straight-line code,
// so independent evaluations (and the arithmetic around them) can overlap; the caller runs
// cr_sincos itself on false, after the rest of its work.
F110_HD bool cr_sincos_fast(double x, double &sn, double &cs, const double (*tab)[4] = kSinCosTab) {
    const bool in = fabs(x) < 1048576.0;
    double k;
    const DD r = sincos_reduce(in ? x : 1.0, k);
    double s, c;
    const bool cert = sincos_table_nb(r, s, c, tab);
    const int q = (int)((int64_t)k & 3);
    const double a = q == 0 ? s : q == 1 ? c : q == 2 ? -s : -c;
    const double b = q == 0 ? c : q == 1 ? -s : q == 2 ? -c : s;
    const bool zero = x == 0.0;
    sn = zero ? x : a;
    cs = zero ? 1.0 : b;
    return zero | (cert & in);
}

// tan x and cos x from one table evaluation (the kinematic model's pair, vehicle_dynamics_st).
// cos: cr_sincos's value where ok_c.  tan: sin / cos in double-double, rounded once at a 2^-64
// relative bound -- the correctly rounded tan where ok_t (glibc's tan, which the reference's
// Numba code calls, is correctly rounded on all but ~0.4 % of arguments; the device library's
// differs more often).  Where a flag is false the caller takes cr_cos / the library tan.
F110_HD void tan_cos_fast(double x, const double (*tab)[4], double &t, double &c, bool &ok_t, bool &ok_c) {
    const bool in = fabs(x) < 1048576.0;
    double k;
    const DD r = sincos_reduce(in ? x : 1.0, k);
    const SinCosDD v = sincos_table_core(r, tab);
    const int q = (int)((int64_t)k & 3);
    const double s_r = v.neg ? -v.s_up : v.s_up, c_r = v.c_up;
    const bool s_ok = v.s_up == v.s_dn, c_ok = v.c_up == v.c_dn;
    const bool zero = x == 0.0;
    const double cq = q == 0 ? c_r : q == 1 ? -s_r : q == 2 ? -c_r : s_r;  // cos(r + q pi/2)
    c = zero ? 1.0 : cq;
    ok_c = zero | (in & ((q & 1) ? s_ok : c_ok));
    // tan(r + q pi/2) = sin r / cos r (q even), -cos r / sin r (q odd)
    // (the table path's low parts carry the t^3 / t^2 terms: up to ~2^-22 of the high parts, so both
    // are renormalised before the division, whose correction divides by the high part only)
    const DD Sn = dd_fast(v.neg ? -v.sh : v.sh, v.neg ? -v.sl : v.sl), Cn = dd_fast(v.ch, v.cl);
    const double nh = (q & 1) ? Cn.h : Sn.h, nl = (q & 1) ? Cn.l : Sn.l;
    const double dh = (q & 1) ? Sn.h : Cn.h, dl = (q & 1) ? Sn.l : Cn.l;
    const double q0 = nh / dh;
    const double rr = (fma(-q0, dh, nh) + nl) - q0 * dl;  // N - q0 D (the product's error exact)
#if defined(__HIP_DEVICE_COMPILE__)
    const double q1 = rr * __builtin_amdgcn_rcp(dh);  // a correction below an ulp of q0: a rough quotient
#else
    const double q1 = rr / dh;
#endif
    const double et = fabs(q0) * 0x1p-64;
    const double t_up = q0 + (q1 + et), t_dn = q0 + (q1 - et);
    t = zero ? x : ((q & 1) ? -t_up : t_up);
    ok_t = zero | (in & (t_up == t_dn) & (dh != 0.0));
}

// tab: kSinCosTab or a copy of it (k_agents reads an LDS copy: one short dependent load per call).
// The branch-free common case inline, the rest (library calls, the series) out of line: one copy
// of it per kernel instead of one per call site (k_agents' code is read once per wave from L2).
__host__ __device__ __attribute__((noinline)) inline void cr_sincos_slow(double x, double &sn, double &cs,
                                                                          const double (*tab)[4]);

F110_HD void cr_sincos(double x, double &sn, double &cs, const double (*tab)[4] = kSinCosTab) {
    if (!cr_sincos_fast(x, sn, cs, tab)) cr_sincos_slow(x, sn, cs, tab);
}

__host__ __device__ __attribute__((noinline)) inline void cr_sincos_slow(double x, double &sn, double &cs,
                                                                          const double (*tab)[4]) {
    if (!(fabs(x) < 1048576.0)) {  // NaN, inf, or beyond the exact reduction
        sn = sin(x);
        cs = cos(x);
        return;
    }
    if (x == 0.0) {  // +-0 (keeps the sign of sin(-0.0))
        sn = x;
        cs = 1.0;
        return;
    }
    double k, s, c;
    const DD r = sincos_reduce(x, k);
    if (!sincos_table(r, s, c, tab)) sincos_series(r, s, c);
    switch ((int)((int64_t)k & 3)) {
        case 0: sn = s; cs = c; break;
        case 1: sn = c; cs = -s; break;
        case 2: sn = -s; cs = -c; break;
        default: sn = -c; cs = s; break;
    }
}

// The series path alone (tests: the table path must give the same bits).
F110_HD void cr_sincos_series(double x, double &sn, double &cs) {
    if (!(fabs(x) < 1048576.0) || x == 0.0) {
        cr_sincos(x, sn, cs);
        return;
    }
    double k, s, c;
    sincos_series(sincos_reduce(x, k), s, c);
    switch ((int)((int64_t)k & 3)) {
        case 0: sn = s; cs = c; break;
        case 1: sn = c; cs = -s; break;
        case 2: sn = -s; cs = -c; break;
        default: sn = -c; cs = s; break;
    }
}

F110_HD double cr_sin(double x) {
    double s, c;
    cr_sincos(x, s, c);
    return s;
}

F110_HD double cr_cos(double x, const double (*tab)[4] = kSinCosTab) {
    double s, c;
    cr_sincos(x, s, c, tab);
    return c;
}

// ------------------------------------------------------------- dynamics --
// accl_constraints, dynamic_models.py:29-60
F110_HD double accl_constraints(double vel, double accl, double v_switch, double a_max, double v_min,
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

// steering_constraint, dynamic_models.py:62-87
F110_HD double steering_constraint(double sa, double sv, double s_min, double s_max, double sv_min,
                                   double sv_max) {
    if ((sa <= s_min && sv <= 0) || (sa >= s_max && sv >= 0))
        sv = 0.;
    else if (sv <= sv_min)
        sv = sv_min;
    else if (sv >= sv_max)
        sv = sv_max;
    return sv;
}

// vehicle_dynamics_ks, dynamic_models.py:90-121: the kinematic single-track
// right-hand side of x[5] = (x, y, steer, v, yaw) under the constrained input.
F110_HD void vehicle_dynamics_ks(const double x[5], double u0_in, double u1_in, const f110_params &p,
                                 double f[5]) {
    const double lwb = p.lf + p.lr;
    const double u0 = steering_constraint(x[2], u0_in, p.s_min, p.s_max, p.sv_min, p.sv_max);
    const double u1 = accl_constraints(x[3], u1_in, p.v_switch, p.a_max, p.v_min, p.v_max);
    double s4, c4;
    cr_sincos(x[4], s4, c4);
    f[0] = x[3] * c4;
    f[1] = x[3] * s4;
    f[2] = u0;
    f[3] = u1;
    double tn, c2;
    bool ok_t, ok_c;
    tan_cos_fast(x[2], kSinCosTab, tn, c2, ok_t, ok_c);
    if (!ok_t) tn = tan(x[2]);
    f[4] = x[3] / lwb * tn;
}

// vehicle_dynamics_st, dynamic_models.py:123-176 (KS branch :152-160 via
// vehicle_dynamics_ks :90-121).  Python's left-to-right order kept.  tn, c2: tan(x[2]) and
// cr_cos(x[2]), the kinematic model's (the caller may have them already, see update_pose_impl).
F110_HD void vehicle_dynamics_st_tc(const double x[7], double u0_in, double u1_in, const f110_params &p,
                                    double f[7], const double (*tab)[4], double tn, double c2) {
    const double mu = p.mu, C_Sf = p.C_Sf, C_Sr = p.C_Sr, lf = p.lf, lr = p.lr, h = p.h, m = p.m, I = p.I;
    double u0 = steering_constraint(x[2], u0_in, p.s_min, p.s_max, p.sv_min, p.sv_max);
    double u1 = accl_constraints(x[3], u1_in, p.v_switch, p.a_max, p.v_min, p.v_max);
    // Both models are evaluated for every car and the car's own is selected
    // (dynamic_models.py:263-283: the kinematic model below |v| = 0.5): the
    // transcendentals and divisions of the two are independent chains, so a
    // wave holding both kinds of car waits for the longer one instead of the
    // sum (this launch is latency-bound: one wave per SIMD).  f[0], f[1] take
    // one sincos of the car's own angle (the yaw, or yaw + slip).
    const bool kinematic = fabs(x[3]) < 0.5;
    const double ang = kinematic ? x[4] : x[6] + x[4];
    double sy, cy;
    const bool sc_ok = cr_sincos_fast(ang, sy, cy, tab);  // (cr_sincos below when not certain)
    // kinematic (vehicle_dynamics_ks re-applies the (idempotent) constraints to u)
    const double lwb = lf + lr;
    const double k0 = steering_constraint(x[2], u0, p.s_min, p.s_max, p.sv_min, p.sv_max);
    const double k1 = accl_constraints(x[3], u1, p.v_switch, p.a_max, p.v_min, p.v_max);
    const double kf4 = x[3] / lwb * tn;
    const double kf5 = u1 / lwb * tn + x[3] / (lwb * (c2 * c2)) * u0;
    // single track
    const double glr_m = kG * lr - u1 * h;
    const double glf_p = kG * lf + u1 * h;
    const double lrlf = lr + lf;
    const double t1 = -mu * m / (x[3] * I * lrlf) * (lf * lf * C_Sf * glr_m + lr * lr * C_Sr * glf_p) * x[5];
    const double t2 = mu * m / (I * lrlf) * (lr * C_Sr * glf_p - lf * C_Sf * glr_m) * x[6];
    const double t3 = mu * m / (I * lrlf) * lf * C_Sf * glr_m * x[2];
    const double s1 = (mu / (x[3] * x[3] * lrlf) * (C_Sr * glf_p * lr - C_Sf * glr_m * lf) - 1) * x[5];
    const double s2 = mu / (x[3] * lrlf) * (C_Sr * glf_p + C_Sf * glr_m) * x[6];
    const double s3 = mu / (x[3] * lrlf) * (C_Sf * glr_m) * x[2];
    if (!sc_ok) cr_sincos(ang, sy, cy, tab);  // rare: after the independent work above
    f[0] = x[3] * cy;
    f[1] = x[3] * sy;
    f[2] = kinematic ? k0 : u0;
    f[3] = kinematic ? k1 : u1;
    f[4] = kinematic ? kf4 : x[5];
    f[5] = kinematic ? kf5 : t1 + t2 + t3;
    f[6] = kinematic ? 0.0 : s1 - s2 + s3;
}

F110_HD void vehicle_dynamics_st(const double x[7], double u0_in, double u1_in, const f110_params &p,
                                 double f[7], const double (*tab)[4] = kSinCosTab) {
    double tn, c2;
    bool ok_t, ok_c;
    tan_cos_fast(x[2], tab, tn, c2, ok_t, ok_c);
    if (!ok_t) tn = tan(x[2]);
    if (!ok_c) c2 = cr_cos(x[2], tab);
    vehicle_dynamics_st_tc(x, u0_in, u1_in, p, f, tab, tn, c2);
}

// The steering angle and speed of RK4's four stages (xs[2], xs[3] of update_pose_impl) depend
// only on themselves: f[2] and f[3] are the constrained inputs, and the model choice |v| < 0.5
// reads the speed.  Their chains are a few compares and products, so they run first, and the
// kinematic model's tan / cos of the four steering angles -- a stage's largest independent work --
// are issued together (k_agents is one wave per SIMD: issue- and latency-bound) instead of one
// pair per stage.  Same operations as vehicle_dynamics_st's, so the same values.
F110_HD void steer_stage_trig(double s2, double s3, double sv, double accl, const f110_params &p, double dt,
                              const double (*tab)[4], double tn[4], double c2[4]) {
    double x2[4], x3[4];
    x2[0] = s2;
    x3[0] = s3;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const double u0 = steering_constraint(x2[j], sv, p.s_min, p.s_max, p.sv_min, p.sv_max);
        const double u1 = accl_constraints(x3[j], accl, p.v_switch, p.a_max, p.v_min, p.v_max);
        const bool kinematic = fabs(x3[j]) < 0.5;
        const double k0 = steering_constraint(x2[j], u0, p.s_min, p.s_max, p.sv_min, p.sv_max);
        const double k1 = accl_constraints(x3[j], u1, p.v_switch, p.a_max, p.v_min, p.v_max);
        const double f2 = kinematic ? k0 : u0, f3 = kinematic ? k1 : u1;
        x2[j + 1] = j < 2 ? s2 + dt * (f2 / 2) : s2 + dt * f2;  // the stages' xs = s + dt k/2, s + dt k
        x3[j + 1] = j < 2 ? s3 + dt * (f3 / 2) : s3 + dt * f3;
    }
    bool okt[4], okc[4], ok = true;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // the four (tan, cos) as one straight-line block
        tan_cos_fast(x2[j], tab, tn[j], c2[j], okt[j], okc[j]);
        ok = ok & okt[j] & okc[j];
    }
    if (!ok) {  // rare: an uncertain rounding
#pragma unroll 1
        for (int j = 0; j < 4; ++j) {
            if (!okt[j]) tn[j] = tan(x2[j]);
            if (!okc[j]) c2[j] = cr_cos(x2[j], tab);
        }
    }
}

// pid, dynamic_models.py:178-221 (v_min = 1e-8 braking quirk included).
F110_HD void pid(double speed, double steer, double cur_speed, double cur_steer, double max_sv, double max_a,
                 double max_v, double min_v, double &accl, double &sv) {
    double steer_diff = steer - cur_steer;
    sv = fabs(steer_diff) > 1e-4 ? (steer_diff / fabs(steer_diff)) * max_sv : 0.0;
    double vel_diff = speed - cur_speed;
    double kp;
    if (cur_speed > 0.)
        kp = vel_diff > 0 ? 10.0 * max_a / max_v : 10.0 * max_a / (-min_v);
    else
        kp = vel_diff > 0 ? 2.0 * max_a / max_v : 2.0 * max_a / (-min_v);
    accl = kp * vel_diff;
}

// RaceCar.update_pose without the scan, base_classes.py:256-417.
// s[7] in/out; b0 = newest buffered steer, b1 = older; cnt = buffer fill.
// RaceCar.update_pose on a state array s (and an accumulator scratch acc) that
// are plain arrays (registers) or volatile LDS arrays (k_step1: every stage
// re-reads s and acc from LDS, so that only one vehicle_dynamics_st evaluation
// is in registers at a time).  Same operations in the same order either way.
template <class V>
F110_HD void update_pose_impl(V s, V acc, double &b0, double &b1, int &cnt, double raw_steer, double vel,
                              const f110_params &p, double dt, int integrator, const double (*tab)[4] = kSinCosTab) {
    double steer;
    if (cnt < 2) {  // :272-274
        steer = 0.0;
        b1 = b0;
        b0 = raw_steer;
        cnt += 1;
    } else {        // :275-278
        steer = b1;
        b1 = b0;
        b0 = raw_steer;
    }
    double accl, sv;
    pid(vel, steer, s[3], s[2], p.sv_max, p.a_max, p.v_max, p.v_min, accl, sv);
    sv = clip(sv, p.sv_min, p.sv_max);
    accl = clip(accl, -p.a_max, p.a_max);
    double k[7], xs[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) xs[i] = s[i];
    if (integrator == F110_INTEGRATOR_RK4) {  // :285-374
        // k1 + 2*k2 + 2*k3 + k4 is summed left to right as the stages come
        // (((k1 + 2k2) + 2k3) + k4: the reference's rounding order), so only
        // one stage's k is live at a time
        double tn[4], c2[4];
        steer_stage_trig(s[2], s[3], sv, accl, p, dt, tab, tn, c2);
        // the four stages as one loop body (one copy of the model's code: k_agents' instructions are
        // read from L2 once per wave), the same operations in the same order as written out
#pragma unroll 1
        for (int st = 0; st < 4; ++st) {
            const double tns = st == 0 ? tn[0] : st == 1 ? tn[1] : st == 2 ? tn[2] : tn[3];
            const double c2s = st == 0 ? c2[0] : st == 1 ? c2[1] : st == 2 ? c2[2] : c2[3];
            vehicle_dynamics_st_tc(xs, sv, accl, p, k, tab, tns, c2s);
            if (st == 3) break;
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                acc[i] = st == 0 ? k[i] : acc[i] + 2 * k[i];
                xs[i] = st < 2 ? s[i] + dt * (k[i] / 2) : s[i] + dt * k[i];
            }
        }
        const double w = dt * (1.0 / 6.0);
#pragma unroll
        for (int i = 0; i < 7; ++i) s[i] = s[i] + w * (acc[i] + k[i]);
    } else {                                  // :376-396
        vehicle_dynamics_st(xs, sv, accl, p, k, tab);
#pragma unroll
        for (int i = 0; i < 7; ++i) s[i] = s[i] + dt * k[i];
    }
    s[2] = clip(s[2], p.s_min, p.s_max);   // :400-401
    s[3] = clip(s[3], p.v_min, p.v_max);
    s[4] = wrap_angle(s[4]);               // :408
    double yr = s[5];                      // :410-412
    if (yr != yr) yr = 0.0;
    else if (isinf(yr)) yr = yr > 0 ? kYawRateCap : -kYawRateCap;
    s[5] = clip(yr, -kYawRateCap, kYawRateCap);
    double sl = s[6];                      // :414-417
    if (sl != sl) sl = 0.0;
    s[6] = clip(sl, -kSlipCap, kSlipCap);
}

F110_HD void update_pose(double s[7], double &b0, double &b1, int &cnt, double raw_steer, double vel,
                         const f110_params &p, double dt, int integrator, const double (*tab)[4] = kSinCosTab) {
    double acc[7];
    update_pose_impl<double *>(s, acc, b0, b1, cnt, raw_steer, vel, p, dt, integrator, tab);
}

// -------------------------------------------------------------- the map --
struct MapView {
    const double *dt;  // [H*W] metres (res * EDT), row-major
    int32_t H, W;
    int64_t n;         // H*W
    double res, ox, oy, oc, os;
    double wres, hres; // width*resolution, height*resolution (laser_models.py:79)
    double inv_res;    // fl(1 / res), for the guarded fast quotient below
};

// xy_2_rc + distance_transform, laser_models.py:55-104: the linear EDT index
// a lookup at (x, y) reads.  Out-of-map (r,c) = (-1,-1) reads dt[-1,-1].
F110_HD int64_t cell_index(const MapView &m, double x, double y) {
    double xt = x - m.ox;
    double yt = y - m.oy;
    double xr = xt * m.oc + yt * m.os;
    double yr = -xt * m.os + yt * m.oc;
    if (xr < 0 || xr >= m.wres || yr < 0 || yr >= m.hres || xr != xr || yr != yr) return m.n - 1;
    int c = (int)(xr / m.res);
    int r = (int)(yr / m.res);
    int64_t lin = (int64_t)r * m.W + c;
    return lin < m.n ? lin : m.n - 1;
}

// int(v / res) for 0 <= v < W*res without the fp64 divide on the common
// path.  fl(v * fl(1/res)) and fl(v / res) are both within 2^-52 relative of
// the exact quotient (< 1e-12 absolute for v/res < 4096), so their integer
// parts agree unless the quotient lies within that distance of an integer;
// inside a 1e-9 guard band the IEEE division decides (bit-exact with
// xy_2_rc's int(x_rot/resolution), laser_models.py:83-84).
F110_HD int trunc_div(double v, double res, double inv_res) {
    double q = v * inv_res;
    int k = (int)q;
    double f = q - (double)k;
    if (f < 1e-9 || f > 1.0 - 1e-9) k = (int)(v / res);
    return k;
}

F110_HD int64_t cell_index_fast(const MapView &m, double x, double y) {
    double xt = x - m.ox;
    double yt = y - m.oy;
    double xr = xt * m.oc + yt * m.os;
    double yr = -xt * m.os + yt * m.oc;
    if (xr < 0 || xr >= m.wres || yr < 0 || yr >= m.hres || xr != xr || yr != yr) return m.n - 1;
    int c = trunc_div(xr, m.res, m.inv_res);
    int r = trunc_div(yr, m.res, m.inv_res);
    int64_t lin = (int64_t)r * m.W + c;
    return lin < m.n ? lin : m.n - 1;
}

// The EDT in 4x4-cell tiles (16 f64 = one 128-B cache line): the 64 lanes of
// a wave trace 64 neighbouring beams whose samples form a short arc of cells
// in ANY direction; square tiles bound the cache lines that arc touches,
// where row-major lines are 16 x 1 cells and an arc along a column touches
// one line per cell.
struct TiledMapView {
    const double *dt;  // [(Hp/4)*(Wp/4)][16], Hp/Wp = H/W rounded up to 4
    int32_t H, W, wt;  // wt = Wp / 4 tiles per tile-row
    int32_t oob;       // tiled index of dt[H-1][W-1] (the reference's dt[-1,-1])
    double res, inv_res, ox, oy, oc, os, wres, hres;
};

// Cells are column-major inside a tile: index = tile * 16 + (c & 3) * 4 +
// (r & 3), so (c >> 2) * 16 + (c & 3) * 4 == c * 4 and the index is
// (r >> 2) * wt * 16 + c * 4 + (r & 3) -- one multiply-add (k_rays_fx).
F110_HD int32_t tiled_index(int32_t wt, int32_t r, int32_t c) {
    return (r >> 2) * wt * 16 + c * 4 + (r & 3);
}

// xy_2_rc + distance_transform (laser_models.py:55-104) on the tiled EDT.
// ROT = false when the map's origin yaw is exactly 0 (cos = 1, sin = 0): then
// x_rot = x_trans*1 + y_trans*0 == x_trans for every finite input (a NaN or
// inf input still lands off-map), so the rotation is skipped bit-exactly.
template <bool ROT>
F110_HD int32_t tiled_cell(const TiledMapView &m, double x, double y) {
    double xr = x - m.ox;
    double yr = y - m.oy;
    if (ROT) {
        const double xt = xr, yt = yr;
        xr = xt * m.oc + yt * m.os;
        yr = -xt * m.os + yt * m.oc;
    }
    const bool inb = (xr >= 0) & (xr < m.wres) & (yr >= 0) & (yr < m.hres);  // false for NaN
    const double qx = xr * m.inv_res, qy = yr * m.inv_res;
#if defined(__HIP_DEVICE_COMPILE__)
    const double fx = __builtin_amdgcn_fract(qx), fy = __builtin_amdgcn_fract(qy);
#else
    const double fx = qx - floor(qx), fy = qy - floor(qy);
#endif
    // the conversions see in-range values only (a NaN or out-of-range double -> int is UB;
    // off-map results are discarded below)
    int32_t c = (int32_t)(inb ? qx : 0.0), r = (int32_t)(inb ? qy : 0.0);
    // guard band (see trunc_div): near an integer the IEEE quotient decides
    const double band = fmax(fabs(fx - 0.5), fabs(fy - 0.5));
    if (inb && band > 0.5 - 1e-9) {
        c = (int32_t)(xr / m.res);
        r = (int32_t)(yr / m.res);
        // x_rot < W*res and y_rot < H*res, yet the rounded quotient can reach W
        // (or H) exactly.  Same cell as cell_index's flat row-major read:
        // dt[r, W] is dt[r+1, 0]; anything past the last cell is dt[-1, -1].
        if (c >= m.W) {
            c = 0;
            ++r;
        }
        if (r >= m.H) return m.oob;
    }
    return inb ? tiled_index(m.wt, r, c) : m.oob;
}

// The ray loop's form of tiled_cell (same cell, bit for bit): the tile index
// in 24-bit multiplies, the IEEE-divide fallback behind a wave-uniform
// branch (taken only when some lane sits within 1e-9 of a cell edge, so the
// common iteration carries no exec-mask juggling), and the EDT read as a
// 32-bit byte offset from the table base (SGPR-base global load).
__device__ __forceinline__ uint32_t tiled_index_u24(int32_t wt, int32_t r, int32_t c) {
    return __umul24((uint32_t)r >> 2, (uint32_t)wt << 4) + (((uint32_t)c << 2) | ((uint32_t)r & 3u));
}

// the same cell as a byte offset into the f64 table
__device__ __forceinline__ uint32_t tiled_offset_u24(int32_t wt, int32_t r, int32_t c) {
    return (__umul24((uint32_t)r >> 2, (uint32_t)wt) << 7) + (((uint32_t)c << 5) | (((uint32_t)r & 3u) << 3));
}

// oob8: the byte offset of m.oob (m.oob << 3), passed by the caller so that a
// loop can keep it in a VGPR (the select below cannot read it from an SGPR
// next to its VCC condition)
template <bool ROT>
__device__ __forceinline__ double tiled_lookup(const TiledMapView &m, double x, double y, uint32_t oob8) {
    double xr = x - m.ox;
    double yr = y - m.oy;
    if (ROT) {
        const double xt = xr, yt = yr;
        xr = xt * m.oc + yt * m.os;
        yr = -xt * m.os + yt * m.oc;
    }
    const bool inb = (xr >= 0) & (xr < m.wres) & (yr >= 0) & (yr < m.hres);  // false for NaN
    const double qx = xr * m.inv_res, qy = yr * m.inv_res;
#if defined(__HIP_DEVICE_COMPILE__)
    const double fx = __builtin_amdgcn_fract(qx), fy = __builtin_amdgcn_fract(qy);
#else
    const double fx = qx - floor(qx), fy = qy - floor(qy);
#endif
    const double band = fmax(fabs(fx - 0.5), fabs(fy - 0.5));
    const bool near = band > 0.5 - 1e-9;  // the guard band of trunc_div (off-map lanes filtered inside)
    // off-map lanes convert 0 (a NaN or out-of-range double -> int is UB); their offset is masked below
    const uint32_t fast = tiled_offset_u24(m.wt, (int32_t)(inb ? qy : 0.0), (int32_t)(inb ? qx : 0.0));
    const uint32_t sel = 0u - (uint32_t)inb;  // branchless select: no exec-mask split per iteration
    uint32_t off = (fast & sel) | (oob8 & ~sel);
#if defined(__HIP_DEVICE_COMPILE__)
    // wave-uniform, rare; the ballot of a bare compare is its lane mask (no
    // VGPR round trip, as a ballot of (inb && near) would need)
    if (__builtin_amdgcn_ballot_w64(near))
#endif
    {
        if (near && inb) {
            int32_t c = (int32_t)(xr / m.res);
            int32_t r = (int32_t)(yr / m.res);
            if (c >= m.W) {  // see tiled_cell
                c = 0;
                ++r;
            }
            off = r >= m.H ? oob8 : tiled_offset_u24(m.wt, r, c);
        }
    }
    return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(m.dt) + off);
}

// ------------------------------------------------------ beam index runs --
// get_scan's beam index (laser_models.py:167-184) is a SEQUENTIAL float
// accumulation t_{i+1} = wrap(fl(t_i + inc)).  Inside one binade [2^(e-1), 2^e)
// every t_i is a multiple of u = ulp and fl(t_i + inc) = t_i + RN_u(inc), so the
// sequence is an exact arithmetic progression until it leaves the binade or
// wraps.  A run {start, count, t0, delta} holds t_{start+k} = t0 + k*delta
// (exact in fp64).  Ties (inc exactly half-way on the u grid) round to even:
// once t/u is even the increment is constant again, so an odd start is one
// single step.  t = 0 and t below kRunTMin (where the ulp grid and the tie
// test's half-ulp reach the subnormals) are single-beam runs.  Runs per scan:
// at most two per binade the indices pass through (a tie's odd start), over
// the binades from inc to theta_dis (twice: before and after the one wrap of
// fov < 2*pi), plus the wrapped start's own binade: max_beam_runs() bounds it
// and f110_create rejects a scan configuration whose bound exceeds kMaxSeg.
struct BeamRun {
    int32_t start, count;
    double t0, delta;
};

F110_HD double first_theta_index(double yaw, double fov, int theta_dis) {
    const double td = (double)theta_dis;
    double t = td * (yaw - fov / 2.) / (2. * kPi);  // :167
    t = fmod(t, td);                                // :170
    while (t < 0) t += td;                          // :171-172
    return t;
}

constexpr double kRunTMin = 0x1p-960;

// Upper bound of build_beam_runs' count for any yaw: per part (before and after the wrap)
// two runs per binade from the one holding inc up to theta_dis, one for a start below inc
// and one at the wrap.
inline int max_beam_runs(double inc, int theta_dis) {
    int e_inc, e_td;
    frexp(inc, &e_inc);
    frexp((double)theta_dis, &e_td);
    const int binades = e_td - e_inc + 1;
    return 2 * (2 * binades + 2);
}

// Returns the number of runs written, or -1 if max_runs is too small.
F110_HD int build_beam_runs(double t, double inc, int theta_dis, int B, BeamRun *runs, int max_runs) {
    const double td = (double)theta_dis;
    int i = 0, n = 0;
    while (i < B) {
        if (n >= max_runs) return -1;
        int run = 1;
        double delta = 0.0;
        if (t >= kRunTMin && t < td) {
            int e;
            frexp(t, &e);  // t in [2^(e-1), 2^e)
            double lim = ldexp(1.0, e);
            if (lim > td) lim = td;
            double v = t + inc;
            if (v < lim) {
                delta = v - t;               // exact (same binade)
                double rem = inc - delta;    // exact (|rem| <= u/2, u >= 2^-52)
                double half_u = ldexp(1.0, e - 54);
                bool tie = fabs(rem) == half_u;
                bool even = (((int64_t)ldexp(t, 53 - e)) & 1) == 0;  // t/u (an integer < 2^53) even
                if (!tie || even) {
                    int64_t span_u = (int64_t)ldexp(lim - t, 53 - e);
                    int64_t d_u = (int64_t)ldexp(delta, 53 - e);
                    // kmax = (span_u - 1) / d_u without a 64-bit integer divide:
                    // both < 2^53, the fp64 quotient is within 1 of it, fixed up exactly
                    int64_t kmax = (int64_t)((double)(span_u - 1) / (double)d_u);
                    if (kmax * d_u > span_u - 1) --kmax;
                    else if ((kmax + 1) * d_u <= span_u - 1) ++kmax;
                    int64_t left = (int64_t)(B - i - 1);
                    run = 1 + (int)(kmax < left ? kmax : left);
                }
            }
        }
        runs[n].start = i;
        runs[n].count = run;
        runs[n].t0 = t;
        runs[n].delta = delta;
        ++n;
        double last = t + (double)(run - 1) * delta;
        i += run;
        t = last + inc;               // :180
        while (t >= td) t -= td;      // :183-184
    }
    return n;
}

// build_beam_runs with the same runs (start, count, t0, delta) and a shorter
// dependent chain per run, for k_agents (one thread per car, latency-bound):
// the exponent and the tie test from the bits of t, and the run length
// kmax = max{k : t + k delta < lim} from an approximate quotient fixed up by
// exact sign tests (fma(k, delta, -span) rounds once, so its sign is the exact
// one), instead of 64-bit integer conversions and an IEEE division.  The
// multiples t + k delta (k <= kmax) all lie in t's binade on its ulp grid, as
// in build_beam_runs.  tests/test_host_lib.py checks the two against each
// other over yaws and scan configurations.
F110_HD int build_beam_runs_fast(double t, double inc, int theta_dis, int B, BeamRun *runs, int max_runs) {
    const double td = (double)theta_dis;
    int i = 0, n = 0;
    while (i < B) {
        if (n >= max_runs) return -1;
        int run = 1;
        double delta = 0.0;
        if (t >= kRunTMin && t < td) {
            int e;
            frexp(t, &e);  // t in [2^(e-1), 2^e)
            double lim = ldexp(1.0, e);
            if (lim > td) lim = td;
            const double v = t + inc;
            if (v < lim) {
                delta = v - t;                // exact (same binade)
                const double rem = inc - delta;
                const bool tie = fabs(rem) == ldexp(1.0, e - 54);
                const uint64_t tb = __builtin_bit_cast(uint64_t, t);
                if (!tie || (tb & 1u) == 0) {  // t's last mantissa bit (t normal): even
                    const double span = lim - t;  // exact
#if defined(__HIP_DEVICE_COMPILE__)
                    const double qa = span * __builtin_amdgcn_rcp(delta);
#else
                    const double qa = span / delta;
#endif
                    // (int)qa is kmax - 1, kmax or kmax + 1 (qa within 2^-20 relative of q); a
                    // quotient beyond 2^30 (> B) is clamped there, where kmax > B - i - 1 anyway:
                    // one exact test each way, branch-free
                    int k = (int)(qa < 0x1p30 ? qa : 0x1p30);
                    k -= fma((double)k, delta, -span) >= 0.0 ? 1 : 0;
                    k += fma((double)(k + 1), delta, -span) < 0.0 ? 1 : 0;
                    const int left = B - i - 1;
                    run = 1 + (k < left ? k : left);
                }
            }
        }
        runs[n].start = i;
        runs[n].count = run;
        runs[n].t0 = t;
        runs[n].delta = delta;
        ++n;
        double last = t + (double)(run - 1) * delta;
        i += run;
        t = last + inc;               // :180
        while (t >= td) t -= td;      // :183-184
    }
    return n;
}

// theta index (as get_scan would have it) of beam b, given its runs.
F110_HD double beam_theta_index(const BeamRun *runs, int n, int b) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {  // last run with start <= b
        int mid = (lo + hi + 1) >> 1;
        if (runs[mid].start <= b) lo = mid; else hi = mid - 1;
    }
    return runs[lo].t0 + (double)(b - runs[lo].start) * runs[lo].delta;
}

// ------------------------------------------------------------- geometry --
F110_HD double dot2(double a0, double a1, double b0, double b1) {  // ndarray.dot of 2-vectors (BLAS)
    return fma(a1, b1, a0 * b0);
}

// get_trmtx + get_vertices, collision_models.py:218-260 -> [rl, rr, fr, fl].
F110_HD void get_vertices(double x, double y, double th, double length, double width, double v[8]) {
    double s, c;
    cr_sincos(th, s, c);
    const double px[4] = {-length / 2, -length / 2, length / 2, length / 2};
    const double py[4] = {width / 2, -width / 2, -width / 2, width / 2};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[2 * k] = c * px[k] + ((-s) * py[k] + x);
        v[2 * k + 1] = s * px[k] + (c * py[k] + y);
    }
}

// indexOfFurthestPoint + support, collision_models.py:81-110
F110_HD void gjk_support(const double *v1, const double *v2, double d0, double d1, double &o0, double &o1) {
    int i = 0, j = 0;
    double b1 = 0, b2 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double p1 = fma(v1[2 * k], d0, v1[2 * k + 1] * d1);
        double p2 = fma(v2[2 * k], -d0, v2[2 * k + 1] * -d1);
        if (k == 0 || p1 > b1) { b1 = p1; i = k; }
        if (k == 0 || p2 > b2) { b2 = p2; j = k; }
    }
    o0 = v1[2 * i] - v2[2 * j];
    o1 = v1[2 * i + 1] - v2[2 * j + 1];
}

F110_HD void triple(double a0, double a1, double b0, double b1, double c0, double c1, double &o0, double &o1) {
    double ac = dot2(a0, a1, c0, c1), bc = dot2(b0, b1, c0, c1);  // tripleProduct :52-64
    o0 = b0 * ac - a0 * bc;
    o1 = b1 * ac - a1 * bc;
}

// collision (2-D GJK), collision_models.py:113-182
F110_HD bool gjk_collision(const double *v1, const double *v2) {
    double sx[3], sy[3];
    int index = 0;
    double p10 = (((v1[0] + v1[2]) + v1[4]) + v1[6]) / 4, p11 = (((v1[1] + v1[3]) + v1[5]) + v1[7]) / 4;
    double p20 = (((v2[0] + v2[2]) + v2[4]) + v2[6]) / 4, p21 = (((v2[1] + v2[3]) + v2[5]) + v2[7]) / 4;
    double d0 = p10 - p20, d1 = p11 - p21;
    if (d0 == 0 && d1 == 0) d0 = 1.0;
    double a0, a1;
    gjk_support(v1, v2, d0, d1, a0, a1);
    sx[0] = a0;
    sy[0] = a1;
    if (dot2(d0, d1, a0, a1) <= 0) return false;
    d0 = -a0;
    d1 = -a1;
    int iter = 0;
    while (iter < 1000) {
        gjk_support(v1, v2, d0, d1, a0, a1);
        ++index;
        sx[index] = a0;
        sy[index] = a1;
        if (dot2(d0, d1, a0, a1) <= 0) return false;
        double ao0 = -a0, ao1 = -a1;
        if (index < 2) {
            double ab0 = sx[0] - a0, ab1 = sy[0] - a1;
            triple(ab0, ab1, ao0, ao1, ab0, ab1, d0, d1);
            if (sqrt(fma(d1, d1, d0 * d0)) < 1e-10) {  // perpendicular(ab)
                d0 = ab1;
                d1 = -1 * ab0;
            }
            continue;
        }
        double ab0 = sx[1] - a0, ab1 = sy[1] - a1;
        double ac0 = sx[0] - a0, ac1 = sy[0] - a1;
        double q0, q1;
        triple(ab0, ab1, ac0, ac1, ac0, ac1, q0, q1);  // acperp
        if (dot2(q0, q1, ao0, ao1) >= 0) {
            d0 = q0;
            d1 = q1;
        } else {
            triple(ac0, ac1, ab0, ab1, ab0, ab1, q0, q1);  // abperp
            if (dot2(q0, q1, ao0, ao1) < 0) return true;
            sx[0] = sx[1];
            sy[0] = sy[1];
            d0 = q0;
            d1 = q1;
        }
        sx[1] = sx[2];
        sy[1] = sy[2];
        --index;
        ++iter;
    }
    return false;
}

// RaceCar.scan_angles[k] (base_classes.py:122-126), the value f110_host_tables
// stores: computed instead of loaded (same operations, no contraction)
F110_HD double beam_angle(int k, double fov, double incr) { return -fov / 2. + (double)k * incr; }

// argmin_k |angles[k] - a| over the uniform beam grid angles[k] = -fov/2 + k*incr
// (get_blocked_view_indices, laser_models.py:310-313).  The grid is strictly
// increasing, so |angles[k]-a| is V-shaped: test the analytic guess +-2 with
// NumPy's first-minimum tie break instead of a 1080-long scan.
F110_HD int nearest_beam(int B, double fov, double incr, double a) {
    if (a != a) return 0;  // np.argmin of an all-NaN array
    double g = (a + fov / 2.0) / incr;
    int k0 = g < 0 ? 0 : (g > (double)(B - 1) ? B - 1 : (int)(g + 0.5));
    int lo = k0 - 2 < 0 ? 0 : k0 - 2;
    int hi = k0 + 2 > B - 1 ? B - 1 : k0 + 2;
    int best = lo;
    double bd = fabs(beam_angle(lo, fov, incr) - a);
    for (int k = lo + 1; k <= hi; ++k) {
        double d = fabs(beam_angle(k, fov, incr) - a);
        if (d < bd) { bd = d; best = k; }
    }
    return best;
}

// One vertex of get_blocked_view_indices (laser_models.py:282-315): the beam
// nearest to the vertex bearing, relative to ego = atan2(sin(yaw), cos(yaw)).
// phi receives the vertex bearing atan2(uy, ux) (used by box_beam_window).
F110_HD int blocked_vertex_beam(double px, double py, double ego, double vx0, double vy0, int B, double fov,
                                double incr, double &phi) {
    double vx = vx0 - px, vy = vy0 - py;
    double nrm = sqrt(vx * vx + vy * vy);
    double ux = vx / nrm, uy = vy / nrm;
    phi = atan2(uy, ux);
    double angle = ego - phi;
    if (angle > kPi) angle = angle - 2 * kPi;
    else if (angle < -kPi) angle = angle + 2 * kPi;
    return nearest_beam(B, fov, incr, -angle);
}

// get_blocked_view_indices, laser_models.py:282-315
F110_HD void blocked_range(double px, double py, double pth, const double v[8], int B, double fov, double incr,
                           int &lo, int &hi) {
    double ey, ex;
    cr_sincos(pth, ey, ex);
    double ego = atan2(ey, ex);
    int mn = 0, mx = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double vx = v[2 * i] - px, vy = v[2 * i + 1] - py;
        double nrm = sqrt(vx * vx + vy * vy);
        double ux = vx / nrm, uy = vy / nrm;
        double angle = ego - atan2(uy, ux);
        if (angle > kPi) angle = angle - 2 * kPi;
        else if (angle < -kPi) angle = angle + 2 * kPi;
        int k = nearest_beam(B, fov, incr, -angle);
        if (i == 0 || k < mn) mn = k;
        if (i == 0 || k > mx) mx = k;
    }
    lo = mn;
    hi = mx;
}

// Which beams of a ray_cast can reach an opponent's box at all.  From scan
// origin o outside the (convex) box, a ray at world angle theta meets an
// edge only if theta lies in the angular interval the box subtends at o.
// Beams more than kBeamMargin outside it miss every edge by a relative
// margin (>= 1e-9 of the edge parameter for o at least kBoxClearance away),
// far above f64 rounding, so the reference's get_range returns inf for all
// four edges and the beam can be skipped.  The filter is off (half = inf)
// when o is within kBoxClearance of a vertex or of an edge's line (which
// includes are_collinear's 1e-8 test: get_range's denom == 0 branch ignores
// the beam direction there), or inside the box.
constexpr double kBeamMargin = 1e-5;
constexpr double kBoxClearance = 1e-3;

F110_HD double wrap_pm_pi(double a) { return a - 2.0 * kPi * rint(a * (0.5 / kPi)); }  // approximate

// The beam-index ranges [r0a, r0b] and [r1a, r1b] (either may be empty) that
// can hold beams of the window (center, half) for a car at yaw oth:
// angle(b) = oth + angles[b] with angles[b] ~ -fov/2 + b*incr.  Padded by 2
// beams; callers still apply the exact per-beam window test.
F110_HD void window_beam_ranges(double oth, double fov, double incr, int B, double center, double half, int &r0a,
                                int &r0b, int &r1a, int &r1b) {
    r0a = 0;
    r0b = B - 1;
    r1a = 1;
    r1b = 0;
    if (!(half < kPi)) return;  // no filter: every beam
    // u(b) = angle(b) - (center - half), taken mod 2pi into [0, 2pi)
    double c0 = oth - fov / 2.0 - (center - half);
    c0 = c0 - 2.0 * kPi * floor(c0 * (0.5 / kPi));
    // in the window iff (c0 + b*incr) mod 2pi <= 2*half
    const double w = 2.0 * half;
    r0a = 0;
    r0b = c0 <= w ? (int)floor((w - c0) / incr) + 2 : -1;
    r1a = (int)ceil((2.0 * kPi - c0) / incr) - 2;
    r1b = (int)floor((2.0 * kPi - c0 + w) / incr) + 2;
    if (r0b > B - 1) r0b = B - 1;
    if (r1a < 0) r1a = 0;
    if (r1b > B - 1) r1b = B - 1;
    if (r1a <= r1b && r0a <= r0b && r1a <= r0b + 1) {  // overlapping: one range
        r0b = r1b > r0b ? r1b : r0b;
        r1a = 1;
        r1b = 0;
    }
}

F110_HD void box_beam_window(double ox, double oy, const double v[8], const double phi_in[4], double &center,
                             double &half) {
    center = 0.0;
    half = INFINITY;
    double phi[4];
    int inside_pos = 0, inside_neg = 0;
    for (int q = 0; q < 4; ++q) {
        const double ax = v[2 * q], ay = v[2 * q + 1];
        const double bx = v[2 * ((q + 1) & 3)], by = v[2 * ((q + 1) & 3) + 1];
        const double dx = ax - ox, dy = ay - oy;
        if (dx * dx + dy * dy < kBoxClearance * kBoxClearance) return;
        // |cross(va - o, o - vb)| = |edge| * distance(o, edge line): no filter
        // within kBoxClearance of any edge line (this also covers
        // are_collinear's 1e-8 test and keeps d1's sign robust for rays whose
        // backward half crosses an edge)
        const double c = dx * (oy - by) - dy * (ox - bx);
        const double ex = bx - ax, ey = by - ay;
        if (fabs(c) < 1e-8 || c * c < kBoxClearance * kBoxClearance * (ex * ex + ey * ey)) return;
        // side of o relative to edge a->b (all one sign: o inside the box)
        const double side = (bx - ax) * (oy - ay) - (by - ay) * (ox - ax);
        inside_pos += side > 0.0;
        inside_neg += side < 0.0;
        // bearing of the vertex from o (any approximation is fine: the margin
        // is 1e-5 rad); phi_in = the blocked-range bearings when available
        phi[q] = phi_in ? phi_in[q] : atan2(dy, dx);
    }
    if (inside_pos == 4 || inside_neg == 4) return;
    double lo = 0.0, hi = 0.0;
    for (int q = 1; q < 4; ++q) {
        const double d = wrap_pm_pi(phi[q] - phi[0]);
        lo = d < lo ? d : lo;
        hi = d > hi ? d : hi;
    }
    if (hi - lo > kPi - 1e-3) return;  // o very close to the box: no filter
    center = phi[0] + 0.5 * (lo + hi);
    half = 0.5 * (hi - lo) + kBeamMargin;
}

// get_range, laser_models.py:249-280, with the beam's (cos, sin)(theta + pi/2)
// hoisted out of the 4-edge loop (same values each call).
F110_HD double get_range(double ox, double oy, double v30, double v31, double va0, double va1, double vb0,
                         double vb1) {
    double v10 = ox - va0, v11 = oy - va1;
    double v20 = vb0 - va0, v21 = vb1 - va1;
    double denom = dot2(v20, v21, v30, v31);
    double distance = INFINITY;
    if (fabs(denom) > 0.0) {
        double d1 = (v20 * v11 - v21 * v10) / denom;
        double d2 = dot2(v10, v11, v30, v31) / denom;
        if (d1 >= 0.0 && d2 >= 0.0 && d2 <= 1.0) distance = d1;
    } else {
        double ba0 = va0 - ox, ba1 = va1 - oy;  // are_collinear(o, va, vb) :232-247
        double ca0 = ox - vb0, ca1 = oy - vb1;
        if (fabs(ba0 * ca1 - ba1 * ca0) < 1e-8) {
            double e0 = va0 - ox, e1 = va1 - oy, f0 = vb0 - ox, f1 = vb1 - oy;
            double da = sqrt(fma(e1, e1, e0 * e0));
            double db = sqrt(fma(f1, f1, f0 * f0));
            distance = da <= db ? da : db;
        }
    }
    return distance;
}

// ----------------------------------------------------------------- noise --
// Philox4x32-10 (Salmon et al., SC'11) keyed by (seed, global env id);
// counter = (beam pair, steps since reset, stream tag).  Scan noise replaces
// numpy default_rng(seed).normal(0, std, B) (laser_models.py:450-452): same
// stream for every agent of an env and restarted at every reset
// (base_classes.py:119,204), like the reference.
struct U4 { uint32_t x, y, z, w; };

F110_HD U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        U4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

F110_HD double u01_open(uint32_t hi, uint32_t lo) {  // (0, 1], 53 bits
    uint64_t v = ((uint64_t)(hi >> 5) << 26) | (uint64_t)(lo >> 6);
    return ((double)v + 1.0) * (1.0 / 9007199254740992.0);
}

// ---------------------------------------------------- NumPy float32 trig --
// np.cos / np.sin on float32 (NumPy 2.2, the x86 SIMD loop of
// umath/loops_trigonometric: Cody-Waite reduction by pi/2 in three fma steps,
// degree-8 cosine / degree-9 sine minimax polynomials on [-pi/4, pi/4],
// quadrant select; |x| beyond 71476.0625 (cos) / 117435.992 (sin) goes to
// libm, here the correctly rounded float of the f64 function).  F110Env.reset
// evaluates start_rot this way when its options are float32
// (f110_env.py:448-451, train_ddpg's dtype).  Bit-exact against the installed
// NumPy on [-pi, pi] and beyond (tests/test_host_lib.py).
F110_HD float np_sincosf(float x, bool cos_op) {
    if (x != x) return x;
    const float ax = x < 0.0f ? -x : x;
    if (ax > (cos_op ? 71476.0625f : 117435.992f)) return (float)(cos_op ? cos((double)x) : sin((double)x));
    const float magic = 0x1.800000p+23f;
    float q = fmaf(x, 0x1.45f306p-1f, magic);  // x * 2/pi, rounded to the nearest integer (one fma)
    q = q - magic;
    float r = fmaf(q, -0x1.921fb0p+00f, x);
    r = fmaf(q, -0x1.5110b4p-22f, r);
    r = fmaf(q, -0x1.846988p-48f, r);
    const float r2 = r * r;
    float c = fmaf(0x1.98e616p-16f, r2, -0x1.6c06dcp-10f);
    c = fmaf(c, r2, 0x1.55553cp-05f);
    c = fmaf(c, r2, -0x1.000000p-01f);
    c = fmaf(c, r2, 0x1.000000p+00f);
    float sn = fmaf(0x1.7d3bbcp-19f, r2, -0x1.a06bbap-13f);
    sn = fmaf(sn, r2, 0x1.11119ap-07f);
    sn = fmaf(sn, r2, -0x1.555556p-03f);
    sn = fmaf(sn, r2, 0.0f);
    sn = fmaf(sn, r, r);
    int iq = (int)q;  // q is integral
    if (cos_op) iq += 1;
    float v = (iq & 1) == 0 ? sn : c;
    if ((iq & 2) == 2) v = 0.0f - v;
    return v;
}

// Philox2x32-10 (Salmon et al., SC'11; passes BigCrush): one 32x32->64
// multiply and one xor3 per round, half the work of Philox4x32 for the 48
// random bits one normal needs.
struct U2 { uint32_t x, y; };

F110_HD U2 philox2x32(uint32_t L, uint32_t R, uint32_t k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p = (uint64_t)0xD256D193u * L;
        const uint32_t hi = (uint32_t)(p >> 32);
        L = hi ^ k ^ R;
        R = (uint32_t)p;
        k += 0x9E3779B9u;
    }
    return {L, R};
}

// the noise key of (seed, env): distinct envs of one seed get distinct keys
// (an odd multiplier is a bijection mod 2^32)
F110_HD uint32_t noise_key(uint64_t seed, uint64_t env) {
    return (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x85EBCA6Bu) ^ ((uint32_t)env * 0x9E3779B9u) ^
           ((uint32_t)(env >> 32) * 0xC2B2AE35u);
}

// N(0,1) noise of the env's stream at `step`: beams b and b + 64 of each
// 128-beam block share one Philox2x32 block (counter (step, p | step_hi <<
// 16) with p = (b >> 7) * 64 + (b & 63), key noise_key(seed, env)) and take
// the two outputs of one Box-Muller transform, rad * cos and rad * sin
// (independent N(0,1)), on 24-bit uniforms in fp32 hardware transcendentals
// (v_log, v_sqrt, v_cos, v_sin: the noise is a statistical quantity, its ~1e-7
// relative precision is far below the 0.01 m std it scales; tails are cut at
// 5.8 sigma).  A lane tracing both beams (k_rays_fxn<2>) draws once for two.
// The key is per env: wave-uniform in the chunked ray kernels.
F110_D void beam_normal_pair_k(uint32_t key, uint64_t step, int p, float &n_lo, float &n_hi) {
    const U2 r = philox2x32((uint32_t)step, (uint32_t)p | ((uint32_t)(step >> 32) << 16), key);
    const float u1 = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
    const float u2 = (float)(r.y >> 8) * (1.0f / 16777216.0f);           // [0, 1)
    const float rad = __builtin_amdgcn_sqrtf(-2.0f * 0.69314718055994531f * __builtin_amdgcn_logf(u1));
    n_lo = rad * __builtin_amdgcn_cosf(u2);  // cos(2 pi u2): beam (b & ~64)
    n_hi = rad * __builtin_amdgcn_sinf(u2);  // sin(2 pi u2): beam (b | 64)
}

F110_D int beam_noise_pair(int b) { return ((b >> 7) << 6) | (b & 63); }

F110_D float beam_normal_k(uint32_t key, uint64_t step, int b) {
    float lo, hi;
    beam_normal_pair_k(key, step, beam_noise_pair(b), lo, hi);
    return (b & 64) ? hi : lo;
}

F110_D float beam_normal(uint64_t seed, uint64_t env, uint64_t step, int b) {
    return beam_normal_k(noise_key(seed, env), step, b);
}

// uniform u32 for (seed, env, episode) — autoreset spawn choice.
F110_HD uint32_t spawn_draw(uint64_t seed, uint64_t env, uint64_t episode) {
    U4 c = {(uint32_t)episode, (uint32_t)(episode >> 32), 0x5BA3Eu, 0u};
    U4 r = philox(c, (uint32_t)seed ^ (uint32_t)env, (uint32_t)(seed >> 32) ^ (uint32_t)(env >> 32) ^ 0xA5A5A5A5u);
    return r.x;
}

}  // namespace f110
