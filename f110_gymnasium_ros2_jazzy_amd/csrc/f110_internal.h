// f110_internal.h — context layout and kernel launchers shared by
// f110_kernels.hip (device) and f110_capi.cpp (host API).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "f110_device.h"

namespace f110 {

// Everything one launch of the fused env-step kernel needs, passed by value.
struct StepArgs {
    MapView map;
    const double *sines, *cosines;            // [theta_dis]  ScanSimulator2D tables
    const double *angles, *beam_cos, *side;   // [B] RaceCar class-level beam tables
    f110_params p;
    int32_t E, A, B, theta_dis, integrator, ego, autoreset, mode;  // mode 0 step, 1 reset
    double fov, eps, max_range, dt, lidar_dist, ttc_thresh, noise_std, inc, beam_incr;
    uint64_t seed;
    int64_t env_offset;
    // persistent per-agent / per-env state (SoA, owned by the context)
    double *st;          // [7][E*A]
    double *sb;          // [2][E*A] steer buffer (newest, older)
    int32_t *scnt;       // [E*A]
    double *start;       // [3][E*A] reset poses (lap logic)
    int32_t *toggles;    // [E*A]
    uint8_t *near_start; // [E*A]
    float *lap_times;    // [E*A]
    float *lap_counts;   // [E*A]
    double *sim_time;    // [E]
    uint8_t *pending;    // [E] autoreset pending
    uint64_t *episode;   // [E]
    uint64_t *nstep;     // [E] steps since reset (noise counter)
    const double *spawn; // [n_spawn][A][3]
    int32_t n_spawn;
    // inputs
    const float *actions;       // [E][A][2]
    const double *reset_poses;  // [E][A][3]
    const uint8_t *reset_mask;  // [E] or null
    f110_outputs out;
    unsigned long long *ctr;    // [2] lookups, rays
};

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

size_t step_lds_bytes(int A, int B);
hipError_t prepare_env_step(size_t lds_bytes);
hipError_t launch_env_step(const StepArgs &a, hipStream_t s);
hipError_t launch_scan_batch(const ScanArgs &a, hipStream_t s);
hipError_t launch_dynamics_batch(const double *x, const double *u, double *f, int64_t M, const f110_params &p,
                                 hipStream_t s);

}  // namespace f110
