/*
 * f110_debug.h -- measurement, diagnostics, A/B scheduling knobs and host
 * test hooks of libf110.so (the same shared library as include/f110.h).
 *
 * None of these is part of the drop-in boundary (include/f110.h): the
 * reference has no counterpart for them.  They are used by bench.py, the
 * profiling scripts and the tests.  Results never depend on them: the
 * counters and timers only observe, and the f110_debug_set_* knobs change
 * which ray kernel variant runs, never what it computes (every variant is
 * bit-identical, tests/test_gpu_batch.py).  Conventions as in f110.h.
 */
#ifndef F110_DEBUG_H
#define F110_DEBUG_H

#include "f110.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- counters -------------------------------------------------------------
 * EDT lookups and rays traced by f110_step/f110_reset/f110_scan_batch since
 * the last reset of the counters (device-side accumulation; reading syncs
 * `stream`).  Used for the measured mean lookups per ray (roofline).
 * k_rays_fxs, the default ray kernel of f110_step, counts only while counting
 * is on (f110_debug_set_simt): its uncounted build keeps the per-trip
 * bookkeeping out of the timed loop; the other ray kernels always count. */
F110_API int f110_read_counters(f110_ctx *ctx, uint64_t *lookups, uint64_t *rays, void *stream);
F110_API int f110_reset_counters(f110_ctx *ctx, void *stream);
/* Diagnostic: the sum over the counter lines of counter idx (0..15): 0
 * lookups, 1 rays, 2 lane slots (f110_debug_read_simt). */
F110_API int f110_debug_read_counter(f110_ctx *ctx, int32_t idx, uint64_t *value, void *stream);
/* SIMT efficiency of the fixed-point ray loops (k_rays_fx / k_rays_fxn /
 * k_rays_fxs, the default kernels) since the last counter reset: loop_lookups
 * = lookups made inside the loop (all lookups less the first one per ray,
 * which k_agents makes), lane_slots = 64 x the wave-level gathers the loop
 * issued (k_rays_fx / k_rays_fxn: trip count x rays per lane; k_rays_fxs:
 * trips x 2 slots, a closed slot's zero-cell gather included), summed over
 * waves; efficiency = loop_lookups / lane_slots.  Other ray
 * kernels, and launches made while the count is off, leave lane_slots as
 * they are.  f110_debug_set_simt(ctx, 1) turns the count on (off by default: its
 * extra atomic per wave costs ~2 % of k_rays).  Diagnostics (no reference
 * counterpart).  While it is on, f110_step runs k_rays_fxs's counting build
 * (lookups, rays, lane slots, other loads: counters 0-3 and 5). */
F110_API int f110_debug_set_simt(f110_ctx *ctx, int32_t on);
F110_API int f110_debug_read_simt(f110_ctx *ctx, uint64_t *loop_lookups, uint64_t *lane_slots, void *stream);

/* Hand-off mask check (multi-agent contexts).  k_agents marks, per car, the
 * 64-beam chunks whose f64 scan k_post_multi's agent ray_cast may read, and
 * the ray kernel stores only those chunks into the hand-off buffer.  mode bit
 * 0: before each ray launch the hand-off buffer is filled with NaN and
 * k_post_multi counts every read of a beam whose chunk bit is clear into
 * counter 6 (f110_debug_read_counter); bit 1: no mask (every chunk stored, the
 * reference for bit-identity); bit 2: every mask empty (a forced miss: the
 * check's own test).  0 restores the default.  Debug only: with the
 * mask correct, outputs are the same bits in every mode. */
F110_API int f110_debug_set_handoff_check(f110_ctx *ctx, int32_t mode);

/* ---- per-kernel timing ----------------------------------------------------
 * Attaches a (start, stop) HIP event pair to the dispatch of each of the
 * three kernels of the next max_steps f110_step/f110_reset calls (k_agents,
 * k_rays, k_post; hipExtLaunchKernel: the kernel's own begin / end
 * timestamps, no marker packet between the kernels).
 * f110_profile_end waits for them and returns the summed milliseconds per
 * kernel and the number of steps recorded.  Used by bench.py for the
 * roofline of the dominant kernel (k_rays). */
F110_API int f110_profile_begin(f110_ctx *ctx, int32_t max_steps);
F110_API int f110_profile_end(f110_ctx *ctx, double ms_out[3], int32_t *steps_out);
/* Before f110_profile_end: the recorded steps' six timestamps (begin / end of
 * k_agents, the ray kernel, k_post) in ms after ref_event (a caller-owned
 * hipEvent_t with timing, recorded before those steps on any stream of the
 * device): out[step][6], up to max_steps steps; steps_out gets the count.
 * bench.py takes the union of the ray kernels' intervals over concurrent
 * stream sub-shards from it (the timed runner's own ray time). */
F110_API int f110_debug_profile_stamps(f110_ctx *ctx, void *ref_event, double *out, int32_t max_steps,
                                       int32_t *steps_out);

/* ---- diagnostics -------------------------------------------------------------
 * Wave trace of the ray kernel (one-wave blocks: k_rays_fx / k_rays_fxn /
 * k_rays_fxs, or the chunked k_rays_tiled on an axis-aligned map without a
 * reset mask): arm != 0 records the next f110_step's ray launch -- per wave
 * (block) {start, end} s_memrealtime ticks (100 MHz), {XCC id << 32 | HW_ID},
 * {item << 32 | car} (item: the chunk, chunk group, or k_rays_fxs's trips << 8
 * | wave of the car).  Entries of waves that did not run stay 0.  host_out
 * [max_waves][4] (or NULL) receives the last trace (waits for `stream`);
 * n_waves gets the buffer's capacity in waves. */
F110_API int f110_debug_wave_trace(f110_ctx *ctx, int32_t arm, uint64_t *host_out, int64_t max_waves,
                                   int64_t *n_waves, void *stream);

/* Ray gate for sub-shards stepped on concurrent streams (one context per
 * sub-shard, one stream each).  A non-null wait_event is waited on (stream
 * side) before every following f110_step / f110_reset ray launch of this
 * context; a non-null record_event is recorded right after it.  Chaining
 * the sub-shards' events in a ring keeps their ray passes in order (never two
 * ray grids competing for the CUs) while their k_agents / k_post launches run
 * beside another sub-shard's ray pass.  Events are caller-owned hipEvent_t;
 * NULL, NULL turns the gate off.  Scheduling only: results are unchanged. */
F110_API int f110_debug_set_ray_gate(f110_ctx *ctx, void *wait_event, void *record_event);

/* Turns the heavy-first ray dispatch off for the following f110_step calls of
 * this context (permanent).  Heavy-first starts the previous
 * step's long waves first so one ray grid does not end on them; when another
 * sub-shard's ray pass runs beside this one on a concurrent stream, that
 * tail is filled anyway and the list upkeep is the larger cost.
 * Scheduling only: results are unchanged. */
F110_API int f110_debug_disable_heavy_first(f110_ctx *ctx);

/* The ray kernel this context launches (>= 0), or a negative error code:
 * 1 k_rays_tiled in flat ray order, 2 tiled chunked, 3 the fixed-point
 * kernels k_rays_fx / k_rays_fxn / k_rays_fxs (the default where their
 * preconditions hold: axis-aligned map, EDT entries 0 or > eps).  Selected at
 * f110_create (env F110_RAY_KERNEL overrides the default, A/B only). */
F110_API int f110_debug_ray_kernel(const f110_ctx *ctx);

/* Rays traced per lane by the fixed-point ray kernel (1: k_rays_fx, 2:
 * k_rays_fxn / k_rays_fxs; size-based default, f110_debug_set_ray_lanes); 1 for the
 * other ray kernels.  Diagnostic, no reference counterpart. */
F110_API int f110_debug_ray_lanes(const f110_ctx *ctx);
/* k_rays_fxs's waves per car for unmasked steps (one wave per car traces the
 * car's 64-beam chunks two at a time, refilling a slot as soon as its chunk
 * ends), or 0 when the context steps with k_rays_fxn / k_rays_fx (heavy-first
 * on, one ray per lane, no padded table).  Default: 1 from 32768 cars. */
F110_API int f110_debug_ray_refill(const f110_ctx *ctx);
/* Set k_rays_fxs's waves per car (0: k_rays_fxn) and, when on, switch the
 * context to the padded EDT (built on first use) and off its heavy-first list.
 * For callers that split one GPU's cars over several contexts
 * (streams.StreamShards): the size rule is about the cars the GPU traces at
 * once, not one context's.  Any time.  Scheduling only: results are unchanged. */
F110_API int f110_debug_set_ray_refill(f110_ctx *ctx, int32_t waves);

/* Sets the rays per lane of the fixed-point ray kernel (1 or 2) before the
 * context's first reset/step.  The size-based default looks at this
 * context's cars only; a caller stepping S contexts concurrently on one GPU
 * (streams.StreamShards) knows the GPU's total and passes the choice for
 * that.  Scheduling only: results are unchanged.
 * Diagnostic / tuning, no reference counterpart. */
F110_API int f110_debug_set_ray_lanes(f110_ctx *ctx, int32_t n);

/* ---- host-side test hooks (no device work) -------------------------------
 * The lookup tables f110_create uploads: ScanSimulator2D sines/cosines
 * (laser_models.py:379-381) and RaceCar's class-level beam tables
 * (base_classes.py:122-158).  Any pointer may be NULL. */
F110_API void f110_host_tables(int32_t theta_dis, int32_t n_beams, double fov, const f110_params *p,
                               double *sines, double *cosines, double *angles, double *beam_cos, double *side);
/* get_scan's sequentially accumulated beam index (laser_models.py:167-184)
 * for every beam at yaw, evaluated through the run decomposition the kernels
 * use.  Returns the number of runs (>0) or a negative error. */
F110_API int f110_host_beam_indices(double yaw, double fov, int32_t theta_dis, int32_t n_beams,
                                    double *theta_index_out);
/* 1 when k_agents' run builder (build_beam_runs_fast) gives the same runs as
 * build_beam_runs at yaw, 0 when not, < 0 on error (host). */
/* cr_sincos's branch-free common case (k_agents' dynamics): ok[i] = 1 where it applies, and
 * there sn / cs are cr_sincos's values (host). */
F110_API void f110_host_sincos_fast(const double *x, int64_t n, double *sn, double *cs, uint8_t *ok);
/* The kinematic model's (tan, cos) from one table evaluation: where ok_t the correctly rounded
 * tan, where ok_c cr_sincos's cos (host). */
F110_API void f110_host_tan_cos_fast(const double *x, int64_t n, double *t, double *c, uint8_t *ok_t, uint8_t *ok_c);
F110_API int f110_host_beam_runs_agree(double yaw, double fov, int32_t theta_dis, int32_t n_beams);

/* xy_2_rc's cell (laser_models.py:55-104) for n points xy [n][2] on an H x W
 * map, through the three device mappings: lin_out[n][3] = row-major index
 * with the IEEE divide (cell_index), with the guarded fast quotient
 * (cell_index_fast), and the 4x4-tiled mapping of the ray kernel translated
 * back to row-major.  Out-of-map points give H*W-1 (the reference's
 * dt[-1, -1]).  Host only; the CPU tests check the three agree on boundary
 * points. */
F110_API int f110_host_cell_index(int32_t H, int32_t W, double resolution, const double origin[3], const double *xy,
                                  int64_t n, int64_t *lin_out);

/* The EDT table f110_create uploads for the fixed-point ray kernels, built on
 * the host: kind 0 the row-major table (rows of W + 1 cells rounded up to 16,
 * dt[-1,-1] in the padding, a 0.0 zero cell after the last row), kind 1 the
 * table padded by `pad` cells of dt[-1,-1] on every side (rows of 511 mod 512
 * cells; not built past its 32-bit / 24-bit offset limits: returns 0).
 * Returns the length in doubles; fills out[] when out_len suffices; meta =
 * {rows, cols, zero-cell byte offset or -1}.  Host test hook. */
F110_API int64_t f110_host_map_table(const uint32_t *edt_k, int32_t H, int32_t W, double res, int32_t kind,
                                     int32_t pad, double *out, int64_t out_len, int64_t meta[3]);

/* The beam-index ranges (r0a..r0b, r1a..r1b; empty when a > b) the agent
 * ray_cast visits for an opponent box whose angular window at the scan
 * origin is center +- half (world frame), for a car at yaw.  Host only; the
 * CPU tests check they contain every beam inside the window. */
/* Host copy of the device's cr_sincos (the ray_cast / box / dynamics sin and
 * cos: double-double evaluation, one rounding, i.e. correctly rounded).  It
 * equals NumPy's (glibc's) np.sin / np.cos except where glibc is itself off
 * by one ulp (< 0.3 % of the sampled arguments, test_cr_sincos_matches_numpy);
 * on those the device differs from the reference's trig by that ulp, which
 * the non-exact budgets (tests/golden/nonexact_beams.json) pin.  Test hook,
 * no reference counterpart. */
F110_API void f110_host_sincos(const double *x, int64_t n, double *sn, double *cs);
/* The same with the table path off (every value by the double-double
 * series): f110_host_sincos must give the same bits (test hook). */
F110_API void f110_host_sincos_series(const double *x, int64_t n, double *sn, double *cs);
/* NumPy's float32 np.cos (cos_op != 0) / np.sin over n values, as the
 * device evaluates F110Env.reset's float32 start_rot (test hook). */
F110_API void f110_host_np_sincosf(const float *x, int64_t n, int32_t cos_op, float *out);
F110_API void f110_host_window_ranges(double yaw, double fov, int32_t n_beams, double center, double half,
                                      int32_t ranges_out[4]);

#ifdef __cplusplus
}
#endif
#endif /* F110_DEBUG_H */
