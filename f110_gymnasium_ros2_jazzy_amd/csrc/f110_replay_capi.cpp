// f110_replay_capi.cpp — host side of the learner's device components
// (include/f110.h, "prioritized experience replay" and "learner
// optimizer"): argument checks, the device allocation at create, and the
// launches of f110_replay.hip / f110_adam.hip.
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "f110_internal.h"

using namespace f110;

int f110_set_error(int code, const std::string &msg);  // f110_capi.cpp

namespace {
int fail(int code, const std::string &msg) { return f110_set_error(code, msg); }
}  // namespace

struct f110_replay {
    int device = 0;
    int64_t max_add = 0;
    int32_t max_batch = 0;
    int64_t known_len = 0;  // a lower bound of the device length seen by f110_replay_length (never shrinks)
    ReplayView v{};
    std::vector<void *> allocs;

    template <class T>
    hipError_t alloc(T **p, size_t n) {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, n * sizeof(T) + 16);
        if (e == hipSuccess) {
            allocs.push_back(q);
            *p = static_cast<T *>(q);
        }
        return e;
    }
};

extern "C" int f110_replay_create(f110_replay **out, int32_t device, int64_t capacity, int32_t obs_dim,
                                  int32_t act_dim, int32_t max_batch, int64_t max_add, double alpha, double eps,
                                  uint64_t seed) {
    if (!out || capacity <= 0 || capacity >= (int64_t)1 << 32 || obs_dim <= 0 || act_dim <= 0 || act_dim > 256 ||
        max_batch <= 0 || max_batch > kReplayMaxBatch || max_add <= 0 || max_add > capacity)
        return fail(F110_E_INVALID,
                    "f110_replay_create: bad arguments (0 < capacity < 2^32, 0 < act_dim <= 256, "
                    "0 < max_batch <= 8192, 0 < max_add <= capacity)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev)
        return fail(F110_E_NODEVICE, "f110_replay_create: no such HIP device");
    if (hipSetDevice(device) != hipSuccess) return fail(F110_E_NODEVICE, "f110_replay_create: hipSetDevice");
    auto *rb = new f110_replay();
    rb->device = device;
    rb->max_add = max_add;
    rb->max_batch = max_batch;
    ReplayView &v = rb->v;
    v.capacity = capacity;
    v.obs_dim = obs_dim;
    v.act_dim = act_dim;
    v.alpha = alpha;
    v.eps = (float)eps;  // ps + self._eps is evaluated in float32 (NEP 50)
    v.seed = seed;
    const size_t cap = (size_t)capacity;
    hipError_t e = rb->alloc(&v.hdr, 1);
    if (e == hipSuccess) e = rb->alloc(&v.obs, cap * obs_dim);
    if (e == hipSuccess) e = rb->alloc(&v.next_obs, cap * obs_dim);
    if (e == hipSuccess) e = rb->alloc(&v.act, cap * act_dim);
    if (e == hipSuccess) e = rb->alloc(&v.reward, cap);
    if (e == hipSuccess) e = rb->alloc(&v.done, cap);
    if (e == hipSuccess) e = rb->alloc(&v.prio, cap);
    if (e == hipSuccess) e = rb->alloc(&v.wt, cap);
    if (e == hipSuccess) e = rb->alloc(&v.keys, cap);
    if (e == hipSuccess) e = rb->alloc(&v.hist, (size_t)kHistRep * 4 * 256);
    if (e == hipSuccess) e = rb->alloc(&v.den_part, kReplayMaxGrid);
    if (e == hipSuccess) e = rb->alloc(&v.part, kReplayMaxGrid);
    if (e == hipSuccess) e = rb->alloc(&v.sel, kReplayMaxBatch);
    if (e == hipSuccess) e = rb->alloc(&v.tie, kTieCap);
    if (e == hipSuccess) e = rb->alloc(&v.pos, (size_t)max_add);
    if (e == hipSuccess) e = hipMemset(v.hdr, 0, sizeof(ReplayHdr));
    if (e == hipSuccess) e = hipMemset(v.prio, 0, cap * sizeof(float));
    if (e == hipSuccess) e = hipMemset(v.wt, 0, cap * sizeof(double));
    if (e == hipSuccess) e = hipMemset(v.hist, 0, (size_t)kHistRep * 4 * 256 * sizeof(uint32_t));
    if (e == hipSuccess) e = prepare_replay(max_batch);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        for (void *q : rb->allocs) (void)hipFree(q);
        delete rb;
        return fail(F110_E_ALLOC, std::string("f110_replay_create: ") + hipGetErrorString(e));
    }
    *out = rb;
    return F110_OK;
}

extern "C" int f110_replay_destroy(f110_replay *rb) {
    if (!rb) return F110_OK;
    (void)hipSetDevice(rb->device);
    for (void *q : rb->allocs) (void)hipFree(q);
    delete rb;
    return F110_OK;
}

static bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

namespace {
int replay_add(f110_replay *rb, const char *fn, const float *obs, int64_t obs_stride, const float *act,
               int64_t act_stride, const float *reward, const double *reward64, const float *next_obs,
               int64_t next_stride, const uint8_t *done, const float *priority, const uint8_t *mask, int mask_skip,
               int64_t n, void *stream) {
    if (!rb) return fail(F110_E_INVALID, std::string(fn) + ": null buffer");
    if (n < 0 || n > rb->max_add) return fail(F110_E_INVALID, std::string(fn) + ": n must be in [0, max_add]");
    if (n == 0) return F110_OK;
    const ReplayView &v = rb->v;
    if (!obs || !act || (!reward && !reward64) || !next_obs || obs_stride < v.obs_dim || next_stride < v.obs_dim ||
        act_stride < v.act_dim)
        return fail(F110_E_INVALID, std::string(fn) + ": null row pointer or stride below the row length");
    if (hipSetDevice(rb->device) != hipSuccess) return fail(F110_E_HIP, std::string(fn) + ": hipSetDevice");
    ReplayRows in{};
    in.obs = obs;
    in.next_obs = next_obs;
    in.act = act;
    in.reward = reward;
    in.reward64 = reward64;
    in.done = done;
    in.priority = priority;
    in.obs_stride = obs_stride;
    in.next_stride = next_stride;
    in.act_stride = act_stride;
    in.vec4 = (v.obs_dim % 4 == 0 && obs_stride % 4 == 0 && next_stride % 4 == 0 && aligned16(obs) &&
               aligned16(next_obs)) ? 1 : 0;
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e = launch_replay_add_index(v, mask, mask_skip, priority, n, s);
    if (e == hipSuccess) e = launch_replay_add_copy(v, in, n, s);
    if (e != hipSuccess) return fail(F110_E_HIP, std::string(fn) + ": " + hipGetErrorString(e));
    return F110_OK;
}
}  // namespace

extern "C" int f110_replay_add(f110_replay *rb, const float *obs, int64_t obs_stride, const float *act,
                               int64_t act_stride, const float *reward, const float *next_obs, int64_t next_stride,
                               const uint8_t *done, const float *priority, const uint8_t *mask, int64_t n,
                               void *stream) {
    return replay_add(rb, "f110_replay_add", obs, obs_stride, act, act_stride, reward, nullptr, next_obs, next_stride,
                      done, priority, mask, 0, n, stream);
}

extern "C" int f110_replay_add_env(f110_replay *rb, const float *obs, int64_t obs_stride, const float *act,
                                   int64_t act_stride, const double *reward, const float *next_obs,
                                   int64_t next_stride, const uint8_t *terminated, const uint8_t *was_reset,
                                   int64_t n, void *stream) {
    if (!reward) return fail(F110_E_INVALID, "f110_replay_add_env: null reward");
    return replay_add(rb, "f110_replay_add_env", obs, obs_stride, act, act_stride, nullptr, reward, next_obs,
                      next_stride, terminated, nullptr, was_reset, 1, n, stream);
}

extern "C" int f110_replay_sample(f110_replay *rb, int32_t batch, double beta, int64_t *idx, float *weights,
                                  float *obs, float *act, float *reward, float *next_obs, float *done,
                                  void *stream) {
    if (!rb || !idx || !weights) return fail(F110_E_INVALID, "f110_replay_sample: null argument");
    if (batch <= 0 || batch > rb->max_batch) return fail(F110_E_INVALID, "f110_replay_sample: batch must be in [1, max_batch]");
    if (obs && (!act || !reward || !next_obs || !done))
        return fail(F110_E_INVALID, "f110_replay_sample: give all batch outputs or none");
    if (hipSetDevice(rb->device) != hipSuccess) return fail(F110_E_HIP, "f110_replay_sample: hipSetDevice");
    ReplayBatch out{};
    out.obs = obs;
    out.next_obs = next_obs;
    out.act = act;
    out.reward = reward;
    out.done = done;
    out.vec4 = (rb->v.obs_dim % 4 == 0 && obs && aligned16(obs) && aligned16(next_obs)) ? 1 : 0;
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e = launch_replay_select(rb->v, batch, beta, idx, weights, rb->known_len >= batch, s);
    if (e == hipSuccess) e = launch_replay_gather(rb->v, batch, idx, out, s);
    if (e != hipSuccess) return fail(F110_E_HIP, std::string("f110_replay_sample: ") + hipGetErrorString(e));
    return F110_OK;
}

extern "C" int f110_replay_update_priorities(f110_replay *rb, const int64_t *idx, const float *values, int64_t n,
                                             int32_t from_td, float add_eps, void *stream) {
    if (!rb || n < 0 || (n > 0 && (!idx || !values)))
        return fail(F110_E_INVALID, "f110_replay_update_priorities: bad arguments");
    if (hipSetDevice(rb->device) != hipSuccess) return fail(F110_E_HIP, "f110_replay_update_priorities: hipSetDevice");
    hipError_t e = launch_replay_update(rb->v, idx, values, n, add_eps, from_td ? 1 : 0, 0, (hipStream_t)stream);
    if (e != hipSuccess) return fail(F110_E_HIP, std::string("f110_replay_update_priorities: ") + hipGetErrorString(e));
    return F110_OK;
}

extern "C" int f110_replay_length(f110_replay *rb, int64_t *length, int64_t *next_idx, void *stream) {
    if (!rb) return fail(F110_E_INVALID, "f110_replay_length: null buffer");
    if (hipSetDevice(rb->device) != hipSuccess) return fail(F110_E_HIP, "f110_replay_length: hipSetDevice");
    ReplayHdr h{};
    hipError_t e = hipMemcpyAsync(&h, rb->v.hdr, sizeof(h), hipMemcpyDeviceToHost, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess) return fail(F110_E_HIP, std::string("f110_replay_length: ") + hipGetErrorString(e));
    if (length) *length = h.length;
    if (next_idx) *next_idx = h.next;
    if (h.length > rb->known_len) rb->known_len = h.length;  // the ring never shrinks
    return F110_OK;
}

extern "C" int f110_replay_arrays(f110_replay *rb, float **priority, float **obs, float **act, float **reward,
                                  float **next_obs, float **done) {
    if (!rb) return fail(F110_E_INVALID, "f110_replay_arrays: null buffer");
    if (priority) *priority = rb->v.prio;
    if (obs) *obs = rb->v.obs;
    if (act) *act = rb->v.act;
    if (reward) *reward = rb->v.reward;
    if (next_obs) *next_obs = rb->v.next_obs;
    if (done) *done = rb->v.done;
    return F110_OK;
}

extern "C" int f110_adam_step(float *param, float *exp_avg, float *exp_avg_sq, const float *grad, int64_t n,
                              double lr, double beta1, double beta2, double eps, void *state, float *target,
                              double tau, void *stream) {
    if (n < 0 || (n > 0 && (!param || !exp_avg || !exp_avg_sq || !grad || !state)))
        return fail(F110_E_INVALID, "f110_adam_step: bad arguments");
    AdamArgs a{};
    a.param = param;
    a.exp_avg = exp_avg;
    a.exp_avg_sq = exp_avg_sq;
    a.grad = grad;
    a.n = n;
    a.lr = lr;
    a.beta1 = beta1;
    a.beta2 = beta2;
    a.eps = eps;
    a.step = static_cast<int64_t *>(state);
    a.target = target;
    a.tau = (float)tau;
    a.done = reinterpret_cast<uint32_t *>(static_cast<int64_t *>(state) + 1);
    hipError_t e = launch_adam(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(F110_E_HIP, std::string("f110_adam_step: ") + hipGetErrorString(e));
    return F110_OK;
}
