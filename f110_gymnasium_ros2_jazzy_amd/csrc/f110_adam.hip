// f110_adam.hip — Adam over one network's flat parameter bucket.
//
// The DDPG learner (ddpg.py) keeps each network's parameters, gradients and
// Adam moments as flat fp32 buffers (the nn.Parameters are views), so one
// launch updates a whole network instead of torch.optim.Adam's per-tensor
// kernels.  The arithmetic is torch.optim.Adam's single-tensor update
// (torch/optim/adam.py, _single_tensor_adam, amsgrad=False, weight_decay=0),
// as agent.py:187-188 configures it, element by element in float32:
//   m = m + (1-b1)*(g - m)               exp_avg.lerp_(grad, 1-beta1)
//   v = v*b2 + ((1-b2)*g)*g              exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1-beta2)
//   p = p + (-lr/bc1) * (m / (sqrt(v)/sqrt(bc2) + eps))
// with bc_i = 1 - beta_i^t from the device step counter t (graph-safe: the
// last block to finish advances it).  With a target buffer the soft target
// update of the same network follows in the same pass (agent.py:340-341,
// target.lerp_(online, tau): t = t + tau * (p - t)): the reference applies it
// after both networks' steps, and neither network changes in between.
#include <hip/hip_runtime.h>

#include "f110_internal.h"

namespace f110 {

constexpr int kAdamPer = 4;

__global__ void __launch_bounds__(256) k_adam(AdamArgs a) {
    const int64_t step = *a.step;
    const double t = (double)(step + 1);
    // The last block to take a ticket advances the step counter.  The ticket is taken as soon as
    // the block has read the counter (the asm makes the atomic wait for that load), not after its
    // updates: the blocks' same-address atomics then overlap their memory work instead of queueing
    // at the end (1.6 us per launch at the critic's 338 blocks).  No fence: the last block hands
    // no data over, and every block's read of the counter has returned before its ticket.
    // atomicInc (old >= lim ? 0 : old + 1): the last ticket also re-arms the counter, and the
    // compiler's wave-level atomic rewrite (which would wait for the result at once) leaves it alone
    uint32_t ticket = 0u;
    if (threadIdx.x == 0) {
        uint32_t lim = gridDim.x - 1;
        asm volatile("" : "+v"(lim) : "v"((uint32_t)step));
        ticket = atomicInc(a.done, lim);  // its result is first needed after the updates
    }
    const float w1 = (float)(1.0 - a.beta1);                        // lerp weight (< 0.5)
    const float b2 = (float)a.beta2, w2 = (float)(1.0 - a.beta2);
    const double bc1 = 1.0 - pow(a.beta1, t), bc2 = 1.0 - pow(a.beta2, t);
    const float step_size = (float)(a.lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    const float eps = (float)a.eps;
    // kAdamPer elements per thread, their loads issued together (one memory round trip), then the
    // updates; a grid-stride loop over such groups
    for (int64_t base = (int64_t)blockIdx.x * 256 * kAdamPer + threadIdx.x; base < a.n;
         base += (int64_t)gridDim.x * 256 * kAdamPer) {
        float g[kAdamPer], m[kAdamPer], v[kAdamPer], p[kAdamPer], q[kAdamPer];
#pragma unroll
        for (int u = 0; u < kAdamPer; ++u) {
            const int64_t i = base + (int64_t)u * 256;
            const bool in = i < a.n;
            g[u] = in ? a.grad[i] : 0.0f;
            m[u] = in ? a.exp_avg[i] : 0.0f;
            v[u] = in ? a.exp_avg_sq[i] : 0.0f;
            p[u] = in ? a.param[i] : 0.0f;
            q[u] = in && a.target ? a.target[i] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < kAdamPer; ++u) {
            const int64_t i = base + (int64_t)u * 256;
            if (i >= a.n) break;
            float mm = m[u] + w1 * (g[u] - m[u]);
            float vv = v[u] * b2;
            vv = vv + (w2 * g[u]) * g[u];
            const float denom = sqrtf(vv) / bc2_sqrt + eps;
            const float pp = p[u] + (-step_size) * (mm / denom);
            a.param[i] = pp;
            a.exp_avg[i] = mm;
            a.exp_avg_sq[i] = vv;
            if (a.target) a.target[i] = q[u] + a.tau * (pp - q[u]);
        }
    }
    if (threadIdx.x == 0 && ticket == gridDim.x - 1) *a.step = step + 1;
}

hipError_t launch_adam(const AdamArgs &a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    // kAdamPer elements per thread (one memory round trip), at most 1024 blocks: few last-block
    // tickets on the one counter
    int64_t g = (a.n + 256 * kAdamPer - 1) / (256 * kAdamPer);
    g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
    hipLaunchKernelGGL(k_adam, dim3((unsigned)g), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace f110
