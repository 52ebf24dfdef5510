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

__global__ void __launch_bounds__(256) k_adam(AdamArgs a) {
    const double t = (double)(*a.step + 1);
    const float w1 = (float)(1.0 - a.beta1);                        // lerp weight (< 0.5)
    const float b2 = (float)a.beta2, w2 = (float)(1.0 - a.beta2);
    const double bc1 = 1.0 - pow(a.beta1, t), bc2 = 1.0 - pow(a.beta2, t);
    const float step_size = (float)(a.lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    const float eps = (float)a.eps;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * 256) {
        const float g = a.grad[i];
        float m = a.exp_avg[i];
        m = m + w1 * (g - m);
        float v = a.exp_avg_sq[i];
        v = v * b2;
        v = v + (w2 * g) * g;
        const float denom = sqrtf(v) / bc2_sqrt + eps;
        const float p = a.param[i] + (-step_size) * (m / denom);
        a.param[i] = p;
        a.exp_avg[i] = m;
        a.exp_avg_sq[i] = v;
        if (a.target) {
            const float t0 = a.target[i];
            a.target[i] = t0 + a.tau * (p - t0);
        }
    }
    // the last block to finish advances the step counter
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const uint32_t done = atomicAdd(a.done, 1u);
        if (done == gridDim.x - 1) {
            *a.step += 1;
            *a.done = 0;
        }
    }
}

hipError_t launch_adam(const AdamArgs &a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    int64_t g = (a.n + 1023) / 1024;
    g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
    hipLaunchKernelGGL(k_adam, dim3((unsigned)g), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace f110
