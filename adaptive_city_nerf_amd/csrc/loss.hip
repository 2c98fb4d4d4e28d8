// loss.hip -- the training loss of the adaptation / meta-training steps on gfx950:
//   nerfs/losses.py:10-32 compute_mse_loss = F.mse_loss(*color_space_transformer(pred, gt, "linear"))
//   nerfs/color_space.py:13-19, 22-66 (gt.clamp(0,1) -> srgb_to_linear -> clamp(0,1); pred.clamp(0,1))
// The reference evaluates this as ~11 elementwise / reduction launches forward and ~5 backward per
// render; in a meta-training step (108 renders) those 5-us launches cost more than the MLP forward.
// Here: one single-workgroup launch forward (the batch is thousands of rays; per-thread double partial
// sums, one fixed reduction order: deterministic) and one elementwise launch backward.
// Float semantics follow the torch ops: scalars as float (12.92f, 0.055f, 1.055f, 0.04045f), powf with
// the float exponent, clamps that pass NaN through, and mse_loss_backward's double `2 / numel` factor.
#include "acn_device.h"
#include "acn_internal.h"

namespace {

using acn::clamp01;
using acn::gt_linear;   // gt (sRGB in [0,1] after the clamp) -> linear, clamped again

constexpr int kThreads = 1024;

__global__ void __launch_bounds__(kThreads) mse_linear_fwd_kernel(const float* __restrict__ pred,
                                                                  const float* __restrict__ gt, int64_t n,
                                                                  float* __restrict__ loss) {
    __shared__ double red[kThreads / 64];
    double acc = 0.0;
    // unrolled: the loads of 8 strides are issued together (same accumulation order per thread)
#pragma unroll 8
    for (int64_t e = threadIdx.x; e < n; e += kThreads) {
        const float d = clamp01(pred[e]) - gt_linear(gt[e]);
        acc += (double)(d * d);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < kThreads / 64; ++i) t += red[i];
        loss[0] = (float)(t / (double)n);
    }
}

// Multi-workgroup form (acn_mse_linear_fwd_ws): G workgroups of 256 threads (G sized for ~2 elements per
// thread, at most 256), thread i of workgroup b sums elements b*256 + i, + G*256, ... in double; the
// workgroup sums in a fixed order into partials[b]; the last workgroup to finish (ticket counter) adds
// partials[0..G) in a fixed tree, writes the loss and resets the counter.  Deterministic (fixed assignment and
// order for a given n).  The time of this launch is memory latency, not arithmetic: a thread's loads are
// issued 4 at a time ahead of the sums (same per-thread order), and the grid is wide enough that a thread
// has one or two such rounds (8 dependent rounds per thread measured 11 us at n = 12000,
// tools/micro/loss_micro.py).
constexpr int kWsThreads = 256;
constexpr int kWsMaxBlocks = 256;
constexpr int kWsPerThread = 2;
__global__ void __launch_bounds__(kWsThreads) mse_linear_fwd_ws_kernel(const float* __restrict__ pred,
                                                                       const float* __restrict__ gt, int64_t n,
                                                                       double* __restrict__ partials,
                                                                       unsigned int* __restrict__ counter,
                                                                       float* __restrict__ loss) {
    __shared__ double red[kWsThreads / 64];
    __shared__ bool last;
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kWsThreads;
    for (int64_t e = (int64_t)blockIdx.x * kWsThreads + threadIdx.x; e < n; e += 4 * stride) {
        float p[4], q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = e + u * stride;
            p[u] = i < n ? pred[i] : 0.0f;
            q[u] = i < n ? gt[i] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (e + u * stride < n) {
                const float d = clamp01(p[u]) - gt_linear(q[u]);
                acc += (double)(d * d);
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < kWsThreads / 64; ++i) t += red[i];
        partials[blockIdx.x] = t;
        __threadfence();
        last = atomicAdd(counter, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    // last workgroup: thread i loads partial i (G <= 256), then a fixed xor tree per wave and the waves in order
    // (deterministic for a given n; a serial in-order sum through one wave measured ~10 us of this launch)
    if (last) {
        __threadfence();
        const unsigned int G = gridDim.x;
        double v = threadIdx.x < G ? __hip_atomic_load(&partials[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : 0.0;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        __syncthreads();   // red[] is reused (thread 0 read it above)
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
        __syncthreads();
        double t = 0.0;
        for (int i = 0; i < kWsThreads / 64; ++i) t += red[i];
        if (threadIdx.x == 0) {
            loss[0] = (float)(t / (double)n);
            counter[0] = 0u;
        }
    }
}

// d loss / d pred: mse_loss_backward (2 / numel * (input - target) * grad_output, in double) through the
// clamp's backward (gradient where 0 <= pred <= 1)
__global__ void __launch_bounds__(256) mse_linear_bwd_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                             int64_t n, const float* __restrict__ g_loss,
                                                             float* __restrict__ g_pred) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const float p = pred[e];
    const float d = clamp01(p) - gt_linear(gt[e]);
    const float g = (float)((2.0 / (double)n) * (double)d * (double)g_loss[0]);
    g_pred[e] = (p >= 0.0f && p <= 1.0f) ? g : 0.0f;
}

}  // namespace

extern "C" int acn_mse_linear_fwd(const float* pred, const float* gt, int64_t n, float* loss, void* stream) {
    ACN_REQUIRE(n >= 1 && pred && gt && loss, "acn_mse_linear_fwd: bad arguments");
    hipLaunchKernelGGL(mse_linear_fwd_kernel, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, pred, gt, n, loss);
    return acn_check_launch("acn_mse_linear_fwd");
}

extern "C" size_t acn_mse_linear_workspace_bytes(void) { return kWsMaxBlocks * sizeof(double) + 16; }

extern "C" int acn_mse_linear_fwd_ws(const float* pred, const float* gt, int64_t n, float* loss, void* workspace,
                                     size_t workspace_bytes, void* stream) {
    ACN_REQUIRE(n >= 1 && pred && gt && loss && workspace, "acn_mse_linear_fwd_ws: bad arguments");
    ACN_REQUIRE(workspace_bytes >= acn_mse_linear_workspace_bytes(), "acn_mse_linear_fwd_ws: workspace too small");
    int64_t g = (n + kWsThreads * kWsPerThread - 1) / (kWsThreads * kWsPerThread);
    g = g < 1 ? 1 : (g > kWsMaxBlocks ? kWsMaxBlocks : g);
    double* partials = (double*)workspace;
    unsigned int* counter = (unsigned int*)((char*)workspace + kWsMaxBlocks * sizeof(double));
    hipLaunchKernelGGL(mse_linear_fwd_ws_kernel, dim3((unsigned)g), dim3(kWsThreads), 0, (hipStream_t)stream, pred, gt,
                       n, partials, counter, loss);
    return acn_check_launch("acn_mse_linear_fwd_ws");
}

extern "C" int acn_mse_linear_bwd(const float* pred, const float* gt, int64_t n, const float* g_loss, float* g_pred,
                                  void* stream) {
    ACN_REQUIRE(n >= 1 && pred && gt && g_loss && g_pred, "acn_mse_linear_bwd: bad arguments");
    hipLaunchKernelGGL(mse_linear_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       pred, gt, n, g_loss, g_pred);
    return acn_check_launch("acn_mse_linear_bwd");
}
