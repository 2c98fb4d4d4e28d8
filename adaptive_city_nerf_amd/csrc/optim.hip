// optim.hip -- the optimizer step of the online adaptation loop on gfx950:
//   torch.nn.utils.clip_grad_norm_(params, max_norm)      (runtime_adapt.py:305-307)
//   torch.optim.Adam(param_groups).step()                  (common/utils.py:57-62, runtime_adapt.py:309)
// over every parameter of the model in ONE launch each (multi-tensor), instead of per-tensor op
// chains.  The reference runs dense Adam over 134M parameters per step (4 experts x 2^24 table
// rows x 2): this step is HBM-bound (28 B moved per parameter: read p, g, m, v; write p, m, v),
// so the kernels stream 16-B vectors with every lane busy and fold the clip coefficient into the
// Adam pass (the clipped gradient is never written back).
//
// Work decomposition: every tensor is cut into chunks of ACN_OPTIM_CHUNK elements; the caller
// passes a device array of tensor descriptors and a chunk -> tensor map, so one grid covers all
// tensors (and no host synchronisation is needed between the norm, the coefficient and the step).
#include "acn_internal.h"

namespace {

constexpr int kThreads = 256;
#ifndef ACN_ADAM_UNROLL
#define ACN_ADAM_UNROLL 4
#endif
#ifndef ACN_ADAM_NT
#define ACN_ADAM_NT 2  // 1: non-temporal stores in the Adam passes, 2: non-temporal loads and stores
#endif
constexpr int kUnroll = ACN_ADAM_UNROLL;  // 16-B vectors in flight per lane and array: 2 blocks per CU need them to cover HBM latency

typedef float f4 __attribute__((ext_vector_type(4)));

// The slotted norm and Adam passes touch every byte once (p, g, m, v of 268M parameters >> the 256 MiB
// Infinity Cache): non-temporal loads and stores, A/B on the C5 step (tools/ab_c5.sh): Adam 1.69 ->
// 1.42 ms, plain / stores-only NT / 2 or 8 vectors in flight all slower.
__device__ __forceinline__ f4 ldv(const f4* a) {
    if (ACN_ADAM_NT >= 2) return __builtin_nontemporal_load(a);
    return *a;
}
__device__ __forceinline__ void stv(f4* a, const f4& v) {
    if (ACN_ADAM_NT >= 1) __builtin_nontemporal_store(v, a);
    else *a = v;
}

__device__ __forceinline__ double block_sum(double v) {
    __shared__ double red[kThreads / 64];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kThreads / 64; ++i) t += red[i];
    return t;  // valid on thread 0
}

// per-chunk sum of squared gradients (double accumulation)
__global__ void __launch_bounds__(kThreads) sumsq_kernel(const acn_param_desc* __restrict__ descs,
                                                         const int32_t* __restrict__ chunk_tensor,
                                                         double* __restrict__ partials) {
    const acn_param_desc d = descs[chunk_tensor[blockIdx.x]];
    const int64_t base = (int64_t)(blockIdx.x - d.first_chunk) * ACN_OPTIM_CHUNK;
    const int64_t n = d.numel - base < ACN_OPTIM_CHUNK ? d.numel - base : ACN_OPTIM_CHUNK;
    const float* g = d.grad + base;
    double acc = 0.0;
    if (d.grad != nullptr) {
        const bool vec = ((reinterpret_cast<uintptr_t>(g) & 15) == 0);
        if (vec) {
            const int64_t n4 = n >> 2;
            const f4* g4 = reinterpret_cast<const f4*>(g);
            int64_t i = threadIdx.x;
            for (; i + (kUnroll - 1) * kThreads < n4; i += kUnroll * kThreads) {  // kUnroll loads in flight
                f4 v[kUnroll];
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) v[u] = ldv(&g4[i + u * kThreads]);
#pragma unroll
                for (int u = 0; u < kUnroll; ++u)
                    acc += (double)v[u][0] * v[u][0] + (double)v[u][1] * v[u][1] + (double)v[u][2] * v[u][2] +
                           (double)v[u][3] * v[u][3];
            }
            for (; i < n4; i += kThreads) {
                const f4 v = ldv(&g4[i]);
                acc += (double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2] + (double)v[3] * v[3];
            }
            for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += kThreads) acc += (double)g[i] * g[i];
        } else {
            for (int64_t i = threadIdx.x; i < n; i += kThreads) acc += (double)g[i] * g[i];
        }
    }
    const double t = block_sum(acc);
    if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// extra (optional): a sum of squares produced elsewhere (the table-gradient scatter's telescoped sum,
// acn_hashgrid_bwd_pairs_sumsq), added to the total and reset to 0 for the next step
__global__ void __launch_bounds__(kThreads) reduce_kernel(const double* __restrict__ partials, int64_t n,
                                                          double* __restrict__ total, double* __restrict__ extra) {
    double acc = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += kThreads) acc += partials[i];
    const double t = block_sum(acc);
    if (threadIdx.x == 0) {
        if (extra) {
            total[0] = t + extra[0];
            extra[0] = 0.0;
        } else {
            total[0] = t;
        }
    }
}

// clip_grad_norm_ (torch/nn/utils/clip_grad.py): total_norm, clip_coef = max_norm / (total_norm +
// 1e-6) clamped to <= 1 (fp32 arithmetic, as the tensor ops there).
__global__ void clip_coef_kernel(const double* __restrict__ total_sumsq, float max_norm, float* __restrict__ out) {
    const float norm = (float)sqrt(total_sumsq[0]);
    float coef = max_norm / (norm + 1e-6f);
    coef = coef > 1.0f ? 1.0f : coef;  // NaN passes through, like torch.clamp
    out[0] = norm;
    out[1] = coef;
}

// GradScaler (torch/amp/grad_scaler.py: _unscale_grads_ + _amp_update_scale_) folded into the clip
// coefficient: the gradients stay scaled in memory and Adam multiplies by clip_coef / scale (exact: the scale
// is a power of two); a non-finite norm skips the step through seg[K] = -1.
__global__ void amp_unscale_coef_kernel(const double* __restrict__ total_sumsq, float max_norm, float* __restrict__ scale_p,
                                        int32_t* __restrict__ tracker, float* __restrict__ found_inf_p, float growth,
                                        float backoff, int growth_interval, float* __restrict__ out,
                                        int64_t* __restrict__ seg, int K) {
    const float scale = scale_p[0];
    const float inv = (float)(1.0 / (double)scale);  // scale.double().reciprocal().float(), as GradScaler
    const float norm = (float)sqrt(total_sumsq[0]) * inv;
    const bool found_inf = !(norm == norm) || norm == INFINITY;
    float coef = 1.0f;
    if (max_norm > 0.0f) {
        coef = max_norm / (norm + 1e-6f);
        coef = coef > 1.0f ? 1.0f : coef;
    }
    out[0] = norm;
    out[1] = coef * inv;
    found_inf_p[0] = found_inf ? 1.0f : 0.0f;
    if (found_inf) {  // torch._amp_update_scale_
        if (seg) seg[K] = -1;
        scale_p[0] = scale * backoff;
        tracker[0] = 0;
    } else {
        const int t = tracker[0] + 1;
        if (t == growth_interval) {
            const float g = scale * growth;
            scale_p[0] = (g == g && g != INFINITY) ? g : scale;  // only a finite grown scale is kept
            tracker[0] = 0;
        } else {
            tracker[0] = t;
        }
    }
}

struct GroupK {
    float lr_neg_step, w1, beta2, one_m_beta2, bc2s, eps, wd;
};
struct GroupsArg {
    GroupK g[ACN_OPTIM_MAX_GROUPS];
};

// torch.optim.Adam, single-tensor semantics (torch/optim/adam.py _single_tensor_adam):
//   g = grad * clip (+ wd * p); m = lerp(m, g, 1 - beta1); v = v * beta2 + (1 - beta2) * g * g
//   p += (-lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
__device__ __forceinline__ void adam_elem(float& p, float gr, float& m, float& v, float scale, const GroupK& k) {
    float g = gr * scale;
    if (k.wd != 0.0f) g = fmaf(k.wd, p, g);       // grad.add(param, alpha=wd) (vectorised fmadd)
    m = fmaf(k.w1, g - m, m);                    // at::lerp, |weight| < 0.5 branch (vectorised fmadd)
    v = v * k.beta2;
    v = v + (k.one_m_beta2 * g) * g;             // addcmul_(g, g, value = 1 - beta2)
    const float denom = sqrtf(v) / k.bc2s + k.eps;
    p = p + (k.lr_neg_step * m) / denom;         // addcdiv_(m, denom, value = -step_size)
}

__device__ __forceinline__ void adam_vec(f4& pp, const f4& gg, f4& mm, f4& vv, float scale, const GroupK& k) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float a = pp[c], b = mm[c], e = vv[c];
        adam_elem(a, gg[c], b, e, scale, k);
        pp[c] = a; mm[c] = b; vv[c] = e;
    }
}

// one chunk of one tensor: 16-B vectors, kUnroll of each array loaded before any is updated
__device__ __forceinline__ void adam_chunk(float* p, const float* g, float* m, float* v, int64_t n, float scale,
                                           const GroupK& k) {
    const uintptr_t align = reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                            reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v);
    int64_t done = 0;
    if ((align & 15) == 0) {
        const int64_t n4 = n >> 2;
        f4* p4 = reinterpret_cast<f4*>(p);
        const f4* g4 = reinterpret_cast<const f4*>(g);
        f4* m4 = reinterpret_cast<f4*>(m);
        f4* v4 = reinterpret_cast<f4*>(v);
        int64_t i = threadIdx.x;
        for (; i + (kUnroll - 1) * kThreads < n4; i += kUnroll * kThreads) {
            f4 pp[kUnroll], gg[kUnroll], mm[kUnroll], vv[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                pp[u] = ldv(&p4[i + u * kThreads]);
                gg[u] = ldv(&g4[i + u * kThreads]);
                mm[u] = ldv(&m4[i + u * kThreads]);
                vv[u] = ldv(&v4[i + u * kThreads]);
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                adam_vec(pp[u], gg[u], mm[u], vv[u], scale, k);
                stv(&p4[i + u * kThreads], pp[u]);
                stv(&m4[i + u * kThreads], mm[u]);
                stv(&v4[i + u * kThreads], vv[u]);
            }
        }
        for (; i < n4; i += kThreads) {
            f4 pp = ldv(&p4[i]), mm = ldv(&m4[i]), vv = ldv(&v4[i]);
            const f4 gg = ldv(&g4[i]);
            adam_vec(pp, gg, mm, vv, scale, k);
            stv(&p4[i], pp);
            stv(&m4[i], mm);
            stv(&v4[i], vv);
        }
        done = n4 << 2;
    }
    for (int64_t i = done + threadIdx.x; i < n; i += kThreads) {
        float a = p[i], b = m[i], e = v[i];
        adam_elem(a, g[i], b, e, scale, k);
        p[i] = a; m[i] = b; v[i] = e;
    }
}

__global__ void __launch_bounds__(kThreads) adam_kernel(const acn_param_desc* __restrict__ descs,
                                                        const int32_t* __restrict__ chunk_tensor, GroupsArg ga,
                                                        const float* __restrict__ grad_scale) {
    const acn_param_desc d = descs[chunk_tensor[blockIdx.x]];
    if (d.grad == nullptr) return;  // parameter without gradient: torch skips it
    const GroupK k = ga.g[d.group];
    const float scale = grad_scale ? grad_scale[1] : 1.0f;
    const int64_t base = (int64_t)(blockIdx.x - d.first_chunk) * ACN_OPTIM_CHUNK;
    const int64_t n = d.numel - base < ACN_OPTIM_CHUNK ? d.numel - base : ACN_OPTIM_CHUNK;
    float* p = d.param + base;
    const float* g = d.grad + base;
    float* m = d.exp_avg + base;
    float* v = d.exp_avg_sq + base;
    adam_chunk(p, g, m, v, n, scale, k);
}

// graph-replayable variant: the per-group constants come from a device table indexed by a device
// step counter that bump_kernel advances once per replay (before adam_table_kernel runs)
__global__ void bump_kernel(int32_t* __restrict__ step_dev) { step_dev[0] += 1; }

__global__ void __launch_bounds__(kThreads) adam_table_kernel(const acn_param_desc* __restrict__ descs,
                                                              const int32_t* __restrict__ chunk_tensor,
                                                              const GroupK* __restrict__ table, int ngroups,
                                                              const int32_t* __restrict__ step_dev, int first_step,
                                                              int table_steps, const float* __restrict__ grad_scale) {
    const int row = step_dev[0] - first_step;
    if (row < 0 || row >= table_steps) return;  // out of the uploaded range: the host re-uploads first
    const acn_param_desc d = descs[chunk_tensor[blockIdx.x]];
    if (d.grad == nullptr) return;
    const GroupK k = table[(int64_t)row * ngroups + d.group];
    const float scale = grad_scale ? grad_scale[1] : 1.0f;
    const int64_t base = (int64_t)(blockIdx.x - d.first_chunk) * ACN_OPTIM_CHUNK;
    const int64_t n = d.numel - base < ACN_OPTIM_CHUNK ? d.numel - base : ACN_OPTIM_CHUNK;
    float* p = d.param + base;
    const float* g = d.grad + base;
    float* m = d.exp_avg + base;
    float* v = d.exp_avg_sq + base;
    adam_chunk(p, g, m, v, n, scale, k);
}

// ---------------------------------------------------------------------------------------------
// Slotted variant (routed container, graph-replayable): tensor t belongs to activity slot
// flags[t] & 0xffff; slot s < K (an expert) is active in this step iff its routed pair count
// seg[K + 1 + s] > 0 (routed.hip), slots >= K (shared parameters) always.  Like torch, an inactive
// expert (grad None in the reference) is skipped entirely: no moment decay, no step increment.  Each
// slot keeps its own device step counter; the constants come from a table of steps 1..table_steps.
// flags bit 16: zero the gradient after reading it (the table gradients are scatter-added into
// persistent buffers, so the next step finds them cleared without a separate memset pass).
constexpr int kSlotZero = 1 << 16;
constexpr int kSlotNormElsewhere = 1 << 17;  // sum of squares supplied by acn_hashgrid_bwd_pairs_sumsq

__device__ __forceinline__ bool slot_active(const int64_t* __restrict__ seg, int K, int slot) {
    if (seg == nullptr) return true;
    if (seg[K] < 0) return false;  // an overflowed bounded exchange step (expert_parallel.py): no slot steps
    return slot >= K || seg[K + 1 + slot] > 0;
}

__global__ void bump_slots_kernel(int32_t* __restrict__ step_dev, const int64_t* __restrict__ seg, int K, int nslots) {
    const int s = threadIdx.x;
    if (s < nslots && slot_active(seg, K, s)) step_dev[s] += 1;
}

// CLIP: the last workgroup to finish (ticket counter, reset for the next call) also runs reduce_kernel's sum
// over the partials (same threads, same order: the same double) and clip_coef_kernel -- one launch instead of
// three, bitwise the same total and coefficient
template <bool CLIP>
__global__ void __launch_bounds__(kThreads) sumsq_slots_kernel(const acn_param_desc* __restrict__ descs,
                                                               const int32_t* __restrict__ chunk_tensor,
                                                               const int32_t* __restrict__ flags,
                                                               const int64_t* __restrict__ seg, int K,
                                                               double* __restrict__ partials,
                                                               double* __restrict__ total = nullptr,
                                                               double* __restrict__ extra = nullptr,
                                                               float max_norm = 0.0f, float* __restrict__ out = nullptr,
                                                               unsigned int* __restrict__ counter = nullptr) {
    const int t = chunk_tensor[blockIdx.x];
    const acn_param_desc d = descs[t];
    double acc = 0.0;
    if (d.grad != nullptr && slot_active(seg, K, flags[t] & 0xffff) && !(flags[t] & kSlotNormElsewhere)) {
        const int64_t base = (int64_t)(blockIdx.x - d.first_chunk) * ACN_OPTIM_CHUNK;
        const int64_t n = d.numel - base < ACN_OPTIM_CHUNK ? d.numel - base : ACN_OPTIM_CHUNK;
        const float* g = d.grad + base;
        if ((reinterpret_cast<uintptr_t>(g) & 15) == 0) {
            const int64_t n4 = n >> 2;
            const f4* g4 = reinterpret_cast<const f4*>(g);
            int64_t i = threadIdx.x;
            for (; i + (kUnroll - 1) * kThreads < n4; i += kUnroll * kThreads) {
                f4 v[kUnroll];
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) v[u] = ldv(&g4[i + u * kThreads]);
#pragma unroll
                for (int u = 0; u < kUnroll; ++u)
                    acc += (double)v[u][0] * v[u][0] + (double)v[u][1] * v[u][1] + (double)v[u][2] * v[u][2] +
                           (double)v[u][3] * v[u][3];
            }
            for (; i < n4; i += kThreads) {
                const f4 v = ldv(&g4[i]);
                acc += (double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2] + (double)v[3] * v[3];
            }
            for (int64_t i2 = (n4 << 2) + threadIdx.x; i2 < n; i2 += kThreads) acc += (double)g[i2] * g[i2];
        } else {
            for (int64_t i = threadIdx.x; i < n; i += kThreads) acc += (double)g[i] * g[i];
        }
    }
    const double tot = block_sum(acc);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
    if constexpr (CLIP) {
        __shared__ bool last;
        if (threadIdx.x == 0) {
            __threadfence();
            last = atomicAdd(counter, 1u) == gridDim.x - 1;
        }
        __syncthreads();
        if (!last) return;
        __threadfence();
        double a2 = 0.0;
        for (int64_t i = threadIdx.x; i < (int64_t)gridDim.x; i += kThreads)
            a2 += __hip_atomic_load(&partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double t = block_sum(a2);
        if (threadIdx.x == 0) {
            double tt = t;
            if (extra) {
                tt = t + extra[0];
                extra[0] = 0.0;
            }
            total[0] = tt;
            const float norm = (float)sqrt(tt);
            float coef = max_norm / (norm + 1e-6f);
            coef = coef > 1.0f ? 1.0f : coef;  // NaN passes through, like torch.clamp
            out[0] = norm;
            out[1] = coef;
            counter[0] = 0u;
        }
    }
}

// adam_chunk + clearing the gradient vectors that were non-zero (most table rows get no gradient; A/B
// measured against rewriting every vector: 1.47-1.52 vs 1.52-1.56 ms over 268M parameters)
__device__ __forceinline__ void adam_chunk_zero(float* p, float* g, float* m, float* v, int64_t n, float scale,
                                                const GroupK& k) {
    const uintptr_t align = reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                            reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v);
    int64_t done = 0;
    if ((align & 15) == 0) {
        const int64_t n4 = n >> 2;
        f4* p4 = reinterpret_cast<f4*>(p);
        f4* g4 = reinterpret_cast<f4*>(g);
        f4* m4 = reinterpret_cast<f4*>(m);
        f4* v4 = reinterpret_cast<f4*>(v);
        const f4 zero = 0.0f;
        int64_t i = threadIdx.x;
        for (; i + (kUnroll - 1) * kThreads < n4; i += kUnroll * kThreads) {
            f4 pp[kUnroll], gg[kUnroll], mm[kUnroll], vv[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                pp[u] = ldv(&p4[i + u * kThreads]);
                gg[u] = ldv(&g4[i + u * kThreads]);
                mm[u] = ldv(&m4[i + u * kThreads]);
                vv[u] = ldv(&v4[i + u * kThreads]);
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const bool nz = gg[u][0] != 0.0f || gg[u][1] != 0.0f || gg[u][2] != 0.0f || gg[u][3] != 0.0f;
                adam_vec(pp[u], gg[u], mm[u], vv[u], scale, k);
                stv(&p4[i + u * kThreads], pp[u]);
                stv(&m4[i + u * kThreads], mm[u]);
                stv(&v4[i + u * kThreads], vv[u]);
                if (nz) stv(&g4[i + u * kThreads], zero);
            }
        }
        for (; i < n4; i += kThreads) {
            f4 pp = ldv(&p4[i]), mm = ldv(&m4[i]), vv = ldv(&v4[i]);
            const f4 gg = ldv(&g4[i]);
            const bool nz = gg[0] != 0.0f || gg[1] != 0.0f || gg[2] != 0.0f || gg[3] != 0.0f;
            adam_vec(pp, gg, mm, vv, scale, k);
            stv(&p4[i], pp);
            stv(&m4[i], mm);
            stv(&v4[i], vv);
            if (nz) stv(&g4[i], zero);
        }
        done = n4 << 2;
    }
    for (int64_t i = done + threadIdx.x; i < n; i += kThreads) {
        float a = p[i], b = m[i], e = v[i];
        adam_elem(a, g[i], b, e, scale, k);
        p[i] = a; m[i] = b; v[i] = e;
        g[i] = 0.0f;
    }
}

// Segment-mapped chunk (the sparse hash-table gradients of the routed step): a tensor whose 64-B segments
// (16 floats = 8 table rows) carry two byte maps -- now[s]: the table scatter added into segment s this
// step; ever[s]: segment s was updated before.  A segment neither touched now nor ever holds m = v = g = 0,
// where torch's Adam (weight_decay 0) leaves p, m, v bit-identical (m' = 0, v' = 0, p' = p + (-step * 0) /
// eps = p): it is skipped, nothing read or written.  A segment not touched now has g = 0 (the gradient
// buffer is cleared after every use): its update reads p, m, v only.  A vector = 4 floats, so segment
// s = vector / 4; the 4 vectors of a segment are 4 consecutive lanes of one wave-instruction (the map
// loads precede the map stores for all of them); the first lane updates the maps.  chunk base is a
// multiple of ACN_OPTIM_CHUNK floats (segment aligned).
#ifndef ACN_ADAM_MAP_PIPE
#define ACN_ADAM_MAP_PIPE 0  // adam_chunk_seg: next iteration's map bytes loaded ahead of this iteration's data
#endif
__device__ __forceinline__ bool seg_live(uint8_t nw, uint8_t ev, int phase) {
    return phase == 0 ? (nw | ev) != 0 : (phase == 1 ? (ev != 0 && nw == 0) : nw != 0);
}

// phase 0: every live segment (now | ever); phase 1 (early pass): only segments touched before but not now --
// their gradient is zero, so the update needs neither the gradient nor the clip coefficient and the maps stay;
// phase 2 (late pass): only the segments touched now (gradient read and cleared, maps updated).
__device__ __forceinline__ void adam_chunk_seg(float* p, float* g, float* m, float* v, int64_t n, float scale,
                                               const GroupK& k, uint8_t* __restrict__ now, uint8_t* __restrict__ ever,
                                               bool clear, int phase = 0) {
    f4* p4 = reinterpret_cast<f4*>(p);
    f4* g4 = reinterpret_cast<f4*>(g);
    f4* m4 = reinterpret_cast<f4*>(m);
    f4* v4 = reinterpret_cast<f4*>(v);
    const int64_t n4 = n >> 2;   // n is a multiple of 16 (checked by the host)
    const f4 zero = 0.0f;
    int64_t i = threadIdx.x;
    // kUnroll vectors per thread per iteration: every map byte first, then all their p / m / v / g loads in
    // flight together (the one-vector loop waited on the map load before each data load: 4.7 TB/s)
#if ACN_ADAM_MAP_PIPE
    // the map bytes of the NEXT iteration are loaded before this iteration's data loads: the compiler may not
    // move them above this iteration's map stores itself (uint8_t stores alias anything), so without this
    // every iteration waited for two dependent memory round trips (map, then data) instead of one.  The
    // prefetched bytes belong to other segments than the ones this iteration clears, so values are unchanged.
    uint8_t nx_nw[kUnroll], nx_ev[kUnroll];
    if (i + (kUnroll - 1) * kThreads < n4) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t sgi = (i + u * kThreads) >> 2;
            nx_nw[u] = now[sgi];
            nx_ev[u] = ever[sgi];
        }
    }
#endif
    for (; i + (kUnroll - 1) * kThreads < n4; i += kUnroll * kThreads) {
        uint8_t nw[kUnroll], ev[kUnroll];
#if ACN_ADAM_MAP_PIPE
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            nw[u] = nx_nw[u];
            ev[u] = nx_ev[u];
        }
        const int64_t inx = i + kUnroll * kThreads;
        if (inx + (kUnroll - 1) * kThreads < n4) {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int64_t sgi = (inx + u * kThreads) >> 2;
                nx_nw[u] = now[sgi];
                nx_ev[u] = ever[sgi];
            }
        }
#else
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t sgi = (i + u * kThreads) >> 2;
            nw[u] = now[sgi];
            ev[u] = ever[sgi];
        }
#endif
        f4 pp[kUnroll], mm[kUnroll], vv[kUnroll], gg[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t iv = i + u * kThreads;
            if (seg_live(nw[u], ev[u], phase)) {
                pp[u] = ldv(&p4[iv]);
                mm[u] = ldv(&m4[iv]);
                vv[u] = ldv(&v4[iv]);
                gg[u] = nw[u] ? ldv(&g4[iv]) : zero;
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t iv = i + u * kThreads;
            if (seg_live(nw[u], ev[u], phase)) {
                adam_vec(pp[u], gg[u], mm[u], vv[u], scale, k);
                stv(&p4[iv], pp[u]);
                stv(&m4[iv], mm[u]);
                stv(&v4[iv], vv[u]);
                if (clear && nw[u] && (gg[u][0] != 0.0f || gg[u][1] != 0.0f || gg[u][2] != 0.0f || gg[u][3] != 0.0f))
                    stv(&g4[iv], zero);
            }
            if (phase != 1 && (iv & 3) == 0 && nw[u]) {
                now[iv >> 2] = 0;
                if (!ev[u]) ever[iv >> 2] = 1;
            }
        }
    }
    for (; i < n4; i += kThreads) {
        const int64_t sgi = i >> 2;
        const uint8_t nw = now[sgi], ev = ever[sgi];
        if (seg_live(nw, ev, phase)) {
            f4 pp = ldv(&p4[i]), mm = ldv(&m4[i]), vv = ldv(&v4[i]);
            const f4 gg = nw ? ldv(&g4[i]) : zero;
            adam_vec(pp, gg, mm, vv, scale, k);
            stv(&p4[i], pp);
            stv(&m4[i], mm);
            stv(&v4[i], vv);
            if (clear && nw && (gg[0] != 0.0f || gg[1] != 0.0f || gg[2] != 0.0f || gg[3] != 0.0f)) stv(&g4[i], zero);
        }
        if (phase != 1 && (i & 3) == 0 && nw) {
            now[sgi] = 0;
            if (!ev) ever[sgi] = 1;
        }
    }
}

#ifndef ACN_ADAM_SEG_LDS
#define ACN_ADAM_SEG_LDS 0  // 1: segment-mapped chunks through an LDS list of their live segments (measured slower)
#endif
// The same update as adam_chunk_seg, with the chunk's live segments (now | ever) first compacted into an LDS
// list (ascending within each 64-segment ballot group), so that every lane of every wave-instruction moves a
// live vector: adam_chunk_seg leaves the lanes of dead segments idle (40% at C5's 60% ever-touched tables),
// which caps the bytes in flight per CU below what HBM needs.  Each vector sees exactly adam_chunk_seg's
// arithmetic (bitwise the dense update); the lists live in LDS only (nothing kept between steps).
__device__ __forceinline__ void adam_chunk_seg_lds(float* p, float* g, float* m, float* v, int64_t n, float scale,
                                                   const GroupK& k, uint8_t* __restrict__ now,
                                                   uint8_t* __restrict__ ever, bool clear) {
    __shared__ uint16_t lst[ACN_OPTIM_CHUNK / 16];
    __shared__ uint8_t flg[ACN_OPTIM_CHUNK / 16];   // bit 0: touched now, bit 1: touched before
    __shared__ int cnt;
    const int nseg = (int)(n >> 4);   // n is a multiple of 16 (checked by the host)
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    for (int s0 = 0; s0 < nseg; s0 += kThreads) {
        const int sg = s0 + (int)threadIdx.x;
        uint8_t nw = 0, ev = 0;
        if (sg < nseg) {
            nw = now[sg];
            ev = ever[sg];
        }
        const bool live = (nw | ev) != 0;
        const uint64_t b = __ballot(live);
        int base = 0;
        if (lane == 0 && b != 0) base = atomicAdd(&cnt, (int)__popcll(b));
        base = __shfl(base, 0);
        if (live) {
            const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            lst[pos] = (uint16_t)sg;
            flg[pos] = (uint8_t)((nw ? 1 : 0) | (ev ? 2 : 0));
        }
    }
    __syncthreads();
    const int nv = cnt * 4;   // 4 vectors per segment, consecutive lanes
    f4* p4 = reinterpret_cast<f4*>(p);
    f4* g4 = reinterpret_cast<f4*>(g);
    f4* m4 = reinterpret_cast<f4*>(m);
    f4* v4 = reinterpret_cast<f4*>(v);
    const f4 zero = 0.0f;
    int i = threadIdx.x;
    for (; i + (kUnroll - 1) * kThreads < nv; i += kUnroll * kThreads) {
        int64_t iv[kUnroll];
        uint8_t fl[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int j = i + u * kThreads;
            iv[u] = (int64_t)lst[j >> 2] * 4 + (j & 3);
            fl[u] = flg[j >> 2];
        }
        f4 pp[kUnroll], mm[kUnroll], vv[kUnroll], gg[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            pp[u] = ldv(&p4[iv[u]]);
            mm[u] = ldv(&m4[iv[u]]);
            vv[u] = ldv(&v4[iv[u]]);
            gg[u] = (fl[u] & 1) ? ldv(&g4[iv[u]]) : zero;
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            adam_vec(pp[u], gg[u], mm[u], vv[u], scale, k);
            stv(&p4[iv[u]], pp[u]);
            stv(&m4[iv[u]], mm[u]);
            stv(&v4[iv[u]], vv[u]);
            if (clear && (fl[u] & 1) && (gg[u][0] != 0.0f || gg[u][1] != 0.0f || gg[u][2] != 0.0f || gg[u][3] != 0.0f))
                stv(&g4[iv[u]], zero);
            if ((iv[u] & 3) == 0 && (fl[u] & 1)) {
                now[iv[u] >> 2] = 0;
                if (!(fl[u] & 2)) ever[iv[u] >> 2] = 1;
            }
        }
    }
    for (; i < nv; i += kThreads) {
        const int64_t ivs = (int64_t)lst[i >> 2] * 4 + (i & 3);
        const uint8_t fs = flg[i >> 2];
        f4 pp = ldv(&p4[ivs]), mm = ldv(&m4[ivs]), vv = ldv(&v4[ivs]);
        const f4 gg = (fs & 1) ? ldv(&g4[ivs]) : zero;
        adam_vec(pp, gg, mm, vv, scale, k);
        stv(&p4[ivs], pp);
        stv(&m4[ivs], mm);
        stv(&v4[ivs], vv);
        if (clear && (fs & 1) && (gg[0] != 0.0f || gg[1] != 0.0f || gg[2] != 0.0f || gg[3] != 0.0f)) stv(&g4[ivs], zero);
        if ((ivs & 3) == 0 && (fs & 1)) {
            now[ivs >> 2] = 0;
            if (!(fs & 2)) ever[ivs >> 2] = 1;
        }
    }
}

#ifdef ACN_ADAM_WPE   // occupancy experiment: waves per SIMD for adam_slots_kernel (compiler default 3 at 166 VGPRs)
#define ACN_ADAM_SLOTS_ATTR __attribute__((amdgpu_waves_per_eu(ACN_ADAM_WPE, ACN_ADAM_WPE)))
#else
#define ACN_ADAM_SLOTS_ATTR
#endif
__global__ void __launch_bounds__(kThreads) ACN_ADAM_SLOTS_ATTR adam_slots_kernel(const acn_param_desc* __restrict__ descs,
                                                              const int32_t* __restrict__ chunk_tensor,
                                                              const int32_t* __restrict__ flags,
                                                              const GroupK* __restrict__ table, int ngroups,
                                                              int table_steps, const int32_t* __restrict__ step_dev,
                                                              const int64_t* __restrict__ seg, int K,
                                                              const float* __restrict__ grad_scale,
                                                              uint8_t* const* __restrict__ segmaps, int phase) {
    const int t = chunk_tensor[blockIdx.x];
    const acn_param_desc d = descs[t];
    const int f = flags[t], slot = f & 0xffff;
    if (d.grad == nullptr) return;
    const bool mapped = segmaps != nullptr && segmaps[2 * t] != nullptr;
    if (phase == 1 && !mapped) return;   // the early pass touches only the mapped tables' untouched segments
    if (seg != nullptr && seg[K] < 0) {
        if (phase == 1) return;
        // a skipped step (AMP found_inf, an overflowed bounded exchange): parameters and moments stay, but the
        // gradients this pass would have cleared are cleared (and the segment marks reset) so the next step
        // starts from zero as after an update
        if (f & kSlotZero) {
            const int64_t base = (int64_t)(blockIdx.x - d.first_chunk) * ACN_OPTIM_CHUNK;
            const int64_t n = d.numel - base < ACN_OPTIM_CHUNK ? d.numel - base : ACN_OPTIM_CHUNK;
            float* g = const_cast<float*>(d.grad) + base;
            uint8_t* now = segmaps ? segmaps[2 * t] : nullptr;
            for (int64_t i = threadIdx.x; i < n; i += kThreads)
                if ((now == nullptr || now[(base + i) >> 4]) && g[i] != 0.0f) g[i] = 0.0f;
            __syncthreads();
            if (now)
                for (int64_t sg = threadIdx.x; sg < (n + 15) >> 4; sg += kThreads) now[(base >> 4) + sg] = 0;
        }
        return;
    }
    if (!slot_active(seg, K, slot)) return;
    const int row = step_dev[slot] - 1;
    if (row < 0 || row >= table_steps) return;  // outside the uploaded table: the host refills first
    const GroupK k = table[(int64_t)row * ngroups + d.group];
    const float scale = grad_scale ? grad_scale[1] : 1.0f;
    const int64_t base = (int64_t)(blockIdx.x - d.first_chunk) * ACN_OPTIM_CHUNK;
    const int64_t n = d.numel - base < ACN_OPTIM_CHUNK ? d.numel - base : ACN_OPTIM_CHUNK;
    float* p = d.param + base;
    float* g = const_cast<float*>(d.grad) + base;
    float* m = d.exp_avg + base;
    float* v = d.exp_avg_sq + base;
    uint8_t* smap = segmaps ? segmaps[2 * t] : nullptr;
    if (smap) {
        const int64_t s0 = base >> 4, nseg = (d.numel + 15) >> 4;
#if ACN_ADAM_SEG_LDS  // (phase 0 only)
        adam_chunk_seg_lds(p, g, m, v, n, scale, k, smap + s0, segmaps[2 * t + 1] + s0, (f & kSlotZero) != 0);
#else
        if (phase != 0)
            adam_chunk_seg(p, g, m, v, n, scale, k, smap + s0, segmaps[2 * t + 1] + s0, (f & kSlotZero) != 0, phase);
        else
            adam_chunk_seg(p, g, m, v, n, scale, k, smap + s0, segmaps[2 * t + 1] + s0, (f & kSlotZero) != 0);
#endif
        (void)nseg;
    } else if (f & kSlotZero) {
        adam_chunk_zero(p, g, m, v, n, scale, k);
    } else {
        adam_chunk(p, g, m, v, n, scale, k);
    }
}

// python-float (double) scalars of _single_tensor_adam for one group at one step, cast to fp32 where
// they meet tensors
void group_consts(const acn_adam_group& g, GroupK& k) {
    const double b1 = g.beta1, b2 = g.beta2;
    const double bc1 = 1.0 - pow(b1, (double)g.step);
    const double bc2 = 1.0 - pow(b2, (double)g.step);
    const double step_size = (double)g.lr / bc1;
    k.lr_neg_step = (float)(-step_size);
    k.w1 = (float)(1.0 - b1);
    k.beta2 = (float)b2;
    k.one_m_beta2 = (float)(1.0 - b2);
    k.bc2s = (float)sqrt(bc2);
    k.eps = (float)g.eps;
    k.wd = (float)g.weight_decay;
}

// descriptors as kernel arguments -> device memory + the chunk -> tensor map (graph capture: the
// addresses are baked into the captured node, no host-to-device copy)
constexpr int kPlanMax = 64;
struct PlanArg {
    acn_param_desc d[kPlanMax];
};

__global__ void __launch_bounds__(kThreads) plan_kernel(PlanArg pa, int n, acn_param_desc* __restrict__ out,
                                                        int32_t* __restrict__ chunk_tensor, int64_t nchunks) {
    for (int i = threadIdx.x; i < n; i += kThreads) out[i] = pa.d[i];
    for (int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x; c < nchunks; c += (int64_t)gridDim.x * kThreads) {
        int t = 0;
        while (t + 1 < n && pa.d[t + 1].first_chunk <= c) ++t;
        chunk_tensor[c] = t;
    }
}

}  // namespace

extern "C" int acn_optim_plan_device(const acn_param_desc* host_descs, int n, acn_param_desc* descs,
                                     int32_t* chunk_tensor, int64_t nchunks, void* stream) {
    ACN_REQUIRE(n >= 1 && n <= kPlanMax, "acn_optim_plan_device: 1 <= n <= %d tensors", kPlanMax);
    ACN_REQUIRE(host_descs && descs && chunk_tensor && nchunks >= 1, "acn_optim_plan_device: bad arguments");
    PlanArg pa{};
    for (int i = 0; i < n; ++i) pa.d[i] = host_descs[i];
    const unsigned blocks = (unsigned)((nchunks + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(plan_kernel, dim3(blocks < 1 ? 1 : blocks), dim3(kThreads), 0, (hipStream_t)stream, pa, n,
                       descs, chunk_tensor, nchunks);
    return acn_check_launch("acn_optim_plan_device");
}

extern "C" size_t acn_adam_table_bytes(int ngroups, int steps) {
    return (size_t)ngroups * (size_t)steps * sizeof(GroupK);
}

extern "C" int acn_adam_table_fill(const acn_adam_group* groups, int ngroups, int first_step, int steps, void* out,
                                   size_t bytes) {
    ACN_REQUIRE(groups && out, "acn_adam_table_fill: NULL pointer");
    ACN_REQUIRE(ngroups >= 1 && ngroups <= ACN_OPTIM_MAX_GROUPS && steps >= 1 && first_step >= 1,
                "acn_adam_table_fill: bad ngroups / steps / first_step");
    ACN_REQUIRE(bytes >= acn_adam_table_bytes(ngroups, steps), "acn_adam_table_fill: buffer too small");
    GroupK* t = reinterpret_cast<GroupK*>(out);
    for (int s = 0; s < steps; ++s)
        for (int i = 0; i < ngroups; ++i) {
            acn_adam_group g = groups[i];
            g.step = first_step + s;
            group_consts(g, t[(size_t)s * ngroups + i]);
        }
    return ACN_OK;
}

extern "C" int acn_adam_step_table(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                                   const void* table, int ngroups, int32_t* step_dev, int first_step, int table_steps,
                                   const float* grad_scale, void* stream) {
    ACN_REQUIRE(nchunks >= 0 && nchunks <= 0x7fffffff, "acn_adam_step_table: bad nchunks");
    ACN_REQUIRE(table && step_dev && ngroups >= 1 && ngroups <= ACN_OPTIM_MAX_GROUPS && table_steps >= 1,
                "acn_adam_step_table: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(bump_kernel, dim3(1), dim3(1), 0, s, step_dev);
    if (nchunks > 0) {
        ACN_REQUIRE(descs && chunk_tensor, "acn_adam_step_table: NULL pointer");
        hipLaunchKernelGGL(adam_table_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, s, descs, chunk_tensor,
                           reinterpret_cast<const GroupK*>(table), ngroups, step_dev, first_step, table_steps,
                           grad_scale);
    }
    return acn_check_launch("acn_adam_step_table");
}

extern "C" int acn_grad_sumsq(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                              double* partials, double* total, void* stream) {
    ACN_REQUIRE(nchunks >= 0, "acn_grad_sumsq: nchunks must be >= 0");
    ACN_REQUIRE(total, "acn_grad_sumsq: NULL total");
    hipStream_t s = (hipStream_t)stream;
    if (nchunks == 0) {
        const hipError_t e = hipMemsetAsync(total, 0, sizeof(double), s);
        return e == hipSuccess ? ACN_OK : acn_set_error((int)e, "acn_grad_sumsq: %s", hipGetErrorString(e));
    }
    ACN_REQUIRE(descs && chunk_tensor && partials, "acn_grad_sumsq: NULL pointer");
    ACN_REQUIRE(nchunks <= 0x7fffffff, "acn_grad_sumsq: too many chunks");
    hipLaunchKernelGGL(sumsq_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, s, descs, chunk_tensor, partials);
    hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kThreads), 0, s, partials, nchunks, total, (double*)nullptr);
    return acn_check_launch("acn_grad_sumsq");
}

extern "C" int acn_clip_coef(const double* total_sumsq, float max_norm, float* out, void* stream) {
    ACN_REQUIRE(total_sumsq && out, "acn_clip_coef: NULL pointer");
    hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, total_sumsq, max_norm, out);
    return acn_check_launch("acn_clip_coef");
}

extern "C" int acn_amp_unscale_coef(const double* total_sumsq, float max_norm, float* scale, int32_t* growth_tracker,
                                    float* found_inf, float growth, float backoff, int growth_interval, float* out,
                                    int64_t* seg, int K, void* stream) {
    ACN_REQUIRE(total_sumsq && scale && growth_tracker && found_inf && out && growth_interval >= 1 &&
                    (seg == nullptr || K >= 0),
                "acn_amp_unscale_coef: bad arguments");
    hipLaunchKernelGGL(amp_unscale_coef_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, total_sumsq, max_norm, scale,
                       growth_tracker, found_inf, growth, backoff, growth_interval, out, seg, K);
    return acn_check_launch("acn_amp_unscale_coef");
}

extern "C" int acn_adam_step(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                             const acn_adam_group* groups, int ngroups, const float* grad_scale, void* stream) {
    ACN_REQUIRE(nchunks >= 0 && nchunks <= 0x7fffffff, "acn_adam_step: bad nchunks");
    if (nchunks == 0) return ACN_OK;
    ACN_REQUIRE(descs && chunk_tensor && groups, "acn_adam_step: NULL pointer");
    ACN_REQUIRE(ngroups >= 1 && ngroups <= ACN_OPTIM_MAX_GROUPS, "acn_adam_step: ngroups must be in [1, %d]",
                ACN_OPTIM_MAX_GROUPS);
    GroupsArg ga{};
    for (int i = 0; i < ngroups; ++i) {
        ACN_REQUIRE(groups[i].step >= 1, "acn_adam_step: group %d step must be >= 1 (incremented before the update)",
                    i);
        group_consts(groups[i], ga.g[i]);
    }
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, (hipStream_t)stream, descs,
                       chunk_tensor, ga, grad_scale);
    return acn_check_launch("acn_adam_step");
}

extern "C" int acn_grad_sumsq_slots(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                                    const int32_t* flags, const int64_t* seg, int K, double* partials, double* total,
                                    void* stream) {
    return acn_grad_sumsq_slots_ex(descs, chunk_tensor, nchunks, flags, seg, K, partials, total, nullptr, stream);
}

extern "C" int acn_grad_sumsq_slots_ex(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                                       const int32_t* flags, const int64_t* seg, int K, double* partials, double* total,
                                       double* extra, void* stream) {
    ACN_REQUIRE(nchunks >= 1 && nchunks <= 0x7fffffff && descs && chunk_tensor && flags && partials && total,
                "acn_grad_sumsq_slots: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(sumsq_slots_kernel<false>, dim3((unsigned)nchunks), dim3(kThreads), 0, s, descs, chunk_tensor,
                       flags, seg, K, partials, nullptr, nullptr, 0.0f, nullptr, nullptr);
    hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kThreads), 0, s, partials, nchunks, total, extra);
    return acn_check_launch("acn_grad_sumsq_slots");
}

extern "C" int acn_grad_clip_slots(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                                   const int32_t* flags, const int64_t* seg, int K, double* partials, double* total,
                                   double* extra, float max_norm, float* out, unsigned int* counter, void* stream) {
    ACN_REQUIRE(nchunks >= 1 && nchunks <= 0x7fffffff && descs && chunk_tensor && flags && partials && total && out &&
                    counter,
                "acn_grad_clip_slots: bad arguments");
    hipLaunchKernelGGL(sumsq_slots_kernel<true>, dim3((unsigned)nchunks), dim3(kThreads), 0, (hipStream_t)stream, descs,
                       chunk_tensor, flags, seg, K, partials, total, extra, max_norm, out, counter);
    return acn_check_launch("acn_grad_clip_slots");
}

extern "C" int acn_adam_step_slots(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                                   const int32_t* flags, const void* table, int ngroups, int table_steps,
                                   int32_t* step_dev, int nslots, const int64_t* seg, int K, const float* grad_scale,
                                   void* stream) {
    ACN_REQUIRE(nchunks >= 1 && nchunks <= 0x7fffffff && descs && chunk_tensor && flags && table && step_dev,
                "acn_adam_step_slots: bad arguments");
    ACN_REQUIRE(ngroups >= 1 && ngroups <= ACN_OPTIM_MAX_GROUPS && table_steps >= 1 && nslots >= 1 && nslots <= 1024,
                "acn_adam_step_slots: bad ngroups / table_steps / nslots");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(bump_slots_kernel, dim3(1), dim3(1024), 0, s, step_dev, seg, K, nslots);
    hipLaunchKernelGGL(adam_slots_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, s, descs, chunk_tensor, flags,
                       reinterpret_cast<const GroupK*>(table), ngroups, table_steps, step_dev, seg, K, grad_scale,
                       (uint8_t* const*)nullptr, 0);
    return acn_check_launch("acn_adam_step_slots");
}

extern "C" int acn_adam_step_slots_segmap(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                                          const int32_t* flags, const void* table, int ngroups, int table_steps,
                                          int32_t* step_dev, int nslots, const int64_t* seg, int K,
                                          const float* grad_scale, uint8_t* const* segmaps, void* stream) {
    ACN_REQUIRE(nchunks >= 1 && nchunks <= 0x7fffffff && descs && chunk_tensor && flags && table && step_dev && segmaps,
                "acn_adam_step_slots_segmap: bad arguments");
    ACN_REQUIRE(ngroups >= 1 && ngroups <= ACN_OPTIM_MAX_GROUPS && table_steps >= 1 && nslots >= 1 && nslots <= 1024,
                "acn_adam_step_slots_segmap: bad ngroups / table_steps / nslots");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(bump_slots_kernel, dim3(1), dim3(1024), 0, s, step_dev, seg, K, nslots);
    hipLaunchKernelGGL(adam_slots_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, s, descs, chunk_tensor, flags,
                       reinterpret_cast<const GroupK*>(table), ngroups, table_steps, step_dev, seg, K, grad_scale,
                       segmaps, 0);
    return acn_check_launch("acn_adam_step_slots_segmap");
}

extern "C" int acn_adam_step_slots_segmap_phase(const acn_param_desc* descs, const int32_t* chunk_tensor,
                                                int64_t nchunks, const int32_t* flags, const void* table, int ngroups,
                                                int table_steps, int32_t* step_dev, int nslots, const int64_t* seg,
                                                int K, const float* grad_scale, uint8_t* const* segmaps, int phase,
                                                void* stream) {
    ACN_REQUIRE(nchunks >= 1 && nchunks <= 0x7fffffff && descs && chunk_tensor && flags && table && step_dev && segmaps,
                "acn_adam_step_slots_segmap_phase: bad arguments");
    ACN_REQUIRE(ngroups >= 1 && ngroups <= ACN_OPTIM_MAX_GROUPS && table_steps >= 1 && nslots >= 1 && nslots <= 1024,
                "acn_adam_step_slots_segmap_phase: bad ngroups / table_steps / nslots");
    ACN_REQUIRE(phase == 1 || phase == 2, "acn_adam_step_slots_segmap_phase: phase must be 1 or 2, got %d", phase);
    hipStream_t s = (hipStream_t)stream;
    if (phase == 1) hipLaunchKernelGGL(bump_slots_kernel, dim3(1), dim3(1024), 0, s, step_dev, seg, K, nslots);
    hipLaunchKernelGGL(adam_slots_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, s, descs, chunk_tensor, flags,
                       reinterpret_cast<const GroupK*>(table), ngroups, table_steps, step_dev, seg, K, grad_scale,
                       segmaps, phase);
    return acn_check_launch("acn_adam_step_slots_segmap_phase");
}
