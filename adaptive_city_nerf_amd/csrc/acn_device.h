// acn_device.h -- device-side building blocks shared by the kernels (gfx950, wave64).
//
// All files are compiled with -ffp-contract=off: every a*b+c here rounds twice unless fmaf() is
// written explicitly, which is what keeps the hash-grid / SH / ray-geometry arithmetic bit-exact
// with the reference's chains of elementwise torch ops.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace acn {

constexpr uint32_t kP1 = 2654435761u;  // models/encodings.py:275 hash primes {1, 2654435761, 805459861}
constexpr uint32_t kP2 = 805459861u;

// models/trunc_exp.py:22-41 (float32 clamp +-88.722839111)
__device__ __forceinline__ float trunc_exp(float x) {
    const float m = 88.722839111f;
    x = x < -m ? -m : x;
    x = x > m ? m : x;   // NaN passes through, as torch.clamp
    return expf(x);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// torch.norm(dim=-1) of a 3-vector on CPU == sqrt(fma(z,z, fma(y,y, x*x)))
__device__ __forceinline__ float norm3(float x, float y, float z) {
    return sqrtf(fmaf(z, z, fmaf(y, y, x * x)));
}

// torch.clamp_min / clamp keeping NaN (torch semantics), unlike fmaxf/fminf
__device__ __forceinline__ float clamp_min_nan(float v, float lo) { return v < lo ? lo : v; }
__device__ __forceinline__ float clamp_nan(float v, float lo, float hi) {
    v = v < lo ? lo : v;
    return v > hi ? hi : v;
}

// lane l's double (l wave-uniform: two scalar readlanes)
__device__ __forceinline__ double lane_f64(double v, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// compute_mse_loss in color_space "linear" (nerfs/losses.py:10-32, color_space.py:13-19, 22-66): pred.clamp(0,1)
// against gt.clamp(0,1) -> srgb_to_linear -> clamp(0,1); float scalars and powf as the torch ops (loss.hip and
// the fused training compositing in render.hip)
__device__ __forceinline__ float clamp01(float x) { return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x); }
__device__ __forceinline__ float srgb_to_linear(float x) {
    return x <= 0.04045f ? x / 12.92f : powf((x + 0.055f) / 1.055f, 2.4f);
}
__device__ __forceinline__ float gt_linear(float g) { return clamp01(srgb_to_linear(clamp01(g))); }

// get_ray_directions (nerfs/ray_sampling.py:122-136) for pixel (i, j)
__device__ __forceinline__ void pixel_dir(int i, int j, float fx, float fy, float cx, float cy, int center,
                                          float& dx, float& dy, float& dz) {
    float fi = (float)i, fj = (float)j;
    if (center) { fi = fi + 0.5f; fj = fj + 0.5f; }
    dx = (fi - cx) / fx;
    dy = -((fj - cy) / fy);
    dz = -1.0f;
    const float n = clamp_min_nan(norm3(dx, dy, dz), 1e-12f);
    dx = dx / n; dy = dy / n; dz = dz / n;
}

// SceneBox.ray_aabb_intersect (scene_box.py:81-107): slab test with eps-signed inverse,
// clamp to [0, max_bound], misses (tmax <= tmin) tagged with invalid_value
__device__ __forceinline__ void slab(const float* o, const float* d, const float* aabb, float eps, float max_bound,
                                     float invalid_value, float& tmin, float& tmax) {
    float t0m = -INFINITY, t1m = INFINITY;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        float rd = d[r];
        if (fabsf(rd) < eps) rd = (rd >= 0.0f) ? eps : -eps;
        const float inv = 1.0f / rd;
        const float t0 = (aabb[r] - o[r]) * inv, t1 = (aabb[3 + r] - o[r]) * inv;
        t0m = fmaxf(t0m, fminf(t0, t1));
        t1m = fminf(t1m, fmaxf(t0, t1));
    }
    tmin = fminf(fmaxf(t0m, 0.0f), max_bound);
    tmax = fminf(fmaxf(t1m, 0.0f), max_bound);
    if (tmax <= tmin) { tmin = invalid_value; tmax = invalid_value; }
}

// torch.linspace(0, 1, S)[i] (CPU and GPU kernels: start + step*i below the middle, end - step*(S-1-i)
// above, each evaluated as one fma)
__device__ __forceinline__ float linspace01(int i, int S) {
    if (S == 1) return 0.0f;
    const float step = 1.0f / (float)(S - 1);
    return i < S / 2 ? fmaf(step, (float)i, 0.0f) : fmaf(-step, (float)(S - 1 - i), 1.0f);
}

// torch.lerp(start, end, w) (ATen Lerp.h; the CPU vector kernel and the GPU kernel both end in one fma)
__device__ __forceinline__ float lerp_t(float start, float end, float w) {
    return fabsf(w) < 0.5f ? fmaf(w, end - start, start) : fmaf(w - 1.0f, end - start, end);
}

// models/encodings.py:27-81 components_from_spherical_harmonics, float32 op order of the torch
// expressions (scalar * tensor evaluated left to right).  kz: an opaque +0.0f (c + 0.0f == c for every nonzero
// coefficient) from callers inside a loop, so the coefficient pairs of packed multiplies are formed per call instead
// of being hoisted out of the loop into VGPRs (render_ws_kernel spilled them); 0 elsewhere.
template <int DEGREE>
__device__ __forceinline__ void sh_components(float x, float y, float z, float* c, float kz = 0.0f) {
    const float xx = x * x, yy = y * y, zz = z * z;
    c[0] = (0.28209479177387814f + kz);
    if (DEGREE > 0) {
        c[1] = (0.4886025119029199f + kz) * y;
        c[2] = (0.4886025119029199f + kz) * z;
        c[3] = (0.4886025119029199f + kz) * x;
    }
    if (DEGREE > 1) {
        c[4] = ((1.0925484305920792f + kz) * x) * y;
        c[5] = ((1.0925484305920792f + kz) * y) * z;
        c[6] = (0.9461746957575601f + kz) * zz - (0.31539156525251999f + kz);
        c[7] = ((1.0925484305920792f + kz) * x) * z;
        c[8] = (0.5462742152960396f + kz) * (xx - yy);
    }
    if (DEGREE > 2) {
        c[9] = ((0.5900435899266435f + kz) * y) * (3.0f * xx - yy);
        c[10] = (((2.890611442640554f + kz) * x) * y) * z;
        c[11] = ((0.4570457994644658f + kz) * y) * (5.0f * zz - (1.0f + kz));
        c[12] = ((0.3731763325901154f + kz) * z) * (5.0f * zz - (3.0f + kz));
        c[13] = ((0.4570457994644658f + kz) * x) * (5.0f * zz - (1.0f + kz));
        c[14] = ((1.445305721320277f + kz) * z) * (xx - yy);
        c[15] = ((0.5900435899266435f + kz) * x) * (xx - (3.0f + kz) * yy);
    }
    if (DEGREE > 3) {
        c[16] = (((2.5033429417967046f + kz) * x) * y) * (xx - yy);
        c[17] = (((1.7701307697799304f + kz) * y) * z) * (3.0f * xx - yy);
        c[18] = (((0.9461746957575601f + kz) * x) * y) * (7.0f * zz - (1.0f + kz));
        c[19] = (((0.6690465435572892f + kz) * y) * z) * (7.0f * zz - (3.0f + kz));
        c[20] = (0.10578554691520431f + kz) * (((35.0f * zz) * zz - (30.0f + kz) * zz) + (3.0f + kz));
        c[21] = (((0.6690465435572892f + kz) * x) * z) * (7.0f * zz - (3.0f + kz));
        c[22] = ((0.47308734787878004f + kz) * (xx - yy)) * (7.0f * zz - (1.0f + kz));
        c[23] = (((1.7701307697799304f + kz) * x) * z) * (xx - (3.0f + kz) * yy);
        c[24] = (0.6258357354491761f + kz) * (xx * (xx - (3.0f + kz) * yy) - yy * (3.0f * xx - yy));
    }
}

// SHEncoder.forward (encodings.py:144-151): d / norm(d).clamp_min(1e-9), then components
template <int DEGREE>
__device__ __forceinline__ void sh_encode(float dx, float dy, float dz, float* c, float kz = 0.0f) {
    const float n = clamp_min_nan(norm3(dx, dy, dz), 1e-9f);
    sh_components<DEGREE>(dx / n, dy / n, dz / n, c, kz);
}

// One level of HashGridEncoder._torch_forward split in two halves so that callers can keep the
// gathers of several levels in flight: hash_issue computes the 8 corner rows and issues their
// loads, hash_finish interpolates once they have landed.  Same arithmetic as hash_level_f2.
// 8-byte table-row load with a cache policy: 0 plain, 1 non-temporal (nt), 2 L1-bypassing
// (relaxed agent-scope atomic load -> global_load_dwordx2 sc1, served by the L2)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
template <int POL>
__device__ __forceinline__ float2 ld_row(const float2* p) {
    if (POL == 1) {
        const f32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const f32x2_t*>(p));
        return make_float2(v[0], v[1]);
    }
    if (POL == 2) {
        const uint64_t u = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        return make_float2(__uint_as_float((uint32_t)u), __uint_as_float((uint32_t)(u >> 32)));
    }
    return *p;
}

struct HashPending {
    float2 f[8];
    float wx, wy, wz;
};

template <int INTERP, int POL = 0>
__device__ __forceinline__ void hash_issue(const float2* __restrict__ tl, float sx, float sy, float sz,
                                           uint32_t mask, HashPending& p) {
    if (INTERP == 0) {
        const uint32_t ix = (uint32_t)(int)rintf(sx), iy = (uint32_t)(int)rintf(sy), iz = (uint32_t)(int)rintf(sz);
        p.f[0] = ld_row<POL>(tl + ((ix ^ (iy * kP1) ^ (iz * kP2)) & mask));
        return;
    }
    const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
    float wx = sx - fx, wy = sy - fy, wz = sz - fz;
    const uint32_t x0 = (uint32_t)(int)fx;
    const uint32_t y0 = (uint32_t)(int)fy * kP1, y1 = y0 + kP1;
    const uint32_t z0 = (uint32_t)(int)fz * kP2, z1 = z0 + kP2;
    const uint32_t x1 = x0 + 1u;
    if (INTERP == 2) {
        wx = (wx * wx) * (3.0f - 2.0f * wx);
        wy = (wy * wy) * (3.0f - 2.0f * wy);
        wz = (wz * wz) * (3.0f - 2.0f * wz);
    }
    const uint32_t a00 = y0 ^ z0, a01 = y0 ^ z1, a10 = y1 ^ z0, a11 = y1 ^ z1;
#if ACN_XPAIR
    // The x-neighbours of a (y, z) corner pair hash to rows i0 = x0^a and i1 = x1^a.  For even x0,
    // i1 = i0 ^ 1: both rows sit in ONE 16-byte block, fetched by a single dwordx4 gather; only
    // lanes with odd x0 issue a second (dwordx2) gather for i1.
    const bool xodd = (x0 & 1u) != 0u;
    const uint32_t aa[4] = {a00, a01, a10, a11};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t i0 = (x0 ^ aa[c]) & mask;
        const float4 q = *reinterpret_cast<const float4*>(tl + (i0 & ~1u));
        const bool hi = (i0 & 1u) != 0u;
        p.f[2 * c] = hi ? make_float2(q.z, q.w) : make_float2(q.x, q.y);
        p.f[2 * c + 1] = hi ? make_float2(q.x, q.y) : make_float2(q.z, q.w);
    }
    if (xodd) {
#pragma unroll
        for (int c = 0; c < 4; ++c) p.f[2 * c + 1] = tl[(x1 ^ aa[c]) & mask];
    }
#else
#if ACN_DIAG_HALF_CORNERS  // diagnostic build only: 4 gathers per level (wrong values)
    p.f[0] = ld_row<POL>(tl + ((x0 ^ a00) & mask));
    p.f[2] = ld_row<POL>(tl + ((x0 ^ a01) & mask));
    p.f[4] = ld_row<POL>(tl + ((x0 ^ a10) & mask));
    p.f[6] = ld_row<POL>(tl + ((x0 ^ a11) & mask));
    p.f[1] = p.f[0]; p.f[3] = p.f[2]; p.f[5] = p.f[4]; p.f[7] = p.f[6];
#else
    p.f[0] = ld_row<POL>(tl + ((x0 ^ a00) & mask));
    p.f[1] = ld_row<POL>(tl + ((x1 ^ a00) & mask));
    p.f[2] = ld_row<POL>(tl + ((x0 ^ a01) & mask));
    p.f[3] = ld_row<POL>(tl + ((x1 ^ a01) & mask));
    p.f[4] = ld_row<POL>(tl + ((x0 ^ a10) & mask));
    p.f[5] = ld_row<POL>(tl + ((x1 ^ a10) & mask));
    p.f[6] = ld_row<POL>(tl + ((x0 ^ a11) & mask));
    p.f[7] = ld_row<POL>(tl + ((x1 ^ a11) & mask));
#endif
#endif
    p.wx = wx;
    p.wy = wy;
    p.wz = wz;
}

// FMA: c = fma(f1, w, f0 * (1 - w)) (one rounding fewer than the reference's f0*(1-w) + f1*w; used
// by the fused field, whose outputs are compared within tolerance)
#ifndef ACN_HASH_PK
#define ACN_HASH_PK 1   // hash_finish on packed fp32 vectors (render.hip is built without the SLP vectorizer)
#endif
template <int INTERP, bool FMA = false>
__device__ __forceinline__ void hash_finish(const HashPending& p, float& o0, float& o1) {
    if (INTERP == 0) {
        o0 = p.f[0].x;
        o1 = p.f[0].y;
        return;
    }
    const float wx = p.wx, wy = p.wy, wz = p.wz;
    const float ax = 1.0f - wx, ay = 1.0f - wy, az = 1.0f - wz;
#if ACN_HASH_PK
    if (!FMA) {   // both features at once on packed fp32 (v_pk_mul_f32 / v_pk_add_f32: per-component IEEE, the same
                  // roundings as the scalar chain below), written as vectors so the packing needs no SLP pass
        auto v2 = [](float2 f) { return f32x2_t{f.x, f.y}; };
        auto lerp2 = [](f32x2_t a, f32x2_t b, float w, float aw) {
            return a * f32x2_t{aw, aw} + b * f32x2_t{w, w};
        };
        const f32x2_t c00 = lerp2(v2(p.f[0]), v2(p.f[1]), wx, ax);
        const f32x2_t c01 = lerp2(v2(p.f[2]), v2(p.f[3]), wx, ax);
        const f32x2_t c10 = lerp2(v2(p.f[4]), v2(p.f[5]), wx, ax);
        const f32x2_t c11 = lerp2(v2(p.f[6]), v2(p.f[7]), wx, ax);
        const f32x2_t c0 = lerp2(c00, c10, wy, ay);
        const f32x2_t c1 = lerp2(c01, c11, wy, ay);
        const f32x2_t o = lerp2(c0, c1, wz, az);
        o0 = o[0];
        o1 = o[1];
        return;
    }
#endif
    auto lerp = [&](float a, float b, float w, float aw) { return FMA ? fmaf(b, w, a * aw) : a * aw + b * w; };
    // f index: bit0 = x1, bit1 = z1, bit2 = y1 (issue order above)
    {
        const float c00 = lerp(p.f[0].x, p.f[1].x, wx, ax);
        const float c01 = lerp(p.f[2].x, p.f[3].x, wx, ax);
        const float c10 = lerp(p.f[4].x, p.f[5].x, wx, ax);
        const float c11 = lerp(p.f[6].x, p.f[7].x, wx, ax);
        const float c0 = lerp(c00, c10, wy, ay);
        const float c1 = lerp(c01, c11, wy, ay);
        o0 = lerp(c0, c1, wz, az);
    }
    {
        const float c00 = lerp(p.f[0].y, p.f[1].y, wx, ax);
        const float c01 = lerp(p.f[2].y, p.f[3].y, wx, ax);
        const float c10 = lerp(p.f[4].y, p.f[5].y, wx, ax);
        const float c11 = lerp(p.f[6].y, p.f[7].y, wx, ax);
        const float c0 = lerp(c00, c10, wy, ay);
        const float c1 = lerp(c01, c11, wy, ay);
        o1 = lerp(c0, c1, wz, az);
    }
}

// Buffer-resource form of hash_issue/hash_finish (Linear/Smoothstep).  The x-neighbours of a
// (y, z) corner pair hash to rows i0 = x0^a and i1 = x1^a; for even x0, i1 = i0 ^ 1, so ONE
// 16-byte gather of the aligned block holding i0 returns both.  The second gather (8 bytes, row
// i1) is only needed by lanes with odd x0: the other lanes pass an out-of-range offset, which the
// buffer's range check turns into a no-op (no cache access).
#ifndef ACN_XPAIR_NOSKIP
#define ACN_XPAIR_NOSKIP 0
#endif
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
struct HashPendingX {
    u32x4_t q[4];
    u32x2_t r[4];
    float wx, wy, wz;
    uint32_t sel;  // bit c: row i0 of corner pair c is the odd row of its block; bit 4: x0 odd
};

template <int INTERP>
__device__ __forceinline__ void hash_issue_x(__amdgpu_buffer_rsrc_t rs, uint32_t lvbase, float sx, float sy, float sz,
                                             uint32_t mask, HashPendingX& p) {
    const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
    float wx = sx - fx, wy = sy - fy, wz = sz - fz;
    const uint32_t x0 = (uint32_t)(int)fx;
    const uint32_t y0 = (uint32_t)(int)fy * kP1, y1 = y0 + kP1;
    const uint32_t z0 = (uint32_t)(int)fz * kP2, z1 = z0 + kP2;
    const uint32_t x1 = x0 + 1u;
    if (INTERP == 2) {
        wx = (wx * wx) * (3.0f - 2.0f * wx);
        wy = (wy * wy) * (3.0f - 2.0f * wy);
        wz = (wz * wz) * (3.0f - 2.0f * wz);
    }
    const uint32_t aa[4] = {y0 ^ z0, y0 ^ z1, y1 ^ z0, y1 ^ z1};
    const bool xodd = (x0 & 1u) != 0u;
    uint32_t sel = xodd ? 16u : 0u;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t i0 = (x0 ^ aa[c]) & mask;
        sel |= (i0 & 1u) << c;
        p.q[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, lvbase + ((i0 & ~1u) << 3), 0, 0);
    }
#if ACN_DIAG_X4ONLY  // diagnostic build only: no second gather (wrong values for odd x0)
#pragma unroll
    for (int c = 0; c < 4; ++c) p.r[c] = u32x2_t{0u, 0u};
#else
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t i1 = (x1 ^ aa[c]) & mask;
        p.r[c] = __builtin_amdgcn_raw_buffer_load_b64(rs, (xodd || ACN_XPAIR_NOSKIP) ? lvbase + (i1 << 3) : 0xFFFFFFF0u, 0, 0);
    }
#endif
    p.wx = wx;
    p.wy = wy;
    p.wz = wz;
    p.sel = sel;
}

// Buffer-resource form of hash_issue, one 8-byte gather per corner (the render's default, ACN_XPAIR == 3): the
// row offsets are 32-bit (lvbase + 8 * row from the expert's table base in the resource), so no 64-bit address
// is formed per corner.  The gathers of the global-address form (hash_issue) returned a wrong row to lanes 48-63
// of one level now and then inside the render kernels; this form never did.
template <int INTERP>
__device__ __forceinline__ void hash_issue_b(__amdgpu_buffer_rsrc_t rs, uint32_t lvbase, float sx, float sy, float sz,
                                             uint32_t mask, HashPending& p) {
    auto ld = [&](uint32_t row) {
        const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rs, lvbase + (row << 3), 0, 0);
        return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
    };
    if (INTERP == 0) {
        const uint32_t ix = (uint32_t)(int)rintf(sx), iy = (uint32_t)(int)rintf(sy), iz = (uint32_t)(int)rintf(sz);
        p.f[0] = ld((ix ^ (iy * kP1) ^ (iz * kP2)) & mask);
        return;
    }
    const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
    float wx = sx - fx, wy = sy - fy, wz = sz - fz;
    const uint32_t x0 = (uint32_t)(int)fx;
    const uint32_t y0 = (uint32_t)(int)fy * kP1, y1 = y0 + kP1;
    const uint32_t z0 = (uint32_t)(int)fz * kP2, z1 = z0 + kP2;
    const uint32_t x1 = x0 + 1u;
    if (INTERP == 2) {   // the constants offset by an opaque +0.0f: formed here, not hoisted into VGPR pairs
        float k3 = 3.0f, k2 = 2.0f;
        asm volatile("" : "+s"(k3), "+s"(k2));
        wx = (wx * wx) * (k3 - k2 * wx);
        wy = (wy * wy) * (k3 - k2 * wy);
        wz = (wz * wz) * (k3 - k2 * wz);
    }
    const uint32_t a00 = y0 ^ z0, a01 = y0 ^ z1, a10 = y1 ^ z0, a11 = y1 ^ z1;
    p.f[0] = ld((x0 ^ a00) & mask);
    p.f[1] = ld((x1 ^ a00) & mask);
    p.f[2] = ld((x0 ^ a01) & mask);
    p.f[3] = ld((x1 ^ a01) & mask);
    p.f[4] = ld((x0 ^ a10) & mask);
    p.f[5] = ld((x1 ^ a10) & mask);
    p.f[6] = ld((x0 ^ a11) & mask);
    p.f[7] = ld((x1 ^ a11) & mask);
    p.wx = wx;
    p.wy = wy;
    p.wz = wz;
}

template <int INTERP>
__device__ __forceinline__ void hash_finish_x(const HashPendingX& p, float& o0, float& o1) {
    HashPending h;
    const bool xodd = (p.sel & 16u) != 0u;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const bool hi = ((p.sel >> c) & 1u) != 0u;
        const u32x4_t q = p.q[c];
        const uint32_t l0 = hi ? q[2] : q[0], l1 = hi ? q[3] : q[1];
        const uint32_t e0 = hi ? q[0] : q[2], e1 = hi ? q[1] : q[3];
        h.f[2 * c] = make_float2(__uint_as_float(l0), __uint_as_float(l1));
        h.f[2 * c + 1] = make_float2(__uint_as_float(xodd ? p.r[c][0] : e0), __uint_as_float(xodd ? p.r[c][1] : e1));
    }
    h.wx = p.wx;
    h.wy = p.wy;
    h.wz = p.wz;
    hash_finish<INTERP>(h, o0, o1);
}

// One level of HashGridEncoder._torch_forward (encodings.py:331-381) for one point.
// tl: this level's table base (row = F floats).  INTERP: 0 nearest, 1 linear, 2 smoothstep.
// Linear/Smoothstep lerp order x -> y -> z exactly as encodings.py:373-379.
template <int INTERP>
__device__ __forceinline__ void hash_level_f2(const float2* __restrict__ tl, float sx, float sy, float sz,
                                              uint32_t mask, float& o0, float& o1) {
    if (INTERP == 0) {
        const uint32_t ix = (uint32_t)(int)rintf(sx), iy = (uint32_t)(int)rintf(sy), iz = (uint32_t)(int)rintf(sz);
        const float2 e = tl[(ix ^ (iy * kP1) ^ (iz * kP2)) & mask];
        o0 = e.x;
        o1 = e.y;
        return;
    }
    const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
    float wx = sx - fx, wy = sy - fy, wz = sz - fz;
    const uint32_t x0 = (uint32_t)(int)fx;
    const uint32_t y0 = (uint32_t)(int)fy * kP1, y1 = y0 + kP1;   // (iy+1)*P1 == iy*P1 + P1 mod 2^32
    const uint32_t z0 = (uint32_t)(int)fz * kP2, z1 = z0 + kP2;
    const uint32_t x1 = x0 + 1u;
    if (INTERP == 2) {
        wx = (wx * wx) * (3.0f - 2.0f * wx);
        wy = (wy * wy) * (3.0f - 2.0f * wy);
        wz = (wz * wz) * (3.0f - 2.0f * wz);
    }
    const uint32_t a00 = y0 ^ z0, a01 = y0 ^ z1, a10 = y1 ^ z0, a11 = y1 ^ z1;
    const float2 f000 = tl[(x0 ^ a00) & mask];
    const float2 f100 = tl[(x1 ^ a00) & mask];
    const float2 f001 = tl[(x0 ^ a01) & mask];
    const float2 f101 = tl[(x1 ^ a01) & mask];
    const float2 f010 = tl[(x0 ^ a10) & mask];
    const float2 f110 = tl[(x1 ^ a10) & mask];
    const float2 f011 = tl[(x0 ^ a11) & mask];
    const float2 f111 = tl[(x1 ^ a11) & mask];
    const float ax = 1.0f - wx, ay = 1.0f - wy, az = 1.0f - wz;
    {
        const float c00 = f000.x * ax + f100.x * wx;
        const float c01 = f001.x * ax + f101.x * wx;
        const float c10 = f010.x * ax + f110.x * wx;
        const float c11 = f011.x * ax + f111.x * wx;
        const float c0 = c00 * ay + c10 * wy;
        const float c1 = c01 * ay + c11 * wy;
        o0 = c0 * az + c1 * wz;
    }
    {
        const float c00 = f000.y * ax + f100.y * wx;
        const float c01 = f001.y * ax + f101.y * wx;
        const float c10 = f010.y * ax + f110.y * wx;
        const float c11 = f011.y * ax + f111.y * wx;
        const float c0 = c00 * ay + c10 * wy;
        const float c1 = c01 * ay + c11 * wy;
        o1 = c0 * az + c1 * wz;
    }
}

// ------------------------------------------------------------------------------------------
// shared by the fused render (render.hip) and the routed training sampler (routed.hip); Cfg is any
// struct with K, cluster_2d, bm, cent[k][3]
// Routing (meta_container.py:97-134), cdist mm-path restated exactly as in the oracle.
// Computed without per-expert arrays (runtime-indexed arrays would live in scratch): a first
// pass gives min distance / denominator (soft) or argmin (hard), then w_k is recomputed per k.
// squared centroid distance of the cdist mm-path, clamped at 0 (NaN -> 0); route_dist = its square root
template <typename Cfg>
__device__ __forceinline__ float route_dist2(const Cfg& cfg, int k, float px, float py, float pz) {
    float s = 0.0f, xn, cn;
    if (cfg.cluster_2d) {
        const float cy = cfg.cent[k][1], cz = cfg.cent[k][2];
        xn = py * py + pz * pz;
        cn = cy * cy + cz * cz;
        s = fmaf(-2.0f * py, cy, s);
        s = fmaf(-2.0f * pz, cz, s);
    } else {
        const float cx = cfg.cent[k][0], cy = cfg.cent[k][1], cz = cfg.cent[k][2];
        xn = (px * px + py * py) + pz * pz;
        cn = (cx * cx + cy * cy) + cz * cz;
        s = fmaf(-2.0f * px, cx, s);
        s = fmaf(-2.0f * py, cy, s);
        s = fmaf(-2.0f * pz, cz, s);
    }
    s = s + xn;
    s = s + cn;
    return s > 0.0f ? s : 0.0f;
}
template <typename Cfg>
__device__ __forceinline__ float route_dist(const Cfg& cfg, int k, float px, float py, float pz) {
    return sqrtf(route_dist2(cfg, k, px, py, pz));
}

struct RouteState {
    float thr, den;  // soft: bm * min dist, sum of masked inverse distances
    int hard;        // hard: argmin
    float thr2;      // soft: thr^2 (1 + 1e-3); a squared distance above it is outside the margin for sure
};
// A squared distance s > thr^2 (1 + 1e-3) (the products rounded ~1e-7 relative) has fl(sqrt(s)) > thr -- sqrt is
// correctly rounded and monotonic -- so its expert is outside the margin (w = 0 exactly) without the square root.
__device__ __forceinline__ float route_thr2(float thr) { return (thr * thr) * 1.001f; }

template <int ROUTE, typename Cfg>
__device__ __forceinline__ RouteState route_prep(const Cfg& cfg, float px, float py, float pz) {
    RouteState st{0.0f, 0.0f, 0, 0.0f};
    if (ROUTE == 1) {
        // min_k max(sqrt(s_k), 1e-6) = max(sqrt(min_k s_k), 1e-6) (monotonic): one square root, not K
        float mins = INFINITY;
        for (int k = 0; k < cfg.K; ++k) mins = fminf(mins, route_dist2(cfg, k, px, py, pz));
        float mind = sqrtf(mins);
        mind = mind < 1e-6f ? 1e-6f : mind;
        st.thr = cfg.bm * mind;
        st.thr2 = route_thr2(st.thr);
        float den = 0.0f;
        for (int k = 0; k < cfg.K; ++k) {
            const float s2 = route_dist2(cfg, k, px, py, pz);
            if (s2 > st.thr2) continue;   // outside the margin: adds 0
            float d = sqrtf(s2);
            d = d < 1e-6f ? 1e-6f : d;
            den = den + ((d <= st.thr) ? 1.0f / d : 0.0f);
        }
        st.den = den < 1e-6f ? 1e-6f : den;
    } else if (ROUTE == 2) {
        float best = INFINITY;
        for (int k = 0; k < cfg.K; ++k) {
            const float d = route_dist(cfg, k, px, py, pz);
            if (d < best || k == 0) { best = d; st.hard = k; }
        }
    }
    return st;
}

template <typename Cfg>
__device__ __forceinline__ float route_weight(const Cfg& cfg, const RouteState& st, int k, float px, float py,
                                              float pz) {
    const float s2 = route_dist2(cfg, k, px, py, pz);
    if (s2 > st.thr2) return 0.0f;   // = 0 / den
    float d = sqrtf(s2);
    d = d < 1e-6f ? 1e-6f : d;
    return ((d <= st.thr) ? 1.0f / d : 0.0f) / st.den;
}

// colour-branch direction encoding (meta_ngp.py:165-168 then encodings.py:144-151)
__device__ __forceinline__ void dir_sh(float dx, float dy, float dz, float (&sh)[16], float kz = 0.0f) {
    const float n = clamp_min_nan(norm3(dx, dy, dz), 1e-9f);
    sh_encode<3>(dx / n, dy / n, dz / n, sh, kz);
}

// t value of sample s (stratified_t_vals, ray_rendering.py:278-287); linspace as torch CPU
__device__ __forceinline__ float lin01(int i, int S) {
    if (S == 1) return 0.0f;
    const float step = 1.0f / (float)(S - 1);
    return i < S / 2 ? fmaf(step, (float)i, 0.0f) : fmaf(-step, (float)(S - 1 - i), 1.0f);
}
__device__ __forceinline__ float tlin(float near, float far, int i, int S) {
    const float u = lin01(i, S);
    return near * (1.0f - u) + far * u;
}
__device__ __forceinline__ float tval(float near, float far, int s, int S, const float* jit) {
    const float ts = tlin(near, far, s, S);
    if (!jit) return ts;
    const float lo = s == 0 ? ts : 0.5f * (tlin(near, far, s - 1, S) + ts);
    const float hi = s == S - 1 ? ts : 0.5f * (ts + tlin(near, far, s + 1, S));
    return lo + (hi - lo) * jit[s];
}

// ---- VALU -> MFMA operand fence (round 5; OFF by default since round 6, §4l).  Round 5 took the
// rare run-to-run differences of the renders (16 columns of one MFMA tile) for stale fp16 B operands and put every
// B fragment through ONE asm statement holding 16 wait states.  Round 6 found their cause elsewhere: the hash-table
// gathers, issued as global loads from 64-bit addresses, now and then returned a wrong row to lanes 48-63 of one
// level (self-check records of the hash features); with the gathers on buffer loads the field repeats, the slots
// self-check builds and the training-MLP repeats show no difference with or without the fence, and hipcc's own
// padding (>= 2 wait states; the box probe needs 1) holds in every kernel (tests/test_hazard_audit.py).  The fence
// cost the meta step 5%, so it is compiled out; -DACN_OPND_FENCE_ON restores it for A/B runs.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
#ifdef ACN_OPND_FENCE_ON
#define ACN_OPND_PAD "s_nop 7\n\ts_nop 7"
#define ACN_OPND_SB0 __builtin_amdgcn_sched_barrier(0);
#define ACN_OPND_ASM(...) asm volatile(__VA_ARGS__)
#else
#define ACN_OPND_PAD ""
#define ACN_OPND_SB0
#define ACN_OPND_ASM(...)
#endif
#define ACN_OPND_CLOB
__device__ __forceinline__ void opnd_fence(f16x8& a) { ACN_OPND_SB0 ACN_OPND_ASM(ACN_OPND_PAD : "+v"(a) : ACN_OPND_CLOB); ACN_OPND_SB0 }
__device__ __forceinline__ void opnd_fence(f16x8& a, f16x8& b) {
    ACN_OPND_SB0 ACN_OPND_ASM(ACN_OPND_PAD : "+v"(a), "+v"(b) : ACN_OPND_CLOB); ACN_OPND_SB0
}
__device__ __forceinline__ void opnd_fence(f16x8& a, f16x8& b, f16x8& c, f16x8& d) {
    ACN_OPND_SB0 ACN_OPND_ASM(ACN_OPND_PAD : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : ACN_OPND_CLOB); ACN_OPND_SB0
}
__device__ __forceinline__ void opnd_fence(f16x8& a, f16x8& b, f16x8& c, f16x8& d, f16x8& e, f16x8& f, f16x8& g,
                                           f16x8& h) {
    ACN_OPND_SB0 ACN_OPND_ASM(ACN_OPND_PAD : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                              : ACN_OPND_CLOB); ACN_OPND_SB0
}
// one plane of N fragments (N = 1, 2, 4, 8)
template <int N>
__device__ __forceinline__ void opnd_fence_n(f16x8 (&x)[N]) {
    static_assert(N == 1 || N == 2 || N == 4 || N == 8, "opnd_fence_n: N in {1, 2, 4, 8}");
    if constexpr (N == 1) opnd_fence(x[0]);
    else if constexpr (N == 2) opnd_fence(x[0], x[1]);
    else if constexpr (N == 4) opnd_fence(x[0], x[1], x[2], x[3]);
    else opnd_fence(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);
}
// hi and lo planes of N fragments (N = 1, 2, 4)
template <int N>
__device__ __forceinline__ void opnd_fence_n(f16x8 (&x)[N], f16x8 (&y)[N]) {
    static_assert(N == 1 || N == 2 || N == 4, "opnd_fence_n: N in {1, 2, 4}");
    if constexpr (N == 1) opnd_fence(x[0], y[0]);
    else if constexpr (N == 2) opnd_fence(x[0], x[1], y[0], y[1]);
    else opnd_fence(x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]);
}

}  // namespace acn
