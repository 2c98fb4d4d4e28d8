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

// models/encodings.py:27-81 components_from_spherical_harmonics, float32 op order of the torch
// expressions (scalar * tensor evaluated left to right).
template <int DEGREE>
__device__ __forceinline__ void sh_components(float x, float y, float z, float* c) {
    const float xx = x * x, yy = y * y, zz = z * z;
    c[0] = 0.28209479177387814f;
    if (DEGREE > 0) {
        c[1] = 0.4886025119029199f * y;
        c[2] = 0.4886025119029199f * z;
        c[3] = 0.4886025119029199f * x;
    }
    if (DEGREE > 1) {
        c[4] = (1.0925484305920792f * x) * y;
        c[5] = (1.0925484305920792f * y) * z;
        c[6] = 0.9461746957575601f * zz - 0.31539156525251999f;
        c[7] = (1.0925484305920792f * x) * z;
        c[8] = 0.5462742152960396f * (xx - yy);
    }
    if (DEGREE > 2) {
        c[9] = (0.5900435899266435f * y) * (3.0f * xx - yy);
        c[10] = ((2.890611442640554f * x) * y) * z;
        c[11] = (0.4570457994644658f * y) * (5.0f * zz - 1.0f);
        c[12] = (0.3731763325901154f * z) * (5.0f * zz - 3.0f);
        c[13] = (0.4570457994644658f * x) * (5.0f * zz - 1.0f);
        c[14] = (1.445305721320277f * z) * (xx - yy);
        c[15] = (0.5900435899266435f * x) * (xx - 3.0f * yy);
    }
    if (DEGREE > 3) {
        c[16] = ((2.5033429417967046f * x) * y) * (xx - yy);
        c[17] = ((1.7701307697799304f * y) * z) * (3.0f * xx - yy);
        c[18] = ((0.9461746957575601f * x) * y) * (7.0f * zz - 1.0f);
        c[19] = ((0.6690465435572892f * y) * z) * (7.0f * zz - 3.0f);
        c[20] = 0.10578554691520431f * (((35.0f * zz) * zz - 30.0f * zz) + 3.0f);
        c[21] = ((0.6690465435572892f * x) * z) * (7.0f * zz - 3.0f);
        c[22] = (0.47308734787878004f * (xx - yy)) * (7.0f * zz - 1.0f);
        c[23] = ((1.7701307697799304f * x) * z) * (xx - 3.0f * yy);
        c[24] = 0.6258357354491761f * (xx * (xx - 3.0f * yy) - yy * (3.0f * xx - yy));
    }
}

// SHEncoder.forward (encodings.py:144-151): d / norm(d).clamp_min(1e-9), then components
template <int DEGREE>
__device__ __forceinline__ void sh_encode(float dx, float dy, float dz, float* c) {
    const float n = clamp_min_nan(norm3(dx, dy, dz), 1e-9f);
    sh_components<DEGREE>(dx / n, dy / n, dz / n, c);
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

}  // namespace acn
