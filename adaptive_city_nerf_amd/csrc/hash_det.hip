// hash_det.hip -- deterministic hash-grid backward (SURVEY §5 "deterministic-mode tests for the hash
// backward, which uses atomics, comparing against a serial CPU scatter-add").
//
// The float-atomic scatter-add of hashgrid_bwd_* (encoders.hip) sums each table row in arrival order,
// so two runs can differ in the last bits.  This mode replaces the atomics by a store pass and a
// per-destination sum pass (cdna_hip_programming.md Guideline 12, "store pass plus a per-destination
// sum pass"):
//   1. one record per (point m, level l, corner c): key = l * T + row, value = the corner's (2-feature)
//      gradient in the forward's chain-rule order ((g * wz') * wy') * wx' -- generated in (m, l, c) order;
//   2. a stable LSD radix sort of the records by key (rocPRIM), so equal keys keep generation order;
//   3. one lane per run of equal keys sums it sequentially in fp32 and stores the row.
// Every row is therefore the fp32 sum of its contributions in (point, corner) order, continued from the row's
// current value: equal, bit for bit, to a serial CPU scatter-add over (point, level, corner)
// (tests/test_hash_det.py), and bitwise reproducible run to run.  It is NOT the reference's own summation
// order: there (models/encodings.py:318-381) each of the 8 corners is a separate gather whose backward
// index_put_(accumulate=True) sums that corner's contributions, and autograd then adds the 8 per-corner
// table gradients.  The caller bounds the workspace (~24 B x 8 x L per point) by chunking the points
// (ops.hashgrid_bwd): chunks run in point order, so the rows continue the same serial sums.
#include <rocprim/device/device_radix_sort.hpp>

#include "acn_device.h"
#include "acn_internal.h"

namespace {

struct ResD {
    int32_t v[ACN_MAX_LEVELS];
};

template <int INTERP>
__global__ void __launch_bounds__(256) det_records_kernel(const float* __restrict__ x01, int64_t M,
                                                          const float2* __restrict__ gout, ResD res, int L, int log2T,
                                                          uint32_t* __restrict__ keys, float2* __restrict__ vals) {
    constexpr int NC = INTERP == 0 ? 1 : 8;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (m, l)
    if (gid >= M * L) return;
    const int64_t m = gid / L;
    const int l = (int)(gid - m * L);
    const float r = (float)res.v[l];
    const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    const uint32_t lbase = (uint32_t)l << log2T;
    const float2 g = gout[m * L + l];
    uint32_t* k = keys + gid * NC;
    float2* v = vals + gid * NC;
    if (INTERP == 0) {
        const uint32_t ix = (uint32_t)(int)rintf(sx), iy = (uint32_t)(int)rintf(sy), iz = (uint32_t)(int)rintf(sz);
        k[0] = lbase | ((ix ^ (iy * acn::kP1) ^ (iz * acn::kP2)) & mask);
        v[0] = g;
        return;
    }
    const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
    float wx = sx - fx, wy = sy - fy, wz = sz - fz;
    if (INTERP == 2) {
        wx = (wx * wx) * (3.0f - 2.0f * wx);
        wy = (wy * wy) * (3.0f - 2.0f * wy);
        wz = (wz * wz) * (3.0f - 2.0f * wz);
    }
    const float ax = 1.0f - wx, ay = 1.0f - wy, az = 1.0f - wz;
    const uint32_t x0 = (uint32_t)(int)fx, y0 = (uint32_t)(int)fy * acn::kP1, z0 = (uint32_t)(int)fz * acn::kP2;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int bx = c >> 2, by = (c >> 1) & 1, bz = c & 1;
        const uint32_t h = ((x0 + (uint32_t)bx) ^ (y0 + (by ? acn::kP1 : 0u)) ^ (z0 + (bz ? acn::kP2 : 0u))) & mask;
        const float fzw = bz ? wz : az, fyw = by ? wy : ay, fxw = bx ? wx : ax;
        k[c] = lbase | h;
        v[c] = make_float2(((g.x * fzw) * fyw) * fxw, ((g.y * fzw) * fyw) * fxw);
    }
}

// one lane per run head: sequential fp32 sum of the run (sorted = generation order within a key)
__global__ void __launch_bounds__(256) det_sum_kernel(const uint32_t* __restrict__ keys, const float2* __restrict__ vals,
                                                      int64_t R, float2* __restrict__ gtable) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const uint32_t key = keys[i];
    if (i > 0 && keys[i - 1] == key) return;
    float2 s = gtable[key];  // the caller's zeroed (or accumulating) gradient row
    for (int64_t j = i; j < R && keys[j] == key; ++j) {
        s.x = s.x + vals[j].x;
        s.y = s.y + vals[j].y;
    }
    gtable[key] = s;
}

int bits_for(uint64_t n) {
    int b = 0;
    while ((1ull << b) < n) ++b;
    return b < 1 ? 1 : b;
}

size_t sort_temp_bytes(int64_t R, int end_bit) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs((void*)nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                              (const float2*)nullptr, (float2*)nullptr, (size_t)R, 0u, (unsigned)end_bit);
    return bytes;
}

size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

}  // namespace

extern "C" size_t acn_hashgrid_bwd_det_workspace_bytes(int64_t M, int L, int log2T, int interp) {
    if (M <= 0 || L < 1 || L > ACN_MAX_LEVELS || log2T < 1) return 0;
    const int64_t R = M * L * (interp == 0 ? 1 : 8);
    const int end_bit = bits_for((uint64_t)L << log2T);
    return 2 * align_up((size_t)R * sizeof(uint32_t)) + 2 * align_up((size_t)R * sizeof(float2)) +
           align_up(sort_temp_bytes(R, end_bit));
}

extern "C" int acn_hashgrid_bwd_det(const float* x01, int64_t M, const float* grad_out, const int32_t* res, int L,
                                    int log2T, int F, int interp, float* grad_table, void* workspace,
                                    size_t workspace_bytes, void* stream) {
    ACN_REQUIRE(M >= 0 && L >= 1 && L <= ACN_MAX_LEVELS && log2T >= 1 && log2T <= 27 && interp >= 0 && interp <= 2,
                "acn_hashgrid_bwd_det: bad grid configuration");
    ACN_REQUIRE(F == 2, "acn_hashgrid_bwd_det: features_per_level must be 2 (the reference configuration)");
    ACN_REQUIRE(((uint64_t)L << log2T) <= (1ull << 32), "acn_hashgrid_bwd_det: L * 2^log2T rows exceed 32-bit keys");
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(x01 && grad_out && res && grad_table && workspace, "acn_hashgrid_bwd_det: NULL pointer");
    ACN_REQUIRE(workspace_bytes >= acn_hashgrid_bwd_det_workspace_bytes(M, L, log2T, interp),
                "acn_hashgrid_bwd_det: workspace too small");
    const int64_t R = M * L * (interp == 0 ? 1 : 8);
    const int end_bit = bits_for((uint64_t)L << log2T);
    char* w = (char*)workspace;
    uint32_t* k0 = (uint32_t*)w;
    w += align_up((size_t)R * sizeof(uint32_t));
    uint32_t* k1 = (uint32_t*)w;
    w += align_up((size_t)R * sizeof(uint32_t));
    float2* v0 = (float2*)w;
    w += align_up((size_t)R * sizeof(float2));
    float2* v1 = (float2*)w;
    w += align_up((size_t)R * sizeof(float2));
    size_t tb = sort_temp_bytes(R, end_bit);
    ResD r{};
    for (int i = 0; i < L; ++i) r.v[i] = res[i];
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)((M * L + 255) / 256)), block(256);
    if (interp == 0) hipLaunchKernelGGL(det_records_kernel<0>, grid, block, 0, s, x01, M, (const float2*)grad_out, r, L, log2T, k0, v0);
    else if (interp == 1) hipLaunchKernelGGL(det_records_kernel<1>, grid, block, 0, s, x01, M, (const float2*)grad_out, r, L, log2T, k0, v0);
    else hipLaunchKernelGGL(det_records_kernel<2>, grid, block, 0, s, x01, M, (const float2*)grad_out, r, L, log2T, k0, v0);
    const hipError_t e = rocprim::radix_sort_pairs((void*)w, tb, k0, k1, v0, v1, (size_t)R, 0u, (unsigned)end_bit, s);
    if (e != hipSuccess) return acn_set_error((int)e, "acn_hashgrid_bwd_det: radix sort failed: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(det_sum_kernel, dim3((unsigned)((R + 255) / 256)), block, 0, s, k1, v1, R, (float2*)grad_table);
    return acn_check_launch("acn_hashgrid_bwd_det");
}
