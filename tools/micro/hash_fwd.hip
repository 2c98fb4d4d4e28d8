// hash_fwd.hip -- A/B microbenchmark of the standalone hash-grid forward (acn_hashgrid_fwd, F = 2,
// linear) access shapes (developer tool, tools/micro/hash_fwd.py).  Same arithmetic in every variant
// (hash_finish's non-FMA lerp order = encoders.hip hash_level_f2), only the gathers and the
// (point, level) -> lane mapping differ:
//   0 plain : one lane per (point, level), 8 dwordx2 gathers (the product kernel before this study)
//   1 xpair : same mapping, x-neighbour rows fetched as one 16-B block (hash_issue_x: 4 dwordx4 + 4
//             dwordx2 only for odd x0)
//   2 band  : xpair + XCD level bands: workgroup v runs on XCD v % 8 and handles levels
//             {2 (v % 8), 2 (v % 8) + 1} of 128 points, so each XCD's L2 sees 2 of the 16 levels
#include "../../adaptive_city_nerf_amd/csrc/acn_device.h"

using namespace acn;

namespace {
struct Res16 {
    int32_t v[16];
};

__global__ void __launch_bounds__(256) fwd_plain(const float* __restrict__ x01, int64_t M, const float2* __restrict__ table,
                                                 Res16 res, int log2T, float2* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = gid >> 4;
    const int l = (int)(gid & 15);
    if (m >= M) return;
    const float r = (float)res.v[l];
    const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    float o0, o1;
    hash_level_f2<1>(table + ((int64_t)l << log2T), sx, sy, sz, mask, o0, o1);
    out[m * 16 + l] = make_float2(o0, o1);
}

__global__ void __launch_bounds__(256) fwd_xpair(const float* __restrict__ x01, int64_t M, const float2* __restrict__ table,
                                                 Res16 res, int log2T, float2* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = gid >> 4;
    const int l = (int)(gid & 15);
    if (m >= M) return;
    const float r = (float)res.v[l];
    const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)table, (short)0, (int)(uint32_t)((16ull << log2T) * 8ull), 0x00020000);
    HashPendingX p;
    hash_issue_x<1>(rs, (uint32_t)l << (log2T + 3), sx, sy, sz, mask, p);
    float o0, o1;
    hash_finish_x<1>(p, o0, o1);
    out[m * 16 + l] = make_float2(o0, o1);
}

__global__ void __launch_bounds__(256) fwd_band(const float* __restrict__ x01, int64_t M, const float2* __restrict__ table,
                                                Res16 res, int log2T, float2* __restrict__ out) {
    const int v = blockIdx.x;
    const int l = 2 * (v & 7) + (threadIdx.x & 1);
    const int64_t m = (int64_t)(v >> 3) * 128 + (threadIdx.x >> 1);
    if (m >= M) return;
    const float r = (float)res.v[l];
    const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)table, (short)0, (int)(uint32_t)((16ull << log2T) * 8ull), 0x00020000);
    HashPendingX p;
    hash_issue_x<1>(rs, (uint32_t)l << (log2T + 3), sx, sy, sz, mask, p);
    float o0, o1;
    hash_finish_x<1>(p, o0, o1);
    out[m * 16 + l] = make_float2(o0, o1);
}
}  // namespace

extern "C" int hf_launch(int variant, const float* x01, int64_t M, const float* table, const int32_t* res, int log2T,
                         float* out, void* stream) {
    if (log2T < 1 || log2T > 24 || M <= 0) return 1;
    Res16 r{};
    for (int i = 0; i < 16; ++i) r.v[i] = res[i];
    hipStream_t s = (hipStream_t)stream;
    if (variant == 0) {
        hipLaunchKernelGGL(fwd_plain, dim3((unsigned)((M * 16 + 255) / 256)), dim3(256), 0, s, x01, M, (const float2*)table, r,
                           log2T, (float2*)out);
    } else if (variant == 1) {
        hipLaunchKernelGGL(fwd_xpair, dim3((unsigned)((M * 16 + 255) / 256)), dim3(256), 0, s, x01, M, (const float2*)table, r,
                           log2T, (float2*)out);
    } else if (variant == 2) {
        hipLaunchKernelGGL(fwd_band, dim3((unsigned)(((M + 127) / 128) * 8)), dim3(256), 0, s, x01, M, (const float2*)table, r,
                           log2T, (float2*)out);
    } else {
        return 2;
    }
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
