// hash_gather.hip -- gather-only microbenchmark of the fused render's hash-table access (developer tool,
// tools/micro/hash_gather.py drives it).  Calibrates the ceiling the render kernel's hash gathers run
// against (VERDICT r02 "Next" 1: the 8.6 TB/s figure of MI355X_MICROARCH.md is for 1,152-B rows; the
// render issues 8-B hashed corner reads).
//
// Same access shape as render_kernel<1,1,0> (render.hip hash_levels8 + acn_device.h hash_issue /
// hash_finish): one wave per ray, the ray's samples in tiles of 32, lane = (sample j = l & 31, half
// h = l >> 5), half h encodes levels 8h .. 8h + 7, eight 8-B corner rows per level from the level's 2^20-row
// fp32 table (16 levels = 128 MiB), D levels' gathers in flight, trilinear interpolation.  Nothing else: no
// MLP, no compositing.  The features are summed per sample and one float per (sample, half) is written so
// the gathers are not dead.  Visiting order: the render's XCD bands (block b runs on XCD b mod 8; XCD x
// takes the x-th contiguous eighth of the rays), or plain grid-stride (band = 0).
#include <hip/hip_runtime.h>

#include "../../adaptive_city_nerf_amd/csrc/acn_device.h"

namespace {

struct Res16 {
    float r[16];
};

template <int D>
__global__ void __launch_bounds__(256) gather_kernel(const float* __restrict__ x01, const float* __restrict__ table,
                                                     Res16 res, int log2T, int N, int S, int band,
                                                     float* __restrict__ out) {
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    int r0, r1, wid, nw;
    if (band) {
        const int nx = gridDim.x / 8, x = blockIdx.x % 8, slot = blockIdx.x / 8;
        r0 = (int)((int64_t)x * N / 8);
        r1 = (int)((int64_t)(x + 1) * N / 8);
        wid = slot * 4 + w;
        nw = nx * 4;
    } else {
        r0 = 0;
        r1 = N;
        wid = blockIdx.x * 4 + w;
        nw = gridDim.x * 4;
    }
    const int tiles = (S + 31) / 32;
    for (int ray = r0 + wid; ray < r1; ray += nw) {
        for (int t = 0; t < tiles; ++t) {
            const int s = t * 32 + j;
            const bool ok = s < S;
            const int64_t m = (int64_t)ray * S + (ok ? s : S - 1);
            const float px = x01[3 * m], py = x01[3 * m + 1], pz = x01[3 * m + 2];
            float acc = 0.0f;
            acn::HashPending pend[D];
            auto issue = [&](int i, acn::HashPending& pp) {
                const int lv = i + 8 * h;
                const float rs = res.r[lv];
                const float2* tl = reinterpret_cast<const float2*>(table) + ((size_t)lv << log2T);
                acn::hash_issue<1, 0>(tl, px * rs, py * rs, pz * rs, mask, pp);
            };
#pragma unroll
            for (int l = 0; l < D - 1; ++l) issue(l, pend[l]);
#pragma unroll
            for (int l = 0; l < 8; ++l) {
                if (l + D - 1 < 8) issue(l + D - 1, pend[(l + D - 1) % D]);
                __builtin_amdgcn_sched_barrier(0);
                float o0, o1;
                acn::hash_finish<1>(pend[l % D], o0, o1);
                acc += o0 + o1;
                __builtin_amdgcn_sched_barrier(0);
            }
            if (ok) out[2 * m + h] = acc;
        }
    }
}

}  // namespace

extern "C" int hg_launch(const float* x01, const float* table, const float* res, int log2T, int N, int S, int depth,
                         int blocks, int band, float* out, void* stream) {
    Res16 r;
    for (int i = 0; i < 16; ++i) r.r[i] = res[i];
    hipStream_t s = (hipStream_t)stream;
    switch (depth) {
        case 1: hipLaunchKernelGGL(gather_kernel<1>, dim3(blocks), dim3(256), 0, s, x01, table, r, log2T, N, S, band, out); break;
        case 2: hipLaunchKernelGGL(gather_kernel<2>, dim3(blocks), dim3(256), 0, s, x01, table, r, log2T, N, S, band, out); break;
        case 3: hipLaunchKernelGGL(gather_kernel<3>, dim3(blocks), dim3(256), 0, s, x01, table, r, log2T, N, S, band, out); break;
        case 4: hipLaunchKernelGGL(gather_kernel<4>, dim3(blocks), dim3(256), 0, s, x01, table, r, log2T, N, S, band, out); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}
