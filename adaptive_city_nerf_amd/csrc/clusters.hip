// clusters.hip -- Voronoi ray -> expert routing of cluster creation (gfx950).
//
// Replaces the per-image tensor pipeline of scripts/create_clusters.py: compute_voronoi_opt
// (:386-556: S samples per ray on the lerp(near, far, linspace(0, 1, S)) grid, squared centroid
// distances in the routing subspace (YZ when cluster_2d), the strict argmin or the
// d2 <= m^2 * min d2 overlap rule, and the per-expert AABB / sample-count streaming of the assigned
// samples) and compute_voronoi_orig (:559-634: torch.cdist distances, ratio to the nearest centroid
// + 1e-8, min over the ray's samples <= boundary_margin).  One lane per ray; the samples and
// centroids stay in registers, so the (N*S, C) distance blocks of the reference never exist.
// Float ops follow the reference's op order (-ffp-contract=off, fmaf where its kernels fuse):
// linspace / lerp as one fma each, x = o + d * t, |x|^2 = sequential sum of squares, and
//   opt:  d2 = (|x|^2 + |c|^2) - 2 * (x . c)          (x . c as the GEMM's fma chain)
//   orig: D  = sqrt(max(0, [-2x, |x|^2, 1] . [c, 1, |c|^2]))   (torch.cdist's mm path, MKL's chain)
//
// Output per ray: bit c of bits[r] = the ray belongs to centroid c (C <= 63).
// AABB streaming (opt modes, update != 0): over the assigned samples x = o + d * t, mins / maxs (C, 3)
// are lowered / raised in place (the caller initialises them to +inf / -inf as the reference does),
// counts (C) gain the number of assigned samples and nan_flag[c] is set when an assigned sample is
// NaN (the reference's torch.minimum / maximum then make that expert's box NaN).  The extremes over
// a ray's assigned samples sit at its smallest / largest assigned t (x = o + d * t rounds
// monotonically in t), so a lane keeps two t's per centroid and boxes are reduced once per wave.
#include "acn_device.h"
#include "acn_internal.h"

namespace {

constexpr int kMaxCentroids = 63;

struct VoronoiArgs {
    const float* rays;   // (N, 8)
    int64_t N;
    int S, C;
    int mode;            // 0 opt strict (margin == 1), 1 opt overlap, 2 orig (cdist ratio)
    int update;          // stream AABBs / counts (opt modes)
    float m2;            // float(boundary_margin ** 2)
    float bm;            // float(boundary_margin)
    float cent[kMaxCentroids][3];
};

__device__ __forceinline__ bool isnan_(float v) { return v != v; }
__device__ __forceinline__ float nanmin(float a, float b) {
    return (isnan_(a) || isnan_(b)) ? __builtin_nanf("") : fminf(a, b);
}

// float min / max atomics through the integer order of IEEE floats (NaN never reaches them)
__device__ __forceinline__ void atomic_min_f(float* addr, float v) {
    if (v >= 0.0f) atomicMin(reinterpret_cast<int*>(addr), __float_as_int(v));
    else atomicMax(reinterpret_cast<unsigned*>(addr), __float_as_uint(v));
}
__device__ __forceinline__ void atomic_max_f(float* addr, float v) {
    if (v >= 0.0f) atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
    else atomicMin(reinterpret_cast<unsigned*>(addr), __float_as_uint(v));
}

// MAXC: register capacity (>= C); K: routing dims (2 = YZ, 3 = XYZ), subspace starts at 3 - K
template <int MAXC, int K>
__global__ void __launch_bounds__(256) voronoi_kernel(VoronoiArgs a, uint64_t* __restrict__ bits,
                                                      float* __restrict__ mins, float* __restrict__ maxs,
                                                      unsigned long long* __restrict__ counts,
                                                      int* __restrict__ nan_flag) {
    constexpr int ST = 3 - K;
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = r < a.N;
    float o[3] = {0.f, 0.f, 0.f}, d[3] = {0.f, 0.f, 0.f}, tn = 0.f, tf = 0.f;
    if (live) {
        const float4 p0 = reinterpret_cast<const float4*>(a.rays + 8 * r)[0];
        const float4 p1 = reinterpret_cast<const float4*>(a.rays + 8 * r)[1];
        o[0] = p0.x; o[1] = p0.y; o[2] = p0.z; d[0] = p0.w; d[1] = p1.x; d[2] = p1.y; tn = p1.z; tf = p1.w;
    }
    // centroid subspace coordinates and squared norms (pow(2).sum(-1): sequential)
    float cs[MAXC][K], cn[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
#pragma unroll
        for (int j = 0; j < K; ++j) cs[c][j] = c < a.C ? a.cent[c][ST + j] : 0.f;
        float s = cs[c][0] * cs[c][0];
#pragma unroll
        for (int j = 1; j < K; ++j) s = s + cs[c][j] * cs[c][j];
        cn[c] = s;
    }
    uint64_t has = 0, nanm = 0;
    float tlo[MAXC], thi[MAXC], rmin[MAXC];
    unsigned cnt[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) { tlo[c] = INFINITY; thi[c] = -INFINITY; rmin[c] = INFINITY; cnt[c] = 0; }

    if (live) {
        for (int s = 0; s < a.S; ++s) {
            const float t = acn::lerp_t(tn, tf, acn::linspace01(s, a.S));
            float x[K];
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = o[ST + j] + d[ST + j] * t;
            float x2 = x[0] * x[0];
#pragma unroll
            for (int j = 1; j < K; ++j) x2 = x2 + x[j] * x[j];
            float v[MAXC];
            if (a.mode == 2) {
#pragma unroll
                for (int c = 0; c < MAXC; ++c) {
                    float acc = (-2.0f * x[0]) * cs[c][0];
#pragma unroll
                    for (int j = 1; j < K; ++j) acc = fmaf(-2.0f * x[j], cs[c][j], acc);
                    acc = fmaf(x2, 1.0f, acc);
                    acc = fmaf(1.0f, cn[c], acc);
                    v[c] = sqrtf(acn::clamp_min_nan(acc, 0.0f));
                }
                float m = v[0];
#pragma unroll
                for (int c = 1; c < MAXC; ++c) if (c < a.C) m = nanmin(m, v[c]);
                const float den = m + 1e-8f;
#pragma unroll
                for (int c = 0; c < MAXC; ++c) rmin[c] = nanmin(rmin[c], v[c] / den);
            } else {
#pragma unroll
                for (int c = 0; c < MAXC; ++c) {
                    float ip = x[0] * cs[c][0];
#pragma unroll
                    for (int j = 1; j < K; ++j) ip = fmaf(x[j], cs[c][j], ip);
                    v[c] = acn::clamp_min_nan((x2 + cn[c]) - 2.0f * ip, 0.0f);
                }
                uint64_t sel = 0;
                if (a.mode == 0) {  // argmin: a NaN wins, else the first minimum
                    int best = 0;
                    float bv = v[0];
#pragma unroll
                    for (int c = 1; c < MAXC; ++c)
                        if (c < a.C && !isnan_(bv) && (v[c] < bv || isnan_(v[c]))) { best = c; bv = v[c]; }
                    sel = 1ull << best;
                } else {
                    float m = v[0];
#pragma unroll
                    for (int c = 1; c < MAXC; ++c) if (c < a.C) m = nanmin(m, v[c]);
                    const float thr = a.m2 * m;
#pragma unroll
                    for (int c = 0; c < MAXC; ++c) if (c < a.C && v[c] <= thr) sel |= 1ull << c;
                }
                has |= sel;
                if (a.update) {
#pragma unroll
                    for (int c = 0; c < MAXC; ++c) {
                        if ((sel >> c) & 1ull) {
                            cnt[c] += 1;
                            if (isnan_(t)) nanm |= 1ull << c;
                            else { tlo[c] = fminf(tlo[c], t); thi[c] = fmaxf(thi[c], t); }
                        }
                    }
                }
            }
        }
        if (a.mode == 2) {
#pragma unroll
            for (int c = 0; c < MAXC; ++c) if (c < a.C && rmin[c] <= a.bm) has |= 1ull << c;
        }
        bits[r] = has;
    }
    if (!a.update) return;  // uniform over the grid
    // per-wave box / count reduction, then one atomic per centroid per wave
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (c >= a.C) break;
        float lo[3], hi[3];
        const bool any = tlo[c] <= thi[c];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float xa = o[j] + d[j] * tlo[c], xb = o[j] + d[j] * thi[c];
            lo[j] = any ? fminf(xa, xb) : INFINITY;
            hi[j] = any ? fmaxf(xa, xb) : -INFINITY;
        }
        unsigned n = cnt[c];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                lo[j] = fminf(lo[j], __shfl_xor(lo[j], off));
                hi[j] = fmaxf(hi[j], __shfl_xor(hi[j], off));
            }
            n += __shfl_xor(n, off);
        }
        const bool nan_any = __ballot((nanm >> c) & 1ull) != 0;
        if (lane == 0) {
            if (n) atomicAdd(counts + c, (unsigned long long)n);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                if (lo[j] <= hi[j]) {
                    atomic_min_f(mins + 3 * c + j, lo[j]);
                    atomic_max_f(maxs + 3 * c + j, hi[j]);
                }
            }
            if (nan_any) atomicOr(nan_flag + c, 1);
        }
    }
}

template <int MAXC>
int launch_c(const VoronoiArgs& a, int k, uint64_t* bits, float* mins, float* maxs, unsigned long long* counts,
             int* nf, hipStream_t s) {
    const unsigned blocks = (unsigned)((a.N + 255) / 256);
    if (k == 2)
        hipLaunchKernelGGL((voronoi_kernel<MAXC, 2>), dim3(blocks), dim3(256), 0, s, a, bits, mins, maxs, counts, nf);
    else
        hipLaunchKernelGGL((voronoi_kernel<MAXC, 3>), dim3(blocks), dim3(256), 0, s, a, bits, mins, maxs, counts, nf);
    return acn_check_launch("acn_voronoi_route");
}

}  // namespace

extern "C" int acn_voronoi_route(const float* rays, int64_t N, int ray_samples, const float* centroids, int n_centroids,
                                 int cluster_2d, double boundary_margin, int orig, int update_aabbs, uint64_t* bits,
                                 float* mins, float* maxs, int64_t* counts, int32_t* nan_flag, void* stream) {
    ACN_REQUIRE(N >= 0 && ray_samples >= 1, "acn_voronoi_route: N >= 0 and ray_samples >= 1 required");
    ACN_REQUIRE(n_centroids >= 1 && n_centroids <= kMaxCentroids, "acn_voronoi_route: 1 <= n_centroids <= 63");
    ACN_REQUIRE(centroids, "acn_voronoi_route: centroids is NULL");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(rays && bits, "acn_voronoi_route: NULL pointer");
    ACN_REQUIRE((((uintptr_t)rays) & 15) == 0, "acn_voronoi_route: rays must be 16-byte aligned");
    const int update = (update_aabbs && !orig) ? 1 : 0;
    ACN_REQUIRE(!update || (mins && maxs && counts && nan_flag), "acn_voronoi_route: AABB buffers are NULL");
    VoronoiArgs a{};
    a.rays = rays; a.N = N; a.S = ray_samples; a.C = n_centroids;
    a.mode = orig ? 2 : (boundary_margin == 1.0 ? 0 : 1);
    a.update = update;
    a.m2 = (float)(boundary_margin * boundary_margin);
    a.bm = (float)boundary_margin;
    for (int c = 0; c < n_centroids; ++c)
        for (int j = 0; j < 3; ++j) a.cent[c][j] = centroids[3 * c + j];
    const int k = cluster_2d ? 2 : 3;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* cnt = reinterpret_cast<unsigned long long*>(counts);
    if (n_centroids <= 4) return launch_c<4>(a, k, bits, mins, maxs, cnt, nan_flag, s);
    if (n_centroids <= 8) return launch_c<8>(a, k, bits, mins, maxs, cnt, nan_flag, s);
    if (n_centroids <= 16) return launch_c<16>(a, k, bits, mins, maxs, cnt, nan_flag, s);
    if (n_centroids <= 32) return launch_c<32>(a, k, bits, mins, maxs, cnt, nan_flag, s);
    return launch_c<63>(a, k, bits, mins, maxs, cnt, nan_flag, s);
}
