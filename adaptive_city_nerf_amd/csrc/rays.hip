// rays.hip -- per-pixel ray generation for full-frame renders (gfx950).
// Replaces get_ray_directions (nerfs/ray_sampling.py:111-136), get_rays / _rays_cam_to_world
// (:50-108, :10-24), SceneBox.ray_aabb_intersect (nerfs/scene_box.py:45-107) and
// clamp_rays_near_far (ray_sampling.py:139-176) with one fused kernel writing (H*W, 8) rays.
#include "acn_device.h"
#include "acn_internal.h"

namespace {

using acn::pixel_dir;
using acn::slab;

__global__ void __launch_bounds__(256) dirs_kernel(int H, int W, float fx, float fy, float cx, float cy, int center,
                                                   float* __restrict__ dirs) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    float dx, dy, dz;
    pixel_dir((int)(p % W), (int)(p / W), fx, fy, cx, cy, center, dx, dy, dz);
    dirs[3 * p] = dx; dirs[3 * p + 1] = dy; dirs[3 * p + 2] = dz;
}

struct Mat34 { float m[12]; };
struct Box { float b[6]; };

// get_rays (ray_sampling.py:50-108) for given camera-frame directions
__global__ void __launch_bounds__(256) rays_from_dirs_kernel(const float* __restrict__ dirs, int64_t N, Mat34 c, int has_aabb,
                                                             Box box, float near_c, float far_c, float eps,
                                                             float max_bound, float invalid_value, float* __restrict__ rays) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    const float dx = dirs[3 * p], dy = dirs[3 * p + 1], dz = dirs[3 * p + 2];
    float dw[3], o[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        dw[r] = fmaf(dz, c.m[4 * r + 2], fmaf(dy, c.m[4 * r + 1], dx * c.m[4 * r + 0]));
        o[r] = c.m[4 * r + 3];
    }
    float tmin = near_c, tmax = far_c;
    if (has_aabb) slab(o, dw, box.b, eps, max_bound, invalid_value, tmin, tmax);
    float* r = rays + 8 * p;
    r[0] = o[0]; r[1] = o[1]; r[2] = o[2]; r[3] = dw[0]; r[4] = dw[1]; r[5] = dw[2]; r[6] = tmin; r[7] = tmax;
}

__global__ void __launch_bounds__(256) ray_aabb_kernel(const float* __restrict__ o, const float* __restrict__ d, int64_t N,
                                                       Box box, float eps, float max_bound, float invalid_value,
                                                       float* __restrict__ tmin, float* __restrict__ tmax) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    float tn, tf;
    slab(o + 3 * p, d + 3 * p, box.b, eps, max_bound, invalid_value, tn, tf);
    tmin[p] = tn; tmax[p] = tf;
}

// clamp_rays_near_far (ray_sampling.py:139-176)
__global__ void __launch_bounds__(256) clamp_kernel(float* __restrict__ rays, int64_t N, int apply, int hn, float nv,
                                                    int hf, float fv, float eps, float invalid_value,
                                                    uint8_t* __restrict__ valid) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    float n = rays[8 * p + 6], f = rays[8 * p + 7];
    if (apply) {
        if (hn) n = fmaxf(n, nv);
        if (hf) f = fminf(f, fv);
    }
    const bool ok = isfinite(n) && isfinite(f) && (f > n + eps);
    if (apply) {
        rays[8 * p + 6] = ok ? n : invalid_value;
        rays[8 * p + 7] = ok ? f : invalid_value;
    }
    if (valid) valid[p] = ok ? 1 : 0;
}

struct RayGenArgs {
    int H, W;
    float fx, fy, cx, cy;
    int center_pixels;
    float c2w[12];
    int has_aabb;
    float aabb[6];
    float near_c, far_c;
    int has_near_ovr, has_far_ovr, apply_clamp;
    float near_ovr, far_ovr;
};

__global__ void __launch_bounds__(256) rays_kernel(RayGenArgs a, float* __restrict__ rays, uint8_t* __restrict__ valid) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)a.H * a.W) return;
    const int j = (int)(p / a.W), i = (int)(p % a.W);
    float dx, dy, dz;
    pixel_dir(i, j, a.fx, a.fy, a.cx, a.cy, a.center_pixels, dx, dy, dz);
    float dw[3], o[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {  // dirs @ R^T (MKL sgemm, K=3, restated as an fma chain)
        dw[r] = fmaf(dz, a.c2w[4 * r + 2], fmaf(dy, a.c2w[4 * r + 1], dx * a.c2w[4 * r + 0]));
        o[r] = a.c2w[4 * r + 3];
    }
    float tmin, tmax;
    if (a.has_aabb) {
        slab(o, dw, a.aabb, 1e-8f, 1e10f, 1e10f, tmin, tmax);   // get_rays defaults (:55-58, :83-89)
    } else {
        tmin = a.near_c;
        tmax = a.far_c;
    }
    bool ok;
    if (a.apply_clamp) {
        if (a.has_near_ovr) tmin = fmaxf(tmin, a.near_ovr);
        if (a.has_far_ovr) tmax = fminf(tmax, a.far_ovr);
        ok = isfinite(tmin) && isfinite(tmax) && (tmax > tmin + 1e-6f);
        if (!ok) { tmin = INFINITY; tmax = INFINITY; }
    } else {
        ok = isfinite(tmin) && isfinite(tmax) && (tmax > tmin + 1e-6f);
    }
    float* r = rays + 8 * p;
    reinterpret_cast<float4*>(r)[0] = make_float4(o[0], o[1], o[2], dw[0]);
    reinterpret_cast<float4*>(r)[1] = make_float4(dw[1], dw[2], tmin, tmax);
    if (valid) valid[p] = ok ? 1 : 0;
}

}  // namespace

extern "C" int acn_get_rays(int H, int W, float fx, float fy, float cx, float cy, int center_pixels, const float* c2w,
                            const float* aabb, float near_c, float far_c, int has_near_ovr, float near_ovr,
                            int has_far_ovr, float far_ovr, int apply_clamp, float* rays, uint8_t* valid,
                            void* stream) {
    ACN_REQUIRE(H >= 0 && W >= 0, "acn_get_rays: H, W must be >= 0");
    ACN_REQUIRE(c2w, "acn_get_rays: c2w is NULL");
    if ((int64_t)H * W == 0) return ACN_OK;
    ACN_REQUIRE(rays, "acn_get_rays: rays is NULL");
    ACN_REQUIRE((((uintptr_t)rays) & 15) == 0, "acn_get_rays: rays must be 16-byte aligned");
    RayGenArgs a{};
    a.H = H; a.W = W; a.fx = fx; a.fy = fy; a.cx = cx; a.cy = cy; a.center_pixels = center_pixels;
    for (int i = 0; i < 12; ++i) a.c2w[i] = c2w[i];
    a.has_aabb = aabb != nullptr;
    if (aabb) for (int i = 0; i < 6; ++i) a.aabb[i] = aabb[i];
    a.near_c = near_c; a.far_c = far_c;
    a.has_near_ovr = has_near_ovr; a.near_ovr = near_ovr;
    a.has_far_ovr = has_far_ovr; a.far_ovr = far_ovr;
    a.apply_clamp = apply_clamp;
    const int64_t n = (int64_t)H * W;
    hipLaunchKernelGGL(rays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a, rays, valid);
    return acn_check_launch("acn_get_rays");
}

extern "C" int acn_ray_directions(int H, int W, float fx, float fy, float cx, float cy, int center_pixels, float* dirs,
                                  void* stream) {
    ACN_REQUIRE(H >= 0 && W >= 0, "acn_ray_directions: H, W must be >= 0");
    const int64_t n = (int64_t)H * W;
    if (n == 0) return ACN_OK;
    ACN_REQUIRE(dirs, "acn_ray_directions: dirs is NULL");
    hipLaunchKernelGGL(dirs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, H, W, fx, fy,
                       cx, cy, center_pixels, dirs);
    return acn_check_launch("acn_ray_directions");
}

extern "C" int acn_rays_from_dirs(const float* dirs, int64_t N, const float* c2w, const float* aabb, float near_c,
                                  float far_c, float eps, float max_bound, float invalid_value, float* rays,
                                  void* stream) {
    ACN_REQUIRE(N >= 0 && c2w, "acn_rays_from_dirs: bad arguments");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(dirs && rays, "acn_rays_from_dirs: NULL pointer");
    Mat34 c;
    for (int i = 0; i < 12; ++i) c.m[i] = c2w[i];
    Box b{};
    if (aabb) for (int i = 0; i < 6; ++i) b.b[i] = aabb[i];
    hipLaunchKernelGGL(rays_from_dirs_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dirs,
                       N, c, aabb != nullptr, b, near_c, far_c, eps, max_bound, invalid_value, rays);
    return acn_check_launch("acn_rays_from_dirs");
}

extern "C" int acn_ray_aabb(const float* origins, const float* dirs, int64_t N, const float* aabb, float eps,
                            float max_bound, float invalid_value, float* tmin, float* tmax, void* stream) {
    ACN_REQUIRE(N >= 0 && aabb, "acn_ray_aabb: bad arguments");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(origins && dirs && tmin && tmax, "acn_ray_aabb: NULL pointer");
    Box b;
    for (int i = 0; i < 6; ++i) b.b[i] = aabb[i];
    hipLaunchKernelGGL(ray_aabb_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, origins,
                       dirs, N, b, eps, max_bound, invalid_value, tmin, tmax);
    return acn_check_launch("acn_ray_aabb");
}

extern "C" int acn_clamp_rays(float* rays, int64_t N, int apply, int has_near_ovr, float near_ovr, int has_far_ovr,
                              float far_ovr, float eps, float invalid_value, uint8_t* valid, void* stream) {
    ACN_REQUIRE(N >= 0, "acn_clamp_rays: N must be >= 0");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(rays, "acn_clamp_rays: NULL rays");
    hipLaunchKernelGGL(clamp_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, rays, N, apply,
                       has_near_ovr, near_ovr, has_far_ovr, far_ovr, eps, invalid_value, valid);
    return acn_check_launch("acn_clamp_rays");
}
