/*
 * occ_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker for the occupancy-grid renderer).
 *
 * The reference's occupancy path (nerfs/ray_rendering.py:349-558, models/inr/meta_ngp.py:318-443)
 * delegates marching to nerfacc 0.5.3 (OccGridEstimator.sampling -> traverse_grids), a third-party
 * CUDA extension that is NOT vendored in /root/reference and not installed here (SURVEY.md §8(c),
 * §8(f)).  This file restates nerfacc 0.5.3's published algorithm in plain C:
 *   - ray_aabb_intersect   (nerfacc/grid.py ray_aabb_intersect; slab test, misses -> miss_value)
 *   - traverse_grids       (nerfacc/grid.py traverse_grids + its CUDA kernel): per ray the 2L
 *     entry/exit times of the L nested level boxes are sorted; between consecutive events the
 *     finest level containing the ray is walked cell by cell with a 3-D DDA (setup_traversal /
 *     single_traversal, eps 1e-6 at both ends); samples sit on ONE global sequence
 *     t_{k+1} = t_k + clamp(t_k * cone_angle, step, 1e10) started at the ray's near plane, and a
 *     sample [t_k, t_{k+1}] is emitted iff its midpoint falls inside an occupied cell.
 * PARITY UNPINNED against nerfacc itself (no nerfacc source, binary or fixture exists here); the
 * reference's own glue around it is pinned by tests/golden/occ_*.npz (make_golden.py runs the
 * reference with a nerfacc stand-in built on this restatement).  Compiled -ffp-contract=off; the
 * HIP kernels (adaptive_city_nerf_amd/csrc/occ.hip) follow the same float op sequence, so sample
 * lists are compared bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* nerfacc device_ray_aabb_intersect: aabb = [xmin, ymin, zmin, xmax, ymax, zmax] */
static int ray_aabb(const float* o, const float* d, const float* aabb, float near_plane, float far_plane,
                    float miss, float* t_min, float* t_max) {
    float tmin = (aabb[0] - o[0]) / d[0], tmax = (aabb[3] - o[0]) / d[0];
    if (tmin > tmax) { float t = tmin; tmin = tmax; tmax = t; }
    float tymin = (aabb[1] - o[1]) / d[1], tymax = (aabb[4] - o[1]) / d[1];
    if (tymin > tymax) { float t = tymin; tymin = tymax; tymax = t; }
    if (tmin > tymax || tymin > tmax) { *t_min = miss; *t_max = miss; return 0; }
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (aabb[2] - o[2]) / d[2], tzmax = (aabb[5] - o[2]) / d[2];
    if (tzmin > tzmax) { float t = tzmin; tzmin = tzmax; tzmax = t; }
    if (tmin > tzmax || tzmin > tmax) { *t_min = miss; *t_max = miss; return 0; }
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    *t_min = fmaxf(tmin, near_plane);
    *t_max = fminf(tmax, far_plane);
    return 1;
}

void oracle_occ_ray_aabb(const float* rays_o, const float* rays_d, int64_t N, const float* aabbs, int n_aabbs,
                         float near_plane, float far_plane, float miss, float* t_mins, float* t_maxs, uint8_t* hits) {
    for (int64_t i = 0; i < N; ++i)
        for (int a = 0; a < n_aabbs; ++a) {
            const int64_t k = i * n_aabbs + a;
            hits[k] = (uint8_t)ray_aabb(rays_o + 3 * i, rays_d + 3 * i, aabbs + 6 * a, near_plane, far_plane, miss,
                                        &t_mins[k], &t_maxs[k]);
        }
}

/* nerfacc calc_dt */
static inline float calc_dt(float t, float cone, float dt_min, float dt_max) {
    float v = t * cone;
    v = fmaxf(v, dt_min);
    return fminf(v, dt_max);
}

#define OCC_MAX_ITERS (1 << 22)

/* clamp((int)v, 0, n-1) (make_int3 truncation then clamp), defined for +-inf / NaN too */
static inline int cell_index(float v, int n) {
    if (!(v >= 0.0f)) return 0;
    if (v >= (float)n) return n - 1;
    const int i = (int)v;
    return i > n - 1 ? n - 1 : i;
}

/* one ray of traverse_grids (first pass when t0 == NULL: count only).  Returns the sample count. */
static int64_t traverse_ray(const float* o, const float* d, float near_plane, float far_plane, const uint8_t* bin,
                            const float* aabbs, int L, const int* res, float step, float cone, float* t0, float* t1) {
    enum { MAXL = 16 };
    float ts[2 * MAXL];
    int ti[2 * MAXL];
    int hit[MAXL];
    for (int l = 0; l < L; ++l) {
        float a, b;
        hit[l] = ray_aabb(o, d, aabbs + 6 * l, -INFINITY, INFINITY, INFINITY, &a, &b);
        ts[l] = a;
        ts[L + l] = b;
    }
    for (int i = 0; i < 2 * L; ++i) ti[i] = i;
    /* torch.sort(cat([t_mins, t_maxs])): stable insertion sort by value (ties keep index order) */
    for (int i = 1; i < 2 * L; ++i) {
        float v = ts[i];
        int x = ti[i], j = i - 1;
        while (j >= 0 && ts[j] > v) { ts[j + 1] = ts[j]; ti[j + 1] = ti[j]; --j; }
        ts[j + 1] = v;
        ti[j + 1] = x;
    }
    const float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
    const float eps = 1e-6f;
    int64_t n = 0;
    int64_t budget = OCC_MAX_ITERS; /* termination guard shared with the HIP kernel (float absorption) */
    float t_last = near_plane;
    int continuous = 0;
    for (int i = 0; i < 2 * L - 1; ++i) {
        const int entering = ti[i] < L;
        int level = ti[i] % L;
        if (!hit[level]) continue;
        if (!entering) {
            if (ti[i + 1] < L) continue; /* leaving into the outside */
            level = ti[i + 1] % L;
            if (!hit[level]) continue;
        }
        const float this_tmin = fmaxf(ts[i], near_plane);
        const float this_tmax = fminf(ts[i + 1], far_plane);
        if (!(this_tmin < this_tmax)) continue; /* nerfacc: this_tmin >= this_tmax (NaN-safe here) */
        if (!continuous) {
            for (;;) { /* march until the midpoint is right after this_tmin */
                if (--budget < 0) return n;
                const float dt = calc_dt(t_last, cone, step, 1e10f);
                if (t_last + dt * 0.5f >= this_tmin) break;
                t_last += dt;
            }
        }
        const float* bmin = aabbs + 6 * level;
        const float* bmax = bmin + 3;
        int cur[3], fin[3], stp[3];
        float tdist[3], delta[3];
        for (int a = 0; a < 3; ++a) {
            const float r = (float)res[a];
            const float vs = (bmax[a] - bmin[a]) / r;
            const float ps = o[a] + d[a] * (this_tmin + eps);
            const float pe = o[a] + d[a] * (this_tmax - eps);
            cur[a] = cell_index((ps - bmin[a]) / (bmax[a] - bmin[a]) * r, res[a]);
            fin[a] = cell_index((pe - bmin[a]) / (bmax[a] - bmin[a]) * r, res[a]);
            const int start = cur[a] + (d[a] > 0.0f ? 1 : 0);
            const float tm = ((bmin[a] + ((float)start * vs)) - o[a]) * inv[a];
            tdist[a] = d[a] == 0.0f ? this_tmax : tm;
            const float sf = d[a] == 0.0f ? 0.0f : (d[a] > 0.0f ? 1.0f : -1.0f);
            stp[a] = (int)sf;
            const float dtmp = vs * inv[a] * sf;
            delta[a] = d[a] == 0.0f ? this_tmax : dtmp;
        }
        const int ovf[3] = {fin[0] + stp[0], fin[1] + stp[1], fin[2] + stp[2]};
        for (;;) {
            float t_trav = fminf(tdist[0], fminf(tdist[1], tdist[2]));
            t_trav = fminf(t_trav, this_tmax);
            const int64_t cell = (int64_t)level * res[0] * res[1] * res[2] + (int64_t)cur[0] * res[1] * res[2] +
                                 (int64_t)cur[1] * res[2] + cur[2];
            if (!bin[cell]) {
                for (;;) {
                    if (--budget < 0) return n;
                    const float dt = calc_dt(t_last, cone, step, 1e10f);
                    if (t_last + dt * 0.5f >= t_trav) break;
                    t_last += dt;
                }
                continuous = 0;
            } else {
                for (;;) {
                    if (--budget < 0) return n;
                    const float dt = calc_dt(t_last, cone, step, 1e10f);
                    if (t_last + dt * 0.5f >= t_trav) break;
                    const float t_next = t_last + dt;
                    if (t0) { t0[n] = t_last; t1[n] = t_next; }
                    ++n;
                    continuous = 1;
                    t_last = t_next;
                    if (t_next >= t_trav) break;
                }
            }
            if (--budget < 0) return n;
            /* single_traversal */
            int ax;
            if (tdist[0] < tdist[1] && tdist[0] < tdist[2]) ax = 0;
            else if (tdist[1] < tdist[2]) ax = 1;
            else ax = 2;
            cur[ax] += stp[ax];
            tdist[ax] += delta[ax];
            if (cur[ax] == ovf[ax]) break;
            /* guard (not in nerfacc, where this case reads out of bounds): a DDA that left the grid
               without meeting its overflow index stops here */
            if (cur[ax] < 0 || cur[ax] >= res[ax]) break;
        }
    }
    return n;
}

/* traverse_grids over N rays.  offsets == NULL: counts[i] <- samples of ray i.  Otherwise ray i
   writes its samples at offsets[i] (ray_idx, t0, t1). */
void oracle_occ_traverse(const float* rays_o, const float* rays_d, int64_t N, const float* near_planes,
                         const float* far_planes, const uint8_t* binaries, const float* aabbs, int L, const int* res,
                         float step, float cone, int64_t* counts, const int64_t* offsets, int64_t* ray_idx,
                         float* t0, float* t1) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < N; ++i) {
        if (!offsets) {
            counts[i] = traverse_ray(rays_o + 3 * i, rays_d + 3 * i, near_planes[i], far_planes[i], binaries, aabbs,
                                     L, res, step, cone, NULL, NULL);
        } else {
            const int64_t b = offsets[i];
            const int64_t n = traverse_ray(rays_o + 3 * i, rays_d + 3 * i, near_planes[i], far_planes[i], binaries,
                                           aabbs, L, res, step, cone, t0 + b, t1 + b);
            for (int64_t k = 0; k < n; ++k) ray_idx[b + k] = i;
        }
    }
}
