/* cluster_oracle.c -- TEST INFRASTRUCTURE ONLY: C restatement of scripts/create_clusters.py's
 * per-ray routing (compute_voronoi_opt :386-556 and compute_voronoi_orig :559-634) and of the ray
 * generation its main() uses (get_ray_directions + get_rays(scene_box, aabb_max_bound=1e10,
 * aabb_invalid_value=inf) + clamp_rays_near_far, :790-803).  Only tests/ and bench.py's cpu_baseline
 * call it (through oracle/cluster_ref.py).
 *
 * Float op order restated from the reference's torch ops on the CPU, checked against the reference
 * itself (tests/golden/clusters.npz, tests/test_cluster_oracle.py):
 *   linspace(0, 1, S)       one fma per element (start + step*i / end - step*(S-1-i))
 *   lerp(near, far, z)      fma(w, far - near, near) for |w| < 0.5, else fma(w - 1, far - near, far)
 *   x = o + d * t           mul, then add
 *   |x|^2 = x.pow(2).sum()  sequential
 *   cdist (orig)            [-2x, |x|^2, 1] . [c, 1, |c|^2] as MKL sgemm's sequential fma chain, then
 *                           clamp_min(0) and sqrt.  torch's CPU sqrt (MKL VML) is not correctly
 *                           rounded: ~0.7% of distances differ by 1 ulp, so only rays whose decision
 *                           sits within an ulp of the margin can differ (the tests bound them).
 *   opt (GPU in the reference, TF32 GEMMs there on Ampere+): d2 = (|x|^2 + |c|^2) - 2 * (x . c) with
 *                           the dot as an fma chain -- parity with the reference unpinned; the HIP
 *                           kernel is pinned to this restatement bit for bit.
 * -ffp-contract=off (Makefile): no implicit FMA contraction.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static float lin01(int i, int S) {
    if (S == 1) return 0.0f;
    const float step = 1.0f / (float)(S - 1);
    return i < S / 2 ? fmaf(step, (float)i, 0.0f) : fmaf(-step, (float)(S - 1 - i), 1.0f);
}

static float lerp_t(float a, float b, float w) {
    return fabsf(w) < 0.5f ? fmaf(w, b - a, a) : fmaf(w - 1.0f, b - a, b);
}

static float nanmin_f(float a, float b) { return (isnan(a) || isnan(b)) ? NAN : fminf(a, b); }

/* rays of one image: directions (RUB), world rays via c2w (3,4), slab test against aabb (2,3) with
 * max_bound 1e10 / invalid inf, then the near/far override (has_* flags) and validity. */
void oracle_cluster_rays(int H, int W, float fx, float fy, float cx, float cy, int center_pixels, const float* c2w,
                         const float* aabb, int has_near, float near_v, int has_far, float far_v, float* rays,
                         uint8_t* valid) {
    for (int64_t p = 0; p < (int64_t)H * W; ++p) {
        const int j = (int)(p / W), i = (int)(p % W);
        float fi = (float)i, fj = (float)j;
        if (center_pixels) { fi = fi + 0.5f; fj = fj + 0.5f; }
        float dx = (fi - cx) / fx, dy = -((fj - cy) / fy), dz = -1.0f;
        const float n = fmaxf(sqrtf(fmaf(dz, dz, fmaf(dy, dy, dx * dx))), 1e-12f);
        dx = dx / n; dy = dy / n; dz = dz / n;
        float d[3], o[3];
        for (int a = 0; a < 3; ++a) {
            d[a] = fmaf(dz, c2w[4 * a + 2], fmaf(dy, c2w[4 * a + 1], dx * c2w[4 * a + 0]));
            o[a] = c2w[4 * a + 3];
        }
        float t0m = -INFINITY, t1m = INFINITY;
        for (int a = 0; a < 3; ++a) {
            float rd = d[a];
            if (fabsf(rd) < 1e-8f) rd = (rd >= 0.0f) ? 1e-8f : -1e-8f;
            const float inv = 1.0f / rd;
            const float t0 = (aabb[a] - o[a]) * inv, t1 = (aabb[3 + a] - o[a]) * inv;
            t0m = fmaxf(t0m, fminf(t0, t1));
            t1m = fminf(t1m, fmaxf(t0, t1));
        }
        float tn = fminf(fmaxf(t0m, 0.0f), 1e10f), tf = fminf(fmaxf(t1m, 0.0f), 1e10f);
        if (tf <= tn) { tn = INFINITY; tf = INFINITY; }
        if (has_near) tn = fmaxf(tn, near_v);
        if (has_far) tf = fminf(tf, far_v);
        const int ok = isfinite(tn) && isfinite(tf) && (tf > tn + 1e-6f);
        if (!ok) { tn = INFINITY; tf = INFINITY; }
        float* r = rays + 8 * p;
        r[0] = o[0]; r[1] = o[1]; r[2] = o[2]; r[3] = d[0]; r[4] = d[1]; r[5] = d[2]; r[6] = tn; r[7] = tf;
        valid[p] = (uint8_t)ok;
    }
}

/* bits[r]: bit c = ray r belongs to centroid c.  mode 0 opt strict, 1 opt overlap, 2 orig.
 * update (opt modes): mins/maxs (C,3) lowered/raised in place by the assigned samples, counts (C)
 * += assigned samples, nan_flag[c] = 1 when an assigned sample is NaN. */
void oracle_voronoi(const float* rays, int64_t N, int S, const float* cents, int C, int cluster_2d, int mode,
                    double boundary_margin, int update, uint64_t* bits, float* mins, float* maxs, int64_t* counts,
                    int32_t* nan_flag) {
    const int st = cluster_2d ? 1 : 0, k = cluster_2d ? 2 : 3;
    const float m2 = (float)(boundary_margin * boundary_margin), bm = (float)boundary_margin;
    float* cs = (float*)malloc(sizeof(float) * 3 * (size_t)C);
    float* cn = (float*)malloc(sizeof(float) * (size_t)C);
    float* v = (float*)malloc(sizeof(float) * (size_t)C);
    float* rmin = (float*)malloc(sizeof(float) * (size_t)C);
    for (int c = 0; c < C; ++c) {
        for (int j = 0; j < k; ++j) cs[3 * c + j] = cents[3 * c + st + j];
        float s = cs[3 * c] * cs[3 * c];
        for (int j = 1; j < k; ++j) s = s + cs[3 * c + j] * cs[3 * c + j];
        cn[c] = s;
    }
    for (int64_t r = 0; r < N; ++r) {
        const float* ry = rays + 8 * r;
        uint64_t has = 0;
        for (int c = 0; c < C; ++c) rmin[c] = INFINITY;
        for (int s = 0; s < S; ++s) {
            const float t = lerp_t(ry[6], ry[7], lin01(s, S));
            float x[3], xf[3];
            for (int a = 0; a < 3; ++a) xf[a] = ry[a] + ry[3 + a] * t;
            for (int j = 0; j < k; ++j) x[j] = xf[st + j];
            float x2 = x[0] * x[0];
            for (int j = 1; j < k; ++j) x2 = x2 + x[j] * x[j];
            if (mode == 2) {
                for (int c = 0; c < C; ++c) {
                    float acc = (-2.0f * x[0]) * cs[3 * c];
                    for (int j = 1; j < k; ++j) acc = fmaf(-2.0f * x[j], cs[3 * c + j], acc);
                    acc = fmaf(x2, 1.0f, acc);
                    acc = fmaf(1.0f, cn[c], acc);
                    v[c] = sqrtf(acc < 0.0f ? 0.0f : acc);
                }
                float m = v[0];
                for (int c = 1; c < C; ++c) m = nanmin_f(m, v[c]);
                const float den = m + 1e-8f;
                for (int c = 0; c < C; ++c) rmin[c] = nanmin_f(rmin[c], v[c] / den);
                continue;
            }
            for (int c = 0; c < C; ++c) {
                float ip = x[0] * cs[3 * c];
                for (int j = 1; j < k; ++j) ip = fmaf(x[j], cs[3 * c + j], ip);
                const float d2 = (x2 + cn[c]) - 2.0f * ip;
                v[c] = d2 < 0.0f ? 0.0f : d2;
            }
            uint64_t sel = 0;
            if (mode == 0) {
                int best = 0;
                float bv = v[0];
                for (int c = 1; c < C; ++c)
                    if (!isnan(bv) && (v[c] < bv || isnan(v[c]))) { best = c; bv = v[c]; }
                sel = 1ull << best;
            } else {
                float m = v[0];
                for (int c = 1; c < C; ++c) m = nanmin_f(m, v[c]);
                const float thr = m2 * m;
                for (int c = 0; c < C; ++c) if (v[c] <= thr) sel |= 1ull << c;
            }
            has |= sel;
            if (update) {
                for (int c = 0; c < C; ++c) {
                    if (!((sel >> c) & 1ull)) continue;
                    counts[c] += 1;
                    if (isnan(t)) { nan_flag[c] = 1; continue; }
                    for (int a = 0; a < 3; ++a) {
                        if (xf[a] < mins[3 * c + a]) mins[3 * c + a] = xf[a];
                        if (xf[a] > maxs[3 * c + a]) maxs[3 * c + a] = xf[a];
                    }
                }
            }
        }
        if (mode == 2)
            for (int c = 0; c < C; ++c) if (rmin[c] <= bm) has |= 1ull << c;
        bits[r] = has;
    }
    free(cs); free(cn); free(v); free(rmin);
}
