// occ.hip -- occupancy-grid ray marching and packed-sample compositing (gfx950).
//
// The reference's occupancy renderer (nerfs/ray_rendering.py:349-558; models/inr/meta_ngp.py:318-443)
// runs on nerfacc 0.5.3 (OccGridEstimator.sampling / traverse_grids / render_weight_from_density /
// accumulate_along_rays; third-party, not vendored).  These kernels restate that
// published algorithm MI355X-first:
//   * the occupancy grid is read as a 1-bit-per-cell image (levels x 128^3 bits = 1 MiB at the
//     reference's 4 x 128^3, L2-resident) derived from the reference's bool `binaries` buffer;
//   * traversal is one lane per ray (the t_{k+1} = t_k + calc_dt(t_k) recurrence is sequential and
//     its float roundings define the samples), in two passes: count, then fill at the offsets the
//     caller's scan produced -- the packed (ray-major) layout nerfacc returns;
//   * the per-expert sample lists of the container renderer are merged per ray with a K-way merge
//     (boundary union, _merge_segments_union ray_rendering.py:196-258) instead of a global sort;
//   * compositing over packed samples is a segmented scan per ray (one wave per ray, 64 samples per
//     step), deterministic (no atomics), with fused backward.
// Float op order of the traversal follows oracle/occ_oracle.c exactly (-ffp-contract=off), so the
// sample lists agree bit for bit with the oracle.
#include "acn_internal.h"

using namespace acn;

namespace {

constexpr int kOccMaxLevels = 8;
constexpr int64_t kOccMaxIters = 1 << 22;  // termination guard (same as the oracle)

__device__ __forceinline__ bool ray_aabb_slab(const float o[3], const float d[3], const float* aabb, float near_plane,
                                              float far_plane, float miss, float& t_min, float& t_max) {
    float tmin = (aabb[0] - o[0]) / d[0], tmax = (aabb[3] - o[0]) / d[0];
    if (tmin > tmax) { const float t = tmin; tmin = tmax; tmax = t; }
    float tymin = (aabb[1] - o[1]) / d[1], tymax = (aabb[4] - o[1]) / d[1];
    if (tymin > tymax) { const float t = tymin; tymin = tymax; tymax = t; }
    if (tmin > tymax || tymin > tmax) { t_min = miss; t_max = miss; return false; }
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (aabb[2] - o[2]) / d[2], tzmax = (aabb[5] - o[2]) / d[2];
    if (tzmin > tzmax) { const float t = tzmin; tzmin = tzmax; tzmax = t; }
    if (tmin > tzmax || tzmin > tmax) { t_min = miss; t_max = miss; return false; }
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    t_min = fmaxf(tmin, near_plane);
    t_max = fminf(tmax, far_plane);
    return true;
}

__device__ __forceinline__ float calc_dt(float t, float cone, float dt_min) {
    return fminf(fmaxf(t * cone, dt_min), 1e10f);
}

__device__ __forceinline__ int cell_index(float v, int n) {
    if (!(v >= 0.0f)) return 0;
    if (v >= (float)n) return n - 1;
    const int i = (int)v;
    return i > n - 1 ? n - 1 : i;
}

// torch.maximum / torch.minimum / amax / amin propagate NaN
__device__ __forceinline__ float nmax(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fmaxf(a, b); }
__device__ __forceinline__ float nmin(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fminf(a, b); }

// _intersect_rays_aabb (ray_rendering.py:170-193): prefilter of the container renderer
__device__ __forceinline__ bool prefilter_hit(const float o[3], const float d[3], float near, float far,
                                              const float* box /*[min3, max3]*/) {
    float tmn = -INFINITY, tmx = INFINITY;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float inv = fabsf(d[a]) > 1e-9f ? 1.0f / d[a] : 1e9f;
        const float t0 = (box[a] - o[a]) * inv, t1 = (box[3 + a] - o[a]) * inv;
        const float lo = nmin(t0, t1), hi = nmax(t0, t1);
        tmn = a == 0 ? lo : nmax(tmn, lo);
        tmx = a == 0 ? hi : nmin(tmx, hi);
    }
    const float te = nmax(tmn, near), tx = nmin(tmx, far);
    return tx > te;
}

struct TraverseArgs {
    const float* rays_o;  // (N, ld_o) rows start with o
    const float* rays_d;  // (N, ld_d)
    int64_t ld_o, ld_d, N;
    const float* near;    // (N)
    const float* far;     // (N)
    const uint32_t* bits; // levels * cells / 32 words, bit c = binaries.flatten()[c]
    float aabbs[kOccMaxLevels][6];
    int32_t L, rx, ry, rz;
    float step, cone;
    int32_t has_prefilter;
    float prefilter[6];
    const float* pf_nf;     // (N, ld_pf): [near, far] of the prefilter (the rays' own columns 6, 7)
    int64_t ld_pf;
    int64_t* counts;        // pass 1 output (N)
    const int64_t* offsets; // pass 2 input (N), NULL in pass 1
    int64_t* ray_idx;       // pass 2 outputs (M)
    float* t0;
    float* t1;
};

// Per-ray event list of traverse_grids: the 2L entry/exit times of the nested level boxes, sorted
// (stable, ties keep index order, as torch.sort on the cat([t_mins, t_maxs]) of nerfacc).
struct RayEvents {
    float ts[2 * kOccMaxLevels];
    int ti[2 * kOccMaxLevels];
    bool hit[kOccMaxLevels];
};

__device__ __forceinline__ void ray_events(const TraverseArgs& a, const float o[3], const float d[3], RayEvents& ev) {
    const int L = a.L;
    for (int l = 0; l < L; ++l) {
        float x, y;
        ev.hit[l] = ray_aabb_slab(o, d, a.aabbs[l], -INFINITY, INFINITY, INFINITY, x, y);
        ev.ts[l] = x;
        ev.ts[L + l] = y;
    }
    for (int i = 0; i < 2 * L; ++i) ev.ti[i] = i;
    for (int i = 1; i < 2 * L; ++i) {
        const float v = ev.ts[i];
        const int x = ev.ti[i];
        int j = i - 1;
        while (j >= 0 && ev.ts[j] > v) { ev.ts[j + 1] = ev.ts[j]; ev.ti[j + 1] = ev.ti[j]; --j; }
        ev.ts[j + 1] = v;
        ev.ti[j + 1] = x;
    }
}

// Level interval of event i (the finest level containing the ray between events i and i+1) or -1.
__device__ __forceinline__ int interval_level(const TraverseArgs& a, const RayEvents& ev, int i, float near_plane,
                                              float far_plane, float& this_tmin, float& this_tmax) {
    const int L = a.L;
    const bool entering = ev.ti[i] < L;
    int level = ev.ti[i] % L;
    if (!ev.hit[level]) return -1;
    if (!entering) {
        if (ev.ti[i + 1] < L) return -1;  // leaving into the outside
        level = ev.ti[i + 1] % L;
        if (!ev.hit[level]) return -1;
    }
    this_tmin = fmaxf(ev.ts[i], near_plane);
    this_tmax = fminf(ev.ts[i + 1], far_plane);
    if (!(this_tmin < this_tmax)) return -1;
    return level;
}

// 3-D DDA over one level's grid between this_tmin and this_tmax (nerfacc setup_traversal /
// single_traversal, eps 1e-6 at both ends).
struct Dda {
    int cur[3], ovf[3], stp[3];
    float tdist[3], delta[3];
    int64_t lbase;
};

__device__ __forceinline__ void dda_setup(const TraverseArgs& a, const float o[3], const float d[3],
                                          const float inv[3], int level, float this_tmin, float this_tmax, Dda& g) {
    const int res[3] = {a.rx, a.ry, a.rz};
    const float eps = 1e-6f;
    const float* bmin = a.aabbs[level];
    const float* bmax = bmin + 3;
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
        const float r = (float)res[ax];
        const float vs = (bmax[ax] - bmin[ax]) / r;
        const float ps = o[ax] + d[ax] * (this_tmin + eps);
        const float pe = o[ax] + d[ax] * (this_tmax - eps);
        g.cur[ax] = cell_index((ps - bmin[ax]) / (bmax[ax] - bmin[ax]) * r, res[ax]);
        const int fin = cell_index((pe - bmin[ax]) / (bmax[ax] - bmin[ax]) * r, res[ax]);
        const int start = g.cur[ax] + (d[ax] > 0.0f ? 1 : 0);
        const float tm = ((bmin[ax] + ((float)start * vs)) - o[ax]) * inv[ax];
        g.tdist[ax] = d[ax] == 0.0f ? this_tmax : tm;
        const float sf = d[ax] == 0.0f ? 0.0f : (d[ax] > 0.0f ? 1.0f : -1.0f);
        g.stp[ax] = (int)sf;
        const float dtmp = vs * inv[ax] * sf;
        g.delta[ax] = d[ax] == 0.0f ? this_tmax : dtmp;
        g.ovf[ax] = fin + g.stp[ax];
    }
    g.lbase = (int64_t)level * ((int64_t)a.rx * a.ry * a.rz);
}

__device__ __forceinline__ int64_t dda_cell(const TraverseArgs& a, const Dda& g) {
    return g.lbase + ((int64_t)g.cur[0] * a.ry + g.cur[1]) * a.rz + g.cur[2];
}

// single_traversal; false when the walk leaves the interval (overflow index, or -- a guard nerfacc
// lacks, where it would read out of bounds -- the grid)
__device__ __forceinline__ bool dda_step(const TraverseArgs& a, Dda& g) {
    const int res[3] = {a.rx, a.ry, a.rz};
    int ax;
    if (g.tdist[0] < g.tdist[1] && g.tdist[0] < g.tdist[2]) ax = 0;
    else if (g.tdist[1] < g.tdist[2]) ax = 1;
    else ax = 2;
    g.cur[ax] += g.stp[ax];
    g.tdist[ax] += g.delta[ax];
    if (g.cur[ax] == g.ovf[ax]) return false;
    if (g.cur[ax] < 0 || g.cur[ax] >= res[ax]) return false;
    return true;
}

__device__ __forceinline__ bool occupied(const uint32_t* bits, int64_t cell) {
    return (bits[cell >> 5] >> (cell & 31)) & 1u;
}

// One ray of traverse_grids (oracle/occ_oracle.c traverse_ray, same float op order).  Writes at most
// `cap` samples to t0/t1 (if non-NULL) and returns the full sample count.
__device__ int64_t traverse_ray(const TraverseArgs& a, const RayEvents& ev, const float o[3], const float d[3],
                                const float inv[3], float near_plane, float far_plane, int64_t cap, float* t0,
                                float* t1) {
    int64_t n = 0, budget = kOccMaxIters;
    float t_last = near_plane;
    bool continuous = false;
    for (int i = 0; i < 2 * a.L - 1; ++i) {
        float this_tmin, this_tmax;
        const int level = interval_level(a, ev, i, near_plane, far_plane, this_tmin, this_tmax);
        if (level < 0) continue;
        if (!continuous) {
            for (;;) {
                if (--budget < 0) return n;
                const float dt = calc_dt(t_last, a.cone, a.step);
                if (t_last + dt * 0.5f >= this_tmin) break;
                t_last += dt;
            }
        }
        Dda g;
        dda_setup(a, o, d, inv, level, this_tmin, this_tmax, g);
        for (;;) {
            float t_trav = fminf(g.tdist[0], fminf(g.tdist[1], g.tdist[2]));
            t_trav = fminf(t_trav, this_tmax);
            if (!occupied(a.bits, dda_cell(a, g))) {
                for (;;) {
                    if (--budget < 0) return n;
                    const float dt = calc_dt(t_last, a.cone, a.step);
                    if (t_last + dt * 0.5f >= t_trav) break;
                    t_last += dt;
                }
                continuous = false;
            } else {
                for (;;) {
                    if (--budget < 0) return n;
                    const float dt = calc_dt(t_last, a.cone, a.step);
                    if (t_last + dt * 0.5f >= t_trav) break;
                    const float t_next = t_last + dt;
                    if (t0 && n < cap) { t0[n] = t_last; t1[n] = t_next; }
                    ++n;
                    continuous = true;
                    t_last = t_next;
                    if (t_next >= t_trav) break;
                }
            }
            if (--budget < 0) return n;
            if (!dda_step(a, g)) break;
        }
    }
    return n;
}

// offsets == NULL: counts[i] <- samples of ray i, and with cap > 0 its first cap samples are written
// to the scratch rows t0/t1 + i * cap (single-pass mode, compacted by occ_compact_kernel); offsets !=
// NULL: ray i writes all its samples at offsets[i] (second pass of the two-pass mode).
__global__ void __launch_bounds__(64) occ_traverse_kernel(TraverseArgs a, int64_t cap) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.N) return;
    const float* po = a.rays_o + i * a.ld_o;
    const float* pd = a.rays_d + i * a.ld_d;
    const float o[3] = {po[0], po[1], po[2]}, d[3] = {pd[0], pd[1], pd[2]};
    const float nr = a.near[i], fr = a.far[i];
    if (a.has_prefilter && !prefilter_hit(o, d, a.pf_nf[i * a.ld_pf], a.pf_nf[i * a.ld_pf + 1], a.prefilter)) {
        if (!a.offsets) a.counts[i] = 0;
        return;
    }
    RayEvents ev;
    ray_events(a, o, d, ev);
    const float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
    if (!a.offsets) {
        a.counts[i] = traverse_ray(a, ev, o, d, inv, nr, fr, cap, cap > 0 ? a.t0 + i * cap : nullptr,
                                   cap > 0 ? a.t1 + i * cap : nullptr);
        return;
    }
    const int64_t b = a.offsets[i];
    const int64_t n = traverse_ray(a, ev, o, d, inv, nr, fr, INT64_MAX, a.t0 + b, a.t1 + b);
    for (int64_t k = 0; k < n; ++k) a.ray_idx[b + k] = i;
}

// single-pass mode: scratch rows (cap per ray) -> packed arrays at the scanned offsets, wave per ray
__global__ void __launch_bounds__(256) occ_compact_kernel(const float* s0, const float* s1, int64_t cap,
                                                          const int64_t* counts, const int64_t* offsets, int64_t N,
                                                          int64_t* ray_idx, float* t0, float* t1) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < N; r += nw) {
        const int64_t n = counts[r], b = offsets[r];
        for (int64_t k = lane; k < n; k += 64) {
            t0[b + k] = s0[r * cap + k];
            t1[b + k] = s1[r * cap + k];
            ray_idx[b + k] = r;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Boundary union of K per-expert packed sample lists (ray_rendering.py:196-258).  Per ray, each
// expert's boundaries t0[0], t1[0], t0[1], t1[1], ... are non-decreasing; the union is the sorted
// set of distinct values (torch.unique(sorted=True)); consecutive pairs are the merged segments.
struct UnionArgs {
    int32_t K;
    int64_t N;
    const int64_t* starts[kMaxK];  // per expert: (N) first sample of each ray
    const int64_t* counts[kMaxK];  // per expert: (N) samples of each ray
    const float* t0[kMaxK];
    const float* t1[kMaxK];
    int64_t* out_counts;           // pass 1
    const int64_t* offsets;        // pass 2
    int64_t* ray_idx;
    float* m0;
    float* m1;
};

__global__ void __launch_bounds__(256) occ_union_kernel(UnionArgs a) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.N) return;
    int64_t pos[kMaxK], end[kMaxK], base[kMaxK];
    for (int k = 0; k < a.K; ++k) {
        base[k] = a.starts[k][r];
        pos[k] = 0;
        end[k] = 2 * a.counts[k][r];
    }
    int64_t nuniq = 0, w = a.offsets ? a.offsets[r] : 0;
    float prev = 0.0f;
    for (;;) {
        int kb = -1;
        float vb = 0.0f;
        for (int k = 0; k < a.K; ++k) {
            if (pos[k] >= end[k]) continue;
            const int64_t e = pos[k];
            const float v = (e & 1) ? a.t1[k][base[k] + (e >> 1)] : a.t0[k][base[k] + (e >> 1)];
            if (kb < 0 || v < vb) { kb = k; vb = v; }
        }
        if (kb < 0) break;
        ++pos[kb];
        if (nuniq > 0 && vb == prev) continue;
        if (a.offsets && nuniq > 0) {
            a.m0[w] = prev;
            a.m1[w] = vb;
            a.ray_idx[w] = r;
            ++w;
        }
        prev = vb;
        ++nuniq;
    }
    if (!a.offsets) a.out_counts[r] = nuniq >= 2 ? nuniq - 1 : 0;
}

// ------------------------------------------------------------------------------------------
// nerfacc render_weight_from_density over packed samples (one wave per ray, 64 samples per step):
// sdt = sigma * (t1 - t0); alpha = 1 - exp(-sdt); trans = exp(-exclusive_sum(sdt)); w = trans * alpha.
// The segmented exclusive sum is carried in double.
__device__ __forceinline__ double wave_incl_scan(double v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const double y = __shfl_up(v, off);
        if (lane >= off) v += y;
    }
    return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

struct PackedWArgs {
    const float *sigmas, *t0, *t1;
    const int64_t *starts, *counts;
    int64_t N;
    float *weights, *trans, *alphas;
};

__global__ void __launch_bounds__(256) packed_weights_kernel(PackedWArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < a.N; r += nw) {
        const int64_t b = a.starts[r], n = a.counts[r];
        double carry = 0.0;
        for (int64_t s0 = 0; s0 < n; s0 += 64) {
            const int64_t i = b + s0 + lane;
            const bool v = s0 + lane < n;
            const float sdt = v ? a.sigmas[i] * (a.t1[i] - a.t0[i]) : 0.0f;
            const double incl = wave_incl_scan((double)sdt, lane);
            const float excl = (float)(carry + incl - (double)sdt);
            if (v) {
                const float alpha = 1.0f - expf(-sdt);
                const float tr = expf(-excl);
                a.weights[i] = tr * alpha;
                if (a.trans) a.trans[i] = tr;
                if (a.alphas) a.alphas[i] = alpha;
            }
            carry += __shfl(incl, 63);
        }
    }
}

// backward of weights w.r.t. sigmas: g_sdt_i = g_w_i * T_i * (1 - a_i) - sum_{k>i} g_w_k * w_k
//                                   (+ g_T_i terms: d T_k / d sdt_i = -T_k for k > i)
struct PackedWBwdArgs {
    const float *sigmas, *t0, *t1, *weights, *trans, *alphas;
    const float *g_w, *g_trans, *g_alphas;  // any may be NULL
    const int64_t *starts, *counts;
    int64_t N;
    float* g_sigmas;
};

__global__ void __launch_bounds__(256) packed_weights_bwd_kernel(PackedWBwdArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < a.N; r += nw) {
        const int64_t b = a.starts[r], n = a.counts[r];
        // total of q_k = g_w_k * w_k + g_T_k * T_k over the ray, then walk front to back
        double tot = 0.0;
        for (int64_t s0 = 0; s0 < n; s0 += 64) {
            const int64_t i = b + s0 + lane;
            double q = 0.0;
            if (s0 + lane < n) {
                if (a.g_w) q += (double)a.g_w[i] * (double)a.weights[i];
                if (a.g_trans) q += (double)a.g_trans[i] * (double)a.trans[i];
            }
            tot += wave_sum_d(q);
        }
        double carry = 0.0;  // sum of q over samples before this step
        for (int64_t s0 = 0; s0 < n; s0 += 64) {
            const int64_t i = b + s0 + lane;
            const bool v = s0 + lane < n;
            double q = 0.0;
            float gs = 0.0f;
            if (v) {
                if (a.g_w) q += (double)a.g_w[i] * (double)a.weights[i];
                if (a.g_trans) q += (double)a.g_trans[i] * (double)a.trans[i];
            }
            const double incl = wave_incl_scan(q, lane);
            if (v) {
                const double after = tot - (carry + incl);  // sum_{k>i} q_k
                const float alpha = a.alphas[i], tr = a.trans[i];
                double g = 0.0;
                if (a.g_w) g += (double)a.g_w[i] * (double)tr * (1.0 - (double)alpha);
                if (a.g_alphas) g += (double)a.g_alphas[i] * (1.0 - (double)alpha);
                g -= after;
                gs = (float)(g * (double)(a.t1[i] - a.t0[i]));
                a.g_sigmas[i] = gs;
            }
            carry += __shfl(incl, 63);
        }
    }
}

// accumulate_along_rays: out[r, c] = sum_i w_i * v_i[c] over ray r's samples (v = NULL: C = 1, v = 1)
struct PackedAccArgs {
    const float* w;
    const float* v;   // (M, C) or NULL
    int32_t C;
    const int64_t *starts, *counts;
    int64_t N;
    float* out;       // (N, C)
};

__global__ void __launch_bounds__(256) packed_accumulate_kernel(PackedAccArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < a.N; r += nw) {
        const int64_t b = a.starts[r], n = a.counts[r];
        for (int c = 0; c < a.C; ++c) {
            float s = 0.0f;
            for (int64_t k = lane; k < n; k += 64) {
                const int64_t i = b + k;
                s += a.v ? a.w[i] * a.v[i * a.C + c] : a.w[i];
            }
            double t = wave_sum_d((double)s);
            if (lane == 0) a.out[r * a.C + c] = (float)t;
        }
    }
}

// backward: g_w_i = sum_c g_out[r_i, c] * v_i[c]; g_v_i[c] = w_i * g_out[r_i, c]
__global__ void __launch_bounds__(256) packed_accumulate_bwd_kernel(const float* w, const float* v, int C,
                                                                     const int64_t* ray_idx, int64_t M,
                                                                     const float* g_out, float* g_w, float* g_v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const int64_t r = ray_idx[i];
    float gw = 0.0f;
    for (int c = 0; c < C; ++c) {
        const float g = g_out[r * C + c];
        gw += v ? g * v[i * C + c] : g;
        if (g_v) g_v[i * C + c] = w[i] * g;
    }
    if (g_w) g_w[i] = gw;
}

// ------------------------------------------------------------------------------------------
// occupancy-grid maintenance (OccGridEstimator._update / mark_invisible_cells)
__global__ void __launch_bounds__(256) occ_pack_bits_kernel(const uint8_t* bin, int64_t n, uint32_t* bits) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w * 32 >= n) return;
    uint32_t m = 0u;
    for (int b = 0; b < 32; ++b) {
        const int64_t c = w * 32 + b;
        if (c < n && bin[c]) m |= 1u << b;
    }
    bits[w] = m;
}

// x = aabb_min + ((coord + u) / res) * (aabb_max - aabb_min)   (nerfacc _update, cell centres jittered)
__global__ void __launch_bounds__(256) occ_cell_points_kernel(const int64_t* idx, int64_t n, const float* u,
                                                              float4 bmin_r, float4 bmax_r, int rx, int ry, int rz,
                                                              float* x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t c = idx[i];
    const int64_t ci = c / ((int64_t)ry * rz), cj = (c / rz) % ry, ck = c % rz;
    const float co[3] = {(float)ci, (float)cj, (float)ck};
    const float rs[3] = {(float)rx, (float)ry, (float)rz};
    const float mn[3] = {bmin_r.x, bmin_r.y, bmin_r.z}, mx[3] = {bmax_r.x, bmax_r.y, bmax_r.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float v = (co[a] + (u ? u[i * 3 + a] : 0.0f)) / rs[a];
        x[i * 3 + a] = mn[a] + v * (mx[a] - mn[a]);
    }
}

// occs[c] = max(occs[c] * decay, occ)  (torch.maximum: NaN propagates)
__global__ void __launch_bounds__(256) occ_ema_kernel(float* occs, const int64_t* cell_ids, const float* occ, int64_t n,
                                                      float decay) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t c = cell_ids[i];
    const float a = occs[c] * decay, b = occ[i];
    occs[c] = nmax(a, b);
}

// sum and count of occs >= 0 (partials per block, double)
__global__ void __launch_bounds__(256) occ_mean_partial_kernel(const float* occs, int64_t n, double* part) {
    double s = 0.0, c = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = occs[i];
        if (v >= 0.0f) { s += (double)v; c += 1.0; }
    }
    __shared__ double ss[4], sc[4];
    s = wave_sum_d(s);
    c = wave_sum_d(c);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) { ss[wv] = s; sc[wv] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = ss[0] + ss[1] + ss[2] + ss[3];
        part[2 * blockIdx.x + 1] = sc[0] + sc[1] + sc[2] + sc[3];
    }
}

// thre = min(mean(occs[occs >= 0]), occ_thre) (NaN when no cell qualifies); binaries = occs > thre
__global__ void __launch_bounds__(256) occ_binarize_kernel(const float* occs, int64_t n, const double* part, int nparts,
                                                           float occ_thre, uint8_t* bin, uint32_t* bits,
                                                           float* thre_out) {
    __shared__ float thre;
    if (threadIdx.x == 0) {
        double s = 0.0, c = 0.0;
        for (int p = 0; p < nparts; ++p) { s += part[2 * p]; c += part[2 * p + 1]; }
        const float mean = c > 0.0 ? (float)(s / c) : __builtin_nanf("");
        thre = mean != mean ? mean : fminf(mean, occ_thre);
        if (blockIdx.x == 0 && thre_out) *thre_out = thre;
    }
    __syncthreads();
    const float t = thre;
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w * 32 >= n) return;
    uint32_t m = 0u;
    for (int b = 0; b < 32; ++b) {
        const int64_t c = w * 32 + b;
        if (c < n) {
            const bool o = occs[c] > t;
            bin[c] = o;
            if (o) m |= 1u << b;
        }
    }
    if (bits) bits[w] = m;
}

// mark_invisible_cells: a cell (coords / (res - 1) mapped into the level box) is visible if some
// camera sees it in front of near_plane inside the image; occs <- 0 if visible else -1.
struct MarkArgs {
    const float* Ks;     // (C, 3, 3) or (1, 3, 3)
    const float* c2w;    // (C, 3, 4) rows of the RDF camera-to-world
    int32_t nK, nc2w, C;
    int32_t width, height;
    float near_plane;
    float bmin[3], bmax[3];
    int32_t rx, ry, rz;
    const int64_t* idx;  // cells of this level to test
    int64_t n;
    float* occs_level;   // occs + level * cells
};

__global__ void __launch_bounds__(256) occ_mark_invisible_kernel(MarkArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int64_t c = a.idx[i];
    const int64_t ci = c / ((int64_t)a.ry * a.rz), cj = (c / a.rz) % a.ry, ck = c % a.rz;
    const float g[3] = {(float)ci / (float)(a.rx - 1), (float)cj / (float)(a.ry - 1), (float)ck / (float)(a.rz - 1)};
    float xw[3];
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) xw[ax] = a.bmin[ax] + g[ax] * (a.bmax[ax] - a.bmin[ax]);
    int count = 0;
    for (int cam = 0; cam < a.C && count == 0; ++cam) {
        const float* P = a.c2w + (int64_t)(a.nc2w == 1 ? 0 : cam) * 12;
        const float* K = a.Ks + (int64_t)(a.nK == 1 ? 0 : cam) * 9;
        // R_w2c = R^T, t_w2c = -R^T t; xc = R^T xw + t_w2c
        float tw[3], xc[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) tw[r] = -(P[0 * 4 + r] * P[3] + P[1 * 4 + r] * P[7] + P[2 * 4 + r] * P[11]);
#pragma unroll
        for (int r = 0; r < 3; ++r) xc[r] = (P[0 * 4 + r] * xw[0] + P[1 * 4 + r] * xw[1] + P[2 * 4 + r] * xw[2]) + tw[r];
        float uvd[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) uvd[r] = K[r * 3 + 0] * xc[0] + K[r * 3 + 1] * xc[1] + K[r * 3 + 2] * xc[2];
        const float u = uvd[0] / uvd[2], v = uvd[1] / uvd[2];
        const bool ok = (uvd[2] >= a.near_plane) && (u >= 0.0f) && (u < (float)a.width) && (v >= 0.0f) &&
                        (v < (float)a.height);
        count += ok ? 1 : 0;
    }
    a.occs_level[c] = count > 0 ? 0.0f : -1.0f;
}

inline unsigned blocks(int64_t n, int per = 256) { return (unsigned)((n + per - 1) / per); }

}  // namespace

// ==========================================================================================
static unsigned ray_waves_grid(int64_t N) {
    const int64_t wgs = (N + 3) / 4;  // 4 waves (rays) per 256-thread block
    return (unsigned)(wgs < 4096 ? (wgs < 1 ? 1 : wgs) : 4096);
}

extern "C" int acn_occ_traverse(const float* rays_o, int64_t ld_o, const float* rays_d, int64_t ld_d, int64_t N,
                                const float* near_planes, const float* far_planes, const uint32_t* bits,
                                const float* aabbs, int levels, const int32_t* res, float step_size, float cone_angle,
                                const float* prefilter_aabb, const float* prefilter_near_far, int64_t ld_pf,
                                int64_t cap, int64_t* counts, const int64_t* offsets, int64_t* ray_indices,
                                float* t_starts, float* t_ends, void* stream) {
    ACN_REQUIRE(N >= 0, "acn_occ_traverse: N must be >= 0");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(levels >= 1 && levels <= kOccMaxLevels, "acn_occ_traverse: levels must be in [1, %d], got %d",
                kOccMaxLevels, levels);
    ACN_REQUIRE(res && res[0] >= 1 && res[1] >= 1 && res[2] >= 1, "acn_occ_traverse: bad resolution");
    ACN_REQUIRE(step_size > 0.0f, "acn_occ_traverse: render_step_size must be > 0 (got %g)", (double)step_size);
    ACN_REQUIRE(cone_angle >= 0.0f, "acn_occ_traverse: cone_angle must be >= 0");
    ACN_REQUIRE(rays_o && rays_d && near_planes && far_planes && bits && aabbs, "acn_occ_traverse: NULL pointer");
    ACN_REQUIRE(ld_o >= 3 && ld_d >= 3, "acn_occ_traverse: rays must be (N, >=3)");
    ACN_REQUIRE(cap >= 0, "acn_occ_traverse: cap must be >= 0");
    if (offsets) ACN_REQUIRE(ray_indices && t_starts && t_ends, "acn_occ_traverse: NULL fill output");
    else ACN_REQUIRE(counts && (cap == 0 || (t_starts && t_ends)), "acn_occ_traverse: NULL count / scratch output");
    TraverseArgs a{};
    a.rays_o = rays_o; a.rays_d = rays_d; a.ld_o = ld_o; a.ld_d = ld_d; a.N = N;
    a.near = near_planes; a.far = far_planes; a.bits = bits;
    for (int l = 0; l < levels; ++l)
        for (int k = 0; k < 6; ++k) a.aabbs[l][k] = aabbs[l * 6 + k];
    a.L = levels; a.rx = res[0]; a.ry = res[1]; a.rz = res[2];
    a.step = step_size; a.cone = cone_angle;
    a.has_prefilter = prefilter_aabb != nullptr;
    if (prefilter_aabb) {
        ACN_REQUIRE(prefilter_near_far && ld_pf >= 2, "acn_occ_traverse: prefilter needs the rays' near/far");
        for (int k = 0; k < 6; ++k) a.prefilter[k] = prefilter_aabb[k];
        a.pf_nf = prefilter_near_far;
        a.ld_pf = ld_pf;
    }
    a.counts = counts; a.offsets = offsets; a.ray_idx = ray_indices; a.t0 = t_starts; a.t1 = t_ends;
    hipLaunchKernelGGL(occ_traverse_kernel, dim3(blocks(N, 64)), dim3(64), 0, (hipStream_t)stream, a,
                       offsets ? (int64_t)0 : cap);
    return acn_check_launch("acn_occ_traverse");
}

extern "C" int acn_occ_compact(const float* scratch_t0, const float* scratch_t1, int64_t cap, const int64_t* counts,
                               const int64_t* offsets, int64_t N, int64_t* ray_indices, float* t_starts, float* t_ends,
                               void* stream) {
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(scratch_t0 && scratch_t1 && counts && offsets && ray_indices && t_starts && t_ends && cap > 0,
                "acn_occ_compact: bad arguments");
    hipLaunchKernelGGL(occ_compact_kernel, dim3(ray_waves_grid(N)), dim3(256), 0, (hipStream_t)stream, scratch_t0,
                       scratch_t1, cap, counts, offsets, N, ray_indices, t_starts, t_ends);
    return acn_check_launch("acn_occ_compact");
}

extern "C" int acn_occ_union(int K, int64_t N, const int64_t* const* starts, const int64_t* const* counts,
                             const float* const* t_starts, const float* const* t_ends, int64_t* out_counts,
                             const int64_t* offsets, int64_t* ray_indices, float* m_starts, float* m_ends,
                             void* stream) {
    ACN_REQUIRE(K >= 1 && K <= kMaxK, "acn_occ_union: K must be in [1, %d]", kMaxK);
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(starts && counts && t_starts && t_ends, "acn_occ_union: NULL pointer");
    if (offsets) ACN_REQUIRE(ray_indices && m_starts && m_ends, "acn_occ_union: NULL fill output");
    else ACN_REQUIRE(out_counts, "acn_occ_union: NULL counts");
    UnionArgs a{};
    a.K = K; a.N = N;
    for (int k = 0; k < K; ++k) {
        ACN_REQUIRE(starts[k] && counts[k], "acn_occ_union: NULL per-expert list %d", k);
        a.starts[k] = starts[k]; a.counts[k] = counts[k]; a.t0[k] = t_starts[k]; a.t1[k] = t_ends[k];
    }
    a.out_counts = out_counts; a.offsets = offsets; a.ray_idx = ray_indices; a.m0 = m_starts; a.m1 = m_ends;
    hipLaunchKernelGGL(occ_union_kernel, dim3(blocks(N)), dim3(256), 0, (hipStream_t)stream, a);
    return acn_check_launch("acn_occ_union");
}

extern "C" int acn_packed_weights_fwd(const float* sigmas, const float* t_starts, const float* t_ends,
                                      const int64_t* chunk_starts, const int64_t* chunk_cnts, int64_t N,
                                      float* weights, float* trans, float* alphas, void* stream) {
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(sigmas && t_starts && t_ends && chunk_starts && chunk_cnts && weights,
                "acn_packed_weights_fwd: NULL pointer");
    PackedWArgs a{sigmas, t_starts, t_ends, chunk_starts, chunk_cnts, N, weights, trans, alphas};
    hipLaunchKernelGGL(packed_weights_kernel, dim3(ray_waves_grid(N)), dim3(256), 0, (hipStream_t)stream, a);
    return acn_check_launch("acn_packed_weights_fwd");
}

extern "C" int acn_packed_weights_bwd(const float* sigmas, const float* t_starts, const float* t_ends,
                                      const float* weights, const float* trans, const float* alphas,
                                      const float* g_weights, const float* g_trans, const float* g_alphas,
                                      const int64_t* chunk_starts, const int64_t* chunk_cnts, int64_t N,
                                      float* g_sigmas, void* stream) {
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(sigmas && t_starts && t_ends && weights && trans && alphas && chunk_starts && chunk_cnts && g_sigmas,
                "acn_packed_weights_bwd: NULL pointer");
    PackedWBwdArgs a{sigmas, t_starts, t_ends, weights, trans, alphas, g_weights, g_trans, g_alphas,
                     chunk_starts, chunk_cnts, N, g_sigmas};
    hipLaunchKernelGGL(packed_weights_bwd_kernel, dim3(ray_waves_grid(N)), dim3(256), 0, (hipStream_t)stream, a);
    return acn_check_launch("acn_packed_weights_bwd");
}

extern "C" int acn_packed_accumulate_fwd(const float* weights, const float* values, int C,
                                         const int64_t* chunk_starts, const int64_t* chunk_cnts, int64_t N,
                                         float* out, void* stream) {
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(C >= 1, "acn_packed_accumulate_fwd: C must be >= 1");
    ACN_REQUIRE(weights && chunk_starts && chunk_cnts && out, "acn_packed_accumulate_fwd: NULL pointer");
    PackedAccArgs a{weights, values, values ? C : 1, chunk_starts, chunk_cnts, N, out};
    hipLaunchKernelGGL(packed_accumulate_kernel, dim3(ray_waves_grid(N)), dim3(256), 0, (hipStream_t)stream, a);
    return acn_check_launch("acn_packed_accumulate_fwd");
}

extern "C" int acn_packed_accumulate_bwd(const float* weights, const float* values, int C, const int64_t* ray_indices,
                                         int64_t M, const float* g_out, float* g_weights, float* g_values,
                                         void* stream) {
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(C >= 1 && weights && ray_indices && g_out, "acn_packed_accumulate_bwd: bad arguments");
    hipLaunchKernelGGL(packed_accumulate_bwd_kernel, dim3(blocks(M)), dim3(256), 0, (hipStream_t)stream, weights,
                       values, values ? C : 1, ray_indices, M, g_out, g_weights, g_values);
    return acn_check_launch("acn_packed_accumulate_bwd");
}

extern "C" int acn_occ_pack_bits(const uint8_t* binaries, int64_t n, uint32_t* bits, void* stream) {
    if (n == 0) return ACN_OK;
    ACN_REQUIRE(binaries && bits, "acn_occ_pack_bits: NULL pointer");
    hipLaunchKernelGGL(occ_pack_bits_kernel, dim3(blocks((n + 31) / 32)), dim3(256), 0, (hipStream_t)stream,
                       binaries, n, bits);
    return acn_check_launch("acn_occ_pack_bits");
}

extern "C" int acn_occ_cell_points(const int64_t* cell_indices, int64_t n, const float* u, const float* aabb,
                                   const int32_t* res, float* x, void* stream) {
    if (n == 0) return ACN_OK;
    ACN_REQUIRE(cell_indices && aabb && res && x, "acn_occ_cell_points: NULL pointer");
    const float4 mn = make_float4(aabb[0], aabb[1], aabb[2], 0.0f), mx = make_float4(aabb[3], aabb[4], aabb[5], 0.0f);
    hipLaunchKernelGGL(occ_cell_points_kernel, dim3(blocks(n)), dim3(256), 0, (hipStream_t)stream, cell_indices, n, u,
                       mn, mx, res[0], res[1], res[2], x);
    return acn_check_launch("acn_occ_cell_points");
}

extern "C" int acn_occ_ema(float* occs, const int64_t* cell_ids, const float* occ, int64_t n, float decay,
                           void* stream) {
    if (n == 0) return ACN_OK;
    ACN_REQUIRE(occs && cell_ids && occ, "acn_occ_ema: NULL pointer");
    hipLaunchKernelGGL(occ_ema_kernel, dim3(blocks(n)), dim3(256), 0, (hipStream_t)stream, occs, cell_ids, occ, n,
                       decay);
    return acn_check_launch("acn_occ_ema");
}

extern "C" size_t acn_occ_binarize_workspace_bytes(void) { return 2 * 1024 * sizeof(double); }

extern "C" int acn_occ_binarize(const float* occs, int64_t n, float occ_thre, uint8_t* binaries, uint32_t* bits,
                                float* thre_out, void* workspace, void* stream) {
    if (n == 0) return ACN_OK;
    ACN_REQUIRE(occs && binaries && workspace, "acn_occ_binarize: NULL pointer");
    hipStream_t s = (hipStream_t)stream;
    const int nparts = 1024;
    hipLaunchKernelGGL(occ_mean_partial_kernel, dim3(nparts), dim3(256), 0, s, occs, n, (double*)workspace);
    int st = acn_check_launch("acn_occ_binarize/mean");
    if (st) return st;
    hipLaunchKernelGGL(occ_binarize_kernel, dim3(blocks((n + 31) / 32)), dim3(256), 0, s, occs, n,
                       (const double*)workspace, nparts, occ_thre, binaries, bits, thre_out);
    return acn_check_launch("acn_occ_binarize");
}

extern "C" int acn_occ_mark_invisible(const float* Ks, int nK, const float* c2w, int nc2w, int width, int height,
                                      float near_plane, const float* aabb, const int32_t* res,
                                      const int64_t* cell_indices, int64_t n, float* occs_level, void* stream) {
    if (n == 0) return ACN_OK;
    ACN_REQUIRE(Ks && c2w && aabb && res && cell_indices && occs_level, "acn_occ_mark_invisible: NULL pointer");
    ACN_REQUIRE(nK >= 1 && nc2w >= 1 && (nK == nc2w || nK == 1 || nc2w == 1),
                "acn_occ_mark_invisible: K and c2w camera counts must match or broadcast");
    ACN_REQUIRE(res[0] > 1 && res[1] > 1 && res[2] > 1, "acn_occ_mark_invisible: resolution must be > 1");
    MarkArgs a{};
    a.Ks = Ks; a.c2w = c2w; a.nK = nK; a.nc2w = nc2w; a.C = nK > nc2w ? nK : nc2w;
    a.width = width; a.height = height; a.near_plane = near_plane;
    for (int k = 0; k < 3; ++k) { a.bmin[k] = aabb[k]; a.bmax[k] = aabb[3 + k]; }
    a.rx = res[0]; a.ry = res[1]; a.rz = res[2];
    a.idx = cell_indices; a.n = n; a.occs_level = occs_level;
    hipLaunchKernelGGL(occ_mark_invisible_kernel, dim3(blocks(n)), dim3(256), 0, (hipStream_t)stream, a);
    return acn_check_launch("acn_occ_mark_invisible");
}
