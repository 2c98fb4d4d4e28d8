// data.hip -- on-device ray routing for episodic task sampling (gfx950).
//
// Replaces the per-ray torch tensor chains of the reference's TaskDataset construction
// (data/task_dataset.py:130-172 _aabb_intersect / _region_segment, :197-227 block ids and cell
// overlaps, :253-352 the 64-step DDA max-overlap policy, :354-418 the alpha-point + 6-neighbour
// max-overlap policy, and the selected-cell overlap recompute + tolerance filter of _route_and_bin
// :544-628) with ONE kernel, one lane per ray, same float op order as the reference's CPU torch ops
// (-ffp-contract=off), so cell assignments are bit-for-bit the reference's.  Binning (stable sort by
// cell) stays on the device in torch; the RNG-driven episode sampling stays on the host generator.
#include "acn_internal.h"

namespace {

__device__ __forceinline__ float nmax2(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fmaxf(a, b); }
__device__ __forceinline__ float nmin2(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fminf(a, b); }

struct RouteArgs {
    const float* rays;    // (N, 8)
    int64_t N;
    float lo[3], hi[3];   // region AABB
    int32_t nx, ny, nz;
    const float* cell_bounds;  // (C, 2, 3) device
    const float* tol_cell;     // (C) per-cell keep tolerance max(1e-6 * |size|, 1e-9)
    float alpha;
    float tol_abs;        // max(1e-6 * median cell diagonal, 1e-9)
    int32_t policy;       // 0 alpha, 1 dda
    int32_t max_steps;
    int64_t* cid;         // out (N): selected cell (valid rays)
    uint8_t* flags;       // out (N): bit0 region-valid, bit1 keep
};

// TaskDataset._aabb_intersect (eps 1e-12) for one ray and box [lo, hi]
__device__ __forceinline__ bool aabb_hit(const float o[3], const float d[3], const float lo[3], const float hi[3],
                                         float& t_entry, float& t_exit) {
    bool miss_parallel = false;
    float te = 0.0f, tx = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const bool parallel = fabsf(d[a]) < 1e-12f;
        const float inv = 1.0f / d[a];
        const float t0 = (lo[a] - o[a]) * inv, t1 = (hi[a] - o[a]) * inv;
        const float mn = nmin2(t0, t1), mx = nmax2(t0, t1);
        te = a == 0 ? mn : nmax2(te, mn);
        tx = a == 0 ? mx : nmin2(tx, mx);
        const bool inside = (o[a] >= lo[a]) && (o[a] <= hi[a]);
        miss_parallel = miss_parallel || (parallel && !inside);
    }
    t_entry = te;
    t_exit = tx;
    return (tx >= te) && !miss_parallel;
}

// _overlap_len_with_cell: clipped to [max(t_entry, 0, near), min(t_exit, far)], 0 on a miss
__device__ __forceinline__ float overlap_len(const float o[3], const float d[3], float near, float far,
                                             const float* cb) {
    float te, tx;
    const bool hit = aabb_hit(o, d, cb, cb + 3, te, tx);
    float t0 = nmax2(te, 0.0f);
    t0 = nmax2(t0, near);
    const float t1 = nmin2(tx, far);
    float len = t1 - t0;
    len = len < 0.0f ? 0.0f : len;  // clamp_min(0) (NaN stays NaN)
    return hit ? len : 0.0f;
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// torch's floor(...).to(int64) followed by a clamp to [0, n): computed in int32.  Values below -1
// and NaN land on 0 as in int64; [2^30, 2^63) saturate to 2^30 (still >= n - 1); x86's conversion of
// >= 2^63 / inf gives INT64_MIN, i.e. 0 after the clamp, reproduced here.
__device__ __forceinline__ int f2i_floor(float v) {
    v = floorf(v);
    if (!(v >= -2.0f && v < 9.22337203685477581e18f)) return -1;
    return (int)fminf(v, 1073741824.0f);
}

__global__ void __launch_bounds__(256) route_kernel(RouteArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.N) return;
    const float* r = a.rays + i * 8;
    const float o[3] = {r[0], r[1], r[2]}, d[3] = {r[3], r[4], r[5]};
    const float near = r[6], far = r[7];
    // _region_segment
    float te, tx;
    const bool hit = aabb_hit(o, d, a.lo, a.hi, te, tx);
    float t0 = nmax2(te, 0.0f);
    t0 = nmax2(t0, near);
    const float t1 = nmin2(tx, far);
    const float seg = t1 - t0;
    if (!(hit && seg > 0.0f)) {
        a.cid[i] = -1;
        a.flags[i] = 0;
        return;
    }
    const int nx = a.nx, ny = a.ny, nz = a.nz;
    const int nyz = ny * nz;
    int cid_final;
    if (a.policy == 0) {
        // alpha point (nudged inside the segment) -> primary block
        float ta = t0 + a.alpha * (t1 - t0);
        ta = ta + 1e-6f * (t1 - t0);
        float rel[3];
        const int n3[3] = {nx, ny, nz};
        int ix[3];
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
            const float p = o[ax] + d[ax] * ta;
            float ext = a.hi[ax] - a.lo[ax];
            ext = ext < 1e-9f ? 1e-9f : ext;
            float v = (p - a.lo[ax]) / ext;
            v = v < 0.0f ? 0.0f : v;
            v = v > 0.99999988f ? 0.99999988f : v;  // clamp(0, 1 - 1e-7) in fp32
            rel[ax] = v;
            ix[ax] = clampi(f2i_floor(rel[ax] * (float)n3[ax]), 0, n3[ax] - 1);
        }
        const int cid_primary = ix[0] * nyz + ix[1] * nz + ix[2];
        // 6 neighbours then the primary; argmax keeps the first maximum (torch.argmax)
        const int dx[7] = {-1, 1, 0, 0, 0, 0, 0}, dy[7] = {0, 0, -1, 1, 0, 0, 0}, dz[7] = {0, 0, 0, 0, -1, 1, 0};
        float best = -1.0f;
        int cid_best = cid_primary;
        for (int k = 0; k < 7; ++k) {
            const int cx = clampi(ix[0] + dx[k], 0, nx - 1), cy = clampi(ix[1] + dy[k], 0, ny - 1),
                      cz = clampi(ix[2] + dz[k], 0, nz - 1);
            const int c = cx * nyz + cy * nz + cz;
            const float len = overlap_len(o, d, near, far, a.cell_bounds + c * 6);
            if (k == 0 || len > best) { best = len; cid_best = c; }
        }
        const float tol = fmaxf(a.tol_abs, 1e-6f * seg);
        cid_final = (best >= tol) ? cid_best : cid_primary;
    } else {
        // _dda_maxoverlap: grid units g = (p - lo) / max(cell, 1e-12)
        float go[3], gd[3];
        const int n3[3] = {nx, ny, nz};
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
            float cell = (a.hi[ax] - a.lo[ax]) / (float)n3[ax];
            cell = cell < 1e-12f ? 1e-12f : cell;
            go[ax] = (o[ax] - a.lo[ax]) / cell;
            gd[ax] = d[ax] / cell;
        }
        int idx[3], st[3];
        float tmax[3], tdel[3];
        const float big = 1e30f;
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
            const float p = go[ax] + gd[ax] * (t0 + 1e-6f);
            idx[ax] = f2i_floor(p);
            const float sg = gd[ax] > 0.0f ? 1.0f : (gd[ax] < 0.0f ? -1.0f : 0.0f);
            st[ax] = (int)sg;
            const float nb = st[ax] > 0 ? floorf(p) + 1.0f : ceilf(p) - 1.0f;
            const float inv = 1.0f / gd[ax];
            float tm = (nb - p) * inv, td = (float)st[ax] * inv;
            if (!(tm == tm) || isinf(tm)) tm = big;  // nan_to_num(nan=big, posinf=big, neginf=big)
            if (!(td == td) || isinf(td)) td = big;
            tmax[ax] = tm;
            tdel[ax] = td;
            idx[ax] = clampi(idx[ax], 0, n3[ax] - 1);
        }
        float t = t0, best_len = 0.0f;
        int best_cid = idx[0] * nyz + idx[1] * nz + idx[2];
        for (int s = 0; s < a.max_steps; ++s) {
            const float m = fminf(fminf(tmax[0], tmax[1]), tmax[2]);
            const float t_next = fminf(m, t1);
            float dt = t_next - t;
            dt = dt < 0.0f ? 0.0f : dt;
            const int c = idx[0] * nyz + idx[1] * nz + idx[2];
            if (dt > best_len) { best_len = dt; best_cid = c; }
            if (t_next >= t1) break;
            const bool ax_ = (tmax[0] <= tmax[1]) && (tmax[0] <= tmax[2]);
            const bool ay_ = !(tmax[0] <= tmax[1]) && (tmax[1] <= tmax[2]);
            const int ax = ax_ ? 0 : (ay_ ? 1 : 2);
            idx[ax] = clampi(idx[ax] + st[ax], 0, n3[ax] - 1);
            tmax[ax] = tmax[ax] + tdel[ax];
            t = t_next;
        }
        cid_final = best_cid;
    }
    // _route_and_bin: recompute the overlap with the selected cell; keep >= that cell's tolerance
    const float len = overlap_len(o, d, near, far, a.cell_bounds + (int64_t)cid_final * 6);
    a.cid[i] = (int64_t)cid_final;
    a.flags[i] = (uint8_t)(1u | ((len >= a.tol_cell[cid_final]) ? 2u : 0u));
}

}  // namespace

extern "C" int acn_route_rays(const float* rays, int64_t N, const float* region_aabb, const int32_t* cells,
                              const float* cell_bounds, const float* tol_cell, float alpha, float tol_abs, int policy,
                              int max_steps, int64_t* cell_ids, uint8_t* flags, void* stream) {
    ACN_REQUIRE(N >= 0, "acn_route_rays: N must be >= 0");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(rays && region_aabb && cells && cell_bounds && tol_cell && cell_ids && flags,
                "acn_route_rays: NULL pointer");
    ACN_REQUIRE(cells[0] >= 1 && cells[1] >= 1 && cells[2] >= 1, "acn_route_rays: cells must be >= 1");
    ACN_REQUIRE(policy == 0 || policy == 1, "acn_route_rays: policy must be 0 (alpha) or 1 (dda)");
    RouteArgs a{};
    a.rays = rays; a.N = N;
    for (int k = 0; k < 3; ++k) { a.lo[k] = region_aabb[k]; a.hi[k] = region_aabb[3 + k]; }
    a.nx = cells[0]; a.ny = cells[1]; a.nz = cells[2];
    a.cell_bounds = cell_bounds; a.tol_cell = tol_cell;
    a.alpha = alpha; a.tol_abs = tol_abs; a.policy = policy; a.max_steps = max_steps;
    a.cid = cell_ids; a.flags = flags;
    hipLaunchKernelGGL(route_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    return acn_check_launch("acn_route_rays");
}

// ---------------------------------------------------------------------------------------------
// Stable binning of the kept rays by cell (_route_and_bin's "sort by cell, keep relative order"):
// a counting sort whose output order equals torch.sort(cid, stable=True) over the region-valid rays
// followed by the keep filter.  The rays are cut into segments of kSegTiles 64-ray tiles, one wave
// per segment (4 per block); a wave prefetches its whole segment, then groups the lanes of each
// tile by cell with ballots (consecutive pixels of an image mostly share a cell: 1-3 groups per
// tile) -- no atomics, ranks inside a group follow lane order, so the scatter is stable.
//   count:   hist[c * nseg + s] = kept rays of cell c in segment s          (cell-major)
//   scan:    per cell (one block each) exclusive scan over the segments, totals[c]
//   starts:  exclusive scan of totals -> starts[c]; counts[c] = totals[c], counts[C] = valid rays
//   scatter: out[starts[c] + hist[c * nseg + s] + running rank] = ray index  (int32)
namespace {

constexpr int kSegTiles = 16;
constexpr int kSeg = 64 * kSegTiles;   // rays per segment
constexpr int kBinWaves = 4;           // waves (segments) per block

__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << __lane_id()) - 1ull; }

__device__ __forceinline__ void seg_load(const int64_t* __restrict__ cid, const uint8_t* __restrict__ flags, int64_t N,
                                         int64_t seg0, int key[kSegTiles], unsigned& n_valid) {
    uint8_t f[kSegTiles];
#pragma unroll
    for (int t = 0; t < kSegTiles; ++t) {
        const int64_t i = seg0 + t * 64 + __lane_id();
        f[t] = i < N ? flags[i] : 0;
    }
#pragma unroll
    for (int t = 0; t < kSegTiles; ++t) {
        const int64_t i = seg0 + t * 64 + __lane_id();
        key[t] = (f[t] & 2) ? (int)cid[i] : -1;
        n_valid += __popcll(__ballot(f[t] & 1));
    }
}

__global__ void __launch_bounds__(64 * kBinWaves) bin_count_kernel(const int64_t* __restrict__ cid,
                                                                   const uint8_t* __restrict__ flags, int64_t N,
                                                                   int nseg, int C, int32_t* __restrict__ hist,
                                                                   int32_t* __restrict__ seg_valid) {
    extern __shared__ int32_t lds[];
    const int w = threadIdx.x >> 6;
    int32_t* h = lds + w * C;
    const int seg = blockIdx.x * kBinWaves + w;
    for (int c = __lane_id(); c < C; c += 64) h[c] = 0;
    __syncthreads();
    if (seg >= nseg) return;  // wave-uniform; no barrier follows
    int key[kSegTiles];
    unsigned nv = 0;
    seg_load(cid, flags, N, (int64_t)seg * kSeg, key, nv);
#pragma unroll
    for (int t = 0; t < kSegTiles; ++t) {
        uint64_t pending = __ballot(key[t] >= 0);
        while (pending) {
            const int src = __ffsll((unsigned long long)pending) - 1;
            const int k = __shfl(key[t], src);
            const uint64_t m = __ballot(key[t] == k);
            if (__lane_id() == src) h[k] += __popcll(m);
            pending &= ~m;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (int c = __lane_id(); c < C; c += 64) hist[(int64_t)c * nseg + seg] = h[c];
    if (__lane_id() == 0) seg_valid[seg] = (int32_t)nv;
}

// block c: exclusive scan of hist[c * nseg .. + nseg) in place, totals[c]
__global__ void __launch_bounds__(256) bin_scan_kernel(int32_t* __restrict__ hist, int nseg,
                                                       int64_t* __restrict__ totals) {
    __shared__ int32_t wsum[4];
    __shared__ int64_t carry_s;
    int32_t* row = hist + (int64_t)blockIdx.x * nseg;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) carry_s = 0;
    __syncthreads();
    for (int base = 0; base < nseg; base += 256) {
        const int j = base + t;
        const int32_t v = j < nseg ? row[j] : 0;
        int32_t x = v;  // wave inclusive scan
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t y = __shfl_up(x, off);
            if (lane >= off) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        int32_t before = 0;
        for (int k = 0; k < w; ++k) before += wsum[k];
        const int64_t carry = carry_s;
        if (j < nseg) row[j] = (int32_t)(carry + before + x - v);
        __syncthreads();
        if (t == 255) carry_s = carry + before + x;
        __syncthreads();
    }
    if (t == 0) totals[blockIdx.x] = carry_s;
}

// single block: starts = exclusive scan of totals; counts[c] = totals[c], counts[C] = valid rays
__global__ void __launch_bounds__(1024) bin_starts_kernel(const int64_t* __restrict__ totals, int C,
                                                          int64_t* __restrict__ starts, int64_t* __restrict__ counts,
                                                          const int32_t* __restrict__ seg_valid, int nseg) {
    __shared__ int64_t part[1024];
    __shared__ int64_t vsum[16];
    const int t = threadIdx.x;
    int64_t v = 0;
    for (int j = t; j < nseg; j += 1024) v += seg_valid[j];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    if ((t & 63) == 0) vsum[t >> 6] = v;
    const int per = (C + 1023) / 1024, lo = t * per, hi = lo + per < C ? lo + per : C;
    int64_t s = 0;
    for (int c = lo; c < hi; ++c) s += totals[c];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int64_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int64_t run = part[t] - s;
    for (int c = lo; c < hi; ++c) {
        starts[c] = run;
        counts[c] = totals[c];
        run += totals[c];
    }
    if (t == 0) {
        int64_t nv = 0;
        for (int k = 0; k < 16; ++k) nv += vsum[k];
        counts[C] = nv;
    }
}

__global__ void __launch_bounds__(64 * kBinWaves) bin_scatter_kernel(const int64_t* __restrict__ cid,
                                                                     const uint8_t* __restrict__ flags, int64_t N,
                                                                     int nseg, int C,
                                                                     const int32_t* __restrict__ hist,
                                                                     const int64_t* __restrict__ starts,
                                                                     int32_t* __restrict__ out) {
    extern __shared__ int32_t lds[];
    const int w = threadIdx.x >> 6;
    int32_t* h = lds + w * C;
    const int seg = blockIdx.x * kBinWaves + w;
    if (seg >= nseg) return;  // no block barrier in this kernel
    for (int c = __lane_id(); c < C; c += 64) h[c] = (int32_t)(starts[c] + hist[(int64_t)c * nseg + seg]);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    int key[kSegTiles];
    unsigned nv = 0;
    const int64_t seg0 = (int64_t)seg * kSeg;
    seg_load(cid, flags, N, seg0, key, nv);
#pragma unroll
    for (int t = 0; t < kSegTiles; ++t) {
        uint64_t pending = __ballot(key[t] >= 0);
        while (pending) {
            const int src = __ffsll((unsigned long long)pending) - 1;
            const int k = __shfl(key[t], src);
            const uint64_t m = __ballot(key[t] == k);
            const int32_t start = h[k];
            if (key[t] == k) out[start + __popcll(m & lanemask_lt())] = (int32_t)(seg0 + t * 64 + __lane_id());
            __builtin_amdgcn_wave_barrier();
            if (__lane_id() == src) h[k] = start + __popcll(m);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            pending &= ~m;
        }
    }
}

int bin_segments(int64_t N) { return (int)((N + kSeg - 1) / kSeg); }

}  // namespace

extern "C" size_t acn_bin_rays_workspace_bytes(int64_t N, int n_cells) {
    const int nseg = bin_segments(N) > 0 ? bin_segments(N) : 1;
    return (size_t)nseg * sizeof(int32_t) + (size_t)n_cells * nseg * sizeof(int32_t) +
           2 * (size_t)n_cells * sizeof(int64_t) + 64;
}

extern "C" int acn_bin_rays(const int64_t* cell_ids, const uint8_t* flags, int64_t N, int n_cells, int32_t* ray_index,
                            int64_t* counts, void* workspace, size_t workspace_bytes, void* stream) {
    ACN_REQUIRE(N >= 0 && N < (int64_t(1) << 31), "acn_bin_rays: N must be in [0, 2^31)");
    ACN_REQUIRE(n_cells >= 1 && n_cells <= 4096, "acn_bin_rays: n_cells must be in [1, 4096]");
    ACN_REQUIRE(workspace_bytes >= acn_bin_rays_workspace_bytes(N, n_cells), "acn_bin_rays: workspace too small");
    ACN_REQUIRE(counts && workspace && (N == 0 || (cell_ids && flags && ray_index)), "acn_bin_rays: NULL pointer");
    hipStream_t s = (hipStream_t)stream;
    const int nseg = bin_segments(N) > 0 ? bin_segments(N) : 1;
    int64_t* totals = (int64_t*)workspace;  // (C) then starts (C), hist (C * nseg), seg_valid (nseg)
    int64_t* starts = totals + n_cells;
    int32_t* hist = (int32_t*)(starts + n_cells);
    int32_t* seg_valid = hist + (size_t)n_cells * nseg;
    const size_t lds = (size_t)kBinWaves * n_cells * sizeof(int32_t);
    const unsigned blocks = (unsigned)((nseg + kBinWaves - 1) / kBinWaves);
    hipLaunchKernelGGL(bin_count_kernel, dim3(blocks), dim3(64 * kBinWaves), lds, s, cell_ids, flags, N, nseg,
                       n_cells, hist, seg_valid);
    hipLaunchKernelGGL(bin_scan_kernel, dim3(n_cells), dim3(256), 0, s, hist, nseg, totals);
    hipLaunchKernelGGL(bin_starts_kernel, dim3(1), dim3(1024), 0, s, totals, n_cells, starts, counts, seg_valid,
                       N > 0 ? nseg : 0);
    if (N > 0)
        hipLaunchKernelGGL(bin_scatter_kernel, dim3(blocks), dim3(64 * kBinWaves), lds, s, cell_ids, flags, N, nseg,
                           n_cells, hist, starts, ray_index);
    return acn_check_launch("acn_bin_rays");
}
