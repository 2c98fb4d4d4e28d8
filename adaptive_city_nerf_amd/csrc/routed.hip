// routed.hip -- (sample, expert) pair lists of the routed container (gfx950).
//
// Replaces the front end of the differentiable container render and its expert dispatch
// (nerfs/ray_rendering.py:262-345 stratified_t_vals / points / id6, models/inr/meta_container.py:
// 97-134 _routing, :300-343 the per-expert nonzero -> index_select -> expert -> index_add_ loop,
// meta_ngp.py:155-168 _world_to_unit / _enc_dir):
//
//   acn_routed_count   : one lane per sample -> t (N,S), routing weights W (M,K) in the reference's
//                        cdist-mm arithmetic, per-256-sample block counts of routed samples per expert,
//                        then one workgroup scans them -> pair segment of every expert (starts[K+1]).
//   acn_routed_scatter : one lane per sample -> for every expert k with w_k > 0, pair record at
//                        starts[k] + (rank of the sample among expert k's samples, in sample order;
//                        the *_tiled expert-parallel forms: in depth-tile order, tile_sample):
//                        sample index, weight, x in expert k's unit box (clamped), SH-4 of the ray
//                        direction; pmap (M,K) = pair index or -1.  Pairs of expert k are therefore
//                        exactly the rows the reference's index_select(nonzero(w[:,k] > 0)) gathers,
//                        in the same order.
//   acn_routed_blend_fwd / _bwd : y_m = sum_k y_pk * w_pk accumulated in expert order from zero
//                        (index_add_); backward dY_p = dY_m * w_p (mul + index_add_ backward).
//
// Pairs are the currency of the expert-parallel layouts too: the pairs of expert k are what an
// all-to-all sends to the GPU that owns expert k (parallel.py).
#include "acn_device.h"
#include "acn_internal.h"

using namespace acn;

namespace {

constexpr int kBlk = 256;  // samples per count / scatter block (4 waves)

struct RouteCfg {
    int32_t K, cluster_2d, routing;  // routing: 1 soft (bm > 1), 2 hard (argmin)
    float bm;
    float cent[kMaxK][3];
};

// Fixed pair layout of the expert-parallel exchange: expert k's segment is [off[k], off[k] + cap[k]) (uniform
// capacity: off[k] = k cap); fixed = 0: the compact layout of acn_routed_count (segments padded to `align`)
struct Caps {
    int32_t fixed;
    int64_t cap[kMaxK];
    int64_t off[kMaxK + 1];
};

// weight of expert k for a sample at p (the reference's rule; hard routing as weight 1 of the argmin:
// 0 + y * 1 == y, identical to index_copy_)
__device__ __forceinline__ void route_row(const RouteCfg& cfg, float px, float py, float pz, float (&w)[kMaxK]) {
    if (cfg.routing == 1) {
        const RouteState st = route_prep<1>(cfg, px, py, pz);
#pragma unroll
        for (int k = 0; k < kMaxK; ++k) w[k] = k < cfg.K ? route_weight(cfg, st, k, px, py, pz) : 0.0f;
    } else {
        const RouteState st = route_prep<2>(cfg, px, py, pz);
#pragma unroll
        for (int k = 0; k < kMaxK; ++k) w[k] = (k < cfg.K && st.hard == k) ? 1.0f : 0.0f;
    }
}

// Sample at traversal position mp.  tile = 0: sample order (mp itself, ray-major).  tile > 0: depth tiles -- the
// rays come in blocks of `tile` consecutive rays (the last one shorter), and a block's rays at sample s precede its
// rays at s + 1.  The pair lists are built in traversal order, so with tiles a wave of an expert's records holds
// neighbouring rays at one depth: neighbouring points, the hash rows they share stay in L2.  A
// bijection of [0, M): every sample is visited once, whatever the order.
__device__ __forceinline__ int64_t tile_sample(int64_t mp, int64_t N, int S, int tile) {
    if (tile <= 0) return mp;
    const int64_t ts = (int64_t)tile * S;
    const int64_t bi = mp / ts;
    const int64_t q = mp - bi * ts;
    const int64_t r0 = bi * tile;
    const int64_t nb = N - r0 < tile ? N - r0 : tile;
    const int64_t s = q / nb;
    return (r0 + (q - s * nb)) * S + s;
}

__global__ void __launch_bounds__(kBlk) routed_count_kernel(const float* __restrict__ rays, int64_t N, int S,
                                                            const float* __restrict__ jit, RouteCfg cfg,
                                                            float* __restrict__ t_out, float* __restrict__ W,
                                                            int32_t* __restrict__ blk_cnt, int tile) {
    __shared__ int wcnt[kBlk / 64][kMaxK];
    const int64_t M = N * (int64_t)S;
    const int64_t mp = (int64_t)blockIdx.x * kBlk + threadIdx.x;
    const int64_t m = mp < M ? tile_sample(mp, N, S, tile) : mp;
    float w[kMaxK];
#pragma unroll
    for (int k = 0; k < kMaxK; ++k) w[k] = 0.0f;
    if (m < M) {
        const int64_t ray = m / S;
        const int s = (int)(m - ray * S);
        const float* rp = rays + ray * 8;
        const float t = tval(rp[6], rp[7], s, S, jit ? jit + ray * S : nullptr);
        t_out[m] = t;
        const float px = rp[0] + rp[3] * t, py = rp[1] + rp[4] * t, pz = rp[2] + rp[5] * t;
        route_row(cfg, px, py, pz, w);
#pragma unroll
        for (int k = 0; k < kMaxK; ++k)
            if (k < cfg.K) W[m * cfg.K + k] = w[k];
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kMaxK; ++k) {
        if (k < cfg.K) {  // wave-uniform
            const uint64_t b = __ballot(w[k] > 0.0f);
            if (lane == 0) wcnt[wave][k] = __popcll(b);
        }
    }
    __syncthreads();
    if (threadIdx.x < cfg.K) {
        int c = 0;
#pragma unroll
        for (int q = 0; q < kBlk / 64; ++q) c += wcnt[q][threadIdx.x];
        blk_cnt[(int64_t)blockIdx.x * cfg.K + threadIdx.x] = c;
    }
}

// one workgroup: per expert, exclusive scan of the block counts (in place) and the segment starts
// cap > 0: fixed layout -- expert k's segment is [k cap, (k + 1) cap) whatever the counts (cap >= M, so no
// segment can overflow): the expert-parallel send buffer, grouped by owner, with host-known split sizes
__global__ void __launch_bounds__(1024) routed_scan_kernel(int32_t* __restrict__ blk_cnt, int64_t nblk, int K,
                                                           int align, Caps caps, int64_t* __restrict__ starts) {
    // wave k scans expert k's block counts: each lane sums a contiguous run of blocks, one inclusive wave
    // scan of the 64 run totals, then each lane writes its run's exclusive prefixes.  Integer sums, so the
    // result equals the serial prefix sums exactly (the previous form had every wave scan all K experts)
    static_assert(kMaxK <= 16, "one wave per expert in a 1024-thread block");
    __shared__ int64_t etot[kMaxK];   // expert k's pair count
    const int tid = threadIdx.x, lane = tid & 63, k = tid >> 6;
    if (k < K) {
        const int64_t per = (nblk + 63) / 64;
        const int64_t b0 = lane * per, b1 = b0 + per < nblk ? b0 + per : nblk;
        int64_t sum = 0;
        for (int64_t b = b0; b < b1; ++b) sum += blk_cnt[b * K + k];
        int64_t v = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t u = __shfl_up(v, off);
            if (lane >= off) v += u;
        }
        int64_t run = v - sum;
        for (int64_t b = b0; b < b1; ++b) {
            const int32_t c = blk_cnt[b * K + k];
            blk_cnt[b * K + k] = (int32_t)run;
            run += c;
        }
        if (lane == 63) etot[k] = v;
    }
    __syncthreads();
    if (tid == 0) {
        int64_t base = 0;
        for (int k = 0; k < K; ++k) {
            const int64_t total = etot[k];
            starts[k] = caps.fixed ? caps.off[k] : base;
            starts[K + 1 + k] = total;                        // real pair count of expert k
            base += (total + align - 1) / align * align;      // segment padded to a multiple of align
        }
        starts[K] = caps.fixed ? caps.off[K] : base;
    }
}

struct BoxCfg {
    float amin[kMaxK][3], ext[kMaxK][3];
    float lo, hi;
};

// XD = 0: x01 (3, expert k's unit box) + sh (16) per pair; XD = 1: xd (6) = [world point, ray direction] per
// pair (the record the expert-parallel layouts send to the expert's owner)
template <int XD>
__global__ void __launch_bounds__(kBlk) routed_scatter_kernel(const float* __restrict__ rays, int64_t N, int S,
                                                              int K, const float* __restrict__ t_vals,
                                                              const float* __restrict__ W,
                                                              const int32_t* __restrict__ blk_off,
                                                              const int64_t* __restrict__ starts, BoxCfg box,
                                                              int32_t* __restrict__ pidx, float* __restrict__ pw,
                                                              float* __restrict__ x01, float* __restrict__ sh_out,
                                                              int32_t* __restrict__ pmap, int32_t* __restrict__ pk,
                                                              int pad, int tile) {
    __shared__ int wcnt[kBlk / 64][kMaxK];
    const int64_t M = N * (int64_t)S;
    if (XD == 0 && pad) {
        // the padding slots of expert k (segment tail past its live count, ALIGN padding): pidx -1, weight 0,
        // a neutral point; disjoint from every pair slot this kernel writes (was routed_pad_kernel, a launch
        // of its own)
        for (int k = blockIdx.x; k < K; k += gridDim.x) {
            const int64_t p0 = starts[k] + starts[K + 1 + k], p1 = starts[k + 1];
            for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
                pidx[p] = -1;
                pw[p] = 0.0f;
                x01[3 * p] = x01[3 * p + 1] = x01[3 * p + 2] = 0.5f;
#pragma unroll
                for (int q = 0; q < 16; ++q) sh_out[16 * p + q] = 0.0f;
                if (pk) pk[p] = k;
            }
        }
    }
    const int64_t mp = (int64_t)blockIdx.x * kBlk + threadIdx.x;   // traversal position (tile_sample)
    const bool live = mp < M;
    const int64_t m = live ? tile_sample(mp, N, S, tile) : mp;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float px = 0.0f, py = 0.0f, pz = 0.0f, sh[16];
    if (live) {
        const int64_t ray = m / S;
        const float* rp = rays + ray * 8;
        const float t = t_vals[m];
        px = rp[0] + rp[3] * t;
        py = rp[1] + rp[4] * t;
        pz = rp[2] + rp[5] * t;
        if (XD) {
            sh[0] = rp[3]; sh[1] = rp[4]; sh[2] = rp[5];
        } else {
            dir_sh(rp[3], rp[4], rp[5], sh);
        }
    }
    const uint64_t below = (1ull << lane) - 1ull;
    for (int k = 0; k < K; ++k) {
        const float wk = live ? W[m * K + k] : 0.0f;
        const uint64_t b = __ballot(wk > 0.0f);
        if (lane == 0) wcnt[wave][k] = __popcll(b);
    }
    __syncthreads();
    for (int k = 0; k < K; ++k) {
        const float wk = live ? W[m * K + k] : 0.0f;
        const uint64_t b = __ballot(wk > 0.0f);  // recomputed (a runtime-indexed array would go to scratch)
        if (!live) continue;
        if (!(wk > 0.0f)) {
            pmap[m * K + k] = -1;
            continue;
        }
        int64_t pos = starts[k] + blk_off[(int64_t)blockIdx.x * K + k] + __popcll(b & below);
        for (int q = 0; q < wave; ++q) pos += wcnt[q][k];
        if (pos >= starts[k + 1]) {   // fixed layout below the expert's count (capacity-bounded exchange):
            pmap[m * K + k] = -1;      // the pair is dropped; the caller sees the count exceed the capacity
            continue;
        }
        pmap[m * K + k] = (int32_t)pos;
        pidx[pos] = (int32_t)m;
        if (pk) pk[pos] = k;
        pw[pos] = wk;
        if (XD) {
            float* o = x01 + pos * 6;
            o[0] = px; o[1] = py; o[2] = pz;
            o[3] = sh[0]; o[4] = sh[1]; o[5] = sh[2];
            continue;
        }
        x01[pos * 3 + 0] = clamp_nan((px - box.amin[k][0]) / box.ext[k][0], box.lo, box.hi);
        x01[pos * 3 + 1] = clamp_nan((py - box.amin[k][1]) / box.ext[k][1], box.lo, box.hi);
        x01[pos * 3 + 2] = clamp_nan((pz - box.amin[k][2]) / box.ext[k][2], box.lo, box.hi);
        float4* o4 = reinterpret_cast<float4*>(sh_out + pos * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) o4[q] = make_float4(sh[4 * q], sh[4 * q + 1], sh[4 * q + 2], sh[4 * q + 3]);
    }
}

__global__ void __launch_bounds__(256) blend_fwd_kernel(const float4* __restrict__ y, const float* __restrict__ pw,
                                                        const int32_t* __restrict__ pmap, int64_t M, int K,
                                                        float4* __restrict__ out) {
    const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (m >= M) return;
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int k = 0; k < K; ++k) {
        const int32_t p = pmap[m * K + k];
        if (p < 0) continue;
        const float4 v = y[p];
        const float w = pw[p];
        acc.x = acc.x + v.x * w;
        acc.y = acc.y + v.y * w;
        acc.z = acc.z + v.z * w;
        acc.w = acc.w + v.w * w;
    }
    out[m] = acc;
}

__global__ void __launch_bounds__(256) blend_bwd_kernel(const float4* __restrict__ g, const int32_t* __restrict__ pidx,
                                                        const float* __restrict__ pw, int64_t P,
                                                        const int64_t* __restrict__ live, float4* __restrict__ gy) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= P || (live && p >= live[0])) return;  // slots past the live count hold no pair
    const int32_t m = pidx[p];
    if (m < 0) {  // padding slot
        gy[p] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        return;
    }
    const float4 v = g[m];
    const float w = pw[p];
    gy[p] = make_float4(v.x * w, v.y * w, v.z * w, v.w * w);
}

// owner side of the expert-parallel layouts: world point + direction records of ONE expert -> x01 in its
// unit box and SH-4 of the direction (the same ops as routed_scatter_kernel<0>)
__global__ void __launch_bounds__(256) xd_unit_sh_kernel(const float* __restrict__ xd, int64_t P, float3 amin, float3 ext,
                                                         float lo, float hi, float* __restrict__ x01,
                                                         float* __restrict__ sh_out) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    const float* r = xd + p * 6;
    x01[p * 3 + 0] = clamp_nan((r[0] - amin.x) / ext.x, lo, hi);
    x01[p * 3 + 1] = clamp_nan((r[1] - amin.y) / ext.y, lo, hi);
    x01[p * 3 + 2] = clamp_nan((r[2] - amin.z) / ext.z, lo, hi);
    float sh[16];
    dir_sh(r[3], r[4], r[5], sh);
    float4* o4 = reinterpret_cast<float4*>(sh_out + p * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) o4[q] = make_float4(sh[4 * q], sh[4 * q + 1], sh[4 * q + 2], sh[4 * q + 3]);
}

unsigned blocks_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

// ---- expert-parallel exchange (expert_parallel.ExpertParallelAdaptStep).  Sender: pairs in the fixed
// layout of acn_routed_count_fixed; slots past a segment's live count get pidx -1, pw 0.
__global__ void __launch_bounds__(256) pad_pairs_kernel(const int64_t* __restrict__ seg, int K, int32_t* __restrict__ pidx,
                                                        float* __restrict__ pw) {
    const int k = blockIdx.y;
    const int64_t p0 = seg[k] + seg[K + 1 + k], p1 = seg[k + 1];
    for (int64_t p = p0 + (int64_t)blockIdx.x * 256 + threadIdx.x; p < p1; p += (int64_t)gridDim.x * 256) {
        pidx[p] = -1;
        pw[p] = 0.0f;
    }
}

// Owner: the received layout is [src s][local expert j][cap] records with live counts cnt[s][j]; the compact
// pair list holds local expert j's records in (s, i) order in a segment padded to `align`.  One thread:
// off[s][j] = sum_{s' < s} cnt[s'][j], seg[j] (padded starts), seg[E] = slots, seg[E + 1 + j] = live count.
// the received layout of a capacity-bounded exchange: sender s's segment of local expert j starts at
// s * row + off[j] and holds at most cap[j] records (uniform: off[j] = j cap, row = E cap)
struct OwnCaps {
    int64_t row;
    int64_t cap[kMaxK];
    int64_t off[kMaxK];
};

__global__ void ep_seg_kernel(const int64_t* __restrict__ cnt, int W, int E, int align, OwnCaps oc,
                              int64_t* __restrict__ off, int64_t* __restrict__ seg) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t base = 0;
    for (int j = 0; j < E; ++j) {
        int64_t run = 0;
        for (int s = 0; s < W; ++s) {
            off[(int64_t)s * E + j] = run;
            const int64_t c = cnt[(int64_t)s * E + j];
            run += c < oc.cap[j] ? c : oc.cap[j];   // a count past the capacity: only cap records were sent
        }
        seg[j] = base;
        seg[E + 1 + j] = run;
        base += (run + align - 1) / align * align;
    }
    seg[E] = base;
}

// per compact slot p < seg[E]: (s, i) of its record, x01 in the expert's unit box + SH-4 (as
// routed_scatter_kernel<0>), pk = j, pflag = 0 (pair) / -1 (padding), back = received-layout index or -1
__global__ void __launch_bounds__(256) ep_gather_kernel(const float* __restrict__ xd, const int64_t* __restrict__ cnt,
                                                        const int64_t* __restrict__ off, const int64_t* __restrict__ seg,
                                                        int W, int E, OwnCaps oc, BoxCfg box, float* __restrict__ x01,
                                                        float* __restrict__ sh_out, int32_t* __restrict__ pk,
                                                        int32_t* __restrict__ pflag, int64_t* __restrict__ back) {
    const int64_t total = seg[E];
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < total; p += (int64_t)gridDim.x * 256) {
        int j = 0;
        while (j + 1 < E && seg[j + 1] <= p) ++j;
        const int64_t q = p - seg[j];
        pk[p] = j;
        if (q >= seg[E + 1 + j]) {  // padding of segment j
            pflag[p] = -1;
            back[p] = -1;
            x01[3 * p] = x01[3 * p + 1] = x01[3 * p + 2] = 0.5f;
            float4* o4 = reinterpret_cast<float4*>(sh_out + p * 16);
#pragma unroll
            for (int c = 0; c < 4; ++c) o4[c] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            continue;
        }
        int s = 0;
        while (s + 1 < W && off[(int64_t)(s + 1) * E + j] <= q) ++s;
        const int64_t i = q - off[(int64_t)s * E + j];
        const int64_t src = (int64_t)s * oc.row + oc.off[j] + i;
        const float* r = xd + src * 6;
        pflag[p] = 0;
        back[p] = src;
        x01[3 * p + 0] = clamp_nan((r[0] - box.amin[j][0]) / box.ext[j][0], box.lo, box.hi);
        x01[3 * p + 1] = clamp_nan((r[1] - box.amin[j][1]) / box.ext[j][1], box.lo, box.hi);
        x01[3 * p + 2] = clamp_nan((r[2] - box.amin[j][2]) / box.ext[j][2], box.lo, box.hi);
        float sh[16];
        dir_sh(r[3], r[4], r[5], sh);
        float4* o4 = reinterpret_cast<float4*>(sh_out + p * 16);
#pragma unroll
        for (int c = 0; c < 4; ++c) o4[c] = make_float4(sh[4 * c], sh[4 * c + 1], sh[4 * c + 2], sh[4 * c + 3]);
    }
}

// owner: field outputs of the compact slots back to the received layout (-> the senders' pair slots)
__global__ void __launch_bounds__(256) ep_scatter_back_kernel(const float4* __restrict__ out, const int64_t* __restrict__ back,
                                                              const int64_t* __restrict__ seg, int E,
                                                              float4* __restrict__ ret) {
    const int64_t total = seg[E];
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < total; p += (int64_t)gridDim.x * 256) {
        const int64_t b = back[p];
        if (b >= 0) ret[b] = out[p];
    }
}

// owner: the senders' dL/d(rgb, sigma) of the received layout -> the compact slots (0 on padding)
__global__ void __launch_bounds__(256) ep_gather_grad_kernel(const float4* __restrict__ gy, const int64_t* __restrict__ back,
                                                             const int64_t* __restrict__ seg, int E,
                                                             float4* __restrict__ gout) {
    const int64_t total = seg[E];
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < total; p += (int64_t)gridDim.x * 256) {
        const int64_t b = back[p];
        gout[p] = b >= 0 ? gy[b] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
}

constexpr unsigned kEpBlocks = 1024;  // fixed grids (graph-replayable): they stride to the device slot count

// The exchange plan of a planned expert-parallel frame (expert_parallel.render_rays_ep_batched): per batch b of
// `batch` consecutive rays and expert k, the number of samples routed to k (w_k > 0) -- the counts acn_routed_count*
// gives that batch's pairs (the same t values and routing arithmetic, route_row), so a batch whose segment
// capacities are these counts moves exactly its live records.  One lane per sample; a wave's lanes of one batch
// add their ballot count with one atomic per expert (integer sums: the result does not depend on the order).
__global__ void __launch_bounds__(kBlk) routed_count_batches_kernel(const float* __restrict__ rays, int64_t N, int S,
                                                                    int64_t batch, const float* __restrict__ jit,
                                                                    RouteCfg cfg, unsigned long long* __restrict__ cnt) {
    const int64_t M = N * (int64_t)S;
    const int lane = threadIdx.x & 63;
    for (int64_t m0 = (int64_t)blockIdx.x * kBlk + (threadIdx.x & ~63); m0 < M; m0 += (int64_t)gridDim.x * kBlk) {
        const int64_t m = m0 + lane;
        const bool live = m < M;
        float w[kMaxK];
#pragma unroll
        for (int k = 0; k < kMaxK; ++k) w[k] = 0.0f;
        int64_t b = 0;
        if (live) {
            const int64_t ray = m / S;
            const int s = (int)(m - ray * S);
            b = ray / batch;
            const float* rp = rays + ray * 8;
            const float t = tval(rp[6], rp[7], s, S, jit ? jit + ray * S : nullptr);
            route_row(cfg, rp[0] + rp[3] * t, rp[1] + rp[4] * t, rp[2] + rp[5] * t, w);
        }
        const int64_t last = (m0 + 63 < M ? m0 + 63 : M - 1) / S / batch;
        const int64_t b0 = m0 / S / batch;
        for (int k = 0; k < cfg.K; ++k) {
            if (b0 == last) {   // wave-uniform: the whole wave in one batch
                const uint64_t bal = __ballot(w[k] > 0.0f);
                if (lane == 0 && bal) atomicAdd(&cnt[b0 * cfg.K + k], (unsigned long long)__popcll(bal));
            } else if (live && w[k] > 0.0f) {
                atomicAdd(&cnt[b * cfg.K + k], 1ull);
            }
        }
    }
}

}  // namespace

extern "C" size_t acn_routed_workspace_bytes(int64_t M, int K) {
    const int64_t nblk = (M + kBlk - 1) / kBlk;
    return (size_t)(M * K) * sizeof(float) + (size_t)(nblk * K) * sizeof(int32_t) + 16;
}

extern "C" int acn_routed_count(const float* rays, int64_t N, int S, const float* jitter, const acn_routing* routing,
                                int align, float* t_vals, int64_t* starts, void* workspace, size_t workspace_bytes,
                                void* stream) {
    ACN_REQUIRE(N >= 0 && S >= 1 && routing && starts && align >= 1, "acn_routed_count: bad arguments");
    const int K = routing->K;
    ACN_REQUIRE(K >= 1 && K <= kMaxK, "acn_routed_count: K = %d outside [1, %d]", K, kMaxK);
    const int64_t M = N * (int64_t)S;
    ACN_REQUIRE(workspace && workspace_bytes >= acn_routed_workspace_bytes(M, K),
                "acn_routed_count: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    if (M == 0) {
        const hipError_t e = hipMemsetAsync(starts, 0, (size_t)(2 * K + 1) * sizeof(int64_t), s);
        return e == hipSuccess ? ACN_OK : acn_set_error((int)e, "acn_routed_count: memset failed");
    }
    ACN_REQUIRE(rays && t_vals, "acn_routed_count: NULL pointer");
    RouteCfg cfg{};
    cfg.K = K;
    cfg.cluster_2d = routing->cluster_2d;
    cfg.bm = routing->boundary_margin;
    cfg.routing = routing->boundary_margin > 1.0f ? 1 : 2;
    for (int k = 0; k < K; ++k)
        for (int a = 0; a < 3; ++a) cfg.cent[k][a] = routing->centroids[k][a];
    float* W = (float*)workspace;
    int32_t* blk = (int32_t*)(W + M * K);
    const int64_t nblk = (M + kBlk - 1) / kBlk;
    hipLaunchKernelGGL(routed_count_kernel, dim3(blocks_for(M, kBlk)), dim3(kBlk), 0, s, rays, N, S, jitter, cfg, t_vals,
                       W, blk, 0);
    Caps caps{};
    hipLaunchKernelGGL(routed_scan_kernel, dim3(1), dim3(1024), 0, s, blk, nblk, K, align, caps, starts);
    return acn_check_launch("acn_routed_count");
}

extern "C" int acn_routed_count_fixed(const float* rays, int64_t N, int S, const float* jitter,
                                      const acn_routing* routing, int64_t cap, float* t_vals, int64_t* starts,
                                      void* workspace, size_t workspace_bytes, void* stream) {
    ACN_REQUIRE(routing && routing->K >= 1 && routing->K <= kMaxK, "acn_routed_count_fixed: bad routing");
    int64_t caps[kMaxK];
    for (int k = 0; k < routing->K; ++k) caps[k] = cap;
    return acn_routed_count_caps(rays, N, S, jitter, routing, caps, t_vals, starts, workspace, workspace_bytes, stream);
}

extern "C" int acn_routed_count_caps(const float* rays, int64_t N, int S, const float* jitter,
                                     const acn_routing* routing, const int64_t* caps_host, float* t_vals,
                                     int64_t* starts, void* workspace, size_t workspace_bytes, void* stream) {
    return acn_routed_count_caps_tiled(rays, N, S, jitter, routing, caps_host, 0, t_vals, starts, workspace,
                                       workspace_bytes, stream);
}

extern "C" int acn_routed_count_caps_tiled(const float* rays, int64_t N, int S, const float* jitter,
                                           const acn_routing* routing, const int64_t* caps_host, int tile_rays,
                                           float* t_vals, int64_t* starts, void* workspace, size_t workspace_bytes,
                                           void* stream) {
    ACN_REQUIRE(N >= 0 && S >= 1 && routing && starts && caps_host && tile_rays >= 0,
                "acn_routed_count_caps: bad arguments");
    const int K = routing->K;
    ACN_REQUIRE(K >= 1 && K <= kMaxK, "acn_routed_count_caps: K = %d outside [1, %d]", K, kMaxK);
    const int64_t M = N * (int64_t)S;
    Caps caps{};
    caps.fixed = 1;
    for (int k = 0; k < K; ++k) {
        ACN_REQUIRE(caps_host[k] >= 0, "acn_routed_count_caps: capacity of expert %d must be >= 0", k);
        caps.cap[k] = caps_host[k];
        caps.off[k + 1] = caps.off[k] + caps_host[k];
    }
    ACN_REQUIRE(workspace && workspace_bytes >= acn_routed_workspace_bytes(M, K),
                "acn_routed_count_caps: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    RouteCfg cfg{};
    cfg.K = K;
    cfg.cluster_2d = routing->cluster_2d;
    cfg.bm = routing->boundary_margin;
    cfg.routing = routing->boundary_margin > 1.0f ? 1 : 2;
    for (int k = 0; k < K; ++k)
        for (int a = 0; a < 3; ++a) cfg.cent[k][a] = routing->centroids[k][a];
    float* W = (float*)workspace;
    int32_t* blk = (int32_t*)(W + M * K);
    const int64_t nblk = (M + kBlk - 1) / kBlk;
    if (M > 0) {
        ACN_REQUIRE(rays && t_vals, "acn_routed_count_caps: NULL pointer");
        hipLaunchKernelGGL(routed_count_kernel, dim3(blocks_for(M, kBlk)), dim3(kBlk), 0, s, rays, N, S, jitter, cfg,
                           t_vals, W, blk, tile_rays);
    }
    hipLaunchKernelGGL(routed_scan_kernel, dim3(1), dim3(1024), 0, s, blk, nblk, K, 1, caps, starts);
    return acn_check_launch("acn_routed_count_caps");
}

extern "C" int acn_routed_scatter(const float* rays, int64_t N, int S, int K, const float* t_vals,
                                  const int64_t* starts, const float* aabb_min, const float* aabb_extent, float lo,
                                  float hi, int align, const void* workspace, int32_t* pidx, float* pw, float* x01,
                                  float* sh, int32_t* pmap, int32_t* pk, void* stream) {
    ACN_REQUIRE(N >= 0 && S >= 1 && K >= 1 && K <= kMaxK && aabb_min && aabb_extent,
                "acn_routed_scatter: bad arguments");
    const int64_t M = N * (int64_t)S;
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(rays && t_vals && starts && workspace && pidx && pw && x01 && sh && pmap,
                "acn_routed_scatter: NULL pointer");
    BoxCfg box{};
    for (int k = 0; k < K; ++k)
        for (int a = 0; a < 3; ++a) {
            box.amin[k][a] = aabb_min[3 * k + a];
            box.ext[k][a] = aabb_extent[3 * k + a];
        }
    box.lo = lo;
    box.hi = hi;
    const float* W = (const float*)workspace;
    const int32_t* blk = (const int32_t*)(W + M * K);
    hipLaunchKernelGGL(routed_scatter_kernel<0>, dim3(blocks_for(M, kBlk)), dim3(kBlk), 0, (hipStream_t)stream, rays,
                       N, S, K, t_vals, W, blk, starts, box, pidx, pw, x01, sh, pmap, pk, align > 1 ? 1 : 0, 0);
    return acn_check_launch("acn_routed_scatter");
}

extern "C" int acn_routed_blend_fwd(const float* y, const float* pw, const int32_t* pmap, int64_t M, int K, float* out,
                                    void* stream) {
    ACN_REQUIRE(M >= 0 && K >= 1 && K <= kMaxK, "acn_routed_blend_fwd: bad arguments");
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(pw && pmap && out, "acn_routed_blend_fwd: NULL pointer");
    hipLaunchKernelGGL(blend_fwd_kernel, dim3(blocks_for(M, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)y, pw, pmap, M, K, (float4*)out);
    return acn_check_launch("acn_routed_blend_fwd");
}

extern "C" int acn_routed_blend_bwd(const float* g, const int32_t* pidx, const float* pw, int64_t P,
                                    const int64_t* live, float* gy, void* stream) {
    ACN_REQUIRE(P >= 0, "acn_routed_blend_bwd: bad arguments");
    if (P == 0) return ACN_OK;
    ACN_REQUIRE(g && pidx && pw && gy, "acn_routed_blend_bwd: NULL pointer");
    hipLaunchKernelGGL(blend_bwd_kernel, dim3(blocks_for(P, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)g, pidx, pw, P, live, (float4*)gy);
    return acn_check_launch("acn_routed_blend_bwd");
}

extern "C" int acn_routed_scatter_xd(const float* rays, int64_t N, int S, int K, const float* t_vals, const int64_t* seg,
                                     const void* workspace, int32_t* pidx, float* pw, float* xd, int32_t* pmap,
                                     int32_t* pk, void* stream) {
    return acn_routed_scatter_xd_tiled(rays, N, S, K, 0, t_vals, seg, workspace, pidx, pw, xd, pmap, pk, stream);
}

extern "C" int acn_routed_scatter_xd_tiled(const float* rays, int64_t N, int S, int K, int tile_rays,
                                           const float* t_vals, const int64_t* seg, const void* workspace,
                                           int32_t* pidx, float* pw, float* xd, int32_t* pmap, int32_t* pk,
                                           void* stream) {
    ACN_REQUIRE(N >= 0 && S >= 1 && K >= 1 && K <= kMaxK && tile_rays >= 0, "acn_routed_scatter_xd: bad arguments");
    const int64_t M = N * (int64_t)S;
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(rays && t_vals && seg && workspace && pidx && pw && xd && pmap, "acn_routed_scatter_xd: NULL pointer");
    BoxCfg box{};
    const float* W = (const float*)workspace;
    const int32_t* blk = (const int32_t*)(W + M * K);
    hipLaunchKernelGGL(routed_scatter_kernel<1>, dim3(blocks_for(M, kBlk)), dim3(kBlk), 0, (hipStream_t)stream, rays,
                       N, S, K, t_vals, W, blk, seg, box, pidx, pw, xd, (float*)nullptr, pmap, pk, 0, tile_rays);
    return acn_check_launch("acn_routed_scatter_xd");
}

extern "C" int acn_xd_unit_sh(const float* xd, int64_t P, const float* aabb_min, const float* aabb_extent, float lo,
                              float hi, float* x01, float* sh, void* stream) {
    ACN_REQUIRE(P >= 0 && aabb_min && aabb_extent, "acn_xd_unit_sh: bad arguments");
    if (P == 0) return ACN_OK;
    ACN_REQUIRE(xd && x01 && sh, "acn_xd_unit_sh: NULL pointer");
    hipLaunchKernelGGL(xd_unit_sh_kernel, dim3(blocks_for(P, 256)), dim3(256), 0, (hipStream_t)stream, xd, P,
                       make_float3(aabb_min[0], aabb_min[1], aabb_min[2]),
                       make_float3(aabb_extent[0], aabb_extent[1], aabb_extent[2]), lo, hi, x01, sh);
    return acn_check_launch("acn_xd_unit_sh");
}

extern "C" int acn_routed_pad_pairs(const int64_t* seg, int K, int64_t max_pad, int32_t* pidx, float* pw, void* stream) {
    ACN_REQUIRE(seg && pidx && pw && K >= 1 && K <= kMaxK && max_pad >= 0, "acn_routed_pad_pairs: bad arguments");
    if (max_pad == 0) return ACN_OK;
    hipLaunchKernelGGL(pad_pairs_kernel, dim3(blocks_for(max_pad, 256) < 256 ? blocks_for(max_pad, 256) : 256, K),
                       dim3(256), 0, (hipStream_t)stream, seg, K, pidx, pw);
    return acn_check_launch("acn_routed_pad_pairs");
}

extern "C" size_t acn_ep_workspace_bytes(int W, int E) { return (size_t)W * (size_t)E * sizeof(int64_t); }

extern "C" int acn_ep_gather(const float* recv_xd, const int64_t* recv_cnt, int W, int E, int64_t cap, int align,
                             const float* aabb_min, const float* aabb_extent, float lo, float hi, int64_t* seg,
                             void* workspace, float* x01, float* sh, int32_t* pk, int32_t* pflag, int64_t* back,
                             void* stream) {
    ACN_REQUIRE(E >= 1 && E <= kMaxK && cap >= 1, "acn_ep_gather: bad arguments");
    int64_t caps[kMaxK];
    for (int j = 0; j < E; ++j) caps[j] = cap;
    return acn_ep_gather_caps(recv_xd, recv_cnt, W, E, caps, align, aabb_min, aabb_extent, lo, hi, seg, workspace, x01,
                              sh, pk, pflag, back, stream);
}

extern "C" int acn_ep_gather_caps(const float* recv_xd, const int64_t* recv_cnt, int W, int E, const int64_t* caps_host,
                                  int align, const float* aabb_min, const float* aabb_extent, float lo, float hi,
                                  int64_t* seg, void* workspace, float* x01, float* sh, int32_t* pk, int32_t* pflag,
                                  int64_t* back, void* stream) {
    ACN_REQUIRE(W >= 1 && E >= 1 && E <= kMaxK && caps_host && align >= 1 && aabb_min && aabb_extent,
                "acn_ep_gather: bad arguments");
    OwnCaps oc{};
    for (int j = 0; j < E; ++j) {
        ACN_REQUIRE(caps_host[j] >= 1, "acn_ep_gather: capacity of local expert %d must be >= 1", j);
        oc.cap[j] = caps_host[j];
        oc.off[j] = oc.row;
        oc.row += caps_host[j];
    }
    ACN_REQUIRE(recv_xd && recv_cnt && seg && workspace && x01 && sh && pk && pflag && back,
                "acn_ep_gather: NULL pointer");
    BoxCfg box{};
    for (int j = 0; j < E; ++j)
        for (int a = 0; a < 3; ++a) {
            box.amin[j][a] = aabb_min[3 * j + a];
            box.ext[j][a] = aabb_extent[3 * j + a];
        }
    box.lo = lo;
    box.hi = hi;
    hipStream_t s = (hipStream_t)stream;
    int64_t* off = (int64_t*)workspace;
    hipLaunchKernelGGL(ep_seg_kernel, dim3(1), dim3(64), 0, s, recv_cnt, W, E, align, oc, off, seg);
    hipLaunchKernelGGL(ep_gather_kernel, dim3(kEpBlocks), dim3(256), 0, s, recv_xd, recv_cnt, (const int64_t*)off,
                       (const int64_t*)seg, W, E, oc, box, x01, sh, pk, pflag, back);
    return acn_check_launch("acn_ep_gather");
}

extern "C" int acn_ep_scatter_back(const float* out, const int64_t* back, const int64_t* seg, int E, float* ret,
                                   void* stream) {
    ACN_REQUIRE(out && back && seg && ret && E >= 1 && E <= kMaxK, "acn_ep_scatter_back: bad arguments");
    hipLaunchKernelGGL(ep_scatter_back_kernel, dim3(kEpBlocks), dim3(256), 0, (hipStream_t)stream, (const float4*)out,
                       back, seg, E, (float4*)ret);
    return acn_check_launch("acn_ep_scatter_back");
}

extern "C" int acn_ep_gather_grad(const float* gy, const int64_t* back, const int64_t* seg, int E, float* gout,
                                  void* stream) {
    ACN_REQUIRE(gy && back && seg && gout && E >= 1 && E <= kMaxK, "acn_ep_gather_grad: bad arguments");
    hipLaunchKernelGGL(ep_gather_grad_kernel, dim3(kEpBlocks), dim3(256), 0, (hipStream_t)stream, (const float4*)gy,
                       back, seg, E, (float4*)gout);
    return acn_check_launch("acn_ep_gather_grad");
}

extern "C" int acn_routed_count_batches(const float* rays, int64_t N, int S, int64_t batch, const float* jitter,
                                        const acn_routing* routing, int64_t* counts, void* stream) {
    ACN_REQUIRE(N >= 0 && S >= 1 && batch >= 1 && routing && counts, "acn_routed_count_batches: bad arguments");
    const int K = routing->K;
    ACN_REQUIRE(K >= 1 && K <= kMaxK, "acn_routed_count_batches: K = %d outside [1, %d]", K, kMaxK);
    const int64_t nb = (N + batch - 1) / batch;
    hipStream_t s = (hipStream_t)stream;
    if (nb > 0) {
        const hipError_t e = hipMemsetAsync(counts, 0, (size_t)(nb * K) * sizeof(int64_t), s);
        if (e != hipSuccess) return acn_set_error((int)e, "acn_routed_count_batches: memset failed");
    }
    const int64_t M = N * (int64_t)S;
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(rays, "acn_routed_count_batches: NULL rays");
    RouteCfg cfg{};
    cfg.K = K;
    cfg.cluster_2d = routing->cluster_2d;
    cfg.bm = routing->boundary_margin;
    cfg.routing = routing->boundary_margin > 1.0f ? 1 : 2;
    for (int k = 0; k < K; ++k)
        for (int a = 0; a < 3; ++a) cfg.cent[k][a] = routing->centroids[k][a];
    const unsigned blocks = blocks_for(M, kBlk) < 8192u ? blocks_for(M, kBlk) : 8192u;
    hipLaunchKernelGGL(routed_count_batches_kernel, dim3(blocks), dim3(kBlk), 0, s, rays, N, S, batch, jitter, cfg,
                       (unsigned long long*)counts);
    return acn_check_launch("acn_routed_count_batches");
}
