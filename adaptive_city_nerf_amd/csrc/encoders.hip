// encoders.hip -- standalone HashGridEncoder forward/backward and SHEncoder forward (gfx950).
//
// Replaces models/encodings.py:331-381 (HashGridEncoder._torch_forward, _hash :308-316, _gather
// :318-329) and :133-151 (SHEncoder.forward).  One lane per (point, level): the L lanes of a
// point are adjacent, so the (M, L*F) output row of a point is written as one contiguous
// L*F*4-byte segment (128 B for the reference's L=16, F=2) and the point's x01 is a broadcast.
#include "acn_device.h"
#include "acn_internal.h"

namespace {

struct Res32 {
    int32_t v[ACN_MAX_LEVELS];
};

template <int INTERP>
__global__ void __launch_bounds__(256) hashgrid_fwd_f2(const float* __restrict__ x01, int64_t M,
                                                       const float2* __restrict__ table, Res32 res,
                                                       int L, int log2T, float2* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = gid / L;
    const int l = (int)(gid - m * L);
    if (m >= M) return;
    const float r = (float)res.v[l];
    const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    const float2* tl = table + ((int64_t)l << log2T);
    float o0, o1;
    acn::hash_level_f2<INTERP>(tl, sx, sy, sz, mask, o0, o1);
    out[m * L + l] = make_float2(o0, o1);
}

// Linear / Smoothstep through a buffer resource over the whole table (the renders' gather form):
// 32-bit row offsets, and the x-neighbours of each (y, z) corner pair come from one 16-B block when x0 is even
// (hash_issue_x: 4 dwordx4 gathers, plus 4 dwordx2 only for odd x0).  The same rows and the same lerp chain as
// hash_level_f2, so the outputs are bitwise those of hashgrid_fwd_f2.  Tables up to 2 GiB (acn_hashgrid_fwd).
#ifndef ACN_HASH_FWD_BUF
#define ACN_HASH_FWD_BUF 1
#endif
template <int INTERP>
__global__ void __launch_bounds__(256) hashgrid_fwd_f2_buf(const float* __restrict__ x01, int64_t M,
                                                           const float2* __restrict__ table, Res32 res, int L,
                                                           int log2T, float2* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = gid / L;
    const int l = (int)(gid - m * L);
    if (m >= M) return;
    const float r = (float)res.v[l];
    const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)table, (short)0, (int)((uint32_t)L << (log2T + 3)), 0x00020000);
    acn::HashPendingX p;
    acn::hash_issue_x<INTERP>(rs, (uint32_t)l << (log2T + 3), sx, sy, sz, mask, p);
    float o0, o1;
    acn::hash_finish_x<INTERP>(p, o0, o1);
    out[m * L + l] = make_float2(o0, o1);
}

// generic feature count (F != 2)
template <int INTERP>
__global__ void __launch_bounds__(256) hashgrid_fwd_gen(const float* __restrict__ x01, int64_t M,
                                                        const float* __restrict__ table, Res32 res, int L,
                                                        int log2T, int F, float* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = gid / L;
    const int l = (int)(gid - m * L);
    if (m >= M) return;
    const float r = (float)res.v[l];
    const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    const float* tl = table + ((int64_t)l << log2T) * F;
    float* o = out + (m * L + l) * F;
    if (INTERP == 0) {
        const uint32_t ix = (uint32_t)(int)rintf(sx), iy = (uint32_t)(int)rintf(sy), iz = (uint32_t)(int)rintf(sz);
        const float* e = tl + (int64_t)((ix ^ (iy * acn::kP1) ^ (iz * acn::kP2)) & mask) * F;
        for (int f = 0; f < F; ++f) o[f] = e[f];
        return;
    }
    const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
    float wx = sx - fx, wy = sy - fy, wz = sz - fz;
    if (INTERP == 2) {
        wx = (wx * wx) * (3.0f - 2.0f * wx);
        wy = (wy * wy) * (3.0f - 2.0f * wy);
        wz = (wz * wz) * (3.0f - 2.0f * wz);
    }
    const uint32_t x0 = (uint32_t)(int)fx, x1 = x0 + 1u;
    const uint32_t y0 = (uint32_t)(int)fy * acn::kP1, y1 = y0 + acn::kP1;
    const uint32_t z0 = (uint32_t)(int)fz * acn::kP2, z1 = z0 + acn::kP2;
    const float* c[8];
    c[0] = tl + (int64_t)((x0 ^ y0 ^ z0) & mask) * F;  // f000
    c[1] = tl + (int64_t)((x0 ^ y0 ^ z1) & mask) * F;  // f001
    c[2] = tl + (int64_t)((x0 ^ y1 ^ z0) & mask) * F;  // f010
    c[3] = tl + (int64_t)((x0 ^ y1 ^ z1) & mask) * F;  // f011
    c[4] = tl + (int64_t)((x1 ^ y0 ^ z0) & mask) * F;  // f100
    c[5] = tl + (int64_t)((x1 ^ y0 ^ z1) & mask) * F;  // f101
    c[6] = tl + (int64_t)((x1 ^ y1 ^ z0) & mask) * F;  // f110
    c[7] = tl + (int64_t)((x1 ^ y1 ^ z1) & mask) * F;  // f111
    const float ax = 1.0f - wx, ay = 1.0f - wy, az = 1.0f - wz;
    for (int f = 0; f < F; ++f) {
        const float c00 = c[0][f] * ax + c[4][f] * wx;
        const float c01 = c[1][f] * ax + c[5][f] * wx;
        const float c10 = c[2][f] * ax + c[6][f] * wx;
        const float c11 = c[3][f] * ax + c[7][f] * wx;
        const float c0 = c00 * ay + c10 * wy;
        const float c1 = c01 * ay + c11 * wy;
        o[f] = c0 * az + c1 * wz;
    }
}

// Backward: autograd of the 8 gathers + lerps.  The gradient of corner (bx,by,bz) is
// ((g * wz') * wy') * wx' in the chain-rule order of the forward lerps, scatter-added with
// no-return fp32 atomics (global_atomic_add_f32), as torch's index_put_(accumulate=True).
template <int INTERP>
__global__ void __launch_bounds__(256) hashgrid_bwd_gen(const float* __restrict__ x01, int64_t M,
                                                        const float* __restrict__ gout, Res32 res, int L,
                                                        int log2T, int F, float* __restrict__ gtable) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = gid / L;
    const int l = (int)(gid - m * L);
    if (m >= M) return;
    const float r = (float)res.v[l];
    const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    float* tl = gtable + ((int64_t)l << log2T) * F;
    const float* g = gout + (m * L + l) * F;
    if (INTERP == 0) {
        const uint32_t ix = (uint32_t)(int)rintf(sx), iy = (uint32_t)(int)rintf(sy), iz = (uint32_t)(int)rintf(sz);
        float* e = tl + (int64_t)((ix ^ (iy * acn::kP1) ^ (iz * acn::kP2)) & mask) * F;
        for (int f = 0; f < F; ++f) unsafeAtomicAdd(e + f, g[f]);
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
    const uint32_t x0 = (uint32_t)(int)fx;
    const uint32_t y0 = (uint32_t)(int)fy * acn::kP1;
    const uint32_t z0 = (uint32_t)(int)fz * acn::kP2;
#pragma unroll
    for (int cidx = 0; cidx < 8; ++cidx) {
        const int bx = cidx >> 2, by = (cidx >> 1) & 1, bz = cidx & 1;
        const uint32_t h = ((x0 + (uint32_t)bx) ^ (y0 + (by ? acn::kP1 : 0u)) ^ (z0 + (bz ? acn::kP2 : 0u))) & mask;
        float* e = tl + (int64_t)h * F;
        for (int f = 0; f < F; ++f) {
            const float gv = ((g[f] * (bz ? wz : az)) * (by ? wy : ay)) * (bx ? wx : ax);
            unsafeAtomicAdd(e + f, gv);
        }
    }
}

// F == 2, Linear/Smoothstep: one lane per (point, level, corner, feature).  A wave covers 4
// consecutive points at ONE level, lanes ordered (point, y/z corner, x corner, feature), so each
// no-return atomic instruction touches ~16 table row pairs (the x-neighbours of a corner pair
// share a 128-B line) instead of the 64 unrelated rows of the lane-per-(point, level) mapping
// (MI355X_MICROARCH.md "Global float atomics": rate set by distinct rows per instruction).  The
// per-corner gradient keeps the forward's chain-rule order ((g * wz) * wy) * wx.
template <int INTERP>
__global__ void __launch_bounds__(256) hashgrid_bwd_f2(const float* __restrict__ x01, int64_t M,
                                                       const float* __restrict__ gout, Res32 res, int L,
                                                       int log2T, float* __restrict__ gtable) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t groups = (M + 3) >> 2;               // groups of 4 points
    const int l = (int)(wave / groups);
    const int64_t m = (wave - (int64_t)l * groups) * 4 + (lane >> 4);
    if (l >= L || m >= M) return;
    const int f = lane & 1, bx = (lane >> 1) & 1, by = (lane >> 3) & 1, bz = (lane >> 2) & 1;
    const float r = (float)res.v[l];
    const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
    float wx = sx - fx, wy = sy - fy, wz = sz - fz;
    if (INTERP == 2) {
        wx = (wx * wx) * (3.0f - 2.0f * wx);
        wy = (wy * wy) * (3.0f - 2.0f * wy);
        wz = (wz * wz) * (3.0f - 2.0f * wz);
    }
    const uint32_t xi = (uint32_t)(int)fx + (uint32_t)bx;
    const uint32_t yi = (uint32_t)(int)fy * acn::kP1 + (by ? acn::kP1 : 0u);
    const uint32_t zi = (uint32_t)(int)fz * acn::kP2 + (bz ? acn::kP2 : 0u);
    const uint32_t h = (xi ^ yi ^ zi) & mask;
    const float gv = ((gout[(m * L + l) * 2 + f] * (bz ? wz : 1.0f - wz)) * (by ? wy : 1.0f - wy)) * (bx ? wx : 1.0f - wx);
    unsafeAtomicAdd(gtable + (((int64_t)l << log2T) + h) * 2 + f, gv);
}

// Run-length-aggregated variant: lane = (sub-group s = lane >> 4, corner, feature) walks PPL
// consecutive points (a stretch of one ray: the training path lays samples out ray-major) at one
// level, summing gradients in a register while the target row repeats and issuing one atomic per
// run.  Coarse levels see long runs (several samples per cell), which is where the per-row atomic
// contention was; waves interleave levels (l = wave % L) so concurrent waves spread over all levels
// instead of all hammering level 0's few thousand rows at once.  Sum order within a run is the
// sample order; across runs it is the (unordered) atomic order, as before.
template <int INTERP, int PPL>
__global__ void __launch_bounds__(256) hashgrid_bwd_rle(const float* __restrict__ x01, int64_t M,
                                                        const float* __restrict__ gout, Res32 res, int L,
                                                        int log2T, float* __restrict__ gtable, int l0) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int l = l0 + (int)(wave % (L - l0));  // levels l0..L-1 (the coarser ones: hashgrid_bwd_merge)
    const int64_t chunk = wave / (L - l0);
    const int64_t m0 = (chunk * 4 + (lane >> 4)) * PPL;
    if (m0 >= M) return;
    const int f = lane & 1, bx = (lane >> 1) & 1, by = (lane >> 3) & 1, bz = (lane >> 2) & 1;
    const float r = (float)res.v[l];
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    const int64_t base = ((int64_t)l << log2T) * 2 + f;
    int64_t cur = -1;
    float acc = 0.0f;
#pragma unroll 4
    for (int i = 0; i < PPL; ++i) {
        const int64_t m = m0 + i;
        if (m >= M) break;
        const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
        const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
        float wx = sx - fx, wy = sy - fy, wz = sz - fz;
        if (INTERP == 2) {
            wx = (wx * wx) * (3.0f - 2.0f * wx);
            wy = (wy * wy) * (3.0f - 2.0f * wy);
            wz = (wz * wz) * (3.0f - 2.0f * wz);
        }
        const uint32_t xi = (uint32_t)(int)fx + (uint32_t)bx;
        const uint32_t yi = (uint32_t)(int)fy * acn::kP1 + (by ? acn::kP1 : 0u);
        const uint32_t zi = (uint32_t)(int)fz * acn::kP2 + (bz ? acn::kP2 : 0u);
        const int64_t a = base + (int64_t)((xi ^ yi ^ zi) & mask) * 2;
        const float gv = ((gout[(m * L + l) * 2 + f] * (bz ? wz : 1.0f - wz)) * (by ? wy : 1.0f - wy)) *
                         (bx ? wx : 1.0f - wx);
        if (a == cur) {
            acc += gv;
        } else {
            if (cur >= 0) unsafeAtomicAdd(gtable + cur, acc);
            cur = a;
            acc = gv;
        }
    }
    if (cur >= 0) unsafeAtomicAdd(gtable + cur, acc);
}

#ifndef ACN_HASH_BWD_PPL
#define ACN_HASH_BWD_PPL 16  // consecutive points per lane in hashgrid_bwd_rle (0: the per-point kernel)
#endif

// ---------------------------------------------------------------------------------------------
// (sample, expert) pair lists of the routed container (routed.hip): slot p belongs to expert pk[p],
// the live slot count is seg[K] on the device (graph-replayable: grids are fixed, loops stride to it).
struct Tables {
    const float2* t[acn::kMaxK];
};
struct GradTables {
    float* t[acn::kMaxK];
};
struct SegMaps {   // per expert: the "touched this step" byte map of its table's 64-B segments (or null)
    uint8_t* t[acn::kMaxK];
};

template <int INTERP, bool BUF = false>
__global__ void __launch_bounds__(256) hashgrid_fwd_pairs(const float* __restrict__ x01, const int32_t* __restrict__ pk,
                                                          const int64_t* __restrict__ seg, int K, Tables tabs,
                                                          Res32 res, int L, int log2T, float2* __restrict__ out) {
    const int64_t n = seg[K] * L;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    for (int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < n; gid += (int64_t)gridDim.x * blockDim.x) {
        const int64_t m = gid / L;
        const int l = (int)(gid - m * L);
        const float r = (float)res.v[l];
        const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
        float o0, o1;
        if (BUF) {
            // buffer gathers (hashgrid_fwd_f2_buf) from the table of the lane's expert: one resource per distinct
            // expert of the wave (a wave's slots normally share one; the loop takes each expert once)
            const int k = pk[m];
            for (;;) {
                const int kw = __builtin_amdgcn_readfirstlane(k);
                if (k == kw) {
                    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                        (void*)tabs.t[kw], (short)0, (int)((uint32_t)L << (log2T + 3)), 0x00020000);
                    acn::HashPendingX p;
                    acn::hash_issue_x<INTERP>(rs, (uint32_t)l << (log2T + 3), sx, sy, sz, mask, p);
                    acn::hash_finish_x<INTERP>(p, o0, o1);
                    break;
                }
            }
        } else {
            const float2* tl = tabs.t[pk[m]] + ((int64_t)l << log2T);
            acn::hash_level_f2<INTERP>(tl, sx, sy, sz, mask, o0, o1);
        }
        out[m * L + l] = make_float2(o0, o1);
    }
}

// hashgrid_bwd_rle over pair slots: the run key is the target address, so a stretch may cross an
// expert boundary; padding slots (pidx < 0) add nothing
// TELE: returning atomics; every run adds new^2 - old^2 (new = old + run sum, the value the atomic
// leaves) to *sq.  Per row these telescope to (final value)^2 - 0, so *sq gains the squared norm of the
// table-gradient update without a pass over the 128 MiB gradient buffers (clip_grad_norm_'s sum of
// squares, runtime_adapt.py:305-307).  Doubles: new^2 and old^2 are exact, so only the differences and
// their sum round (~1e-16 relative).
template <int INTERP, int PPL, bool TELE, bool MARK_ONLY = false>
__global__ void __launch_bounds__(256) hashgrid_bwd_pairs(const float* __restrict__ x01, const int32_t* __restrict__ pk,
                                                          const int32_t* __restrict__ pidx,
                                                          const int64_t* __restrict__ seg, int K,
                                                          const float* __restrict__ gout, GradTables gt, Res32 res,
                                                          int L, int log2T, int l0, double* __restrict__ sq,
                                                          SegMaps smaps) {
    const int lane = threadIdx.x & 63;
    const int64_t M = seg[K];
    const int64_t nwaves = ((M + 4 * PPL - 1) / (4 * PPL)) * (L - l0);
    const int f = lane & 1, bx = (lane >> 1) & 1, by = (lane >> 3) & 1, bz = (lane >> 2) & 1;
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    double tsq = 0.0;
    auto flush = [&](float* a, float v) {
        if (MARK_ONLY) return;   // acn_hashgrid_pairs_mark: segment maps only
        if (TELE) {
            const float o = atomicAdd(a, v);
            const float nv = o + v;
            tsq += (double)nv * (double)nv - (double)o * (double)o;
        } else {
            unsafeAtomicAdd(a, v);
        }
    };
    for (int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; wave < nwaves;
         wave += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int l = l0 + (int)(wave % (L - l0));
        const int64_t chunk = wave / (L - l0);
        const int64_t m0 = (chunk * 4 + (lane >> 4)) * PPL;
        const float r = (float)res.v[l];
        const int64_t base = ((int64_t)l << log2T) * 2 + f;
        float* cur = nullptr;
        uint8_t* cseg = nullptr;   // the segment-map byte of cur's 64-B segment (segment maps on)
        float acc = 0.0f;
        for (int i = 0; i < PPL; ++i) {
            const int64_t m = m0 + i;
            if (m >= M) break;
            if (pidx[m] < 0) continue;
            const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
            const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
            float wx = sx - fx, wy = sy - fy, wz = sz - fz;
            if (INTERP == 2) {
                wx = (wx * wx) * (3.0f - 2.0f * wx);
                wy = (wy * wy) * (3.0f - 2.0f * wy);
                wz = (wz * wz) * (3.0f - 2.0f * wz);
            }
            const uint32_t xi = (uint32_t)(int)fx + (uint32_t)bx;
            const uint32_t yi = (uint32_t)(int)fy * acn::kP1 + (by ? acn::kP1 : 0u);
            const uint32_t zi = (uint32_t)(int)fz * acn::kP2 + (bz ? acn::kP2 : 0u);
            const int kk = pk[m];
            const uint32_t row = (xi ^ yi ^ zi) & mask;
            float* a = gt.t[kk] + base + (int64_t)row * 2;
            const float gv = MARK_ONLY ? 0.0f : ((gout[(m * L + l) * 2 + f] * (bz ? wz : 1.0f - wz)) *
                                                 (by ? wy : 1.0f - wy)) * (bx ? wx : 1.0f - wx);
            if (a == cur) {
                acc += gv;
            } else {
                if (cur) {
                    flush(cur, acc);
                    if (cseg && f == 0) *cseg = 1;   // idempotent plain byte store (feature 1 shares the row)
                }
                cur = a;
                cseg = smaps.t[kk] ? smaps.t[kk] + ((((int64_t)l << log2T) + row) >> 3) : nullptr;
                acc = gv;
            }
        }
        if (cur) {
            flush(cur, acc);
            if (cseg && f == 0) *cseg = 1;
        }
    }
    if (TELE) {  // one double atomic per wave
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) tsq += __shfl_xor(tsq, off);
        if (lane == 0 && tsq != 0.0) atomicAdd(sq, tsq);
    }
}

// ---------------------------------------------------------------------------------------------
// Coarse levels of the table-gradient scatter, merged per workgroup.  At the coarse
// levels many samples -- of one ray and of neighbouring rays -- add into the same rows, but a lane's run
// merge only sees one corner of one sample stream.  Here a workgroup takes a chunk of C_l consecutive
// slots at one level, accumulates every (slot, corner) contribution into an LDS hash table keyed by
// (table, 64-B segment) with LDS float atomics, then flushes each touched segment as 16 consecutive
// floats (4 segments per wave-instruction = the full-rate shape of MI355X_MICROARCH.md 'Global float
// atomics').  Memory-side requests fall from one per (run, corner pair) to one per distinct segment of
// the chunk.  A full table (more distinct segments than kMergeNE) falls back to direct atomics for the
// overflowing contributions.  Sums stay fp32; their order is as unordered as the atomics they replace.
constexpr int kMergeLogNE = 10, kMergeNE = 1 << kMergeLogNE;
constexpr uint32_t kMergeEmpty = 0xffffffffu;
struct MergeCfg {
    int LM;                   // levels 0 .. LM-1 are merged here
    int clog2[ACN_MAX_LEVELS];  // chunk of 2^clog2[l] slots per workgroup item at level l
};

template <int INTERP>
__global__ void __launch_bounds__(256) hashgrid_bwd_merge(const float* __restrict__ x01, const int32_t* __restrict__ pk,
                                                          const int32_t* __restrict__ pidx,
                                                          const int64_t* __restrict__ seg, int K, int64_t Mhost,
                                                          const float* __restrict__ gout, GradTables gt, Res32 res,
                                                          int L, int log2T, MergeCfg cfg) {
    __shared__ uint32_t keys[kMergeNE];
    __shared__ __attribute__((aligned(16))) float vals[kMergeNE * 16];
    const int64_t M = seg ? seg[K] : Mhost;
    int64_t items = 0;
    for (int l = 0; l < cfg.LM; ++l) items += (M + (1ll << cfg.clog2[l]) - 1) >> cfg.clog2[l];
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
        int l = 0;
        int64_t rem = it;
        for (; l < cfg.LM - 1; ++l) {
            const int64_t n = (M + (1ll << cfg.clog2[l]) - 1) >> cfg.clog2[l];
            if (rem < n) break;
            rem -= n;
        }
        const int64_t m0 = rem << cfg.clog2[l], m1 = min(M, m0 + (1ll << cfg.clog2[l]));
        for (int i = threadIdx.x; i < kMergeNE; i += blockDim.x) keys[i] = kMergeEmpty;
        for (int i = threadIdx.x; i < kMergeNE * 4; i += blockDim.x)
            reinterpret_cast<float4*>(vals)[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        __syncthreads();
        const float r = (float)res.v[l];
        // lanes as in hashgrid_bwd_rle: (stream q, corner, feature f); a lane run-merges 16 consecutive
        // slots of its stream and adds each finished run into the LDS table (LDS atomics on runs, not on
        // every contribution: coarse cells repeat along a ray)
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
        const int f = lane & 1, bx = (lane >> 1) & 1, by = (lane >> 3) & 1, bz = (lane >> 2) & 1;
        auto add_run = [&](uint32_t kx, uint32_t row, float v) {
            const uint32_t key = (kx << 24) | (row >> 3);
            uint32_t h = (key * 2654435761u) >> (32 - kMergeLogNE);
            for (int probe = 0; probe < 32; ++probe) {
                uint32_t cur = keys[h];
                if (cur == kMergeEmpty) cur = atomicCAS(&keys[h], kMergeEmpty, key);
                if (cur == kMergeEmpty || cur == key) {
                    atomicAdd(&vals[h * 16 + (row & 7) * 2 + f], v);
                    return;
                }
                h = (h + 1) & (kMergeNE - 1);
            }
            unsafeAtomicAdd(gt.t[kx] + (((int64_t)l << log2T) + row) * 2 + f, v);  // table crowded
        };
        for (int64_t sb = m0 + (int64_t)w * 64; sb < m1; sb += (int64_t)nw * 64) {
            const int64_t mb = sb + (lane >> 4) * 16;
            uint32_t cur_row = 0xffffffffu, cur_k = 0;
            float acc = 0.0f;
            for (int i = 0; i < 16; ++i) {
                const int64_t m = mb + i;
                if (m >= m1) break;
                if (pidx && pidx[m] < 0) continue;
                const uint32_t kx = pk ? (uint32_t)pk[m] : 0u;
                const float sx = x01[3 * m] * r, sy = x01[3 * m + 1] * r, sz = x01[3 * m + 2] * r;
                const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
                float wx = sx - fx, wy = sy - fy, wz = sz - fz;
                if (INTERP == 2) {
                    wx = (wx * wx) * (3.0f - 2.0f * wx);
                    wy = (wy * wy) * (3.0f - 2.0f * wy);
                    wz = (wz * wz) * (3.0f - 2.0f * wz);
                }
                const uint32_t xi = (uint32_t)(int)fx + (uint32_t)bx;
                const uint32_t yi = (uint32_t)(int)fy * acn::kP1 + (by ? acn::kP1 : 0u);
                const uint32_t zi = (uint32_t)(int)fz * acn::kP2 + (bz ? acn::kP2 : 0u);
                const uint32_t row = (xi ^ yi ^ zi) & mask;
                const float gv = ((gout[(m * L + l) * 2 + f] * (bz ? wz : 1.0f - wz)) * (by ? wy : 1.0f - wy)) *
                                 (bx ? wx : 1.0f - wx);
                if (row == cur_row && kx == cur_k) {
                    acc += gv;
                } else {
                    if (cur_row != 0xffffffffu) add_run(cur_k, cur_row, acc);
                    cur_row = row;
                    cur_k = kx;
                    acc = gv;
                }
            }
            if (cur_row != 0xffffffffu) add_run(cur_k, cur_row, acc);
        }
        __syncthreads();
        // flush: 16 consecutive lanes per segment
        for (int i = threadIdx.x; i < kMergeNE * 16; i += blockDim.x) {
            const uint32_t key = keys[i >> 4];
            const float v = vals[i];
            if (key != kMergeEmpty && v != 0.0f)
                unsafeAtomicAdd(gt.t[key >> 24] + ((int64_t)l << log2T) * 2 + (int64_t)(key & 0xffffffu) * 16 + (i & 15), v);
        }
        __syncthreads();
    }
}

#ifndef ACN_HASH_BWD_MERGE
// coarse levels merged per workgroup in the pair-list scatter (C5; 0: every level on the run-merge kernel).  Off:
// measured slower on the C5 step (hash backward 0.36 -> 0.76 / 0.79 / 0.89 ms merging 3 / 6 / 8 levels,
// tools/ab_c5.sh) -- a coarse chunk is one workgroup's serial work (few items in flight), and the
// runs of neighbouring lanes collide on the same LDS entries; it also cannot telescope the clip norm or mark the
// segment maps the C5 step needs
#define ACN_HASH_BWD_MERGE 0
#endif
#ifndef ACN_HASH_BWD_MERGE_SA
// the same for the standalone scatter (acn_hashgrid_bwd: the meta-training query step, whose batch is ~6x C5's):
// 6 merged levels there cut the scatter 855 -> 795 us and the meta step 1.1%
#define ACN_HASH_BWD_MERGE_SA 6
#endif

MergeCfg merge_cfg(int L, int log2T, int levels = ACN_HASH_BWD_MERGE) {
    MergeCfg c{};
    c.LM = levels < L ? levels : L;
    if (log2T > 27) c.LM = 0;  // the LDS key holds a 24-bit segment index
    // chunks sized so a chunk's distinct segments stay well under kMergeNE at the reference grid
    // (tools/hash_bwd_analysis.py on the C5 batch: level 0 ~13k segments per 104k slots ... level 5 ~230k)
    const int lg[8] = {12, 11, 10, 9, 8, 8, 7, 7};
    for (int l = 0; l < ACN_MAX_LEVELS; ++l) c.clog2[l] = l < 8 ? lg[l] : 7;
    return c;
}

template <int DEGREE>
__global__ void __launch_bounds__(256) sh_fwd_kernel(const float* __restrict__ d, int64_t M,
                                                     float* __restrict__ out) {
    constexpr int C = (DEGREE + 1) * (DEGREE + 1);
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    float c[C];
    acn::sh_encode<DEGREE>(d[3 * m], d[3 * m + 1], d[3 * m + 2], c);
#pragma unroll
    for (int i = 0; i < C; ++i) out[m * C + i] = c[i];
}

}  // namespace

extern "C" int acn_hashgrid_fwd(const float* x01, int64_t M, const float* table, const int32_t* res, int L,
                                int log2T, int F, int interp, float* out, void* stream) {
    ACN_REQUIRE(M >= 0, "acn_hashgrid_fwd: M must be >= 0");
    ACN_REQUIRE(L >= 1 && L <= ACN_MAX_LEVELS, "acn_hashgrid_fwd: levels must be in [1, %d], got %d", ACN_MAX_LEVELS, L);
    ACN_REQUIRE(log2T >= 1 && log2T <= 30, "acn_hashgrid_fwd: log2_hashmap_size must be in [1, 30], got %d", log2T);
    ACN_REQUIRE(F >= 1 && F <= 64, "acn_hashgrid_fwd: features_per_level must be in [1, 64], got %d", F);
    ACN_REQUIRE(interp >= 0 && interp <= 2, "acn_hashgrid_fwd: bad interpolation %d", interp);
    ACN_REQUIRE(res != nullptr, "acn_hashgrid_fwd: res is NULL");
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(x01 && table && out, "acn_hashgrid_fwd: NULL pointer");
    Res32 r{};
    for (int i = 0; i < L; ++i) r.v[i] = res[i];
    const int64_t threads = M * L;
    const dim3 grid((unsigned)((threads + 255) / 256)), block(256);
    hipStream_t s = (hipStream_t)stream;
    if (F == 2) {
        const bool buf = ACN_HASH_FWD_BUF && interp != 0 && ((uint64_t)L << (log2T + 3)) <= (1ull << 31);
        if (buf && interp == 1) hipLaunchKernelGGL(hashgrid_fwd_f2_buf<1>, grid, block, 0, s, x01, M, (const float2*)table, r, L, log2T, (float2*)out);
        else if (buf) hipLaunchKernelGGL(hashgrid_fwd_f2_buf<2>, grid, block, 0, s, x01, M, (const float2*)table, r, L, log2T, (float2*)out);
        else if (interp == 0) hipLaunchKernelGGL(hashgrid_fwd_f2<0>, grid, block, 0, s, x01, M, (const float2*)table, r, L, log2T, (float2*)out);
        else if (interp == 1) hipLaunchKernelGGL(hashgrid_fwd_f2<1>, grid, block, 0, s, x01, M, (const float2*)table, r, L, log2T, (float2*)out);
        else hipLaunchKernelGGL(hashgrid_fwd_f2<2>, grid, block, 0, s, x01, M, (const float2*)table, r, L, log2T, (float2*)out);
    } else {
        if (interp == 0) hipLaunchKernelGGL(hashgrid_fwd_gen<0>, grid, block, 0, s, x01, M, table, r, L, log2T, F, out);
        else if (interp == 1) hipLaunchKernelGGL(hashgrid_fwd_gen<1>, grid, block, 0, s, x01, M, table, r, L, log2T, F, out);
        else hipLaunchKernelGGL(hashgrid_fwd_gen<2>, grid, block, 0, s, x01, M, table, r, L, log2T, F, out);
    }
    return acn_check_launch("acn_hashgrid_fwd");
}

extern "C" int acn_hashgrid_bwd(const float* x01, int64_t M, const float* grad_out, const int32_t* res, int L,
                                int log2T, int F, int interp, float* grad_table, void* stream) {
    ACN_REQUIRE(M >= 0, "acn_hashgrid_bwd: M must be >= 0");
    ACN_REQUIRE(L >= 1 && L <= ACN_MAX_LEVELS, "acn_hashgrid_bwd: levels must be in [1, %d], got %d", ACN_MAX_LEVELS, L);
    ACN_REQUIRE(log2T >= 1 && log2T <= 30, "acn_hashgrid_bwd: log2_hashmap_size must be in [1, 30], got %d", log2T);
    ACN_REQUIRE(F >= 1 && F <= 64, "acn_hashgrid_bwd: features_per_level must be in [1, 64], got %d", F);
    ACN_REQUIRE(interp >= 0 && interp <= 2, "acn_hashgrid_bwd: bad interpolation %d", interp);
    ACN_REQUIRE(res != nullptr, "acn_hashgrid_bwd: res is NULL");
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(x01 && grad_out && grad_table, "acn_hashgrid_bwd: NULL pointer");
    Res32 r{};
    for (int i = 0; i < L; ++i) r.v[i] = res[i];
    hipStream_t s = (hipStream_t)stream;
    if (F == 2 && interp != 0 && ACN_HASH_BWD_PPL > 0) {
        constexpr int PPL = ACN_HASH_BWD_PPL > 0 ? ACN_HASH_BWD_PPL : 1;
        const MergeCfg mc = merge_cfg(L, log2T, ACN_HASH_BWD_MERGE_SA);
        if (mc.LM > 0) {
            GradTables t{};
            t.t[0] = grad_table;
            int64_t items = 0;
            for (int l = 0; l < mc.LM; ++l) items += (M + (1ll << mc.clog2[l]) - 1) >> mc.clog2[l];
            const dim3 mgrid((unsigned)(items < 1024 ? items : 1024)), block(256);
            if (interp == 1) hipLaunchKernelGGL(hashgrid_bwd_merge<1>, mgrid, block, 0, s, x01, nullptr, nullptr, nullptr, 1, M, grad_out, t, r, L, log2T, mc);
            else hipLaunchKernelGGL(hashgrid_bwd_merge<2>, mgrid, block, 0, s, x01, nullptr, nullptr, nullptr, 1, M, grad_out, t, r, L, log2T, mc);
        }
        if (mc.LM < L) {
            const int64_t waves = ((M + 4 * PPL - 1) / (4 * PPL)) * (L - mc.LM);
            const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
            if (interp == 1) hipLaunchKernelGGL((hashgrid_bwd_rle<1, PPL>), grid, block, 0, s, x01, M, grad_out, r, L, log2T, grad_table, mc.LM);
            else hipLaunchKernelGGL((hashgrid_bwd_rle<2, PPL>), grid, block, 0, s, x01, M, grad_out, r, L, log2T, grad_table, mc.LM);
        }
        return acn_check_launch("acn_hashgrid_bwd");
    }
    if (F == 2 && interp != 0) {
        const int64_t waves = ((M + 3) / 4) * L;
        const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
        if (interp == 1) hipLaunchKernelGGL(hashgrid_bwd_f2<1>, grid, block, 0, s, x01, M, grad_out, r, L, log2T, grad_table);
        else hipLaunchKernelGGL(hashgrid_bwd_f2<2>, grid, block, 0, s, x01, M, grad_out, r, L, log2T, grad_table);
        return acn_check_launch("acn_hashgrid_bwd");
    }
    const int64_t threads = M * L;
    const dim3 grid((unsigned)((threads + 255) / 256)), block(256);
    if (interp == 0) hipLaunchKernelGGL(hashgrid_bwd_gen<0>, grid, block, 0, s, x01, M, grad_out, r, L, log2T, F, grad_table);
    else if (interp == 1) hipLaunchKernelGGL(hashgrid_bwd_gen<1>, grid, block, 0, s, x01, M, grad_out, r, L, log2T, F, grad_table);
    else hipLaunchKernelGGL(hashgrid_bwd_gen<2>, grid, block, 0, s, x01, M, grad_out, r, L, log2T, F, grad_table);
    return acn_check_launch("acn_hashgrid_bwd");
}

extern "C" int acn_sh_fwd(const float* d, int64_t M, int levels, float* out, void* stream) {
    ACN_REQUIRE(levels >= 1 && levels <= 5, "acn_sh_fwd: Supported levels in [1, 5], got %d", levels);
    ACN_REQUIRE(M >= 0, "acn_sh_fwd: M must be >= 0");
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(d && out, "acn_sh_fwd: NULL pointer");
    const dim3 grid((unsigned)((M + 255) / 256)), block(256);
    hipStream_t s = (hipStream_t)stream;
    switch (levels) {
        case 1: hipLaunchKernelGGL(sh_fwd_kernel<0>, grid, block, 0, s, d, M, out); break;
        case 2: hipLaunchKernelGGL(sh_fwd_kernel<1>, grid, block, 0, s, d, M, out); break;
        case 3: hipLaunchKernelGGL(sh_fwd_kernel<2>, grid, block, 0, s, d, M, out); break;
        case 4: hipLaunchKernelGGL(sh_fwd_kernel<3>, grid, block, 0, s, d, M, out); break;
        default: hipLaunchKernelGGL(sh_fwd_kernel<4>, grid, block, 0, s, d, M, out); break;
    }
    return acn_check_launch("acn_sh_fwd");
}

extern "C" int acn_hashgrid_fwd_pairs(const float* x01, const int32_t* pk, const int64_t* seg, int K,
                                      const float* const* tables, const int32_t* res, int L, int log2T, int interp,
                                      float* out, void* stream) {
    ACN_REQUIRE(K >= 1 && K <= acn::kMaxK && tables && res && seg && x01 && pk && out,
                "acn_hashgrid_fwd_pairs: bad arguments");
    ACN_REQUIRE(L >= 1 && L <= ACN_MAX_LEVELS && log2T >= 1 && log2T <= 30 && interp >= 0 && interp <= 2,
                "acn_hashgrid_fwd_pairs: bad grid configuration");
    Res32 r{};
    for (int i = 0; i < L; ++i) r.v[i] = res[i];
    Tables t{};
    for (int k = 0; k < K; ++k) t.t[k] = (const float2*)tables[k];
    const dim3 grid(2048), block(256);  // grid-stride to the device slot count
    hipStream_t s = (hipStream_t)stream;
    if (interp == 0) hipLaunchKernelGGL(hashgrid_fwd_pairs<0>, grid, block, 0, s, x01, pk, seg, K, t, r, L, log2T, (float2*)out);
    else if (ACN_HASH_FWD_BUF && ((uint64_t)L << (log2T + 3)) <= (1ull << 31)) {
        if (interp == 1) hipLaunchKernelGGL((hashgrid_fwd_pairs<1, true>), grid, block, 0, s, x01, pk, seg, K, t, r, L, log2T, (float2*)out);
        else hipLaunchKernelGGL((hashgrid_fwd_pairs<2, true>), grid, block, 0, s, x01, pk, seg, K, t, r, L, log2T, (float2*)out);
    }
    else if (interp == 1) hipLaunchKernelGGL(hashgrid_fwd_pairs<1>, grid, block, 0, s, x01, pk, seg, K, t, r, L, log2T, (float2*)out);
    else hipLaunchKernelGGL(hashgrid_fwd_pairs<2>, grid, block, 0, s, x01, pk, seg, K, t, r, L, log2T, (float2*)out);
    return acn_check_launch("acn_hashgrid_fwd_pairs");
}

extern "C" int acn_hashgrid_bwd_pairs(const float* x01, const int32_t* pk, const int32_t* pidx, const int64_t* seg,
                                      int K, const float* grad_out, float* const* grad_tables, const int32_t* res,
                                      int L, int log2T, int interp, void* stream) {
    return acn_hashgrid_bwd_pairs_sumsq(x01, pk, pidx, seg, K, grad_out, grad_tables, res, L, log2T, interp, nullptr,
                                        stream);
}

extern "C" int acn_hashgrid_bwd_pairs_sumsq(const float* x01, const int32_t* pk, const int32_t* pidx,
                                            const int64_t* seg, int K, const float* grad_out,
                                            float* const* grad_tables, const int32_t* res, int L, int log2T,
                                            int interp, double* table_sumsq, void* stream) {
    return acn_hashgrid_bwd_pairs_segmap(x01, pk, pidx, seg, K, grad_out, grad_tables, res, L, log2T, interp,
                                         table_sumsq, nullptr, stream);
}

extern "C" int acn_hashgrid_bwd_pairs_segmap(const float* x01, const int32_t* pk, const int32_t* pidx,
                                             const int64_t* seg, int K, const float* grad_out,
                                             float* const* grad_tables, const int32_t* res, int L, int log2T,
                                             int interp, double* table_sumsq, uint8_t* const* seg_now,
                                             void* stream) {
    ACN_REQUIRE(K >= 1 && K <= acn::kMaxK && grad_tables && res && seg && x01 && pk && pidx && grad_out,
                "acn_hashgrid_bwd_pairs: bad arguments");
    ACN_REQUIRE(L >= 1 && L <= ACN_MAX_LEVELS && log2T >= 1 && log2T <= 30 && (interp == 1 || interp == 2),
                "acn_hashgrid_bwd_pairs: Linear / Smoothstep interpolation only");
    Res32 r{};
    for (int i = 0; i < L; ++i) r.v[i] = res[i];
    GradTables t{};
    for (int k = 0; k < K; ++k) t.t[k] = grad_tables[k];
    SegMaps sm{};
    if (seg_now)
        for (int k = 0; k < K; ++k) sm.t[k] = seg_now[k];
    const dim3 grid(2048), block(256);
    hipStream_t s = (hipStream_t)stream;
    const MergeCfg mc = merge_cfg(L, log2T);
    ACN_REQUIRE(!(table_sumsq && mc.LM > 0), "acn_hashgrid_bwd_pairs_sumsq: not available with the merged coarse "
                "levels (ACN_HASH_BWD_MERGE)");
    ACN_REQUIRE(!(seg_now && mc.LM > 0), "acn_hashgrid_bwd_pairs_segmap: not available with the merged coarse levels");
    if (mc.LM > 0) {  // fixed grid (graph-replayable): items are counted from the device slot count
        if (interp == 1) hipLaunchKernelGGL(hashgrid_bwd_merge<1>, dim3(512), block, 0, s, x01, pk, pidx, seg, K, (int64_t)0, grad_out, t, r, L, log2T, mc);
        else hipLaunchKernelGGL(hashgrid_bwd_merge<2>, dim3(512), block, 0, s, x01, pk, pidx, seg, K, (int64_t)0, grad_out, t, r, L, log2T, mc);
    }
    if (mc.LM < L) {
#define ACN_BWD_PAIRS(I, T) hipLaunchKernelGGL((hashgrid_bwd_pairs<I, 16, T>), grid, block, 0, s, x01, pk, pidx, seg, K, grad_out, t, r, L, log2T, mc.LM, table_sumsq, sm)
        if (table_sumsq) { if (interp == 1) ACN_BWD_PAIRS(1, true); else ACN_BWD_PAIRS(2, true); }
        else { if (interp == 1) ACN_BWD_PAIRS(1, false); else ACN_BWD_PAIRS(2, false); }
#undef ACN_BWD_PAIRS
    }
    return acn_check_launch("acn_hashgrid_bwd_pairs");
}

extern "C" int acn_hashgrid_pairs_mark(const float* x01, const int32_t* pk, const int32_t* pidx, const int64_t* seg,
                                       int K, const int32_t* res, int L, int log2T, int interp,
                                       uint8_t* const* seg_now, void* stream) {
    ACN_REQUIRE(K >= 1 && K <= acn::kMaxK && res && seg && x01 && pk && pidx && seg_now,
                "acn_hashgrid_pairs_mark: bad arguments");
    ACN_REQUIRE(L >= 1 && L <= ACN_MAX_LEVELS && log2T >= 1 && log2T <= 30 && (interp == 1 || interp == 2),
                "acn_hashgrid_pairs_mark: Linear / Smoothstep interpolation only");
    Res32 r{};
    for (int i = 0; i < L; ++i) r.v[i] = res[i];
    GradTables t{};
    SegMaps sm{};
    for (int k = 0; k < K; ++k) {
        sm.t[k] = seg_now[k];
        t.t[k] = reinterpret_cast<float*>(seg_now[k]);   // address arithmetic only: nothing is written through it
    }
    hipStream_t s = (hipStream_t)stream;
    if (interp == 1)
        hipLaunchKernelGGL((hashgrid_bwd_pairs<1, 16, false, true>), dim3(2048), dim3(256), 0, s, x01, pk, pidx, seg, K,
                           (const float*)nullptr, t, r, L, log2T, 0, (double*)nullptr, sm);
    else
        hipLaunchKernelGGL((hashgrid_bwd_pairs<2, 16, false, true>), dim3(2048), dim3(256), 0, s, x01, pk, pidx, seg, K,
                           (const float*)nullptr, t, r, L, log2T, 0, (double*)nullptr, sm);
    return acn_check_launch("acn_hashgrid_pairs_mark");
}
