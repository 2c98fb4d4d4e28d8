// render.hip -- fused field (hash grid -> sigma MLP -> colour MLP) and fused stratified render
// for gfx950 (MI355X).  Replaces the chunked torch-op chains of
//   nerfs/ray_rendering.py:290-345 render_rays_stratified (+ stratified_t_vals :262-287,
//   _get_bg_rgb :23-45, volume_render :114-165),
//   models/inr/meta_container.py:275-343 MetaContainer.forward (+ _routing :97-134,
//   background_color :347-382),
//   models/inr/meta_ngp.py:155-241 MetaNGP._world_to_unit / density / color / forward.
//
// Execution model: one wave owns one ray at a time and walks it front to back in tiles of 32
// samples.  Inside a tile the 64 lanes are (sample j = lane & 31, half h = lane >> 5); half h
// hash-encodes levels 8h..8h+7 of sample j, which is exactly the B-operand layout of
// v_mfma_f32_32x32x2_f32 for the first layer (k-step s pairs feature 16*0+s with 16*1+s).  Every
// MLP layer is H^T = W . X^T on fp32 MFMA (exact fp32 fma chains: parity mode), with the layer's
// accumulator registers feeding the next layer's B operand directly (no LDS round trip).  The
// packed weights of up to two experts sit in LDS (58 KB each); more experts read them from L2.
// Compositing uses a 32-lane exclusive prefix product of (1 - alpha + 1e-10) in double (torch's
// CPU cumprod accumulates in double), carries transmittance across tiles, and stops the ray once
// T < tau (early ray termination; tau = 0 disables it).
#include "acn_device.h"
#include "acn_internal.h"

using namespace acn;

#ifndef ACN_MLP_F16X3
#define ACN_MLP_F16X3 1  // MLP on v_mfma_f32_32x32x16_f16 with a 3-term fp16 split (hi*hi + hi*lo + lo*hi)
#endif

#ifndef ACN_SLOTS
#define ACN_SLOTS 1  // routed K > 2: stage the two most needed experts per workgroup (render_slots_kernel)
#endif

#ifndef ACN_XPAIR
#define ACN_XPAIR 2  // hash gathers: 2 buffer loads of x-paired 16-B blocks (default); 3 buffer loads,
                     // one 8-B row per corner; 0 global loads from 64-bit addresses (round 5: wrong rows in lanes 48-63)
#endif
#ifndef ACN_LEVEL_PARITY
#define ACN_LEVEL_PARITY 0  // 1: half h encodes levels 2i+h (instruction i = two adjacent levels)
#endif
#ifndef ACN_FINE_POL
#define ACN_FINE_POL 0      // load policy (ld_row) of the gathers of the finest levels
#endif
#ifndef ACN_FINE_FROM
#define ACN_FINE_FROM 8     // first gather step i (0..7) that uses ACN_FINE_POL
#endif


typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int rho(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// An opaque zero / copy produced inside the loop body: the packed-weight reads and per-lane
// level selections derived from it cannot be hoisted out of the ray/tile loops by LICM (the
// hoisted values would exceed the 128-VGPR budget of 4 waves/SIMD and get spilled to scratch).
__device__ __forceinline__ int opaque_s(int v) {
    asm volatile("" : "+s"(v));
    return v;
}
__device__ __forceinline__ int opaque_v(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// ------------------------------------------------------------------------------------------
// weight packing
struct PackSrc {
    const float *sig_w0, *sig_b0, *sig_w1, *sig_b1, *sigh_w, *sigh_b, *geo_w, *geo_b;
    const float *col_w0, *col_b0, *col_w1, *col_b1, *col_w2, *col_b2;
};
struct PackArgs {
    PackSrc e[kMaxK];
};

// decode a local index of an A-operand segment with NS k-steps per tile
__device__ __forceinline__ void decode_a(int li, int NS, int& t, int& s, int& i, int& h) {
    const int q = li & 3, lane = (li >> 2) & 63, tg = li >> 8;
    const int g = tg % (NS / 4);
    t = tg / (NS / 4);
    s = 4 * g + q;
    i = lane & 31;
    h = lane >> 5;
}

// ---- fp16x3 image (ACN_MLP_F16X3): the same layer regions [PK_W1, PK_WC3) hold, per layer, NT
// output tiles x NK k-steps (K = 16) x {hi, lo} A fragments of v_mfma_f32_32x32x16_f16, one
// 16-B [8 x f16] chunk per lane (lane l: row l & 31, half h = l >> 5, element e <-> k = 8h + e).
// The B operand of a layer is its input in the accumulator layout, so element e of half h at
// k-step s is input row xrow_acc(s, h, e) (cdna_hip_programming.md §3, "accumulator tile as the
// next MFMA's operand"); the A image is permuted to pair with it.  hi = f16(w),
// lo = f16(w - hi): the three products keep ~22 bits of every weight and activation.
__device__ __forceinline__ int xrow_acc(int s, int h, int e) {
    return 32 * (s >> 1) + 16 * (s & 1) + 8 * (e >> 2) + 4 * h + (e & 3);
}
// input = hash features: element e of k-step s of half h is feat[8s + e] of that half
__device__ __forceinline__ int xcol_feat(int s, int h, int e) {
    const int i = 8 * s + e;
    return ACN_LEVEL_PARITY ? 4 * (i >> 1) + 2 * h + (i & 1) : 16 * h + i;
}

__device__ float xweight(const PackSrc& p, int layer, int row, int s, int h, int e) {
    switch (layer) {
        case 0: return p.sig_w0[row * 32 + xcol_feat(s, h, e)];                 // sigma_trunk.0 (64, 32)
        case 1: return p.sig_w1[row * 64 + xrow_acc(s, h, e)];                  // sigma_trunk.1 (64, 64)
        case 2: {                                                               // [sigma_head; geo; 0] x 64
            const int k = xrow_acc(s, h, e);
            if (row == 0) return p.sigh_w[k];
            if (row <= kGeo) return p.geo_w[(row - 1) * 64 + k];
            return 0.0f;
        }
        case 3: {                                                               // color_mlp.0 on head rows
            const int r = xrow_acc(s, h, e);                                    // 0 sraw, 1..15 geo, 16..31 sh
            return r == 0 ? 0.0f : p.col_w0[row * 31 + (r - 1)];
        }
        default: return p.col_w1[row * 64 + xrow_acc(s, h, e)];                 // color_mlp.1 (64, 64)
    }
}

__device__ float pack_value_x3(const PackSrc& p, int idx) {
    int base, NK, layer;
    if (idx < PK_W2) { base = PK_W1; NK = 2; layer = 0; }
    else if (idx < PK_WH) { base = PK_W2; NK = 4; layer = 1; }
    else if (idx < PK_WC1) { base = PK_WH; NK = 4; layer = 2; }
    else if (idx < PK_WC2) { base = PK_WC1; NK = 2; layer = 3; }
    else { base = PK_WC2; NK = 4; layer = 4; }
    const int li = idx - base;
    const int q = li & 3, lane = (li >> 2) & 63, frag = li >> 8;
    const int part = frag & 1, ts = frag >> 1, s = ts % NK, T = ts / NK;
    const int row = 32 * T + (lane & 31), h = lane >> 5;
    uint32_t bits = 0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const float w = xweight(p, layer, row, s, h, 2 * q + u);
        const _Float16 hi = (_Float16)w;
        const _Float16 v = part ? (_Float16)(w - (float)hi) : hi;
        bits |= (uint32_t)__builtin_bit_cast(uint16_t, v) << (16 * u);
    }
    return __uint_as_float(bits);
}

__device__ float pack_value(const PackSrc& p, int idx) {
    int t, s, i, h;
    if (ACN_MLP_F16X3 && idx < PK_WC3) return pack_value_x3(p, idx);
    if (idx < PK_W2) {  // sigma_trunk.0 (64, 32): k = 16h + s
        decode_a(idx - PK_W1, 16, t, s, i, h);
        const int col = ACN_LEVEL_PARITY ? 4 * (s >> 1) + 2 * h + (s & 1) : 16 * h + s;
        return p.sig_w0[(i + 32 * t) * 32 + col];
    }
    if (idx < PK_WH) {  // sigma_trunk.1 (64, 64): k = rho(r, h) + 32 Tin, s = 16 Tin + r
        decode_a(idx - PK_W2, 32, t, s, i, h);
        return p.sig_w1[(i + 32 * t) * 64 + rho(s & 15, h) + 32 * (s >> 4)];
    }
    if (idx < PK_WC1) {  // [sigma_head; geo_head; 0] (32 rows) x 64
        decode_a(idx - PK_WH, 32, t, s, i, h);
        const int k = rho(s & 15, h) + 32 * (s >> 4);
        if (i == 0) return p.sigh_w[k];
        if (i <= kGeo) return p.geo_w[(i - 1) * 64 + k];
        return 0.0f;
    }
    if (idx < PK_WC2) {  // color_mlp.0 (64, 31) on head rows rho: 0 -> sigma_raw (weight 0),
        decode_a(idx - PK_WC1, 16, t, s, i, h);  // 1..15 geo, 16..31 SH  => column rho - 1
        const int r = rho(s, h);
        return r == 0 ? 0.0f : p.col_w0[(i + 32 * t) * 31 + (r - 1)];
    }
    if (idx < PK_WC3) {  // color_mlp.1 (64, 64)
        decode_a(idx - PK_WC2, 32, t, s, i, h);
        return p.col_w1[(i + 32 * t) * 64 + rho(s & 15, h) + 32 * (s >> 4)];
    }
    if (idx < PK_B) {  // color_mlp.2 (3, 64), VALU layout [h][c][T*16 + r]
        const int li = idx - PK_WC3;
        const int hh = li / 96, c = (li % 96) / 32, tr = li % 32;
        return p.col_w2[c * 64 + rho(tr & 15, hh) + 32 * (tr >> 4)];
    }
    if (idx < PK_BC3) {  // bias fragments [tile][h][r]
        const int li = idx - PK_B;
        const int tile = li / 32, hh = (li / 16) & 1, r = li & 15;
        const int row = rho(r, hh);
        switch (tile) {
            case 0: case 1: return p.sig_b0[row + 32 * (tile - 0)];
            case 2: case 3: return p.sig_b1[row + 32 * (tile - 2)];
            case 4: return row == 0 ? p.sigh_b[0] : (row <= kGeo ? p.geo_b[row - 1] : 0.0f);
            case 5: case 6: return p.col_b0[row + 32 * (tile - 5)];
            default: return p.col_b1[row + 32 * (tile - 7)];
        }
    }
    const int li = idx - PK_BC3;
    return li < 3 ? p.col_b2[li] : 0.0f;
}

__global__ void __launch_bounds__(256) pack_kernel(PackArgs args, int K, float* __restrict__ out) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = blockIdx.y;
    if (idx >= PK_FLOATS || k >= K) return;
    out[(size_t)k * PK_FLOATS + idx] = pack_value(args.e[k], idx);
}

// ------------------------------------------------------------------------------------------
// one 32-sample tile of one expert's field.  W: packed image (LDS or global, by inlining).
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

__device__ __forceinline__ f32x16 bias_frag(const float* W, int tile, int h) {
    const float* b = W + PK_B + (tile * 2 + h) * 16;
    const f32x4 a = ld4(b), c = ld4(b + 4), d = ld4(b + 8), e = ld4(b + 12);
    f32x16 v;
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = c[0]; v[5] = c[1]; v[6] = c[2]; v[7] = c[3];
    v[8] = d[0]; v[9] = d[1]; v[10] = d[2]; v[11] = d[3];
    v[12] = e[0]; v[13] = e[1]; v[14] = e[2]; v[15] = e[3];
    return v;
}

// a [tile][h][16] fragment image (per-ray folded colour bias)
__device__ __forceinline__ f32x16 bias_frag_at(const float* cb, int tile, int h) {
    const float* b = cb + (tile * 2 + h) * 16;
    const f32x4 a = ld4(b), c = ld4(b + 4), d = ld4(b + 8), e = ld4(b + 12);
    f32x16 v;
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = c[0]; v[5] = c[1]; v[6] = c[2]; v[7] = c[3];
    v[8] = d[0]; v[9] = d[1]; v[10] = d[2]; v[11] = d[3];
    v[12] = e[0]; v[13] = e[1]; v[14] = e[2]; v[15] = e[3];
    return v;
}

// ---- fp16x3 MLP building blocks
__device__ __forceinline__ f32x16 mfma16(const f16x8& a, const f16x8& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16x8 ldh8(const float* p) { return *reinterpret_cast<const f16x8*>(p); }

// split 8 fp32 values into hi = f16(x), lo = f16(x - hi)
__device__ __forceinline__ void split8(const float* x, f16x8& hi, f16x8& lo) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const _Float16 a = (_Float16)x[e];
        hi[e] = a;
        lo[e] = (_Float16)(x[e] - (float)a);
    }
}
// B fragments of a 64-row input held as two accumulator tiles: k-step s = 2 * tile + half-tile
__device__ __forceinline__ void split_acc2(const f32x16& a0, const f32x16& a1, f16x8 (&bh)[4], f16x8 (&bl)[4]) {
    float x[8];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const f32x16& a = (s >> 1) ? a1 : a0;
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = a[8 * (s & 1) + e];
        split8(x, bh[s], bl[s]);
    }
}

// out[T] = bias + W . X over NK k-steps of 16, three fp16 products per k-step (small terms first).
// The B fragments (bh, bl: v_cvt_pk_f16_f32 results) pass through the operand fence first (acn_device.h,
// DESIGN.md §4j): the round-4 pad at this point (ACN_X3_NOP) was placed by position, and the compiler still
// sank the last conversions past it into the k-step loop, 2 wait states before their MFMA.
// REV: k-steps in reverse order (colour layer 0 with per-lane SH: the SH k-step first, the order the per-ray
// fold accumulates in, so the result is bit-identical to fold_sh_bias + the folded layer)
template <int NT, int NK, bool REV = false>
__device__ __forceinline__ void layer_x3(const float* W, int seg, const float* bias_base, int bt, int lane, int h,
                                         f16x8 (&bh)[NK], f16x8 (&bl)[NK], f32x16 (&out)[NT],
                                         int nk_used = NK) {
    if (nk_used == 1) opnd_fence(bh[REV ? NK - 1 : 0], bl[REV ? NK - 1 : 0]);
    else opnd_fence_n<NK>(bh, bl);
#pragma unroll
    for (int T = 0; T < NT; ++T) out[T] = bias_frag_at(bias_base, bt + T, h);
#pragma unroll
    for (int si = 0; si < NK; ++si) {
        if (si >= nk_used) break;
        const int s = REV ? NK - 1 - si : si;
#pragma unroll
        for (int T = 0; T < NT; ++T) {
            const float* fp = W + seg + (((T * NK + s) * 2) * 64 + lane) * 4;
            const f16x8 ahi = ldh8(fp), alo = ldh8(fp + 256);
            out[T] = mfma16(alo, bh[s], out[T]);
            out[T] = mfma16(ahi, bl[s], out[T]);
            out[T] = mfma16(ahi, bh[s], out[T]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}


// Per-ray fold of colour layer 0's SH columns (meta_ngp.py:171-190: the direction, hence its SH
// encoding, is constant along a ray): cb[tile][h][r] = b_c0[row] + sum_m W_c0[row][15+m] sh[m]
// for row = rho(r, h) + 32 tile, computed once per ray with the 8 SH k-steps of the packed
// colour-layer-0 image (B = this half's SH rows, identical in every column).  Lanes j == 0 of
// each half store the fragment; the wave reads it back per tile instead of the plain bias.
__device__ __forceinline__ void fold_sh_bias(const float* W, const float (&shv)[8], int lane, float* cb) {
    const int h = lane >> 5;
    f32x16 q0 = bias_frag(W, BT_C1, h), q1 = bias_frag(W, BT_C1 + 1, h);
#if ACN_MLP_F16X3
    {   // k-step 1 of the colour-layer-0 image = head rows 16..31 = this half's SH values (shv)
        f16x8 sh_hi, sh_lo;
        split8(shv, sh_hi, sh_lo);
        opnd_fence(sh_hi, sh_lo);   // the fold had no pad at all
        const float* f0 = W + PK_WC1 + (((0 * 2 + 1) * 2) * 64 + lane) * 4;
        const float* f1 = W + PK_WC1 + (((1 * 2 + 1) * 2) * 64 + lane) * 4;
        const f16x8 h0 = ldh8(f0), l0 = ldh8(f0 + 256), h1 = ldh8(f1), l1 = ldh8(f1 + 256);
        q0 = mfma16(l0, sh_hi, q0); q0 = mfma16(h0, sh_lo, q0); q0 = mfma16(h0, sh_hi, q0);
        q1 = mfma16(l1, sh_hi, q1); q1 = mfma16(h1, sh_lo, q1); q1 = mfma16(h1, sh_hi, q1);
    }
#else
#pragma unroll
    for (int g = 2; g < 4; ++g) {
        const f32x4 w0 = ld4(W + PK_WC1 + ((0 * 4 + g) * 64 + lane) * 4);
        const f32x4 w1 = ld4(W + PK_WC1 + ((1 * 4 + g) * 64 + lane) * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            q0 = mfma32(w0[q], shv[4 * (g - 2) + q], q0);
            q1 = mfma32(w1[q], shv[4 * (g - 2) + q], q1);
        }
    }
#endif
    if ((lane & 31) == 0) {
        f32x4* d0 = reinterpret_cast<f32x4*>(cb + (0 * 2 + h) * 16);
        f32x4* d1 = reinterpret_cast<f32x4*>(cb + (1 * 2 + h) * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f32x4 a, b;
            a[0] = q0[4 * i]; a[1] = q0[4 * i + 1]; a[2] = q0[4 * i + 2]; a[3] = q0[4 * i + 3];
            b[0] = q1[4 * i]; b[1] = q1[4 * i + 1]; b[2] = q1[4 * i + 2]; b[3] = q1[4 * i + 3];
            d0[i] = a;
            d1[i] = b;
        }
    }
}

#ifndef ACN_FAST_VALU
#define ACN_FAST_VALU 0  // 1: one-instruction ReLU (v_max_f32), FMA lerps, reciprocal world->unit
#endif
__device__ __forceinline__ void relu16(f32x16& v) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
        // ACN_FAST_VALU: v_max_f32 (NaN -> 0 inside the fused MLP; a NaN sample still renders NaN
        // because its t / dist are NaN); else compare + select, NaN-propagating like torch.relu
        v[i] = ACN_FAST_VALU ? fmaxf(v[i], 0.0f) : (v[i] < 0.0f ? 0.0f : v[i]);
}

// 64 -> 64 layer: out tiles (o0, o1) = bias + W . [in0; in1].  A fragments are double
// buffered one 4-k-step group ahead; the scheduling barrier stops the compiler from hoisting
// every ds_read of the layer (64 VGPRs) above the MFMAs.
__device__ __forceinline__ void layer64x64(const float* W, int seg, int btile, int lane, int h,
                                           const f32x16& in0, const f32x16& in1, f32x16& o0, f32x16& o1) {
    o0 = bias_frag(W, btile, h);
    o1 = bias_frag(W, btile + 1, h);
    f32x4 n0 = ld4(W + seg + ((0 * 8 + 0) * 64 + lane) * 4);
    f32x4 n1 = ld4(W + seg + ((1 * 8 + 0) * 64 + lane) * 4);
#pragma unroll
    for (int gi = 0; gi < 8; ++gi) {
        const f32x4 a0 = n0, a1 = n1;
        if (gi < 7) {
            n0 = ld4(W + seg + ((0 * 8 + gi + 1) * 64 + lane) * 4);
            n1 = ld4(W + seg + ((1 * 8 + gi + 1) * 64 + lane) * 4);
        }
        const int tin = gi >> 2, g = gi & 3;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float b = tin ? in1[4 * g + q] : in0[4 * g + q];
            o0 = mfma32(a0[q], b, o0);
            o1 = mfma32(a1[q], b, o1);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

#ifndef ACN_HASH_DEPTH
// levels whose gathers are in flight together (1 = issue + wait per level).  3 with the depth tiles: C2 3.89 -> 3.92e9,
// C3 2.745 -> 2.755e9 against 2 (profiles/r06ag_hash_depth_ab.jsonl); 1 loses 3-4% on C3 / C4; 4 spills
#define ACN_HASH_DEPTH 3
#endif

#ifndef ACN_FIELD_CHECK
#define ACN_FIELD_CHECK 0
#endif
#if ACN_FIELD_CHECK
__device__ uint32_t g_fchk[3];   // diagnostic: tiles whose hash features differed between two evaluations, lane mask
constexpr unsigned kFchkMax = 4096;
__device__ float g_fchk_rec[40 * kFchkMax];
__device__ unsigned g_fchk_n;
#endif
#if ACN_DIAG_PHASE  // diagnostic build only: per-wave timestamp taken right after the hash phase
__shared__ uint64_t g_diag_stamp[16];
#endif

// level encoded by half h at gather step i (its features sit at feat[2i], feat[2i+1])
__device__ __forceinline__ int level_of(int i, int h) { return ACN_LEVEL_PARITY ? 2 * i + h : i + 8 * h; }

// Hash-encode this half's 8 levels (encodings.py:331-381) with the gathers of ACN_HASH_DEPTH
// levels in flight: level step i+D-1 is issued before step i is interpolated.
template <int INTERP>
__device__ __forceinline__ void hash_levels8(const ExpertMeta& em, int log2T, int h, float x0, float x1, float x2,
                                             float (&feat)[16]) {
    constexpr int D = INTERP == 2 ? 1 : ACN_HASH_DEPTH;   // Smoothstep: one level in flight (its spill-free depth)
    const uint32_t mask = (uint32_t)((1ull << log2T) - 1ull);
#if ACN_XPAIR == 2
    if (INTERP != 0) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)em.table, (short)0, (int)(uint32_t)((16ull << log2T) * 8ull), 0x00020000);
        HashPendingX px[D];
        auto issue_x = [&](int i, HashPendingX& pp) {
            const int lv = level_of(i, h);
            const float res = (float)(ACN_LEVEL_PARITY ? (h ? em.res[2 * i + 1] : em.res[2 * i])
                                                       : (h ? em.res[8 + i] : em.res[i]));
            hash_issue_x<INTERP>(rs, (uint32_t)lv << (log2T + 3), x0 * res, x1 * res, x2 * res, mask, pp);
        };
#pragma unroll
        for (int l = 0; l < D - 1; ++l) issue_x(l, px[l]);
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            if (l + D - 1 < 8) issue_x(l + D - 1, px[(l + D - 1) % D]);
            __builtin_amdgcn_sched_barrier(0);
            hash_finish_x<INTERP>(px[l % D], feat[2 * l], feat[2 * l + 1]);
            __builtin_amdgcn_sched_barrier(0);
        }
        return;
    }
#endif
    HashPending pend[D];
#if ACN_XPAIR == 3
    // the expert's 16 level tables (F = 2) in one buffer resource: level lv starts at byte lv << (log2T + 3)
    const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
        (void*)em.table, (short)0, (int)(uint32_t)((16ull << log2T) * 8ull), 0x00020000);
#endif
    auto issue = [&](int i, HashPending& pp) {
        const int lv = level_of(i, h);
        const float res = (float)(ACN_LEVEL_PARITY ? (h ? em.res[2 * i + 1] : em.res[2 * i])
                                                   : (h ? em.res[8 + i] : em.res[i]));
#if ACN_XPAIR == 3
        hash_issue_b<INTERP>(rsb, (uint32_t)lv << (log2T + 3), x0 * res, x1 * res, x2 * res, mask, pp);
        return;
#endif
        const float2* tl = reinterpret_cast<const float2*>(em.table) + ((size_t)lv << log2T);
        if (i >= ACN_FINE_FROM)
            hash_issue<INTERP, ACN_FINE_POL>(tl, x0 * res, x1 * res, x2 * res, mask, pp);
        else
            hash_issue<INTERP, 0>(tl, x0 * res, x1 * res, x2 * res, mask, pp);
    };
#pragma unroll
    for (int l = 0; l < D - 1; ++l) issue(l, pend[l]);
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        if (l + D - 1 < 8) issue(l + D - 1, pend[(l + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        hash_finish<INTERP, ACN_FAST_VALU != 0>(pend[l % D], feat[2 * l], feat[2 * l + 1]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Field of one expert on this lane's sample (x world point, shv = this half's SH rows).
// Returns rgb (after sigmoid) on every lane and sigma_raw on every lane.
// FOLD: the colour MLP's SH columns + bias were folded per ray into cb (LDS, [tile][h][16],
// see fold_sh_bias): colour layer 0 then only runs the 8 k-steps of the [sigma_raw, geo] rows.
// SHFIRST (with FOLD false): colour layer 0 runs unfolded on per-lane SH rows, the SH k-step before the
// [sigma_raw, geo] one -- bit for bit the folded result of a ray whose lanes all carry its SH (the render of
// compacted samples of several rays, ep_field_kernel)
template <int INTERP, bool FOLD, bool SHFIRST = false, bool FCHK = false>
__device__ __forceinline__ void field_tile(const float* W, const ExpertMeta& em, int log2T, float px, float py,
                                           float pz, const float (&shv)[8], const float* cb, int lane, float& rr,
                                           float& rg, float& rb, float& sraw) {
    W = W + opaque_s(0);
    const int h = opaque_v(lane >> 5);
    // _world_to_unit (meta_ngp.py:155-158)
    const float eps = 1e-6f, hi = 1.0f - 1e-6f;
#if ACN_FAST_VALU  // multiply by the host-computed reciprocal extent (<= 1 ulp from the division)
    const float x0 = clamp_nan((px - em.amin[0]) * em.rext[0], eps, hi);
    const float x1 = clamp_nan((py - em.amin[1]) * em.rext[1], eps, hi);
    const float x2 = clamp_nan((pz - em.amin[2]) * em.rext[2], eps, hi);
#else
    const float x0 = clamp_nan((px - em.amin[0]) / em.ext[0], eps, hi);
    const float x1 = clamp_nan((py - em.amin[1]) / em.ext[1], eps, hi);
    const float x2 = clamp_nan((pz - em.amin[2]) / em.ext[2], eps, hi);
#endif
    float feat[16];
#if ACN_DIAG_NOHASH  // diagnostic build only: no gathers
#pragma unroll
    for (int i = 0; i < 16; ++i) feat[i] = x0 * (float)(i + 1) - x1 + x2 * (float)i;
#else
    hash_levels8<INTERP>(em, log2T, h, x0, x1, x2, feat);
#endif
#if ACN_FIELD_CHECK  // diagnostic build only: the hash encoding evaluated twice; differing lanes are counted
    if constexpr (FCHK) {
        float f2[16];
        hash_levels8<INTERP>(em, log2T, h, x0, x1, x2, f2);
        bool bad = false;
#pragma unroll
        for (int i = 0; i < 16; ++i) bad |= __float_as_uint(f2[i]) != __float_as_uint(feat[i]);
        const uint64_t bm = __ballot(bad);
        if (bm && lane == 0) {
            atomicAdd(&g_fchk[0], 1u);
            atomicOr(&g_fchk[1], (uint32_t)bm);
            atomicOr(&g_fchk[2], (uint32_t)(bm >> 32));
        }
        if (bad) {   // per differing lane: lane, table pointer, unit point, both feature vectors
            const unsigned q = atomicAdd(&g_fchk_n, 1u);
            if (q < kFchkMax) {
                float* o = g_fchk_rec + 40 * q;
                const uint64_t tp = (uint64_t)(uintptr_t)em.table;
                o[0] = __uint_as_float((uint32_t)lane); o[1] = __uint_as_float((uint32_t)tp);
                o[2] = __uint_as_float((uint32_t)(tp >> 32)); o[3] = x0; o[4] = x1; o[5] = x2;
                o[6] = __uint_as_float((uint32_t)log2T); o[7] = __uint_as_float((uint32_t)h);
#pragma unroll
                for (int i = 0; i < 16; ++i) { o[8 + i] = feat[i]; o[24 + i] = f2[i]; }
            }
        }
    }
#endif
#if ACN_DIAG_PHASE
    {
        const uint64_t tnow = __builtin_amdgcn_s_memtime();
        if (lane == 0) g_diag_stamp[threadIdx.x >> 6] = tnow;
    }
#endif
#if ACN_DIAG_NOMLP  // diagnostic build only: no MLP
    {
        float a = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; ++i) a += feat[i];
        rr = a; rg = feat[1]; rb = feat[2]; sraw = __shfl(feat[3], lane & 31);
        return;
    }
#endif
#if ACN_MLP_F16X3
    f32x16 d0, d1;
    {
        // sigma_trunk.0: 32 -> 64 (ReLU)
        f16x8 fh[2], fl[2];
        split8(feat, fh[0], fl[0]);
        split8(feat + 8, fh[1], fl[1]);
        f32x16 a[2];
        layer_x3<2, 2>(W, PK_W1, W + PK_B, BT_L1, lane, h, fh, fl, a);
        relu16(a[0]);
        relu16(a[1]);
        // sigma_trunk.1: 64 -> 64 (ReLU)
        f16x8 bh[4], bl[4];
        split_acc2(a[0], a[1], bh, bl);
        f32x16 b[2];
        layer_x3<2, 4>(W, PK_W2, W + PK_B, BT_L2, lane, h, bh, bl, b);
        relu16(b[0]);
        relu16(b[1]);
        // heads: rows 0 sigma_head, 1..15 geo_head (16..31 carry SH when not folded)
        split_acc2(b[0], b[1], bh, bl);
        f32x16 hd[1];
        layer_x3<1, 4>(W, PK_WH, W + PK_B, BT_H, lane, h, bh, bl, hd);
        if (!FOLD) {
#pragma unroll
            for (int r = 8; r < 16; ++r) hd[0][r] = shv[r - 8];
        }
        sraw = __shfl(hd[0][0], lane & 31);
        // color_mlp.0: [geo(15), sh(16)] -> 64 (ReLU); FOLD: bias from cb, only k-step 0 (rows 0..15)
        f16x8 ch[2], cl[2];
        {
            float x[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = hd[0][e];
            split8(x, ch[0], cl[0]);
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = hd[0][8 + e];
            split8(x, ch[1], cl[1]);
        }
        f32x16 c[2];
        if (FOLD) layer_x3<2, 2>(W, PK_WC1, cb, 0, lane, h, ch, cl, c, 1);   // per-ray folded bias
        else if (SHFIRST) layer_x3<2, 2, true>(W, PK_WC1, W + PK_B, BT_C1, lane, h, ch, cl, c);
        else layer_x3<2, 2>(W, PK_WC1, W + PK_B, BT_C1, lane, h, ch, cl, c);
        relu16(c[0]);
        relu16(c[1]);
        // color_mlp.1: 64 -> 64 (ReLU)
        split_acc2(c[0], c[1], bh, bl);
        f32x16 dd[2];
        layer_x3<2, 4>(W, PK_WC2, W + PK_B, BT_C2, lane, h, bh, bl, dd);
        d0 = dd[0];
        d1 = dd[1];
        relu16(d0);
        relu16(d1);
    }
#else
    // sigma_trunk.0: 32 -> 64 (ReLU)
    f32x16 a0 = bias_frag(W, BT_L1, h), a1 = bias_frag(W, BT_L1 + 1, h);
    {
        f32x4 n0 = ld4(W + PK_W1 + ((0 * 4 + 0) * 64 + lane) * 4);
        f32x4 n1 = ld4(W + PK_W1 + ((1 * 4 + 0) * 64 + lane) * 4);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 w0 = n0, w1 = n1;
            if (g < 3) {
                n0 = ld4(W + PK_W1 + ((0 * 4 + g + 1) * 64 + lane) * 4);
                n1 = ld4(W + PK_W1 + ((1 * 4 + g + 1) * 64 + lane) * 4);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a0 = mfma32(w0[q], feat[4 * g + q], a0);
                a1 = mfma32(w1[q], feat[4 * g + q], a1);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    relu16(a0);
    relu16(a1);
    // sigma_trunk.1: 64 -> 64 (ReLU)
    f32x16 b0, b1;
    layer64x64(W, PK_W2, BT_L2, lane, h, a0, a1, b0, b1);
    relu16(b0);
    relu16(b1);
    // heads: rows 0 sigma_head, 1..15 geo_head; rows 16..31 carry the SH features through
    // (zero weights, accumulator initialised with SH): the colour MLP input [geo, sh].
    f32x16 hd = bias_frag(W, BT_H, h);
    if (!FOLD) {
#pragma unroll
        for (int r = 8; r < 16; ++r) hd[r] = shv[r - 8];
    }
    {
        f32x4 n = ld4(W + PK_WH + (0 * 64 + lane) * 4);
#pragma unroll
        for (int gi = 0; gi < 8; ++gi) {
            const f32x4 w = n;
            if (gi < 7) n = ld4(W + PK_WH + ((gi + 1) * 64 + lane) * 4);
            const int tin = gi >> 2, g = gi & 3;
#pragma unroll
            for (int q = 0; q < 4; ++q) hd = mfma32(w[q], tin ? b1[4 * g + q] : b0[4 * g + q], hd);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // sigma_raw = row 0, held by lane j of half 0
    sraw = __shfl(hd[0], lane & 31);
    // color_mlp.0: [geo(15), sh(16)] -> 64 (ReLU); with FOLD only the 8 k-steps of rows 0..15
    f32x16 c0, c1;
    if (FOLD) {
        c0 = bias_frag_at(cb, 0, h);
        c1 = bias_frag_at(cb, 1, h);
    } else {
        c0 = bias_frag(W, BT_C1, h);
        c1 = bias_frag(W, BT_C1 + 1, h);
    }
    {
        constexpr int NG = FOLD ? 2 : 4;
        constexpr bool RV = SHFIRST && !FOLD;   // groups 2, 3 (SH rows) first: the fold's order
        auto gq = [](int i) { return RV ? (i + 2) & 3 : i; };
        f32x4 n0 = ld4(W + PK_WC1 + ((0 * 4 + gq(0)) * 64 + lane) * 4);
        f32x4 n1 = ld4(W + PK_WC1 + ((1 * 4 + gq(0)) * 64 + lane) * 4);
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            const int g = gq(gi);
            const f32x4 w0 = n0, w1 = n1;
            if (gi < NG - 1) {
                n0 = ld4(W + PK_WC1 + ((0 * 4 + gq(gi + 1)) * 64 + lane) * 4);
                n1 = ld4(W + PK_WC1 + ((1 * 4 + gq(gi + 1)) * 64 + lane) * 4);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c0 = mfma32(w0[q], hd[4 * g + q], c0);
                c1 = mfma32(w1[q], hd[4 * g + q], c1);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    relu16(c0);
    relu16(c1);
    // color_mlp.1: 64 -> 64 (ReLU)
    f32x16 d0, d1;
    layer64x64(W, PK_WC2, BT_C2, lane, h, c0, c1, d0, d1);
    relu16(d0);
    relu16(d1);
#endif
    // color_mlp.2: 64 -> 3 on the VALU (a 3-row MFMA tile would waste 29/32 of the pipe):
    // each half dots its 32 features, the halves are summed with a cross-half swap.
    const float* w3 = W + PK_WC3 + h * 96;
    float o[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float acc = 0.0f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 wa = ld4(w3 + c * 32 + 4 * g);
            const f32x4 wb = ld4(w3 + c * 32 + 16 + 4 * g);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                acc = fmaf(wa[q], d0[4 * g + q], acc);
                acc = fmaf(wb[q], d1[4 * g + q], acc);
            }
        }
        o[c] = acc;
    }
    const f32x4 b3 = ld4(W + PK_BC3);
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = (o[c] + __shfl_xor(o[c], 32)) + b3[c];
    rr = sigmoidf_(o[0]);
    rg = sigmoidf_(o[1]);
    rb = sigmoidf_(o[2]);
}

// Container forward of this lane's sample over all experts (meta_container.py:300-343):
// soft: y = sum_k (y_k * w_k) accumulated in expert order from zero (index_add_); hard: copy.
// FOLD: cb points at this wave's per-expert folded colour biases ([k][64] floats in LDS) and
// *folded is the wave-uniform mask of experts already folded for the current ray.
template <int INTERP, int ROUTE, bool FOLD>
__device__ __forceinline__ void container_tile(const FieldCfg& cfg, const float* Wbase, float px, float py, float pz,
                                               const float (&shv)[8], float* cb, uint32_t* folded, int lane,
                                               float& yr, float& yg, float& yb, float& ys) {
    if (ROUTE == 0) {
        if (FOLD && !(*folded & 1u)) {
            fold_sh_bias(Wbase, shv, lane, cb);
            *folded |= 1u;
        }
        field_tile<INTERP, FOLD>(Wbase, cfg.ex[0], cfg.log2T, px, py, pz, shv, cb, lane, yr, yg, yb, ys);
        ys = trunc_exp(ys);
        return;
    }
    const RouteState st = route_prep<ROUTE>(cfg, px, py, pz);
    yr = yg = yb = ys = 0.0f;
    for (int k = 0; k < cfg.K; ++k) {
        const float wk = (ROUTE == 1) ? route_weight(cfg, st, k, px, py, pz) : 0.0f;
        const bool need = (ROUTE == 1) ? (wk > 0.0f) : (st.hard == k);
        if (__ballot(need) == 0ull) continue;  // wave-uniform skip of experts no sample needs
        const float* Wk = Wbase + (size_t)k * PK_FLOATS;
        float* cbk = FOLD ? cb + k * 64 : nullptr;
        if (FOLD && !((*folded >> k) & 1u)) {
            fold_sh_bias(Wk, shv, lane, cbk);
            *folded |= 1u << k;
        }
        float r, g, b, s;
        field_tile<INTERP, FOLD>(Wk, cfg.ex[k], cfg.log2T, px, py, pz, shv, cbk, lane, r, g, b, s);
        s = trunc_exp(s);
        if (need) {
            if (ROUTE == 1) {
                yr = yr + r * wk;
                yg = yg + g * wk;
                yb = yb + b * wk;
                ys = ys + s * wk;
            } else {
                yr = r; yg = g; yb = b; ys = s;
            }
        }
    }
}

// SH rows of the head tile held by half h: rows 16+4h..19+4h and 24+4h..27+4h
__device__ __forceinline__ void sh_rows_for_half(const float (&sh)[16], int h, float (&shv)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        shv[i] = h ? sh[4 + i] : sh[i];
        shv[4 + i] = h ? sh[12 + i] : sh[8 + i];
    }
}

// ------------------------------------------------------------------------------------------
template <int KL>
__device__ __forceinline__ void stage_weights(float* smem, const float* __restrict__ packed) {
    const f32x4* src = reinterpret_cast<const f32x4*>(packed);
    f32x4* dst = reinterpret_cast<f32x4*>(smem);
    for (int i = threadIdx.x; i < KL * PK_FLOATS / 4; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

struct FieldParams {
    const float* x;
    int64_t M, ld;
    const float* packed;
    float* out;
};

// acn_field_fwd: 32 points per wave-tile, grid-stride over tiles.
template <int INTERP, int KL, int ROUTE>
__global__ void __launch_bounds__(1024, 4) field_kernel(FieldCfg cfg, FieldParams p) {
    __shared__ __attribute__((aligned(16))) float smem[(KL > 0 ? KL : 1) * PK_FLOATS];
    const float* W = p.packed;
    if (KL > 0) {
        stage_weights<KL>(smem, p.packed);
        W = smem;
    }
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t ntiles = (p.M + 31) / 32;
    for (int64_t tile = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave; tile < ntiles; tile += nw) {
        const int64_t m = tile * 32 + j;
        const int64_t mc = m < p.M ? m : p.M - 1;
        const float* xr = p.x + mc * p.ld;
        const float px = xr[0], py = xr[1], pz = xr[2];
        float sh[16], shv[8];
        dir_sh(xr[3], xr[4], xr[5], sh);
        sh_rows_for_half(sh, h, shv);
        float yr, yg, yb, ys;
        container_tile<INTERP, ROUTE, false>(cfg, W, px, py, pz, shv, nullptr, nullptr, lane, yr, yg, yb, ys);
        if (h == 0 && m < p.M) {
            f32x4 v;
            v[0] = yr; v[1] = yg; v[2] = yb; v[3] = ys;
            *reinterpret_cast<f32x4*>(p.out + 4 * m) = v;
        }
    }
}

// ------------------------------------------------------------------------------------------
// compositing of one 32-sample tile (ray_rendering.py:137-159).  Transmittance is carried in
// double (torch's CPU cumprod accumulates in double); the weighted sums are kept as per-lane
// float partials across tiles and reduced across lanes once per ray, in double.
struct RayAcc {
    double T;
    float r, g, b, d, a;
};

#ifndef ACN_COMPOSITE_DPP
#define ACN_COMPOSITE_DPP 1
#endif
// a double moved by one DPP control (both 32-bit halves); lanes without a source (or outside ROWMASK)
// get the multiplicative identity 1.0
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROWMASK, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0x3ff00000, (int)(uint32_t)(b >> 32), CTRL, ROWMASK, 0xF, false);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// sum over the 32 lanes of half 0 (both halves hold the same per-sample partials): DPP inside each
// 16-lane row, then rows 0 and 1 through readlanes (a wave-uniform result)
template <int CTRL>
__device__ __forceinline__ double dpp_add_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
    return v + __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double wave32_sum(double v) {
#if ACN_COMPOSITE_DPP
    v = dpp_add_f64<0xB1>(v);   // quad_perm [1,0,3,2]
    v = dpp_add_f64<0x4E>(v);   // quad_perm [2,3,0,1]
    v = dpp_add_f64<0x141>(v);  // row_half_mirror
    v = dpp_add_f64<0x140>(v);  // row_mirror
    return lane_f64(v, 0) + lane_f64(v, 16);
#else
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) v += __shfl_xor(v, off, 32);
    return v;
#endif
}

__device__ __forceinline__ void composite_tile(RayAcc& acc, bool valid, float cr, float cg, float cb, float sig,
                                               float t, float dist, int j, float* wout) {
    // rgb.clamp(0,1), sigma.clamp_min(0) (* sigma_scale) are applied by the caller
    dist = clamp_min_nan(dist, 1e-4f);
    float alpha = 1.0f - expf(-sig * dist);
    alpha = clamp_nan(alpha, 0.0f, (float)(1.0 - 1e-7));
    float x = (1.0f - alpha) + 1e-10f;
    if (!valid) { x = 1.0f; alpha = 0.0f; }
    double incl = (double)x;
#if ACN_COMPOSITE_DPP
    // inclusive product over the 32 samples of each lane half on DPP (no LDS): row_shr 1/2/4/8 inside
    // each 16-lane row, then row_bcast:15 carries row 0's (row 2's) product into row 1 (row 3); lanes
    // without a source keep the identity 1.0.  Both halves hold the same samples, so lane 31 = lane 63.
    incl *= dpp_f64<0x111, 0xF>(incl);
    incl *= dpp_f64<0x112, 0xF>(incl);
    incl *= dpp_f64<0x114, 0xF>(incl);
    incl *= dpp_f64<0x118, 0xF>(incl);
    incl *= dpp_f64<0x142, 0xA>(incl);
    double excl = dpp_f64<0x138, 0xF>(incl);  // wave_shr:1
    if (j == 0) excl = 1.0;
#else
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) {
        const double y = __shfl_up(incl, off, 32);
        if (j >= off) incl *= y;
    }
    double excl = __shfl_up(incl, 1, 32);
    if (j == 0) excl = 1.0;
#endif
    const float Ts = (float)(acc.T * excl);
    const float w = alpha * Ts;
    if (wout) *wout = w;
    if (valid) {
        acc.r += w * cr;
        acc.g += w * cg;
        acc.b += w * cb;
        acc.d += w * t;
        acc.a += w;
    }
#if ACN_COMPOSITE_DPP
    acc.T = acc.T * lane_f64(incl, 31);
#else
    acc.T = acc.T * __shfl(incl, 31, 32);
#endif
}

__device__ __forceinline__ void finish_ray(const RayAcc& acc, float& r, float& g, float& b, float& d, float& a) {
    r = (float)wave32_sum((double)acc.r);
    g = (float)wave32_sum((double)acc.g);
    b = (float)wave32_sum((double)acc.b);
    d = (float)wave32_sum((double)acc.d);
    a = (float)wave32_sum((double)acc.a);
}

struct BgArgs {
    int32_t mode, hidden;
    float color[3];
    const float *w1, *b1, *w2, *b2;
};

// background_color (meta_container.py:360-367): F.normalize -> SH(4) -> Linear ReLU -> Linear Sigmoid
__device__ __forceinline__ void background(const BgArgs& bg, float dx, float dy, float dz, int lane, float (&out)[3]) {
    if (bg.mode == ACN_BG_CONST) { out[0] = bg.color[0]; out[1] = bg.color[1]; out[2] = bg.color[2]; return; }
    if (bg.mode != ACN_BG_MLP) { out[0] = out[1] = out[2] = 0.0f; return; }
    const float n = clamp_min_nan(norm3(dx, dy, dz), 1e-12f);
    float sh[16];
    sh_encode<3>(dx / n, dy / n, dz / n, sh, __int_as_float(opaque_s(0)));   // +0.0f, opaque (acn_device.h)
    float hv = 0.0f;
    // an opaque lane index: the per-lane weight addresses below are formed here, per call, not hoisted out of
    // the callers' ray loops by LICM (four 64-bit addresses held across render_ws_kernel's loop spilled)
    lane = opaque_v(lane);
    if (lane < bg.hidden) {
        float s = 0.0f;
        for (int k = 0; k < 16; ++k) s = fmaf(sh[k], bg.w1[lane * 16 + k], s);
        hv = s + bg.b1[lane];
        hv = hv < 0.0f ? 0.0f : hv;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float v = lane < bg.hidden ? hv * bg.w2[c * bg.hidden + lane] : 0.0f;
#if ACN_COMPOSITE_DPP
        v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
        v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
        v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
        v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
        v = (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
            (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
#else
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
#endif
        out[c] = sigmoidf_(v + bg.b2[c]);
    }
}

struct RenderParams {
    const float* rays;
    int64_t N;
    int32_t S;
    const float* jitter;
    const float* packed;
    float sigma_scale, tau;
    float *rgb, *depth, *weights, *acc;
    const int32_t* order;  // optional visiting order (ray_order_kernel); NULL = rays in the given order
    const int32_t* norder; // render_slots_kernel: device count of `order` entries (the multi-expert rays of the
                           // split routed render); NULL = N
};

#ifndef ACN_SHFOLD
#define ACN_SHFOLD 1
#endif

// t of sample i without jitter, branch-free (same roundings as lin01/tlin)
__device__ __forceinline__ float tlin_sel(float near, float far, int i, int S, float step) {
    const float a = fmaf(step, (float)i, 0.0f);
    const float b = fmaf(-step, (float)(S - 1 - i), 1.0f);
    const float u = i < S / 2 ? a : b;
    return near * (1.0f - u) + far * u;
}

#ifndef ACN_SLOTS_PROF
#define ACN_SLOTS_PROF 0   // diagnostic build: per-ray section stamps of render_slots_kernel (acn_debug_slprof_fetch)
#endif
#if ACN_SLOTS_PROF
constexpr int kSlProfRays = 1 << 20;
__device__ unsigned long long g_slprof[kSlProfRays * 6];
#define SL_MARK(ray, i) if (lane == 0 && (ray) < kSlProfRays) g_slprof[(ray) * 6 + (i)] = wall_clock64();
#else
#define SL_MARK(ray, i)
#endif
// One ray, front to back in 32-sample tiles: t-values -> field(px, py, pz, shv, folded, y...) ->
// volume_render conditioning -> compositing -> background -> outputs.  `field` evaluates the
// (routed) container for this lane's sample; it is a template callable so the single-expert, the
// LDS-resident and the slot-staged kernels share this body.
template <class FieldFn>
__device__ __forceinline__ void render_ray(const RenderParams& p, const BgArgs& bg, int64_t ray, int lane, float step,
                                           FieldFn&& field) {
    const int j = lane & 31, h = lane >> 5;
    const int S = p.S;
#if ACN_DIAG_CLOCK || ACN_DIAG_PHASE
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#endif
#if ACN_DIAG_CLOCK  // diagnostic build only: depth[ray] <- in-kernel shader clock (MHz) over the ray
    const uint64_t diag_t0 = __builtin_amdgcn_s_memtime(), diag_r0 = __builtin_amdgcn_s_memrealtime();
#endif
#if ACN_DIAG_WAVETIME  // diagnostic build only: rgb[ray] <- bit patterns of (start, end) 100-MHz stamps, HW ids
    const uint32_t diag_w0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
    const float* rp = p.rays + ray * 8;
    const float ox = rp[0], oy = rp[1], oz = rp[2], dx = rp[3], dy = rp[4], dz = rp[5];
    const float near = rp[6], far = rp[7];
    const float* jit = p.jitter ? p.jitter + ray * S : nullptr;
    float sh[16], shv[8];
    dir_sh(dx, dy, dz, sh);
    sh_rows_for_half(sh, h, shv);
    uint32_t folded = 0u;
#if ACN_DIAG_PHASE
    uint32_t dg_hash = 0u, dg_mlp = 0u, dg_comp = 0u, dg_n = 0u;
#endif
    RayAcc acc{1.0, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    int s0 = 0;
    for (; s0 < S; s0 += 32) {
        const int s = s0 + j;
        const bool valid = s < S;
        const int sc = valid ? s : S - 1;
        float t, dist;
        if (!jit) {  // eval: dist = t[i+1] - t[i], the last one repeated (ray_rendering.py:144-145)
            const int i0 = sc < S - 1 ? sc : S - 2;
            const float ta = tlin_sel(near, far, i0, S, step), tb = tlin_sel(near, far, i0 + 1, S, step);
            t = sc < S - 1 ? ta : tb;
            dist = tb - ta;
        } else {
            t = tval(near, far, sc, S, jit);
            const float tn = (sc < S - 1) ? tval(near, far, sc + 1, S, jit) : t;
            const float tp = (sc == S - 1 && S > 1) ? tval(near, far, sc - 1, S, jit) : t;
            dist = (sc < S - 1) ? (tn - t) : (t - tp);
        }
        const float px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;
        float yr, yg, yb, ys;
#if ACN_DIAG_PHASE
        const uint64_t dA = __builtin_amdgcn_s_memtime();
#endif
        field(sc, px, py, pz, shv, folded, yr, yg, yb, ys);
        if (s0 == 0) { SL_MARK(ray, 3) }
#if ACN_DIAG_PHASE
        const uint64_t dB = __builtin_amdgcn_s_memtime();
        const uint32_t dS = __builtin_amdgcn_readfirstlane((uint32_t)g_diag_stamp[wave]);
        dg_hash += dS - (uint32_t)dA;
        dg_mlp += (uint32_t)dB - dS;
        dg_n += 1u;
#endif
        // volume_render input conditioning (:140-143)
        yr = clamp_nan(yr, 0.0f, 1.0f);
        yg = clamp_nan(yg, 0.0f, 1.0f);
        yb = clamp_nan(yb, 0.0f, 1.0f);
        float sig = clamp_min_nan(ys, 0.0f);
        if (p.sigma_scale != 1.0f) sig = sig * p.sigma_scale;
        float wv;
        composite_tile(acc, valid, yr, yg, yb, sig, t, dist, j, &wv);
        if (p.weights && valid && h == 0) p.weights[ray * S + s] = wv;
#if ACN_DIAG_PHASE
        dg_comp += (uint32_t)__builtin_amdgcn_s_memtime() - (uint32_t)dB;
#endif
        const int stop = __builtin_amdgcn_readfirstlane((int)(acc.T < (double)p.tau));
        if (stop) { s0 += 32; break; }
    }
    SL_MARK(ray, 4)
    if (p.weights && h == 0)  // samples skipped by early termination carry zero weight
        for (int s = s0 + j; s < S; s += 32) p.weights[ray * S + s] = 0.0f;
    float bgc[3];
    background(bg, dx, dy, dz, lane, bgc);
    float r, g, b, dd, a;
    finish_ray(acc, r, g, b, dd, a);
    if (lane == 0) {
        if (bg.mode != ACN_BG_NONE) {
            const float om = 1.0f - a;
            r = r + om * bgc[0];
            g = g + om * bgc[1];
            b = b + om * bgc[2];
        }
        p.rgb[ray * 3 + 0] = r;
        p.rgb[ray * 3 + 1] = g;
        p.rgb[ray * 3 + 2] = b;
        p.depth[ray] = dd;
        p.acc[ray] = a;
#if ACN_DIAG_CLOCK
        p.depth[ray] = (float)(__builtin_amdgcn_s_memtime() - diag_t0) * 100.0f /
                       (float)(__builtin_amdgcn_s_memrealtime() - diag_r0);
#endif
#if ACN_DIAG_WAVETIME
        p.rgb[ray * 3 + 0] = __int_as_float((int)diag_w0);
        p.rgb[ray * 3 + 1] = __int_as_float((int)(uint32_t)__builtin_amdgcn_s_memrealtime());
        p.rgb[ray * 3 + 2] = __int_as_float((int)((__builtin_amdgcn_s_getreg((31 << 11) | 4) & 0xffffu) |
                                                   (__builtin_amdgcn_s_getreg((31 << 11) | 20) << 16)));
#endif
#if ACN_DIAG_PHASE  // cycles per tile: depth <- hash phase, acc <- MLP phase, rgb.r <- compositing
        p.depth[ray] = (float)dg_hash / (float)dg_n;
        p.acc[ray] = (float)dg_mlp / (float)dg_n;
        p.rgb[ray * 3] = (float)dg_comp / (float)dg_n;
#endif
    }
}

template <int INTERP, int KL, int ROUTE>
__global__ void __launch_bounds__(1024, 4) render_kernel(FieldCfg cfg, BgArgs bg, RenderParams p) {
    constexpr bool FOLD = ACN_SHFOLD != 0;
    constexpr int KF = ROUTE == 0 ? 1 : (KL == 2 ? 2 : kMaxK);  // experts a ray may fold
    __shared__ __attribute__((aligned(16))) float smem[(KL > 0 ? KL : 1) * PK_FLOATS];
    __shared__ __attribute__((aligned(16))) float cbuf[FOLD ? 16 * KF * 64 : 4];
    const float* W = p.packed;
    if (KL > 0) {
        stage_weights<KL>(smem, p.packed);
        W = smem;
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably uniform: ray data in SGPRs
    float* cb = FOLD ? cbuf + wave * KF * 64 : nullptr;
    const float step = 1.0f / (float)(p.S - 1);
    // XCD bands: workgroups are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), so
    // when the grid is a multiple of 8, XCD x walks the x-th contiguous eighth of the visiting order.
    // With a spatially coherent order (ray_order_kernel, or pixel-ordered full frames) each XCD's
    // 4 MB L2 then serves the hash cells of one image region instead of the whole frame.
    const int64_t wpb = blockDim.x >> 6;
    int64_t pos, hi, stride;
    if ((gridDim.x & 7) == 0) {
        const int64_t chunk = (p.N + 7) >> 3;
        const int64_t lo = min(p.N, (int64_t)(blockIdx.x & 7) * chunk);
        hi = min(p.N, lo + chunk);
        pos = lo + (int64_t)(blockIdx.x >> 3) * wpb + wave;
        stride = (int64_t)(gridDim.x >> 3) * wpb;
    } else {
        hi = p.N;
        pos = (int64_t)blockIdx.x * wpb + wave;
        stride = (int64_t)gridDim.x * wpb;
    }
    for (; pos < hi; pos += stride) {
        const int64_t ray = p.order ? (int64_t)__builtin_amdgcn_readfirstlane(p.order[pos]) : pos;
        render_ray(p, bg, ray, lane, step,
                   [&](int, float px, float py, float pz, const float (&shv)[8], uint32_t& folded, float& yr, float& yg,
                       float& yb, float& ys) {
                       container_tile<INTERP, ROUTE, FOLD>(cfg, W, px, py, pz, shv, cb, &folded, lane, yr, yg, yb, ys);
                   });
    }
}

// ------------------------------------------------------------------------------------------
// Single-expert render with the workgroup's field tiles shared (render_ws_kernel, the C2 path when there is no
// early termination).  render_kernel gives every wave one ray, and all 4096 waves of a C2 batch are resident
// at once, so a CU runs until its slowest ray ends: the per-wave timeline (tools/micro/wave_times.py) shows rays
// of 190-295 us in a 297 us launch, 12 of 16 waves resident on average.  Here the 16 rays of a round are
// split into their 32-sample tiles (the field's MFMA unit), and the waves take tiles from an LDS counter
// (tile-major, so wave w starts on ray w's first tile, as before).  A tile's field values (rgb, sigma per
// sample) go to LDS; the wave whose tile completes a ray composites that ray from LDS with render_ray's exact
// sequence (t, dist, conditioning, composite_tile in tile order, background, reductions), so every output is
// bit-identical to render_kernel.  Early ray termination needs the tiles in order: tau > 0 keeps render_kernel.
#ifndef ACN_RENDER_WS
#define ACN_RENDER_WS 1
#endif
constexpr int kWsMaxS = 256;   // LDS field buffer: 16 rays x kWsMaxS samples x 16 B = 64 KB
#ifndef ACN_WS_CHECK
#define ACN_WS_CHECK 0   // diagnostic self-check build (tools/dbg/selfcheck.py)
#endif
#ifndef ACN_WS_PREFOLD
#define ACN_WS_PREFOLD 1  // fold each round ray's SH colour bias once, at the round start (not per tile)
#endif
#ifndef ACN_WS_DTILE
// R > 0: depth tiles -- a field tile = R of the round's 16 rays at 32 / R consecutive samples, instead of one ray's
// 32 consecutive samples (0).  A wave's gathers then come from neighbouring rays at nearby depths, whose points
// share hash lines at more levels than one ray's consecutive samples do.  C2: 3.72e9 (0) -> 3.79 (16) / 3.89 (8) /
// 3.90 (4) / 3.86e9 (2) ray-samples/s (profiles/r06y_ws_dtile_ab.jsonl); outputs bit-identical (the field of a
// sample does not depend on its tile-mates; compositing reads LDS per ray as before).  The self-check build
// (ACN_WS_CHECK) keeps ray tiles.
#define ACN_WS_DTILE (ACN_WS_CHECK ? 0 : 8)
#endif

// composite one ray from its samples' field values in LDS (ys[s] = rgb, sigma of sample s, as the field tile
// returned them): render_ray's exact sequence without early termination -- t and dist, the volume_render
// conditioning, composite_tile in tile order, weights, background, the double reductions, the outputs
__device__ __forceinline__ void composite_ray_lds(const RenderParams& p, const BgArgs& bg, int64_t ray,
                                                  const f32x4* __restrict__ ys, int lane, float step) {
    const int j = lane & 31, h = lane >> 5;
    const int S = p.S;
    const float* rq = p.rays + ray * 8;
    const float dx = rq[3], dy = rq[4], dz = rq[5];
    const float near = rq[6], far = rq[7];
    const float* jit = p.jitter ? p.jitter + ray * S : nullptr;
    RayAcc acc{1.0, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (int s0 = 0; s0 < S; s0 += 32) {
        const int s = s0 + j;
        const bool valid = s < S;
        const int sc = valid ? s : S - 1;
        float t, dist;
        if (!jit) {
            const int i0 = sc < S - 1 ? sc : S - 2;
            const float ta = tlin_sel(near, far, i0, S, step), tb = tlin_sel(near, far, i0 + 1, S, step);
            t = sc < S - 1 ? ta : tb;
            dist = tb - ta;
        } else {
            t = tval(near, far, sc, S, jit);
            const float tn = (sc < S - 1) ? tval(near, far, sc + 1, S, jit) : t;
            const float tp = (sc == S - 1 && S > 1) ? tval(near, far, sc - 1, S, jit) : t;
            dist = (sc < S - 1) ? (tn - t) : (t - tp);
        }
        const f32x4 y = ys[sc];
        const float cr = clamp_nan(y[0], 0.0f, 1.0f);
        const float cg = clamp_nan(y[1], 0.0f, 1.0f);
        const float cbl = clamp_nan(y[2], 0.0f, 1.0f);
        float sig = clamp_min_nan(y[3], 0.0f);
        if (p.sigma_scale != 1.0f) sig = sig * p.sigma_scale;
        float wv;
        composite_tile(acc, valid, cr, cg, cbl, sig, t, dist, j, &wv);
        if (p.weights && valid && h == 0) p.weights[ray * S + s] = wv;
    }
    float bgc[3];
    background(bg, dx, dy, dz, lane, bgc);
    float r, g, b, dd, a;
    finish_ray(acc, r, g, b, dd, a);
    if (lane == 0) {
        if (bg.mode != ACN_BG_NONE) {
            const float om = 1.0f - a;
            r = r + om * bgc[0];
            g = g + om * bgc[1];
            b = b + om * bgc[2];
        }
        p.rgb[ray * 3 + 0] = r;
        p.rgb[ray * 3 + 1] = g;
        p.rgb[ray * 3 + 2] = b;
        p.depth[ray] = dd;
        p.acc[ray] = a;
    }
}

template <int INTERP>
__global__ void __launch_bounds__(1024, 4) render_ws_kernel(FieldCfg cfg, BgArgs bg, RenderParams p) {
    constexpr bool FOLD = ACN_SHFOLD != 0;
    __shared__ __attribute__((aligned(16))) float smem[PK_FLOATS];
    __shared__ __attribute__((aligned(16))) float cbuf[FOLD ? 16 * 64 : 4];
    __shared__ __attribute__((aligned(16))) f32x4 ybuf[16 * kWsMaxS];
    __shared__ int qhead;
    __shared__ int done[16];
    stage_weights<1>(smem, p.packed);
    const float* W = smem;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* cb = FOLD ? cbuf + wave * 64 : nullptr;
    const int S = p.S;
    const int T = (S + 31) >> 5;
    const float step = 1.0f / (float)(S - 1);
    // the rays of a round: 16 consecutive positions, XCD bands as in render_kernel
    int64_t base, hi, stride;
    if ((gridDim.x & 7) == 0) {
        const int64_t chunk = (p.N + 7) >> 3;
        const int64_t lo = min(p.N, (int64_t)(blockIdx.x & 7) * chunk);
        hi = min(p.N, lo + chunk);
        base = lo + (int64_t)(blockIdx.x >> 3) * 16;
        stride = (int64_t)(gridDim.x >> 3) * 16;
    } else {
        hi = p.N;
        base = (int64_t)blockIdx.x * 16;
        stride = (int64_t)gridDim.x * 16;
    }
    for (; base < hi; base += stride) {   // block-uniform
        // the lane index re-derived per round through an opaque copy: the per-lane LDS addresses and constants
        // formed from it stay inside the loop instead of being hoisted into registers held across it (spilled)
        const int tid = opaque_v((int)threadIdx.x);
        const int lane = tid & 63, j = lane & 31, h = lane >> 5;
        const float kz = __int_as_float(opaque_s(0));   // +0.0f for the SH coefficients (acn_device.h)
        const int nr = (int)min((int64_t)16, hi - base);
        if (tid == 0) qhead = 0;
        if (tid < 16) done[tid] = 0;
        constexpr bool PRE = FOLD && ACN_WS_PREFOLD;
        if (PRE && wave < nr) {
            // wave w folds round slot w's colour bias into cbuf[w] once; every tile of that ray reads it there
            const int64_t r0 = p.order ? (int64_t)__builtin_amdgcn_readfirstlane(p.order[base + wave]) : base + wave;
            const float* rp = p.rays + r0 * 8;
            float sh[16], sv[8];
            dir_sh(rp[3], rp[4], rp[5], sh, kz);
            sh_rows_for_half(sh, h, sv);
            fold_sh_bias(W, sv, lane, cbuf + wave * 64);
        }
        __syncthreads();
#if ACN_WS_DTILE
        static_assert(!ACN_WS_DTILE || (FOLD && ACN_WS_PREFOLD && !ACN_WS_CHECK), "depth tiles read the pre-folded bias");
        static_assert(16 % (ACN_WS_DTILE > 0 ? ACN_WS_DTILE : 1) == 0, "ACN_WS_DTILE: rays per tile divide 16");
        {
            // tile = R rays of one group of the round at D = 32 / R consecutive samples; lane j: slot g R + j % R,
            // sample q D + j / R (both halves of the tile: the same sample).  Slots past the round's rays repeat
            // its last ray and write nothing.
            constexpr int R = ACN_WS_DTILE, D = 32 / R, NG = 16 / R;
            const int ND = (S + D - 1) / D;
            const float shz[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
            int gcur = -1;
            int slot = 0;
            float ox = 0.0f, oy = 0.0f, oz = 0.0f, dx = 0.0f, dy = 0.0f, dz = 0.0f, near = 0.0f, far = 0.0f;
            const float* jit = nullptr;
            for (;;) {
                int item = 0;
                if (lane == 0) item = __hip_atomic_fetch_add(&qhead, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                item = __builtin_amdgcn_readlane(item, 0);
                if (item >= NG * ND) break;
                const int g = NG == 1 ? 0 : item % NG, q = NG == 1 ? item : item / NG;
                if (g != gcur) {   // wave-uniform
                    slot = g * R + (j % R);
                    const int ls = slot < nr ? slot : nr - 1;
                    const int64_t ray = p.order ? (int64_t)p.order[base + ls] : base + ls;
                    const float* rp = p.rays + ray * 8;
                    ox = rp[0], oy = rp[1], oz = rp[2], dx = rp[3], dy = rp[4], dz = rp[5];
                    near = rp[6], far = rp[7];
                    jit = p.jitter ? p.jitter + ray * S : nullptr;
                    gcur = g;
                }
                const int s = q * D + j / R;
                const int sc = s < S ? s : S - 1;
                float t;
                if (!jit) {
                    const int i0 = sc < S - 1 ? sc : S - 2;
                    const float ta = tlin_sel(near, far, i0, S, step), tb = tlin_sel(near, far, i0 + 1, S, step);
                    t = sc < S - 1 ? ta : tb;
                } else {
                    t = tval(near, far, sc, S, jit);
                }
                const float px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;
                uint32_t fl = 1u;
                float yr, yg, yb, ys;
                container_tile<INTERP, 0, FOLD>(cfg, W, px, py, pz, shz, cbuf + slot * 64, &fl, lane, yr, yg, yb, ys);
                if (h == 0 && s < S && slot < nr) {
                    f32x4 v;
                    v[0] = yr, v[1] = yg, v[2] = yb, v[3] = ys;
                    ybuf[slot * kWsMaxS + s] = v;
                }
            }
            __syncthreads();   // every sample of the round's rays is in ybuf
            if (wave < nr) {
                const int64_t ray_w = p.order ? (int64_t)__builtin_amdgcn_readfirstlane(p.order[base + wave]) : base + wave;
                composite_ray_lds(p, bg, ray_w, ybuf + wave * kWsMaxS, lane, step);
            }
            __syncthreads();
            continue;
        }
#endif
        int64_t cur = -1;
        uint32_t folded = 0u;
        float shv[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        float ox = 0.0f, oy = 0.0f, oz = 0.0f, dx = 0.0f, dy = 0.0f, dz = 0.0f, near = 0.0f, far = 0.0f;
        const float* jit = nullptr;
        for (;;) {
            int item = 0;
            if (lane == 0) item = __hip_atomic_fetch_add(&qhead, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            item = __builtin_amdgcn_readlane(item, 0);
            if (item >= nr * T) break;
            const int tile = item / nr, slot = item - tile * nr;
            const int64_t ray = p.order ? (int64_t)__builtin_amdgcn_readfirstlane(p.order[base + slot]) : base + slot;
            if (ray != cur) {
                const float* rp = p.rays + ray * 8;
                ox = rp[0], oy = rp[1], oz = rp[2], dx = rp[3], dy = rp[4], dz = rp[5];
                near = rp[6], far = rp[7];
                jit = p.jitter ? p.jitter + ray * S : nullptr;
                if (!PRE || ACN_WS_CHECK) {
                    float sh[16];
                    dir_sh(dx, dy, dz, sh, kz);
                    sh_rows_for_half(sh, h, shv);
                    if (!PRE) folded = 0u;
                }
                cur = ray;
            }
            if (PRE) {   // the slot's pre-folded bias (shv is not read by a folded field tile)
                cb = cbuf + slot * 64;
                folded = 1u;
            }
            const int s = tile * 32 + j;
            const int sc = s < S ? s : S - 1;
            float t;
            if (!jit) {
                const int i0 = sc < S - 1 ? sc : S - 2;
                const float ta = tlin_sel(near, far, i0, S, step), tb = tlin_sel(near, far, i0 + 1, S, step);
                t = sc < S - 1 ? ta : tb;
            } else {
                t = tval(near, far, sc, S, jit);
            }
            const float px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;
            float yr, yg, yb, ys;
            container_tile<INTERP, 0, FOLD>(cfg, W, px, py, pz, shv, cb, &folded, lane, yr, yg, yb, ys);
#if ACN_WS_CHECK  // diagnostic build only: the tile evaluated twice; a differing lane poisons its sample (NaN rgb).
            {   // The second evaluation runs colour layer 0 unfolded, SH k-step first: bit for bit the fold + folded
                // layer (field_tile), so a stale operand in the per-ray fold is caught as well
                float cr, cg, cbb, cs;
                field_tile<INTERP, false, true>(W, cfg.ex[0], cfg.log2T, px, py, pz, shv, nullptr, lane, cr, cg, cbb, cs);
                cs = trunc_exp(cs);
                if (__float_as_uint(cr) != __float_as_uint(yr) || __float_as_uint(cg) != __float_as_uint(yg) ||
                    __float_as_uint(cbb) != __float_as_uint(yb) || __float_as_uint(cs) != __float_as_uint(ys))
                    yr = __int_as_float(0x7fc00000);
            }
#endif
            if (h == 0 && s < S) {
                f32x4 v;
                v[0] = yr, v[1] = yg, v[2] = yb, v[3] = ys;
                ybuf[slot * kWsMaxS + s] = v;
            }
            // the wave's LDS writes are ordered before its count (workgroup-scope release / acquire)
            int old = 0;
            if (lane == 0) old = __hip_atomic_fetch_add(&done[slot], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            old = __builtin_amdgcn_readlane(old, 0);
            if (old != T - 1) continue;
            // this tile completed the ray: composite it (render_ray's sequence, no early termination)
            composite_ray_lds(p, bg, ray, ybuf + slot * kWsMaxS, lane, step);
        }
        __syncthreads();   // ybuf / qhead / done reused by the next round
    }
}

// ------------------------------------------------------------------------------------------
// Routed render with more than two experts (C3 / C4).  LDS holds two expert SLOTS; per round of
// 16 rays (one per wave) the workgroup routes every sample of its rays, counts how many waves
// need each expert, and stages the two most needed ones into the slots (only when they change --
// with rays sorted by owning expert, parallel.expert_sorted_plan, a workgroup's rays mostly need
// the same one or two experts, so staging is rare).  A sample whose expert is not resident is
// evaluated from the packed image in global memory (L2), without the SH fold.
#ifndef ACN_SLOTS_SINGLE
#define ACN_SLOTS_SINGLE 1  // single-expert rays (kSingleRay) skip the per-sample routing and blend
#endif
// Bit kSingleRay of the returned mask: every sample of the ray is routed to ONE expert with weight
// exactly 1.0f (soft: (1/d)/den with den = 1/d; hard: always), so the container's blend
// 0 + y_k * 1.0f is y_k bit for bit and the ray can skip the per-sample routing and blend.
constexpr uint32_t kSingleRay = 1u << 31;
// The expert bits and the exactness test of route_prep<1> + route_weight for one sample, without the
// quotients: w_k = ((d_k <= thr) ? 1/d_k : 0) / den is > 0 exactly when d_k <= thr and d_k is finite
// (den >= 1e-6 and finite), and is exactly 0 or 1 on every expert when at most one finite d_k is inside
// the margin and, if one is, (1/d_k) / max(1/d_k, 1e-6) == 1 (den is then 0 + 1/d_k: the other terms
// add +0).  With two or more inside, the ray has two bits and is never a single-expert ray, so its
// exactness does not matter.  One square root per sample for the minimum, and one per expert near the margin
// only (route_thr2), instead of 3K square roots and 3K divisions.
__device__ __forceinline__ void soft_route_bits(const FieldCfg& cfg, float px, float py, float pz, uint32_t& m,
                                                bool& exact) {
    // min_k max(sqrt(max(s_k, 0)), 1e-6) = max(sqrt(min_k max(s_k, 0)), 1e-6): sqrt and the clamps are
    // monotonic, so the minimum is taken on the squared distances (one square root instead of K)
    float mins = INFINITY;
    for (int k = 0; k < cfg.K; ++k) mins = fminf(mins, route_dist2(cfg, k, px, py, pz));
    float mind = sqrtf(mins);
    mind = mind < 1e-6f ? 1e-6f : mind;
    const float thr = cfg.bm * mind, thr2 = route_thr2(thr);
    int cnt = 0;
    float dsel = 1.0f;
    for (int k = 0; k < cfg.K; ++k) {
        const float s2 = route_dist2(cfg, k, px, py, pz);
        if (s2 > thr2) continue;   // outside the margin (route_thr2)
        float d = sqrtf(s2);
        d = d < 1e-6f ? 1e-6f : d;
        if (d <= thr && d < INFINITY) {
            m |= 1u << k;
            ++cnt;
            dsel = d;
        }
    }
    if (cnt == 1) {
        const float inv = 1.0f / dsel;
        const float den = inv < 1e-6f ? 1e-6f : inv;
        exact = exact && (inv / den == 1.0f);
    }
}
__device__ __forceinline__ uint32_t ray_expert_mask(const FieldCfg& cfg, int route, const RenderParams& p, int64_t ray,
                                                    bool live, float step, int lane) {
    uint32_t m = 0u;
    bool exact = true;
    if (live) {
        const float* rp = p.rays + ray * 8;
        const float ox = rp[0], oy = rp[1], oz = rp[2], dx = rp[3], dy = rp[4], dz = rp[5];
        const float near = rp[6], far = rp[7];
        const float* jit = p.jitter ? p.jitter + ray * p.S : nullptr;
        for (int s = lane; s < p.S; s += 64) {
            const float t = jit ? tval(near, far, s, p.S, jit) : tlin_sel(near, far, s, p.S, step);
            const float px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;
            if (route == 1) {
                soft_route_bits(cfg, px, py, pz, m, exact);
            } else {
                m |= 1u << route_prep<2>(cfg, px, py, pz).hard;
            }
        }
    }
    uint32_t any = 0u;  // OR over the wave: one ballot per expert (scalar), no LDS round trips
    for (int k = 0; k < cfg.K; ++k)
        if (__ballot((m >> k) & 1u) != 0ull) any |= 1u << k;
    if (ACN_SLOTS_SINGLE && __builtin_popcount(any) == 1 && __ballot(!exact) == 0ull) any |= kSingleRay;
    return any;
}

#ifndef ACN_ORDER_DIAG
#define ACN_ORDER_DIAG 0  // diagnostic builds of ray_order_kernel (1-3: stop after a phase; wrong orders)
#endif
#ifndef ACN_SLOTS_BAND
#define ACN_SLOTS_BAND 0
#endif
#ifndef ACN_SLOTS_CHECK
#define ACN_SLOTS_CHECK 0   // diagnostic self-check build (tools/dbg/selfcheck.py; 2: mismatches recorded)
#endif
#if ACN_SLOTS_CHECK > 1
constexpr unsigned kChkMax = 4096;
__device__ float g_chk[16 * kChkMax];
__device__ unsigned g_chk_n;
#endif
#ifndef ACN_SLOTS_THREADS
#define ACN_SLOTS_THREADS 512  // 2 waves/SIMD, 256 VGPRs: the 1024-thread build spills and was measured wrong
#endif
// `folded` (per ray, wave-uniform): bits 0-1 = LDS slot 0 / 1 folded; bit 3 = cbg holds the fold of expert
// (folded >> 4) & 31, the expert read from global memory last (its fold is reused while it stays the same)
__device__ __forceinline__ bool cbg_holds(uint32_t folded, int k) {
    return (folded & 8u) && (int)((folded >> 4) & 31u) == k;
}
__device__ __forceinline__ uint32_t cbg_set(uint32_t folded, int k) {
    return (folded & 7u) | 8u | ((uint32_t)k << 4);
}
// the field of one 32-sample tile in render_slots_kernel: LDS slot experts, the rest from the packed images
// in global memory (folded colour bias in cb[slot] / cbg); single = one expert with weight 1.0f on every sample
template <int INTERP, int ROUTE, bool FOLD>
__device__ __forceinline__ void slots_field(const FieldCfg& cfg, const RenderParams& p, const float* smem, float* cb,
                                            float* cbg, int k0, int k1, bool single, int k_single, float px, float py,
                                            float pz, const float (&shv)[8], uint32_t& folded, int lane, float& yr,
                                            float& yg, float& yb, float& ys) {
        if (single) {  // wave-uniform: one expert, weight 1.0f on every sample
            const int k = k_single;
            const int sl = (k == k0) ? 0 : ((k == k1) ? 1 : -1);
            float sg;
            if (sl >= 0) {
                const float* Wk = smem + sl * PK_FLOATS;
                float* cbk = FOLD ? cb + sl * 64 : nullptr;
                if (FOLD && !((folded >> sl) & 1u)) {
                    fold_sh_bias(Wk, shv, lane, cbk);
                    folded |= 1u << sl;
                }
                field_tile<INTERP, FOLD, false, ACN_FIELD_CHECK != 0>(Wk, cfg.ex[k], cfg.log2T, px, py, pz, shv, cbk, lane, yr,
                                         yg, yb, sg);
            } else {
                const float* Wg = p.packed + (size_t)k * PK_FLOATS;
                if (FOLD && !cbg_holds(folded, k)) {
                    fold_sh_bias(Wg, shv, lane, cbg);
                    folded = cbg_set(folded, k);
                }
                field_tile<INTERP, FOLD, false, ACN_FIELD_CHECK != 0>(Wg, cfg.ex[k], cfg.log2T, px, py, pz, shv, cbg, lane, yr,
                                         yg, yb, sg);
            }
            ys = trunc_exp(sg);
            return;
        }
    #if ACN_DIAG_SLOTS_NOMULTI  // diagnostic build only: the multi-expert blend path removed (register study)
        yr = yg = yb = ys = 0.0f;
        return;
    #endif
        const RouteState st = route_prep<ROUTE>(cfg, px, py, pz);
        yr = yg = yb = ys = 0.0f;
        for (int k = 0; k < cfg.K; ++k) {
            const float wk = (ROUTE == 1) ? route_weight(cfg, st, k, px, py, pz) : 0.0f;
            const bool need = (ROUTE == 1) ? (wk > 0.0f) : (st.hard == k);
            if (__ballot(need) == 0ull) continue;
            float r, g, b, sg;
            const int sl = (k == k0) ? 0 : ((k == k1) ? 1 : -1);
            if (sl >= 0) {
                const float* Wk = smem + sl * PK_FLOATS;
                float* cbk = FOLD ? cb + sl * 64 : nullptr;
                if (FOLD && !((folded >> sl) & 1u)) {
                    fold_sh_bias(Wk, shv, lane, cbk);
                    folded |= 1u << sl;
                }
                field_tile<INTERP, FOLD, false, ACN_FIELD_CHECK != 0>(Wk, cfg.ex[k], cfg.log2T, px, py, pz, shv, cbk, lane, r, g,
                                         b, sg);
            } else {
    #if ACN_SLOTS_NOFALLBACK  // diagnostic only: non-resident experts skipped
                r = g = b = sg = 0.0f;
    #else
                const float* Wg = p.packed + (size_t)k * PK_FLOATS;
                if (FOLD && !cbg_holds(folded, k)) {
                    fold_sh_bias(Wg, shv, lane, cbg);
                    folded = cbg_set(folded, k);
                }
                field_tile<INTERP, FOLD, false, ACN_FIELD_CHECK != 0>(Wg, cfg.ex[k], cfg.log2T, px, py, pz, shv, cbg, lane, r, g,
                                         b, sg);
    #endif
            }
            sg = trunc_exp(sg);
            if (need) {
                if (ROUTE == 1) {
                    yr = yr + r * wk;
                    yg = yg + g * wk;
                    yb = yb + b * wk;
                    ys = ys + sg * wk;
                } else {
                    yr = r; yg = g; yb = b; ys = sg;
                }
            }
        }
}

template <int INTERP, int ROUTE>
__global__ void __launch_bounds__(ACN_SLOTS_THREADS, ACN_SLOTS_THREADS / 256) render_slots_kernel(FieldCfg cfg, BgArgs bg, RenderParams p) {
    constexpr bool FOLD = ACN_SHFOLD != 0;
    __shared__ __attribute__((aligned(16))) float smem[2 * PK_FLOATS];
    // per wave: the folded SH bias of the two LDS slots and of the expert read from L2 (every expert's
    // colour layer 0 runs folded, wherever its weights are read from: a ray's arithmetic must not depend on
    // which experts its workgroup round keeps in LDS -- that choice depends on the other rays of the batch)
    __shared__ __attribute__((aligned(16))) float cbuf[FOLD ? (ACN_SLOTS_THREADS / 64) * 3 * 64 : 4];
    // per-round expert counts, three buffers by round index: round q counts into cnt[q % 3], every wave reads
    // that buffer after the round's barrier, and thread 0 clears cnt[(q + 2) % 3] (read in round q - 1, before
    // this barrier; written again in round q + 2, after the next one) -- one barrier per round, not three
    __shared__ int cnt[3][kMaxK];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* cb = FOLD ? cbuf + wave * 3 * 64 : nullptr;
    float* cbg = FOLD ? cb + 2 * 64 : nullptr;
    const float step = 1.0f / (float)(p.S - 1);
    if (threadIdx.x < 3 * kMaxK) (&cnt[0][0])[threadIdx.x] = 0;
    __syncthreads();
    // the two LDS slots' experts: wave-uniform registers, updated identically by every wave from the counts
    int sk0 = -1, sk1 = -1, rbuf = 0;
    const int64_t waves_per_wg = blockDim.x >> 6;
    // XCD bands (as render_kernel): with the grid a multiple of 8, XCD x walks the x-th contiguous
    // eighth of the rays, so a frame's neighbouring rays share one L2 (ACN_SLOTS_BAND=0: interleaved)
    int64_t first = (int64_t)blockIdx.x * waves_per_wg, lim = p.norder ? (int64_t)p.norder[0] : p.N,
            gstride = (int64_t)gridDim.x * waves_per_wg;
    if (ACN_SLOTS_BAND && (gridDim.x & 7) == 0 && !p.norder) {
        const int64_t chunk = (((p.N + 7) >> 3) + waves_per_wg - 1) / waves_per_wg * waves_per_wg;
        const int64_t lo = min(p.N, (int64_t)(blockIdx.x & 7) * chunk);
        lim = min(p.N, lo + chunk);
        first = lo + (int64_t)(blockIdx.x >> 3) * waves_per_wg;
        gstride = (int64_t)(gridDim.x >> 3) * waves_per_wg;
    }
    for (int64_t base = first; base < lim; base += gstride) {
        const bool live = base + wave < lim;
        const int64_t ray = !live ? 0 : (p.order ? (int64_t)__builtin_amdgcn_readfirstlane(p.order[base + wave])
                                                 : base + wave);
        if (live) { SL_MARK(ray, 0) }
        const uint32_t m = ray_expert_mask(cfg, ROUTE, p, ray, live, step, lane);
        if (live) { SL_MARK(ray, 1) }
        int* cq = cnt[rbuf];
        if (lane == 0)
            for (int k = 0; k < cfg.K; ++k)
                if ((m >> k) & 1u) atomicAdd(&cq[k], 1);
        __syncthreads();   // this round's counts complete; every wave is done with the previous round's slots
        {
            // the two most needed experts (the same choice in every wave: same counts, same slot state)
            int b0 = -1, b1 = -1;
            for (int k = 0; k < cfg.K; ++k) {
                const int c = cq[k];
                if (c == 0) continue;
                if (b0 < 0 || c > cq[b0]) { b1 = b0; b0 = k; }
                else if (b1 < 0 || c > cq[b1]) b1 = k;
            }
            b0 = __builtin_amdgcn_readfirstlane(b0);
            b1 = __builtin_amdgcn_readfirstlane(b1);
            const int rclear = rbuf == 0 ? 2 : rbuf - 1;   // (q + 2) % 3
            if (threadIdx.x < kMaxK) cnt[rclear][threadIdx.x] = 0;
            rbuf = rbuf == 2 ? 0 : rbuf + 1;
            // keep an expert in the slot it already occupies
            if (b0 == sk1 || b1 == sk0) { const int t = b0; b0 = b1; b1 = t; }
            const bool rs0 = b0 >= 0 && b0 != sk0, rs1 = b1 >= 0 && b1 != sk1;
            if (b0 >= 0) sk0 = b0;
            if (b1 >= 0) sk1 = b1;
            if (rs0 || rs1) {   // block-uniform
                for (int sl = 0; sl < 2; ++sl) {
                    if (sl == 0 ? !rs0 : !rs1) continue;
                    const f32x4* src = reinterpret_cast<const f32x4*>(p.packed + (size_t)(sl == 0 ? sk0 : sk1) * PK_FLOATS);
                    f32x4* dst = reinterpret_cast<f32x4*>(smem + sl * PK_FLOATS);
                    for (int i = threadIdx.x; i < PK_FLOATS / 4; i += blockDim.x) dst[i] = src[i];
                }
                __syncthreads();
            }
        }
#if ACN_DIAG_NOSLOTS  // diagnostic build only: every expert from global memory
        const int k0 = -1, k1 = -1;
#else
        const int k0 = sk0, k1 = sk1;
#endif
        if (live) { SL_MARK(ray, 2) }
        if (live) {
            const bool single = (m & kSingleRay) != 0u;
            const int k_single = __builtin_ctz(m | kSingleRay);
            render_ray(p, bg, ray, lane, step,
                       [&](int sc_, float px, float py, float pz, const float (&shv)[8], uint32_t& folded, float& yr, float& yg,
                           float& yb, float& ys) {
                           (void)sc_;
                           slots_field<INTERP, ROUTE, FOLD>(cfg, p, smem, cb, cbg, k0, k1, single, k_single, px, py,
                                                            pz, shv, folded, lane, yr, yg, yb, ys);
#if ACN_SLOTS_CHECK  // diagnostic build only: the tile evaluated again with every fold redone; a differing lane
                     // poisons its sample (NaN rgb: tools/dbg/selfcheck.py)
                           uint32_t f2 = 0u;
                           float cr, cg, cbb, cs;
                           slots_field<INTERP, ROUTE, FOLD>(cfg, p, smem, cb, cbg, k0, k1, single, k_single, px, py,
                                                            pz, shv, f2, lane, cr, cg, cbb, cs);
                           if (__float_as_uint(cr) != __float_as_uint(yr) || __float_as_uint(cg) != __float_as_uint(yg) ||
                               __float_as_uint(cbb) != __float_as_uint(yb) || __float_as_uint(cs) != __float_as_uint(ys)) {
#if ACN_SLOTS_CHECK > 1   // record the mismatch (tools/dbg/selfcheck.py --detail)
                               const unsigned q = atomicAdd(&g_chk_n, 1u);
                               if (q < kChkMax) {
                                   float* o = g_chk + 16 * q;
                                   o[0] = (float)ray; o[1] = (float)sc_; o[2] = single ? 1.0f : 0.0f; o[3] = (float)k_single;
                                   o[4] = (float)k0; o[5] = (float)k1; o[6] = yr; o[7] = cr; o[8] = yg; o[9] = cg;
                                   o[10] = yb; o[11] = cbb; o[12] = ys; o[13] = cs; o[14] = (float)lane;
                                   o[15] = (float)folded;
                               }
#endif
                               yr = __int_as_float(0x7fc00000);
                           }
#endif
                       });
            SL_MARK(ray, 5)
        }
    }
}

// Routed render in depth tiles (render_wss_kernel: C3 / C4 without early termination).  render_slots_kernel gives
// every wave one ray and its 32-sample tiles; here, as in render_ws_kernel, the 8 rays of a workgroup round are
// cut into tiles of R rays x 32 / R consecutive samples (ACN_WSS_DTILE), so a wave's hash gathers come from
// neighbouring rays at nearby depths.  Per round: every wave routes its ray's samples (ray_expert_mask), the
// counts pick the two most needed experts for the LDS slots (render_slots_kernel's rule; the others are read
// from the packed images in global memory), the waves take tiles from an LDS counter and put each sample's
// blended (rgb, sigma) in LDS, and after a barrier wave w composites ray w with render_ray's sequence
// (composite_ray_lds).  A tile mixes rays, so colour layer 0 runs unfolded on each lane's own SH rows, SH k-steps
// first (field_tile SHFIRST: bit for bit the folded layer), and the blend is the general path (for a
// single-expert ray 0 + y * 1.0f == y): every output equals render_slots_kernel's (tests/test_k8.py).
#ifndef ACN_RENDER_WSS
#define ACN_RENDER_WSS 1
#endif
// Rounds (RW = rays per round, LDS ybuf = RW x kWssMaxS(RW) samples x 16 B = 32 KB beside the two expert images):
// 16 rays (two per wave) in tiles of 16 rays x 2 samples up to S = 128, else 8 rays in tiles of 8 x 4.  C4-S96:
// 3.12e9 (8 / 8 x 4) -> 3.17e9 (16 / 8 x 4) -> 3.27e9 (16 / 16 x 2) ray-samples/s (profiles/r06ac_wss_rounds_ab.jsonl)
#ifndef ACN_WSS_DTILE8
#define ACN_WSS_DTILE8 8     // rays per tile in 8-ray rounds
#endif
#ifndef ACN_WSS_DTILE16
#define ACN_WSS_DTILE16 16   // rays per tile in 16-ray rounds
#endif
#ifndef ACN_WSS_RAYS16
#define ACN_WSS_RAYS16 1     // 0: 8-ray rounds at every S
#endif
constexpr int kWssMaxS(int rw) { return rw == 8 ? kWsMaxS : 128; }
template <int INTERP, int ROUTE, int RW>
__global__ void __launch_bounds__(ACN_SLOTS_THREADS, ACN_SLOTS_THREADS / 256) render_wss_kernel(FieldCfg cfg, BgArgs bg, RenderParams p) {
    constexpr int kWssRays = RW, kWssPerWave = RW / (ACN_SLOTS_THREADS / 64), kMaxS = kWssMaxS(RW);
    constexpr int R = RW == 8 ? ACN_WSS_DTILE8 : ACN_WSS_DTILE16, D = 32 / R, NG = kWssRays / R;
    static_assert(kWssRays % R == 0 && 32 % R == 0, "ACN_WSS_DTILE*: rays per tile");
    __shared__ __attribute__((aligned(16))) float smem[2 * PK_FLOATS];
    __shared__ __attribute__((aligned(16))) f32x4 ybuf[kWssRays * kMaxS];
    static_assert(kWssPerWave >= 1 && kWssRays == kWssPerWave * (ACN_SLOTS_THREADS / 64), "rays per round");
    __shared__ int cnt[kMaxK];
    __shared__ int qhead;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int S = p.S;
    const float step = 1.0f / (float)(S - 1);
    const int ND = (S + D - 1) / D;
    int sk0 = -1, sk1 = -1;
    const int64_t lim = p.norder ? (int64_t)p.norder[0] : p.N;
    for (int64_t base = (int64_t)blockIdx.x * kWssRays; base < lim; base += (int64_t)gridDim.x * kWssRays) {
        const int tid = opaque_v((int)threadIdx.x);
        const int lane = tid & 63, j = lane & 31, h = lane >> 5;
        const int nr = (int)min((int64_t)kWssRays, lim - base);
        if (tid < kMaxK) cnt[tid] = 0;
        if (tid == 0) qhead = 0;
        __syncthreads();   // the previous round's composites are done with ybuf; counts cleared
        for (int u = 0; u < kWssPerWave; ++u) {   // wave w routes round slots w, w + 8, ...
            const int sl = wave + u * (ACN_SLOTS_THREADS / 64);
            const bool live = sl < nr;
            const int64_t ray = !live ? 0 : (p.order ? (int64_t)__builtin_amdgcn_readfirstlane(p.order[base + sl])
                                                     : base + sl);
            const uint32_t m = ray_expert_mask(cfg, ROUTE, p, ray, live, step, lane);
            if (lane == 0)
                for (int k = 0; k < cfg.K; ++k)
                    if ((m >> k) & 1u) atomicAdd(&cnt[k], 1);
        }
        __syncthreads();
        {   // the two most needed experts (render_slots_kernel's choice and slot keeping)
            int b0 = -1, b1 = -1;
            for (int k = 0; k < cfg.K; ++k) {
                const int c = cnt[k];
                if (c == 0) continue;
                if (b0 < 0 || c > cnt[b0]) { b1 = b0; b0 = k; }
                else if (b1 < 0 || c > cnt[b1]) b1 = k;
            }
            b0 = __builtin_amdgcn_readfirstlane(b0);
            b1 = __builtin_amdgcn_readfirstlane(b1);
            if (b0 == sk1 || b1 == sk0) { const int t = b0; b0 = b1; b1 = t; }
            const bool rs0 = b0 >= 0 && b0 != sk0, rs1 = b1 >= 0 && b1 != sk1;
            if (b0 >= 0) sk0 = b0;
            if (b1 >= 0) sk1 = b1;
            if (rs0 || rs1) {   // block-uniform
                for (int sl = 0; sl < 2; ++sl) {
                    if (sl == 0 ? !rs0 : !rs1) continue;
                    const f32x4* src = reinterpret_cast<const f32x4*>(p.packed + (size_t)(sl == 0 ? sk0 : sk1) * PK_FLOATS);
                    f32x4* dst = reinterpret_cast<f32x4*>(smem + sl * PK_FLOATS);
                    for (int i = tid; i < PK_FLOATS / 4; i += blockDim.x) dst[i] = src[i];
                }
                __syncthreads();
            }
        }
        const int k0 = sk0, k1 = sk1;
        int gcur = -1, slot = 0;
        float ox = 0.0f, oy = 0.0f, oz = 0.0f, dx = 0.0f, dy = 0.0f, dz = 0.0f, near = 0.0f, far = 0.0f;
        float shv[8];
        const float* jit = nullptr;
        for (;;) {
            int item = 0;
            if (lane == 0) item = __hip_atomic_fetch_add(&qhead, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            item = __builtin_amdgcn_readlane(item, 0);
            if (item >= NG * ND) break;
            const int g = NG == 1 ? 0 : item % NG, q = NG == 1 ? item : item / NG;
            if (g != gcur) {   // wave-uniform: this lane's ray of group g
                slot = g * R + (j % R);
                const int ls = slot < nr ? slot : nr - 1;
                const int64_t rr = p.order ? (int64_t)p.order[base + ls] : base + ls;
                const float* rp = p.rays + rr * 8;
                ox = rp[0], oy = rp[1], oz = rp[2], dx = rp[3], dy = rp[4], dz = rp[5];
                near = rp[6], far = rp[7];
                jit = p.jitter ? p.jitter + rr * S : nullptr;
                float sh[16];
                dir_sh(dx, dy, dz, sh);
                sh_rows_for_half(sh, h, shv);
                gcur = g;
            }
            const int s = q * D + j / R;
            const int sc = s < S ? s : S - 1;
            float t;
            if (!jit) {
                const int i0 = sc < S - 1 ? sc : S - 2;
                const float ta = tlin_sel(near, far, i0, S, step), tb = tlin_sel(near, far, i0 + 1, S, step);
                t = sc < S - 1 ? ta : tb;
            } else {
                t = tval(near, far, sc, S, jit);
            }
            const float px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;
            const RouteState st = route_prep<ROUTE>(cfg, px, py, pz);
            float yr = 0.0f, yg = 0.0f, yb = 0.0f, ys = 0.0f;
            for (int k = 0; k < cfg.K; ++k) {
                const float wk = (ROUTE == 1) ? route_weight(cfg, st, k, px, py, pz) : 0.0f;
                const bool need = (ROUTE == 1) ? (wk > 0.0f) : (st.hard == k);
                if (__ballot(need) == 0ull) continue;
                float r, gg, b, sg;
                if (k == k0 || k == k1)   // wave-uniform; separate call sites keep LDS and global reads of the image
                    field_tile<INTERP, false, true>(smem + (k == k0 ? 0 : PK_FLOATS), cfg.ex[k], cfg.log2T, px, py, pz,
                                                    shv, nullptr, lane, r, gg, b, sg);
                else
                    field_tile<INTERP, false, true>(p.packed + (size_t)k * PK_FLOATS, cfg.ex[k], cfg.log2T, px, py, pz,
                                                    shv, nullptr, lane, r, gg, b, sg);
                sg = trunc_exp(sg);
                if (need) {
                    if (ROUTE == 1) {
                        yr = yr + r * wk;
                        yg = yg + gg * wk;
                        yb = yb + b * wk;
                        ys = ys + sg * wk;
                    } else {
                        yr = r; yg = gg; yb = b; ys = sg;
                    }
                }
            }
            if (h == 0 && s < S && slot < nr) {
                f32x4 v;
                v[0] = yr, v[1] = yg, v[2] = yb, v[3] = ys;
                ybuf[slot * kMaxS + s] = v;
            }
        }
        __syncthreads();   // every sample of the round's rays is in ybuf
        for (int u = 0; u < kWssPerWave; ++u) {
            const int sl = wave + u * (ACN_SLOTS_THREADS / 64);
            if (sl >= nr) break;
            const int64_t ray = p.order ? (int64_t)__builtin_amdgcn_readfirstlane(p.order[base + sl]) : base + sl;
            composite_ray_lds(p, bg, ray, ybuf + sl * kMaxS, lane, step);
        }
    }
}

// inclusive scan over the 64 lanes of a wave on DPP: row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast:15 / :31 carry the row totals upward (gfx9-family DPP)
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return v;
}
// lanes of this wave (among `valid`) holding the same 6-bit digit, and how many of them sit below this lane
__device__ __forceinline__ uint64_t same_digit_lanes(bool valid, int dig) {
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 6; ++b) {
        const uint64_t bb = __ballot(valid && ((dig >> b) & 1));
        m &= ((dig >> b) & 1) ? bb : ~bb;
    }
    return m;
}
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
constexpr int kRtThreads = 512;   // ep_field_kernel: two workgroups per CU (16 waves)
#ifndef ACN_EP_BANDS
#define ACN_EP_BANDS 1                // ep_field_kernel: XCD bands over each expert's wave-tiles
#endif
constexpr int kRtWaves = kRtThreads / 64;
constexpr int kEpMaxSeg = 1024;   // W * E segments of the compact received layout (ep_field_kernel)

// ------------------------------------------------------------------------------------------
// One expert per GPU, render (expert_parallel.ExpertParallelRenderer).  The routed render of
// routed render split at its expert boundary: the senders' (sample, expert) pairs travel to the
// experts' owners as 24-B [world point, direction] records in the fixed layout of acn_routed_count_fixed.
//   ep_field_kernel     owner: each owned expert's field on the records received from every sender, in the
//                       received layout [sender][local expert][cap] -> (rgb, sigma) per record, the same
//                       per-(sample, expert) arithmetic as the fused routed render (LDS-staged image, SH-first
//                       colour layer 0 on per-lane SH), so a ray renders bit for bit as on one GPU;
//   ep_composite_kernel sender: the blend sum_k y_k w_k in ascending k from zero (meta_container.py:320-337)
//                       read from the returned pair slots, then render_kernel's compositing / background /
//                       outputs (ray_rendering.py:114-165): no (N,S,4) field tensor.
template <int INTERP>
__global__ void __launch_bounds__(kRtThreads, 4) ep_field_kernel(FieldCfg cfg, const float* __restrict__ xd,
                                                                  const int64_t* __restrict__ cnt, int W, int E,
                                                                  int64_t cap, const float* __restrict__ packed,
                                                                  float* __restrict__ ret) {
    __shared__ __attribute__((aligned(16))) float Wsl[PK_FLOATS];
    __shared__ int64_t pre[kEpMaxSeg];   // cap == 0 (compact layout): start of segment (w, e), row-major
    // lane from mbcnt (re-derivable anywhere): threadIdx.x is not held across the expert loop (it was spilled)
    const int lane = (int)__lane_id(), j = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t G = (int64_t)gridDim.x * kRtWaves;
    const bool compact = cap == 0;
    if (compact && wave == 0 && lane == 0) {
        int64_t o = 0;
        for (int q = 0; q < W * E; ++q) {
            pre[q] = o;
            o += cnt[q];
        }
    }
    __syncthreads();
    const int64_t cap_eff = compact ? INT64_MAX : cap;
    int slot = -1;
    for (int e = 0; e < E; ++e) {
        int64_t T = 0;   // wave-tiles of local expert e over all senders (records past cap were not sent)
        for (int w = 0; w < W; ++w) {
            const int64_t c = min(cnt[(int64_t)w * E + e], cap_eff);
            T += (c + 31) >> 5;
        }
        // XCD bands (as render_kernel): with the grid a multiple of 8, XCD x takes the x-th contiguous eighth of the
        // expert's wave-tiles, so consecutive records (a ray's samples, neighbouring rays) share one XCD's L2
        int64_t g0 = (int64_t)blockIdx.x * kRtWaves + wave, gend = T, gstep = G;
        if (ACN_EP_BANDS && (gridDim.x & 7) == 0) {
            const int64_t chunk = (T + 7) >> 3;
            const int64_t lo = min(T, (int64_t)(blockIdx.x & 7) * chunk);
            gend = min(T, lo + chunk);
            g0 = lo + (int64_t)(blockIdx.x >> 3) * kRtWaves + wave;
            gstep = (int64_t)(gridDim.x >> 3) * kRtWaves;
        }
        if (g0 - wave >= gend) continue;   // block-uniform: no tile of this expert for this workgroup
        if (slot != e) {
            __syncthreads();   // every wave is done with the previous expert's image
            const f32x4* src = reinterpret_cast<const f32x4*>(packed + (size_t)e * PK_FLOATS);
            f32x4* dst = reinterpret_cast<f32x4*>(Wsl);
            // opaque thread index: the unrolled copy's per-lane offsets are formed here, not held across the loop
            for (int i = opaque_v(wave * 64 + (int)__lane_id()); i < PK_FLOATS / 4; i += kRtThreads) dst[i] = src[i];
            __syncthreads();
            slot = e;
        }
        for (int64_t g = g0; g < gend; g += gstep) {
            int64_t tl = g, c = 0;
            int w = 0;
            for (; w < W; ++w) {   // sender of wave-tile g
                c = min(cnt[(int64_t)w * E + e], cap_eff);
                const int64_t nt = (c + 31) >> 5;
                if (tl < nt) break;
                tl -= nt;
            }
            const int64_t i = tl * 32 + j;
            const bool valid = i < c;
            const int64_t seg0 = compact ? pre[w * E + e] : ((int64_t)w * E + e) * cap;
            const int64_t rec = seg0 + (valid ? i : c - 1);
            const float* r = xd + rec * 6;
            const float px = r[0], py = r[1], pz = r[2];
            float sh[16], shv[8];
            dir_sh(r[3], r[4], r[5], sh);
            sh_rows_for_half(sh, h, shv);
            float rr, rg, rb, sg;
            field_tile<INTERP, false, true>(Wsl, cfg.ex[e], cfg.log2T, px, py, pz, shv, nullptr, lane, rr, rg, rb, sg);
            sg = trunc_exp(sg);
            if (valid && h == 0)
                *reinterpret_cast<f32x4*>(ret + 4 * (seg0 + i)) = f32x4{rr, rg, rb, sg};
        }
    }
}

template <int ROUTE>
__global__ void __launch_bounds__(1024) ep_composite_kernel(BgArgs bg, RenderParams p, const float* __restrict__ yr,
                                                            const float* __restrict__ pw,
                                                            const int32_t* __restrict__ pmap, int K) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const float step = 1.0f / (float)(p.S - 1);
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t ray = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave; ray < p.N; ray += nw) {
        render_ray(p, bg, ray, lane, step,
                   [&](int sc, float, float, float, const float (&)[8], uint32_t&, float& yr_, float& yg, float& yb,
                       float& ys) {
                       const int64_t m = ray * p.S + sc;
                       f32x4 a = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                       for (int k = 0; k < K; ++k) {
                           const int32_t q = pmap[m * K + k];
                           if (q < 0) continue;
                           const f32x4 y = *reinterpret_cast<const f32x4*>(yr + 4 * (int64_t)q);
                           if (ROUTE == 1) {
                               const float wk = pw[q];
                               a[0] = a[0] + y[0] * wk;
                               a[1] = a[1] + y[1] * wk;
                               a[2] = a[2] + y[2] * wk;
                               a[3] = a[3] + y[3] * wk;
                           } else {
                               a = y;
                           }
                       }
                       yr_ = a[0];
                       yg = a[1];
                       yb = a[2];
                       ys = a[3];
                   });
    }
}

// volume_render of one ray (one wave, 32-sample tiles; both lane halves hold the same samples) over
// fetch(sc) = the (N,S,4) rgb_sigma row of sample sc: rgb, depth, acc wave-uniform, weights row written
__device__ __forceinline__ float4 ld_rs(const float* v) { return make_float4(v[0], v[1], v[2], v[3]); }
template <class Fetch>
__device__ __forceinline__ void vr_fwd_ray(Fetch fetch, const float* __restrict__ t, int S, int raw_rgb, int raw_sigma,
                                           float sigma_scale, int j, int h, float* wrow, float& r, float& g, float& b,
                                           float& dd, float& a) {
    RayAcc acc{1.0, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (int s0 = 0; s0 < S; s0 += 32) {
        const int s = s0 + j;
        const bool valid = s < S;
        const int sc = valid ? s : S - 1;
        const float4 v = fetch(sc);
        float cr = v.x, cg = v.y, cb = v.z, sg = v.w;
        if (raw_rgb) { cr = sigmoidf_(cr); cg = sigmoidf_(cg); cb = sigmoidf_(cb); }
        else { cr = clamp_nan(cr, 0.0f, 1.0f); cg = clamp_nan(cg, 0.0f, 1.0f); cb = clamp_nan(cb, 0.0f, 1.0f); }
        sg = raw_sigma ? trunc_exp(sg) : clamp_min_nan(sg, 0.0f);
        if (sigma_scale != 1.0f) sg = sg * sigma_scale;
        const float dist = (sc < S - 1) ? (t[sc + 1] - t[sc]) : (t[sc] - t[sc - 1]);
        float wv;
        composite_tile(acc, valid, cr, cg, cb, sg, t[sc], dist, j, &wv);
        if (wrow && valid && h == 0) wrow[s] = wv;
    }
    finish_ray(acc, r, g, b, dd, a);
}

// standalone volume_render: one wave per ray
__global__ void __launch_bounds__(256) volume_render_kernel(const float* __restrict__ rs, const float* __restrict__ tv,
                                                            const float* __restrict__ bgp, int64_t N, int S,
                                                            int raw_rgb, int raw_sigma, float sigma_scale,
                                                            float* rgb, float* depth, float* weights, float* accp) {
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t ray = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); ray < N; ray += nw) {
        float r, g, b, dd, a;
        vr_fwd_ray([&](int sc) { return ld_rs(rs + (ray * S + sc) * 4); }, tv + ray * S, S, raw_rgb, raw_sigma,
                   sigma_scale, j, h, weights ? weights + ray * S : nullptr, r, g, b, dd, a);
        if (lane == 0) {
            if (bgp) {
                const float om = 1.0f - a;
                r = r + om * bgp[3 * ray];
                g = g + om * bgp[3 * ray + 1];
                b = b + om * bgp[3 * ray + 2];
            }
            rgb[3 * ray] = r; rgb[3 * ray + 1] = g; rgb[3 * ray + 2] = b;
            depth[ray] = dd;
            accp[ray] = a;
        }
    }
}

// Backward of volume_render (ray_rendering.py:137-165), the gradients autograd produces through
// clamp / exp / cumprod / the three weighted sums, one wave per ray in two forward sweeps over
// 32-sample tiles: sweep 1 rebuilds w_i = alpha_i T_i (T in double, as the forward) and the ray
// total G = sum_k g_k w_k of g_k = dL/dw_k = G_rgb.(c_k - bg) + G_depth t_k + G_acc + G_w,k;
// sweep 2 carries the inclusive prefix P_i of g_k w_k (double) so the suffix sum of
//   dL/dalpha_i = g_i T_i - (1 / x_i) sum_{k>i} g_k w_k,   x_i = 1 - alpha_i + 1e-10,
// is G - P_i.  Then alpha's clamp mask, d(1 - exp(-sigma delta))/dsigma = delta exp(-sigma delta),
// sigma_scale and clamp_min(0)'s mask; rgb gets w_i G_rgb under clamp(0,1)'s mask; bg gets
// (1 - acc) G_rgb.  t_vals get no gradient (stratified_t_vals runs under no_grad).
// fetch(sc) as vr_fwd_ray; store(s, grad) receives sample s's dL/d(rgb_sigma) on the h == 0 lanes; returns
// acc = sum w (double, wave-uniform) for the background gradient.
template <class Fetch, class Store>
__device__ __forceinline__ double vr_bwd_ray(Fetch fetch, Store store, const float* __restrict__ t, int S,
                                             float sigma_scale, float gr, float gg, float gb, float gd, float ga,
                                             float br, float bgg, float bb, const float* __restrict__ gwrow, int j,
                                             int h) {
    double G = 0.0, acc = 0.0;
    for (int pass = 0; pass < 2; ++pass) {
        double T = 1.0, P = 0.0;
        for (int s0 = 0; s0 < S; s0 += 32) {
            const int s = s0 + j;
            const bool valid = s < S;
            const int sc = valid ? s : S - 1;
            const float4 v = fetch(sc);
            const float cr = clamp_nan(v.x, 0.0f, 1.0f), cg = clamp_nan(v.y, 0.0f, 1.0f),
                        cb = clamp_nan(v.z, 0.0f, 1.0f);
            float sg = clamp_min_nan(v.w, 0.0f);
            if (sigma_scale != 1.0f) sg = sg * sigma_scale;
            float dist = (sc < S - 1) ? (t[sc + 1] - t[sc]) : (t[sc] - t[sc - 1]);
            dist = clamp_min_nan(dist, 1e-4f);
            const float e = expf(-sg * dist);
            const float a = 1.0f - e;
            const float alpha = clamp_nan(a, 0.0f, (float)(1.0 - 1e-7));
            float x = (1.0f - alpha) + 1e-10f;
            if (!valid) x = 1.0f;
            double incl = (double)x;
#pragma unroll
            for (int off = 1; off < 32; off <<= 1) {
                const double y = __shfl_up(incl, off, 32);
                if (j >= off) incl *= y;
            }
            double excl = __shfl_up(incl, 1, 32);
            if (j == 0) excl = 1.0;
            const float Ts = (float)(T * excl);
            const float w = valid ? alpha * Ts : 0.0f;
            float g = gr * (cr - br) + gg * (cg - bgg) + gb * (cb - bb) + gd * t[sc] + ga;
            if (gwrow && valid) g += gwrow[s];
            const double gw = valid ? (double)g * (double)w : 0.0;
            if (pass == 0) {
                G += gw;
                acc += (double)w;
            } else {
                double pre = gw;  // inclusive prefix of g_k w_k over the tile
#pragma unroll
                for (int off = 1; off < 32; off <<= 1) {
                    const double y = __shfl_up(pre, off, 32);
                    if (j >= off) pre += y;
                }
                const double suffix = G - (P + pre);
                const float dalpha = (float)((double)g * (double)Ts - suffix / (double)x);
                const bool amask = (a >= 0.0f) && (a <= (float)(1.0 - 1e-7));
                float dsig = amask ? dalpha * dist * e : 0.0f;
                if (sigma_scale != 1.0f) dsig = dsig * sigma_scale;
                const float gsr = (v.w >= 0.0f) ? dsig : 0.0f;
                if (valid && h == 0)
                    store(s, make_float4((v.x >= 0.0f && v.x <= 1.0f) ? w * gr : 0.0f,
                                         (v.y >= 0.0f && v.y <= 1.0f) ? w * gg : 0.0f,
                                         (v.z >= 0.0f && v.z <= 1.0f) ? w * gb : 0.0f, gsr));
                P += __shfl(pre, 31, 32);
            }
            T = T * __shfl(incl, 31, 32);
        }
        if (pass == 0) {
            G = wave32_sum(G);
            acc = wave32_sum(acc);
        }
    }
    return acc;
}

__global__ void __launch_bounds__(256) volume_render_bwd_kernel(
    const float* __restrict__ rs, const float* __restrict__ tv, const float* __restrict__ bgp, int64_t N, int S,
    float sigma_scale, const float* __restrict__ g_rgb, const float* __restrict__ g_depth,
    const float* __restrict__ g_w, const float* __restrict__ g_acc, float* __restrict__ g_rs,
    float* __restrict__ g_bg) {
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t ray = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); ray < N; ray += nw) {
        const float gr = g_rgb ? g_rgb[3 * ray] : 0.0f, gg = g_rgb ? g_rgb[3 * ray + 1] : 0.0f,
                    gb = g_rgb ? g_rgb[3 * ray + 2] : 0.0f;
        const float gd = g_depth ? g_depth[ray] : 0.0f, ga = g_acc ? g_acc[ray] : 0.0f;
        const float br = bgp ? bgp[3 * ray] : 0.0f, bgg = bgp ? bgp[3 * ray + 1] : 0.0f,
                    bb = bgp ? bgp[3 * ray + 2] : 0.0f;
        const double acc = vr_bwd_ray(
            [&](int sc) { return ld_rs(rs + (ray * S + sc) * 4); },
            [&](int s, float4 o) { *reinterpret_cast<float4*>(g_rs + (ray * S + s) * 4) = o; }, tv + ray * S, S,
            sigma_scale, gr, gg, gb, gd, ga, br, bgg, bb, g_w ? g_w + ray * S : nullptr, j, h);
        if (g_bg && lane == 0) {
            const float om = 1.0f - (float)acc;
            g_bg[3 * ray] = om * gr;
            g_bg[3 * ray + 1] = om * gg;
            g_bg[3 * ray + 2] = om * gb;
        }
    }
}

// Fused training compositing of the routed adaptation step (routed_train.RoutedAdaptStep: linear colour space,
// background from the SH-4 MLP head), one wave per ray:
//   rs  = the routed blend of the pair outputs (blend_fwd_kernel; meta_container.py:322-337)
//   bg  = background_color(dirs) (background_kernel), dirs = rays[:, 3:6] written out for the head's backward
//   rgb = volume_render(rs, t, bg) (ray_rendering.py:137-165), the linear-space MSE's gradient
//         (mse_linear_bwd_kernel; losses.py:10-32), volume_render's backward (vr_bwd_ray) and the blend's
//         backward into the pair slots (blend_bwd_kernel; padding slots below the live count get zeros)
// -- the arithmetic of those kernels, in one launch instead of eight (the gradients bitwise those kernels').  The
// reported loss: a double sum per workgroup in ray order, the last workgroup to finish adds the G partials in index
// order (deterministic; mse_linear_fwd_ws sums element-strided, so the two losses agree after the float cast at the
// tested sizes, not by construction).
constexpr int kCmThreads = 256;
constexpr int kCmMaxBlocks = 4096;
#ifndef ACN_CM_PROF
#define ACN_CM_PROF 0   // diagnostic build: per-ray section timestamps (acn_debug_cmprof_fetch)
#endif
#if ACN_CM_PROF
__device__ unsigned long long g_cmprof[4096 * 8];
__device__ unsigned long long g_cmblk[4096 * 4];
#define CM_MARK(i) if (lane == 0 && ray < 4096) g_cmprof[ray * 8 + (i)] = wall_clock64();
#define CM_BLK(i) if (threadIdx.x == 0 && blockIdx.x < 4096) g_cmblk[blockIdx.x * 4 + (i)] = wall_clock64();
#else
#define CM_MARK(i)
#define CM_BLK(i)
#endif
constexpr int kCmMaxS = 1024;   // the per-wave LDS rows of S float4 + S float (4 waves: 80 KB at S = 1024)
// a wave's LDS writes visible to its own later reads (in-order LDS; keeps the compiler from reordering)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__global__ void __launch_bounds__(kCmThreads) composite_mse_train_kernel(
    BgArgs bg, const float* __restrict__ rays, const float4* __restrict__ y, const float* __restrict__ pw,
    const int32_t* __restrict__ pmap, int K, const float* __restrict__ tv, const float* __restrict__ gt, int64_t N,
    int S, const float* __restrict__ g_loss, float* __restrict__ rgb_out, float* __restrict__ dirs_out,
    float* __restrict__ g_bg, float4* __restrict__ gy, const int32_t* __restrict__ pidx,
    const int64_t* __restrict__ live, int64_t P, double* __restrict__ partials, unsigned int* __restrict__ counter,
    float* __restrict__ loss) {
    extern __shared__ float4 cm_rows[];   // [4 waves][S] float4: blended rgb_sigma, then dL/d(rgb_sigma); then
                                          // [4 waves][S] float: the ray's t_vals
    __shared__ double red[kCmThreads / 64];
    __shared__ bool last;
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wv = threadIdx.x >> 6;
    CM_BLK(0)
    float4* row = cm_rows + wv * S;
    float* trow = reinterpret_cast<float*>(cm_rows + (kCmThreads / 64) * S) + wv * S;
    const int64_t nw = (int64_t)gridDim.x * (kCmThreads >> 6);
    const int64_t n = 3 * N;
    const float gl = g_loss[0];
    double lsum = 0.0;
    // a sample's pair slots and weights: all its loads issued together (kept in registers for S <= 128, the
    // blend backward reuses them)
    int32_t pp[2][ACN_MAX_EXPERTS];
    float w[2][ACN_MAX_EXPERTS];
    auto load_pairs = [&](int64_t m, int u) {
        const int32_t* pm = pmap + m * K;
#pragma unroll
        for (int k = 0; k < ACN_MAX_EXPERTS; ++k) pp[u][k] = k < K ? pm[k] : -1;
#pragma unroll
        for (int k = 0; k < ACN_MAX_EXPERTS; ++k) w[u][k] = pp[u][k] >= 0 ? pw[pp[u][k]] : 0.0f;
    };
    for (int64_t ray = (int64_t)blockIdx.x * (kCmThreads >> 6) + wv; ray < N; ray += nw) {
        CM_MARK(0)
        const float dx = rays[8 * ray + 3], dy = rays[8 * ray + 4], dz = rays[8 * ray + 5];
        const int64_t m0 = ray * S;
        const float* tg = tv + m0;
        // blend (blend_fwd_kernel's order: acc + y_k w_k over k), every lane its own samples, 128 per round
        for (int s0 = 0; s0 < S; s0 += 128) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int s = s0 + 64 * u + lane;
                if (s < S) {
                    load_pairs(m0 + s, u);
                    trow[s] = tg[s];
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int s = s0 + 64 * u + lane;
                if (s >= S) continue;
                float4 v[ACN_MAX_EXPERTS];
#pragma unroll
                for (int k = 0; k < ACN_MAX_EXPERTS; ++k)
                    if (pp[u][k] >= 0) v[k] = y[pp[u][k]];
                float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
                for (int k = 0; k < ACN_MAX_EXPERTS; ++k) {
                    if (pp[u][k] < 0) continue;
                    acc.x = acc.x + v[k].x * w[u][k];
                    acc.y = acc.y + v[k].y * w[u][k];
                    acc.z = acc.z + v[k].z * w[u][k];
                    acc.w = acc.w + v[k].w * w[u][k];
                }
                row[s] = acc;
            }
        }
        CM_MARK(1)
        const float gt3[3] = {gt[3 * ray], gt[3 * ray + 1], gt[3 * ray + 2]};
        float c[3];
        background(bg, dx, dy, dz, lane, c);
        if (lane < 3) dirs_out[3 * ray + lane] = lane == 0 ? dx : (lane == 1 ? dy : dz);
        wave_lds_sync();
        CM_MARK(2)
        auto fetch = [&](int sc) { return row[sc]; };
        float r, g, b, dd, a;
        vr_fwd_ray(fetch, trow, S, 0, 0, 1.0f, j, h, nullptr, r, g, b, dd, a);
        const float om = 1.0f - a;
        const float pr[3] = {r + om * c[0], g + om * c[1], b + om * c[2]};
        float gq[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const float d = clamp01(pr[q]) - gt_linear(gt3[q]);
            lsum += (double)(d * d);
            const float gv = (float)((2.0 / (double)n) * (double)d * (double)gl);
            gq[q] = (pr[q] >= 0.0f && pr[q] <= 1.0f) ? gv : 0.0f;
        }
        if (lane == 0) {
            rgb_out[3 * ray] = pr[0];
            rgb_out[3 * ray + 1] = pr[1];
            rgb_out[3 * ray + 2] = pr[2];
        }
        CM_MARK(3)
        // the backward's second sweep reads sample s, then writes its gradient over it (same lane, same tile)
        const double acc = vr_bwd_ray(fetch, [&](int s, float4 o) { row[s] = o; }, trow, S, 1.0f, gq[0], gq[1],
                                      gq[2], 0.0f, 0.0f, c[0], c[1], c[2], nullptr, j, h);
        if (g_bg && lane == 0) {
            const float omb = 1.0f - (float)acc;
            g_bg[3 * ray] = omb * gq[0];
            g_bg[3 * ray + 1] = omb * gq[1];
            g_bg[3 * ray + 2] = omb * gq[2];
        }
        wave_lds_sync();
        CM_MARK(4)
        // blend backward (blend_bwd_kernel): every pair slot of sample s gets dL/d(rgb_sigma)_s * w
        for (int s0 = 0; s0 < S; s0 += 128) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int s = s0 + 64 * u + lane;
                if (s >= S) continue;
                if (S > 128) load_pairs(m0 + s, u);   // else: still in registers from the blend
                const float4 o = row[s];
#pragma unroll
                for (int k = 0; k < ACN_MAX_EXPERTS; ++k)
                    if (pp[u][k] >= 0)
                        gy[pp[u][k]] = make_float4(o.x * w[u][k], o.y * w[u][k], o.z * w[u][k], o.w * w[u][k]);
            }
        }
        wave_lds_sync();
        CM_MARK(5)
    }
    CM_BLK(1)
    // padding slots of the pair segments (pidx < 0 below the live count): zero gradients, as blend_bwd_kernel
    const int64_t nl = live ? (live[0] < P ? live[0] : P) : P;
    for (int64_t p = (int64_t)blockIdx.x * kCmThreads + threadIdx.x; p < nl; p += (int64_t)gridDim.x * kCmThreads)
        if (pidx[p] < 0) gy[p] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    CM_BLK(2)
    if (lane == 0) red[wv] = lsum;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < kCmThreads / 64; ++i) t += red[i];
        partials[blockIdx.x] = t;
        __threadfence();
        last = atomicAdd(counter, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (last) {   // the G partials in a fixed tree (thread i: partials i, i + 256, ...; xor tree; waves in order)
        __threadfence();
        double v = 0.0;
        for (unsigned int i = threadIdx.x; i < gridDim.x; i += kCmThreads)
            v += __hip_atomic_load(&partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) red[wv] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int i = 0; i < kCmThreads / 64; ++i) t += red[i];
            loss[0] = (float)(t / (double)n);
            counter[0] = 0u;
        }
        CM_BLK(3)
    }
}

// MetaContainer._routing as a standalone op: W (M, K) soft weights, or hard (M) argmin
__global__ void __launch_bounds__(256) routing_kernel(FieldCfg cfg, const float* __restrict__ pts, int64_t M, int64_t ld,
                                                      float* __restrict__ W, int32_t* __restrict__ hard) {
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    const float px = pts[m * ld], py = pts[m * ld + 1], pz = pts[m * ld + 2];
    if (cfg.routing == 1) {
        const RouteState st = route_prep<1>(cfg, px, py, pz);
        for (int k = 0; k < cfg.K; ++k) W[m * cfg.K + k] = route_weight(cfg, st, k, px, py, pz);
    } else {
        const RouteState st = route_prep<2>(cfg, px, py, pz);
        hard[m] = st.hard;
    }
}

// MetaContainer.background_color for N directions: one wave per direction
__global__ void __launch_bounds__(256) background_kernel(BgArgs bg, const float* __restrict__ d, int64_t N,
                                                         float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < N; i += nw) {
        float c[3];
        background(bg, d[3 * i], d[3 * i + 1], d[3 * i + 2], lane, c);
        if (lane < 3) out[3 * i + lane] = lane == 0 ? c[0] : (lane == 1 ? c[1] : c[2]);
    }
}

// Background head backward (the autograd of MetaContainer.background_color's bg_mlp, meta_container.py
// :347-382): per ray the forward is re-run (lane j = hidden unit j), then with do = g (1 - y) y
// (sigmoid_backward), dW2[c][j] += do_c h_j, db2 += do, dh_j = sum_c W2[c][j] do_c where h_j > 0
// (threshold_backward), dW1[j][:] += dh_j sh, db1[j] += dh_j.  Every wave of the fixed grid keeps its
// lane's sums for its rays (grid-stride) and writes them once; bg_bwd_reduce_kernel adds the waves'
// copies in wave order (deterministic, no atomics).
constexpr int kBgWaves = 256;   // 64 workgroups x 4 waves
constexpr int kBgLane = 23;     // per lane: dW1 row (16), db1, dW2 column (3), db2 (3, lane 0)
__global__ void __launch_bounds__(256) background_bwd_kernel(BgArgs bg, const float* __restrict__ d, int64_t N,
                                                             const float* __restrict__ g,
                                                             float* __restrict__ partial) {
    const int lane = threadIdx.x & 63;
    const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    float a[kBgLane];
#pragma unroll
    for (int i = 0; i < kBgLane; ++i) a[i] = 0.0f;
    const int H = bg.hidden;
    for (int64_t r = wave; r < N; r += kBgWaves) {
        const float dx = d[3 * r], dy = d[3 * r + 1], dz = d[3 * r + 2];
        const float n = clamp_min_nan(norm3(dx, dy, dz), 1e-12f);
        float sh[16];
        sh_encode<3>(dx / n, dy / n, dz / n, sh);
        float hv = 0.0f;
        if (lane < H) {
            float s = 0.0f;
            for (int k = 0; k < 16; ++k) s = fmaf(sh[k], bg.w1[lane * 16 + k], s);
            hv = s + bg.b1[lane];
            hv = hv < 0.0f ? 0.0f : hv;
        }
        float dov[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float v = lane < H ? hv * bg.w2[c * H + lane] : 0.0f;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            const float y = sigmoidf_(v + bg.b2[c]);
            dov[c] = (g[3 * r + c] * (1.0f - y)) * y;
        }
        if (lane < H) {
            float dh = 0.0f;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                a[17 + c] += dov[c] * hv;
                dh += bg.w2[c * H + lane] * dov[c];
            }
            dh = hv > 0.0f ? dh : 0.0f;
#pragma unroll
            for (int k = 0; k < 16; ++k) a[k] += dh * sh[k];
            a[16] += dh;
        }
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < 3; ++c) a[20 + c] += dov[c];
        }
    }
    float* dst = partial + ((int64_t)wave * 64 + lane) * kBgLane;
#pragma unroll
    for (int i = 0; i < kBgLane; ++i) dst[i] = a[i];
}

// gw1 (H,16), gb1 (H), gw2 (3,H), gb2 (3): the sum of the waves' copies, in wave order
__global__ void __launch_bounds__(256) bg_bwd_reduce_kernel(const float* __restrict__ partial, int H,
                                                            float* __restrict__ gw1, float* __restrict__ gb1,
                                                            float* __restrict__ gw2, float* __restrict__ gb2) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;  // (lane, slot)
    if (e >= 64 * kBgLane) return;
    const int lane = e / kBgLane, i = e - lane * kBgLane;
    if (i >= 20 ? lane != 0 : lane >= H) return;
    // wave order, 32 copies' loads in flight per round (8 dependent rounds instead of 32: the launch is
    // memory latency, 13.7 us per call with 8 in flight)
    float s = 0.0f;
    for (int w0 = 0; w0 < kBgWaves; w0 += 32) {
        float v[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) v[u] = partial[((int64_t)(w0 + u) * 64 + lane) * kBgLane + i];
#pragma unroll
        for (int u = 0; u < 32; ++u) s += v[u];
    }
    if (i < 16) gw1[lane * 16 + i] = s;
    else if (i == 16) gb1[lane] = s;
    else if (i < 20) gw2[(i - 17) * H + lane] = s;
    else gb2[i - 20] = s;
}

// ------------------------------------------------------------------------------------------
int g_num_cus = 0;
int num_cus() {
    if (g_num_cus == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            g_num_cus = n;
        else
            g_num_cus = 256;
    }
    return g_num_cus;
}

int check_expert(const acn_expert& e, int k) {
    ACN_REQUIRE(e.table, "expert %d: hash table is NULL", k);
    if (e.L != 16 || e.F != 2)
        return acn_set_error(ACN_ERR_UNSUPPORTED, "expert %d: fused path needs levels*features = 16*2 (got %d*%d)", k, e.L, e.F);
    ACN_REQUIRE(e.log2T >= 1 && e.log2T <= 30, "expert %d: log2_hashmap_size must be in [1, 30]", k);
    ACN_REQUIRE(e.interp >= 0 && e.interp <= 2, "expert %d: bad interpolation", k);
    const float* ptrs[] = {e.sig_w0, e.sig_b0, e.sig_w1, e.sig_b1, e.sigh_w, e.sigh_b, e.geo_w,
                           e.geo_b, e.col_w0, e.col_b0, e.col_w1, e.col_b1, e.col_w2, e.col_b2};
    for (const float* q : ptrs) ACN_REQUIRE(q, "expert %d: NULL MLP weight/bias pointer", k);
    return ACN_OK;
}

// Builds FieldCfg + packs weights into the workspace.  Returns status; sets *interp.
int prepare(const acn_expert* experts, const acn_routing* routing, int active_module, void* workspace,
            size_t workspace_bytes, hipStream_t s, FieldCfg& cfg, int& interp, int& Keval, bool do_pack) {
    ACN_REQUIRE(experts && routing, "NULL experts/routing");
    const int K = routing->K;
    ACN_REQUIRE(K >= 1 && K <= ACN_MAX_EXPERTS, "routing.K must be in [1, %d], got %d", ACN_MAX_EXPERTS, K);
    ACN_REQUIRE(active_module < K, "active_module %d out of range for K=%d", active_module, K);
    const int k0 = active_module >= 0 ? active_module : 0;
    Keval = active_module >= 0 ? 1 : K;
    ACN_REQUIRE(workspace && workspace_bytes >= (size_t)Keval * PK_BYTES, "workspace too small: need %zu bytes",
                (size_t)Keval * PK_BYTES);
    ACN_REQUIRE(((uintptr_t)workspace & 15) == 0, "workspace must be 16-byte aligned");
    interp = experts[k0].interp;
    const int log2T = experts[k0].log2T;
    PackArgs pa{};
    for (int i = 0; i < Keval; ++i) {
        const acn_expert& e = experts[k0 + i];
        int st = check_expert(e, k0 + i);
        if (st) return st;
        if (e.interp != interp || e.log2T != log2T)
            return acn_set_error(ACN_ERR_UNSUPPORTED, "experts must share interpolation and log2_hashmap_size");
        ExpertMeta& m = cfg.ex[i];
        m.table = e.table;
        for (int a = 0; a < 3; ++a) {
            m.amin[a] = e.aabb_min[a];
            m.ext[a] = e.aabb_extent[a];
            m.rext[a] = 1.0f / e.aabb_extent[a];
        }
        for (int l = 0; l < 16; ++l) m.res[l] = e.res[l];
        pa.e[i] = PackSrc{e.sig_w0, e.sig_b0, e.sig_w1, e.sig_b1, e.sigh_w, e.sigh_b, e.geo_w, e.geo_b,
                          e.col_w0, e.col_b0, e.col_w1, e.col_b1, e.col_w2, e.col_b2};
    }
    cfg.K = Keval;
    cfg.log2T = log2T;
    cfg.cluster_2d = routing->cluster_2d;
    cfg.bm = routing->boundary_margin;
    // single expert (active_module, or K == 1 whose soft weight is exactly 1 / argmin is 0): no routing
    if (active_module >= 0 || K == 1) cfg.routing = 0;
    else cfg.routing = routing->boundary_margin > 1.0f ? 1 : 2;
    for (int k = 0; k < K && active_module < 0; ++k)
        for (int a = 0; a < 3; ++a) cfg.cent[k][a] = routing->centroids[k][a];
    if (do_pack) {
        hipLaunchKernelGGL(pack_kernel, dim3((PK_FLOATS + 255) / 256, Keval), dim3(256), 0, s, pa, Keval,
                           (float*)workspace);
        return acn_check_launch("acn_pack_experts");
    }
    return ACN_OK;
}

}  // namespace

// interpolation x weight residency x routing.  Single-expert launches (ROUTE 0) use one LDS image;
// routed launches keep K <= 2 experts in LDS and read K > 2 packed images from L2.
#define ACN_DISPATCH_I(L, I)                                           \
    do {                                                               \
        if (cfg.routing == 0) L(I, 1, 0);                              \
        else if (cfg.routing == 1) { if (K == 2) L(I, 2, 1); else L(I, 0, 1); } \
        else { if (K == 2) L(I, 2, 2); else L(I, 0, 2); }              \
    } while (0)
#define ACN_DISPATCH(L)                                                \
    do {                                                               \
        if (interp == 1) ACN_DISPATCH_I(L, 1);                         \
        else if (interp == 0) ACN_DISPATCH_I(L, 0);                    \
        else ACN_DISPATCH_I(L, 2);                                     \
    } while (0)

// Training-path sampler: stratified_t_vals (ray_rendering.py:262-287, jitter from caller uniforms), the
// sample points o + d t (:318-320), MetaNGP._world_to_unit (meta_ngp.py:155-158) of the expert's box and
// the colour-branch SH of the ray direction (meta_ngp.py:165-168, encodings.py:144-151), one lane per
// sample, the same roundings as those torch ops (bitwise).  Replaces ~20 elementwise launches per call.
__global__ void __launch_bounds__(256) sample_train_kernel(const float* __restrict__ rays, int64_t N, int S,
                                                           const float* __restrict__ jit, float3 amin, float3 ext,
                                                           float lo, float hi, float* __restrict__ t_out,
                                                           float* __restrict__ x01, float* __restrict__ sh_out) {
    const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (m >= N * (int64_t)S) return;
    const int64_t ray = m / S;
    const int s = (int)(m - ray * S);
    const float* rp = rays + ray * 8;
    const float ox = rp[0], oy = rp[1], oz = rp[2], dx = rp[3], dy = rp[4], dz = rp[5];
    const float t = tval(rp[6], rp[7], s, S, jit ? jit + ray * S : nullptr);
    t_out[m] = t;
    const float px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;
    x01[m * 3 + 0] = clamp_nan((px - amin.x) / ext.x, lo, hi);
    x01[m * 3 + 1] = clamp_nan((py - amin.y) / ext.y, lo, hi);
    x01[m * 3 + 2] = clamp_nan((pz - amin.z) / ext.z, lo, hi);
    float sh[16];
    dir_sh(dx, dy, dz, sh);
    float4* o4 = reinterpret_cast<float4*>(sh_out + m * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) o4[q] = make_float4(sh[4 * q], sh[4 * q + 1], sh[4 * q + 2], sh[4 * q + 3]);
}

// Visiting order of a small batch (N <= ACN_ORDER_MAX): rays grouped by direction, so that the XCD
// bands of render_kernel become compact image regions (a random pixel batch otherwise spreads every
// XCD's samples over the whole frame and its 4 MB L2 serves the hash cells of all of it).  One
// workgroup: the batch's mean direction m and an orthonormal pair (e1, e2) perpendicular to it; every
// ray's gnomonic coordinates (d.e1 / d.m, d.e2 / d.m) (for one camera: its image-plane position),
// quantised to a 64 x 64 grid over the batch's bounding box and Z-ordered; a STABLE sort of the rays by
// cell (two 6-bit LSD radix passes, rank inside a wave by ballot multisplit, so rays of one cell keep
// their index order and the visiting order is reproducible run to run).
// Only the order changes: each ray is still rendered alone and its outputs written at its own index,
// so results are bit-identical to the given order.  Rays with a non-finite direction or d.m <= 0
// go to the last cell.
#define ACN_ORDER_MAX 8192
#define ACN_ORDER_BINS 4096
#ifndef ACN_ORDER_COUNTING
#define ACN_ORDER_COUNTING 1  // stable counting sort with per-cell ranks (0: the two stable radix passes always)
#endif
__device__ __forceinline__ uint32_t spread6(uint32_t v) {
    v &= 63u;
    v = (v | (v << 4)) & 0x30Fu;
    v = (v | (v << 2)) & 0x333u;
    v = (v | (v << 1)) & 0x555u;
    return v;
}
// workgroup-wide reductions (1024 threads = 16 waves) of 3 sums / 4 maxima; every thread gets the result
// DPP within each 16-lane row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then the
// four row results through scalar readlanes: no LDS round trips (a ds_bpermute shuffle ladder costs six
// dependent LDS latencies per value)
template <int OP>
__device__ __forceinline__ float wave_reduce(float v) {
    auto op = [](float a, float b) { return OP == 0 ? a + b : fmaxf(a, b); };
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return op(op(r0, r1), op(r2, r3));
}
template <int OP>
__device__ __forceinline__ void block_reduce3(float& a, float& b, float& c, float* red) {
    a = wave_reduce<OP>(a), b = wave_reduce<OP>(b), c = wave_reduce<OP>(c);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = a, red[16 + w] = b, red[32 + w] = c;
    __syncthreads();
    a = red[0], b = red[16], c = red[32];
    for (int k = 1; k < 16; ++k) a += red[k], b += red[16 + k], c += red[32 + k];
    __syncthreads();  // red[] reuse
}
__device__ __forceinline__ void block_reduce4max(float& a, float& b, float& c, float& d, float* red) {
    a = wave_reduce<1>(a), b = wave_reduce<1>(b), c = wave_reduce<1>(c), d = wave_reduce<1>(d);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = a, red[16 + w] = b, red[32 + w] = c, red[48 + w] = d;
    __syncthreads();
    for (int k = 0; k < 16; ++k)
        a = fmaxf(a, red[k]), b = fmaxf(b, red[16 + k]), c = fmaxf(c, red[32 + k]), d = fmaxf(d, red[48 + k]);
    __syncthreads();
}
__device__ __forceinline__ bool dir_ok(float x, float y, float z) {
    const float n2 = x * x + y * y + z * z;
    return n2 > 0.0f && n2 < 3.0e38f;  // finite, non-zero
}
// One stable LSD radix pass over N <= ACN_ORDER_MAX 16-bit keys by digit (key >> shift) & 63, 1024 threads.
// Wave w owns the contiguous input block [w B, (w + 1) B); per (digit, wave) counts cnt[digit * 16 + w]
// are scanned digit-major, so the output keeps every digit's elements in input order: within a wave
// chunk by the lanes below with the same digit, across chunks by the wave's running offset, across
// waves by the scan.  iin == NULL: the input indices are the positions.  FINAL: write idx to order[].
template <bool FINAL>
__device__ __forceinline__ void radix_pass6(const uint16_t* kin, const uint16_t* iin, int shift, int N, int* cnt,
                                            int* wsum, uint16_t* kout, uint16_t* iout, int32_t* __restrict__ order) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int B = (((N + 15) >> 4) + 63) & ~63;
    const int lo = w * B, hi = min(N, lo + B);
    cnt[tid] = 0;
    __syncthreads();
    for (int p0 = lo; p0 < hi; p0 += 64) {
        const int pos = p0 + lane;
        const bool v = pos < hi;
        const int dig = v ? (kin[pos] >> shift) & 63 : 0;
        const uint64_t m = same_digit_lanes(v, dig);
        if (v && lanes_below(m) == 0) cnt[dig * 16 + w] += __popcll(m);
    }
    __syncthreads();
    const int val = cnt[tid];
    const int incl = wave_incl_scan(val);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int base = incl - val;
    for (int k = 0; k < w; ++k) base += wsum[k];
    cnt[tid] = base;
    __syncthreads();
    for (int p0 = lo; p0 < hi; p0 += 64) {
        const int pos = p0 + lane;
        const bool v = pos < hi;
        const uint16_t key = v ? kin[pos] : (uint16_t)0;
        const int dig = (key >> shift) & 63;
        const uint64_t m = same_digit_lanes(v, dig);
        const int below = lanes_below(m);
        const int run = v ? cnt[dig * 16 + w] : 0;
        if (v) {
            const int dst = run + below;
            const int idx = iin ? (int)iin[pos] : pos;
            if (FINAL) {
                order[dst] = idx;
            } else {
                kout[dst] = key;
                iout[dst] = (uint16_t)idx;
            }
        }
        if (v && below == 0) cnt[dig * 16 + w] = run + __popcll(m);
    }
    __syncthreads();
}
__global__ void __launch_bounds__(1024) ray_order_kernel(const float* __restrict__ rays, int N,
                                                         int32_t* __restrict__ order) {
    constexpr int PER = ACN_ORDER_MAX / 1024;
    __shared__ int cnt[1024];
    __shared__ __attribute__((aligned(16))) float dir[3][ACN_ORDER_MAX];
    __shared__ uint16_t cell_of[ACN_ORDER_MAX];
    __shared__ int wsum[16];
    __shared__ float red[16 * 4];
    const int tid = threadIdx.x;
    // one pass over global memory, every load of the thread in flight at once
    float sx = 0.0f, sy = 0.0f, sz = 0.0f;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int i = tid + q * 1024;
        if (i < N) {
            const float* rp = rays + (int64_t)i * 8;
            const float x = rp[3], y = rp[4], z = rp[5];
            dir[0][i] = x, dir[1][i] = y, dir[2][i] = z;
            if (dir_ok(x, y, z)) {
                const float r = rsqrtf(x * x + y * y + z * z);
                sx += x * r, sy += y * r, sz += z * r;
            }
        }
    }
#if ACN_ORDER_DIAG == 3  // diagnostic only (tools/order_diag.sh): loads, then the identity order
    for (int i = tid; i < N; i += 1024) order[i] = i + (int)(sx * 0.0f);
    return;
#endif
    block_reduce3<0>(sx, sy, sz, red);
    const float mn = sqrtf(sx * sx + sy * sy + sz * sz);
    float mx = 0.0f, my = 0.0f, mz = 1.0f;
    if (mn > 0.0f && mn < 3.0e38f) mx = sx / mn, my = sy / mn, mz = sz / mn;
    // e1 = normalize(m x a) with a the axis least aligned with m; e2 = m x e1
    float ax = 0.0f, ay = 0.0f, az = 0.0f;
    if (fabsf(mx) <= fabsf(my) && fabsf(mx) <= fabsf(mz)) ax = 1.0f;
    else if (fabsf(my) <= fabsf(mz)) ay = 1.0f;
    else az = 1.0f;
    float e1x = my * az - mz * ay, e1y = mz * ax - mx * az, e1z = mx * ay - my * ax;
    const float e1n = rsqrtf(e1x * e1x + e1y * e1y + e1z * e1z);
    e1x *= e1n, e1y *= e1n, e1z *= e1n;
    const float e2x = my * e1z - mz * e1y, e2y = mz * e1x - mx * e1z, e2z = mx * e1y - my * e1x;
    auto coords = [&](int i, float& u, float& v) -> bool {
        const float x = dir[0][i], y = dir[1][i], z = dir[2][i];
        if (!dir_ok(x, y, z)) return false;
        const float dm = x * mx + y * my + z * mz;
        if (!(dm > 0.0f)) return false;
        u = (x * e1x + y * e1y + z * e1z) / dm;
        v = (x * e2x + y * e2y + z * e2z) / dm;
        return fabsf(u) < 1.0e30f && fabsf(v) < 1.0e30f;
    };
    float umin = 3.0e38f, vmin = 3.0e38f, umax = -3.0e38f, vmax = -3.0e38f;
    // each thread's (u, v) kept in registers for the cell pass below (one coordinate pass over dir[], not two)
    float cu[PER], cv[PER];
    bool cok[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int i = tid + q * 1024;
        cok[q] = i < N && coords(i, cu[q], cv[q]);
        if (cok[q]) umin = fminf(umin, cu[q]), umax = fmaxf(umax, cu[q]), vmin = fminf(vmin, cv[q]), vmax = fmaxf(vmax, cv[q]);
    }
#if ACN_ORDER_DIAG == 2  // diagnostic only: + mean direction and the coordinate pass, identity order
    for (int i = tid; i < N; i += 1024) order[i] = i + (int)(umin * 0.0f + umax * 0.0f);
    return;
#endif
#if ACN_ORDER_DIAG == 1  // diagnostic only: fixed range instead of the bounding-box reduction
    umin = -2.0f, vmin = -2.0f, umax = 2.0f, vmax = 2.0f;
#else
    umin = -umin, vmin = -vmin;  // one max-reduction for all four
    block_reduce4max(umin, vmin, umax, vmax, red);
    umin = -umin, vmin = -vmin;
#endif
    const float su = umax > umin ? 63.999f / (umax - umin) : 0.0f;
    const float sv = vmax > vmin ? 63.999f / (vmax - vmin) : 0.0f;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int i = tid + q * 1024;
        if (i >= N) break;
        int c = ACN_ORDER_BINS - 1;
        if (cok[q]) {
            const uint32_t qu = (uint32_t)fminf(fmaxf((cu[q] - umin) * su, 0.0f), 63.0f);
            const uint32_t qv = (uint32_t)fminf(fmaxf((cv[q] - vmin) * sv, 0.0f), 63.0f);
            c = (int)(spread6(qu) | (spread6(qv) << 1));
        }
        cell_of[i] = (uint16_t)c;
    }
    __syncthreads();  // dir[] is free from here on
#if ACN_ORDER_COUNTING
    // Counting sort by cell, made stable per cell afterwards: histogram (LDS atomics), scan, an unordered
    // scatter of the indices into their cell's slice, then every element's rank inside its slice = the number
    // of slice members with a smaller index (cells hold a few rays each: 4096 rays over 4096 cells).  A cell
    // holding more than kOrderSlice rays (degenerate batches: many identical directions) takes the two
    // stable radix passes instead, so the rank scan never goes quadratic.
    {
        constexpr int kOrderSlice = 64;
        int* bins = reinterpret_cast<int*>(&dir[2][0]);     // ACN_ORDER_BINS ints: counts, then slice ends
        int* start = reinterpret_cast<int*>(&dir[1][0]);    // ACN_ORDER_BINS ints: slice starts
        uint16_t* lst = reinterpret_cast<uint16_t*>(&dir[0][0]);
        __shared__ int maxc;
        if (tid == 0) maxc = 0;
        for (int b = tid; b < ACN_ORDER_BINS; b += 1024) bins[b] = 0;
        __syncthreads();
        int mloc = 0;
        for (int i = tid; i < N; i += 1024) {
            const int c = atomicAdd(&bins[cell_of[i]], 1) + 1;
            mloc = c > mloc ? c : mloc;
        }
        if (mloc > kOrderSlice) atomicMax(&maxc, mloc);
        __syncthreads();
        if (maxc == 0) {
            constexpr int BPT = ACN_ORDER_BINS / 1024;          // consecutive bins per thread
            int c[BPT], tot = 0;
#pragma unroll
            for (int q = 0; q < BPT; ++q) tot += (c[q] = bins[tid * BPT + q]);
            const int lane = tid & 63, w = tid >> 6;
            const int incl = wave_incl_scan(tot);
            if (lane == 63) wsum[w] = incl;
            __syncthreads();
            int base = incl - tot;
            for (int k = 0; k < w; ++k) base += wsum[k];
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                start[tid * BPT + q] = base;
                bins[tid * BPT + q] = base;   // scatter cursor, ends at the slice end
                base += c[q];
            }
            __syncthreads();
            for (int i = tid; i < N; i += 1024) lst[atomicAdd(&bins[cell_of[i]], 1)] = (uint16_t)i;
            __syncthreads();
            for (int i = tid; i < N; i += 1024) {
                const int cl = cell_of[i], s0 = start[cl], s1 = bins[cl];
                int r = 0;
                for (int j = s0; j < s1; ++j) r += (int)lst[j] < i ? 1 : 0;
                order[s0 + r] = i;
            }
            return;
        }
        __syncthreads();
    }
#endif
    uint16_t* key1 = reinterpret_cast<uint16_t*>(&dir[0][0]);
    uint16_t* idx1 = reinterpret_cast<uint16_t*>(&dir[1][0]);
    radix_pass6<false>(cell_of, nullptr, 0, N, cnt, wsum, key1, idx1, nullptr);
    radix_pass6<true>(key1, idx1, 6, N, cnt, wsum, nullptr, nullptr, order);
}

extern "C" size_t acn_workspace_bytes(int K) { return (size_t)(K < 1 ? 1 : K) * PK_BYTES; }

extern "C" size_t acn_render_order_bytes(int64_t N) {
    if (N < 1) return 0;
    return N <= ACN_ORDER_MAX ? (size_t)N * sizeof(int32_t) : 0;
}

extern "C" int acn_ray_order(const float* rays, int64_t N, int32_t* order, void* stream) {
    ACN_REQUIRE(N >= 1 && N <= ACN_ORDER_MAX, "acn_ray_order: N must be in [1, %d], got %lld", ACN_ORDER_MAX,
                (long long)N);
    ACN_REQUIRE(rays && order, "acn_ray_order: NULL pointer");
    hipLaunchKernelGGL(ray_order_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, rays, (int)N, order);
    return acn_check_launch("acn_ray_order");
}

extern "C" int acn_pack_experts(const acn_expert* experts, const acn_routing* routing, int active_module,
                                void* workspace, size_t workspace_bytes, void* stream) {
    FieldCfg cfg{};
    int interp, K;
    return prepare(experts, routing, active_module, workspace, workspace_bytes, (hipStream_t)stream, cfg, interp, K,
                   true);
}

extern "C" int acn_field_fwd(const float* x, int64_t M, int64_t ld, const acn_expert* experts,
                             const acn_routing* routing, int active_module, void* workspace, size_t workspace_bytes,
                             float* out, void* stream) {
    ACN_REQUIRE(M >= 0 && ld >= 6, "acn_field_fwd: x must be (N, D>=6)");
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(x && out, "acn_field_fwd: NULL pointer");
    hipStream_t s = (hipStream_t)stream;
    FieldCfg cfg{};
    int interp, K;
    int st = prepare(experts, routing, active_module, workspace, workspace_bytes, s, cfg, interp, K, false);
    if (st) return st;
    FieldParams p{x, M, ld, (const float*)workspace, out};
    const int64_t ntiles = (M + 31) / 32;
    const int64_t wgs = (ntiles + 15) / 16;
    const dim3 grid((unsigned)(wgs < num_cus() ? wgs : num_cus())), block(1024);
#define ACN_FIELD_LAUNCH(I, KL, R) hipLaunchKernelGGL((field_kernel<I, KL, R>), grid, block, 0, s, cfg, p)
    ACN_DISPATCH(ACN_FIELD_LAUNCH);
#undef ACN_FIELD_LAUNCH
    return acn_check_launch("acn_field_fwd");
}

extern "C" int acn_render_stratified_fwd(const float* rays, int64_t N, int S, const float* jitter,
                                         const acn_expert* experts, const acn_routing* routing, int active_module,
                                         const acn_background* bg, float sigma_scale, float tau, void* workspace,
                                         size_t workspace_bytes, float* rgb, float* depth, float* weights, float* acc,
                                         void* stream) {
    return acn_render_stratified_fwd_ordered(rays, N, S, jitter, experts, routing, active_module, bg, sigma_scale, tau,
                                             workspace, workspace_bytes, rgb, depth, weights, acc, nullptr, 0, stream);
}

extern "C" int acn_render_stratified_fwd_ordered(const float* rays, int64_t N, int S, const float* jitter,
                                                 const acn_expert* experts, const acn_routing* routing,
                                                 int active_module, const acn_background* bg, float sigma_scale,
                                                 float tau, void* workspace, size_t workspace_bytes, float* rgb,
                                                 float* depth, float* weights, float* acc, void* order_scratch,
                                                 size_t order_bytes, void* stream) {
    ACN_REQUIRE(N >= 0, "acn_render_stratified_fwd: N must be >= 0");
    ACN_REQUIRE(S >= 2, "acn_render_stratified_fwd: ray_samples must be >= 2, got %d", S);
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(rays && rgb && depth && acc, "acn_render_stratified_fwd: NULL pointer");
    ACN_REQUIRE(bg, "acn_render_stratified_fwd: NULL background");
    if (bg->mode == ACN_BG_MLP) {
        ACN_REQUIRE(bg->w1 && bg->b1 && bg->w2 && bg->b2, "background MLP pointers are NULL");
        ACN_REQUIRE(bg->hidden >= 1 && bg->hidden <= 64, "bg_hidden must be in [1, 64], got %d", bg->hidden);
    }
    hipStream_t s = (hipStream_t)stream;
    FieldCfg cfg{};
    int interp, K;
    int st = prepare(experts, routing, active_module, workspace, workspace_bytes, s, cfg, interp, K, false);
    if (st) return st;
    BgArgs b{bg->mode, bg->hidden, {bg->color[0], bg->color[1], bg->color[2]}, bg->w1, bg->b1, bg->w2, bg->b2};
    RenderParams p{rays, N, S, jitter, (const float*)workspace, sigma_scale, tau, rgb, depth, weights, acc, nullptr};
    int64_t wgs = (N + 15) / 16;
    if ((num_cus() & 7) == 0) wgs = (wgs + 7) & ~(int64_t)7;  // whole XCD bands (render_kernel)
    const dim3 grid((unsigned)(wgs < num_cus() ? wgs : num_cus())), block(1024);
    const bool slots = ACN_SLOTS && cfg.routing != 0 && K != 2;  // render_slots_kernel keeps its own order
    if (order_scratch && !slots && N <= ACN_ORDER_MAX && order_bytes >= (size_t)N * sizeof(int32_t)) {
        hipLaunchKernelGGL(ray_order_kernel, dim3(1), dim3(1024), 0, s, rays, (int)N, (int32_t*)order_scratch);
        p.order = (const int32_t*)order_scratch;
    }
    const bool wss = ACN_RENDER_WSS && S <= kWssMaxS(8) && !(tau > 0.0f);   // routed, no early termination: depth tiles
    const bool wss16 = ACN_WSS_RAYS16 && S <= kWssMaxS(16);
#define ACN_RENDER_LAUNCH(I, KL, R)                                                                    \
    do {                                                                                              \
        if (ACN_SLOTS && KL == 0 && R != 0 && wss && wss16) hipLaunchKernelGGL((render_wss_kernel<I, (R == 0 ? 1 : R), 16>), grid, dim3(ACN_SLOTS_THREADS), 0, s, cfg, b, p); \
        else if (ACN_SLOTS && KL == 0 && R != 0 && wss) hipLaunchKernelGGL((render_wss_kernel<I, (R == 0 ? 1 : R), 8>), grid, dim3(ACN_SLOTS_THREADS), 0, s, cfg, b, p); \
        else if (ACN_SLOTS && KL == 0 && R != 0) hipLaunchKernelGGL((render_slots_kernel<I, (R == 0 ? 1 : R)>), grid, dim3(ACN_SLOTS_THREADS), 0, s, cfg, b, p); \
        else hipLaunchKernelGGL((render_kernel<I, KL, R>), grid, block, 0, s, cfg, b, p);            \
    } while (0)
    if (ACN_RENDER_WS && cfg.routing == 0 && S <= kWsMaxS && !(tau > 0.0f)) {
        // one expert, no early termination: the workgroup shares its rays' field tiles (bit-identical outputs)
        if (interp == 1) hipLaunchKernelGGL(render_ws_kernel<1>, grid, block, 0, s, cfg, b, p);
        else if (interp == 0) hipLaunchKernelGGL(render_ws_kernel<0>, grid, block, 0, s, cfg, b, p);
        else hipLaunchKernelGGL(render_ws_kernel<2>, grid, block, 0, s, cfg, b, p);
        return acn_check_launch("acn_render_stratified_fwd");
    }
    ACN_DISPATCH(ACN_RENDER_LAUNCH);
#undef ACN_RENDER_LAUNCH
    return acn_check_launch("acn_render_stratified_fwd");
}

extern "C" int acn_volume_render_fwd(const float* rgb_sigma, const float* t_vals, const float* bg, int64_t N, int S,
                                     int raw_rgb, int raw_sigma, float sigma_scale, float* rgb, float* depth,
                                     float* weights, float* acc, void* stream) {
    ACN_REQUIRE(N >= 0 && S >= 2, "acn_volume_render_fwd: need N >= 0 and S >= 2 (got S=%d)", S);
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(rgb_sigma && t_vals && rgb && depth && acc, "acn_volume_render_fwd: NULL pointer");
    const int64_t wgs = (N + 3) / 4;
    const dim3 grid((unsigned)(wgs < 4096 ? wgs : 4096)), block(256);
    hipLaunchKernelGGL(volume_render_kernel, grid, block, 0, (hipStream_t)stream, rgb_sigma, t_vals, bg, N, S, raw_rgb,
                       raw_sigma, sigma_scale, rgb, depth, weights, acc);
    return acn_check_launch("acn_volume_render_fwd");
}

extern "C" int acn_volume_render_bwd(const float* rgb_sigma, const float* t_vals, const float* bg, int64_t N, int S,
                                     float sigma_scale, const float* g_rgb, const float* g_depth,
                                     const float* g_weights, const float* g_acc, float* g_rgb_sigma, float* g_bg,
                                     void* stream) {
    ACN_REQUIRE(N >= 0 && S >= 2, "acn_volume_render_bwd: need N >= 0 and S >= 2 (got S=%d)", S);
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(rgb_sigma && t_vals && g_rgb_sigma, "acn_volume_render_bwd: NULL pointer");
    ACN_REQUIRE(!g_bg || bg, "acn_volume_render_bwd: g_bg requested without bg");
    const int64_t wgs = (N + 3) / 4;
    const dim3 grid((unsigned)(wgs < 8192 ? wgs : 8192)), block(256);
    hipLaunchKernelGGL(volume_render_bwd_kernel, grid, block, 0, (hipStream_t)stream, rgb_sigma, t_vals, bg, N, S,
                       sigma_scale, g_rgb, g_depth, g_weights, g_acc, g_rgb_sigma, g_bg);
    return acn_check_launch("acn_volume_render_bwd");
}

extern "C" size_t acn_composite_mse_train_workspace_bytes(void) { return kCmMaxBlocks * sizeof(double) + 16; }

extern "C" int acn_routed_composite_mse_train(const float* rays, int64_t N, int S, const float* t_vals,
                                              const float* pair_out, const float* pair_w, const int32_t* pmap, int K,
                                              const int32_t* pidx, int64_t P, const int64_t* live,
                                              const acn_background* bg, const float* rgbs, const float* g_loss,
                                              float* rgb, float* dirs, float* g_bg, float* g_pair_out, float* loss,
                                              void* workspace, size_t workspace_bytes, void* stream) {
    ACN_REQUIRE(N >= 1 && S >= 2 && S <= kCmMaxS && K >= 1 && K <= ACN_MAX_EXPERTS && P >= 0 && bg,
                "acn_routed_composite_mse_train: bad sizes (N=%lld S=%d K=%d P=%lld)", (long long)N, S, K,
                (long long)P);
    ACN_REQUIRE(rays && t_vals && pmap && rgbs && g_loss && rgb && dirs && loss && workspace &&
                    (P == 0 || (pair_out && pair_w && pidx && g_pair_out)),
                "acn_routed_composite_mse_train: NULL pointer");
    ACN_REQUIRE(workspace_bytes >= acn_composite_mse_train_workspace_bytes(),
                "acn_routed_composite_mse_train: workspace too small");
    ACN_REQUIRE(((uintptr_t)pair_out & 15) == 0 && ((uintptr_t)g_pair_out & 15) == 0,
                "acn_routed_composite_mse_train: pair buffers must be 16-byte aligned");
    if (bg->mode == ACN_BG_MLP) {
        ACN_REQUIRE(bg->w1 && bg->b1 && bg->w2 && bg->b2, "background MLP pointers are NULL");
        ACN_REQUIRE(bg->hidden >= 1 && bg->hidden <= 64, "bg_hidden must be in [1, 64], got %d", bg->hidden);
    }
    BgArgs b{bg->mode, bg->hidden, {bg->color[0], bg->color[1], bg->color[2]}, bg->w1, bg->b1, bg->w2, bg->b2};
    int64_t wgs = (N + 3) / 4;
    wgs = wgs < kCmMaxBlocks ? wgs : kCmMaxBlocks;
    double* partials = (double*)workspace;
    unsigned int* counter = (unsigned int*)((char*)workspace + kCmMaxBlocks * sizeof(double));
    const size_t lds = (size_t)(kCmThreads / 64) * S * (sizeof(float4) + sizeof(float));
    hipLaunchKernelGGL(composite_mse_train_kernel, dim3((unsigned)wgs), dim3(kCmThreads), lds, (hipStream_t)stream, b,
                       rays, (const float4*)pair_out, pair_w, pmap, K, t_vals, rgbs, N, S, g_loss, rgb, dirs, g_bg,
                       (float4*)g_pair_out, pidx, live, P, partials, counter, loss);
    return acn_check_launch("acn_routed_composite_mse_train");
}

extern "C" int acn_routing_fwd(const float* pts, int64_t M, int64_t ld, const acn_routing* routing, float* weights,
                               int32_t* hard, void* stream) {
    ACN_REQUIRE(routing && routing->K >= 1 && routing->K <= ACN_MAX_EXPERTS, "acn_routing_fwd: bad routing");
    ACN_REQUIRE(M >= 0 && ld >= 3, "acn_routing_fwd: pts must be (N, >=3)");
    if (M == 0) return ACN_OK;
    const bool soft = routing->boundary_margin > 1.0f;
    ACN_REQUIRE(pts && (soft ? weights != nullptr : hard != nullptr), "acn_routing_fwd: NULL pointer");
    FieldCfg cfg{};
    cfg.K = routing->K;
    cfg.cluster_2d = routing->cluster_2d;
    cfg.bm = routing->boundary_margin;
    cfg.routing = soft ? 1 : 2;
    for (int k = 0; k < cfg.K; ++k)
        for (int a = 0; a < 3; ++a) cfg.cent[k][a] = routing->centroids[k][a];
    hipLaunchKernelGGL(routing_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, (hipStream_t)stream, cfg, pts, M,
                       ld, weights, hard);
    return acn_check_launch("acn_routing_fwd");
}

extern "C" size_t acn_background_bwd_workspace_bytes(void) { return (size_t)kBgWaves * 64 * kBgLane * sizeof(float); }

extern "C" int acn_background_bwd(const float* dirs, int64_t N, const acn_background* bg, const float* g_out,
                                  float* g_w1, float* g_b1, float* g_w2, float* g_b2, void* workspace,
                                  size_t workspace_bytes, void* stream) {
    ACN_REQUIRE(N >= 1 && bg && dirs && g_out && g_w1 && g_b1 && g_w2 && g_b2 && workspace,
                "acn_background_bwd: bad arguments");
    ACN_REQUIRE(bg->mode == ACN_BG_MLP && bg->w1 && bg->b1 && bg->w2 && bg->b2, "acn_background_bwd: MLP background only");
    ACN_REQUIRE(bg->hidden >= 1 && bg->hidden <= 64, "bg_hidden must be in [1, 64], got %d", bg->hidden);
    ACN_REQUIRE(workspace_bytes >= acn_background_bwd_workspace_bytes(), "acn_background_bwd: workspace too small");
    BgArgs b{bg->mode, bg->hidden, {bg->color[0], bg->color[1], bg->color[2]}, bg->w1, bg->b1, bg->w2, bg->b2};
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(background_bwd_kernel, dim3(kBgWaves / 4), dim3(256), 0, s, b, dirs, N, g_out, (float*)workspace);
    hipLaunchKernelGGL(bg_bwd_reduce_kernel, dim3((64 * kBgLane + 255) / 256), dim3(256), 0, s, (const float*)workspace,
                       bg->hidden, g_w1, g_b1, g_w2, g_b2);
    return acn_check_launch("acn_background_bwd");
}

extern "C" int acn_background_fwd(const float* dirs, int64_t N, const acn_background* bg, float* out, void* stream) {
    ACN_REQUIRE(N >= 0 && bg, "acn_background_fwd: bad arguments");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(dirs && out, "acn_background_fwd: NULL pointer");
    if (bg->mode == ACN_BG_MLP) {
        ACN_REQUIRE(bg->w1 && bg->b1 && bg->w2 && bg->b2, "background MLP pointers are NULL");
        ACN_REQUIRE(bg->hidden >= 1 && bg->hidden <= 64, "bg_hidden must be in [1, 64], got %d", bg->hidden);
    }
    BgArgs b{bg->mode, bg->hidden, {bg->color[0], bg->color[1], bg->color[2]}, bg->w1, bg->b1, bg->w2, bg->b2};
    const int64_t wgs = (N + 3) / 4;
    hipLaunchKernelGGL(background_kernel, dim3((unsigned)(wgs < 8192 ? wgs : 8192)), dim3(256), 0, (hipStream_t)stream,
                       b, dirs, N, out);
    return acn_check_launch("acn_background_fwd");
}

// ==========================================================================================
// Occupancy-grid renderer over PACKED samples (render_expert_occ ray_rendering.py:467-558 and the
// container's soft-MoE render_rays_occ :349-464, after nerfacc's marching / the boundary union):
// per ray, samples [t0, t1) at their midpoints -> field (single expert, or every expert whose
// routing weight exceeds 1e-8 with sigma-weighted blending BEFORE compositing) -> nerfacc
// compositing (alpha = 1 - exp(-sigma*dt), T = exp(-exclusive_sum(sigma*dt)), w = T*alpha) ->
// rgb / depth (at t_mid) / acc + (1 - acc) * background.  One wave per ray, 32 samples per tile,
// the MFMA field tile and SH fold of the stratified kernels; no (M,6) / (M,4) intermediates.
namespace {

struct OccRenderParams {
    const float* rays;
    int64_t ld, N;
    const int64_t *starts, *counts;
    const float *t0, *t1;
    const float* packed;
    float *rgb, *depth, *weights, *acc;
};

// meta_container blend of render_rays_occ (:426-449): s = clamp_min(sum_k W_k sigma_k, 1e-12),
// rgb = sum_k (W_k sigma_k) rgb_k / s, experts evaluated only where W_k > 1e-8.
template <int INTERP, int ROUTE, bool FOLD>
__device__ __forceinline__ void container_tile_occ(const FieldCfg& cfg, const float* Wbase, float px, float py,
                                                   float pz, const float (&shv)[8], float* cb, uint32_t* folded,
                                                   int lane, float& yr, float& yg, float& yb, float& ys) {
    if (ROUTE == 0) {
        container_tile<INTERP, 0, FOLD>(cfg, Wbase, px, py, pz, shv, cb, folded, lane, yr, yg, yb, ys);
        return;
    }
    const RouteState st = route_prep<ROUTE>(cfg, px, py, pz);
    float ns = 0.0f, nr = 0.0f, ng = 0.0f, nb = 0.0f;
    for (int k = 0; k < cfg.K; ++k) {
        const float wk = (ROUTE == 1) ? route_weight(cfg, st, k, px, py, pz) : (st.hard == k ? 1.0f : 0.0f);
        const bool need = wk > 1e-8f;
        if (__ballot(need) == 0ull) continue;
        const float* Wk = Wbase + (size_t)k * PK_FLOATS;
        float* cbk = FOLD ? cb + k * 64 : nullptr;
        if (FOLD && !((*folded >> k) & 1u)) {
            fold_sh_bias(Wk, shv, lane, cbk);
            *folded |= 1u << k;
        }
        float r, g, b, s;
        field_tile<INTERP, FOLD>(Wk, cfg.ex[k], cfg.log2T, px, py, pz, shv, cbk, lane, r, g, b, s);
        s = trunc_exp(s);
        if (need) {
            const float ws = wk * s;
            ns = ns + ws;
            nr = nr + ws * r;
            ng = ng + ws * g;
            nb = nb + ws * b;
        }
    }
    const float sn = clamp_min_nan(ns, 1e-12f);
    yr = nr / sn;
    yg = ng / sn;
    yb = nb / sn;
    ys = sn;
}

template <class FieldFn>
__device__ __forceinline__ void render_ray_packed(const OccRenderParams& p, const BgArgs& bg, int64_t ray, int lane,
                                                  FieldFn&& field) {
    const int j = lane & 31, h = lane >> 5;
    const float* rp = p.rays + ray * p.ld;
    const float ox = rp[0], oy = rp[1], oz = rp[2], dx = rp[3], dy = rp[4], dz = rp[5];
    const int64_t b = p.starts[ray], n = p.counts[ray];
    float sh[16], shv[8];
    dir_sh(dx, dy, dz, sh);
    sh_rows_for_half(sh, h, shv);
    uint32_t folded = 0u;
    double carry = 0.0;
    float ar = 0.0f, ag = 0.0f, ab = 0.0f, ad = 0.0f, aa = 0.0f;
    for (int64_t s0 = 0; s0 < n; s0 += 32) {
        const bool valid = s0 + j < n;
        const int64_t idx = b + (valid ? s0 + j : n - 1);
        const float ta = p.t0[idx], tb = p.t1[idx];
        const float tm = 0.5f * (ta + tb);
        const float px = ox + dx * tm, py = oy + dy * tm, pz = oz + dz * tm;
        float yr, yg, yb, ys;
        field(px, py, pz, shv, folded, yr, yg, yb, ys);
        const float sdt = valid ? ys * (tb - ta) : 0.0f;
        double incl = (double)sdt;
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) {
            const double y = __shfl_up(incl, off, 32);
            if (j >= off) incl += y;
        }
        const float excl = (float)(carry + incl - (double)sdt);
        const float alpha = 1.0f - expf(-sdt);
        const float w = expf(-excl) * alpha;
        if (valid && h == 0) {
            if (p.weights) p.weights[idx] = w;
            ar += w * yr;
            ag += w * yg;
            ab += w * yb;
            ad += w * tm;
            aa += w;
        }
        carry += __shfl(incl, 31, 32);
    }
    float bgc[3];
    background(bg, dx, dy, dz, lane, bgc);
    const float r = (float)wave32_sum((double)ar), g = (float)wave32_sum((double)ag), bb = (float)wave32_sum((double)ab);
    const float dd = (float)wave32_sum((double)ad), a = (float)wave32_sum((double)aa);
    if (lane == 0) {
        float orr = r, og = g, ob = bb;
        if (bg.mode != ACN_BG_NONE) {
            const float om = 1.0f - a;
            orr = r + om * bgc[0];
            og = g + om * bgc[1];
            ob = bb + om * bgc[2];
        }
        p.rgb[ray * 3 + 0] = orr;
        p.rgb[ray * 3 + 1] = og;
        p.rgb[ray * 3 + 2] = ob;
        p.depth[ray] = dd;
        p.acc[ray] = a;
    }
}

template <int INTERP, int KL, int ROUTE>
__global__ void __launch_bounds__(1024, 4) occ_render_kernel(FieldCfg cfg, BgArgs bg, OccRenderParams p) {
    constexpr bool FOLD = ACN_SHFOLD != 0;
    constexpr int KF = ROUTE == 0 ? 1 : (KL == 2 ? 2 : kMaxK);
    __shared__ __attribute__((aligned(16))) float smem[(KL > 0 ? KL : 1) * PK_FLOATS];
    __shared__ __attribute__((aligned(16))) float cbuf[FOLD ? 16 * KF * 64 : 4];
    const float* W = p.packed;
    if (KL > 0) {
        stage_weights<KL>(smem, p.packed);
        W = smem;
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* cb = FOLD ? cbuf + wave * KF * 64 : nullptr;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t ray = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave; ray < p.N; ray += nw) {
        render_ray_packed(p, bg, ray, lane,
                          [&](float px, float py, float pz, const float (&shv)[8], uint32_t& folded, float& yr,
                              float& yg, float& yb, float& ys) {
                              container_tile_occ<INTERP, ROUTE, FOLD>(cfg, W, px, py, pz, shv, cb, &folded, lane, yr,
                                                                      yg, yb, ys);
                          });
    }
}

}  // namespace

extern "C" int acn_render_packed_fwd(const float* rays, int64_t ld, int64_t N, const int64_t* chunk_starts,
                                     const int64_t* chunk_cnts, const float* t_starts, const float* t_ends,
                                     const acn_expert* experts, const acn_routing* routing, int active_module,
                                     const acn_background* bg, void* workspace, size_t workspace_bytes, float* rgb,
                                     float* depth, float* weights, float* acc, void* stream) {
    ACN_REQUIRE(N >= 0 && ld >= 6, "acn_render_packed_fwd: rays must be (N, >=6)");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(rays && chunk_starts && chunk_cnts && rgb && depth && acc, "acn_render_packed_fwd: NULL pointer");
    ACN_REQUIRE(bg, "acn_render_packed_fwd: NULL background");
    if (bg->mode == ACN_BG_MLP) {
        ACN_REQUIRE(bg->w1 && bg->b1 && bg->w2 && bg->b2, "background MLP pointers are NULL");
        ACN_REQUIRE(bg->hidden >= 1 && bg->hidden <= 64, "bg_hidden must be in [1, 64], got %d", bg->hidden);
    }
    hipStream_t s = (hipStream_t)stream;
    FieldCfg cfg{};
    int interp, K;
    int st = prepare(experts, routing, active_module, workspace, workspace_bytes, s, cfg, interp, K, false);
    if (st) return st;
    BgArgs b{bg->mode, bg->hidden, {bg->color[0], bg->color[1], bg->color[2]}, bg->w1, bg->b1, bg->w2, bg->b2};
    OccRenderParams p{rays, ld, N, chunk_starts, chunk_cnts, t_starts, t_ends, (const float*)workspace,
                      rgb, depth, weights, acc};
    const int64_t wgs = (N + 15) / 16;
    const dim3 grid((unsigned)(wgs < num_cus() ? wgs : num_cus())), block(1024);
#define ACN_OCC_LAUNCH(I, KL, R) hipLaunchKernelGGL((occ_render_kernel<I, KL, R>), grid, block, 0, s, cfg, b, p)
    ACN_DISPATCH(ACN_OCC_LAUNCH);
#undef ACN_OCC_LAUNCH
    return acn_check_launch("acn_render_packed_fwd");
}

extern "C" int acn_sample_stratified(const float* rays, int64_t N, int S, const float* jitter, const float* aabb_min,
                                     const float* aabb_extent, float lo, float hi, float* t_vals, float* x01,
                                     float* sh, void* stream) {
    ACN_REQUIRE(N >= 0 && S >= 1 && aabb_min && aabb_extent, "acn_sample_stratified: bad arguments");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(rays && t_vals && x01 && sh, "acn_sample_stratified: NULL pointer");
    const int64_t M = N * (int64_t)S;
    const float3 mn = make_float3(aabb_min[0], aabb_min[1], aabb_min[2]);
    const float3 ex = make_float3(aabb_extent[0], aabb_extent[1], aabb_extent[2]);
    hipLaunchKernelGGL(sample_train_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       rays, N, S, jitter, mn, ex, lo, hi, t_vals, x01, sh);
    return acn_check_launch("acn_sample_stratified");
}

extern "C" int acn_ep_field_fwd(const float* recv_xd, const int64_t* recv_cnt, int W, int E, int64_t cap,
                                const acn_expert* experts, const void* packed, size_t packed_bytes, float* ret,
                                void* stream) {
    return acn_ep_field_fwd_compact(recv_xd, recv_cnt, W, E, cap, cap, experts, packed, packed_bytes, ret, stream);
}

extern "C" int acn_ep_field_fwd_compact(const float* recv_xd, const int64_t* recv_cnt, int W, int E, int64_t cap,
                                        int64_t max_cnt, const acn_expert* experts, const void* packed,
                                        size_t packed_bytes, float* ret, void* stream) {
    ACN_REQUIRE(W >= 1 && E >= 1 && E <= kMaxK && cap >= 0 && (int64_t)W * E <= kEpMaxSeg && (cap > 0 || max_cnt >= 0),
                "acn_ep_field_fwd: bad arguments");
    ACN_REQUIRE(recv_xd && recv_cnt && experts && packed && ret, "acn_ep_field_fwd: NULL pointer");
    acn_routing rt{};
    rt.K = E;
    rt.boundary_margin = 1.0f;
    FieldCfg cfg{};
    int interp, K;
    int st = prepare(experts, &rt, -1, (void*)packed, packed_bytes, (hipStream_t)stream, cfg, interp, K, false);
    if (st) return st;
    int64_t g = 2 * (int64_t)num_cus();
    // wave-tiles to cover: W E segments of at most cap records (compact: at most max_cnt records each)
    const int64_t tiles = (int64_t)W * E * (((cap > 0 ? cap : max_cnt) + 31) / 32);
    const int64_t need = (tiles + kRtWaves - 1) / kRtWaves;
    if (need < g) g = need < 1 ? 1 : need;
    const dim3 grid((unsigned)g), block(kRtThreads);
    hipStream_t s = (hipStream_t)stream;
    if (interp == 1)
        hipLaunchKernelGGL(ep_field_kernel<1>, grid, block, 0, s, cfg, recv_xd, recv_cnt, W, E, cap, (const float*)packed, ret);
    else if (interp == 0)
        hipLaunchKernelGGL(ep_field_kernel<0>, grid, block, 0, s, cfg, recv_xd, recv_cnt, W, E, cap, (const float*)packed, ret);
    else
        hipLaunchKernelGGL(ep_field_kernel<2>, grid, block, 0, s, cfg, recv_xd, recv_cnt, W, E, cap, (const float*)packed, ret);
    return acn_check_launch("acn_ep_field_fwd");
}

extern "C" int acn_ep_composite(const float* rays, int64_t N, int S, const float* jitter, const float* yr, const float* pw,
                                const int32_t* pmap, int K, int hard, const acn_background* bg, float sigma_scale,
                                float tau, float* rgb, float* depth, float* weights, float* acc, void* stream) {
    ACN_REQUIRE(N >= 0 && S >= 2 && K >= 1 && K <= kMaxK, "acn_ep_composite: bad arguments");
    if (N == 0) return ACN_OK;
    ACN_REQUIRE(rays && yr && pw && pmap && bg && rgb && depth && acc, "acn_ep_composite: NULL pointer");
    if (bg->mode == ACN_BG_MLP) {
        ACN_REQUIRE(bg->w1 && bg->b1 && bg->w2 && bg->b2, "background MLP pointers are NULL");
        ACN_REQUIRE(bg->hidden >= 1 && bg->hidden <= 64, "bg_hidden must be in [1, 64], got %d", bg->hidden);
    }
    BgArgs b{bg->mode, bg->hidden, {bg->color[0], bg->color[1], bg->color[2]}, bg->w1, bg->b1, bg->w2, bg->b2};
    RenderParams p{rays, N, S, jitter, nullptr, sigma_scale, tau, rgb, depth, weights, acc, nullptr};
    int64_t wgs = (N + 15) / 16;
    const int64_t cap_g = 4 * (int64_t)num_cus();
    const dim3 grid((unsigned)(wgs < cap_g ? wgs : cap_g)), block(1024);
    hipStream_t s = (hipStream_t)stream;
    if (hard) hipLaunchKernelGGL(ep_composite_kernel<2>, grid, block, 0, s, b, p, yr, pw, pmap, K);
    else hipLaunchKernelGGL(ep_composite_kernel<1>, grid, block, 0, s, b, p, yr, pw, pmap, K);
    return acn_check_launch("acn_ep_composite");
}

#if ACN_SLOTS_PROF
extern "C" int acn_debug_slprof_fetch(unsigned long long* host, int max_rays) {
    const int m = max_rays < kSlProfRays ? max_rays : kSlProfRays;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_slprof), (size_t)m * 6 * sizeof(unsigned long long)) == hipSuccess
               ? m : -1;
}
#endif
#if ACN_CM_PROF
extern "C" int acn_debug_cmprof_fetch(unsigned long long* host, int max_rays) {
    const int m = max_rays < 4096 ? max_rays : 4096;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cmprof), (size_t)m * 8 * sizeof(unsigned long long)) == hipSuccess
               ? m : -1;
}
extern "C" int acn_debug_cmblk_fetch(unsigned long long* host, int max_blocks) {
    const int m = max_blocks < 4096 ? max_blocks : 4096;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cmblk), (size_t)m * 4 * sizeof(unsigned long long)) == hipSuccess
               ? m : -1;
}
#endif
#if ACN_FIELD_CHECK
extern "C" int acn_debug_fchk_fetch(uint32_t* host) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fchk), 3 * sizeof(uint32_t)) != hipSuccess) return -1;
    const uint32_t z[3] = {0u, 0u, 0u};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_fchk), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// records of the differing lanes (40 floats each); returns how many were recorded, clears the count
extern "C" int acn_debug_fchk_records(float* host, int max_records) {
    unsigned n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_fchk_n), sizeof(n)) != hipSuccess) return -1;
    n = n < kFchkMax ? n : kFchkMax;
    const unsigned m = n < (unsigned)max_records ? n : (unsigned)max_records;
    if (m && hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fchk_rec), (size_t)m * 40 * sizeof(float)) != hipSuccess) return -1;
    const unsigned z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_fchk_n), &z, sizeof(z)) != hipSuccess) return -1;
    return (int)m;
}
#endif
#if ACN_SLOTS_CHECK > 1
// diagnostic build only: copy out (and clear) the recorded self-check mismatches; returns their count
extern "C" int acn_debug_check_fetch(float* host, int max_records) {
    unsigned n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_chk_n), sizeof(n)) != hipSuccess) return -1;
    const unsigned m = n < (unsigned)max_records ? n : (unsigned)max_records;
    if (m && hipMemcpyFromSymbol(host, HIP_SYMBOL(g_chk), (size_t)m * 16 * sizeof(float)) != hipSuccess) return -1;
    const unsigned z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_chk_n), &z, sizeof(z)) != hipSuccess) return -1;
    return (int)n;
}
#endif
