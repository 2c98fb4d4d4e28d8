// mlp_train.hip -- the expert MLP of the training path on fp32 MFMA (gfx950).
//
// Replaces the differentiable MetaLinear chain of MetaNGP.density / color (models/inr/meta_ngp.py:
// 171-241, models/metamodule/metamodule.py: F.linear per layer, ReLU blocks, trunc_exp, cat with the SH
// encoding, sigmoid) and its autograd backward: ~11 small GEMMs, ~40 elementwise kernels and the bias
// reductions per call become
//   acn_mlp_train_fwd: one launch -> out (M, 4) = [sigmoid(rgb), trunc_exp(sigma)] and the layer
//                      inputs the weight gradients need, each with a ones column (the bias term);
//   acn_mlp_train_bwd: one launch -> d(hash features) (M, 32) and every layer's output gradient
//                      (after the ReLU / sigmoid / trunc_exp derivative);
// then one GEMM per layer on the caller's side gives [dW | db] = dY^T . [X | 1] (large-K GEMMs).
//
// Execution: one wave per 32-sample tile, lanes (sample j = lane & 31, half h = lane >> 5).  Every
// layer is Y^T = W . X^T on v_mfma_f32_32x32x2_f32 (exact fp32 fma chains) with the layer input in the
// accumulator layout of the previous layer (row rho(r, h) of sample j in register r), so activations
// never leave registers inside a pass; k-step (t, r) pairs input features 32t + rho(r, 0/1), which is
// what each half's lanes hold.  Backward layers are dX^T = W^T . dY^T the same way.  Weights are
// staged in LDS row-major with odd strides (conflict-free for both the row and column access).
// Architecture (the fused paths' reference configuration, nerf_runner.py:102-121): hash features 32
// -> 64 -> 64 (ReLU) -> [geo 15 | sigma 1] ; [geo, SH 16] -> 64 -> 64 (ReLU) -> 3 (sigmoid).
#include "acn_device.h"
#include "acn_internal.h"

// This file is compiled twice into libacnerf.so: the default build (fp16x3 layer products) exports the
// acn_mlp_* entry points, a second object built with -DACN_TRAIN_F16X3=0 -DACN_MLP_SUFFIX=_exact exports
// the exact-fp32 variants as acn_mlp_*_exact (a runtime precision switch: ops.set_train_mlp_precision).
#ifndef ACN_MLP_SUFFIX
#define ACN_MLP_SUFFIX
#endif
#define ACN_MLP_CAT2(a, b) a##b
#define ACN_MLP_CAT(a, b) ACN_MLP_CAT2(a, b)
#define ACN_MLP_API(name) ACN_MLP_CAT(name, ACN_MLP_SUFFIX)

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

// Saved / gradient tensors are feature-major per group of GS samples: element (sample m, feature f) at
// [m / GS][f][m % GS], so a wave's 32 lanes (32 consecutive samples) write 128 contiguous bytes per
// feature, and the weight-gradient GEMM of a layer is a batched (out x GS) . (GS x in) over groups.
constexpr int GS = 2048;
constexpr int SS = 325;                 // saved features: [h0|1 33][a1|1 65][a2|1 65][cin|1 32][c1|1 65][c2|1 65]
constexpr int O_H0 = 0, O_A1 = 33, O_A2 = 98, O_CIN = 163, O_C1 = 195, O_C2 = 260;
constexpr int DS = 275;                 // gradient row: [da1 64][da2 64][dhead 16][dc1 64][dc2 64][drgb 3]
constexpr int G_A1 = 0, G_A2 = 64, G_HD = 128, G_C1 = 144, G_C2 = 208, G_RGB = 272;

#ifndef ACN_TRAIN_F16X3
#define ACN_TRAIN_F16X3 1  // layer products as the fp32-accurate 3-term fp16 split (0: exact fp32 MFMA)
#endif
// ACN_TRAIN_AMP (third object, acn_mlp_*_amp): the reference's use_amp arithmetic -- the chain run under
// torch.autocast(float16) (runtime_adapt.py:249-259, meta_core.py:38, configs/train.json:37).  F.linear casts
// its input and weights to fp16 and addmm returns fp16 (one fp16 x fp16 product per term, fp32 accumulation,
// the bias added, one rounding to fp16); ReLU / sigmoid / trunc_exp (custom_fwd without cast_inputs) run on
// the fp16 tensors and round their results to fp16; the backward mirrors it (the output gradient cast to
// fp16, each dX and [dW | db] rounded to fp16 once).  No per-wave rescaling: values past fp16's range
// overflow / underflow exactly as under autocast -- the loss scale (GradScaler) is the caller's.
#ifndef ACN_TRAIN_AMP
#define ACN_TRAIN_AMP 0
#endif
#if ACN_TRAIN_AMP && !ACN_TRAIN_F16X3
#error "ACN_TRAIN_AMP builds on the fp16 weight image (ACN_TRAIN_F16X3=1)"
#endif
// round to fp16 and back (the identity outside the AMP build)
__device__ __forceinline__ float amp_r(float x) {
#if ACN_TRAIN_AMP
    return (float)(_Float16)x;
#else
    return x;
#endif
}

// LDS weight image: row-major, W0 64x32, W1 64x64, Whead 32x64 (geo rows 0..14, sigma row 15, rows
// 16..31 zero), Wc0 64x31 (col 31 = 0), Wc1 64x64, Wc2 32x64 (rows 3..31 zero), then the biases
// (zero-padded to 32 rows likewise).  Padding every layer to whole 32-row tiles lets the kernels read
// operands unconditionally (no exec-masked LDS loads).  fp32 build: one float per weight, odd strides
// cols + 1 (conflict-free row and column access).  fp16x3 build: each layer region holds a plane of
// hi = f16(w) then a plane of lo = f16(w - hi), row-major f16 with strides cols + 4 halves (a lane's 4
// consecutive k-elements are one 8-B read; rows 2 banks apart); biases stay fp32.
constexpr int S32 = ACN_TRAIN_F16X3 ? 36 : 33, S64 = ACN_TRAIN_F16X3 ? 68 : 65;
constexpr int L_W0 = 0, L_W1 = L_W0 + 64 * S32, L_WH = L_W1 + 64 * S64, L_WC0 = L_WH + 32 * S64, L_WC1 = L_WC0 + 64 * S32,
              L_WC2 = L_WC1 + 64 * S64, L_B0 = L_WC2 + 32 * S64, L_B1 = L_B0 + 64, L_BH = L_B1 + 64, L_BC0 = L_BH + 32,
              L_BC1 = L_BC0 + 64, L_BC2 = L_BC1 + 64, L_FLOATS = L_BC2 + 32;
static_assert(L_FLOATS % 4 == 0, "16-B staging");
static_assert(L_B0 % 4 == 0 && L_B1 % 4 == 0 && L_BH % 4 == 0 && L_BC0 % 4 == 0 && L_BC1 % 4 == 0 && L_BC2 % 4 == 0,
              "16-B bias reads (fwd_layer)");

struct MlpPtrs {
    const float *w0, *b0, *w1, *b1, *wsh, *bsh, *wg, *bg, *wc0, *bc0, *wc1, *bc1, *wc2, *bc2;
};

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int rho(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
// values the compiler must treat as unknown per loop iteration, so loop-invariant LDS weight reads and
// lane-address arithmetic are not hoisted out of the tile loop (and then spilled)
__device__ __forceinline__ int opaque_s(int v) {
    asm volatile("" : "+s"(v));
    return v;
}
__device__ __forceinline__ int opaque_v(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// the heads' activations and the first backward step (torch's derivative chain: sigmoid_backward
// g * (1 - y) * y; trunc_exp backward g * exp(xc) = g * y; threshold_backward (ReLU) g where the output > 0).
// AMP: sigmoid / exp of the fp16 pre-activations rounded to fp16; trunc_exp clamps at fp16(11.089866488) =
// 11.09375 (clamp's scalar is cast to the tensor's dtype; exp(11.09375) > 65504, so the clamped maximum is
// inf, as in the reference); the incoming gradient is cast to fp16 and each product rounded once.
__device__ __forceinline__ float out_rgb(float x) { return amp_r(acn::sigmoidf_(x)); }
__device__ __forceinline__ float out_sigma(float x) {
#if ACN_TRAIN_AMP
    const float m = 11.09375f;
    x = x < -m ? -m : x;
    x = x > m ? m : x;
    return amp_r(expf(x));
#else
    return acn::trunc_exp(x);
#endif
}
__device__ __forceinline__ float grad_rgb(float g, float y) { return amp_r((amp_r(g) * (1.0f - y)) * y); }
__device__ __forceinline__ float grad_sigma(float g, float y) { return amp_r(amp_r(g) * y); }

__device__ __forceinline__ int64_t fm_index(int64_t m, int nfeat, int f) {
    return (m / GS) * ((int64_t)nfeat * GS) + (int64_t)f * GS + (m % GS);
}

// the padded LDS image, built once per call (one element per thread), then copied by every block of
// the MLP kernels with 16-B loads
// weight (row, col) of layer region `layer` (0 W0, 1 W1, 2 head, 3 Wc0, 4 Wc1, 5 Wc2), zero in the padding
__device__ __forceinline__ float layer_w(const MlpPtrs& p, int layer, int r, int c) {
    switch (layer) {
        case 0: return c < 32 ? p.w0[r * 32 + c] : 0.0f;
        case 1: return c < 64 ? p.w1[r * 64 + c] : 0.0f;
        case 2: return c < 64 && r < 16 ? (r < 15 ? p.wg[r * 64 + c] : p.wsh[c]) : 0.0f;
        case 3: return c < 31 ? p.wc0[r * 31 + c] : 0.0f;
        case 4: return c < 64 ? p.wc1[r * 64 + c] : 0.0f;
        default: return c < 64 && r < 3 ? p.wc2[r * 64 + c] : 0.0f;
    }
}

__device__ __forceinline__ float pack_elem(const MlpPtrs& p, int e) {
    if (e < L_B0) {
        int layer, base, rows, ld;
        if (e < L_W1) { layer = 0; base = L_W0; rows = 64; ld = S32; }
        else if (e < L_WH) { layer = 1; base = L_W1; rows = 64; ld = S64; }
        else if (e < L_WC0) { layer = 2; base = L_WH; rows = 32; ld = S64; }
        else if (e < L_WC1) { layer = 3; base = L_WC0; rows = 64; ld = S32; }
        else if (e < L_WC2) { layer = 4; base = L_WC1; rows = 64; ld = S64; }
        else { layer = 5; base = L_WC2; rows = 32; ld = S64; }
        const int q = e - base;
#if ACN_TRAIN_F16X3
        // region = hi plane then lo plane, each rows x ld f16 row-major; this dword = halves (2c, 2c + 1)
        const int plane_dw = rows * ld / 2, part = q / plane_dw, hq = 2 * (q % plane_dw);
        const int r = hq / ld, c = hq % ld;
        uint32_t bits = 0;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const float w = layer_w(p, layer, r, c + u);
            const _Float16 hi = (_Float16)w;
            const _Float16 v = part ? (_Float16)(w - (float)hi) : hi;
            bits |= (uint32_t)__builtin_bit_cast(uint16_t, v) << (16 * u);
        }
        return __uint_as_float(bits);
#else
        (void)rows;
        return layer_w(p, layer, q / ld, q % ld);
#endif
    }
    if (e < L_B1) return p.b0[e - L_B0];
    if (e < L_BH) return p.b1[e - L_B1];
    if (e < L_BC0) { const int q = e - L_BH; return q < 15 ? p.bg[q] : (q == 15 ? p.bsh[0] : 0.0f); }
    if (e < L_BC1) return p.bc0[e - L_BC0];
    if (e < L_BC2) return p.bc1[e - L_BC1];
    const int q = e - L_BC2;
    return q < 3 ? p.bc2[q] : 0.0f;
}

__global__ void __launch_bounds__(256) mlp_pack_kernel(MlpPtrs p, float* __restrict__ img) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e < L_FLOATS) img[e] = pack_elem(p, e);
}

// the images of K experts at once (routed pair lists): blockIdx.y = expert
struct MlpPtrsK {
    MlpPtrs e[acn::kMaxK];
};
__global__ void __launch_bounds__(256) mlp_pack_multi_kernel(MlpPtrsK p, float* __restrict__ imgs) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e < L_FLOATS) imgs[(int64_t)blockIdx.y * L_FLOATS + e] = pack_elem(p.e[blockIdx.y], e);
}

__device__ __forceinline__ void stage_weights(const float* __restrict__ img, float* s) {
    const float4* src = reinterpret_cast<const float4*>(img);
    float4* dst = reinterpret_cast<float4*>(s);
    for (int e = threadIdx.x; e < L_FLOATS / 4; e += blockDim.x) dst[e] = src[e];
}

#if ACN_TRAIN_F16X3
// ---- fp16x3 layers: every product as hi*hi + hi*lo + lo*hi of hi = f16(x), lo = f16(x - hi) on
// v_mfma_f32_32x32x16_f16 with fp32 accumulation (dropping lo*lo: ~2^-22 relative, like the fused render,
// DESIGN.md 4).  fp16's range is handled per layer and wave: the layer input (activations, or the
// output gradients in the backward, which sit far below fp16's normal range) is multiplied by a
// wave-uniform power of two that brings its max |x| into [2^13, 2^14) and the accumulator is multiplied
// back -- both exact.  B operand = the input in the accumulator layout of the previous layer: k-element
// e of lane half h at k-step s is register 8 (s & 1) + e of tile s >> 1, i.e. input row xrow(s, h, e).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma_h(const f16x8& a, const f16x8& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int xrow(int s, int h, int e) { return 32 * (s >> 1) + 16 * (s & 1) + 8 * (e >> 2) + 4 * h + (e & 3); }

// wave-uniform exponent k with max |x| * 2^k in [2^13, 2^14) (0 for an all-zero / non-finite tile set)
template <int KT>
__device__ __forceinline__ int tile_scale_exp(const f32x16 (&X)[KT]) {
    // max of |x| as the integer order of the magnitude bits (NaN sorts above inf: the tile then gets k = 0)
    uint32_t m = 0u;
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t b = __float_as_uint(X[t][r]) & 0x7fffffffu;
            m = b > m ? b : m;
        }
    // within each row of 16 lanes on DPP (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror),
    // then the four rows through scalar readlanes: no LDS round trip
    auto dmax = [](uint32_t v, uint32_t w) { return v > w ? v : w; };
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0xB1, 0xF, 0xF, false));
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x4E, 0xF, 0xF, false));
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x141, 0xF, 0xF, false));
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x140, 0xF, 0xF, false));
    uint32_t w = dmax(dmax((uint32_t)__builtin_amdgcn_readlane((int)m, 0), (uint32_t)__builtin_amdgcn_readlane((int)m, 16)),
                      dmax((uint32_t)__builtin_amdgcn_readlane((int)m, 32), (uint32_t)__builtin_amdgcn_readlane((int)m, 48)));
    if (w == 0u || w >= 0x7f800000u) return 0;      // all zero, or inf / NaN present
    // max = f * 2^e, f in [0.5, 1): the biased exponent field gives e (subnormals: treat as 2^-126)
    const int be = (int)(w >> 23);
    const int e = (be == 0 ? -126 : be - 127) + 1;
    int k = 14 - e;
    return k > 100 ? 100 : (k < -100 ? -100 : k);
}

template <int KT>
__device__ __forceinline__ void split_tiles(const f32x16 (&X)[KT], int k, f16x8 (&bh)[2 * KT], f16x8 (&bl)[2 * KT]) {
    // hi = f16(x), lo = f16(x - hi) (the difference is exact), both rounded to nearest even; per pair of
    // elements the compiler emits one packed scale (v_pk_mul_f32), two packed conversions
    // (v_cvt_pk_f16_f32), two f16 -> f32 conversions and one packed subtraction -- no inline assembly, so
    // the compiler's hazard tracking sees every instruction.  hi + lo keeps ~22 bits of x (a truncating
    // hi, v_cvt_pkrtz, doubles lo and quadruples the dropped lo*lo term).
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    const float sc = ldexpf(1.0f, k);
    const f32x2 sc2 = {sc, sc};
#pragma unroll
    for (int s = 0; s < 2 * KT; ++s) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x2 x = (f32x2){X[s >> 1][8 * (s & 1) + 2 * q], X[s >> 1][8 * (s & 1) + 2 * q + 1]} * sc2;
            const f16x2 h = __builtin_convertvector(x, f16x2);
            const f16x2 l = __builtin_convertvector(x - __builtin_convertvector(h, f32x2), f16x2);
            bh[s][2 * q] = h[0];
            bh[s][2 * q + 1] = h[1];
            bl[s][2 * q] = l[0];
            bl[s][2 * q + 1] = l[1];
        }
    }
}

// AMP: the layer input cast to fp16 as F.linear under autocast does (B operand layout as split_tiles)
template <int KT>
__device__ __forceinline__ void cvt_tiles(const f32x16 (&X)[KT], f16x8 (&bh)[2 * KT]) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int s = 0; s < 2 * KT; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f16x2 h = __builtin_convertvector(((f32x2){X[s >> 1][8 * (s & 1) + 2 * q], X[s >> 1][8 * (s & 1) + 2 * q + 1]}), f16x2);
            bh[s][2 * q] = h[0];
            bh[s][2 * q + 1] = h[1];
        }
}

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f16x8 cat44(const f16x4& a, const f16x4& b) {
    return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

#ifndef ACN_MLP_KPIPE
#define ACN_MLP_KPIPE 1   // fp16x3 fwd_layer / bwd_layer: the next k-step's A operands read ahead (0: at their k-step)
#endif
#ifndef ACN_MLP_BIASV
#define ACN_MLP_BIASV 1   // fp16x3 fwd_layer epilogue: 16-B bias reads (0: one LDS read per element)
#endif
#ifndef ACN_MLP_ILV
// fp16x3 layer products: the output tiles' MFMA chains interleaved per k-step.  Off: meta 61.73 -> 62.03 ms with
// it (the producers of mlp_bwd_dw_pc_kernel 214 -> 217.5 us), C5 1.743 -> 1.728 ms
#define ACN_MLP_ILV 0
#endif
// Y[to] (rows 32to..) = b + W . X  (W: hi / lo planes of 32*NT padded rows, ld = stride in halves,
// ROWS = rows of the region; X: KT input tiles)
template <int NT, int KT, int ROWS>
__device__ __forceinline__ void fwd_layer(const float* W, int ld, const float* b, const f32x16 (&X)[KT],
                                          f32x16 (&Y)[NT], int lane) {
    const int i = lane & 31, h = lane >> 5;
#if ACN_TRAIN_AMP
    (void)ROWS;
    f16x8 bh[2 * KT];
    cvt_tiles<KT>(X, bh);
    acn::opnd_fence_n<2 * KT>(bh);   // VALU -> MFMA operand fence (acn_device.h)
    const _Float16* Wh = reinterpret_cast<const _Float16*>(W);
#pragma unroll
    for (int to = 0; to < NT; ++to) {
        const int ro = (32 * to + i) * ld;
        f32x16 acc = 0.0f;
#pragma unroll
        for (int s = 0; s < 2 * KT; ++s) {
            const int c0 = ro + 32 * (s >> 1) + 16 * (s & 1) + 4 * h;
            const f16x8 ahi = cat44(*reinterpret_cast<const f16x4*>(Wh + c0), *reinterpret_cast<const f16x4*>(Wh + c0 + 8));
            acc = mfma_h(ahi, bh[s], acc);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) Y[to][r] = amp_r(acc[r] + amp_r(b[32 * to + rho(r, h)]));
    }
#else
    const int k = tile_scale_exp<KT>(X);
    const float usc = ldexpf(1.0f, -k);
    f16x8 bh[2 * KT], bl[2 * KT];
    split_tiles<KT>(X, k, bh, bl);
    acn::opnd_fence_n<2 * KT>(bh, bl);
    const _Float16* Wh = reinterpret_cast<const _Float16*>(W);
    const _Float16* Wlo = Wh + ROWS * ld;
#if ACN_MLP_ILV
    // the NT output tiles' chains interleaved, k-step by k-step, with the k-step's A operands of every tile read
    // first (each tile's own chain keeps its order: the same sums bit for bit); Y is the accumulator
#pragma unroll
    for (int to = 0; to < NT; ++to) Y[to] = 0.0f;
#pragma unroll
    for (int s = 0; s < 2 * KT; ++s) {
        f16x8 ahi[NT], alo[NT];
#pragma unroll
        for (int to = 0; to < NT; ++to) {
            const int c0 = (32 * to + i) * ld + 32 * (s >> 1) + 16 * (s & 1) + 4 * h;
            ahi[to] = cat44(*reinterpret_cast<const f16x4*>(Wh + c0), *reinterpret_cast<const f16x4*>(Wh + c0 + 8));
            alo[to] = cat44(*reinterpret_cast<const f16x4*>(Wlo + c0), *reinterpret_cast<const f16x4*>(Wlo + c0 + 8));
        }
#pragma unroll
        for (int to = 0; to < NT; ++to) Y[to] = mfma_h(alo[to], bh[s], Y[to]);
#pragma unroll
        for (int to = 0; to < NT; ++to) Y[to] = mfma_h(ahi[to], bl[s], Y[to]);
#pragma unroll
        for (int to = 0; to < NT; ++to) Y[to] = mfma_h(ahi[to], bh[s], Y[to]);
    }
#pragma unroll
    for (int to = 0; to < NT; ++to)
#pragma unroll
        for (int r = 0; r < 16; ++r) Y[to][r] = __builtin_fmaf(Y[to][r], usc, b[32 * to + rho(r, h)]);
#else
#pragma unroll
    for (int to = 0; to < NT; ++to) {
        const int ro = (32 * to + i) * ld;
        f32x16 acc = 0.0f;
#if ACN_MLP_KPIPE
        // the next k-step's A operands are read while this k-step's MFMAs run (same chain, same order)
        auto lda = [&](int s, f16x8& ahi, f16x8& alo) {
            const int c0 = ro + 32 * (s >> 1) + 16 * (s & 1) + 4 * h;
            ahi = cat44(*reinterpret_cast<const f16x4*>(Wh + c0), *reinterpret_cast<const f16x4*>(Wh + c0 + 8));
            alo = cat44(*reinterpret_cast<const f16x4*>(Wlo + c0), *reinterpret_cast<const f16x4*>(Wlo + c0 + 8));
        };
        f16x8 ahi, alo;
        lda(0, ahi, alo);
#pragma unroll
        for (int s = 0; s < 2 * KT; ++s) {
            f16x8 nhi = ahi, nlo = alo;
            if (s + 1 < 2 * KT) lda(s + 1, nhi, nlo);
            acc = mfma_h(alo, bh[s], acc);
            acc = mfma_h(ahi, bl[s], acc);
            acc = mfma_h(ahi, bh[s], acc);
            ahi = nhi;
            alo = nlo;
        }
#else
#pragma unroll
        for (int s = 0; s < 2 * KT; ++s) {
            const int c0 = ro + 32 * (s >> 1) + 16 * (s & 1) + 4 * h;
            const f16x8 ahi = cat44(*reinterpret_cast<const f16x4*>(Wh + c0), *reinterpret_cast<const f16x4*>(Wh + c0 + 8));
            const f16x8 alo = cat44(*reinterpret_cast<const f16x4*>(Wlo + c0), *reinterpret_cast<const f16x4*>(Wlo + c0 + 8));
            acc = mfma_h(alo, bh[s], acc);
            acc = mfma_h(ahi, bl[s], acc);
            acc = mfma_h(ahi, bh[s], acc);
        }
#endif
        // acc * 2^-k + b in one rounding (the scaling itself is exact); the bias rows rho(4q .. 4q + 3, h) are 4
        // consecutive floats, read as one 16-B vector each (the image's bias regions are 16-B aligned)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#if ACN_MLP_BIASV
            typedef float f32x4b __attribute__((ext_vector_type(4)));
            const f32x4b bv = *reinterpret_cast<const f32x4b*>(b + 32 * to + 8 * q + 4 * h);
#pragma unroll
            for (int e = 0; e < 4; ++e) Y[to][4 * q + e] = __builtin_fmaf(acc[4 * q + e], usc, bv[e]);
#else
#pragma unroll
            for (int e = 0; e < 4; ++e)
                Y[to][4 * q + e] = __builtin_fmaf(acc[4 * q + e], usc, b[32 * to + rho(4 * q + e, h)]);
#endif
        }
    }
#endif
#endif
}

#ifndef ACN_BWD_TR16
#define ACN_BWD_TR16 1  // transposed weight reads of the backward layers on ds_read_b64_tr_b16 (0: ds_read_u16)
#endif
typedef __fp16 hf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) hf16x4 lds_hf16x4;
// ds_read_b64_tr_b16 (gfx950): per 16-lane group, lane 4q + p supplies the address of row q, columns 4p..4p+3
// of a 4 x 16 block of 16-bit elements; lane i of the group receives column i, row q in element q.  The
// address must point into LDS, 8-B aligned; EXEC must be all ones (every caller is wave-uniform).
__device__ __forceinline__ f16x4 ds_read_tr16(const _Float16* p) {
    return __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_hf16x4*)(p)));
}

// dX[ti] (input features 32ti..) = W^T . dY  (W rows = output features; k-steps whose 16 rows are all
// >= NROW are skipped at compile time, padding rows inside a k-step are zero in the image).  The A operand
// of lane (i, h) at k-step s is column 32 ti + i of W at rows xrow(s, h, 0..7) = base + 4h + 0..3 and
// base + 8 + 4h + 0..3: two 4-row blocks, each one transposed read per plane (lane (g, q, p) of 16-lane
// group g addresses row base [+ 8] + 4h + q, columns 32 ti + 16 (g & 1) + 4p).
template <int NT, int KT, int NROW, int ROWS>
__device__ __forceinline__ void bwd_layer(const float* W, int ld, const f32x16 (&dY)[KT], f32x16 (&dX)[NT],
                                          int lane) {
    const int i = lane & 31, h = lane >> 5;
#if ACN_TRAIN_AMP
    f16x8 bh[2 * KT];
    cvt_tiles<KT>(dY, bh);
    acn::opnd_fence_n<2 * KT>(bh);
#else
    const int k = tile_scale_exp<KT>(dY);
    const float usc = ldexpf(1.0f, -k);
    f16x8 bh[2 * KT], bl[2 * KT];
    split_tiles<KT>(dY, k, bh, bl);
    acn::opnd_fence_n<2 * KT>(bh, bl);
#endif
    const _Float16* Wh = reinterpret_cast<const _Float16*>(W);
    const _Float16* Wlo = Wh + ROWS * ld;
#if ACN_BWD_TR16
    const int trow = 4 * h + ((lane >> 2) & 3), tcol = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
#endif
#if ACN_MLP_ILV && ACN_BWD_TR16 && !ACN_TRAIN_AMP
    // as fwd_layer: the NT input tiles' chains interleaved per k-step, operands read first; dX is the accumulator
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) dX[ti] = 0.0f;
#pragma unroll
    for (int s = 0; s < 2 * KT; ++s) {
        if (32 * (s >> 1) + 16 * (s & 1) >= NROW) continue;
        f16x8 ahi[NT], alo[NT];
#pragma unroll
        for (int ti = 0; ti < NT; ++ti) {
            const int o = (32 * (s >> 1) + 16 * (s & 1) + trow) * ld + 32 * ti + tcol;
            ahi[ti] = cat44(ds_read_tr16(Wh + o), ds_read_tr16(Wh + o + 8 * ld));
            alo[ti] = cat44(ds_read_tr16(Wlo + o), ds_read_tr16(Wlo + o + 8 * ld));
        }
#pragma unroll
        for (int ti = 0; ti < NT; ++ti) dX[ti] = mfma_h(alo[ti], bh[s], dX[ti]);
#pragma unroll
        for (int ti = 0; ti < NT; ++ti) dX[ti] = mfma_h(ahi[ti], bl[s], dX[ti]);
#pragma unroll
        for (int ti = 0; ti < NT; ++ti) dX[ti] = mfma_h(ahi[ti], bh[s], dX[ti]);
    }
#pragma unroll
    for (int ti = 0; ti < NT; ++ti)
#pragma unroll
        for (int r = 0; r < 16; ++r) dX[ti][r] = dX[ti][r] * usc;
    return;
#endif
#if ACN_MLP_KPIPE && ACN_BWD_TR16 && !ACN_TRAIN_AMP
    // as fwd_layer: the next live k-step's A operands are read while this k-step's MFMAs run (same chain, order)
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
        auto ldb = [&](int s, f16x8& ahi, f16x8& alo) {
            const int o = (32 * (s >> 1) + 16 * (s & 1) + trow) * ld + 32 * ti + tcol;
            ahi = cat44(ds_read_tr16(Wh + o), ds_read_tr16(Wh + o + 8 * ld));
            alo = cat44(ds_read_tr16(Wlo + o), ds_read_tr16(Wlo + o + 8 * ld));
        };
        f32x16 acc = 0.0f;
        f16x8 ahi, alo;
        ldb(0, ahi, alo);
#pragma unroll
        for (int s = 0; s < 2 * KT; ++s) {
            if (32 * (s >> 1) + 16 * (s & 1) >= NROW) continue;
            f16x8 nhi = ahi, nlo = alo;
            if (s + 1 < 2 * KT && 32 * ((s + 1) >> 1) + 16 * ((s + 1) & 1) < NROW) ldb(s + 1, nhi, nlo);
            acc = mfma_h(alo, bh[s], acc);
            acc = mfma_h(ahi, bl[s], acc);
            acc = mfma_h(ahi, bh[s], acc);
            ahi = nhi;
            alo = nlo;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) dX[ti][r] = acc[r] * usc;
    }
    return;
#endif
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
        f32x16 acc = 0.0f;
#pragma unroll
        for (int s = 0; s < 2 * KT; ++s) {
            if (32 * (s >> 1) + 16 * (s & 1) >= NROW) continue;
            f16x8 ahi, alo;
#if ACN_BWD_TR16
            {
                const int o = (32 * (s >> 1) + 16 * (s & 1) + trow) * ld + 32 * ti + tcol;
                ahi = cat44(ds_read_tr16(Wh + o), ds_read_tr16(Wh + o + 8 * ld));
#if !ACN_TRAIN_AMP
                alo = cat44(ds_read_tr16(Wlo + o), ds_read_tr16(Wlo + o + 8 * ld));
#endif
            }
#else
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int o = xrow(s, h, e) * ld + 32 * ti + i;
                ahi[e] = Wh[o];
                alo[e] = Wlo[o];
            }
#endif
#if ACN_TRAIN_AMP
            (void)alo;
            acc = mfma_h(ahi, bh[s], acc);
#else
            acc = mfma_h(alo, bh[s], acc);
            acc = mfma_h(ahi, bl[s], acc);
            acc = mfma_h(ahi, bh[s], acc);
#endif
        }
#if ACN_TRAIN_AMP
#pragma unroll
        for (int r = 0; r < 16; ++r) dX[ti][r] = amp_r(acc[r]);
#else
#pragma unroll
        for (int r = 0; r < 16; ++r) dX[ti][r] = acc[r] * usc;
#endif
    }
}
#else
// Y[to] (rows 32to..) = b + W . X  (W: 32*NT padded rows, ld = stride; X: KT input tiles).  The A operands
// of an output tile are read into registers before its MFMA chain.
template <int NT, int KT, int ROWS>
__device__ __forceinline__ void fwd_layer(const float* W, int ld, const float* b, const f32x16 (&X)[KT],
                                          f32x16 (&Y)[NT], int lane) {
    const int i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int to = 0; to < NT; ++to) {
        const float* wr = W + (32 * to + i) * ld;
        float a[KT][16];
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) a[t][r] = wr[32 * t + rho(r, h)];
#pragma unroll
        for (int r = 0; r < 16; ++r) Y[to][r] = b[32 * to + rho(r, h)];
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) Y[to] = mfma32(a[t][r], X[t][r], Y[to]);
    }
}

// dX[ti] (input features 32ti..) = W^T . dY  (W rows = output features; k-steps whose rows are all
// >= NROW are skipped at compile time, the other lane half reads zero padding rows)
template <int NT, int KT, int NROW, int ROWS>
__device__ __forceinline__ void bwd_layer(const float* W, int ld, const f32x16 (&dY)[KT], f32x16 (&dX)[NT],
                                          int lane) {
    const int i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
        float a[KT][16];
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (32 * t + rho(r, 0) < NROW) a[t][r] = W[(32 * t + rho(r, h)) * ld + 32 * ti + i];
        dX[ti] = 0.0f;
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (32 * t + rho(r, 0) < NROW) dX[ti] = mfma32(a[t][r], dY[t][r], dX[ti]);
    }
}

#endif

template <int NT>
__device__ __forceinline__ void relu(f32x16 (&Y)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) Y[t][r] = Y[t][r] > 0.0f ? Y[t][r] : 0.0f;
}

// feature-major (GS groups) <-> accumulator tiles of sample m
template <int NT>
__device__ __forceinline__ void load_fm(const float* src, int nall, int off, int nfeat, int64_t m, bool ok, int h,
                                        f32x16 (&X)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = 32 * t + rho(r, h);
            X[t][r] = (ok && f < nfeat) ? src[fm_index(m, nall, off + f)] : 0.0f;
        }
}
template <int NT>
__device__ __forceinline__ void store_fm(float* dst, int nall, int off, int nfeat, int64_t m, bool ok, int h,
                                         const f32x16 (&X)[NT]) {
    if (!ok) return;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = 32 * t + rho(r, h);
            if (f < nfeat) dst[fm_index(m, nall, off + f)] = amp_r(X[t][r]);
        }
}

// row-major (M, stride) <-> accumulator tiles of sample (base + j)
template <int NT>
__device__ __forceinline__ void load_tiles(const float* src, int64_t stride, int off, int nfeat, int64_t m, bool ok,
                                           int h, f32x16 (&X)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = 32 * t + rho(r, h);
            X[t][r] = (ok && f < nfeat) ? src[m * stride + off + f] : 0.0f;
        }
}
template <int NT>
__device__ __forceinline__ void store_tiles(float* dst, int64_t stride, int off, int nfeat, int64_t m, bool ok, int h,
                                            const f32x16 (&X)[NT]) {
    if (!ok) return;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = 32 * t + rho(r, h);
            if (f < nfeat) dst[m * stride + off + f] = X[t][r];
        }
}

// forward of one tile: everything the backward needs is recomputable from h0 + sh, but the weight
// gradients need the layer inputs in memory anyway, so they are saved here
__device__ __forceinline__ void tile_forward(const float* Wl, const float* h0, const float* sh, int64_t m, bool ok,
                                             int lane, f32x16 (&X0)[1], f32x16 (&A1)[2], f32x16 (&A2)[2],
                                             f32x16 (&Hd)[1], f32x16 (&Cin)[1], f32x16 (&C1)[2], f32x16 (&C2)[2],
                                             f32x16 (&Rg)[1]) {
    const int h = lane >> 5;
    load_tiles<1>(h0, 32, 0, 32, m, ok, h, X0);
    fwd_layer<2, 1, 64>(Wl + L_W0, S32, Wl + L_B0, X0, A1, lane);
    relu<2>(A1);
    fwd_layer<2, 2, 64>(Wl + L_W1, S64, Wl + L_B1, A1, A2, lane);
    relu<2>(A2);
    fwd_layer<1, 2, 32>(Wl + L_WH, S64, Wl + L_BH, A2, Hd, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int f = rho(r, h);
        Cin[0][r] = f < 15 ? Hd[0][r] : ((ok && f < 31) ? sh[m * 16 + (f - 15)] : 0.0f);
    }
    fwd_layer<2, 1, 64>(Wl + L_WC0, S32, Wl + L_BC0, Cin, C1, lane);
    relu<2>(C1);
    fwd_layer<2, 2, 64>(Wl + L_WC1, S64, Wl + L_BC1, C1, C2, lane);
    relu<2>(C2);
    fwd_layer<1, 2, 32>(Wl + L_WC2, S64, Wl + L_BC2, C2, Rg, lane);
}

#ifndef ACN_FWD_VLOAD
#define ACN_FWD_VLOAD 0   // mlp_fwd_kernel<false>: the producers' vector h0 / SH loads below (0: per-element loads)
#endif
#ifndef ACN_DW_PIPE
#define ACN_DW_PIPE 1   // dw_blocks (fp32 stage): next k-step's LDS reads in flight, blocks' MFMAs interleaved
#endif
// Prefetched per-sample inputs of the producer waves (mlp_bwd_dw_pc_kernel): whole 16-B vectors at a clamped
// sample index (no per-element exec branches), issued well ahead of their use and masked for samples past the
// end only where they are consumed -- a scheduling barrier after the loads keeps the compiler from sinking them
// to their uses.  The values are those load_tiles / tile_forward / dw_round's output-gradient reads take.
struct X0Raw {
    float4 v[4];   // h0 row elements rho(4q .. 4q + 3, h) = 8q + 4h + 0..3
};
__device__ __forceinline__ void load_x0raw(const float* __restrict__ h0, int64_t m, bool ok, int h, X0Raw& x) {
    const float4* p = reinterpret_cast<const float4*>(h0 + (ok ? m : 0) * 32 + 4 * h);
#pragma unroll
    for (int q = 0; q < 4; ++q) x.v[q] = p[2 * q];
}
__device__ __forceinline__ void x0_tile(const X0Raw& x, bool ok, f32x16 (&X)[1]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        X[0][4 * q] = ok ? x.v[q].x : 0.0f;
        X[0][4 * q + 1] = ok ? x.v[q].y : 0.0f;
        X[0][4 * q + 2] = ok ? x.v[q].z : 0.0f;
        X[0][4 * q + 3] = ok ? x.v[q].w : 0.0f;
    }
}
struct PcIn {      // issued after the forward's first layer (its h0 tile's registers are free by then)
    float s[9];    // SH row value of accumulator row r = 7 .. 15 (rho(r, h) - 15, clamped; rows r < 7 are geo)
    float o[3], g[3];   // outputs / output gradients: h == 0 lanes rgb, h == 1 lanes sigma (in all three)
};
template <bool OG>   // OG: also the output / output-gradient values (the backward's producers)
__device__ __forceinline__ void load_pcin(const float* __restrict__ sh, const float* __restrict__ out,
                                          const float* __restrict__ gout, int64_t m, bool ok, int h, PcIn& in) {
    const int64_t mc = ok ? m : 0;
#pragma unroll
    for (int r = 7; r < 16; ++r) {
        const int f = rho(r, h) - 15;
        in.s[r - 7] = sh[mc * 16 + (f < 0 ? 0 : (f > 15 ? 15 : f))];
    }
    if (OG) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            in.o[c] = out[mc * 4 + (h ? 3 : c)];
            in.g[c] = gout[mc * 4 + (h ? 3 : c)];
        }
    }
}
__device__ __forceinline__ float opaque_f(float v) {   // pins a prefetched value's first use (and its wait) here
    asm volatile("" : "+v"(v));
    return v;
}
// tile_forward on a prefetched h0 tile, issuing the SH / output loads behind the first layer (bitwise the same
// layers and values)
template <bool OG = true>
__device__ __forceinline__ void tile_forward_x(const float* Wl, const X0Raw& x0, const float* __restrict__ sh,
                                               const float* __restrict__ out, const float* __restrict__ gout,
                                               int64_t m, bool ok, int lane, PcIn& in, f32x16 (&A1)[2],
                                               f32x16 (&A2)[2], f32x16 (&Hd)[1], f32x16 (&Cin)[1],
                                               f32x16 (&C1)[2], f32x16 (&C2)[2], f32x16 (&Rg)[1]) {
    const int h = lane >> 5;
    {
        f32x16 X0[1];
        x0_tile(x0, ok, X0);
        fwd_layer<2, 1, 64>(Wl + L_W0, S32, Wl + L_B0, X0, A1, lane);
    }
    relu<2>(A1);
    __builtin_amdgcn_sched_barrier(0);
    load_pcin<OG>(sh, out, gout, m, ok, h, in);
    __builtin_amdgcn_sched_barrier(0);
    fwd_layer<2, 2, 64>(Wl + L_W1, S64, Wl + L_B1, A1, A2, lane);
    relu<2>(A2);
    fwd_layer<1, 2, 32>(Wl + L_WH, S64, Wl + L_BH, A2, Hd, lane);
    __builtin_amdgcn_sched_barrier(0);
    float sv[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) sv[k] = opaque_f(in.s[k]);   // unconditional: selects below, no branches
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int f = rho(r, h);
        Cin[0][r] = f < 15 ? Hd[0][r] : ((ok && f < 31 && r >= 7) ? sv[r >= 7 ? r - 7 : 0] : 0.0f);
    }
    fwd_layer<2, 1, 64>(Wl + L_WC0, S32, Wl + L_BC0, Cin, C1, lane);
    relu<2>(C1);
    fwd_layer<2, 2, 64>(Wl + L_WC1, S64, Wl + L_BC1, C1, C2, lane);
    relu<2>(C2);
    fwd_layer<1, 2, 32>(Wl + L_WC2, S64, Wl + L_BC2, C2, Rg, lane);
}

// SAVE: write the layer inputs for the split backward (keeps every activation live to the end of the tile:
// ~250 VGPRs, 4-wave blocks).  The no-save instantiation -- every fused-path call -- needs ~124 registers, so it
// runs 8-wave blocks: two blocks (the 72 KB weight image each) = four waves per SIMD.
template <bool SAVE>
__global__ void __launch_bounds__(SAVE ? 256 : 512) mlp_fwd_kernel(const float* __restrict__ img, const float* __restrict__ h0,
                                                      const float* __restrict__ sh, int64_t M,
                                                      float* __restrict__ out, float* __restrict__ save) {
    __shared__ __attribute__((aligned(16))) float Wl[L_FLOATS];
    stage_weights(img, Wl);
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int64_t ntiles = (M + 31) / 32;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t tile = wave; tile < ntiles; tile += nwaves) {
        const int64_t m = tile * 32 + j;
        const bool ok = m < M;
        f32x16 X0[1], A1[2], A2[2], Hd[1], Cin[1], C1[2], C2[2], Rg[1];
        // opaque base: the LDS weight reads are re-issued per tile instead of hoisted out of the loop into
        // ~240 held registers (one wave per SIMD; with it the no-save form fits two)
        if (!SAVE && ACN_FWD_VLOAD) {   // vector loads of h0, SH behind the first layer (no per-element branches)
            X0Raw x0;
            load_x0raw(h0, m, ok, h, x0);
            PcIn in;
            tile_forward_x<false>(Wl + opaque_s(0), x0, sh, nullptr, nullptr, m, ok, lane, in, A1, A2, Hd, Cin, C1,
                                  C2, Rg);
        } else {
            tile_forward(Wl + opaque_s(0), h0, sh, m, ok, lane, X0, A1, A2, Hd, Cin, C1, C2, Rg);
        }
        if (ok) {
            if (h == 0) {
#pragma unroll
                for (int c = 0; c < 3; ++c) out[m * 4 + c] = out_rgb(Rg[0][c]);
            } else {
                out[m * 4 + 3] = out_sigma(Hd[0][7]);  // row 15 = sigma head (lane half 1, reg 7)
            }
            if (SAVE) {
                // layer inputs (+ ones columns for the bias gradient), feature-major
#pragma unroll
                for (int r = 0; r < 16; ++r) save[fm_index(m, SS, O_H0 + rho(r, h))] = amp_r(h0[m * 32 + rho(r, h)]);
                store_fm<2>(save, SS, O_A1, 64, m, ok, h, A1);
                store_fm<2>(save, SS, O_A2, 64, m, ok, h, A2);
                store_fm<1>(save, SS, O_CIN, 31, m, ok, h, Cin);
                store_fm<2>(save, SS, O_C1, 64, m, ok, h, C1);
                store_fm<2>(save, SS, O_C2, 64, m, ok, h, C2);
                if (h == 0) {
                    save[fm_index(m, SS, O_H0 + 32)] = 1.0f;
                    save[fm_index(m, SS, O_A1 + 64)] = 1.0f;
                    save[fm_index(m, SS, O_A2 + 64)] = 1.0f;
                } else {
                    save[fm_index(m, SS, O_CIN + 31)] = 1.0f;
                    save[fm_index(m, SS, O_C1 + 64)] = 1.0f;
                    save[fm_index(m, SS, O_C2 + 64)] = 1.0f;
                }
            }
        }
    }
}

// torch's derivative chain: sigmoid_backward g * (1 - y) * y; trunc_exp backward g * exp(xc) = g * y;
// threshold_backward (ReLU) g where the saved output > 0
__global__ void __launch_bounds__(256) mlp_bwd_kernel(const float* __restrict__ img, const float* __restrict__ save,
                                                      const float* __restrict__ out, const float* __restrict__ gout,
                                                      int64_t M, float* __restrict__ gsave,
                                                      float* __restrict__ gh0) {
    __shared__ __attribute__((aligned(16))) float Wl[L_FLOATS];
    stage_weights(img, Wl);
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int64_t ntiles = (M + 31) / 32;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t tile = wave; tile < ntiles; tile += nwaves) {
        const int64_t m = tile * 32 + j;
        const bool ok = m < M;
        // output-layer gradients (rgb rows 0..2 of the colour head; sigma = head row 15)
        f32x16 dRg[1], dHd[1];
        dRg[0] = 0.0f;
        dHd[0] = 0.0f;
        float dsig = 0.0f;
        if (ok) {
            if (h == 0) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float y = out[m * 4 + c];
                    dRg[0][c] = grad_rgb(gout[m * 4 + c], y);
                }
            } else {
                dsig = grad_sigma(gout[m * 4 + 3], out[m * 4 + 3]);
            }
        }
        store_fm<1>(gsave, DS, G_RGB, 3, m, ok, h, dRg);
        f32x16 G2[2], G1[2], Gc[1], mask[2];
        bwd_layer<2, 1, 3, 32>(Wl + L_WC2, S64, dRg, G2, lane);
        load_fm<2>(save, SS, O_C2, 64, m, ok, h, mask);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) G2[t][r] = mask[t][r] > 0.0f ? G2[t][r] : 0.0f;
        store_fm<2>(gsave, DS, G_C2, 64, m, ok, h, G2);
        bwd_layer<2, 2, 64, 64>(Wl + L_WC1, S64, G2, G1, lane);
        load_fm<2>(save, SS, O_C1, 64, m, ok, h, mask);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) G1[t][r] = mask[t][r] > 0.0f ? G1[t][r] : 0.0f;
        store_fm<2>(gsave, DS, G_C1, 64, m, ok, h, G1);
        bwd_layer<1, 2, 64, 64>(Wl + L_WC0, S32, G1, Gc, lane);  // d cin: rows 0..14 = d geo (SH rows dropped)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, h);
            dHd[0][r] = f < 15 ? Gc[0][r] : (f == 15 ? dsig : 0.0f);
        }
        store_fm<1>(gsave, DS, G_HD, 16, m, ok, h, dHd);
        f32x16 GA2[2], GA1[2], GH[1];
        bwd_layer<2, 1, 16, 32>(Wl + L_WH, S64, dHd, GA2, lane);
        load_fm<2>(save, SS, O_A2, 64, m, ok, h, mask);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) GA2[t][r] = mask[t][r] > 0.0f ? GA2[t][r] : 0.0f;
        store_fm<2>(gsave, DS, G_A2, 64, m, ok, h, GA2);
        bwd_layer<2, 2, 64, 64>(Wl + L_W1, S64, GA2, GA1, lane);
        load_fm<2>(save, SS, O_A1, 64, m, ok, h, mask);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) GA1[t][r] = mask[t][r] > 0.0f ? GA1[t][r] : 0.0f;
        store_fm<2>(gsave, DS, G_A1, 64, m, ok, h, GA1);
        bwd_layer<1, 2, 64, 64>(Wl + L_W0, S32, GA1, GH, lane);
        if (gh0) store_tiles<1>(gh0, 32, 0, 32, m, ok, h, GH);
    }
}

// ---------------------------------------------------------------------------------------------
// Fused backward with the weight gradients (acn_mlp_train_bwd_dw).  A workgroup of 4 waves takes 4 tiles
// (128 samples) per round; each wave re-runs the forward of its tile from h0 / sh (the same tile_forward
// as mlp_fwd_kernel, so the activations are bit-identical) instead of reading saved activations, and runs
// the backward chain layer by layer.  At each layer the 4 waves put dY and X of their tiles into one
// shared LDS stage [feature][128 samples]; after a barrier, wave w forms its share of that layer's
// [dW | db] over all 128 samples on v_mfma_f32_16x16x4_f32 (row block w of the 64-row layers, column
// block w of the sigma / colour heads), accumulating in registers that live for the whole kernel:
// every gradient element has exactly one owner wave, so there are no atomics, and a workgroup writes
// its 13,715 partial sums once at the end (mlp_dw_reduce_kernel adds the workgroups' copies).
// Nothing per sample is written except dL/dh0.
constexpr int D_W0 = 0, D_B0 = 2048, D_W1 = 2112, D_B1 = 6208, D_WSH = 6272, D_BSH = 6336, D_WG = 6337,
              D_BG = 7297, D_WC0 = 7312, D_BC0 = 9296, D_WC1 = 9360, D_BC1 = 13456, D_WC2 = 13520, D_BC2 = 13712,
              NDW = 13715;
constexpr int SW = 132;                  // stage row stride (floats): 128 samples + 4, 16-B aligned rows
constexpr int X_ROW = 64;                // stage rows 0..63 = dY, 64..127 = X
constexpr int MAX_DW_BLOCKS = 256;       // partial copies (workgroups) of the fused backward

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int NT>
__device__ __forceinline__ void relu_mask(f32x16 (&G)[NT], const f32x16 (&Y)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) G[t][r] = Y[t][r] > 0.0f ? G[t][r] : 0.0f;
}

#ifndef ACN_DW_F16X3
// weight-gradient contraction on the fp16x3 split as well.  Off: measured slower (fused backward 352 ->
// 383 us at M = 384k, meta step 79.1 -> 82.8 ms): with one wave per SIMD the dW phase is bound by the
// staging (split + two f16 planes written per element) and LDS traffic, not by the fp32 MFMAs it saves.
// The AMP build always takes the fp16 stage with ONE plane: its dY and X are fp16 values already, so one
// v_mfma_f32_16x16x16_f16 product per term is exact (fp32 accumulation), as autocast's fp16 GEMM computes it
#define ACN_DW_F16X3 ACN_TRAIN_AMP
#endif
#if ACN_TRAIN_AMP && !ACN_DW_F16X3
#error "the AMP build contracts [dW | db] on the fp16 stage"
#endif
constexpr int kStagePlanes = ACN_TRAIN_AMP ? 1 : 2;   // fp16 stage: hi (+ lo for the fp16x3 split)
#ifndef ACN_DW_CSPLIT
#define ACN_DW_CSPLIT 0   // fp32 stage, fp16x3 split by the consumer waves (producer / consumer kernel only)
#endif
#if ACN_DW_CSPLIT && (ACN_DW_F16X3 || !ACN_TRAIN_F16X3)
#error "ACN_DW_CSPLIT is a variant of the default build's fp32-stage backward"
#endif

struct StageScale {
    int kY, kX;  // power-of-two exponents the staged dY / X carry (0: unscaled fp32 stage)
};

#if ACN_DW_F16X3
// ---- fp16x3 weight gradients.  The stage holds f16 planes (hi, then lo) of [144 rows][SH halves]:
// rows 0..63 dY, 64..127 X, row 128 ones (rows 129..143 zero) -- the bias sums come out of the MFMA as
// the contraction with the ones row.  dY and X are scaled by workgroup-uniform powers of two (the
// contraction mixes the four waves' samples): each wave publishes its max |dY| and max |X| before the
// stage barrier and all waves take the maximum of the four.  Per round and block the 128-sample
// contraction is 8 k-steps of v_mfma_f32_16x16x16_f16 x 3 products into a temporary, added to the
// persistent fp32 accumulator times 2^-(kY + kX).
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
constexpr int SH = 136;                   // stage row stride (halves): 128 samples + 8, 16-B aligned rows
constexpr int ST_ROWS = 144, ST_ONES = 128;
constexpr int ST_FLOATS = kStagePlanes * ST_ROWS * SH / 2;  // one or two f16 planes
__device__ __forceinline__ f32x4 mfma16h(const f16x4& a, const f16x4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}
typedef f32x4 BiasAcc;

__device__ __forceinline__ void stage_init(float* st) {  // the ones row (both planes zero elsewhere there)
    _Float16* hp = reinterpret_cast<_Float16*>(st);
    _Float16* lp = hp + ST_ROWS * SH;
    for (int e = threadIdx.x; e < (ST_ROWS - ST_ONES) * SH; e += blockDim.x) {
        hp[ST_ONES * SH + e] = (_Float16)(e < SH ? 1.0f : 0.0f);
        if (kStagePlanes == 2) lp[ST_ONES * SH + e] = (_Float16)0.0f;
    }
}

// max |x| bits of this wave's tiles (wave-uniform; DPP + readlanes)
template <int NT>
__device__ __forceinline__ uint32_t wave_absmax_bits(const f32x16 (&T)[NT]) {
    uint32_t m = 0u;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t b = __float_as_uint(T[t][r]) & 0x7fffffffu;
            m = b > m ? b : m;
        }
    auto dmax = [](uint32_t v, uint32_t w) { return v > w ? v : w; };
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0xB1, 0xF, 0xF, false));
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x4E, 0xF, 0xF, false));
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x141, 0xF, 0xF, false));
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x140, 0xF, 0xF, false));
    return dmax(dmax((uint32_t)__builtin_amdgcn_readlane((int)m, 0), (uint32_t)__builtin_amdgcn_readlane((int)m, 16)),
                dmax((uint32_t)__builtin_amdgcn_readlane((int)m, 32), (uint32_t)__builtin_amdgcn_readlane((int)m, 48)));
}
__device__ __forceinline__ int exp_for_bits(uint32_t w) {  // as tile_scale_exp
    if (w == 0u || w >= 0x7f800000u) return 0;
    const int be = (int)(w >> 23);
    const int k = 14 - ((be == 0 ? -126 : be - 127) + 1);
    return k > 100 ? 100 : (k < -100 ? -100 : k);
}

template <int NT>
__device__ __forceinline__ void stage_put(float* st, int row0, const f32x16 (&T)[NT], int k, int w, int lane) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    _Float16* hp = reinterpret_cast<_Float16*>(st);
    _Float16* lp = hp + ST_ROWS * SH;
    const int j = lane & 31, h = lane >> 5;
    const float sc = ldexpf(1.0f, k);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const f32x2 x = (f32x2){T[t][r], T[t][r + 1]} * (f32x2){sc, sc};
            const f16x2 hi = __builtin_convertvector(x, f16x2);
            const int o0 = (row0 + 32 * t + rho(r, h)) * SH + 32 * w + j, o1 = (row0 + 32 * t + rho(r + 1, h)) * SH + 32 * w + j;
            hp[o0] = hi[0];
            hp[o1] = hi[1];
            if (kStagePlanes == 2) {
                const f16x2 lo = __builtin_convertvector(x - __builtin_convertvector(hi, f32x2), f16x2);
                lp[o0] = lo[0];
                lp[o1] = lo[1];
            }
        }
}
// the producer / consumer kernel's put (AMP: unscaled fp16 values)
template <int NT>
__device__ __forceinline__ void stage_put(float* st, int row0, const f32x16 (&T)[NT], int w, int lane) {
    stage_put<NT>(st, row0, T, 0, w, lane);
}

// acc[n] += dY[16 rows from arow] . X[16 features from xrow + 16 n]^T over the 128 staged samples,
// bacc (column 0) += the dY rows' sums; lane (i = l & 15, q = l >> 4) supplies k-elements = samples
// 32 q + 4 t + 0..3 of k-step t
template <int NCB, bool PIPE = false>   // PIPE: the fp32 stage's option (unused on the fp16 stage)
__device__ __forceinline__ void dw_blocks(const float* st, int arow, int xrow, f32x4 (&acc)[NCB], BiasAcc& bacc,
                                          StageScale sc, int lane) {
#if ACN_DIAG_NODW  // diagnostic build only: no weight-gradient contraction
    return;
#endif
    const _Float16* hp = reinterpret_cast<const _Float16*>(st);
    const _Float16* lp = hp + ST_ROWS * SH;
    const int i = lane & 15, q = lane >> 4;
    const int oa = (arow + i) * SH + 32 * q, ob = (xrow + i) * SH + 32 * q, oo = (ST_ONES + i) * SH + 32 * q;
    f32x4 tmp[NCB], tb = 0.0f;
#pragma unroll
    for (int n = 0; n < NCB; ++n) tmp[n] = 0.0f;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const f16x4 ah = *reinterpret_cast<const f16x4*>(hp + oa + 4 * t);
        const f16x4 on = *reinterpret_cast<const f16x4*>(hp + oo + 4 * t);
        if (kStagePlanes == 2) {
            const f16x4 al = *reinterpret_cast<const f16x4*>(lp + oa + 4 * t);
            tb = mfma16h(al, on, tb);
            tb = mfma16h(ah, on, tb);
#pragma unroll
            for (int n = 0; n < NCB; ++n) {
                const f16x4 bh = *reinterpret_cast<const f16x4*>(hp + ob + 16 * n * SH + 4 * t);
                const f16x4 bl = *reinterpret_cast<const f16x4*>(lp + ob + 16 * n * SH + 4 * t);
                tmp[n] = mfma16h(al, bh, tmp[n]);
                tmp[n] = mfma16h(ah, bl, tmp[n]);
                tmp[n] = mfma16h(ah, bh, tmp[n]);
            }
        } else {   // AMP: dY, X are fp16 values -- one exact product per term
            tb = mfma16h(ah, on, tb);
#pragma unroll
            for (int n = 0; n < NCB; ++n) {
                const f16x4 bh = *reinterpret_cast<const f16x4*>(hp + ob + 16 * n * SH + 4 * t);
                tmp[n] = mfma16h(ah, bh, tmp[n]);
            }
        }
    }
    const float ua = ldexpf(1.0f, -sc.kY), uab = ldexpf(1.0f, -(sc.kY + sc.kX));
#pragma unroll
    for (int n = 0; n < NCB; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[n][r] = __builtin_fmaf(tmp[n][r], uab, acc[n][r]);
#pragma unroll
    for (int r = 0; r < 4; ++r) bacc[r] = __builtin_fmaf(tb[r], ua, bacc[r]);
}

// one layer's stage round: publish this wave's maxima, barrier (previous readers done, maxima visible),
// put dY / X scaled by the workgroup maxima, barrier
template <int NO, int NI>
__device__ __forceinline__ StageScale stage_layer(float* st, const f32x16 (&dY)[NO], const f32x16 (&X)[NI], int w,
                                                  int lane) {
#if ACN_TRAIN_AMP   // fp16 values already: no rescaling (what autocast's GEMM sees)
    __syncthreads();
    stage_put<NO>(st, 0, dY, 0, w, lane);
    stage_put<NI>(st, X_ROW, X, 0, w, lane);
    __syncthreads();
    return StageScale{0, 0};
#endif
    __shared__ uint32_t smax[8];
    const uint32_t my = wave_absmax_bits<NO>(dY), mx = wave_absmax_bits<NI>(X);
    if (lane == 0) {
        smax[w] = my;
        smax[4 + w] = mx;
    }
    __syncthreads();
    uint32_t ay = 0u, ax = 0u;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        ay = smax[v] > ay ? smax[v] : ay;
        ax = smax[4 + v] > ax ? smax[4 + v] : ax;
    }
    const StageScale sc{exp_for_bits(ay), exp_for_bits(ax)};
    stage_put<NO>(st, 0, dY, sc.kY, w, lane);
    stage_put<NI>(st, X_ROW, X, sc.kX, w, lane);
    __syncthreads();
    return sc;
}
#else
constexpr int ST_FLOATS = 128 * SW;
typedef float BiasAcc;
__device__ __forceinline__ void stage_init(float*) {}
// rows of accumulator-layout tiles -> stage[row0 + feature][32 * w + sample] (all 32 * NT rows; rows past a
// layer's width hold zeros in the tiles)
template <int NT>
__device__ __forceinline__ void stage_put(float* st, int row0, const f32x16 (&T)[NT], int w, int lane) {
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) st[(row0 + 32 * t + rho(r, h)) * SW + 32 * w + j] = amp_r(T[t][r]);  // AMP: fp16 X
}

#if ACN_DW_CSPLIT
// Consumer-side fp16x3 (ACN_DW_CSPLIT): the producers put fp32 values as before and publish the layer's
// workgroup max |dY| / |X| (pc_publish); each consumer scales what it reads by those powers of two, splits
// into hi / lo fp16 and contracts on v_mfma_f32_16x16x16_f16 (hi*hi + hi*lo + lo*hi): one MFMA per product
// term covers the 16 samples the four fp32 16x16x4 MFMAs did.  The bias sums stay the exact fp32 VALU sums.
typedef _Float16 f16x4d __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16hd(const f16x4d& a, const f16x4d& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}
template <int NT>
__device__ __forceinline__ uint32_t wave_absmax_bits(const f32x16 (&T)[NT]) {
    uint32_t m = 0u;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t b = __float_as_uint(T[t][r]) & 0x7fffffffu;
            m = b > m ? b : m;
        }
    auto dmax = [](uint32_t v, uint32_t w) { return v > w ? v : w; };
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0xB1, 0xF, 0xF, false));
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x4E, 0xF, 0xF, false));
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x141, 0xF, 0xF, false));
    m = dmax(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x140, 0xF, 0xF, false));
    return dmax(dmax((uint32_t)__builtin_amdgcn_readlane((int)m, 0), (uint32_t)__builtin_amdgcn_readlane((int)m, 16)),
                dmax((uint32_t)__builtin_amdgcn_readlane((int)m, 32), (uint32_t)__builtin_amdgcn_readlane((int)m, 48)));
}
__device__ __forceinline__ int exp_for_bits(uint32_t w) {  // as tile_scale_exp
    if (w == 0u || w >= 0x7f800000u) return 0;
    const int be = (int)(w >> 23);
    const int k = 14 - ((be == 0 ? -126 : be - 127) + 1);
    return k > 100 ? 100 : (k < -100 ? -100 : k);
}
__device__ __forceinline__ void split4(const f32x4& x, float sc, f16x4d& hi, f16x4d& lo) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const f32x2 v = (f32x2){x[2 * u], x[2 * u + 1]} * (f32x2){sc, sc};
        const f16x2 h = __builtin_convertvector(v, f16x2);
        const f16x2 l = __builtin_convertvector(v - __builtin_convertvector(h, f32x2), f16x2);
        hi[2 * u] = h[0];
        hi[2 * u + 1] = h[1];
        lo[2 * u] = l[0];
        lo[2 * u + 1] = l[1];
    }
}
#endif

// acc[n] += dY[16 rows from arow] . X[16 features from xrow + 16 n]^T over the 128 staged samples;
// lane (i = l & 15, q = l >> 4) supplies k = sample 32 q + kk (4 k-steps per 16-B read).  bsum += this
// lane's share of the bias row sum (the A operand is dY itself).
template <int NCB, bool PIPE = (ACN_DW_PIPE != 0)>
__device__ __forceinline__ void dw_blocks(const float* st, int arow, int xrow, f32x4 (&acc)[NCB], float& bsum,
                                          StageScale sc, int lane) {
#if ACN_DIAG_NODW  // diagnostic build only: no weight-gradient contraction
    return;
#endif
    const int i = lane & 15, q = lane >> 4;
    const float* pa = st + (arow + i) * SW + 32 * q;
    const float* pb = st + (xrow + i) * SW + 32 * q;
#if ACN_DW_CSPLIT
    const float sa = ldexpf(1.0f, sc.kY), sb = ldexpf(1.0f, sc.kX), uab = ldexpf(1.0f, -(sc.kY + sc.kX));
    f32x4 tmp[NCB];
#pragma unroll
    for (int n = 0; n < NCB; ++n) tmp[n] = 0.0f;
#pragma unroll
    for (int k4 = 0; k4 < 8; ++k4) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(pa + 4 * k4);
        bsum += (a[0] + a[1]) + (a[2] + a[3]);
        f16x4d ah, al;
        split4(a, sa, ah, al);
#pragma unroll
        for (int n = 0; n < NCB; ++n) {
            const f32x4 b = *reinterpret_cast<const f32x4*>(pb + 16 * n * SW + 4 * k4);
            f16x4d bh, bl;
            split4(b, sb, bh, bl);
            tmp[n] = mfma16hd(al, bh, tmp[n]);
            tmp[n] = mfma16hd(ah, bl, tmp[n]);
            tmp[n] = mfma16hd(ah, bh, tmp[n]);
        }
    }
#pragma unroll
    for (int n = 0; n < NCB; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[n][r] = __builtin_fmaf(tmp[n][r], uab, acc[n][r]);
    return;
#else
    (void)sc;
#endif
    if (PIPE) {
    // software-pipelined: the next k-step's A / B vectors are read while this one's MFMAs run, and the MFMAs
    // of the NCB independent blocks alternate (each block's own chain keeps its k order: the same sums bit for
    // bit as the plain loop below)
    f32x4 a = *reinterpret_cast<const f32x4*>(pa);
    f32x4 b[NCB];
#pragma unroll
    for (int n = 0; n < NCB; ++n) b[n] = *reinterpret_cast<const f32x4*>(pb + 16 * n * SW);
#pragma unroll
    for (int k4 = 0; k4 < 8; ++k4) {
        f32x4 an = a, bn[NCB];
#pragma unroll
        for (int n = 0; n < NCB; ++n) bn[n] = b[n];
        if (k4 < 7) {
            an = *reinterpret_cast<const f32x4*>(pa + 4 * (k4 + 1));
#pragma unroll
            for (int n = 0; n < NCB; ++n) bn[n] = *reinterpret_cast<const f32x4*>(pb + 16 * n * SW + 4 * (k4 + 1));
        }
        bsum += (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int n = 0; n < NCB; ++n) acc[n] = mfma16(a[e], b[n][e], acc[n]);
        a = an;
#pragma unroll
        for (int n = 0; n < NCB; ++n) b[n] = bn[n];
    }
    return;
    }
#pragma unroll
    for (int k4 = 0; k4 < 8; ++k4) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(pa + 4 * k4);
        bsum += (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
        for (int n = 0; n < NCB; ++n) {
            const f32x4 b = *reinterpret_cast<const f32x4*>(pb + 16 * n * SW + 4 * k4);
            acc[n] = mfma16(a[0], b[0], acc[n]);
            acc[n] = mfma16(a[1], b[1], acc[n]);
            acc[n] = mfma16(a[2], b[2], acc[n]);
            acc[n] = mfma16(a[3], b[3], acc[n]);
        }
    }
}

// one layer's stage round: barrier (previous readers done), put dY / X, barrier
template <int NO, int NI>
__device__ __forceinline__ StageScale stage_layer(float* st, const f32x16 (&dY)[NO], const f32x16 (&X)[NI], int w,
                                                  int lane) {
#if ACN_DW_CSPLIT   // the workgroup's max |dY| / |X| travel with the stage (the consumer-side split's scales)
    __shared__ uint32_t smax_c[8];
    const uint32_t my = wave_absmax_bits<NO>(dY), mx = wave_absmax_bits<NI>(X);
    if (lane == 0) {
        smax_c[w] = my;
        smax_c[4 + w] = mx;
    }
#endif
    __syncthreads();
#if ACN_DW_CSPLIT   // read between the barriers: no wave can overwrite them (next layer) before all have read
    uint32_t ay = 0u, ax = 0u;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        ay = smax_c[v] > ay ? smax_c[v] : ay;
        ax = smax_c[4 + v] > ax ? smax_c[4 + v] : ax;
    }
#endif
    stage_put<NO>(st, 0, dY, w, lane);
    stage_put<NI>(st, X_ROW, X, w, lane);
    __syncthreads();
#if ACN_DW_CSPLIT
    return StageScale{exp_for_bits(ay), exp_for_bits(ax)};
#endif
    return StageScale{0, 0};
}
#endif

// D (16x16x4 layout: lane l, reg r = row 4 (l >> 4) + r, col l & 15) of one block -> dst rows / cols
template <typename Put>
__device__ __forceinline__ void flush_block(const f32x4& d, int lane, Put put) {
#pragma unroll
    for (int r = 0; r < 4; ++r) put(4 * (lane >> 4) + r, lane & 15, d[r]);
}

// expert of pair slot p (segment starts seg[0..K], routed.hip)
__device__ __forceinline__ int seg_expert(const int64_t* seg, int K, int64_t p) {
    int k = 0;
    while (k + 1 < K && seg[k + 1] <= p) ++k;
    return k;
}

// the 14 weight-gradient blocks of one wave (56 accumulator registers) and its bias partial sums
struct DwAcc {
    f32x4 aWC2[1], aWC1[4], aWC0[2], aHD[1], aW1[4], aW0[2];
    BiasAcc bWC2, bWC1, bWC0, bHD, bW1, bW0;
};

__device__ __forceinline__ void dw_zero(DwAcc& a) {
    a.aWC2[0] = 0.0f; a.aHD[0] = 0.0f;
#pragma unroll
    for (int n = 0; n < 4; ++n) { a.aWC1[n] = 0.0f; a.aW1[n] = 0.0f; }
#pragma unroll
    for (int n = 0; n < 2; ++n) { a.aWC0[n] = 0.0f; a.aW0[n] = 0.0f; }
    a.bWC2 = a.bWC1 = a.bWC0 = a.bHD = a.bW1 = a.bW0 = 0.0f;
}

#ifndef ACN_DW_PC
#define ACN_DW_PC 1  // mlp_bwd_dw_pc_kernel (producer / consumer waves) for acn_mlp_train_bwd_dw
#endif
#ifndef ACN_DW_DIAG
#define ACN_DW_DIAG 0  // diagnostic builds: shader-clock cycles per phase of mlp_bwd_dw_kernel (acn_mlp_dw_diag)
#endif
#if ACN_DW_DIAG
__device__ unsigned long long g_dw_diag[MAX_DW_BLOCKS * 4][8];
struct DwClock {
    uint64_t c[8];
    uint64_t t;
};
#define DW_T0(dc) (dc).t = __builtin_amdgcn_s_memtime()
#define DW_LAP(dc, i)                                              \
    do {                                                           \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();        \
        (dc).c[i] += now_ - (dc).t;                                \
        (dc).t = now_;                                             \
    } while (0)
#else
struct DwClock {};
#define DW_T0(dc) (void)0
#define DW_LAP(dc, i) (void)0
#endif

// one round: wave w re-runs the forward of its tile (samples m = tile * 32 + j), runs the backward chain
// and adds its share of every layer's [dW | db] over the workgroup's 128 samples; barriers inside
__device__ __forceinline__ void dw_round(const float* W, float* st, const float* __restrict__ h0,
                                         const float* __restrict__ sh, const float* __restrict__ out,
                                         const float* __restrict__ gout, int64_t m, bool ok, int w, int lane,
                                         float* __restrict__ gh0, DwAcc& a, DwClock& dc) {
    const int h = lane >> 5;
    f32x16 A1[2], A2[2], Hd[1], Cin[1], C1[2], C2[2], Rg[1];
    DW_T0(dc);
    {
        f32x16 X0[1];
        tile_forward(W, h0, sh, m, ok, lane, X0, A1, A2, Hd, Cin, C1, C2, Rg);
    }
    DW_LAP(dc, 0);
    f32x16 dRg[1], dHd[1];
    dRg[0] = 0.0f;
    float dsig = 0.0f;
    if (ok) {
        if (h == 0) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float y = out[m * 4 + c];
                dRg[0][c] = grad_rgb(gout[m * 4 + c], y);
            }
        } else {
            dsig = grad_sigma(gout[m * 4 + 3], out[m * 4 + 3]);
        }
    }
    DW_LAP(dc, 4);
    // colour head 3 x 64: column block w, rows 0..15 (0..2 live)
    {
        const StageScale sc = stage_layer<1, 2>(st, dRg, C2, w, lane);
        DW_LAP(dc, 1);
        dw_blocks<1>(st, 0, X_ROW + 16 * w, a.aWC2, a.bWC2, sc, lane);
        DW_LAP(dc, 2);
    }
    f32x16 G2[2], G1[2], Gc[1];
    bwd_layer<2, 1, 3, 32>(W + L_WC2, S64, dRg, G2, lane);
    relu_mask<2>(G2, C2);
    DW_LAP(dc, 3);
    // colour layer 1, 64 x 64: row block w
    {
        const StageScale sc = stage_layer<2, 2>(st, G2, C1, w, lane);
        DW_LAP(dc, 1);
        dw_blocks<4>(st, 16 * w, X_ROW, a.aWC1, a.bWC1, sc, lane);
        DW_LAP(dc, 2);
    }
    bwd_layer<2, 2, 64, 64>(W + L_WC1, S64, G2, G1, lane);
    relu_mask<2>(G1, C1);
    DW_LAP(dc, 3);
    // colour layer 0, 64 x 31 (input 31 = zero column): row block w
    {
        const StageScale sc = stage_layer<2, 1>(st, G1, Cin, w, lane);
        DW_LAP(dc, 1);
        dw_blocks<2>(st, 16 * w, X_ROW, a.aWC0, a.bWC0, sc, lane);
        DW_LAP(dc, 2);
    }
    bwd_layer<1, 2, 64, 64>(W + L_WC0, S32, G1, Gc, lane);  // d cin: rows 0..14 = d geo (SH rows dropped)
    DW_LAP(dc, 3);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int f = rho(r, h);
        dHd[0][r] = f < 15 ? Gc[0][r] : (f == 15 ? dsig : 0.0f);
    }
    // heads [geo 15 | sigma 1] x 64: column block w
    {
        const StageScale sc = stage_layer<1, 2>(st, dHd, A2, w, lane);
        DW_LAP(dc, 1);
        dw_blocks<1>(st, 0, X_ROW + 16 * w, a.aHD, a.bHD, sc, lane);
        DW_LAP(dc, 2);
    }
    f32x16 GA2[2], GA1[2], GH[1];
    bwd_layer<2, 1, 16, 32>(W + L_WH, S64, dHd, GA2, lane);
    relu_mask<2>(GA2, A2);
    DW_LAP(dc, 3);
    // sigma trunk 1, 64 x 64: row block w
    {
        const StageScale sc = stage_layer<2, 2>(st, GA2, A1, w, lane);
        DW_LAP(dc, 1);
        dw_blocks<4>(st, 16 * w, X_ROW, a.aW1, a.bW1, sc, lane);
        DW_LAP(dc, 2);
    }
    bwd_layer<2, 2, 64, 64>(W + L_W1, S64, GA2, GA1, lane);
    relu_mask<2>(GA1, A1);
    DW_LAP(dc, 3);
    // sigma trunk 0, 64 x 32: row block w
    f32x16 X0[1];
    load_tiles<1>(h0, 32, 0, 32, m, ok, h, X0);  // reloaded (L2-hot) rather than kept live
    {
        const StageScale sc = stage_layer<2, 1>(st, GA1, X0, w, lane);
        DW_LAP(dc, 1);
        dw_blocks<2>(st, 16 * w, X_ROW, a.aW0, a.bW0, sc, lane);
        DW_LAP(dc, 2);
    }
    if (gh0) {
        bwd_layer<1, 2, 64, 64>(W + L_W0, S32, GA1, GH, lane);
        store_tiles<1>(gh0, 32, 0, 32, m, ok, h, GH);
    }
    DW_LAP(dc, 5);
}

// one copy of the 13,715 partial sums: every element has exactly one owner (wave, lane, register)
__device__ __forceinline__ void dw_flush(DwAcc& a, float* __restrict__ dst, int w, int lane0) {
    const int cw = 16 * w;
    flush_block(a.aWC2[0], lane0, [&](int o, int c, float v) { if (o < 3) dst[D_WC2 + 64 * o + cw + c] = v; });
    flush_block(a.aHD[0], lane0, [&](int o, int c, float v) {
        dst[o < 15 ? D_WG + 64 * o + cw + c : D_WSH + cw + c] = v;
    });
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        flush_block(a.aWC1[n], lane0, [&](int o, int c, float v) { dst[D_WC1 + 64 * (cw + o) + 16 * n + c] = v; });
        flush_block(a.aW1[n], lane0, [&](int o, int c, float v) { dst[D_W1 + 64 * (cw + o) + 16 * n + c] = v; });
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        flush_block(a.aWC0[n], lane0, [&](int o, int c, float v) {
            if (16 * n + c < 31) dst[D_WC0 + 31 * (cw + o) + 16 * n + c] = v;
        });
        flush_block(a.aW0[n], lane0, [&](int o, int c, float v) { dst[D_W0 + 32 * (cw + o) + 16 * n + c] = v; });
    }
#if ACN_DW_F16X3
    // bias rows = column 0 of the ones-row contraction blocks: lanes 0, 16, 32, 48 hold rows 4 (l >> 4) + r
    if ((lane0 & 15) == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * (lane0 >> 4) + r;
            if (w == 0) {
                if (i < 3) dst[D_BC2 + i] = a.bWC2[r];
                dst[i < 15 ? D_BG + i : D_BSH] = a.bHD[r];
            }
            dst[D_BC1 + cw + i] = a.bWC1[r];
            dst[D_BC0 + cw + i] = a.bWC0[r];
            dst[D_B1 + cw + i] = a.bW1[r];
            dst[D_B0 + cw + i] = a.bW0[r];
        }
    }
#else
    // bias rows: lane (i, q) holds the sum over samples 32 q .. 32 q + 31 of row i of its row block
    auto red = [](float v) { v += __shfl_xor(v, 16); return v + __shfl_xor(v, 32); };
    const float bWC2 = red(a.bWC2), bHD = red(a.bHD), bWC1 = red(a.bWC1), bWC0 = red(a.bWC0), bW1 = red(a.bW1),
                bW0 = red(a.bW0);
    if (lane0 < 16) {
        const int i = lane0;
        if (w == 0) {
            if (i < 3) dst[D_BC2 + i] = bWC2;
            dst[i < 15 ? D_BG + i : D_BSH] = bHD;
        }
        dst[D_BC1 + cw + i] = bWC1;
        dst[D_BC0 + cw + i] = bWC0;
        dst[D_B1 + cw + i] = bW1;
        dst[D_B0 + cw + i] = bW0;
    }
#endif
}

__global__ void __launch_bounds__(256) mlp_bwd_dw_kernel(const float* __restrict__ img, const float* __restrict__ h0,
                                                         const float* __restrict__ sh, const float* __restrict__ out,
                                                         const float* __restrict__ gout, int64_t M,
                                                         float* __restrict__ gh0, float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float Wl[L_FLOATS];
    __shared__ __attribute__((aligned(16))) float st_base[ST_FLOATS];
    stage_weights(img, Wl);
    stage_init(st_base);
    __syncthreads();
    const int lane0 = threadIdx.x & 63, j = lane0 & 31, w = threadIdx.x >> 6;
    const int64_t ntiles = (M + 31) / 32;
    DwAcc a;
    dw_zero(a);
    DwClock dc{};
    // rounds are uniform over the workgroup (barriers inside): tiles past the end have zero gradients
    for (int64_t base = (int64_t)blockIdx.x * 4; base < ntiles; base += (int64_t)gridDim.x * 4) {
        const int64_t m = (base + w) * 32 + j;
        dw_round(Wl + opaque_s(0), st_base + opaque_s(0), h0, sh, out, gout, m, m < M, w, opaque_v(lane0), gh0, a, dc);
    }
    DW_T0(dc);
    dw_flush(a, partial + (int64_t)blockIdx.x * NDW, w, lane0);
#if ACN_DW_DIAG
    DW_LAP(dc, 6);
    if (lane0 == 0)
        for (int i = 0; i < 8; ++i) g_dw_diag[blockIdx.x * 4 + w][i] = dc.c[i];
#endif
}

// Producer / consumer form of the fused backward (8-wave workgroups, two waves per SIMD).  Waves 0-3
// (producers) run exactly the per-tile work of dw_round -- forward recompute, the dX chain, ReLU masks --
// and put each layer's dY / X into the shared stage; waves 4-7 (consumers) hold the weight-gradient
// accumulators of the same row / column blocks wave w - 4 owned in dw_round and contract the stage.  Per
// layer: producers put -> barrier -> [producers: dX of the layer | consumers: dW of the layer] -> barrier,
// so the MFMA-bound contraction overlaps the producers' VALU-bound split / ReLU / dX work instead of
// following it, and neither role carries the other's registers.  The barrier that frees the stage for the
// next round sits at the HEAD of the producers' round (after the forward recompute), not at the end of the
// previous one, so the consumers' last layer (sigma trunk 0) runs beside the producers' dL/dh0 and their next
// forward recompute instead of in front of them.  Every wave executes the same barriers per
// round and the same rounds; with the fp32 stage the sums, their order and every output are those of
// mlp_bwd_dw_kernel bit for bit (same owners, same stage, same k order).
//   fp16 stages: the AMP build puts fp16 values unscaled (one plane); the fp16x3 stage (ACN_DW_F16X3 in the
// default build) scales dY and X by workgroup-uniform powers of two: each producer wave publishes its max
// |dY| / |X| of the NEXT layer right after computing that layer's dY (before the barrier that ends the
// current layer), into one of two alternating LDS slots -- so the consumers, which read the current layer's
// exponents after its put barrier, never race the producers' next publish; one extra barrier per round
// publishes the first layer's maxima.
#ifndef ACN_DIAG_NOPROD
#define ACN_DIAG_NOPROD 0
#endif
#if ACN_DIAG_NOPROD
#define PC_BWD(...) (void)0
#else
#define PC_BWD(...) __VA_ARGS__
#endif
__device__ __forceinline__ void pc_sync() { __syncthreads(); }
#ifndef ACN_DW_PRIO
#define ACN_DW_PRIO 0   // wave priority in mlp_bwd_dw_pc_kernel: 1 producers raised, 2 consumers raised (A/B)
#endif
#ifndef ACN_DW_PREFETCH
#define ACN_DW_PREFETCH 1   // producers: vector loads of h0 / SH / outputs issued ahead of their use (0: in place)
#endif
#ifndef ACN_DW_HEADSYNC
#define ACN_DW_HEADSYNC 1   // the stage-free barrier at the head of the producers' round (0: at the end, round 5)
#endif
constexpr bool kPcScaled = (ACN_DW_F16X3 && !ACN_TRAIN_AMP) || ACN_DW_CSPLIT;

template <int NO, int NI>
__device__ __forceinline__ void pc_publish(uint32_t* smax, const f32x16 (&dY)[NO], const f32x16 (&X)[NI], int w,
                                           int lane) {
#if (ACN_DW_F16X3 && !ACN_TRAIN_AMP) || ACN_DW_CSPLIT
    const uint32_t my = wave_absmax_bits<NO>(dY), mx = wave_absmax_bits<NI>(X);
    if (lane == 0) {
        smax[w] = my;
        smax[4 + w] = mx;
    }
#else
    (void)smax; (void)dY; (void)X; (void)w; (void)lane;
#endif
}
__device__ __forceinline__ StageScale pc_scale(const uint32_t* smax) {
#if (ACN_DW_F16X3 && !ACN_TRAIN_AMP) || ACN_DW_CSPLIT
    uint32_t ay = 0u, ax = 0u;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        ay = smax[v] > ay ? smax[v] : ay;
        ax = smax[4 + v] > ax ? smax[4 + v] : ax;
    }
    return StageScale{exp_for_bits(ay), exp_for_bits(ax)};
#else
    (void)smax;
    return StageScale{0, 0};
#endif
}
template <int NO, int NI>
__device__ __forceinline__ void pc_put(float* st, const f32x16 (&dY)[NO], const f32x16 (&X)[NI], const uint32_t* smax,
                                       int w, int lane) {
#if ACN_DW_F16X3
    const StageScale sc = pc_scale(smax);
    stage_put<NO>(st, 0, dY, sc.kY, w, lane);
    stage_put<NI>(st, X_ROW, X, sc.kX, w, lane);
#else
    (void)smax;
    stage_put<NO>(st, 0, dY, w, lane);
    stage_put<NI>(st, X_ROW, X, w, lane);
#endif
}

// layer L (1 = colour head ... 6 = sigma trunk 0) uses maxima slot (L - 1) & 1
__device__ __forceinline__ void pc_producer_round(const float* W, float* st, uint32_t* smax,
                                                  const float* __restrict__ h0, const float* __restrict__ sh,
                                                  const float* __restrict__ out, const float* __restrict__ gout,
                                                  int64_t m, bool ok, int w, int lane, float* __restrict__ gh0,
                                                  X0Raw& X0n, int64_t mn, bool okn) {
    const int h = lane >> 5;
    uint32_t* s0 = smax;
    uint32_t* s1 = smax + 8;
    f32x16 A1[2], A2[2], Hd[1], Cin[1], C1[2], C2[2], Rg[1];
#if ACN_DW_PREFETCH
    // X0n holds this round's h0 tile (loaded during the previous round); the SH row and the output / output-
    // gradient vectors are issued before the forward recompute and consumed after its first layers
    PcIn in;
#endif
#if ACN_DIAG_NOPROD  // diagnostic build only: no forward recompute (zero activations): the consumers' time
    A1[0] = A1[1] = A2[0] = A2[1] = Hd[0] = Cin[0] = C1[0] = C1[1] = C2[0] = C2[1] = Rg[0] = 0.0f;
    (void)sh;
#elif ACN_DW_PREFETCH
    tile_forward_x(W, X0n, sh, out, gout, m, ok, lane, in, A1, A2, Hd, Cin, C1, C2, Rg);
    __builtin_amdgcn_sched_barrier(0);
#else
    {
        f32x16 X0[1];
        tile_forward(W, h0, sh, m, ok, lane, X0, A1, A2, Hd, Cin, C1, C2, Rg);
    }
#endif
    f32x16 dRg[1], dHd[1];
    dRg[0] = 0.0f;
    float dsig = 0.0f;
#if ACN_DW_PREFETCH
    {   // selects, not a branch: a branch would let the compiler sink the prefetched loads into it
        const bool rgb = ok && h == 0, sg = ok && h != 0;
        float gv[3], ov[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            gv[c] = opaque_f(in.g[c]);
            ov[c] = opaque_f(in.o[c]);
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) dRg[0][c] = rgb ? grad_rgb(gv[c], ov[c]) : 0.0f;
        dsig = sg ? grad_sigma(gv[0], ov[0]) : 0.0f;
    }
#else
    if (ok) {
        if (h == 0) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float y = out[m * 4 + c];
                dRg[0][c] = grad_rgb(gout[m * 4 + c], y);
            }
        } else {
            dsig = grad_sigma(gout[m * 4 + 3], out[m * 4 + 3]);
        }
    }
#endif
    // colour head
    if (kPcScaled) {
        pc_publish<1, 2>(s0, dRg, C2, w, lane);
        pc_sync();
    }
    if (ACN_DW_HEADSYNC) pc_sync();   // the consumers have finished the previous round's last layer: stage free
    pc_put<1, 2>(st, dRg, C2, s0, w, lane);
    pc_sync();
    f32x16 G2[2], G1[2], Gc[1];
    PC_BWD(bwd_layer<2, 1, 3, 32>(W + L_WC2, S64, dRg, G2, lane));
    relu_mask<2>(G2, C2);
    pc_publish<2, 2>(s1, G2, C1, w, lane);
    pc_sync();
    // colour layer 1
    pc_put<2, 2>(st, G2, C1, s1, w, lane);
    pc_sync();
    PC_BWD(bwd_layer<2, 2, 64, 64>(W + L_WC1, S64, G2, G1, lane));
    relu_mask<2>(G1, C1);
    pc_publish<2, 1>(s0, G1, Cin, w, lane);
    pc_sync();
    // colour layer 0
    pc_put<2, 1>(st, G1, Cin, s0, w, lane);
    pc_sync();
    PC_BWD(bwd_layer<1, 2, 64, 64>(W + L_WC0, S32, G1, Gc, lane));
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int f = rho(r, h);
        dHd[0][r] = f < 15 ? Gc[0][r] : (f == 15 ? dsig : 0.0f);
    }
    pc_publish<1, 2>(s1, dHd, A2, w, lane);
    pc_sync();
    // heads
    pc_put<1, 2>(st, dHd, A2, s1, w, lane);
    pc_sync();
    f32x16 GA2[2], GA1[2], GH[1];
    PC_BWD(bwd_layer<2, 1, 16, 32>(W + L_WH, S64, dHd, GA2, lane));
    relu_mask<2>(GA2, A2);
    pc_publish<2, 2>(s0, GA2, A1, w, lane);
    pc_sync();
    // sigma trunk 1
    pc_put<2, 2>(st, GA2, A1, s0, w, lane);
    pc_sync();
    f32x16 X0[1];
#if ACN_DW_PREFETCH
    X0Raw x0c;
    load_x0raw(h0, m, ok, h, x0c);   // reloaded (L2-hot) for the last layer, issued before this layer's dX
    __builtin_amdgcn_sched_barrier(0);
#endif
    PC_BWD(bwd_layer<2, 2, 64, 64>(W + L_W1, S64, GA2, GA1, lane));
    relu_mask<2>(GA1, A1);
#if ACN_DW_PREFETCH
    __builtin_amdgcn_sched_barrier(0);
    x0_tile(x0c, ok, X0);
#else
    load_tiles<1>(h0, 32, 0, 32, m, ok, h, X0);
#endif
    pc_publish<2, 1>(s1, GA1, X0, w, lane);
    pc_sync();
    // sigma trunk 0
    pc_put<2, 1>(st, GA1, X0, s1, w, lane);
    pc_sync();
#if ACN_DW_PREFETCH
    load_x0raw(h0, mn, okn, h, X0n);   // the next round's h0 tile, behind dL/dh0 and the consumers' last layer
    __builtin_amdgcn_sched_barrier(0);
#else
    (void)X0n; (void)mn; (void)okn;
#endif
    if (gh0) {   // overlaps the consumers' last layer (and the next round's forward recompute follows)
        PC_BWD(bwd_layer<1, 2, 64, 64>(W + L_W0, S32, GA1, GH, lane));
        store_tiles<1>(gh0, 32, 0, 32, m, ok, h, GH);
    }
    if (!ACN_DW_HEADSYNC) pc_sync();
}

template <bool PIPE = (ACN_DW_PIPE != 0)>
__device__ __forceinline__ void pc_consumer_round(const float* st, const uint32_t* smax, int w, int lane, DwAcc& a) {
    const uint32_t* s0 = smax;
    const uint32_t* s1 = smax + 8;
    if (kPcScaled) pc_sync();
    if (ACN_DW_HEADSYNC) pc_sync();   // stage free (the producers' round-head barrier)
    pc_sync();
    dw_blocks<1, PIPE>(st, 0, X_ROW + 16 * w, a.aWC2, a.bWC2, pc_scale(s0), lane);
    pc_sync();
    pc_sync();
    dw_blocks<4, PIPE>(st, 16 * w, X_ROW, a.aWC1, a.bWC1, pc_scale(s1), lane);
    pc_sync();
    pc_sync();
    dw_blocks<2, PIPE>(st, 16 * w, X_ROW, a.aWC0, a.bWC0, pc_scale(s0), lane);
    pc_sync();
    pc_sync();
    dw_blocks<1, PIPE>(st, 0, X_ROW + 16 * w, a.aHD, a.bHD, pc_scale(s1), lane);
    pc_sync();
    pc_sync();
    dw_blocks<4, PIPE>(st, 16 * w, X_ROW, a.aW1, a.bW1, pc_scale(s0), lane);
    pc_sync();
    pc_sync();
    dw_blocks<2, PIPE>(st, 16 * w, X_ROW, a.aW0, a.bW0, pc_scale(s1), lane);
    if (!ACN_DW_HEADSYNC) pc_sync();
}

__global__ void __launch_bounds__(512) mlp_bwd_dw_pc_kernel(const float* __restrict__ img, const float* __restrict__ h0,
                                                            const float* __restrict__ sh, const float* __restrict__ out,
                                                            const float* __restrict__ gout, int64_t M,
                                                            float* __restrict__ gh0, float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float Wl[L_FLOATS];
    __shared__ __attribute__((aligned(16))) float st_base[ST_FLOATS];
    __shared__ uint32_t pc_smax[16];   // two alternating slots of the 4 producers' max |dY|, |X| bits
    stage_weights(img, Wl);
    stage_init(st_base);   // the fp16 stage's ones row (bias sums); nothing for the fp32 stage
    __syncthreads();
    const int lane0 = threadIdx.x & 63, j = lane0 & 31;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), w = wv & 3;
    const int64_t ntiles = (M + 31) / 32;
    // rounds are uniform over the workgroup (the same 12 -- 13 with the scaled stage -- barriers per round in
    // both roles)
    if (wv < 4) {
        if (ACN_DW_PRIO == 1) __builtin_amdgcn_s_setprio(2);   // the producers' chain is the critical path
        const int64_t step = (int64_t)gridDim.x * 4;
        X0Raw X0n;
#if ACN_DW_PREFETCH
        {
            const int64_t m0 = ((int64_t)blockIdx.x * 4 + w) * 32 + j;
            load_x0raw(h0, m0, m0 < M, lane0 >> 5, X0n);
        }
#endif
        for (int64_t base = (int64_t)blockIdx.x * 4; base < ntiles; base += step) {
            const int64_t m = (base + w) * 32 + j, mn = m + step * 32;
            pc_producer_round(Wl + opaque_s(0), st_base + opaque_s(0), pc_smax, h0, sh, out, gout, m, m < M, w,
                              opaque_v(lane0), gh0, X0n, mn, mn < M);
        }
    } else {
        if (ACN_DW_PRIO == 2) __builtin_amdgcn_s_setprio(2);
        DwAcc a;
        dw_zero(a);
        for (int64_t base = (int64_t)blockIdx.x * 4; base < ntiles; base += (int64_t)gridDim.x * 4)
            pc_consumer_round(st_base + opaque_s(0), pc_smax, w, opaque_v(lane0), a);
        dw_flush(a, partial + (int64_t)blockIdx.x * NDW, w, lane0);
    }
}

// Pair-list variant (routed container): workgroup b takes the contiguous rounds [b R / G, (b+1) R / G)
// (R = seg[K] / 128 from the device); when the expert of the next round differs, the running sums go
// to copy (b, expert) and restart, and the new expert's image is staged.  mlp_dw_reduce_pairs_kernel
// adds, per expert, the copies of the workgroups whose range met that expert's rounds (in b order:
// deterministic, no atomics).  Padding slots carry zero output gradients.
__global__ void __launch_bounds__(256) mlp_bwd_dw_pairs_kernel(const float* __restrict__ imgs,
                                                               const float* __restrict__ h0,
                                                               const float* __restrict__ sh,
                                                               const float* __restrict__ out,
                                                               const float* __restrict__ gout,
                                                               const int64_t* __restrict__ seg, int K,
                                                               float* __restrict__ gh0, float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float Wl[L_FLOATS];
    __shared__ __attribute__((aligned(16))) float st_base[ST_FLOATS];
    stage_init(st_base);  // published by the staging barrier of the first round
    const int lane0 = threadIdx.x & 63, j = lane0 & 31, w = threadIdx.x >> 6;
    const int64_t R = seg[K] / 128, G = gridDim.x;
    const int64_t r0 = (int64_t)blockIdx.x * R / G, r1 = ((int64_t)blockIdx.x + 1) * R / G;
    DwAcc a;
    dw_zero(a);
    int cur = -1;
    for (int64_t rd = r0; rd < r1; ++rd) {
        const int k = seg_expert(seg, K, rd * 128);
        if (k != cur) {
            if (cur >= 0) {
                dw_flush(a, partial + ((int64_t)blockIdx.x * K + cur) * NDW, w, lane0);
                dw_zero(a);
            }
            __syncthreads();
            stage_weights(imgs + (int64_t)k * L_FLOATS, Wl);
            __syncthreads();
            cur = k;
        }
        const int64_t m = (rd * 4 + w) * 32 + j;
        DwClock dcp{};
        dw_round(Wl + opaque_s(0), st_base + opaque_s(0), h0, sh, out, gout, m, true, w, opaque_v(lane0), gh0, a, dcp);
    }
    if (cur >= 0) dw_flush(a, partial + ((int64_t)blockIdx.x * K + cur) * NDW, w, lane0);
}

// dw[e] = sum over the nblk partial copies: a block sums 32 consecutive elements, its 8 thread rows
// stride over the copies (128-B coalesced rows), then the rows are added in LDS
__global__ void __launch_bounds__(256) mlp_dw_reduce_kernel(const float* __restrict__ partial, int nblk,
                                                            float* __restrict__ dw) {
    __shared__ float red[8][32];
    const int c = threadIdx.x & 31, row = threadIdx.x >> 5;
    const int e = blockIdx.x * 32 + c;
    float s = 0.0f;
    if (e < NDW) {
        // same summation order; unrolled so the loads of 8 copies are in flight together (a dependent
        // load per iteration made this a chain of 32 memory latencies: 11.5 us per call)
#pragma unroll 8
        for (int b = row; b < nblk; b += 8) s += partial[(int64_t)b * NDW + e];
    }
    red[row][c] = s;
    __syncthreads();
    if (row == 0 && e < NDW) {
        float t = red[0][c];
#pragma unroll
        for (int k = 1; k < 8; ++k) t += red[k][c];
        dw[e] = amp_r(t);  // AMP: the fp16 GEMM output rounding of [dW | db]
    }
}


// ---------------------------------------------------------------------------------------------
// Routed pair lists (routed.hip): slots grouped by expert, every expert's segment padded to a multiple
// of 128 (one round = 4 tiles = 128 slots of ONE expert); the slot count seg[K] lives on the device, so
// grids are fixed and the kernels stride to it (HIP-graph replayable).  A workgroup stages the weight
// image of the expert of its current round and restages when the expert changes.

__global__ void __launch_bounds__(256) mlp_fwd_pairs_kernel(const float* __restrict__ imgs, const float* __restrict__ h0,
                                                            const float* __restrict__ sh,
                                                            const int64_t* __restrict__ seg, int K,
                                                            float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float Wl[L_FLOATS];
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31, w = threadIdx.x >> 6;
    const int64_t rounds = seg[K] / 128;
    int cur = -1;
    for (int64_t rd = blockIdx.x; rd < rounds; rd += gridDim.x) {
        const int k = seg_expert(seg, K, rd * 128);
        if (k != cur) {
            __syncthreads();
            stage_weights(imgs + (int64_t)k * L_FLOATS, Wl);
            __syncthreads();
            cur = k;
        }
        const int64_t m = (rd * 4 + w) * 32 + j;
        f32x16 X0[1], A1[2], A2[2], Hd[1], Cin[1], C1[2], C2[2], Rg[1];
        tile_forward(Wl, h0, sh, m, true, lane, X0, A1, A2, Hd, Cin, C1, C2, Rg);
        if (h == 0) {
#pragma unroll
            for (int c = 0; c < 3; ++c) out[m * 4 + c] = out_rgb(Rg[0][c]);
        } else {
            out[m * 4 + 3] = out_sigma(Hd[0][7]);
        }
    }
}

// Producer / consumer form of the pair-list backward (the routed container's C5 step): mlp_bwd_dw_pc_kernel's
// roles, barriers and prefetch over mlp_bwd_dw_pairs_kernel's contiguous round range per workgroup.  When the
// expert of the next round differs, both roles pass two barriers around the restaging of that expert's image
// (the consumers first write their running sums to copy (b, expert) and restart), so the barrier sequence
// stays the same in both roles.  Same owners, same stage, same k order as dw_round: bitwise the outputs of
// mlp_bwd_dw_pairs_kernel.
#ifndef ACN_DW_PAIRS_PC
#define ACN_DW_PAIRS_PC 1   // 0: mlp_bwd_dw_pairs_kernel (one role per wave)
#endif
#if ACN_DW_PAIRS_PC
__global__ void __launch_bounds__(512) mlp_bwd_dw_pairs_pc_kernel(const float* __restrict__ imgs,
                                                                  const float* __restrict__ h0,
                                                                  const float* __restrict__ sh,
                                                                  const float* __restrict__ out,
                                                                  const float* __restrict__ gout,
                                                                  const int64_t* __restrict__ seg, int K,
                                                                  float* __restrict__ gh0, float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float Wl[L_FLOATS];
    __shared__ __attribute__((aligned(16))) float st_base[ST_FLOATS];
    __shared__ uint32_t pc_smax[16];
    stage_init(st_base);   // published by the staging barriers of the first round
    const int lane0 = threadIdx.x & 63, j = lane0 & 31;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), w = wv & 3;
    const int64_t R = seg[K] / 128, G = gridDim.x;
    const int64_t r0 = (int64_t)blockIdx.x * R / G, r1 = ((int64_t)blockIdx.x + 1) * R / G;
    // one pass per run of rounds of one expert: both roles restage that expert's image between two barriers, the
    // consumers zero their sums before the run and write copy (b, expert) after it (no accumulator state
    // crosses a run, so the compiler keeps the sums in place)
    int64_t rd = r0;
    if (wv < 4) {
        X0Raw X0n;
#if ACN_DW_PREFETCH
        if (r0 < r1) load_x0raw(h0, (r0 * 4 + w) * 32 + j, true, lane0 >> 5, X0n);
#endif
        while (rd < r1) {
            const int k = seg_expert(seg, K, rd * 128);
            __syncthreads();
            stage_weights(imgs + (int64_t)k * L_FLOATS, Wl);
            __syncthreads();
            for (; rd < r1 && seg_expert(seg, K, rd * 128) == k; ++rd) {
                const int64_t m = (rd * 4 + w) * 32 + j, mn = m + 128;
                pc_producer_round(Wl + opaque_s(0), st_base + opaque_s(0), pc_smax, h0, sh, out, gout, m, true, w,
                                  opaque_v(lane0), gh0, X0n, mn, rd + 1 < r1);
            }
        }
    } else {
        while (rd < r1) {
            const int k = seg_expert(seg, K, rd * 128);
            __syncthreads();
            stage_weights(imgs + (int64_t)k * L_FLOATS, Wl);
            __syncthreads();
            DwAcc a;
            dw_zero(a);
            for (; rd < r1 && seg_expert(seg, K, rd * 128) == k; ++rd)
                // the unpipelined contraction: the pipelined one's register allocation here leaves a 6-state
                // WAR-on-C gap under tests/test_hazard_audit.py's margin
                pc_consumer_round<false>(st_base + opaque_s(0), pc_smax, w, opaque_v(lane0), a);
            dw_flush(a, partial + ((int64_t)blockIdx.x * K + k) * NDW, w, lane0);
        }
    }
}
#endif

// dw[k][e] = sum over the workgroups b whose round range [b R / G, (b+1) R / G) met expert k's rounds of
// copy (b, k); zero for an expert without pairs.  grid (NDW / 32, K)
__global__ void __launch_bounds__(256) mlp_dw_reduce_pairs_kernel(const float* __restrict__ partial,
                                                                  const int64_t* __restrict__ seg, int K, int G,
                                                                  float* __restrict__ dw) {
    __shared__ float red[8][32];
    const int c = threadIdx.x & 31, row = threadIdx.x >> 5;
    const int k = blockIdx.y;
    const int e = blockIdx.x * 32 + c;
    const int64_t R = seg[K] / 128, k0 = seg[k] / 128, k1 = seg[k + 1] / 128;
    float s = 0.0f;
    if (e < NDW && k1 > k0) {
        // only the workgroups whose round range [b R / G, (b+1) R / G) meets [k0, k1) hold a copy (the
        // ranges are monotone in b: stop past k1); same summation order as before, the loads issued
        // unconditionally (every copy slot is allocated) so 8 copies are in flight together -- a
        // load under the condition made this a chain of memory latencies (40 us per step at K = 8)
        // first b whose range can meet [k0, k1): (b + 1) R / G > k0 needs b >= k0 G / R - 1
        const int64_t bf = R > 0 ? (k0 * G) / R - 1 : 0;
        const int b0 = (int)((bf < 0 ? 0 : bf) & ~(int64_t)7) + row;  // same residue mod 8: same order
#pragma unroll 8
        for (int b = b0; b < G; b += 8) {
            const int64_t lo = (int64_t)b * R / G, hi = ((int64_t)b + 1) * R / G;
            if (lo >= k1) break;
            const float v = partial[((int64_t)b * K + k) * NDW + e];
            if (lo < hi && hi > k0) s += v;
        }
    }
    red[row][c] = s;
    __syncthreads();
    if (row == 0 && e < NDW) {
        float t = red[0][c];
#pragma unroll
        for (int q = 1; q < 8; ++q) t += red[q][c];
        dw[(int64_t)k * NDW + e] = amp_r(t);
    }
}

MlpPtrs ptrs(const acn_mlp* w) {
    return MlpPtrs{w->w0, w->b0, w->w1, w->b1, w->wsh, w->bsh, w->wg, w->bg,
                   w->wc0, w->bc0, w->wc1, w->bc1, w->wc2, w->bc2};
}

unsigned grid_for(int64_t M) {  // 4 waves per block, grid-stride over 32-sample tiles, ~2 blocks per CU
    const int64_t tiles = (M + 31) / 32, blocks = (tiles + 3) / 4;
    return (unsigned)(blocks < 512 ? (blocks < 1 ? 1 : blocks) : 512);
}

}  // namespace

extern "C" size_t ACN_MLP_API(acn_mlp_workspace_bytes)(void) { return (size_t)L_FLOATS * sizeof(float); }

extern "C" int ACN_MLP_API(acn_mlp_train_fwd)(const float* h0, const float* sh, int64_t M, const acn_mlp* w, float* out,
                                 float* save, void* workspace, void* stream) {
    ACN_REQUIRE(M >= 0 && w && workspace, "acn_mlp_train_fwd: bad arguments");
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(h0 && sh && out, "acn_mlp_train_fwd: NULL pointer");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(mlp_pack_kernel, dim3((L_FLOATS + 255) / 256), dim3(256), 0, s, ptrs(w), (float*)workspace);
    if (save)
        hipLaunchKernelGGL(mlp_fwd_kernel<true>, dim3(grid_for(M)), dim3(256), 0, s, (const float*)workspace, h0, sh, M,
                           out, save);
    else {
        const int64_t blocks = ((M + 31) / 32 + 7) / 8;
        hipLaunchKernelGGL(mlp_fwd_kernel<false>, dim3((unsigned)(blocks < 512 ? blocks : 512)), dim3(512), 0, s,
                           (const float*)workspace, h0, sh, M, out, save);
    }
    return acn_check_launch("acn_mlp_train_fwd");
}

extern "C" int ACN_MLP_API(acn_mlp_train_bwd)(const float* save, const float* out, const float* gout, int64_t M, const acn_mlp* w,
                                 float* gsave, float* gh0, void* workspace, void* stream) {
    ACN_REQUIRE(M >= 0 && w && workspace, "acn_mlp_train_bwd: bad arguments");
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(save && out && gout && gsave, "acn_mlp_train_bwd: NULL pointer");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(mlp_pack_kernel, dim3((L_FLOATS + 255) / 256), dim3(256), 0, s, ptrs(w), (float*)workspace);
    hipLaunchKernelGGL(mlp_bwd_kernel, dim3(grid_for(M)), dim3(256), 0, s, (const float*)workspace, save, out, gout,
                       M, gsave, gh0);
    return acn_check_launch("acn_mlp_train_bwd");
}

#if ACN_DW_DIAG
extern "C" int ACN_MLP_API(acn_mlp_dw_diag)(unsigned long long* host, int nblk) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dw_diag), (size_t)nblk * 4 * 8 * sizeof(unsigned long long));
}
#endif

extern "C" size_t ACN_MLP_API(acn_mlp_dw_workspace_bytes)(void) {
    return ((size_t)L_FLOATS + (size_t)MAX_DW_BLOCKS * NDW) * sizeof(float);
}

namespace {
// the fused backward + the copy reduction, on a packed weight image
int bwd_dw_launch(const float* h0, const float* sh, const float* out, const float* gout, int64_t M, const float* img,
                  float* dw, float* gh0, float* partial, hipStream_t s) {
    const int64_t tiles = (M + 31) / 32, want = (tiles + 3) / 4;
    const int nblk = (int)(want < MAX_DW_BLOCKS ? want : MAX_DW_BLOCKS);
#if ACN_DW_PC
    hipLaunchKernelGGL(mlp_bwd_dw_pc_kernel, dim3(nblk), dim3(512), 0, s, img, h0, sh, out, gout, M, gh0, partial);
#else
    hipLaunchKernelGGL(mlp_bwd_dw_kernel, dim3(nblk), dim3(256), 0, s, img, h0, sh, out, gout, M, gh0, partial);
#endif
    hipLaunchKernelGGL(mlp_dw_reduce_kernel, dim3((NDW + 31) / 32), dim3(256), 0, s, (const float*)partial, nblk,
                       dw);
    return acn_check_launch("acn_mlp_train_bwd_dw");
}
}  // namespace

extern "C" int ACN_MLP_API(acn_mlp_train_bwd_dw)(const float* h0, const float* sh, const float* out, const float* gout, int64_t M,
                                    const acn_mlp* w, float* dw, float* gh0, void* workspace, void* stream) {
    ACN_REQUIRE(M >= 0 && w && workspace && dw, "acn_mlp_train_bwd_dw: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    if (M == 0) {
        const hipError_t e = hipMemsetAsync(dw, 0, (size_t)NDW * sizeof(float), s);
        return e == hipSuccess ? ACN_OK : acn_set_error((int)e, "acn_mlp_train_bwd_dw: memset failed");
    }
    ACN_REQUIRE(h0 && sh && out && gout, "acn_mlp_train_bwd_dw: NULL pointer");
    float* img = (float*)workspace;
    float* partial = img + L_FLOATS;  // L_FLOATS is a multiple of 4: 16-B aligned
    hipLaunchKernelGGL(mlp_pack_kernel, dim3((L_FLOATS + 255) / 256), dim3(256), 0, s, ptrs(w), img);
    return bwd_dw_launch(h0, sh, out, gout, M, img, dw, gh0, partial, s);
}

// the same backward on the image acn_mlp_train_fwd packed into ITS workspace for the same weights (one
// pack per forward + backward pair instead of two); workspace: acn_mlp_dw_workspace_bytes() as above
extern "C" int ACN_MLP_API(acn_mlp_train_bwd_dw_img)(const float* h0, const float* sh, const float* out, const float* gout,
                                        int64_t M, const float* img, float* dw, float* gh0, void* workspace,
                                        void* stream) {
    ACN_REQUIRE(M >= 0 && img && workspace && dw, "acn_mlp_train_bwd_dw_img: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    if (M == 0) {
        const hipError_t e = hipMemsetAsync(dw, 0, (size_t)NDW * sizeof(float), s);
        return e == hipSuccess ? ACN_OK : acn_set_error((int)e, "acn_mlp_train_bwd_dw_img: memset failed");
    }
    ACN_REQUIRE(h0 && sh && out && gout, "acn_mlp_train_bwd_dw_img: NULL pointer");
    return bwd_dw_launch(h0, sh, out, gout, M, img, dw, gh0, (float*)workspace + L_FLOATS, s);
}

// ---------------------------------------------------------------------------------------------
// routed pair lists
constexpr int PAIR_DW_BLOCKS = 256;

extern "C" size_t ACN_MLP_API(acn_mlp_pairs_workspace_bytes)(int K) {
    return ((size_t)K * L_FLOATS + (size_t)PAIR_DW_BLOCKS * K * NDW) * sizeof(float);
}

extern "C" int ACN_MLP_API(acn_mlp_pack_pairs)(const acn_mlp* const* w, int K, void* workspace, void* stream) {
    ACN_REQUIRE(w && workspace && K >= 1 && K <= acn::kMaxK, "acn_mlp_pack_pairs: bad arguments");
    MlpPtrsK pk{};
    for (int k = 0; k < K; ++k) {
        ACN_REQUIRE(w[k], "acn_mlp_pack_pairs: NULL expert %d", k);
        pk.e[k] = ptrs(w[k]);
    }
    hipLaunchKernelGGL(mlp_pack_multi_kernel, dim3((L_FLOATS + 255) / 256, K), dim3(256), 0, (hipStream_t)stream, pk,
                       (float*)workspace);
    return acn_check_launch("acn_mlp_pack_pairs");
}

extern "C" int ACN_MLP_API(acn_mlp_train_fwd_pairs)(const float* h0, const float* sh, const int64_t* seg, int K,
                                       const void* workspace, float* out, void* stream) {
    ACN_REQUIRE(h0 && sh && seg && workspace && out && K >= 1 && K <= acn::kMaxK,
                "acn_mlp_train_fwd_pairs: bad arguments");
    hipLaunchKernelGGL(mlp_fwd_pairs_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, (const float*)workspace, h0,
                       sh, seg, K, out);
    return acn_check_launch("acn_mlp_train_fwd_pairs");
}

extern "C" int ACN_MLP_API(acn_mlp_train_bwd_dw_pairs)(const float* h0, const float* sh, const float* out, const float* gout,
                                          const int64_t* seg, int K, void* workspace, float* dw, float* gh0,
                                          void* stream) {
    ACN_REQUIRE(h0 && sh && out && gout && seg && workspace && dw && K >= 1 && K <= acn::kMaxK,
                "acn_mlp_train_bwd_dw_pairs: bad arguments");
    const float* imgs = (const float*)workspace;
    float* partial = (float*)workspace + (size_t)K * L_FLOATS;
    hipStream_t s = (hipStream_t)stream;
#if ACN_DW_PAIRS_PC
    hipLaunchKernelGGL(mlp_bwd_dw_pairs_pc_kernel, dim3(PAIR_DW_BLOCKS), dim3(512), 0, s, imgs, h0, sh, out, gout, seg, K,
                       gh0, partial);
#else
    hipLaunchKernelGGL(mlp_bwd_dw_pairs_kernel, dim3(PAIR_DW_BLOCKS), dim3(256), 0, s, imgs, h0, sh, out, gout, seg, K,
                       gh0, partial);
#endif
    hipLaunchKernelGGL(mlp_dw_reduce_pairs_kernel, dim3((NDW + 31) / 32, K), dim3(256), 0, s, (const float*)partial,
                       seg, K, PAIR_DW_BLOCKS, dw);
    return acn_check_launch("acn_mlp_train_bwd_dw_pairs");
}
