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

// LDS weight image: row-major, stride = cols + 1 (odd): W0 64x32, W1 64x64, Whead 16x64 (geo rows 0..14,
// sigma row 15), Wc0 64x31 (col 31 = 0), Wc1 64x64, Wc2 3x64, then the biases
constexpr int L_W0 = 0, L_W1 = L_W0 + 64 * 33, L_WH = L_W1 + 64 * 65, L_WC0 = L_WH + 16 * 65, L_WC1 = L_WC0 + 64 * 33,
              L_WC2 = L_WC1 + 64 * 65, L_B0 = L_WC2 + 3 * 65, L_B1 = L_B0 + 64, L_BH = L_B1 + 64, L_BC0 = L_BH + 16,
              L_BC1 = L_BC0 + 64, L_BC2 = L_BC1 + 64, L_FLOATS = (L_BC2 + 4 + 3) / 4 * 4;

struct MlpPtrs {
    const float *w0, *b0, *w1, *b1, *wsh, *bsh, *wg, *bg, *wc0, *bc0, *wc1, *bc1, *wc2, *bc2;
};

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int rho(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ int64_t fm_index(int64_t m, int nfeat, int f) {
    return (m / GS) * ((int64_t)nfeat * GS) + (int64_t)f * GS + (m % GS);
}

// the padded LDS image, built once per call (one element per thread), then copied by every block of
// the MLP kernels with 16-B loads
__global__ void __launch_bounds__(256) mlp_pack_kernel(MlpPtrs p, float* __restrict__ img) {
    {
        const int e = blockIdx.x * 256 + threadIdx.x;
        if (e >= L_FLOATS) return;
        float v = 0.0f;
        if (e < L_W1) { const int r = e / 33, c = e % 33; v = c < 32 ? p.w0[r * 32 + c] : 0.0f; }
        else if (e < L_WH) { const int q = e - L_W1, r = q / 65, c = q % 65; v = c < 64 ? p.w1[r * 64 + c] : 0.0f; }
        else if (e < L_WC0) {
            const int q = e - L_WH, r = q / 65, c = q % 65;
            v = c < 64 ? (r < 15 ? p.wg[r * 64 + c] : p.wsh[c]) : 0.0f;
        }
        else if (e < L_WC1) { const int q = e - L_WC0, r = q / 33, c = q % 33; v = c < 31 ? p.wc0[r * 31 + c] : 0.0f; }
        else if (e < L_WC2) { const int q = e - L_WC1, r = q / 65, c = q % 65; v = c < 64 ? p.wc1[r * 64 + c] : 0.0f; }
        else if (e < L_B0) { const int q = e - L_WC2, r = q / 65, c = q % 65; v = c < 64 ? p.wc2[r * 64 + c] : 0.0f; }
        else if (e < L_B1) v = p.b0[e - L_B0];
        else if (e < L_BH) v = p.b1[e - L_B1];
        else if (e < L_BC0) { const int q = e - L_BH; v = q < 15 ? p.bg[q] : p.bsh[0]; }
        else if (e < L_BC1) v = p.bc0[e - L_BC0];
        else if (e < L_BC2) v = p.bc1[e - L_BC1];
        else { const int q = e - L_BC2; v = q < 3 ? p.bc2[q] : 0.0f; }
        img[e] = v;
    }
}

__device__ __forceinline__ void stage_weights(const float* __restrict__ img, float* s) {
    const float4* src = reinterpret_cast<const float4*>(img);
    float4* dst = reinterpret_cast<float4*>(s);
    for (int e = threadIdx.x; e < L_FLOATS / 4; e += blockDim.x) dst[e] = src[e];
}

// Y[to] (rows 32to..) = b + W . X  (W rows < nrow, ld = stride; X: KT input tiles)
template <int NT, int KT>
__device__ __forceinline__ void fwd_layer(const float* W, int ld, int nrow, const float* b, const f32x16 (&X)[KT],
                                          f32x16 (&Y)[NT], int lane) {
    const int i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int to = 0; to < NT; ++to) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 32 * to + rho(r, h);
            Y[to][r] = row < nrow ? b[row] : 0.0f;
        }
        const int wrow = 32 * to + i;
        const float* wr = W + (wrow < nrow ? wrow : 0) * ld;
        const bool live = wrow < nrow;
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) Y[to] = mfma32(live ? wr[32 * t + rho(r, h)] : 0.0f, X[t][r], Y[to]);
    }
}

// dX[ti] (input features 32ti..) = W^T . dY  (W rows = output features < nrow)
template <int NT, int KT>
__device__ __forceinline__ void bwd_layer(const float* W, int ld, int nrow, const f32x16 (&dY)[KT], f32x16 (&dX)[NT],
                                          int lane) {
    const int i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
        dX[ti] = 0.0f;
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int orow = 32 * t + rho(r, h);
                dX[ti] = mfma32(orow < nrow ? W[orow * ld + 32 * ti + i] : 0.0f, dY[t][r], dX[ti]);
            }
    }
}

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
            if (f < nfeat) dst[fm_index(m, nall, off + f)] = X[t][r];
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
                                             int lane, f32x16 (&A1)[2], f32x16 (&A2)[2], f32x16 (&Hd)[1],
                                             f32x16 (&Cin)[1], f32x16 (&C1)[2], f32x16 (&C2)[2], f32x16 (&Rg)[1]) {
    const int h = lane >> 5;
    f32x16 X0[1];
    load_tiles<1>(h0, 32, 0, 32, m, ok, h, X0);
    fwd_layer<2, 1>(Wl + L_W0, 33, 64, Wl + L_B0, X0, A1, lane);
    relu<2>(A1);
    fwd_layer<2, 2>(Wl + L_W1, 65, 64, Wl + L_B1, A1, A2, lane);
    relu<2>(A2);
    fwd_layer<1, 2>(Wl + L_WH, 65, 16, Wl + L_BH, A2, Hd, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int f = rho(r, h);
        Cin[0][r] = f < 15 ? Hd[0][r] : ((ok && f < 31) ? sh[m * 16 + (f - 15)] : 0.0f);
    }
    fwd_layer<2, 1>(Wl + L_WC0, 33, 64, Wl + L_BC0, Cin, C1, lane);
    relu<2>(C1);
    fwd_layer<2, 2>(Wl + L_WC1, 65, 64, Wl + L_BC1, C1, C2, lane);
    relu<2>(C2);
    fwd_layer<1, 2>(Wl + L_WC2, 65, 3, Wl + L_BC2, C2, Rg, lane);
}

__global__ void __launch_bounds__(256) mlp_fwd_kernel(const float* __restrict__ img, const float* __restrict__ h0,
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
        f32x16 A1[2], A2[2], Hd[1], Cin[1], C1[2], C2[2], Rg[1];
        tile_forward(Wl, h0, sh, m, ok, lane, A1, A2, Hd, Cin, C1, C2, Rg);
        if (ok) {
            if (h == 0) {
#pragma unroll
                for (int c = 0; c < 3; ++c) out[m * 4 + c] = acn::sigmoidf_(Rg[0][c]);
            } else {
                out[m * 4 + 3] = acn::trunc_exp(Hd[0][7]);  // row 15 = sigma head (lane half 1, reg 7)
            }
            if (save) {
                // layer inputs (+ ones columns for the bias gradient), feature-major
#pragma unroll
                for (int r = 0; r < 16; ++r) save[fm_index(m, SS, O_H0 + rho(r, h))] = h0[m * 32 + rho(r, h)];
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
                    dRg[0][c] = (gout[m * 4 + c] * (1.0f - y)) * y;
                }
            } else {
                dsig = gout[m * 4 + 3] * out[m * 4 + 3];
            }
        }
        store_fm<1>(gsave, DS, G_RGB, 3, m, ok, h, dRg);
        f32x16 G2[2], G1[2], Gc[1], mask[2];
        bwd_layer<2, 1>(Wl + L_WC2, 65, 3, dRg, G2, lane);
        load_fm<2>(save, SS, O_C2, 64, m, ok, h, mask);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) G2[t][r] = mask[t][r] > 0.0f ? G2[t][r] : 0.0f;
        store_fm<2>(gsave, DS, G_C2, 64, m, ok, h, G2);
        bwd_layer<2, 2>(Wl + L_WC1, 65, 64, G2, G1, lane);
        load_fm<2>(save, SS, O_C1, 64, m, ok, h, mask);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) G1[t][r] = mask[t][r] > 0.0f ? G1[t][r] : 0.0f;
        store_fm<2>(gsave, DS, G_C1, 64, m, ok, h, G1);
        bwd_layer<1, 2>(Wl + L_WC0, 33, 64, G1, Gc, lane);  // d cin: rows 0..14 = d geo (SH rows dropped)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, h);
            dHd[0][r] = f < 15 ? Gc[0][r] : (f == 15 ? dsig : 0.0f);
        }
        store_fm<1>(gsave, DS, G_HD, 16, m, ok, h, dHd);
        f32x16 GA2[2], GA1[2], GH[1];
        bwd_layer<2, 1>(Wl + L_WH, 65, 16, dHd, GA2, lane);
        load_fm<2>(save, SS, O_A2, 64, m, ok, h, mask);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) GA2[t][r] = mask[t][r] > 0.0f ? GA2[t][r] : 0.0f;
        store_fm<2>(gsave, DS, G_A2, 64, m, ok, h, GA2);
        bwd_layer<2, 2>(Wl + L_W1, 65, 64, GA2, GA1, lane);
        load_fm<2>(save, SS, O_A1, 64, m, ok, h, mask);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) GA1[t][r] = mask[t][r] > 0.0f ? GA1[t][r] : 0.0f;
        store_fm<2>(gsave, DS, G_A1, 64, m, ok, h, GA1);
        bwd_layer<1, 2>(Wl + L_W0, 33, 64, GA1, GH, lane);
        if (gh0) store_tiles<1>(gh0, 32, 0, 32, m, ok, h, GH);
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

extern "C" size_t acn_mlp_workspace_bytes(void) { return (size_t)L_FLOATS * sizeof(float); }

extern "C" int acn_mlp_train_fwd(const float* h0, const float* sh, int64_t M, const acn_mlp* w, float* out,
                                 float* save, void* workspace, void* stream) {
    ACN_REQUIRE(M >= 0 && w && workspace, "acn_mlp_train_fwd: bad arguments");
    if (M == 0) return ACN_OK;
    ACN_REQUIRE(h0 && sh && out, "acn_mlp_train_fwd: NULL pointer");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(mlp_pack_kernel, dim3((L_FLOATS + 255) / 256), dim3(256), 0, s, ptrs(w), (float*)workspace);
    hipLaunchKernelGGL(mlp_fwd_kernel, dim3(grid_for(M)), dim3(256), 0, s, (const float*)workspace, h0, sh, M, out,
                       save);
    return acn_check_launch("acn_mlp_train_fwd");
}

extern "C" int acn_mlp_train_bwd(const float* save, const float* out, const float* gout, int64_t M, const acn_mlp* w,
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
