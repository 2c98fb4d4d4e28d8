// acn_internal.h -- shared host/device definitions of libacnerf (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/acnerf.h"

// ------------------------------------------------------------------------------------------
// error plumbing (capi_common.cpp)
int acn_set_error(int code, const char* fmt, ...);
int acn_check_launch(const char* what);

#define ACN_REQUIRE(cond, ...)                                 \
    do {                                                       \
        if (!(cond)) return acn_set_error(ACN_ERR_ARG, __VA_ARGS__); \
    } while (0)

// ------------------------------------------------------------------------------------------
// Packed per-expert MLP image (floats).  Built on device by acn_pack_kernel from the reference's
// nn.Linear tensors (or fast weights) and staged into LDS by the fused kernels.
//
// MFMA v_mfma_f32_32x32x2_f32: lane l holds A[i=l&31][k=l>>5], B[k=l>>5][j=l&31];
// D[row][col]: col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5) for accumulator register r.
// We compute H^T = W . X^T, i.e. rows = output features, columns = the 32 samples of a tile, so a
// layer's D registers are directly the next layer's B operand (k-step (tile T, reg r) pairs the
// two lane halves' rows rho(r, h) = (r&3)+8(r>>2)+4h+32T).  A is read from LDS as float4 groups
// of 4 consecutive k-steps: [tile][kstep/4][lane][4], one conflict-free ds_read_b128 per lane.
namespace acn {

constexpr int kHashFeat = 32;   // L*F of the fused path (L=16, F=2)
constexpr int kHidden = 64;
constexpr int kGeo = 15;
constexpr int kSH = 16;

constexpr int PK_W1 = 0;                    // sigma_trunk.0: 2 tiles x 16 ksteps x 64
constexpr int PK_W2 = PK_W1 + 2 * 16 * 64;  // sigma_trunk.1: 2 tiles x 32 ksteps x 64
constexpr int PK_WH = PK_W2 + 2 * 32 * 64;  // [sigma_head; geo_head; 0]: 1 tile x 32 ksteps x 64
constexpr int PK_WC1 = PK_WH + 1 * 32 * 64; // color_mlp.0 on [sraw*0, geo, sh]: 2 x 16 x 64
constexpr int PK_WC2 = PK_WC1 + 2 * 16 * 64;// color_mlp.1: 2 x 32 x 64
constexpr int PK_WC3 = PK_WC2 + 2 * 32 * 64;// color_mlp.2 (VALU): [h][c][32]
constexpr int PK_B = PK_WC3 + 2 * 3 * 32;   // bias fragments: 9 tiles x [h][16]
constexpr int PK_BC3 = PK_B + 9 * 32;       // color_mlp.2 bias (3) + pad
constexpr int PK_FLOATS = ((PK_BC3 + 4 + 63) / 64) * 64;
constexpr int PK_BYTES = PK_FLOATS * 4;
// bias tile indices
constexpr int BT_L1 = 0, BT_L2 = 2, BT_H = 4, BT_C1 = 5, BT_C2 = 7;

// per-expert runtime metadata passed by value in kernel arguments
struct ExpertMeta {
    const float* table;
    float amin[3];
    float ext[3];
    float rext[3];   // 1 / ext (host)
    int32_t res[16];
};

constexpr int kMaxK = ACN_MAX_EXPERTS;

struct FieldCfg {
    ExpertMeta ex[kMaxK];
    int32_t K;              // experts evaluated (1 when active_module is set)
    int32_t log2T;
    int32_t routing;        // 0: single expert (ex[0], weight 1), 1: soft, 2: hard
    int32_t cluster_2d;
    float bm;
    float cent[kMaxK][3];
};

}  // namespace acn
