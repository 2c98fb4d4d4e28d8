/*
 * acnerf.h -- C ABI of libacnerf.so, the MI355X (gfx950) volumetric ray renderer for the
 * psklavos1/adaptive-city-nerf stratified render hot path.
 *
 * Every entry point takes plain device pointers + sizes + a hipStream_t (as void*), launches
 * hand-written CDNA4 kernels on that stream and returns an int status: 0 = ok, > 0 = hipError_t,
 * < 0 = argument / unsupported-configuration error.  No C++ exception crosses the ABI; the
 * message of the last failure on the calling thread is available from acn_last_error().
 *
 * Ownership: the caller owns every buffer (inputs, outputs and the workspace); the library
 * never allocates or frees device memory and keeps no pointer past the call.  Functions are
 * stateless and reentrant (the reference's viewer renders from a callback thread while an
 * adaptation thread runs: viewer/viewer.py:712-848, viewer/engine/controller.py:220).
 *
 * Each function names the reference interface it replaces (file:line under the reference repo).
 */
#ifndef ACNERF_H
#define ACNERF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACN_ABI_VERSION 1

#define ACN_OK 0
#define ACN_ERR_ARG (-1)          /* shape / argument error (mirrors the reference's asserts) */
#define ACN_ERR_UNSUPPORTED (-2)  /* configuration the fused kernels do not implement */

#define ACN_MAX_LEVELS 32
#define ACN_MAX_EXPERTS 16

/* interpolation modes of HashGridEncoder (models/encodings.py:158, :340-364) */
#define ACN_INTERP_NEAREST 0
#define ACN_INTERP_LINEAR 1
#define ACN_INTERP_SMOOTHSTEP 2

/* One Instant-NGP expert (MetaNGP, models/inr/meta_ngp.py:15-241).  Pointers are device memory
 * holding the reference's own tensors (state-dict layout, nn.Linear weights (out, in) row-major),
 * or the fast weights of a `params` dict (models/metamodule/metamodule.py:140-156).
 * The fused kernels implement the reference's configured architecture (nerf_runner.py:102-121):
 * L*F = 32 hash features, sigma_trunk 2 x 64 (ReLU), sigma_head 64->1, geo_head 64->15,
 * SH levels 4 (16 comps), color_mlp 31->64->64 (ReLU) ->3, sigmoid rgb.                       */
typedef struct acn_expert {
    const float* table;            /* xyz_encoder.hash_table (L << log2T, F) */
    int32_t L, log2T, F, interp;
    int32_t res[ACN_MAX_LEVELS];   /* xyz_encoder.level_resolutions (host values) */
    float aabb_min[3];             /* scene_box.min               (meta_ngp.py:157) */
    float aabb_extent[3];          /* aabb_extent buffer          (meta_ngp.py:37)  */
    const float *sig_w0, *sig_b0;  /* sigma_trunk.0.linear  (64, 32), (64,) */
    const float *sig_w1, *sig_b1;  /* sigma_trunk.1.linear  (64, 64), (64,) */
    const float *sigh_w, *sigh_b;  /* sigma_head            (1, 64),  (1,)  */
    const float *geo_w, *geo_b;    /* geo_head              (15, 64), (15,) */
    const float *col_w0, *col_b0;  /* color_mlp.0.linear    (64, 31), (64,) */
    const float *col_w1, *col_b1;  /* color_mlp.1.linear    (64, 64), (64,) */
    const float *col_w2, *col_b2;  /* color_mlp.2           (3, 64),  (3,)  */
} acn_expert;

/* MetaContainer routing (models/inr/meta_container.py:97-134): soft inverse-distance weights
 * when boundary_margin > 1, else nearest centroid.                                           */
typedef struct acn_routing {
    int32_t K;                     /* number of experts */
    int32_t cluster_2d;            /* 1: route on (y, z) (coord idx (1, 2)), 0: on (x, y, z) */
    float boundary_margin;         /* bm (>= 1) */
    float centroids[ACN_MAX_EXPERTS][3];
} acn_routing;

/* Background (ray_rendering.py:23-79 _get_bg_rgb / get_bg_default_color, and
 * MetaContainer.background_color meta_container.py:347-382).                                */
#define ACN_BG_NONE 0              /* bg_color_default == "none" */
#define ACN_BG_CONST 1             /* white / black */
#define ACN_BG_MLP 2               /* use_bg_nerf: SH(4) -> Linear(16,H) ReLU -> Linear(H,3) Sigmoid */
typedef struct acn_background {
    int32_t mode;
    int32_t hidden;                /* H (bg_hidden, default 32; <= 64) */
    float color[3];                /* ACN_BG_CONST */
    const float *w1, *b1;          /* bg_mlp.0 (H, 16), (H,) device */
    const float *w2, *b2;          /* bg_mlp.2 (3, H),  (3,) device */
} acn_background;

/* ---------------------------------------------------------------------------------------- */
int acn_version(void);                              /* ACN_ABI_VERSION */
int acn_last_error(char* buf, size_t n);            /* thread-local message of the last failure */

/* HashGridEncoder._torch_forward (models/encodings.py:331-381): x01 (M,3) -> out (M, L*F),
 * level-major / feature-minor.  res: host pointer to L level resolutions.                     */
int acn_hashgrid_fwd(const float* x01, int64_t M, const float* table, const int32_t* res, int L,
                     int log2T, int F, int interp, float* out, void* stream);

/* Backward of the same gathers (autograd of table[idx], encodings.py:324-327): grad_table +=
 * scatter of grad_out (M, L*F).  grad_table must be zero-initialised by the caller.           */
int acn_hashgrid_bwd(const float* x01, int64_t M, const float* grad_out, const int32_t* res,
                     int L, int log2T, int F, int interp, float* grad_table, void* stream);

/* SHEncoder.forward torch fallback (models/encodings.py:133-151, :27-81): d (M,3) unnormalised
 * -> out (M, levels^2), levels in [1, 5].                                                     */
int acn_sh_fwd(const float* d, int64_t M, int levels, float* out, void* stream);

/* Bytes of device workspace the fused field / render entry points need for K experts. */
size_t acn_workspace_bytes(int K);

/* Pack the MLP weights of the experts the next field/render call evaluates (all K, or only
 * experts[active_module] when active_module >= 0) into the workspace, in the MFMA operand order
 * the fused kernels stage into LDS.  Must be re-run whenever any of those weights change (the
 * Python layer re-packs when a tensor's version counter moves or fast weights are passed).    */
int acn_pack_experts(const acn_expert* experts, const acn_routing* routing, int active_module,
                     void* workspace, size_t workspace_bytes, void* stream);

/* MetaContainer.forward / MetaNGP.forward (meta_container.py:275-343, meta_ngp.py:226-241):
 * x (M, ld>=6) rows [xyz, dir, ...] -> out (M, 4) = [rgb, sigma].  active_module >= 0 runs only
 * that expert (no routing), as the reference's `active_module` argument does.  `experts` holds
 * routing->K entries; `workspace` must hold acn_pack_experts() output for the same arguments. */
int acn_field_fwd(const float* x, int64_t M, int64_t ld, const acn_expert* experts,
                  const acn_routing* routing, int active_module, void* workspace,
                  size_t workspace_bytes, float* out, void* stream);

/* volume_render (nerfs/ray_rendering.py:114-165): rgb_sigma (N,S,4), t_vals (N,S), bg (N,3) or
 * NULL -> rgb (N,3), depth (N), weights (N,S) or NULL, acc (N).                              */
int acn_volume_render_fwd(const float* rgb_sigma, const float* t_vals, const float* bg, int64_t N,
                          int S, int raw_rgb, int raw_sigma, float sigma_scale, float* rgb,
                          float* depth, float* weights, float* acc, void* stream);

/* Backward of volume_render (raw_rgb = raw_sigma = 0, the reference's stratified call): given the
 * forward inputs and dL/d(rgb (N,3), depth (N), weights (N,S), acc (N)) -- any of them NULL for zero --
 * writes dL/drgb_sigma (N,S,4) and, if g_bg != NULL, dL/dbg (N,3).  The autograd of
 * ray_rendering.py:137-165 (clamp masks, exp, cumprod, weighted sums); t_vals get no gradient.       */
int acn_volume_render_bwd(const float* rgb_sigma, const float* t_vals, const float* bg, int64_t N, int S,
                          float sigma_scale, const float* g_rgb, const float* g_depth, const float* g_weights,
                          const float* g_acc, float* g_rgb_sigma, float* g_bg, void* stream);

/* Training-path sampler (the differentiable render_rays_stratified's non-differentiable front):
 * stratified_t_vals (ray_rendering.py:262-287; jitter (N,S) uniforms or NULL), points o + d t
 * (:318-320), MetaNGP._world_to_unit (meta_ngp.py:155-158) with HOST aabb_min / aabb_extent (3 floats
 * each) and clamp [lo, hi], and the colour-branch SH-4 of the ray direction (meta_ngp.py:165-168).
 * Outputs t_vals (N,S), x01 (N*S,3), sh (N*S,16); bitwise equal to those torch ops.               */
int acn_sample_stratified(const float* rays, int64_t N, int S, const float* jitter, const float* aabb_min,
                          const float* aabb_extent, float lo, float hi, float* t_vals, float* x01, float* sh,
                          void* stream);

/* Fused render_rays_stratified (ray_rendering.py:290-345 + stratified_t_vals :262-287 +
 * _get_bg_rgb :23-45 + volume_render :114-165) with the field of every expert evaluated in the
 * same kernel.  rays (N,8) [o, d, near, far]; jitter (N,S) uniforms of the training-mode draw
 * (:286) or NULL for eval; tau: early-ray-termination threshold on transmittance (0 = off; the
 * reference has none, the composite error is bounded by 2*tau).  Outputs as volume_render.
 * `workspace` must hold acn_pack_experts() output for the same experts / routing / module.    */
int acn_render_stratified_fwd(const float* rays, int64_t N, int S, const float* jitter,
                              const acn_expert* experts, const acn_routing* routing,
                              int active_module, const acn_background* bg, float sigma_scale,
                              float tau, void* workspace, size_t workspace_bytes, float* rgb,
                              float* depth, float* weights, float* acc, void* stream);

/* Bytes of caller scratch acn_render_stratified_fwd_ordered uses to re-order a batch of N rays
 * (0 when N is outside the re-ordered range 1..8192: the call then renders in the given order). */
size_t acn_render_order_bytes(int64_t N);

/* The visiting order acn_render_stratified_fwd_ordered uses for a batch of 1 <= N <= 8192 rays (the
 * reference renders rays independently, ray_rendering.py:290-345, so only the order of the work
 * changes): order[0..N) is a permutation of 0..N-1 grouping the rays by a Z-ordered 64 x 64 cell of
 * their direction about the batch mean; the sort is stable, so rays of one cell stay in index order
 * and the order is the same on every call.  Exposed for tests and tools.                         */
int acn_ray_order(const float* rays, int64_t N, int32_t* order, void* stream);

/* acn_render_stratified_fwd with a caller-owned scratch of acn_render_order_bytes(N) bytes (NULL /
 * too small = no re-ordering).  Small batches are first sorted by ray direction (Z-order) so that
 * each XCD renders one compact image region and its L2 serves that region's hash cells; every ray
 * is still rendered alone and written at its own index, so the outputs are bit-identical to
 * acn_render_stratified_fwd.  Same reference function (ray_rendering.py:290-345).              */
int acn_render_stratified_fwd_ordered(const float* rays, int64_t N, int S, const float* jitter,
                                      const acn_expert* experts, const acn_routing* routing,
                                      int active_module, const acn_background* bg, float sigma_scale,
                                      float tau, void* workspace, size_t workspace_bytes, float* rgb,
                                      float* depth, float* weights, float* acc, void* order_scratch,
                                      size_t order_bytes, void* stream);

/* get_ray_directions + get_rays + clamp_rays_near_far (nerfs/ray_sampling.py:111-136, :50-108,
 * :139-176) with SceneBox.ray_aabb_intersect (nerfs/scene_box.py:45-107).  c2w: host (3,4)
 * row-major; aabb: host (2,3) or NULL (then near/far constants are used); the override flags
 * reproduce near_far_override=(n|None, f|None); apply_clamp=0 reproduces override None.
 * Writes rays (H*W, 8) and valid (H*W) bytes (valid may be NULL).                             */
int acn_get_rays(int H, int W, float fx, float fy, float cx, float cy, int center_pixels,
                 const float* c2w, const float* aabb, float near_c, float far_c, int has_near_ovr,
                 float near_ovr, int has_far_ovr, float far_ovr, int apply_clamp, float* rays,
                 uint8_t* valid, void* stream);

/* get_ray_directions (ray_sampling.py:111-136): dirs (H*W, 3) unit camera-frame directions. */
int acn_ray_directions(int H, int W, float fx, float fy, float cx, float cy, int center_pixels, float* dirs,
                       void* stream);

/* get_rays (ray_sampling.py:50-108) for given directions (N,3): rays (N,8).  c2w host (3,4);
 * aabb host (2,3) -> SceneBox.ray_aabb_intersect(eps, max_bound, invalid_value), or NULL ->
 * constant near_c / far_c.                                                                   */
int acn_rays_from_dirs(const float* dirs, int64_t N, const float* c2w, const float* aabb, float near_c,
                       float far_c, float eps, float max_bound, float invalid_value, float* rays,
                       void* stream);

/* SceneBox.ray_aabb_intersect (nerfs/scene_box.py:45-107): origins, dirs (N,3) -> tmin, tmax (N). */
int acn_ray_aabb(const float* origins, const float* dirs, int64_t N, const float* aabb, float eps,
                 float max_bound, float invalid_value, float* tmin, float* tmax, void* stream);

/* clamp_rays_near_far (ray_sampling.py:139-176) in place on rays (N,8); apply=0 reproduces
 * near_far_override=None (valid mask only).  valid (N) bytes may be NULL.                     */
int acn_clamp_rays(float* rays, int64_t N, int apply, int has_near_ovr, float near_ovr, int has_far_ovr,
                   float far_ovr, float eps, float invalid_value, uint8_t* valid, void* stream);

/* MetaContainer._routing (meta_container.py:97-134): pts (M, ld>=3) -> soft weights (M, K) when
 * boundary_margin > 1, else hard assignment (M) int32.                                        */
int acn_routing_fwd(const float* pts, int64_t M, int64_t ld, const acn_routing* routing, float* weights,
                    int32_t* hard, void* stream);

/* MetaContainer.background_color (meta_container.py:347-382): dirs (N,3) -> rgb (N,3). */
int acn_background_fwd(const float* dirs, int64_t N, const acn_background* bg, float* out, void* stream);
/* Backward of the MLP background head (the autograd of bg_mlp in MetaContainer.background_color,
 * meta_container.py:347-382) for dL/d(bg rgb) g_out (N,3): writes (overwrites) the gradients of
 * bg_mlp.0.weight (H,16), .0.bias (H), bg_mlp.2.weight (3,H), .2.bias (3).  Deterministic (per-wave sums
 * added in wave order); workspace of acn_background_bwd_workspace_bytes(). */
size_t acn_background_bwd_workspace_bytes(void);
int acn_background_bwd(const float* dirs, int64_t N, const acn_background* bg, const float* g_out, float* g_w1,
                       float* g_b1, float* g_w2, float* g_b2, void* workspace, size_t workspace_bytes, void* stream);

/* The routed adaptation step's compositing, loss and their backward in one launch (replaces, in
 * routed_train.RoutedAdaptStep, acn_routed_blend_fwd + acn_background_fwd + the dirs copy +
 * acn_volume_render_fwd + acn_mse_linear_fwd_ws + acn_mse_linear_bwd + acn_volume_render_bwd +
 * acn_routed_blend_bwd with the same arithmetic).  Reference: the train-mode render_rays +
 * compute_mse_loss + loss.backward() down to the experts' outputs, runtime_adapt.py:286-304,
 * meta_container.py:322-337 (blend), ray_rendering.py:137-165 (compositing), losses.py:10-32 (linear MSE).
 *   rays (N,8), t_vals (N,S); pair_out (P,4) / pair_w (P) / pidx (P) / pmap (N*S,K) the routed pairs of
 *   acn_routed_scatter, live (device int64, may be NULL = P) the live pair count; rgbs (N,3) targets;
 *   g_loss (device float) dL/dloss (1, or the AMP loss scale).
 * Writes rgb (N,3), dirs (N,3) = rays[:,3:6] (for acn_background_bwd), g_bg (N,3) dL/d(background rgb)
 * (may be NULL), g_pair_out (P,4) dL/d(pair outputs) (padding slots below live: 0), loss (device float,
 * deterministic double sum).  pair_out / g_pair_out 16-byte aligned; workspace of
 * acn_composite_mse_train_workspace_bytes(), zeroed once (its counter returns to 0 after each call). */
size_t acn_composite_mse_train_workspace_bytes(void);
int acn_routed_composite_mse_train(const float* rays, int64_t N, int S, const float* t_vals, const float* pair_out,
                                   const float* pair_w, const int32_t* pmap, int K, const int32_t* pidx, int64_t P,
                                   const int64_t* live, const acn_background* bg, const float* rgbs,
                                   const float* g_loss, float* rgb, float* dirs, float* g_bg, float* g_pair_out,
                                   float* loss, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Optimizer step of the online adaptation loop (pipelines/online_stage/runtime_adapt.py:305-309):
 * torch.nn.utils.clip_grad_norm_(params, max_norm) followed by torch.optim.Adam(param_groups)
 * .step() (common/utils.py:57-62), multi-tensor.  The caller keeps, in DEVICE memory, one
 * descriptor per parameter tensor and a chunk -> tensor map: tensor t covers chunks
 * [first_chunk, first_chunk + ceil(numel / ACN_OPTIM_CHUNK)).                                   */
#define ACN_OPTIM_CHUNK 65536
#define ACN_OPTIM_MAX_GROUPS 8
typedef struct acn_param_desc {
    float* param;                  /* the parameter (updated in place) */
    const float* grad;             /* its gradient, or NULL (parameter skipped, as torch does) */
    float* exp_avg;                /* Adam state 'exp_avg'    (same numel) */
    float* exp_avg_sq;             /* Adam state 'exp_avg_sq' (same numel) */
    int64_t numel;
    int32_t group;                 /* index into the acn_adam_group array */
    int32_t first_chunk;
} acn_param_desc;

/* One torch.optim.Adam param group (host memory).  `step` is the value AFTER this step's
 * increment (torch increments state['step'] before the update).                                */
typedef struct acn_adam_group {
    double lr, beta1, beta2, eps, weight_decay;
    int32_t step, pad;
} acn_adam_group;

/* Sum of squared gradients over all described tensors: per-chunk partials (nchunks doubles,
 * caller workspace) then *total (device double).                                               */
int acn_grad_sumsq(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                   double* partials, double* total, void* stream);

/* clip_grad_norm_ coefficient from a (possibly all-reduced) total: out[0] = total_norm (fp32),
 * out[1] = min(1, max_norm / (total_norm + 1e-6)).  Device pointers.                            */
int acn_clip_coef(const double* total_sumsq, float max_norm, float* out, void* stream);

/* Adam update of every described tensor (torch.optim.Adam single-tensor arithmetic), gradients
 * multiplied on the fly by grad_scale[1] (the clip coefficient) when grad_scale != NULL.        */
int acn_adam_step(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                  const acn_adam_group* groups, int ngroups, const float* grad_scale, void* stream);

/* The same update, replayable inside a captured hipGraph: the per-group constants of steps
 * first_step .. first_step + table_steps - 1 are precomputed on the host (acn_adam_table_fill into
 * acn_adam_table_bytes of host memory, then copied to the device by the caller); each call first
 * advances the device step counter *step_dev by one, then updates with the table row of that step
 * (a step outside the table leaves the parameters untouched -- the caller refills in time).      */
/* Descriptors given in host memory (n <= 64) written to device memory together with the chunk ->
 * tensor map by one kernel whose arguments carry them (capturable: no host-to-device copy).     */
int acn_optim_plan_device(const acn_param_desc* host_descs, int n, acn_param_desc* descs, int32_t* chunk_tensor,
                          int64_t nchunks, void* stream);
size_t acn_adam_table_bytes(int ngroups, int steps);
int acn_adam_table_fill(const acn_adam_group* groups, int ngroups, int first_step, int steps, void* out, size_t bytes);
int acn_adam_step_table(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks, const void* table,
                        int ngroups, int32_t* step_dev, int first_step, int table_steps, const float* grad_scale,
                        void* stream);

/* Slotted form for the routed container (graph-replayable, no host synchronisation): tensor t belongs
 * to activity slot flags[t] & 0xffff.  Slot s < K (expert s) is active in a step iff its routed pair
 * count seg[K+1+s] > 0 (acn_routed_count), slots >= K always; an inactive slot is skipped like a
 * torch parameter whose grad is None (no moment decay, no step increment).  step_dev[nslots]: per-slot
 * step counters, advanced on the device for the active slots before the update; table: the per-group
 * constants of steps 1..table_steps (acn_adam_table_fill with first_step 1).  flags bit 16: clear the
 * gradient after reading it.  The norm skips inactive slots likewise.                             */
int acn_grad_sumsq_slots(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                         const int32_t* flags, const int64_t* seg, int K, double* partials, double* total,
                         void* stream);
/* As acn_grad_sumsq_slots, but tensors whose flag has bit 17 set are skipped and *extra (a device double:
 * the table gradients' sum of squares from acn_hashgrid_bwd_pairs_sumsq) is added to the total, then
 * reset to 0 (ready for the next step).  extra may be NULL. */
int acn_grad_sumsq_slots_ex(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                            const int32_t* flags, const int64_t* seg, int K, double* partials, double* total,
                            double* extra, void* stream);
/* acn_grad_sumsq_slots_ex followed by acn_clip_coef(total, max_norm, out) in ONE launch (the last workgroup to
 * finish reduces the partials and writes total, out[0] = norm, out[1] = clip coefficient): bitwise the same
 * results.  counter: a device uint zeroed once (returns to 0 after each call). */
int acn_grad_clip_slots(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                        const int32_t* flags, const int64_t* seg, int K, double* partials, double* total,
                        double* extra, float max_norm, float* out, unsigned int* counter, void* stream);
int acn_adam_step_slots(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                        const int32_t* flags, const void* table, int ngroups, int table_steps, int32_t* step_dev,
                        int nslots, const int64_t* seg, int K, const float* grad_scale, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Occupancy-grid renderer.  The reference delegates this to nerfacc 0.5.3
 * (third-party, not vendored): OccGridEstimator.sampling -> traverse_grids, render_weight_from_density,
 * accumulate_along_rays, pack_info; its own glue is nerfs/ray_rendering.py:170-258, :349-558 and
 * models/inr/meta_ngp.py:242-443.  Packed sample lists are ray-major: ray r owns samples
 * [chunk_starts[r], chunk_starts[r] + chunk_cnts[r]) (nerfacc's packed_info columns).            */

/* OccGridEstimator.sampling's traverse_grids (marching through `levels` nested grids of res[3]
 * cells, aabbs host (levels, 6) [min3, max3]).  bits: the `binaries` buffer as one bit per cell
 * (acn_occ_pack_bits).  near/far (N) device.  prefilter_aabb (host [min3, max3]) or NULL: rays that
 * miss it over [near, far] = prefilter_near_far[i * ld_pf + {0, 1}] (the rays' own columns;
 * ray_rendering.py:170-193 _intersect_rays_aabb) get no samples.
 * offsets == NULL: counts (N) <- samples per ray; with cap > 0 the first cap samples of ray i are also
 *   written to the scratch rows t_starts/t_ends + i * cap (single pass; acn_occ_compact packs them
 *   when every count <= cap).
 * offsets != NULL: ray i writes all its samples at offsets[i] (ray_indices, t_starts, t_ends).      */
int acn_occ_traverse(const float* rays_o, int64_t ld_o, const float* rays_d, int64_t ld_d, int64_t N,
                     const float* near_planes, const float* far_planes, const uint32_t* bits,
                     const float* aabbs, int levels, const int32_t* res, float step_size, float cone_angle,
                     const float* prefilter_aabb, const float* prefilter_near_far, int64_t ld_pf, int64_t cap,
                     int64_t* counts, const int64_t* offsets, int64_t* ray_indices, float* t_starts,
                     float* t_ends, void* stream);

/* Packs the scratch rows of a single-pass acn_occ_traverse (all counts <= cap) at offsets (the
 * exclusive scan of counts): ray_indices, t_starts, t_ends (M).                                 */
int acn_occ_compact(const float* scratch_t0, const float* scratch_t1, int64_t cap, const int64_t* counts,
                    const int64_t* offsets, int64_t N, int64_t* ray_indices, float* t_starts, float* t_ends,
                    void* stream);

/* _merge_segments_union (ray_rendering.py:196-258): per ray, the sorted distinct boundaries of the
 * K experts' segments; consecutive pairs become the merged segments.  starts/counts/t_starts/t_ends
 * are HOST arrays of K device pointers (per expert: (N) chunk starts and counts over the global rays,
 * (M_k) t values).  Two passes as acn_occ_traverse.                                             */
int acn_occ_union(int K, int64_t N, const int64_t* const* starts, const int64_t* const* counts,
                  const float* const* t_starts, const float* const* t_ends, int64_t* out_counts,
                  const int64_t* offsets, int64_t* ray_indices, float* m_starts, float* m_ends, void* stream);

/* Fused occupancy render over packed samples: render_expert_occ (ray_rendering.py:467-558) when
 * active_module >= 0 or K == 1, the container's soft-MoE blend of render_rays_occ (:406-464)
 * otherwise; nerfacc compositing; background as acn_render_stratified_fwd.  rays (N, ld>=6) [o, d].
 * weights (M) or NULL.                                                                        */
int acn_render_packed_fwd(const float* rays, int64_t ld, int64_t N, const int64_t* chunk_starts,
                          const int64_t* chunk_cnts, const float* t_starts, const float* t_ends,
                          const acn_expert* experts, const acn_routing* routing, int active_module,
                          const acn_background* bg, void* workspace, size_t workspace_bytes, float* rgb,
                          float* depth, float* weights, float* acc, void* stream);

/* nerfacc render_weight_from_density over packed samples: weights, trans, alphas (M) (trans / alphas
 * may be NULL).                                                                                */
int acn_packed_weights_fwd(const float* sigmas, const float* t_starts, const float* t_ends,
                           const int64_t* chunk_starts, const int64_t* chunk_cnts, int64_t N,
                           float* weights, float* trans, float* alphas, void* stream);

/* Backward of acn_packed_weights_fwd w.r.t. sigmas given dL/d(weights, trans, alphas) (any NULL). */
int acn_packed_weights_bwd(const float* sigmas, const float* t_starts, const float* t_ends,
                           const float* weights, const float* trans, const float* alphas,
                           const float* g_weights, const float* g_trans, const float* g_alphas,
                           const int64_t* chunk_starts, const int64_t* chunk_cnts, int64_t N,
                           float* g_sigmas, void* stream);

/* nerfacc accumulate_along_rays: out (N, C) = per-ray sum of weights * values (values (M, C) or
 * NULL for C = 1 and values = 1).  Deterministic segmented sums.                                */
int acn_packed_accumulate_fwd(const float* weights, const float* values, int C, const int64_t* chunk_starts,
                              const int64_t* chunk_cnts, int64_t N, float* out, void* stream);

/* Backward of acn_packed_accumulate_fwd given dL/dout (N, C): g_weights (M), g_values (M, C) (either NULL). */
int acn_packed_accumulate_bwd(const float* weights, const float* values, int C, const int64_t* ray_indices,
                              int64_t M, const float* g_out, float* g_weights, float* g_values, void* stream);

/* OccGridEstimator maintenance.  acn_occ_pack_bits: binaries (n bytes, the bool buffer) -> one bit
 * per cell (ceil(n/32) words).  acn_occ_cell_points: jittered cell positions of one level
 * (nerfacc _update: aabb_min + (coords + u) / res * extent); u (n, 3) device or NULL, aabb / res
 * host.  acn_occ_ema: occs[c] = max(occs[c] * decay, occ).  acn_occ_binarize: thre =
 * min(mean(occs[occs >= 0]), occ_thre); binaries = occs > thre (+ bits, thre_out optional), all on
 * device, workspace of acn_occ_binarize_workspace_bytes().  acn_occ_mark_invisible
 * (mark_invisible_cells): Ks (nK, 3, 3), c2w (nc2w, 3, 4) device; occs_level[c] = 0 if some camera
 * sees cell c (coords / (res - 1) in the level box) in front of near_plane, else -1.            */
int acn_occ_pack_bits(const uint8_t* binaries, int64_t n, uint32_t* bits, void* stream);
int acn_occ_cell_points(const int64_t* cell_indices, int64_t n, const float* u, const float* aabb,
                        const int32_t* res, float* x, void* stream);
int acn_occ_ema(float* occs, const int64_t* cell_ids, const float* occ, int64_t n, float decay, void* stream);
size_t acn_occ_binarize_workspace_bytes(void);
int acn_occ_binarize(const float* occs, int64_t n, float occ_thre, uint8_t* binaries, uint32_t* bits,
                     float* thre_out, void* workspace, void* stream);
int acn_occ_mark_invisible(const float* Ks, int nK, const float* c2w, int nc2w, int width, int height,
                           float near_plane, const float* aabb, const int32_t* res,
                           const int64_t* cell_indices, int64_t n, float* occs_level, void* stream);

/* ---------------------------------------------------------------------------------------------
 * The expert MLP of the training path (mlp_train.hip).  Replaces the differentiable MetaLinear chain
 * of MetaNGP.density / color (models/inr/meta_ngp.py:171-241) and its autograd backward for the
 * reference configuration (hash features 32 -> 64 -> 64 ReLU -> geo 15 + sigma 1; [geo, SH 16] ->
 * 64 -> 64 ReLU -> 3 sigmoid).  Pointers: device weights in the reference's nn.Linear layout (out, in)
 * -- module parameters or fast weights.                                                          */
typedef struct acn_mlp {
    const float *w0, *b0;          /* sigma_trunk.0.linear (64, 32), (64) */
    const float *w1, *b1;          /* sigma_trunk.1.linear (64, 64), (64) */
    const float *wsh, *bsh;        /* sigma_head (1, 64), (1)             */
    const float *wg, *bg;          /* geo_head (15, 64), (15)             */
    const float *wc0, *bc0;        /* color_mlp.0.linear (64, 31), (64)   */
    const float *wc1, *bc1;        /* color_mlp.1.linear (64, 64), (64)   */
    const float *wc2, *bc2;        /* color_mlp.2 (3, 64), (3)            */
} acn_mlp;

/* h0 (M, 32) hash features, sh (M, 16) SH of the directions -> out (M, 4) = [sigmoid(rgb), trunc_exp(
 * sigma)]; save or NULL: the layer inputs with ones columns, features [h0|1][a1|1][a2|1][cin|1][c1|1]
 * [c2|1] (widths 33, 65, 65, 32, 65, 65 = 325), stored feature-major per group of 2048 samples:
 * (ceil(M / 2048), 325, 2048), samples past M zero (caller-initialised).  workspace:
 * acn_mlp_workspace_bytes() device bytes (the padded weight image).                              */
size_t acn_mlp_workspace_bytes(void);
int acn_mlp_train_fwd(const float* h0, const float* sh, int64_t M, const acn_mlp* w, float* out, float* save,
                      void* workspace, void* stream);
/* Backward from dL/dout (M, 4): gsave (ceil(M / 2048), 275, 2048) = per-layer output gradients [da1 64]
 * [da2 64][dhead 16: geo 0..14, sigma 15][dc1 64][dc2 64][drgb 3] (after the ReLU / trunc_exp / sigmoid
 * derivatives; samples past M zero, caller-initialised), and gh0 (M, 32) = dL/dh0 (NULL: skipped).
 * [dW | db] of a layer = sum over groups of gsave_block . save_block^T.                          */
int acn_mlp_train_bwd(const float* save, const float* out, const float* gout, int64_t M, const acn_mlp* w,
                      float* gsave, float* gh0, void* workspace, void* stream);
/* Fused backward with the weight gradients (no saved activations): re-runs the forward from h0 / sh,
 * back-propagates dL/dout (M, 4) (out = the forward's output) and writes
 *   dw (13715 floats) = the 14 gradients concatenated in acn_mlp order, each in the nn.Linear layout:
 *     w0 64x32 @0, b0 @2048, w1 64x64 @2112, b1 @6208, wsh 1x64 @6272, bsh @6336, wg 15x64 @6337,
 *     bg @7297, wc0 64x31 @7312, bc0 @9296, wc1 64x64 @9360, bc1 @13456, wc2 3x64 @13520, bc2 @13712;
 *   gh0 (M, 32) = dL/dh0 (NULL: skipped).
 * Replaces the autograd backward of the MetaLinear chain incl. its weight-gradient GEMMs
 * (torch.autograd over models/inr/meta_ngp.py:171-241).  Sums run in a different order than torch's
 * (fp32 MFMA + workgroup partials); not bitwise reproducible run to run (LDS float atomics).
 * workspace: acn_mlp_dw_workspace_bytes() device bytes.                                           */
size_t acn_mlp_dw_workspace_bytes(void);
int acn_mlp_train_bwd_dw(const float* h0, const float* sh, const float* out, const float* gout, int64_t M,
                         const acn_mlp* w, float* dw, float* gh0, void* workspace, void* stream);
/* acn_mlp_train_bwd_dw on a packed weight image instead of acn_mlp pointers: img = the workspace of the
 * acn_mlp_train_fwd call for the same weights (that call packs them there; reusing it saves the backward's
 * own pack launch).  The weights must not have changed since that forward.                          */
int acn_mlp_train_bwd_dw_img(const float* h0, const float* sh, const float* out, const float* gout, int64_t M,
                             const float* img, float* dw, float* gh0, void* workspace, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Episodic task routing (data.hip).  Replaces TaskDataset's region clip + micro-cell assignment
 * (data/task_dataset.py:130-172 _aabb_intersect/_region_segment, :229-352 DDA max overlap,
 * :354-418 alpha point + 6-neighbour max overlap, :544-598 selected-cell overlap >= tolerance).
 * rays (N, 8) device; region_aabb[6], cells[3] (nx, ny, nz) host; cell_bounds (C, 2, 3) and
 * tol_cell (C) device (C = nx*ny*nz, x-major); alpha = assignment_checkpoint; tol_abs =
 * max(1e-6 * median cell diagonal, 1e-9); policy 0 alpha / 1 dda (max_steps DDA steps).
 * Out: cell_ids (N) int64 (-1 when the ray misses the region segment), flags (N) u8: bit0 the ray
 * has a positive segment in the region, bit1 its overlap with the selected cell passes tol_cell.  */
int acn_route_rays(const float* rays, int64_t N, const float* region_aabb, const int32_t* cells,
                   const float* cell_bounds, const float* tol_cell, float alpha, float tol_abs, int policy,
                   int max_steps, int64_t* cell_ids, uint8_t* flags, void* stream);

/* Per-cell ray lists of _route_and_bin (data/task_dataset.py:575-628: sort the region-valid rays by
 * cell, keep relative order, drop rays failing the keep tolerance): a stable counting sort of the
 * rays with flags bit1 set by cell_ids.  ray_index (>= kept rays) int32 device receives the ray
 * indices cell after cell, ascending inside a cell; counts (n_cells + 1) int64 device receives
 * the kept rays per cell and, last, the number of region-valid rays (flags bit0).  N < 2^31,
 * n_cells <= 4096; workspace of acn_bin_rays_workspace_bytes(N, n_cells) device bytes.          */
size_t acn_bin_rays_workspace_bytes(int64_t N, int n_cells);
int acn_bin_rays(const int64_t* cell_ids, const uint8_t* flags, int64_t N, int n_cells, int32_t* ray_index,
                 int64_t* counts, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Cluster creation (clusters.hip).  Replaces scripts/create_clusters.py's per-image routing:
 * compute_voronoi_opt (:386-556) and, with orig != 0, compute_voronoi_orig (:559-634).
 * rays (N, 8) device (16-B aligned); centroids (C, 3) host, C <= 63; routing in YZ when cluster_2d.
 * bits (N) uint64 device: bit c = ray belongs to centroid c (ray_samples samples on
 * lerp(near, far, linspace(0, 1, S)); strict argmin when boundary_margin == 1, else
 * d2 <= margin^2 * min d2; orig: min over samples of dist / (nearest + 1e-8) <= margin).
 * update_aabbs (ignored with orig, as the reference): mins / maxs (C, 3) device lowered / raised in
 * place by the assigned samples, counts (C) int64 += assigned samples, nan_flag (C) int32 set when
 * an assigned sample is NaN.                                                                     */
int acn_voronoi_route(const float* rays, int64_t N, int ray_samples, const float* centroids, int n_centroids,
                      int cluster_2d, double boundary_margin, int orig, int update_aabbs, uint64_t* bits,
                      float* mins, float* maxs, int64_t* counts, int32_t* nan_flag, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Routed container, differentiable path (routed.hip).  Replaces the expert dispatch of
 * MetaContainer.forward under autograd (models/inr/meta_container.py:97-134 _routing, :300-343
 * nonzero -> index_select -> expert -> index_add_) and the sample front end of
 * render_rays_stratified (nerfs/ray_rendering.py:262-320) for M = N*S samples:
 *   acn_routed_count   -> t_vals (N,S) (jitter (N,S) uniforms or NULL), and seg[2K+1] (int64, device):
 *                         expert k's (sample, expert) pairs occupy [seg[k], seg[k] + seg[K+1+k]) and its
 *                         segment [seg[k], seg[k+1]) is padded to a multiple of `align` (seg[K] = total
 *                         slots).  workspace: acn_routed_workspace_bytes(M, K) device bytes (kept for
 *                         the scatter).
 *   acn_routed_scatter -> per pair: pidx (sample index), pw (routing weight), x01 (3, expert k's unit
 *                         box clamped to [lo, hi], _world_to_unit meta_ngp.py:155-158), sh (16, SH-4 of
 *                         the ray direction, meta_ngp.py:165-168); pmap (M,K) pair index or -1; pk
 *                         (optional) the expert of every slot.  Padding slots: pidx -1, pw 0, x01 0.5,
 *                         sh 0.  Buffers must hold seg[K] slots (M*K + K*align always suffices).
 *                         aabb_min / aabb_extent: HOST (K,3) floats.  Pairs of expert k are in sample
 *                         order (= index_select(nonzero(w[:, k] > 0))).
 *   acn_routed_blend_fwd -> out (M,4) = sum_k y[p_k] * w[p_k] in expert order from zero (index_add_)
 *   acn_routed_blend_bwd -> gy (P,4) = g[pidx] * pw  (backward of the weighted index_add_; 0 on padding);
 *                         live (device, nullable): slots at or past *live (e.g. seg + K) are not touched */
size_t acn_routed_workspace_bytes(int64_t M, int K);
int acn_routed_count(const float* rays, int64_t N, int S, const float* jitter, const acn_routing* routing, int align,
                     float* t_vals, int64_t* seg, void* workspace, size_t workspace_bytes, void* stream);
int acn_routed_scatter(const float* rays, int64_t N, int S, int K, const float* t_vals, const int64_t* seg,
                       const float* aabb_min, const float* aabb_extent, float lo, float hi, int align,
                       const void* workspace, int32_t* pidx, float* pw, float* x01, float* sh, int32_t* pmap,
                       int32_t* pk, void* stream);
int acn_routed_blend_fwd(const float* y, const float* pw, const int32_t* pmap, int64_t M, int K, float* out,
                         void* stream);
int acn_routed_blend_bwd(const float* g, const int32_t* pidx, const float* pw, int64_t P, const int64_t* live,
                         float* gy, void* stream);

/* Deterministic HashGridEncoder backward: records (row, corner gradient) in (point, level,
 * corner) order, a stable radix sort by row, one sequential fp32 sum per row -- every row is the sum of
 * its contributions in point order, as a serial CPU scatter-add (encodings.py:318-329); bitwise
 * reproducible.  F = 2.  grad_table is accumulated into (zero it first).  workspace:
 * acn_hashgrid_bwd_det_workspace_bytes(M, L, log2T, interp) device bytes.                          */
size_t acn_hashgrid_bwd_det_workspace_bytes(int64_t M, int L, int log2T, int interp);
int acn_hashgrid_bwd_det(const float* x01, int64_t M, const float* grad_out, const int32_t* res, int L, int log2T,
                         int F, int interp, float* grad_table, void* workspace, size_t workspace_bytes, void* stream);

/* Expert-parallel records (parallel.py, SURVEY §8(e) "one expert per GPU"):
 *   acn_routed_scatter_xd -> the pairs of acn_routed_count (align 1) as xd (P,6) = [world point o + d t,
 *                            ray direction], with pidx / pw / pmap / pk as acn_routed_scatter: the 24-B
 *                            record sent to the GPU owning the pair's expert.
 *   acn_xd_unit_sh        -> owner side: x01 (P,3) in the expert's unit box (HOST aabb_min / extent,
 *                            clamped to [lo, hi]) and SH-4 (P,16) of the direction, as acn_routed_scatter. */
int acn_routed_scatter_xd(const float* rays, int64_t N, int S, int K, const float* t_vals, const int64_t* seg,
                          const void* workspace, int32_t* pidx, float* pw, float* xd, int32_t* pmap, int32_t* pk,
                          void* stream);
int acn_xd_unit_sh(const float* xd, int64_t P, const float* aabb_min, const float* aabb_extent, float lo, float hi,
                   float* x01, float* sh, void* stream);

/* Sync-free expert-parallel exchange (expert_parallel.ExpertParallelAdaptStep, SURVEY §8(e) C5 with one
 * expert block per GPU; replaces the per-expert nonzero / index_select dispatch of meta_container.py:300-337
 * across ranks).  Every buffer has a host-known fixed capacity, so the all-to-alls use constant split
 * sizes and nothing is read back to the host:
 *   acn_routed_count_fixed -> as acn_routed_count, but expert k's segment is [k cap, (k+1) cap); seg[K+1+k] =
 *                             live count.  cap >= N*S never overflows; a smaller cap (an exchange sized to the
 *                             live records) keeps the first cap pairs of an expert in sample order, the scatter
 *                             drops the rest (pmap -1) and seg[K+1+k] > cap tells the caller to redo the batch
 *                             with a larger cap.  With experts numbered by owner (contiguous blocks) the pair
 *                             buffer IS the send buffer of the all-to-all.  Consumers clamp counts to cap.
 *   acn_routed_pad_pairs   -> pidx -1, pw 0 on every segment's slots past its live count (max_pad: a bound
 *                             on one segment's padding, e.g. cap).
 *   acn_ep_gather          -> owner side: records received as [src][local expert j][cap] (W x E x cap xd
 *                             records, live counts recv_cnt (W, E) int64, device) -> compact pair slots per
 *                             local expert in (src, index) order, segments padded to `align`: seg[2E+1]
 *                             (device), x01 (HOST aabb_min / extent (E,3), clamped to [lo, hi]), SH-4, pk (local
 *                             expert), pflag (0 pair / -1 padding, the pidx of the pair kernels), back (index
 *                             into the received layout or -1).  Slot buffers hold W*E*cap + E*align slots.
 *                             workspace: acn_ep_workspace_bytes(W, E).
 *   acn_ep_scatter_back    -> ret[back[p]] = out[p] (float4 per slot): field outputs to the received layout
 *   acn_ep_gather_grad     -> gout[p] = gy[back[p]] (0 on padding): the senders' dL/d(rgb, sigma) to the slots */
int acn_routed_count_fixed(const float* rays, int64_t N, int S, const float* jitter, const acn_routing* routing,
                           int64_t cap, float* t_vals, int64_t* seg, void* workspace, size_t workspace_bytes,
                           void* stream);
int acn_routed_pad_pairs(const int64_t* seg, int K, int64_t max_pad, int32_t* pidx, float* pw, void* stream);
/* Per-expert capacities (HOST arrays): acn_routed_count_caps lays expert k's pairs at [sum_{j<k} caps[j], + caps[k]);
 * acn_ep_gather_caps reads sender s's records of local expert j at s * sum(caps) + sum_{i<j} caps[i].  The
 * uniform-capacity forms above are these with every capacity equal (an exchange sized per expert to the
 * live records: expert_parallel.ExpertParallelAdaptStep(capacity="adaptive")).  A capacity may be 0 (the
 * planned exchange: capacities = the counts of acn_routed_count_batches, so the layout is compact).          */
int acn_routed_count_caps(const float* rays, int64_t N, int S, const float* jitter, const acn_routing* routing,
                          const int64_t* caps, float* t_vals, int64_t* seg, void* workspace, size_t workspace_bytes,
                          void* stream);
/* Depth-tiled pair order (the expert-parallel render, expert_parallel.ExpertParallelRenderer(tile_rays=...)): as
 * acn_routed_count_caps / acn_routed_scatter_xd, with every expert's pairs laid out in depth-tile order instead of
 * sample order -- blocks of tile_rays consecutive rays (the last one shorter), a block's rays at sample s before its
 * rays at s + 1.  The same pairs, counts and segments, pmap / pidx pointing at the new positions; tile_rays 0 IS
 * the sample order of the forms above.  The owner evaluates records in arrival order, so a wave holds neighbouring
 * rays at one depth (the busiest C4 owner rank 29.7 -> 15.5 ms).  Both calls of a batch must use the
 * same tile_rays.  No reference counterpart (the order is the sender's free choice: results go back by position). */
int acn_routed_count_caps_tiled(const float* rays, int64_t N, int S, const float* jitter, const acn_routing* routing,
                                const int64_t* caps, int tile_rays, float* t_vals, int64_t* seg, void* workspace,
                                size_t workspace_bytes, void* stream);
int acn_routed_scatter_xd_tiled(const float* rays, int64_t N, int S, int K, int tile_rays, const float* t_vals,
                                const int64_t* seg, const void* workspace, int32_t* pidx, float* pw, float* xd,
                                int32_t* pmap, int32_t* pk, void* stream);
int acn_ep_gather_caps(const float* recv_xd, const int64_t* recv_cnt, int W, int E, const int64_t* caps, int align,
                       const float* aabb_min, const float* aabb_extent, float lo, float hi, int64_t* seg,
                       void* workspace, float* x01, float* sh, int32_t* pk, int32_t* pflag, int64_t* back,
                       void* stream);
size_t acn_ep_workspace_bytes(int W, int E);
int acn_ep_gather(const float* recv_xd, const int64_t* recv_cnt, int W, int E, int64_t cap, int align,
                  const float* aabb_min, const float* aabb_extent, float lo, float hi, int64_t* seg, void* workspace,
                  float* x01, float* sh, int32_t* pk, int32_t* pflag, int64_t* back, void* stream);
int acn_ep_scatter_back(const float* out, const int64_t* back, const int64_t* seg, int E, float* ret, void* stream);
int acn_ep_gather_grad(const float* gy, const int64_t* back, const int64_t* seg, int E, float* gout, void* stream);

/* One expert per GPU, render (expert_parallel.ExpertParallelRenderer): the fused routed render split at its
 * expert boundary (render_rays_stratified ray_rendering.py:290-345 with MetaContainer.forward's per-expert
 * loop meta_container.py:300-337 distributed over the ranks).
 *   acn_ep_field_fwd -> owner: the field of its E experts (`experts`, packed by acn_pack_experts with a routing
 *                       of K = E, active_module -1) on the records received as [src][local expert][cap] with live
 *                       counts recv_cnt (W, E) (clamped to cap) -> ret (W*E*cap, 4) (rgb, sigma) in the same
 *                       layout; per record the arithmetic of the fused routed render.
 *   acn_ep_composite -> sender: per sample y = 0 + sum_k y_k w_k over its pairs in ascending k (pmap (N*S, K)
 *                       pair index or -1, yr (pairs, 4) the returned field outputs, pw the weights; hard != 0:
 *                       y = y_k, index_copy_), then compositing, background and outputs as
 *                       acn_render_stratified_fwd (weights may be NULL).                                   */
int acn_ep_field_fwd(const float* recv_xd, const int64_t* recv_cnt, int W, int E, int64_t cap,
                     const acn_expert* experts, const void* packed, size_t packed_bytes, float* ret, void* stream);
/* acn_ep_field_fwd_compact -> as acn_ep_field_fwd; cap = 0 selects the COMPACT received layout of a planned
 *                       exchange: segment (src w, local expert e) holds exactly recv_cnt[w][e] records, segments in
 *                       row-major (w, e) order with no gaps (W * E <= 1024); max_cnt = the largest recv_cnt (host,
 *                       sizes the grid).  cap > 0: the fixed layout of acn_ep_field_fwd (max_cnt ignored). */
int acn_ep_field_fwd_compact(const float* recv_xd, const int64_t* recv_cnt, int W, int E, int64_t cap, int64_t max_cnt,
                             const acn_expert* experts, const void* packed, size_t packed_bytes, float* ret,
                             void* stream);
/* acn_routed_count_batches -> the plan of a planned expert-parallel frame: counts (ceil(N / batch), K) int64
 *                       (device) = per batch of `batch` consecutive rays, the samples routed to each expert
 *                       (w_k > 0; the counts acn_routed_count / _caps give that batch, same t and routing
 *                       arithmetic).  Replaces nothing in the reference: it sizes the all-to-all that stands in
 *                       for MetaContainer.forward's per-expert index_select (meta_container.py:307-321). */
int acn_routed_count_batches(const float* rays, int64_t N, int S, int64_t batch, const float* jitter,
                             const acn_routing* routing, int64_t* counts, void* stream);
int acn_ep_composite(const float* rays, int64_t N, int S, const float* jitter, const float* yr, const float* pw,
                     const int32_t* pmap, int K, int hard, const acn_background* bg, float sigma_scale, float tau,
                     float* rgb, float* depth, float* weights, float* acc, void* stream);

/* Per-expert kernels over routed pair slots (segments padded to multiples of 128, slot count seg[K] on the
 * device; fixed grids that stride to it, so a whole step is capturable in a hipGraph):
 *   acn_hashgrid_fwd_pairs : h0 (slots, L*2) of every slot through its expert's table (tables: HOST array
 *                            of K device pointers); all experts share res[L], log2T, F = 2.
 *   acn_hashgrid_bwd_pairs : scatter-add of dL/dh0 into every expert's table gradient (grad_tables: HOST
 *                            array of K device pointers; float atomics); padding slots (pidx < 0) skipped.
 *   acn_mlp_pack_pairs     : the K experts' MLP images into workspace (acn_mlp_pairs_workspace_bytes(K)).
 *   acn_mlp_train_fwd_pairs / acn_mlp_train_bwd_dw_pairs : the fused expert MLP forward / backward (as
 *                            acn_mlp_train_fwd / _bwd_dw) per slot with its expert's weights; dw (K, 13715)
 *                            per-expert [dW | db] (zeros for an expert without pairs; summed in a fixed
 *                            order: deterministic), gh0 (slots, 32).                                   */
int acn_hashgrid_fwd_pairs(const float* x01, const int32_t* pk, const int64_t* seg, int K, const float* const* tables,
                           const int32_t* res, int L, int log2T, int interp, float* out, void* stream);
int acn_hashgrid_bwd_pairs(const float* x01, const int32_t* pk, const int32_t* pidx, const int64_t* seg, int K,
                           const float* grad_out, float* const* grad_tables, const int32_t* res, int L, int log2T,
                           int interp, void* stream);
/* acn_hashgrid_bwd_pairs that also adds, to the device double *table_sumsq, the change of the squared
 * norm of the gradient tables (returning atomics: sum of new^2 - old^2, which telescopes per row), i.e.
 * the tables' share of clip_grad_norm_'s sum of squares (runtime_adapt.py:305-307) when the tables start
 * the step at zero -- no pass over the K x 128 MiB gradients.  Not combinable with the merged coarse
 * levels (ACN_HASH_BWD_MERGE builds: returns an error). */
int acn_hashgrid_bwd_pairs_sumsq(const float* x01, const int32_t* pk, const int32_t* pidx, const int64_t* seg,
                                 int K, const float* grad_out, float* const* grad_tables, const int32_t* res, int L,
                                 int log2T, int interp, double* table_sumsq, void* stream);
size_t acn_mlp_pairs_workspace_bytes(int K);
int acn_mlp_pack_pairs(const acn_mlp* const* w, int K, void* workspace, void* stream);
int acn_mlp_train_fwd_pairs(const float* h0, const float* sh, const int64_t* seg, int K, const void* workspace,
                            float* out, void* stream);
int acn_mlp_train_bwd_dw_pairs(const float* h0, const float* sh, const float* out, const float* gout,
                               const int64_t* seg, int K, void* workspace, float* dw, float* gh0, void* stream);

/* ---- training loss (round 2): nerfs/losses.py:10-32 compute_mse_loss with color_space="linear"
 * (nerfs/color_space.py:13-19, 22-66): loss = mean((clamp(pred,0,1) - clamp(srgb_to_linear(clamp(gt,0,1)),0,1))^2)
 * over n = 3 * rays floats.  fwd: one workgroup, double partials, deterministic; writes loss[0].
 * bwd: g_pred = 2/n * (clamp(pred) - gt_lin) * g_loss[0] where 0 <= pred <= 1, else 0 (mse_loss_backward
 * through clamp's backward).  g_loss is a DEVICE scalar (graph-replayable). */
int acn_mse_linear_fwd(const float* pred, const float* gt, int64_t n, float* loss, void* stream);
/* The same loss over up to 256 workgroups (deterministic: fixed per-thread assignment and reduction order
 * for a given n; a last-workgroup ticket adds the workgroup sums in order).  workspace: a device buffer of
 * acn_mse_linear_workspace_bytes(), ZEROED once before first use (the call leaves its counter at 0 again);
 * one workspace per stream. */
size_t acn_mse_linear_workspace_bytes(void);
int acn_mse_linear_fwd_ws(const float* pred, const float* gt, int64_t n, float* loss, void* workspace,
                          size_t workspace_bytes, void* stream);
int acn_mse_linear_bwd(const float* pred, const float* gt, int64_t n, const float* g_loss, float* g_pred,
                       void* stream);


/* The training MLP in exact fp32 (v_mfma_f32_32x32x2_f32 layer products instead of the fp32-accurate fp16x3
 * split): the same ten entry points, suffixed _exact, same arguments and semantics; workspaces must come
 * from the _exact size functions (the weight image layout differs).  mlp_train.hip compiled a second time
 * with -DACN_TRAIN_F16X3=0 (a runtime precision switch for parity studies: DESIGN.md 4). */
size_t acn_mlp_workspace_bytes_exact(void);
int acn_mlp_train_fwd_exact(const float* h0, const float* sh, int64_t M, const acn_mlp* w, float* out, float* save,
                      void* workspace, void* stream);
int acn_mlp_train_bwd_exact(const float* save, const float* out, const float* gout, int64_t M, const acn_mlp* w,
                      float* gsave, float* gh0, void* workspace, void* stream);
size_t acn_mlp_dw_workspace_bytes_exact(void);
int acn_mlp_train_bwd_dw_exact(const float* h0, const float* sh, const float* out, const float* gout, int64_t M,
                         const acn_mlp* w, float* dw, float* gh0, void* workspace, void* stream);
int acn_mlp_train_bwd_dw_img_exact(const float* h0, const float* sh, const float* out, const float* gout, int64_t M,
                             const float* img, float* dw, float* gh0, void* workspace, void* stream);
size_t acn_mlp_pairs_workspace_bytes_exact(int K);
int acn_mlp_pack_pairs_exact(const acn_mlp* const* w, int K, void* workspace, void* stream);
int acn_mlp_train_fwd_pairs_exact(const float* h0, const float* sh, const int64_t* seg, int K, const void* workspace,
                            float* out, void* stream);
int acn_mlp_train_bwd_dw_pairs_exact(const float* h0, const float* sh, const float* out, const float* gout,
                               const int64_t* seg, int K, void* workspace, float* dw, float* gh0, void* stream);

/* The training MLP in the reference's use_amp arithmetic (the MetaLinear chain under torch.autocast(float16):
 * pipelines/online_stage/runtime_adapt.py:249-259, pipelines/offline_stage/meta_core.py:38, configs/train.json:37):
 * one fp16 x fp16 MFMA product per term with fp32 accumulation, every layer output, activation, dX and
 * [dW | db] rounded to fp16 once, the incoming gradient cast to fp16; no internal rescaling (the caller's
 * loss scale -- acn_amp_unscale_coef -- keeps the gradients in fp16's range, as GradScaler does).  The same ten
 * entry points, suffixed _amp; workspaces from the _amp size functions.  mlp_train.hip compiled a third
 * time with -DACN_TRAIN_AMP=1. */
size_t acn_mlp_workspace_bytes_amp(void);
int acn_mlp_train_fwd_amp(const float* h0, const float* sh, int64_t M, const acn_mlp* w, float* out, float* save,
                          void* workspace, void* stream);
int acn_mlp_train_bwd_amp(const float* save, const float* out, const float* gout, int64_t M, const acn_mlp* w,
                          float* gsave, float* gh0, void* workspace, void* stream);
size_t acn_mlp_dw_workspace_bytes_amp(void);
int acn_mlp_train_bwd_dw_amp(const float* h0, const float* sh, const float* out, const float* gout, int64_t M,
                             const acn_mlp* w, float* dw, float* gh0, void* workspace, void* stream);
int acn_mlp_train_bwd_dw_img_amp(const float* h0, const float* sh, const float* out, const float* gout, int64_t M,
                                 const float* img, float* dw, float* gh0, void* workspace, void* stream);
size_t acn_mlp_pairs_workspace_bytes_amp(int K);
int acn_mlp_pack_pairs_amp(const acn_mlp* const* w, int K, void* workspace, void* stream);
int acn_mlp_train_fwd_pairs_amp(const float* h0, const float* sh, const int64_t* seg, int K, const void* workspace,
                                float* out, void* stream);
int acn_mlp_train_bwd_dw_pairs_amp(const float* h0, const float* sh, const float* out, const float* gout,
                                   const int64_t* seg, int K, void* workspace, float* dw, float* gh0, void* stream);

/* torch.cuda.amp.GradScaler's unscale_ + clip_grad_norm_ + step-skip + update in one device launch
 * (replaces scaler.unscale_(optimizer); clip_grad_norm_(params, max_norm); scaler.step(optimizer);
 * scaler.update() of runtime_adapt.py:261-268 for the fused Adam paths).  total_sumsq = sum of squares of the
 * SCALED gradients (acn_grad_sumsq*); scale (float32[1]), growth_tracker (int32[1]) and found_inf (float32[1])
 * are device scalars -- GradScaler's own _scale / _growth_tracker tensors can be passed.  Writes out[0] = the
 * unscaled total norm, out[1] = the Adam gradient multiplier clip_coef / scale (clip_coef = 1 when max_norm
 * <= 0); when the norm is not finite (an inf / NaN gradient: GradScaler's found_inf) the step is skipped --
 * seg[K] = -1 (the slotted Adam's no-step gate; seg may be NULL for callers that test found_inf) -- and the
 * scale backs off (x backoff, tracker 0); otherwise tracker += 1 and, at growth_interval, the scale grows
 * (x growth, tracker 0: torch._amp_update_scale_).  Powers of two keep the unscaling exact. */
int acn_amp_unscale_coef(const double* total_sumsq, float max_norm, float* scale, int32_t* growth_tracker,
                         float* found_inf, float growth, float backoff, int growth_interval, float* out, int64_t* seg,
                         int K, void* stream);

/* Segment maps of the hash-table gradients (routed step): per expert table two byte maps over
 * its 64-B segments (8 rows of 2 features): now[s] = the scatter added into segment s this step, ever[s] = it
 * was updated by an earlier step.
 *   acn_hashgrid_bwd_pairs_segmap -> acn_hashgrid_bwd_pairs_sumsq that also sets now[] of every segment it adds
 *                                   into (seg_now: HOST array of K device byte maps, nullable).
 *   acn_adam_step_slots_segmap    -> acn_adam_step_slots where tensor t with segmaps[2t] != NULL (device array
 *                                   of 2 * ntensors byte-map pointers: now, ever) skips segments never touched
 *                                   (m = v = g = 0: torch's Adam with weight_decay 0 leaves them bit-identical),
 *                                   reads no gradient for segments not touched this step (g = 0 there), then
 *                                   sets ever |= now and clears now.  Mapped tensors: numel a multiple of 16,
 *                                   group weight_decay 0, 16-B aligned.  Exact: bitwise the dense update. */
int acn_hashgrid_bwd_pairs_segmap(const float* x01, const int32_t* pk, const int32_t* pidx, const int64_t* seg, int K,
                                  const float* grad_out, float* const* grad_tables, const int32_t* res, int L,
                                  int log2T, int interp, double* table_sumsq, uint8_t* const* seg_now, void* stream);
/* acn_hashgrid_pairs_mark -> only the now[] marks of acn_hashgrid_bwd_pairs_segmap (no gradient written): the
 * segment maps of a step whose table gradients came from the deterministic sort-based backward. */
int acn_hashgrid_pairs_mark(const float* x01, const int32_t* pk, const int32_t* pidx, const int64_t* seg, int K,
                            const int32_t* res, int L, int log2T, int interp, uint8_t* const* seg_now, void* stream);
int acn_adam_step_slots_segmap(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                               const int32_t* flags, const void* table, int ngroups, int table_steps, int32_t* step_dev,
                               int nslots, const int64_t* seg, int K, const float* grad_scale, uint8_t* const* segmaps,
                               void* stream);
/* The same update in two passes, so most of its bytes can run beside the step's forward / backward on a
 * second stream (routed_train.RoutedAdaptStep):
 *   phase 1 (early, once the now[] marks of the step are set -- acn_hashgrid_pairs_mark after the pair
 *            scatter): advances the active slots' step counters and updates the mapped tensors' segments touched
 *            before but not now -- their gradient is zero, so neither the gradient nor the clip coefficient is
 *            read; maps unchanged;
 *   phase 2 (late, after the clip coefficient): the mapped segments touched now and every unmapped tensor
 *            (maps and gradients updated / cleared as in acn_adam_step_slots_segmap); no counter bump.
 * Each element sees exactly acn_adam_step_slots_segmap's arithmetic (bitwise the same update). */
int acn_adam_step_slots_segmap_phase(const acn_param_desc* descs, const int32_t* chunk_tensor, int64_t nchunks,
                                     const int32_t* flags, const void* table, int ngroups, int table_steps,
                                     int32_t* step_dev, int nslots, const int64_t* seg, int K, const float* grad_scale,
                                     uint8_t* const* segmaps, int phase, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ACNERF_H */
