/*
 * nrt.h -- C ABI of libnrt_hip.so, the MI355X (gfx950) ray-march render path.
 *
 * The reference (prashantraina/neural_raytracing, pytorch3d/pathtracer) has no FFI: its hot path
 * sits behind duck-typed Python objects.  Each entry point below replaces one of those Python
 * call sites; the comment on each names the reference file:line it stands in for.  The Python
 * host layer (neural_raytracing_amd/pathtracer) binds these with ctypes.
 *
 * Conventions
 *   - All array pointers are DEVICE memory owned by the caller unless the name says host_.
 *   - Every compute call is stream-ordered on the caller's hipStream_t (passed as void*);
 *     nothing synchronises the device and nothing allocates device memory except the
 *     *_create functions (weights are packed once) and nrt_workspace_* helpers.
 *   - Rays are [P, 6] float32 = origin(3) || direction(3), P = N*W*H*B flattened in the
 *     reference's [N, W, H, B] order.
 *   - Return value: 0 on success, negative NRT_E* on error; nrt_last_error() returns a
 *     thread-local message for the last failure on the calling thread.
 *   - precision: NRT_FP32 computes every MLP layer with exact-f32 MFMA (v_mfma_f32_32x32x2_f32 /
 *     16x16x4_f32) and matches the CPU restatement to ~1e-6; NRT_FP16 uses v_mfma_f32_32x32x16_f16
 *     with f32 accumulation (the throughput path, judged by PSNR against FP32); NRT_FP32_SPLIT is
 *     NRT_FP32 except that the SDF march + coarse scan of the ring-engine SDFs runs every layer on
 *     v_mfma_f32_16x16x32_f16 with each f32 operand split into two f16 halves and three products
 *     (hi*hi + hi*lo + lo*hi, f32 accumulation): FP32 accuracy (22-bit operands, fewer
 *     accumulation roundings than an fma chain) at FP16 matrix-core throughput.  NRT_MIXED is
 *     NRT_FP32_SPLIT except that the ring-engine SDF march + scan runs at FP16 and every decision
 *     FP16 cannot make (a step whose value lies within the "mixed_refine_d" bound of eps or of
 *     max_t, a scan whose two smallest values lie within "mixed_refine_s") is taken again on the
 *     split engine; sdf(best), the normals and the shading are split.
 */
#ifndef NRT_H_
#define NRT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NRT_OK 0
#define NRT_EINVAL (-1)
#define NRT_EUNSUPPORTED (-2)
#define NRT_EHIP (-3)
#define NRT_ENOMEM (-4)

#define NRT_FP32 0
#define NRT_FP16 1
#define NRT_FP32_SPLIT 2
#define NRT_MIXED 3

/* activations (neural_blocks.py:26 leaky_relu default; sdfs.py:29 softplus) */
#define NRT_ACT_LEAKY_RELU 0
#define NRT_ACT_SOFTPLUS 1
#define NRT_ACT_NONE 2
#define NRT_ACT_SIGMOID 3
#define NRT_ACT_RELU 4

const char* nrt_last_error(void);
int nrt_version(void);
/* 1 when the library was built for gfx950 and a device is visible; 0 otherwise */
int nrt_device_ok(void);

/* ---------------------------------------------------------------------------------------
 * SkipConnMLP (neural_blocks.py:12-86 + utils.py:33-40 fourier2)
 * ------------------------------------------------------------------------------------- */
typedef struct nrt_mlp nrt_mlp;

typedef struct {
  int32_t in_size;     /* input features (3 for points)                                   */
  int32_t hidden;      /* hidden width, multiple of 32 (32..256)                          */
  int32_t num_layers;  /* hidden Linear layers (skip-concat layers counted)               */
  int32_t out;         /* output features (<= 96)                                         */
  int32_t freqs;       /* Fourier features F: basis is [in_size, F]                       */
  int32_t skip;        /* skip period: layer i concatenates the encoding iff              */
                       /*   i != num_layers-1 && i % skip == 0   (neural_blocks.py:48,82) */
  int32_t latent;      /* latent_size appended to the encoding                            */
  int32_t activation;  /* NRT_ACT_*                                                       */
} nrt_mlp_desc;

/* Pack host float32 weights (torch layout).  host_basis: [in_size, F] (basis_p).
 * host_weights[l], host_biases[l] for l = 0 (init: [hidden, dp]), 1..num_layers (layers[i]:
 * [hidden, hidden (+dp if skip)]), num_layers+1 (out: [out, hidden]); dp = in+2F+latent.
 * Replaces the per-call eager Linear chain (neural_blocks.py:75-86). */
int nrt_mlp_create(const nrt_mlp_desc* desc, const float* host_basis,
                   const float* const* host_weights, const float* const* host_biases,
                   nrt_mlp** out);
int nrt_mlp_destroy(nrt_mlp* mlp);
/* Re-pack an MLP handle from the caller's DEVICE weights after an optimiser step (training,
 * SURVEY §8f rank 1; the same nn.Linear layouts as nrt_mlp_create, stream-ordered, no host copy):
 * refreshes the fragments nrt_mlp_forward / nrt_mlp_backward / nrt_mlp_grad_backward read and the
 * FP32 and fp32-split march streams.  A refreshed handle no longer serves the FP16 ring march or
 * shading programs (those calls fall back or fail); render with a handle from nrt_mlp_create. */
int nrt_mlp_refresh(nrt_mlp* mlp, const float* const* device_weights,
                    const float* const* device_biases, void* stream);

/* y[M, out] = SkipConnMLP(x[M, in], latent[M, latent]) -- neural_blocks.py:75-86 */
int nrt_mlp_forward(const nrt_mlp* mlp, const float* x, const float* latent, int64_t M,
                    float* y, int precision, void* stream);
/* y[k][M, out] = mlps[k](x) for n same-shape MLPs without latent on one input: the NeuralBSDF
 * components of a spatially varying mixture on the shared Rusinkiewicz features (bsdfs.py:
 * 634-637, called per component there).  At FP32 the shading MLP shapes run as one launch on
 * the ring engine (n x the row blocks, up to 16 MLPs a launch); other shapes and precisions are
 * n nrt_mlp_forward calls.  Each y[k] equals nrt_mlp_forward(mlps[k], ...) bit for bit.
 * save (training; NULL for none): one device buffer of nrt_mlp_save_bytes(mlps[k], M) bytes per
 * MLP; the forward also stores the activations the backward needs (every hidden layer's and the
 * Fourier encoding), so nrt_mlp_backward_saved does not evaluate the forward again -- the torch
 * autograd contract (the forward saves, the backward reads).  FP32 only; NRT_EUNSUPPORTED for
 * MLPs whose nrt_mlp_save_bytes is 0. */
int nrt_mlp_forward_multi(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                          float* const* y, void* const* save, int precision, void* stream);
/* Bytes of one MLP's saved activations for M rows; 0 when the MLP has no saving forward (the
 * shading shapes of the ring backward only: see option "bwd_ring"). */
size_t nrt_mlp_save_bytes(const nrt_mlp* mlp, int64_t M);

/* Backward of nrt_mlp_forward in FP32 (torch autograd through
 * SkipConnMLP.forward, neural_blocks.py:75-86): given dy [M, out] = dL/dy, writes
 *   dx [M, in] and dlatent [M, latent] (each may be NULL),
 *   dweights[l] [R_l, C_l] and dbiases[l] [R_l] for l = 0 (init), 1..num_layers (hidden),
 *   num_layers + 1 (out), in the torch nn.Linear layouts (host arrays of device pointers; the
 *   arrays or single entries may be NULL).  Gradients are overwritten, not accumulated.
 * workspace: nrt_mlp_backward_workspace_bytes(mlp, M) bytes of device memory. */
size_t nrt_mlp_backward_workspace_bytes(const nrt_mlp* mlp, int64_t M);
int nrt_mlp_backward(const nrt_mlp* mlp, const float* x, const float* latent, int64_t M,
                     const float* dy, float* dx, float* dlatent, float* const* dweights,
                     float* const* dbiases, void* workspace, void* stream);

/* nrt_mlp_backward for n MLPs of one shape (no latent) on the same input x [M, in] -- the
 * NeuralBSDFs of a ComposeSpatialVarying mixture, which all read param_rusin(wi, wo)
 * (bsdfs.py:634-637) -- in one backward launch and one weight-gradient launch.  dy[i] [M, out],
 * dx[i] [M, in] (the array or entries may be NULL); dweights / dbiases are flat host arrays of
 * n x (num_layers + 2) device pointers, MLP-major.  Per MLP the same results as nrt_mlp_backward
 * up to the split-K summation order of the weight gradients.
 * workspace: nrt_mlp_backward_multi_workspace_bytes(mlps, n, M) bytes. */
size_t nrt_mlp_backward_multi_workspace_bytes(const nrt_mlp* const* mlps, int n, int64_t M);
int nrt_mlp_backward_multi(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                           const float* const* dy, float* const* dx, float* const* dweights,
                           float* const* dbiases, void* workspace, void* stream);
/* nrt_mlp_backward_multi from the activations nrt_mlp_forward_multi saved (saved[i], Ms rows):
 * the backward chain and the weight gradients only.  Row i of this call (x [M, in], dy[i]) is
 * saved row rows[i] (int32 [M]; NULL: M == Ms and row i) -- the rows with a gradient, compacted
 * by the caller.  Same gradients as nrt_mlp_backward_multi on those rows, bit for bit.
 * workspace: nrt_mlp_backward_multi_workspace_bytes(mlps, n, M) bytes. */
int nrt_mlp_backward_saved(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                           const int32_t* rows, const void* const* saved, int64_t Ms,
                           const float* const* dy, float* const* dx, float* const* dweights,
                           float* const* dbiases, void* workspace, void* stream);

/* Double backward of the input gradient (SDF.autograd_diff with
 * create_graph=True, sdfs.py:184-197, differentiated again by loss.backward()): for
 * g(x) = d(sum_o y_o)/dx [M, in] (torch.autograd.grad with grad_outputs = ones) and v [M, in] =
 * dL/dg, writes dweights[l], dbiases[l] = d(sum_rows v . g)/dW_l, /db_l in the nn.Linear layouts
 * (FP32; latent is held constant; x is not differentiated).  Gradients are overwritten.
 * workspace: nrt_mlp_grad_backward_workspace_bytes(mlp, M) bytes of device memory. */
size_t nrt_mlp_grad_backward_workspace_bytes(const nrt_mlp* mlp, int64_t M);
int nrt_mlp_grad_backward(const nrt_mlp* mlp, const float* x, const float* latent, int64_t M,
                          const float* v, float* const* dweights, float* const* dbiases,
                          void* workspace, void* stream);

/* ---------------------------------------------------------------------------------------
 * Signed distance fields (shapes/sdfs.py)
 * ------------------------------------------------------------------------------------- */
typedef struct nrt_sdf nrt_sdf;

/* SPHERE_SDF = |p| - 1 (sdfs.py:13) */
int nrt_sdf_create_unit_sphere(nrt_sdf** out);
/* a bare SkipConnMLP with out=1 used as the SDF */
int nrt_sdf_create_mlp(const nrt_mlp* mlp, nrt_sdf** out);
/* SphereSDF (sdfs.py:16-44): smooth_min_k(|(I+tfs_i) p - c_i| - r_i) + shift(p).
 * host_centers [n,3], host_radii [n], host_tfs [n,3,3]; shift may be NULL. */
int nrt_sdf_create_sphere_blob(int32_t n, const float* host_centers, const float* host_radii,
                               const float* host_tfs, float k, const nrt_mlp* shift,
                               nrt_sdf** out);
/* Rewrite a sphere-blob SDF's sphere table from device tensors (same layout as the host
 * arguments of nrt_sdf_create_sphere_blob), stream-ordered: the training path's per-step update
 * after an optimiser step, with no host round trip.  NRT_EINVAL for other SDF kinds. */
int nrt_sdf_refresh_spheres(nrt_sdf* sdf, const float* device_centers, const float* device_radii,
                            const float* device_tfs, void* stream);
int nrt_sdf_destroy(nrt_sdf* sdf);

/* out[M] = sdf(p[M,3]) */
int nrt_sdf_eval(const nrt_sdf* sdf, const float* p, int64_t M, float* out, int precision,
                 void* stream);
/* out[M,3] = d sdf / d p  (SDF.autograd_diff, sdfs.py:184-197; f32 backward) */
int nrt_sdf_grad(const nrt_sdf* sdf, const float* p, int64_t M, float* grad, void* stream);

/* SphereSDF's smooth-min part for training (sdfs.py:37-43, utils.py:386-387; replaces the
 * torch ops of SphereSDF.forward and of SDF.autograd_diff's create_graph=True gradient,
 * sdfs.py:184-197, when the points carry no gradient): value[P] = -log(max(sum_i exp(-k sd_i),
 * 1e-4)) / k with sd_i = |(I + tfs_i) p - c_i| - R_i, and grad[P,3] = d value / d p (either
 * output may be NULL).  centers [n,3], radii [n], tfs [n,3,3] are the module's device tensors;
 * n <= 1260. */
int nrt_sphere_smoothmin_forward(const float* p, int64_t P, const float* centers,
                                 const float* radii, const float* tfs, int32_t n, float k,
                                 float* value, float* grad, void* stream);
/* The backward of both outputs with respect to the sphere parameters (for grad: the double
 * backward of the normal): dcenters [n,3], dradii [n], dtfs [n,3,3] (each may be NULL) are
 * overwritten with sum_points dvalue . d value / d theta + dgrad . d grad / d theta; dvalue [P]
 * and dgrad [P,3] may be NULL (no gradient).  Deterministic (fixed-order sums).
 * workspace: nrt_sphere_smoothmin_workspace_bytes(P) bytes. */
size_t nrt_sphere_smoothmin_workspace_bytes(int64_t P);
int nrt_sphere_smoothmin_backward(const float* p, int64_t P, const float* centers,
                                  const float* radii, const float* tfs, int32_t n, float k,
                                  const float* dvalue, const float* dgrad, float* dcenters,
                                  float* dradii, float* dtfs, void* workspace, void* stream);

typedef struct {
  int32_t max_steps;   /* SDF.max_steps (sdfs.py:96; scripts set 32/64/256)               */
  float epsilon;       /* SDF.epsilon 1e-3                                                 */
  float max_t;         /* intersect(max_t=10)                                              */
  int32_t primary;     /* 1: run the 128-step coarse scan (SDF.throughput, sdfs.py:232)     */
  double scan_max_t;   /* dist + random.random()*(2/128), computed by the caller           */
  int32_t precision;   /* NRT_FP32 / NRT_FP16 / NRT_FP32_SPLIT / NRT_MIXED                  */
  int32_t* scan_index; /* optional [P] output: the coarse-scan argmin idxs (sdfs.py:243-246), so a
                          training caller can rebuild best_pos = o + idx*step*d; NULL = unused  */
  /* Batched tiles (pathtrace's chunk_size^2 tile loop in one call, main.py:63-90): when not NULL,
   * a DEVICE array of per-group scan_max_t values (one random.random() draw per tile,
   * sdfs.py:236); ray r uses group r / group_rays and scan_max_t is ignored.  NULL = one group. */
  const double* scan_max_t_groups;
  int64_t group_rays;
} nrt_march_params;

/* SDF.intersect (sdfs.py:111-160) for P rays.  Outputs (each [P] or [P,3]):
 *   t, hit (uint8), p (offset by 5*eps*n on hits), n (unit normal, 0 on misses),
 *   raw_n (un-normalised gradient, 0 on misses; may be NULL), wi = to_local(-d) (NULL ok),
 *   throughput (-1000*sdf(best scan point); untouched when primary == 0).
 * hit_idx[P] / hit_count[1] (int32, optional): compacted indices of hit rays (any order).
 * workspace: nrt_intersect_workspace_bytes(P) bytes of device memory. */
size_t nrt_intersect_workspace_bytes(const nrt_sdf* sdf, int64_t P);
int nrt_sdf_intersect(const nrt_sdf* sdf, const float* rays, int64_t P,
                      const nrt_march_params* params, float* t, uint8_t* hit, float* p, float* n,
                      float* raw_n, float* wi, float* throughput, int32_t* hit_idx,
                      int32_t* hit_count, void* workspace, void* stream);

/* SDF.intersect_test (sdfs.py:162-181): visible[P] = (t >= max_t[P]) | still-marching,
 * march from t0 = 100*eps.  max_t is per ray (scene.py:296 passes the light distance). */
int nrt_sdf_occlusion(const nrt_sdf* sdf, const float* rays, int64_t P, const float* max_t,
                      int32_t max_steps, float epsilon, uint8_t* visible, int precision,
                      void* stream);

/* SDF callables the library cannot pack (SDF(sdf=f) with f any function of p: a warp or a
 * displacement around a packed SDF, edit_dtu.py:86-100).  The caller evaluates f on the query
 * points q[P,3] between steps; these do the rest of sdfs.py:111-181, elementwise in ray order.
 *
 * March (sdfs.py:118-133): first call dists = NULL (t = 0, remaining = 1, hit = 0); every later
 * call consumes dists = f(q) of the step just taken (hit |= remaining & d <= eps, remaining &=
 * !hit-now, t += d where still remaining).  prep = 1 then applies the next step's remaining &=
 * t < max_t; every call writes q = r_o + t r_d (after the last step: the march's p).
 * Replaces the loop at sdfs.py:118-131 (reference: torch ops around self.sdf). */
int nrt_march_callable_step(const float* rays, int64_t P, const float* dists, float epsilon,
                            float max_t, int prep, float* t, uint8_t* remaining, uint8_t* hit,
                            float* q, void* stream);
/* Coarse scan (SDF.throughput, sdfs.py:232-249): sd = f(scan point j) for j = 0 .. 128 (point 0
 * = r_o); keeps the first strict minimum (curr_min, idx).  prep = 1 writes scan point j + 1
 * (r_o + (float)(step (j+1)) r_d), prep = 2 writes best_pos = r_o + ((float)idx (float)step) r_d. */
int nrt_scan_callable_step(const float* rays, int64_t P, const float* sd, int32_t j, double step,
                           int prep, float* curr_min, int32_t* idx, float* q, void* stream);
/* Shadow march (SDF.intersect_test, sdfs.py:162-181): phase 0 sets depth = t0 (= 1e2 eps,
 * rounded to f32 by the caller), remaining = 1 and q; phase 1 consumes dists (depth += d where
 * remaining, then remaining &= d >= eps) and writes q; phase 2 consumes the last step and writes
 * visible = depth >= max_t[i] | remaining. */
int nrt_occlusion_callable_step(const float* rays, int64_t P, const float* dists, float epsilon,
                                float t0, const float* max_t, int phase, float* depth,
                                uint8_t* remaining, float* q, uint8_t* visible, void* stream);

/* ---------------------------------------------------------------------------------------
 * Lights (lights/lights.py) and BSDFs (bsdf/bsdfs.py)
 * ------------------------------------------------------------------------------------- */
typedef struct nrt_light nrt_light;
typedef struct nrt_bsdf nrt_bsdf;

/* LightField (lights.py:155-195): 10x256 MLP -> direction/magnitude, colour = sigmoid(c) */
int nrt_light_create_field(const nrt_mlp* mlp, const float* host_color3, nrt_light** out);
/* PointLights (lights.py:40-110), one light */
int nrt_light_create_point(const float* host_location3, const float* host_intensity3,
                           float constant, float linear, float square, float scale,
                           nrt_light** out);
/* pytorch3d.renderer.PointLights as a pathtracer light (renderer/lighting.py:221-304, the light
 * of utils.sphere_examples, utils.py:409-431): d = (loc - p) / (1e-7 + |loc - p|),
 * Le = scale * intensity / (1e-7 + |loc - p|)^2, intensity = ambient_color; one light */
int nrt_light_create_renderer_point(const float* host_location3, const float* host_intensity3,
                                    float scale, nrt_light** out);
int nrt_light_destroy(nrt_light* light);

#define NRT_BSDF_NEURAL 0     /* NeuralBSDF (bsdfs.py:613-637): act(MLP(param_rusin2))     */
#define NRT_BSDF_DIFFUSE 1    /* Diffuse (bsdfs.py:78-118)                                 */
#define NRT_BSDF_CONDUCTOR 2  /* Conductor (bsdfs.py:345-388)                              */

typedef struct {
  int32_t kind;          /* NRT_BSDF_*                                                     */
  const nrt_mlp* mlp;    /* NEURAL only                                                    */
  int32_t activation;    /* NEURAL: act; DIFFUSE: preprocess (NONE = x/pi, SIGMOID, ...);  */
                         /* CONDUCTOR: act on specular                                      */
  float params[4];       /* DIFFUSE: reflectance rgb; CONDUCTOR: specular rgb, eta         */
} nrt_bsdf_component;

/* ComposeSpatialVarying (bsdfs.py:482-536): sum_j sigmoid(sp_var(p))_j * f_j.
 * spatial may be NULL for a single component (weight 1, no sigmoid). */
int nrt_bsdf_create(int32_t n, const nrt_bsdf_component* components, const nrt_mlp* spatial,
                    nrt_bsdf** out);
int nrt_bsdf_destroy(nrt_bsdf* bsdf);

/* Direct.sample's emitter + BSDF block (integrators.py:173-189) for the hit rays listed in
 * hit_idx[0 .. *hit_count): light sample at p, wo = to_local(frame(n), d_light),
 * rgb[i] = (sum_j k_j f_j(wi, wo)) * Le.  rgb of rays not listed is left untouched.
 * weights_out [P, n_components] (optional): the sigmoid spatial weights
 * (it.normalized_weights, bsdfs.py:520). */
int nrt_shade_direct(const nrt_bsdf* bsdf, const nrt_light* light, const float* p,
                     const float* n, const float* wi, const int32_t* hit_idx,
                     const int32_t* hit_count, int64_t P, float* rgb, float* weights_out,
                     int precision, void* stream);

/* Direct.sample with w_isect=True (integrators.py:163 -> sample_emitter_dir_w_isect,
 * scene.py:290-298): for each listed hit ray, a point-light sample, a shadow ray
 * [p, d_light] marched like SDF.intersect_test (sdfs.py:162-181; t0 = 100*eps, max_steps,
 * max_t = light distance), Le = 0 where occluded, then the shading of nrt_shade_direct.
 * visible_out [P] (optional) receives the visibility per hit-list position.  Needs a point light
 * (NRT_EUNSUPPORTED otherwise: the reference's LightField samples carry no distance).
 * workspace: nrt_shadow_workspace_bytes(P) bytes of device memory. */
size_t nrt_shadow_workspace_bytes(int64_t P);
int nrt_shade_direct_shadowed(const nrt_bsdf* bsdf, const nrt_light* light, const nrt_sdf* sdf,
                              int32_t max_steps, float epsilon, const float* p, const float* n,
                              const float* wi, const int32_t* hit_idx, const int32_t* hit_count,
                              int64_t P, float* rgb, float* weights_out, uint8_t* visible_out,
                              void* workspace, int precision, void* stream);

/* Direct shading with a LEARNED occlusion term: sample_emitter_dir_w_learned_occ
 * (scene.py:301-319, selected by Direct/Path when w_isect is a SkipConnMLP,
 * integrators.py:164-166 and :289-291).  As nrt_shade_direct_shadowed, but an occluded sample keeps
 * sigmoid(occ([p, dir_to_elev_azim(d)])) * Le instead of 0 (utils.py:490-494 for elev/azim).
 * occ: an nrt_mlp mapping 5 -> 1 (broadcast over RGB) or 5 -> 3.  Same workspace size. */
int nrt_shade_direct_learned_occ(const nrt_bsdf* bsdf, const nrt_light* light, const nrt_sdf* sdf,
                                 const nrt_mlp* occ, int32_t max_steps, float epsilon,
                                 const float* p, const float* n, const float* wi,
                                 const int32_t* hit_idx, const int32_t* hit_count, int64_t P,
                                 float* rgb, float* weights_out, uint8_t* visible_out,
                                 void* workspace, int precision, void* stream);

/* One bounce of Path.sample (integrators.py:309-350) over the rays with active[i] != 0:
 *   result[i] += throughput[i] * f(wi, wo_light) * Le   (the emitter term; shadow rays toward the
 *                point light when shadow != 0, as w_isect=True; with occ != NULL as well, an
 *                occluded Le is scaled by the learned occlusion, as nrt_shade_direct_learned_occ)
 *   BSDF sample (ComposeSpatialVarying.sample, bsdfs.py:500-513; NeuralBSDF / Diffuse components)
 *     from injected uniforms: u_comp [P, n_components, 2] (each component's sampler draw, in
 *     component order) and u_sel [P] (inverse CDF of k / sum k, standing in for multinomial)
 *   throughput[i] = clamp(spectrum_sel, 1e-10) * throughput[i]; active[i] &= any(throughput > 0)
 *   rays_out[i] = [p, from_local(frame(n), wo_sel)]  (inactive rays: [p, (0,0,1)])
 * The caller intersects rays_out (primary = 0) and clears active where it missed.  sdf may be
 * NULL when shadow == 0.  workspace: nrt_path_workspace_bytes(P). */
size_t nrt_path_workspace_bytes(int64_t P);
int nrt_path_bounce(const nrt_bsdf* bsdf, const nrt_light* light, const nrt_sdf* sdf,
                    int32_t shadow, const nrt_mlp* occ, int32_t max_steps, float epsilon,
                    const float* p, const float* n, const float* wi, int64_t P, uint8_t* active,
                    float* throughput, float* result, const float* u_comp, const float* u_sel,
                    float* rays_out, void* workspace, int precision, void* stream);

/* ---------------------------------------------------------------------------------------
 * Cameras (cameras/cameras.py) and the tile composite (main.py:85-90, integrators.py:251)
 * ------------------------------------------------------------------------------------- */
#define NRT_CAM_NERF 0   /* NeRFCamera.sample_positions (cameras.py:23-54)                   */
#define NRT_CAM_DTU 1    /* DTUCamera.sample_positions + lift (cameras.py:132-192)           */
#define NRT_CAM_FOV 2    /* FoVPerspectiveCameras.sample_positions (renderer/cameras.py:539)  */

typedef struct {
  int32_t kind;
  int32_t size;            /* `size` argument of pathtrace                                  */
  float focal;             /* NERF                                                          */
  float mat[16];           /* NERF: c2w [3,4] row-major; DTU: pose [4,4];                   */
                           /* FOV: inverse full-projection [4,4] (row-vector convention)    */
  float intrinsic[16];     /* DTU: K [4,4]                                                  */
  float origin[3];         /* FOV: camera centre                                            */
} nrt_camera;

/* rays[(n*W + x)*H + y][6] for tile rows x in [x0, x0+W), cols y in [y0, y0+H) of camera n.
 * Pixel (x, y) uses u = y0+y, v = x0+x (main.py:71 stacks [gy, gx]) unless `positions`
 * ([W, H, 2] device, (u, v) per pixel, the reference's position_samples) is given.
 * noise (device, uniforms in [0,1), NULL = none; with_noise is the jitter amplitude):
 *   NERF: [2, W, H] -- u plane then v plane (two rand_like draws, cameras.py:35-36);
 *   FOV:  [W, H, 2] -- interleaved (one sampler draw, renderer/cameras.py:553-555);
 *   DTU ignores it (cameras.py:156-192 never reads with_noise). */
int nrt_raygen(const nrt_camera* host_cams, int32_t N, int32_t x0, int32_t y0, int32_t W,
               int32_t H, float with_noise, const float* noise, const float* positions,
               float* rays, void* stream);

/* SurfaceInteraction.set_normals + to_local(-d) (interaction.py:73-78, sdfs.py:158-159):
 * frame[P,9] = coordinate_system(n) as [s | t | n] columns (row-major 3x3, may be NULL) and
 * wi[P,3] = to_local(frame, -d) (may be NULL). */
/* Sphere (shapes/shapes.py:31-97): the analytic ray / sphere hit in the reference's float32 op
 * order (quad_solve :11-18; nearest root >= 1e-8; p = o + t d + 1e-5 n, n = normalize(p - c)).
 * center: 3 host floats; radius: the python float (sqr_radius = radius^2 in double, then f32).  Optional outputs (NULL = skip): t, hit, p, n (needs p), upper = the far
 * root (intersect_limits, :78-91), hit_idx + hit_count (compacted hit list, count zeroed here).
 * intersect_test (:70-77) is the hit output alone. */
int nrt_sphere_intersect(const float* center, double radius, const float* rays, int64_t P,
                         float* t, uint8_t* hit, float* p, float* n, float* upper,
                         int32_t* hit_idx, int32_t* hit_count, void* stream);
/* SphereCloud (shapes/shapes.py:99-206): the nearest hit over N spheres per ray.  spheres:
 * device [N][4] floats (centre x, y, z, radius).  split_n, t_max: intersect's arguments (the
 * chunk of spheres per pass; a root counts when in [1e-8, t_max), the best distance starts at
 * t_max).  Outputs as nrt_sphere_intersect's (NULL = skip; hit is intersect_test's answer).  The
 * reference's own broadcasting is well-formed for one sphere, where the results are its bit for
 * bit; more spheres follow the same per-ray statements (the nearest sphere's index within its
 * chunk of split_n names the normal's centre, as the reference keeps it). */
int nrt_sphere_cloud_intersect(const float* spheres, int64_t N, int64_t split_n, double t_max,
                               const float* rays, int64_t P, float* t, uint8_t* hit, float* p,
                               float* n, int32_t* hit_idx, int32_t* hit_count, void* stream);
int nrt_frames(const float* rays, const float* n, int64_t P, float* frame, float* wi,
               void* stream);

/* image[n, X0+x, Y0+y, :] for the tile = rgb (3 ch) and, when alpha_from_throughput,
 * sigmoid(throughput) as the 4th channel (NeRFIntegrator, integrators.py:249-257); pixels
 * whose hit==0 take `background` when fill_misses (main.py:88-89).  img_w, img_h, channels
 * describe the destination [N, img_w, img_h, channels] float32 image. */
int nrt_composite(const float* rgb, const float* throughput, const uint8_t* hit, int32_t N,
                  int32_t W, int32_t H, int32_t alpha_from_throughput, int32_t fill_misses,
                  float background, float* image, int32_t img_w, int32_t img_h,
                  int32_t channels, int32_t X0, int32_t Y0, void* stream);

/* One fused pathtrace tile (main.py:63-90) of Direct / NeRFIntegrator(Direct) (integrators.py:
 * 156-206, 243-257) in one call: nrt_raygen -> nrt_sdf_intersect (march, coarse scan when
 * params->primary, normals) -> nrt_shade_direct -> nrt_composite into image[N, img_w, img_h,
 * channels] at (X0, Y0).  noise: the camera's uniforms as nrt_raygen takes them (NULL: no
 * jitter); with_alpha = 1 (NeRFIntegrator: channels 4, alpha = sigmoid(throughput), misses kept)
 * or 0 (Direct: channels 3, misses = background).  workspace: nrt_render_tile_workspace_bytes
 * bytes of device memory (every intermediate; nothing is allocated).  The same launches as the
 * Python chain render.render_tile, so the results are bit-identical. */
size_t nrt_render_tile_workspace_bytes(const nrt_sdf* sdf, int32_t N, int32_t W, int32_t H);
int nrt_render_tile(const nrt_camera* host_cams, int32_t N, int32_t x0, int32_t y0, int32_t W,
                    int32_t H, float with_noise, const float* noise, const nrt_sdf* sdf,
                    const nrt_march_params* params, const nrt_bsdf* bsdf, const nrt_light* light,
                    int32_t with_alpha, float background, float* image, int32_t img_w,
                    int32_t img_h, int32_t channels, int32_t X0, int32_t Y0, void* workspace,
                    void* stream);

/* ---------------------------------------------------------------------------------------
 * NeRFLE (shapes/nerf.py:153-214), driven by NeRFReproduce.sample (integrators.py:260-267):
 * for each ray and each depth ts[s] (the caller's linspace(0, 2 + random()*0.1, S)),
 * first = MLP_5x128(o + ts[s] d) -> (alpha_raw, latent[64]),
 * rgb_s = sigmoid(MLP_8x64([latent, d, light])), composited with the reference's weights
 * (alpha = 1 - exp(-relu(alpha_raw) t), rolled cumprod with the last entry 1).
 * light[light_dim] (device) is the point light's location (envmap=False, light_dim 3) or
 * its envmap encoding from nrt_light_envmap (envmap=True, light_dim 3 bins^2).
 * first: 3 -> 65, second: (67 + light_dim) -> 3.  ts[S] device; rgb [P,3].  FP16 with the
 * default shapes runs the fused k_nerfle16 kernel -- for the envmap too: the envmap is one
 * constant per call, so its share of the colour MLP's input (W[:, env] env in the init and skip
 * layers, env B[env, :] in the Fourier projection) is folded into one constant input column of
 * the kernel's 70-input program, rebuilt when the envmap changes (one 4 light_dim-byte read-back
 * and a stream synchronisation per call).
 * workspace: nrt_nerfle_workspace_bytes(P, S, light_dim) bytes of device memory.
 * ------------------------------------------------------------------------------------- */
size_t nrt_nerfle_workspace_bytes(int64_t P, int32_t S, int32_t light_dim);
/* The workspace the call with these MLPs and precision actually needs: 16 B per sample on the
 * fused FP16 kernel (alpha_raw + rgb_raw), nrt_nerfle_workspace_bytes otherwise (the unfused
 * path's [P S, 65 / 70] intermediates) -- so a caller chunks by the path that runs. */
size_t nrt_nerfle_workspace_bytes_for(const nrt_mlp* first, const nrt_mlp* second, int64_t P,
                                      int32_t S, int32_t light_dim, int32_t precision);
int nrt_nerfle_forward(const nrt_mlp* first, const nrt_mlp* second, const float* rays, int64_t P,
                       const float* ts, int32_t S, const float* light, int32_t light_dim,
                       float* rgb, void* workspace, int precision, void* stream);

/* PlainNeRF (shapes/nerf.py:9-74; replaces PlainNeRF.forward, nerf.py:46-74): per ray and depth
 * ts[s] (the caller's linspace(0.4, 2 + random()*0.1, S)),
 *   first_out = first(o + ts[s] d, latent[row])            (3 + latent L -> 1 + I)
 *   rgb_s = tanh(second(dir_to_elev_azim(d), [first_out[1:], latent[row]]))   (2 + (I+L) -> 3)
 *   sigma = relu(first_out[0] + noise[s * P + p])           (noise NULL: none; the reference
 *                                                              draws randn * 1e-3, nerf.py:66)
 * composited with the NeRFLE weights, rgb[p] = (sum_s w_s rgb_s + 1) / 2.  latent is [rows, L]
 * device memory; ray p uses row p / rays_per_latent (the reference's latent[None, :, None, None,
 * None] indexes the camera axis of [N, W, H, B] rays: rays_per_latent = W*H*B).
 * workspace: nrt_plain_nerf_workspace_bytes(first, second, P, S) bytes. */
size_t nrt_plain_nerf_workspace_bytes(const nrt_mlp* first, const nrt_mlp* second, int64_t P,
                                      int32_t S);
int nrt_plain_nerf_forward(const nrt_mlp* first, const nrt_mlp* second, const float* rays,
                           int64_t P, const float* ts, int32_t S, const float* latent,
                           int64_t rays_per_latent, const float* noise, float* rgb,
                           void* workspace, int precision, void* stream);

/* NeRFLE's envmap light encoding (nerf.py:183-191): PointLights.envmap (lights.py:81-88) at
 * elev_azim_to_dir (utils.py:478-486) of meshgrid(linspace(0, 180, bins), linspace(0, 45, bins))
 * -> out[bins^2 * 3] (device).  Point lights only (NRT_EUNSUPPORTED otherwise). */
int nrt_light_envmap(const nrt_light* light, int32_t bins, float* out, void* stream);

/* ---------------------------------------------------------------------------------------
 * Kernel timing (bench / profiling aid; no reference counterpart)
 * When enabled, the heavy launches (k_intersect, k_sdf_grad, k_shade_direct, k_mlp_forward)
 * are bracketed by hipEvents on the stream they run on.  nrt_profile_read synchronises those
 * events and returns the summed duration and launch count of kernel `name`.
 * ------------------------------------------------------------------------------------- */
#define NRT_PROF_TIMING 1 /* hipEvents around the profiled launches */
#define NRT_PROF_EVALS 2  /* count the ring marches' SDF evaluations (one device atomic per
                             wave-evaluation: enable it in an untimed pass only) */
void nrt_profile_enable(int flags);
void nrt_profile_reset(void);
int nrt_profile_read(const char* name, double* total_ms, int64_t* launches);
/* SDF evaluations (ray x point) the ring marches (k_march16 / k_scan_best16 / k_march32 /
 * k_scan_best32) executed while NRT_PROF_EVALS was enabled, since the last nrt_profile_reset: the
 * executed work behind the algorithmic count (every ray at every march step and scan point,
 * sdfs.py:119-131, 232-249), which the lane-level job lists lower.  Synchronises. */
int nrt_profile_evals(uint64_t* evals);
/* Rays the NRT_MIXED refinement re-marched on the split engine (the flagged rays, nrt_ring_mixed
 * step 2) while NRT_PROF_EVALS was enabled, since the last nrt_profile_reset.  Synchronises. */
int nrt_profile_refined(uint64_t* rays);
/* Algorithmic FLOP of the timed launches of kernel `name` since the last nrt_profile_reset, as
 * the entries that launch it count them (the MLP backward and weight-gradient launches of the
 * training path: every multiply-add of the layers' products at their real widths, 2 FLOP each);
 * 0 for launches that record none.  With nrt_profile_read's time it gives a roofline fraction. */
int nrt_profile_flop(const char* name, double* flop);

/* ---------------------------------------------------------------------------------------
 * Runtime options (no reference counterpart: the reference has one eager implementation).
 * Process-wide, read when a call launches its kernels; the library reads no environment
 * variables.  Each option selects between implementations that the parity tests hold to the
 * same oracle bar, or sets a schedule that does not change results:
 *   "ring16"        1  FP16 SDF march / normals on the LDS-ring engine (0: per-wave kernels)
 *   "ring32"        1  FP32 SDF march on the FP32 ring engine k_march32 (0: per-wave k_intersect)
 *   "normals16"     1  after an FP16 ring march, normals by FP16 forward mode (k_normal16);
 *                      0: the FP32 backward (k_sdf_grad) -- FP32-accurate normals
 *   "scan_best32"   1  FP16 primary march: the throughput -1000 sdf(best) (sdfs.py:137, 249) is
 *                      evaluated by the FP32 engine (k_scan_best32) at the FP16 scan's argmin;
 *                      0: by the FP16 engine (k_scan_best16) -- the x1000 logit amplifies FP16
 *                      SDF error into alpha
 *   "march_blocks"  0  persistent-grid size of the ring marches (0: every resident slot);
 *                      results are bit-identical for every value
 *   "shade_program" 1  FP16 shading MLPs in one fused program kernel (0: per component)
 *   "nerf_fused"    1  FP16 NeRFLE in the fused k_nerfle16 (0: separate MLP launches)
 *   "max_waves"     0  waves per block (1..4) of the per-wave kernels (0: 4)
 *   "shade_ring"    1  FP32 / fp32-split shading MLPs (LightField 10x256, spatial weights 16x256,
 *                      NeuralBSDF 6x96) on the row-program ring kernels k_light32 / k_bsdf32 and
 *                      k_light3 / k_bsdf3 (0: the per-wave k_shade_direct)
 *   "normals_ring"  1  after an FP32 / fp32-split ring march, normals by forward mode on the same
 *                      engine (k_normal32 / k_normal3; 0: the per-wave FP32 backward k_sdf_grad)
 *   "xcd_lines"     0  1: ring marches deal rays to waves XCD by XCD (each 32-ray line of the
 *                      outputs stored by waves of one XCD); measured: more HBM write traffic
 *                      than the plain strided deal (0), kept for A/B runs; bit-identical results
 *   "mixed_refine_d" 20000 NRT_MIXED: a ray is marched again at FP32 accuracy when one of its
 *                      FP16 steps lies within d * (1 + step/16) of eps (or its next t of max_t);
 *                      1e-7 units (the FP16 SDF error of the headline scene is <= 7.3e-5; slowly
 *                      converging rays need the larger bound)
 *   "mixed_restart"  1  1: a flagged ray marches again from t = 0; 0: it resumes at the flagged
 *                      step (cheaper, but keeps the FP16 drift of t: measured 1,464 step flips);
 *                      2: at its first step within "mixed_zone" of a surface (zone 0.2: 18 step
 *                      flips for 2.5 ms less; kept for A/B)
 *   "mixed_zone"     500000  restart 2's zone, 1e-7 units
 *   "bwd_colsplit"   1  nrt_mlp_backward(_multi): 1 = the column-split kernels (a block of one
 *                      wave per 32-column row block on the same 32 rows; the encoding in global
 *                      tiles where that doubles the blocks per CU), 2 = the same with the encoding
 *                      in the LDS slab unless fewer than two blocks fit, 0 = one wave per 32 rows
 *                      (round 3).  Gradients bit-equal across values.  nrt_mlp_grad_backward
 *                      follows the option too: any nonzero value selects its column-split
 *                      kernel (k_mlp_grad_backward32_cs, the slab in LDS; 1 and 2 run the same
 *                      kernel there), 0 the per-wave kernel.
 *   "bwd_ring"       1  nrt_mlp_backward(_multi) of the shading MLPs' shapes (LightField 10x256
 *                      F=16, spatial weights 16x256 F=128, NeuralBSDF 6x96 F=64: leaky_relu, 3
 *                      inputs, no latent) on the FP32 ring engine (16-row tiles, the weights and
 *                      the transposed weights streamed through a block-shared LDS ring, dZ kept in
 *                      registers between layers); 0: the bwd_colsplit kernels.  Same gradients to
 *                      FP32 rounding (different summation order), both held to float64 autograd
 *   "wgrad_tile"     0  1: weight gradients (every backward) on k_wgrad_tile -- 128 x 128 output
 *                      tiles of four waves, the batch rows staged through LDS (operands read twice
 *                      per layer), each layer's bias summed from the staged dZ -- instead of
 *                      k_wgrad_batch (64 x 64 tiles fed by direct loads); measured 10 % slower on
 *                      the training step (1.06 vs 0.96 ms a launch: MFMA busy 0.36 vs 0.51, 32 % of
 *                      wave time parked at the stage barriers).  Deterministic either way; the two
 *                      differ by the split-K slice count (FP32 summation order)
 *   "train_save"     1  nrt_mlp_save_bytes > 0 for the ring backward's shapes (the training
 *                      forward saves its activations, nrt_mlp_backward_saved skips the forward
 *                      evaluation); 0: nrt_mlp_save_bytes returns 0 (the backward recomputes)
 *   "mixed_drift"    0  1: the flag bound is d * (1 + a per-ray drift estimate built from the
 *                      ratio of consecutive step values) instead of d * (1 + step/16); measured
 *                      to flag more rays for the same accuracy (152 vs 133 ms), kept for A/B
 *   "ring_occlusion" 1  shadow rays (nrt_sdf_occlusion, the shadowed shading entries) march on
 *                      the ring engine of the precision (k_occl16 / k_occl32 / k_occl3); 0: the
 *                      per-wave k_occlusion; same visibility bar either way
 *   "mixed_refine_s" 2000 NRT_MIXED: sdf(best) re-evaluates the scan's runner-up when the FP16
 *                      minimum and runner-up lie within s (1e-7 units)
 *   "march_queue"    2  nrt_sdf_intersect's ring marches: 1 = one launch-wide job queue (waves
 *                      take 16 jobs at a time from [every ray's march][every ray's scan
 *                      segments] through a device counter) instead of per-wave job lists, 0 =
 *                      the lists, 2 = the queue for batches of >= 131,072 rays (64 a resident
 *                      wave; the 800^2 frame 1 % faster, the 38,400-ray training march 1-5 %
 *                      slower on it); same results (a ray's values do not depend on the schedule)
 *   "march_stage"    1  under the launch queue, the plain ring marches (k_march32 / k_march16 /
 *                      k_march3) stage each wave's finished packed t and whole-scan keys in LDS
 *                      per 16-ray line and write whole lines (fewer, coalesced write requests);
 *                      0: one 4- / 8-byte store per ray; the same words either way
 * nrt_set_option returns NRT_EINVAL for an unknown name or a negative value.
 * ------------------------------------------------------------------------------------- */
int nrt_set_option(const char* name, int64_t value);
int nrt_get_option(const char* name, int64_t* value);
/* every option back to its default */
int nrt_reset_options(void);

#ifdef __cplusplus
}
#endif
#endif /* NRT_H_ */
