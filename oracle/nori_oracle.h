/*
 * nori_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's `path_mis` hot path (rogerbarton/optix-renderer,
 * Nori). Used exclusively by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg, as the checker / reported CPU baseline -- never by the product
 * path (optix-renderer_amd/), which must fail loudly without its HIP library.
 *
 * Pinning: the reference cannot be compiled in this image (include/nori/common.h
 * needs IlmBase's ImathPlatform.h; src/utils/bvh.cpp and block.cpp need TBB headers;
 * none are present and stand-in headers are not allowed), so this restatement is
 * pinned by the reference's own fixtures: the pcg32 known-answer output
 * (ext/pcg32/pcg32-demo.out, also regenerated from the reference's pcg32-demo.cpp
 * into oracle/_ref/), the scene t-tests scenes/pa4/tests/test-{furnace,direct}.xml,
 * the BSDF t-test scenes/pa3/tests/ttest-microfacet.xml and the chi^2 test
 * scenes/pa3/tests/chi2test-microfacet.xml. See DESIGN.md "Oracle".
 */
#ifndef NORI_ORACLE_H
#define NORI_ORACLE_H

#include <stdint.h>

#include "nori_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct no_scene no_scene;

enum { NO_SAMPLER_PER_PATH = 0, NO_SAMPLER_NORI_BLOCK = 1 };
/* or'ed into no_render's sampler_mode: depth-of-field lens samples drawn from one sequential stream inside the
 * serial render loop, literally as the reference's single-thread render does (perspective.cpp:118-122); requires
 * blocks == NULL, n_threads == 1, s0 == 0. Without it each ray's lens sample is reached by pcg32::advance. */
enum { NO_RENDER_LENS_SERIAL = 0x100 };

/* copies the scene and builds the BVH with a serial restatement of BVH::build */
int no_scene_create(const nh_scene_desc *desc, no_scene **out);
void no_scene_free(no_scene *s);
/* export the oracle's BVH (reference layout) for comparison with the product builder */
int no_bvh_info(const no_scene *s, uint32_t *n_nodes, uint32_t *n_indices);
/* the oracle's own EnvMap::calculateProbs CDF (W*H+1 entries) and normalization */
int no_env_cdf(const no_scene *s, const float **cdf, uint32_t *n, float *normalization);
int no_bvh_export(const no_scene *s, nh_bvh_node *nodes, uint32_t *indices);

/* the oracle's restated Eigen arithmetic on n cases of 36 floats (oracle/eigen_probe.cpp layout) -> 28 floats
   each, for the bit-for-bit comparison with the reference's Eigen */
int no_eigen_ops(int32_t n, const float *in, float *out);
/* the oracle's normal-map arithmetic on n cases of 13 floats (s3 t3 n3 v3 intensity, oracle/normalmap_probe.cpp "ops"
   layout) -> 15 floats each: normalize(TBN * v) (mesh.cpp:176-182), the sphere's re-derived frame n', t', b'
   (sphere.cpp:117-120) and PNGTexture::eval's normal-map blend of v (PNGTexture.cpp:155-161) */
int no_normal_ops(int32_t n, const float *in, float *out);

/* SimpleDenoiser::denoise (src/denoiser/simple.cpp:29-76) in place on an (W+2b)(H+2b)x4 RGBW ImageBlock,
   serial row-major order (the reference with one thread) */
int no_denoise_simple(float *rgbw, int32_t width, int32_t height, int32_t border, const nh_denoiser *p);

/* BVH::rayIntersect over a ray batch (closest or any hit) */
int no_trace_rays(const no_scene *s, const nh_ray_soa *rays, int32_t n, int32_t any_hit, nh_hit_soa *out);

/* pcg32 restatement: seed / next for KAT tests */
void no_pcg32_seed(uint64_t *state, uint64_t *inc, uint64_t initstate, uint64_t initseq);
uint32_t no_pcg32_next(uint64_t *state, uint64_t *inc);
/* the per-(pixel, sample) seeding contract used by the GPU path */
void no_path_seed(uint64_t seed, uint64_t pixel_index, uint64_t sample_index, uint64_t *state, uint64_t *inc);

/* render sample rounds [s0, s1) into an (W+2b)(H+2b)x4 RGBW master block (accumulating).
 * blocks: optional list of 32x32 block ids to render (NULL = all). Per-path sampler mode
 * accepts any round range; NORI_BLOCK mode requires s0 == 0 (per-block streams persist
 * across rounds, render.cpp:315-320). n_threads >= 1. Returns invalid-sample count in
 * *n_invalid (may be NULL). */
int no_render(const no_scene *s, int32_t sampler_mode, uint64_t seed, int32_t s0, int32_t s1,
              const int32_t *blocks, int32_t n_blocks, int32_t n_threads, float *rgbw, uint64_t *n_invalid);

/* one camera path under the per-path contract: radiance and pixel jitter */
int no_path_radiance(const no_scene *s, uint64_t seed, int32_t px, int32_t py, int32_t sample, float *rgb3,
                     float *jitter2);

/* StudentsTTest scene branch (src/utils/ttest.cpp:191-240): n paths from a sequential
 * pcg32 stream (state/inc in/out, default-constructed = PCG32_DEFAULT_*). Returns
 * Welford mean/variance of the luminance. */
int no_ttest_scene(const no_scene *s, uint64_t *state, uint64_t *inc, int32_t n, double *mean, double *variance);
/* StudentsTTest BSDF branch (ttest.cpp:147-190) */
int no_ttest_bsdf(const nh_bsdf *b, float angle_deg, uint64_t *state, uint64_t *inc, int32_t n, double *mean,
                  double *variance);
/* BSDF sample/pdf for the chi^2 test: wi local, sample 2D -> wo, weight, pdf(wo) */
int no_bsdf_sample(const nh_bsdf *b, const float *wi, const float *sample, float *wo, float *weight3,
                   float *pdf, int32_t *measure);
float no_bsdf_pdf(const nh_bsdf *b, const float *wi, const float *wo);
/* Texture<Color3f>::eval of the scene's albedo texture `texture` (1-based, nh_bsdf.albedo_texture) at n uv
 * pairs: rgb = 3n floats */
int no_texture_eval(const no_scene *s, uint32_t texture, int32_t n, const float *u, const float *v, float *rgb);
int no_bsdf_pdf_batch(const nh_bsdf *b, const float *wi, int32_t n, const float *wo, float *out);
/* ChiSquareTest histogram (src/utils/chi2test.cpp:150-170), rng state in/out */
int no_chi2_histogram(const nh_bsdf *b, const float *wi, uint64_t *state, uint64_t *inc, int32_t n, int32_t res_theta,
                      int32_t res_phi, double *obs);

#ifdef __cplusplus
}
#endif
#endif
