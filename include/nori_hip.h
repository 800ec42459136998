/*
 * nori_hip.h -- C-ABI boundary of the MI355X-native Nori `path_mis` hot path.
 *
 * Everything crossing this boundary is plain C: PODs, pointers and sizes. No
 * C++ types, no exceptions, no torch types. Every call returns an int status
 * (NH_OK == 0); the message of the last failure on a context is available via
 * nh_last_error(), and for the context-free host calls via nh_host_last_error().
 *
 * What each entry point replaces in the reference (rogerbarton/optix-renderer,
 * paths relative to the reference root):
 *
 *   nh_scene_load_xml     loadFromXML + Scene::cloneAndInit/update
 *                         (src/utils/parser.cpp:28-378, src/utils/scene.cpp:59-202)
 *   nh_bvh_build          BVH::build (src/utils/bvh.cpp:54-380)
 *   nh_create/nh_destroy  OptixState context creation (include/nori/optix/OptixState.cpp:39-74)
 *   nh_upload_scene       OptixState::preRender scene/SBT upload
 *                         (include/nori/optix/OptixState.render.cpp:19-85, OptixState.cpp:344-411)
 *   nh_upload_bvh         OptixState GAS/IAS build (include/nori/optix/OptixState.as.cpp:47-248)
 *   nh_trace_rays         BVH::rayIntersect / Scene::rayIntersect
 *                         (src/utils/bvh.cpp:402-460, include/nori/scene.h:114-137)
 *   nh_render             RenderThread::renderThreadMain sample loop + renderBlock + PathMISIntegrator::Li
 *                         (src/utils/render.cpp:281-347, :421-459; src/integrators/path_mis.cpp:16-150)
 *                         and the OptiX subframe launch (include/nori/optix/OptixState.cpp:485-510)
 *   nh_get_framebuffer    ImageBlock master (src/utils/block.cpp:38-134); toBitmap is nh_framebuffer_to_rgb
 *   nh_reduce_framebuffers  (new) RCCL sum of per-GPU RGBW framebuffers over xGMI
 *   nh_denoise            Denoiser::denoise on the master ImageBlock after the render loop
 *                         (src/utils/render.cpp:368-369): SimpleDenoiser (src/denoiser/simple.cpp:29-76,
 *                         computeVarianceFromImage src/utils/common.cpp:339-398); the GPU counterpart of
 *                         OptixState::denoise (include/nori/optix/OptixState.denoiser.cpp:123-150)
 *
 * Conventions (mirroring the reference's threading contract):
 *   - input pointers are host-owned and only read during the call;
 *   - calls on one nh_ctx are serialised by the caller; distinct contexts may be
 *     driven from distinct host threads (one per GPU).
 */
#ifndef NORI_HIP_H
#define NORI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NH_OK 0
#define NH_ERR_INVALID 1
#define NH_ERR_IO 2
#define NH_ERR_DEVICE 3
#define NH_ERR_UNSUPPORTED 4
#define NH_ERR_STATE 5

/* ---- scene description (flattened Nori scene graph) --------------------- */

enum { NH_SHAPE_MESH = 0, NH_SHAPE_SPHERE = 1 };
enum { NH_BSDF_DIFFUSE = 0, NH_BSDF_MIRROR = 1, NH_BSDF_DIELECTRIC = 2, NH_BSDF_MICROFACET = 3 };
enum { NH_EMITTER_AREA = 0, NH_EMITTER_POINT = 1, NH_EMITTER_ENVMAP = 2 };
/* path_mis (src/integrators/path_mis.cpp), path_mats (path_mats.cpp), the single-bounce
 * direct_ems / direct_mats / direct_mis (direct_ems.cpp, direct_mats.cpp, direct_mis.cpp), the
 * point-light `direct` integrator (direct.cpp, scenes/pa1) and the `normals` integrator of the normal-map scenes
 * (normals.cpp: |shFrame.toWorld(direction)|, the envmap on a miss) */
enum { NH_INTEGRATOR_PATH_MIS = 0, NH_INTEGRATOR_PATH_MATS = 1, NH_INTEGRATOR_DIRECT_EMS = 2,
       NH_INTEGRATOR_DIRECT_MATS = 3, NH_INTEGRATOR_DIRECT_MIS = 4, NH_INTEGRATOR_DIRECT = 5,
       NH_INTEGRATOR_NORMALS = 6 };

/* One Nori Shape (src/shapes/mesh.cpp, src/shapes/sphere.cpp). Mesh data lives in
 * the scene-wide concatenated arrays at the given offsets. */
typedef struct nh_shape {
    int32_t type;            /* NH_SHAPE_* */
    int32_t bsdf;            /* index into nh_scene_desc.bsdfs (every shape has one; default diffuse 0.5) */
    int32_t emitter;         /* index into nh_scene_desc.emitters, or -1 */
    uint32_t v_offset;       /* first vertex in V/N/UV/T/BT */
    uint32_t n_vertices;
    uint32_t f_offset;       /* first face in F (face indices are local to the shape) */
    uint32_t n_faces;
    int32_t has_normals;     /* N present (per vertex) */
    int32_t has_uvs;         /* UV present (per vertex); tangents T/BT present iff both */
    float center[3];         /* sphere */
    float radius;            /* sphere */
    float bbox_min[3];       /* Shape::getBoundingBox() */
    float bbox_max[3];
    uint32_t pdf_offset;     /* mesh area DiscretePDF: n_faces+1 CDF entries in area_cdf */
    float pdf_normalization; /* DiscretePDF::getNormalization() = 1/sum(area) */
    uint32_t normal_map;     /* 1 + index into nh_scene_desc.textures of the shape's <texture name="normal"> child
                                (Shape::addChild, src/shapes/shape.cpp:138-147), 0 = none. It perturbs the shading
                                frame: meshes with normals and uvs take normalize(TBN * eval(uv)) (mesh.cpp:165-185),
                                spheres re-derive their frame from shFrame.toWorld(eval(uv)) (sphere.cpp:115-121) */
} nh_shape;

/* One Nori BSDF (src/bsdf/{diffuse,mirror,dielectric,microfacet}.cpp). */
typedef struct nh_bsdf {
    int32_t type;            /* NH_BSDF_* */
    float albedo[3];         /* diffuse: constant albedo texture */
    float alpha;             /* microfacet: Beckmann roughness */
    float int_ior, ext_ior;  /* dielectric / microfacet */
    float kd[3];             /* microfacet diffuse base */
    float ks;                /* microfacet: 1 - max(kd) */
    uint32_t albedo_texture; /* diffuse: 1 + index into nh_scene_desc.textures of its Texture<Color3f> albedo
                                child (diffuse.cpp:70-91); 0 = the constant albedo above */
} nh_bsdf;

/* A Texture<Color3f> child of a BSDF, evaluated at the hit's uv (Intersection::uv, BSDFQueryRecord::uv):
 *   NH_TEXTURE_CONSTANT     ConstantTexture (src/textures/consttexture.cpp): value1
 *   NH_TEXTURE_CHECKERBOARD Checkerboard<Color3f> (src/textures/checkerboard.cpp:29-47): value1 / value2 by the
 *                           parity of the cell of uv / scale - delta
 *   NH_TEXTURE_PNG          PNGTexture (src/textures/PNGTexture.cpp:125-160): nearest texel of an sRGB-decoded RGBA
 *                           image (row 0 of the PNG first) at texel_offset in nh_scene_desc.texels; with
 *                           linear = 1 (sRGB = false, the default for a texture named "normal", PNGTexture.cpp:26)
 *                           the texels hold the normal-map decode of loadFromFile (x / 255 * 2 - 1 with every third
 *                           float of the RGBA array normalized as a Vector3f, PNGTexture.cpp:85-95) and eval blends
 *                           the texel by intensity and normalizes it (:155-161) */
enum { NH_TEXTURE_CONSTANT = 0, NH_TEXTURE_CHECKERBOARD = 1, NH_TEXTURE_PNG = 2 };
typedef struct nh_texture {
    int32_t type;            /* NH_TEXTURE_* */
    float value1[3];         /* constant value / checkerboard value1 */
    float value2[3];         /* checkerboard value2 */
    float delta[2];          /* checkerboard Point2f delta */
    float scale[2];          /* checkerboard Vector2f scale */
    int32_t width, height;   /* png */
    uint64_t texel_offset;   /* png: first texel (4 floats) in nh_scene_desc.texels */
    float scale_u, scale_v;  /* png scaleU / scaleV */
    float offset_u, offset_v;/* png offsetU / offsetV (non-spherical lookups) */
    int32_t spherical;       /* png sphericalTexture */
    float rotation[9];       /* png spherical lookups: the eulerAngles rotation (PNGTexture.cpp:133-139), row-major;
                                identity for eulerAngles = 0 */
    int32_t linear;          /* png: sRGB = false (normal-map decode + eval's intensity blend and normalize) */
    float intensity;         /* png, linear: PNGTexture intensity [1] */
    int32_t pad;
} nh_texture;

/* One Nori Emitter (src/emitters/{arealight,pointlight}.cpp). */
typedef struct nh_emitter {
    int32_t type;            /* NH_EMITTER_* */
    int32_t shape;           /* area light: owning shape */
    float radiance[3];       /* area: radiance; point: power */
    float light_prob;        /* lightWeight (emitter DiscretePDF weight) */
    float position[3];       /* point light */
    float pad;
} nh_emitter;

/* PerspectiveCamera after update() (src/cameras/perspective.cpp:48-96). Row-major 4x4. */
typedef struct nh_camera {
    int32_t width, height;
    float sample_to_camera[16];
    float camera_to_world[16];
    float inv_output_size[2];
    float near_clip, far_clip;
    /* after cloneAndInit's fstop <-> lensRadius coupling (perspective.cpp:37-42). lens_radius > 1e-4 (Epsilon):
       thin lens (perspective.cpp:114-130); camera ray k of the serial render order (round, BlockGenerator
       spiral, x-major pixels) takes draws 2k, 2k+1 of a default-state pcg32 -- the reference's static sampler */
    float lens_radius, focal_distance;
    /* which of those two draws is the lens sample's x: Independent::next2D builds Point2f(nextFloat(), nextFloat())
       (independent.cpp:74-78), whose argument evaluation order C++ leaves unspecified. NH_LENS_DRAWS_RTL (the
       loader's default): x = draw 2k+1, y = draw 2k, as g++ compiles it (oracle/normalmap_probe.cpp "order");
       NH_LENS_DRAWS_LTR: x = draw 2k, as clang compiles it */
    int32_t lens_draw_order;
} nh_camera;
enum { NH_LENS_DRAWS_LTR = 0, NH_LENS_DRAWS_RTL = 1 };

/* Tabulated reconstruction filter as ImageBlock::init builds it (src/utils/block.cpp:54-70). */
typedef struct nh_filter {
    float radius;
    int32_t border;          /* ceil(radius - 0.5) */
    float lookup_factor;     /* NORI_FILTER_RESOLUTION / radius */
    float table[33];         /* NORI_FILTER_RESOLUTION + 1 entries, last = 0 */
} nh_filter;

/* EnvMap emitter (src/emitters/environmentmap.cpp) with its albedo texture: a png_texture
 * (src/textures/PNGTexture.cpp, sRGB-decoded RGBA floats, PNG row 0 first) or the constant 0.5
 * fallback as a 1x1 texture. */
typedef struct nh_envmap {
    int32_t width, height;        /* texture size (getWidth/getHeight); 1x1 for constant textures */
    const float *rgba;            /* width*height*4 floats (PNGTexture::data) */
    float radiance[3];            /* EnvMap radiance multiplier */
    float scale_u, scale_v;       /* PNGTexture scaleU/scaleV */
    float offset_u, offset_v;     /* PNGTexture offsetU/offsetV (non-spherical lookups) */
    int32_t spherical;            /* PNGTexture sphericalTexture */
    int32_t constant;             /* ConstantTexture: eval ignores uv */
    const float *cdf;             /* EnvMap::calculateProbs DiscretePDF: width*height+1 CDF entries */
    float normalization;          /* DiscretePDF::getNormalization() */
    float rotation[9];            /* spherical lookups: the png_texture's eulerAngles rotation (PNGTexture.cpp:133-139),
                                     row-major; identity for eulerAngles = 0 */
} nh_envmap;

/* <denoiser> of the scene (Scene::m_denoiser, src/utils/scene.cpp:242-245): SimpleDenoiser's parameters after
 * its constructor's clamps (src/denoiser/simple.cpp:15-24): sigma_d = clamp(sigma_d [0], Epsilon, 10),
 * sigma_vr = clamp(sigma_vr [0.6], Epsilon, 10), range = clamp(range [1], 0, 50), amount = clamp(amount [1], 1, 10) */
enum { NH_DENOISER_NONE = 0, NH_DENOISER_SIMPLE = 1 };
typedef struct nh_denoiser {
    int32_t type;            /* NH_DENOISER_* */
    float sigma_d;           /* spatial Gaussian sigma (pixels) */
    float sigma_vr;          /* range sigma of the variance-scaled L1 colour distance */
    int32_t range;           /* window half-size: (2 range + 1)^2 pixels */
    int32_t amount;          /* passes */
} nh_denoiser;

typedef struct nh_scene_desc {
    nh_camera camera;
    nh_filter filter;
    int32_t integrator;      /* NH_INTEGRATOR_* */
    int32_t sample_count;    /* sampler sampleCount */
    uint32_t n_shapes;
    const nh_shape *shapes;
    uint32_t n_bsdfs;
    const nh_bsdf *bsdfs;
    uint32_t n_emitters;
    const nh_emitter *emitters;
    const float *emitter_cdf;     /* Scene::emitterDpdf CDF, n_emitters+1 entries */
    int32_t envmap;               /* emitter index of the environment map, or -1 */
    uint32_t n_vertices;          /* total over all meshes */
    const float *V;               /* 3 floats per vertex */
    const float *N;               /* 3 per vertex (zeros for meshes without normals) */
    const float *UV;              /* 2 per vertex */
    const float *T;               /* 3 per vertex: accumulated tangents (mesh.cpp:165-190 uses normalised) */
    const float *BT;              /* 3 per vertex */
    uint32_t n_faces;
    const uint32_t *F;            /* 3 per face, local to the owning shape */
    uint32_t n_area_cdf;
    const float *area_cdf;        /* concatenated per-mesh area CDFs */
    nh_envmap env;                /* valid when envmap >= 0 */
    nh_denoiser denoiser;         /* type NH_DENOISER_NONE when the scene has none */
    uint32_t n_textures;          /* BSDF albedo textures (nh_bsdf.albedo_texture) */
    const nh_texture *textures;
    uint64_t n_texels;            /* RGBA texels of every png texture, 4 floats each */
    const float *texels;
    float normals_direction[3];   /* NH_INTEGRATOR_NORMALS: its `direction` point [0, 0, 1] (normals.cpp:10-12) */
} nh_scene_desc;

/* ---- BVH in the reference's own layout (include/nori/bvh.h:127-165) ---- */

/* 32-byte node: word0 = flag | (size_or_axis << 1), word1 = leaf start / right child. */
typedef struct nh_bvh_node {
    uint32_t word0;
    uint32_t word1;
    float bbox_min[3];
    float bbox_max[3];
} nh_bvh_node;

typedef struct nh_bvh_desc {
    uint32_t n_nodes;
    const nh_bvh_node *nodes;
    uint32_t n_indices;           /* == primitive count */
    const uint32_t *indices;      /* global primitive ids in leaf order */
    uint32_t n_shapes;
    const uint32_t *shape_offset; /* n_shapes+1 prefix sums of primitive counts (BVH::m_shapeOffset) */
    float bbox_min[3], bbox_max[3];
    uint32_t max_depth;           /* deepest node level (root = 0): bounds the traversal stack */
} nh_bvh_desc;

/* ---- ray batches for the traversal entry point -------------------------- */

typedef struct nh_ray_soa {
    const float *ox, *oy, *oz;
    const float *dx, *dy, *dz;
    const float *mint, *maxt;     /* Ray3f semantics: mint == 1e-4f triggers the adaptive epsilon */
} nh_ray_soa;

typedef struct nh_hit_soa {
    uint8_t *hit;                 /* 0/1 */
    float *t, *u, *v;             /* closest-hit only */
    uint32_t *prim;               /* global primitive id, closest-hit only */
    uint32_t *shape;              /* shape index, closest-hit only */
} nh_hit_soa;

/* ---- rendering ------------------------------------------------------------ */

enum { NH_MODE_MEGAKERNEL = 0, NH_MODE_WAVEFRONT = 1 };
/* Visit orders of BVH::rayIntersect (src/utils/bvh.cpp:402-460); all three return the reference's hit.
 *   REFERENCE  binary tree, left child first (the reference's order)
 *   ORDERED    binary tree, nearer child first
 *   WIDE       4-wide collapse of the same tree (same boxes), nearer child first; nh_render uses it
 *              for deep trees whenever the traversal is not REFERENCE */
enum { NH_TRAVERSAL_REFERENCE = 0, NH_TRAVERSAL_ORDERED = 1, NH_TRAVERSAL_WIDE = 2 };

typedef struct nh_render_req {
    int32_t sample_begin;         /* sample rounds [sample_begin, sample_end) */
    int32_t sample_end;
    uint64_t seed;                /* base of the per-(pixel, sample) pcg32 seeding contract */
    int32_t n_blocks;             /* number of 32x32 image blocks this context renders; 0 = all */
    const int32_t *blocks;        /* block ids (by*nbx+bx) when n_blocks > 0 */
    int32_t mode;                 /* NH_MODE_* */
    int32_t traversal;            /* NH_TRAVERSAL_* */
    int32_t clear;                /* zero the framebuffer first */
    int32_t collect_stats;        /* 1: count BVH nodes/prims visited (calibration, slower) */
} nh_render_req;

typedef struct nh_render_stats {
    double kernel_ms_path;        /* summed device time of the path-tracing kernel(s) */
    double kernel_ms_splat;       /* summed device time of the ImageBlock splat kernel */
    double kernel_ms_extend;      /* wavefront: closest-hit kernel */
    double kernel_ms_shadow;      /* wavefront: any-hit kernel */
    double kernel_ms_shade;       /* wavefront: shading kernels */
    uint64_t launches_path, launches_splat, launches_extend, launches_shadow, launches_shade;
    uint64_t samples;             /* camera samples traced */
    uint64_t ray_queries;         /* closest + any-hit queries (collect_stats) */
    uint64_t nodes_visited;       /* BVH inner-node pops (collect_stats) */
    uint64_t boxes_tested;        /* child boxes tested (collect_stats) */
    uint64_t prims_tested;        /* primitive intersection tests (collect_stats) */
    uint64_t invalid_samples;     /* ImageBlock::put drops (NaN/Inf/negative) */
    /* wavefront mode: the any-hit kernel's share of ray_queries / nodes_visited / boxes_tested /
       prims_tested (the rest is the extend kernel's) */
    uint64_t shadow_queries, shadow_nodes_visited, shadow_boxes_tested, shadow_prims_tested;
    /* wavefront mode, always counted (host side, from the queue counts): path-state bytes the
       shade kernels load + store, and the queue bytes of the extend / any-hit kernels */
    uint64_t shade_state_bytes, extend_queue_bytes, shadow_queue_bytes, paths_shaded;
    /* wavefront mode: the tail kernel that finishes the last few live paths of a chunk in place */
    double kernel_ms_tail;
    uint64_t launches_tail;
    /* bytes of one BVH node as counted in nodes_visited: 64 (binary tree) or 128 (the 4-wide
       collapse, NH_TRAVERSAL_WIDE), for the last render */
    uint64_t node_bytes;
    /* the tail kernel's share of ray_queries / nodes_visited / boxes_tested / prims_tested (closest
       + any hit), and of that its any-hit part (also counted in shadow_*), collect_stats only */
    uint64_t tail_queries, tail_nodes_visited, tail_boxes_tested, tail_prims_tested;
    uint64_t tail_shadow_queries, tail_shadow_nodes_visited, tail_shadow_boxes_tested, tail_shadow_prims_tested;
    /* 1 when the last wavefront render traversed an LDS copy of the BVH (scenes of a few KB): its node
       and primitive reads then come from LDS, not HBM */
    uint64_t lds_scene;
    /* 1 when the last wavefront render ran one fused bounce kernel per bounce (shade + any-hit +
       closest-hit, LDS-staged BVHs): its time is in kernel_ms_shade, extend/shadow times are 0 */
    uint64_t fused_bounce;
    /* RCCL communicator cliques created by nh_reduce_framebuffers with this context as root (a clique
       is reused while the same contexts reduce again) */
    uint64_t comm_inits;
    /* nh_denoise / nh_denoise_image: summed device time and kernel launches */
    double kernel_ms_denoise;
    uint64_t launches_denoise;
    /* wavefront chunks whose tail kernel ran on a tail slot's stream, decoupled from the chunk's path pool
       (RR-ahead pipeline with several pools: the pool took the next chunk meanwhile) */
    uint64_t tails_async;
    /* wavefront path pools the last render drove (NH_POOLS, else 2, or 3 for scenes with mirror / dielectric BSDFs) */
    uint64_t pools_active;
    /* 1 when the last wavefront render traced each bounce's closest-hit and any-hit queries in one persistent
       launch (deep BVHs, 4-wide tree): its time is in kernel_ms_extend, kernel_ms_shadow stays 0 */
    uint64_t trace_fused;
    /* RR-ahead tail kernel (wf_tail_rr), collect_stats only: cycles its lanes spent in the shade body, the light
       sample's any-hit query, the next closest hit and the next vertex's head (clock64, summed over lanes), the
       path-bounces it ran and its longest chain (bounces of one path) */
    uint64_t tail_cycles_body, tail_cycles_shadow, tail_cycles_closest, tail_cycles_head;
    uint64_t tail_bounces, tail_max_bounces;
    /* the same four phase sums and the path-bounce count for the bounces the tail's cooperative finish ran (a path
       carried by a 16-lane group once <= 4 remain in its wave): the latency of one bounce of the last chains */
    uint64_t tail_coop_cycles_body, tail_coop_cycles_shadow, tail_coop_cycles_closest, tail_coop_cycles_head;
    uint64_t tail_coop_bounces;
    /* RR-ahead bounce kernel (wf_bounce_rr), collect_stats only: cycles its lanes spent loading the path (state and
       the Intersection of its hit), in the body, the any-hit query, the closest hit, the head and ranking + storing
       the survivors (clock64, summed over lanes), and the path-bounces it ran */
    uint64_t bounce_cycles_load, bounce_cycles_body, bounce_cycles_shadow, bounce_cycles_closest, bounce_cycles_head;
    uint64_t bounce_cycles_store, bounce_bounces;
} nh_render_stats;

typedef struct nh_scene nh_scene;
typedef struct nh_bvh nh_bvh;
typedef struct nh_ctx nh_ctx;

/* host-side scene ingestion */
int nh_scene_load_xml(const char *path, nh_scene **out);
/* <test> roots (src/utils/ttest.cpp) hold several <scene>s: load the index-th one */
int nh_scene_load_xml_index(const char *path, int32_t index, nh_scene **out);
int nh_scene_get_desc(const nh_scene *scene, nh_scene_desc *out);
/* overrides used by benchmarks and tests (camera resize recomputes the projection) */
int nh_scene_set_resolution(nh_scene *scene, int32_t width, int32_t height);
int nh_scene_set_sample_count(nh_scene *scene, int32_t spp);
int nh_scene_set_bsdf(nh_scene *scene, uint32_t shape, const nh_bsdf *bsdf);
/* append a texture to the scene's texture table (png: texels = width*height*4 floats, copied); returns its
   index + 1 for nh_bsdf.albedo_texture, or 0 on error (nh_host_last_error) */
uint32_t nh_scene_add_texture(nh_scene *scene, const nh_texture *tex, const float *texels);
/* give a shape a normal map (Shape::addChild of a <texture name="normal">, src/shapes/shape.cpp:138-147):
   texture = a value nh_scene_add_texture returned, 0 removes it */
int nh_scene_set_normal_map(nh_scene *scene, uint32_t shape, uint32_t texture);
/* the thin-lens sample's draw order (nh_camera.lens_draw_order): NH_LENS_DRAWS_RTL or NH_LENS_DRAWS_LTR */
int nh_scene_set_lens_draw_order(nh_scene *scene, int32_t order);
/* PNGTexture::loadFromFile's byte -> float loop over lodepng's RGBA8 array (PNGTexture.cpp:78-95): srgb != 0
   InverseGammaCorrect(b / 255) per byte; srgb == 0 the normal-map decode b / 255 * 2 - 1 with every third float
   of the array normalized as an Eigen Vector3f (the triples run over RGBA data, so they straddle pixels -- the
   reference's behaviour, reproduced). out: n floats. */
int nh_texture_decode(const uint8_t *rgba8, uint64_t n, int32_t srgb, float *out);
int nh_scene_set_integrator(nh_scene *scene, int32_t integrator);
void nh_scene_free(nh_scene *scene);
const char *nh_host_last_error(void);
/* Parity hook for the loader's transform arithmetic (the Eigen operations of parser.cpp:308-360,
 * transform.h:73-86, transform.cpp:9-10 and perspective.cpp:68-95 as the product restates them). One
 * request line in the protocol of oracle/eigen_xform_probe.cpp (floats as 8-hex-digit bit patterns:
 * "inv", "xf", "cam", "pt", "vec", "nrm"); writes the reply floats to out and returns their count, or
 * -1 (nh_host_last_error) for a malformed request or too small a cap. */
int nh_debug_transform(const char *request, float *out, int32_t cap);

int nh_bvh_build(const nh_scene_desc *scene, int32_t n_threads, nh_bvh **out);
int nh_bvh_get_desc(const nh_bvh *bvh, nh_bvh_desc *out);
void nh_bvh_free(nh_bvh *bvh);

/* ImageBlock::toBitmap (src/utils/block.cpp:76-82): rgbw with border -> W*H*3 rgb */
int nh_framebuffer_to_rgb(const float *rgbw, int32_t width, int32_t height, int32_t border, float *rgb);
/* Bitmap::save equivalents: PFM (always available) and uncompressed OpenEXR */
int nh_write_pfm(const char *path, const float *rgb, int32_t width, int32_t height);
/* PNG decode as PNGTexture::loadFromFile's lodepng call (8-bit RGBA, row 0 first); rgba may be
   NULL (or cap too small) to query the size */
int nh_image_load_png(const char *path, uint8_t *rgba, size_t cap, int32_t *width, int32_t *height);
int nh_write_exr(const char *path, const float *rgb, int32_t width, int32_t height);
/* Bitmap::saveToLDR (src/utils/bitmap.cpp:122-140): sRGB gamma (GammaCorrect, :109-112), bytes
 * (uint8_t)Clamp(255 * v + 0.5, 0, 255) per channel, written as an 8-bit RGB PNG. nh_rgb_to_ldr
 * produces the bytes only (3 per pixel, row 0 first). */
int nh_rgb_to_ldr(const float *rgb, int32_t width, int32_t height, uint8_t *rgb8);
int nh_write_png(const char *path, const float *rgb, int32_t width, int32_t height);

/* device side */
int nh_get_device_count(int *n);
int nh_create(int device, nh_ctx **out);
void nh_destroy(nh_ctx *ctx);
int nh_upload_scene(nh_ctx *ctx, const nh_scene_desc *scene);
int nh_upload_bvh(nh_ctx *ctx, const nh_bvh_desc *bvh);
int nh_trace_rays(nh_ctx *ctx, const nh_ray_soa *rays, int32_t n, int32_t any_hit, int32_t traversal, nh_hit_soa *out);
int nh_render(nh_ctx *ctx, const nh_render_req *req);
int nh_synchronize(nh_ctx *ctx);
int nh_get_framebuffer(nh_ctx *ctx, float *rgbw, size_t n_floats);
/* device pointer of the (W+2b)(H+2b)x4 fp32 framebuffer, for collectives issued by the caller;
   completes every submitted render first (the wavefront pipeline advances only inside library calls) */
int nh_framebuffer_device_ptr(nh_ctx *ctx, void **dptr, size_t *n_floats);
int nh_get_stats(nh_ctx *ctx, nh_render_stats *out);
int nh_reset_stats(nh_ctx *ctx);
/* single-process multi-GPU: RCCL sum of the framebuffers of n contexts into ctxs[root] (n = 1 included:
   a one-rank reduce). The communicator clique is created on the first call for a set of contexts and
   reused by later calls with the same contexts in the same order; it is destroyed with the contexts. */
int nh_reduce_framebuffers(nh_ctx **ctxs, int32_t n, int32_t root);
/* SimpleDenoiser::denoise (src/denoiser/simple.cpp:29-76) in place on the context's master ImageBlock (its
   interior W x H pixels; the border is left as is), after completing every submitted render. The pixels are
   updated in the row-major order of the reference's loops -- a pixel reads the already denoised values of
   the pixels before it and the previous pass's values of the others -- which is what the reference computes
   with one TBB thread (with more, its rows race). params->type must be NH_DENOISER_SIMPLE, the other fields
   within the constructor's clamps. Finite framebuffer values are assumed (ImageBlock::put drops the others). */
int nh_denoise(nh_ctx *ctx, const nh_denoiser *params);
/* the same on a caller's host ImageBlock: (width + 2 border) x (height + 2 border) x 4 floats, in place */
int nh_denoise_image(nh_ctx *ctx, float *rgbw, int32_t width, int32_t height, int32_t border,
                     const nh_denoiser *params);
const char *nh_last_error(const nh_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* NORI_HIP_H */
