/*
 * A scene handed to the C-ABI field by field, without the XML loader -- what a Nori build binding the
 * library through per-plugin export hooks (Shape/BSDF/Emitter/Camera::getHipRecord,
 * shaped like the reference's getOptix* hooks, include/nori/bsdf.h:122, emitter.h:159, shape.h:194-201,
 * camera.h:86) produces from its live objects. The records below are what those hooks would write:
 *   camera   PerspectiveCamera::update (src/cameras/perspective.cpp:48-96): sampleToCamera, cameraToWorld
 *   filter   GaussianFilter (src/cameras/rfilter.cpp:31-47) tabulated as ImageBlock::init (block.cpp:54-70)
 *   meshes   Mesh::update area DiscretePDF (src/shapes/mesh.cpp:35-48)
 *   emitters Scene::emitterDpdf (one area light)
 * The scene is rendered through nh_render (wavefront, ordered traversal) and compared with the CPU
 * oracle (test infrastructure, oracle/) on the same description. Exit 0 when rel-L2 < 1e-4.
 *
 * usage: manual_scene [spp]
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nori_hip.h"
#include "nori_oracle.h"

#define W 64
#define H 48

/* row-major 4x4 inverse (Gauss-Jordan in double) */
static int inv4(const double *m, double *out) {
    double a[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) a[i][j] = j < 4 ? m[4 * i + j] : (j - 4 == i);
    for (int c = 0; c < 4; ++c) {
        int p = c;
        for (int r = c + 1; r < 4; ++r)
            if (fabs(a[r][c]) > fabs(a[p][c])) p = r;
        if (fabs(a[p][c]) < 1e-12) return 1;
        for (int j = 0; j < 8; ++j) { double t = a[c][j]; a[c][j] = a[p][j]; a[p][j] = t; }
        const double d = a[c][c];
        for (int j = 0; j < 8; ++j) a[c][j] /= d;
        for (int r = 0; r < 4; ++r)
            if (r != c) {
                const double f = a[r][c];
                for (int j = 0; j < 8; ++j) a[r][j] -= f * a[c][j];
            }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = a[i][j + 4];
    return 0;
}

/* PerspectiveCamera::update: sampleToCamera = (scale(0.5, -0.5 aspect, 1) * translate(1, -1/aspect, 0) *
 * perspective)^-1, camera at the origin looking down +z (cameraToWorld = identity) */
static void camera(nh_camera *c, float fov_deg, float near_clip, float far_clip) {
    memset(c, 0, sizeof(*c));
    c->width = W;
    c->height = H;
    const double aspect = (double)W / H, recip = 1.0 / (far_clip - near_clip);
    const double cot = 1.0 / tan(fov_deg * 3.14159265358979323846 / 360.0);
    const double persp[16] = {cot, 0, 0, 0, 0, cot, 0, 0, 0, 0, far_clip * recip, -near_clip * far_clip * recip, 0, 0, 1, 0};
    const double st[16] = {0.5, 0, 0, 0.5, 0, -0.5 * aspect, 0, 0.5, 0, 0, 1, 0, 0, 0, 0, 1};  /* scale * translate */
    double m[16], inv[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += st[4 * i + k] * persp[4 * k + j];
            m[4 * i + j] = s;
        }
    if (inv4(m, inv)) abort();
    for (int i = 0; i < 16; ++i) {
        c->sample_to_camera[i] = (float)inv[i];
        c->camera_to_world[i] = (i % 5 == 0) ? 1.f : 0.f;
    }
    c->inv_output_size[0] = 1.f / W;
    c->inv_output_size[1] = 1.f / H;
    c->near_clip = near_clip;
    c->far_clip = far_clip;
}

static void gaussian_filter(nh_filter *f, float radius, float stddev) {
    f->radius = radius;
    f->border = (int)ceilf(radius - 0.5f);
    f->lookup_factor = 32 / radius;
    const float alpha = -1.0f / (2.0f * stddev * stddev);
    for (int i = 0; i < 32; ++i) {
        const float x = (radius * i) / 32;
        const float v = (float)exp((double)(alpha * x * x)) - (float)exp((double)(alpha * radius * radius));
        f->table[i] = v > 0 ? v : 0;
    }
    f->table[32] = 0.f;
}

/* Mesh::update: triangle-area CDF, normalised, last entry 1 */
static float area_cdf(const float *V, const unsigned *F, unsigned nf, float *cdf) {
    cdf[0] = 0.f;
    for (unsigned i = 0; i < nf; ++i) {
        const float *p0 = V + 3 * F[3 * i], *p1 = V + 3 * F[3 * i + 1], *p2 = V + 3 * F[3 * i + 2];
        const float a[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
        const float b[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
        const float c[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
        cdf[i + 1] = cdf[i] + 0.5f * sqrtf(c[0] * c[0] + (c[1] * c[1] + c[2] * c[2]));
    }
    const float sum = cdf[nf], norm = 1.0f / sum;
    for (unsigned i = 1; i <= nf; ++i) cdf[i] *= norm;
    cdf[nf] = 1.0f;
    return norm;
}

static void mesh_bbox(nh_shape *s, const float *V) {
    for (int a = 0; a < 3; ++a) { s->bbox_min[a] = INFINITY; s->bbox_max[a] = -INFINITY; }
    for (unsigned v = s->v_offset; v < s->v_offset + s->n_vertices; ++v)
        for (int a = 0; a < 3; ++a) {
            s->bbox_min[a] = fminf(s->bbox_min[a], V[3 * v + a]);
            s->bbox_max[a] = fmaxf(s->bbox_max[a], V[3 * v + a]);
        }
}

int main(int argc, char **argv) {
    const int spp = argc > 1 ? atoi(argv[1]) : 8;
    /* floor quad (y = -1) and a light quad (y = 1.5, facing down), as two meshes of one vertex array */
    static const float V[] = {-3, -1, 1,  3, -1, 1,  3, -1, 8,  -3, -1, 8,
                              -0.6f, 1.5f, 3.4f,  0.6f, 1.5f, 3.4f,  0.6f, 1.5f, 4.6f,  -0.6f, 1.5f, 4.6f};
    static const unsigned F[] = {0, 2, 1, 0, 3, 2, /* light, local indices: */ 0, 1, 2, 0, 2, 3};
    static float N[3 * 8], UV[2 * 8], T[3 * 8], BT[3 * 8];
    nh_shape shapes[4];
    memset(shapes, 0, sizeof(shapes));
    shapes[0].type = NH_SHAPE_MESH; shapes[0].bsdf = 0; shapes[0].emitter = -1;
    shapes[0].v_offset = 0; shapes[0].n_vertices = 4; shapes[0].f_offset = 0; shapes[0].n_faces = 2;
    shapes[1].type = NH_SHAPE_MESH; shapes[1].bsdf = 0; shapes[1].emitter = 0;
    shapes[1].v_offset = 4; shapes[1].n_vertices = 4; shapes[1].f_offset = 2; shapes[1].n_faces = 2;
    /* two spheres: a Beckmann microfacet one and a mirror one */
    const float sc[2][4] = {{-0.8f, -0.3f, 4.2f, 0.7f}, {0.9f, -0.45f, 3.6f, 0.55f}};
    for (int i = 0; i < 2; ++i) {
        nh_shape *s = &shapes[2 + i];
        s->type = NH_SHAPE_SPHERE; s->bsdf = 1 + i; s->emitter = -1;
        for (int a = 0; a < 3; ++a) {
            s->center[a] = sc[i][a];
            s->bbox_min[a] = sc[i][a] - sc[i][3];
            s->bbox_max[a] = sc[i][a] + sc[i][3];
        }
        s->radius = sc[i][3];
    }
    float cdf[6];
    shapes[0].pdf_offset = 0;
    shapes[0].pdf_normalization = area_cdf(V, F, 2, cdf);
    shapes[1].pdf_offset = 3;
    shapes[1].pdf_normalization = area_cdf(V + 3 * 4, F + 6, 2, cdf + 3);
    mesh_bbox(&shapes[0], V);
    mesh_bbox(&shapes[1], V);

    nh_bsdf bsdfs[3];
    memset(bsdfs, 0, sizeof(bsdfs));
    bsdfs[0].type = NH_BSDF_DIFFUSE;
    bsdfs[0].albedo[0] = 0.7f; bsdfs[0].albedo[1] = 0.6f; bsdfs[0].albedo[2] = 0.5f;
    bsdfs[1].type = NH_BSDF_MICROFACET;  /* microfacet.cpp:33-54: ks = 1 - max(kd) */
    bsdfs[1].alpha = 0.25f; bsdfs[1].int_ior = 1.5046f; bsdfs[1].ext_ior = 1.000277f;
    bsdfs[1].kd[0] = 0.2f; bsdfs[1].kd[1] = 0.35f; bsdfs[1].kd[2] = 0.5f; bsdfs[1].ks = 1.0f - 0.5f;
    bsdfs[2].type = NH_BSDF_MIRROR;

    nh_emitter em;
    memset(&em, 0, sizeof(em));
    em.type = NH_EMITTER_AREA;
    em.shape = 1;
    em.radiance[0] = em.radiance[1] = em.radiance[2] = 12.f;
    em.light_prob = 1.f;
    static const float emitter_cdf[2] = {0.f, 1.f};

    nh_scene_desc d;
    memset(&d, 0, sizeof(d));
    camera(&d.camera, 50.f, 1e-4f, 1e4f);
    gaussian_filter(&d.filter, 2.0f, 0.5f);
    d.integrator = NH_INTEGRATOR_PATH_MIS;
    d.sample_count = spp;
    d.n_shapes = 4; d.shapes = shapes;
    d.n_bsdfs = 3; d.bsdfs = bsdfs;
    d.n_emitters = 1; d.emitters = &em; d.emitter_cdf = emitter_cdf;
    d.envmap = -1;
    d.n_vertices = 8; d.V = V; d.N = N; d.UV = UV; d.T = T; d.BT = BT;
    d.n_faces = 4; d.F = F;
    d.n_area_cdf = 6; d.area_cdf = cdf;

    nh_bvh *bvh = NULL;
    nh_ctx *ctx = NULL;
    if (nh_bvh_build(&d, 0, &bvh) != NH_OK) { fprintf(stderr, "bvh: %s\n", nh_host_last_error()); return 2; }
    nh_bvh_desc bd;
    nh_bvh_get_desc(bvh, &bd);
    if (nh_create(0, &ctx) != NH_OK) { fprintf(stderr, "no device\n"); return 2; }
    if (nh_upload_scene(ctx, &d) != NH_OK || nh_upload_bvh(ctx, &bd) != NH_OK) {
        fprintf(stderr, "upload: %s\n", nh_last_error(ctx));
        return 2;
    }
    nh_render_req q;
    memset(&q, 0, sizeof(q));
    q.sample_begin = 0; q.sample_end = spp; q.seed = 77;
    q.mode = NH_MODE_WAVEFRONT; q.traversal = NH_TRAVERSAL_ORDERED; q.clear = 1;
    if (nh_render(ctx, &q) != NH_OK) { fprintf(stderr, "render: %s\n", nh_last_error(ctx)); return 2; }
    const size_t n = 4 * (size_t)(W + 2 * d.filter.border) * (H + 2 * d.filter.border);
    float *g = calloc(n, sizeof(float)), *r = calloc(n, sizeof(float));
    if (nh_get_framebuffer(ctx, g, n) != NH_OK) { fprintf(stderr, "fb: %s\n", nh_last_error(ctx)); return 2; }
    nh_render_stats st;
    nh_get_stats(ctx, &st);

    no_scene *os = NULL;  /* the oracle on the same description */
    if (no_scene_create(&d, &os) != NH_OK) return 2;
    uint64_t inv = 0;
    if (no_render(os, NO_SAMPLER_PER_PATH, 77, 0, spp, NULL, 0, 8, r, &inv) != NH_OK) return 2;
    double num = 0, den = 0, mean = 0;
    int same = 1;
    for (size_t i = 0; i < n; ++i) {
        const double e = (double)g[i] - r[i];
        num += e * e;
        den += (double)r[i] * r[i];
        mean += r[i];
        same &= memcmp(&g[i], &r[i], 4) == 0;
    }
    const double rel = sqrt(num / (den > 0 ? den : 1e-300));
    printf("manual-scene %dx%d %d spp: rel-L2 %.3e bit-identical %d mean %.4f fused %llu samples %llu\n", W, H, spp,
           rel, same, mean / n, (unsigned long long)st.fused_bounce, (unsigned long long)st.samples);
    no_scene_free(os);
    nh_destroy(ctx);
    nh_bvh_free(bvh);
    free(g);
    free(r);
    return rel < 1e-4 && mean > 1e-3 ? 0 : 1;
}
