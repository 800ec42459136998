// nori_hip: headless equivalent of the reference's `nori <scene.xml>` entry
// (src/utils/main.cpp:32-114 + RenderThread::renderThreadMain, render.cpp:232-419),
// rendering the scene's path_mis / path_mats integrator on one MI355X through the
// C-ABI, applying the scene's <denoiser> (render.cpp:368-369), and writing <scene>.exr next to the input
// (Bitmap::save, bitmap.cpp:82-110).
//
//   nori_hip scene.xml [--spp N] [--width W --height H] [--device D] [--ordered] [--pfm out.pfm] [--png]
// --png also writes <scene>.png as Bitmap::saveToLDR (bitmap.cpp:122-140; the reference's hdrToLdr).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nori_hip.h"

static int die(const char *what, const char *msg) {
    std::fprintf(stderr, "nori_hip: %s: %s\n", what, msg);
    return 1;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: nori_hip scene.xml [--spp N] [--width W --height H] [--device D] [--ordered] [--pfm out] [--png]\n");
        return 1;
    }
    std::string scene_path = argv[1], pfm;
    bool png = false;
    int spp = 0, w = 0, h = 0, device = 0, traversal = NH_TRAVERSAL_REFERENCE;
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() { return i + 1 < argc ? argv[++i] : (char *)"0"; };
        if (a == "--spp") spp = std::atoi(next());
        else if (a == "--width") w = std::atoi(next());
        else if (a == "--height") h = std::atoi(next());
        else if (a == "--device") device = std::atoi(next());
        else if (a == "--ordered") traversal = NH_TRAVERSAL_ORDERED;
        else if (a == "--pfm") pfm = next();
        else if (a == "--png") png = true;
        else return die("argument", a.c_str());
    }
    nh_scene *scene = nullptr;
    if (nh_scene_load_xml(scene_path.c_str(), &scene)) return die("load", nh_host_last_error());
    if (w > 0 && h > 0) nh_scene_set_resolution(scene, w, h);
    if (spp > 0) nh_scene_set_sample_count(scene, spp);
    nh_scene_desc desc;
    nh_scene_get_desc(scene, &desc);
    auto t0 = std::chrono::steady_clock::now();
    nh_bvh *bvh = nullptr;
    if (nh_bvh_build(&desc, 0, &bvh)) return die("bvh", nh_host_last_error());
    nh_bvh_desc bd;
    nh_bvh_get_desc(bvh, &bd);
    auto t1 = std::chrono::steady_clock::now();
    nh_ctx *ctx = nullptr;
    if (nh_create(device, &ctx)) return die("device", "cannot create a context on the requested GPU");
    if (nh_upload_scene(ctx, &desc) || nh_upload_bvh(ctx, &bd)) return die("upload", nh_last_error(ctx));
    nh_render_req req;
    std::memset(&req, 0, sizeof(req));
    req.sample_begin = 0;
    req.sample_end = desc.sample_count;
    req.mode = NH_MODE_MEGAKERNEL;
    req.traversal = traversal;
    req.clear = 1;
    auto t2 = std::chrono::steady_clock::now();
    if (nh_render(ctx, &req)) return die("render", nh_last_error(ctx));
    nh_synchronize(ctx);
    auto t3 = std::chrono::steady_clock::now();
    // Denoiser::denoise on the master block after the render loop (render.cpp:368-369)
    if (desc.denoiser.type != NH_DENOISER_NONE && nh_denoise(ctx, &desc.denoiser))
        return die("denoise", nh_last_error(ctx));
    const int W = desc.camera.width, H = desc.camera.height, B = desc.filter.border;
    std::vector<float> rgbw(4 * (size_t)(W + 2 * B) * (H + 2 * B)), rgb(3 * (size_t)W * H);
    nh_get_framebuffer(ctx, rgbw.data(), rgbw.size());
    nh_framebuffer_to_rgb(rgbw.data(), W, H, B, rgb.data());
    std::string out = scene_path;
    auto dot = out.find_last_of('.');
    if (dot != std::string::npos) out = out.substr(0, dot);
    if (png) nh_write_png((out + ".png").c_str(), rgb.data(), W, H);
    out += ".exr";
    nh_write_exr(out.c_str(), rgb.data(), W, H);
    if (!pfm.empty()) nh_write_pfm(pfm.c_str(), rgb.data(), W, H);
    double bvh_s = std::chrono::duration<double>(t1 - t0).count();
    double rs = std::chrono::duration<double>(t3 - t2).count();
    double msps = (double)W * H * desc.sample_count / rs / 1e6;
    std::printf("nori_hip: %dx%d %d spp, BVH %u nodes (%.3f s), render %.3f s = %.2f Msamples/s -> %s\n", W, H,
                desc.sample_count, bd.n_nodes, bvh_s, rs, msps, out.c_str());
    nh_destroy(ctx);
    nh_bvh_free(bvh);
    nh_scene_free(scene);
    return 0;
}
