"""Time nh_denoise_image (SimpleDenoiser, GPU) at a given size; prints ms per pass from HIP events."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "optix-renderer_amd"))
import numpy as np
import nori_hip as nh

def main():
    for (h, w, r) in [(600, 800, 7), (1024, 1024, 7), (1024, 1024, 2)]:
        rng = np.random.default_rng(1)
        blk = rng.random((h + 4, w + 4, 4)).astype(np.float32)
        p = nh.simple_denoiser(6.0, 1.5, r, 1)
        ctx = nh.Context(0)
        ctx.denoise_image(blk, 2, p)
        ctx.reset_stats()
        t = time.perf_counter()
        ctx.denoise_image(blk, 2, p)
        wall = (time.perf_counter() - t) * 1e3
        s = ctx.stats()
        print(f"{w}x{h} range {r}: {s['kernel_ms_denoise']:.2f} ms device ({s['launches_denoise']} launches), {wall:.1f} ms wall", flush=True)

main()
