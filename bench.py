"""Benchmark of the MI355X path_mis hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--mode wavefront]

Workload (N=1, BASELINE.json configs[1]): Cornell box diffuse-only (C2: both spheres
diffuse), 1024x1024, 256 spp, path_mis, per-path pcg32 seeding. One step = `--rounds`
(default 16) sample rounds over the whole image = one nh_render call: the wavefront pipeline
(generate, then extend / any-hit / shade per bounce until no path is alive) or, with
--mode megakernel, one path-kernel launch; then one ImageBlock splat. The default K=16 steps
render the full 256 spp. Multi-GPU: one process per GPU (torchrun), 32x32 image blocks dealt
round-robin to ranks (tile shard); a step is `--rounds` x N sample rounds over each rank's 1/N
of the blocks, so every GPU traces the same 16.7M samples per step at any N (weak scaling: at N
GPUs the K steps render N x K x rounds spp of the same image); one RCCL reduce (sum) of the RGBW
framebuffer to rank 0 inside the timed region.

The JSON line also carries:
  roofline      the dominant kernel (largest summed HIP-event time on the context's stream):
                  wf_shade    path-state bytes loaded + stored (counted by construction from
                              the queue counts)
                  wf_extend   BVH nodes x 64 B + primitive tests x 48 B (in-kernel counters in
                              a calibration launch on the same seeds) + 48 B ray/hit per query
                  nh_path_kernel (megakernel) nodes x 64 + prims x 48 + 20 B record per path
                ... / average launch duration, against 8 TB/s HBM; traffic = HBM bytes per
                launch from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json)
                when one exists for this workload, else null
  cpu_baseline  the CPU oracle (oracle/, a restatement of the reference's path_mis) timed on
                this host on a bounded sample of the same workload (rank 0, N=1 only)
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "optix-renderer_amd"))

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
NODE_BYTES, PRIM_BYTES, RECORD_BYTES = 64, 48, 20
EXTEND_IO_BYTES = 4 + 32 + 16


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=16)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--rounds", type=int, default=16, help="sample rounds per step")
    p.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "bumpy1m"])
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--traversal", default="ordered", choices=["ordered", "reference"])
    p.add_argument("--mode", default="wavefront", choices=["megakernel", "wavefront"])
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-calibrate", action="store_true")
    p.add_argument("--pools", type=int, default=2,
                   help="wavefront path pools in flight (2: a chunk's last bounces overlap the next chunk)")
    p.add_argument("--roofline-steps", type=int, default=4,
                   help="with --pools > 1: steps of the serialized pass that times the kernels for the roofline")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl = RCCL over xGMI (production); gloo = host-side reduce, for rehearsing the "
                        "multi-process flow with several ranks on one GPU")
    return p.parse_args()


def build_scene(args, tmp):
    """SURVEY.md 8(d) configurations. Returns (xml, W, H, description, default spp per step count)."""
    import scenegen
    if args.config in ("c1", "c2", "c4"):
        w = args.width or (2048 if args.config == "c4" else 1024)
        h = args.height or w
        xml = scenegen.cbox_xml(tmp, "c2" if args.config == "c2" else "c1", width=w, height=h)
        desc = f"Cornell box ({'diffuse-only' if args.config == 'c2' else 'mirror+dielectric'}) {w}x{h}"
    elif args.config == "c5":
        w = args.width or 4096
        h = args.height or w
        xml, ntri = scenegen.c5_xml(tmp, width=w, height=h)
        desc = f"C5: 10 flattened bumpy meshes ({ntri} tris) + png envmap + area light {w}x{h}"
    else:
        w = args.width or 1024
        h = args.height or w
        n_phi = 1000 if args.config == "c3" else 2000
        xml, ntri = scenegen.bumpy_cbox_xml(tmp, n_phi, 250, width=w, height=h)
        desc = f"cbox + synthetic bumpy sphere ({ntri} tris, Beckmann microfacet) {w}x{h}"
    return xml, w, h, desc


def pmc_traffic(workload_key):
    """HBM bytes per path-kernel launch from a committed rocprofv3 PMC summary, if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        data = json.load(open(path))
        return data.get(workload_key, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def roofline(args, calib, st, W, H, R):
    """Roofline of the dominant kernel. Algorithmic bytes come from the calibration launch's
    in-kernel counters (same seeds as the first timed step), scaled per sample; the time is the
    kernel's summed HIP-event duration over the timed region on the context's stream.
      megakernel: nh_path_kernel -- BVH nodes x 64 B + primitive tests x 48 B (closest, probe and
                  shadow queries) + 20 B sample record per path
      wavefront:  the dominant stage -- wf_shade: path-state bytes; wf_extend: the closest-hit
                  share of nodes/prims + 48 B per query (ray 32 B in, hit 16 B out)"""
    paths = calib["samples"]
    NODE_BYTES = calib.get("node_bytes") or 64  # 128 when the 4-wide tree was traversed
    if args.mode == "wavefront":
        # dominant stage by measured time
        stage = max(("extend", "shadow", "shade"), key=lambda k: st[f"kernel_ms_{k}"])
        q = calib["ray_queries"] - calib["shadow_queries"]
        nodes = calib["nodes_visited"] - calib["shadow_nodes_visited"]
        prims = calib["prims_tested"] - calib["shadow_prims_tested"]
        if stage == "shade":
            bytes_calib = calib["shade_state_bytes"]
        elif stage == "extend":
            bytes_calib = nodes * NODE_BYTES + prims * PRIM_BYTES + calib["extend_queue_bytes"]
        else:
            bytes_calib = (calib["shadow_nodes_visited"] * NODE_BYTES + calib["shadow_prims_tested"] * PRIM_BYTES
                           + calib["shadow_queue_bytes"])
        launches, ms, kernel = max(st[f"launches_{stage}"], 1), st[f"kernel_ms_{stage}"], f"wf_{stage}"
    else:
        q, nodes, prims = calib["ray_queries"], calib["nodes_visited"], calib["prims_tested"]
        bytes_calib = nodes * NODE_BYTES + prims * PRIM_BYTES + paths * RECORD_BYTES
        launches, ms, kernel = max(st["launches_path"], 1), st["kernel_ms_path"], "nh_path_kernel"
    bytes_per_sample = bytes_calib / paths
    avg_ms = ms / launches
    bytes_per_launch = bytes_per_sample * st["samples"] / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    key = f"{args.config}_{W}x{H}_r{R}_{args.traversal}_{args.mode}"
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            # PMC summaries are recorded for single-GPU runs (per-rank launches are smaller at N > 1)
            "traffic": pmc_traffic(key) if int(os.environ.get("WORLD_SIZE", "1")) == 1 else None,
            "kernel": kernel, "avg_launch_ms": round(avg_ms, 4), "launches": launches,
            "algorithmic_bytes_per_launch": int(bytes_per_launch),
            "bytes_per_sample": round(bytes_per_sample, 1),
            "node_bytes": NODE_BYTES,
            "queries_per_sample": round(q / paths, 3),
            "nodes_per_query": round(nodes / max(q, 1), 3),
            "prims_per_query": round(prims / max(q, 1), 3),
            "splat_ms_per_launch": round(st["kernel_ms_splat"] / max(st["launches_splat"], 1), 4)}
    if args.mode == "wavefront":
        roof["stage_ms"] = {k: round(st[f"kernel_ms_{k}"], 3) for k in ("extend", "shadow", "shade", "tail", "splat")}
        # every traversal/shade stage against HBM, algorithmic bytes as above (per-sample from calibration)
        per = {"shade": calib["shade_state_bytes"],
               "extend": nodes * NODE_BYTES + prims * PRIM_BYTES + calib["extend_queue_bytes"],
               "extend_queue_only": calib["extend_queue_bytes"],
               "shadow": (calib["shadow_nodes_visited"] * NODE_BYTES + calib["shadow_prims_tested"] * PRIM_BYTES
                          + calib["shadow_queue_bytes"])}
        roof["stage_gbs"] = {}
        for k, b in per.items():
            t = st["kernel_ms_" + k.split("_")[0]]
            if t > 0:
                roof["stage_gbs"][k] = round(b / paths * st["samples"] / (t * 1e-3) / 1e9, 1)
    return roof


def cpu_baseline(scene, budget_s, seed):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import nori_oracle as no
    threads = int(os.environ.get("NH_CPU_THREADS", "16"))
    threads = max(1, min(threads, os.cpu_count() or 1))
    orc = no.OracleScene(scene)
    rgbw = None
    t0 = time.perf_counter()
    rounds = 0
    while True:
        rgbw = orc.render(rounds, rounds + 1, seed=seed, threads=threads, rgbw=rgbw)
        rounds += 1
        if time.perf_counter() - t0 >= budget_s or rounds >= 256:
            break
    dt = time.perf_counter() - t0
    n = rounds * orc.width * orc.height
    return {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{rounds} spp of the same {orc.width}x{orc.height} image ({n} samples, {dt:.1f} s), "
                      f"oracle/nori_oracle.cpp restatement of path_mis, {threads} threads"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = 0  # rehearsal: every rank on GPU 0
            dist.init_process_group("gloo")
    import nori_hip as nh

    tmp = tempfile.mkdtemp(prefix="nh_bench_")
    xml, W, H, scene_desc = build_scene(args, tmp)
    scene = nh.Scene(xml)
    t0 = time.perf_counter()
    bvh = nh.Bvh(scene, n_threads=16)
    bvh_s = time.perf_counter() - t0
    ctx = nh.Context(local)
    t0 = time.perf_counter()
    ctx.upload(scene, bvh)
    upload_s = time.perf_counter() - t0
    blocks = nh.tile_shard(W, H, world, rank) if world > 1 else None
    trav = nh.TRAVERSAL_ORDERED if args.traversal == "ordered" else nh.TRAVERSAL_REFERENCE
    mode = nh.MODE_WAVEFRONT if args.mode == "wavefront" else nh.MODE_MEGAKERNEL
    # rounds per step and rank: each rank's 1/N of the image for N x --rounds rounds (weak scaling)
    R = args.rounds * world
    os.environ["NH_POOLS"] = str(args.pools)

    # calibration launch (in-kernel counters; same seeds as the first timed step)
    calib = None
    if not args.no_calibrate:
        ctx.reset_stats()
        ctx.render(0, R, seed=args.seed, blocks=blocks, traversal=trav, clear=True, stats=True, mode=mode)
        calib = ctx.stats()

    # warmup (rounds past the timed range, separate framebuffer content)
    for w in range(args.warmup):
        ctx.render(R * (args.steps + w), R * (args.steps + w + 1), seed=args.seed, blocks=blocks, traversal=trav,
                   clear=(w == 0), mode=mode)
    ctx.synchronize()
    ctx.reset_stats()
    if dist is not None:
        import torch
        ctx.synchronize()
        dist.barrier()
    ctx.render(0, 0, seed=args.seed, blocks=blocks, traversal=trav, clear=True)
    ctx.synchronize()
    t_start = time.perf_counter()
    for s in range(args.steps):
        ctx.render(s * R, (s + 1) * R, seed=args.seed, blocks=blocks, traversal=trav, clear=False, mode=mode)
    if dist is not None:
        ctx.synchronize()
        if args.dist_backend == "nccl":
            ptr, n = ctx.framebuffer_device_ptr()
            fb = _wrap_device(ptr, n, local)
            dist.reduce(fb, dst=0, op=dist.ReduceOp.SUM)
            torch.cuda.synchronize()
        else:
            fb = torch.from_numpy(ctx.framebuffer().reshape(-1))
            dist.reduce(fb, dst=0, op=dist.ReduceOp.SUM)
    ctx.synchronize()
    t_end = time.perf_counter()
    elapsed = t_end - t_start
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=f"cuda:{local}" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = ctx.stats()
    total_samples = W * H * R * args.steps
    roof_pass = None
    if args.mode == "wavefront" and args.pools > 1 and calib is not None and args.roofline_steps > 0:
        # Kernels of overlapping pools share the GPU, so their event durations are no kernel roofline:
        # time the kernels in a serialized pass (one pool) over the same workload instead.
        os.environ["NH_POOLS"] = "1"
        ctx.reset_stats()
        base = R * (args.steps + args.warmup)
        for s in range(args.roofline_steps):
            ctx.render(base + s * R, base + (s + 1) * R, seed=args.seed, blocks=blocks, traversal=trav, mode=mode)
        ctx.synchronize()
        st = ctx.stats()
        roof_pass = f"serialized pass: {args.roofline_steps} steps with one path pool (kernels alone on the GPU)"
        os.environ["NH_POOLS"] = str(args.pools)

    if rank == 0:
        value = total_samples / elapsed / 1e6
        # roofline of the path megakernel (dominant kernel)
        roof = None
        if calib is not None and calib["samples"] > 0:
            roof = roofline(args, calib, st, W, H, R)
            roof["timed"] = roof_pass or "the timed region"
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(scene, args.cpu_seconds, args.seed)
        line = {
            "metric": "Msamples/sec (whole node) + traversal HBM GB/s, cbox 1024x1024 256spp",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference Cornell box scene files, per-path pcg32 seeds)",
            "config": {"workload": f"{scene_desc}, {R * args.steps} spp, path_mis", "config": args.config,
                       "width": W, "height": H, "spp": R * args.steps, "rounds_per_step": R,
                       "mode": args.mode, "traversal": args.traversal, "pools": args.pools,
                       "parallelism": (f"tile-shard x{world} + {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} reduce"
                                       if world > 1 else "single GPU"),
                       "bvh_build_s": round(bvh_s, 3), "upload_s": round(upload_s, 3)},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _wrap_device(ptr, n, device):
    """torch view of the context's device framebuffer (fp32, n elements) for RCCL."""
    import torch

    class _CAI:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 3}

    return torch.as_tensor(_CAI(), device=f"cuda:{device}")


if __name__ == "__main__":
    main()
