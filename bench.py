"""Benchmark of the MI355X path_mis hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--mode wavefront] [--scaling weak|strong]

Workload (N=1, BASELINE.json configs[1]): Cornell box diffuse-only (C2: both spheres
diffuse), 1024x1024, 256 spp, path_mis, per-path pcg32 seeding. One step = `--rounds`
(default 16) sample rounds over the whole image = one nh_render call: the wavefront pipeline
(per bounce: closest-hit traversal, any-hit traversal, shade; a tail kernel finishes the last
paths) or, with --mode megakernel, one path-kernel launch; then the ImageBlock splat. The
default K=16 steps render the full 256 spp.

Multi-GPU: one process per GPU (torchrun; `python bench.py --gpus N` without a launcher starts the N ranks
itself as a child torch.distributed.run), 32x32 image blocks dealt round-robin to ranks (tile
shard), one RCCL reduce (sum) of the RGBW framebuffer to rank 0 inside the timed region, max
time over ranks. --scaling weak (default): a step is N x --rounds sample rounds over each rank's
1/N of the blocks, so every GPU traces the same 16.7M samples per step at any N. --scaling
strong: a fixed image (C4, 2048^2, --rounds x --steps spp) split over the ranks by blocks.
`value` = all ranks' samples / the max-over-ranks time.

The JSON line also carries:
  roofline      the dominant kernel (largest summed HIP-event time) against the 8 TB/s HBM peak:
                algorithmic HBM bytes per launch / average launch duration (see roofline()); every
                stage's figures under `stages` (HBM GB/s, and for an LDS-staged BVH the algorithmic
                traversal work rate separately, never compared with the HBM peak); `traffic` = HBM
                bytes per launch from the committed rocprofv3 PMC summary of the same command
                (profiles/pmc_traffic.json, named in `traffic_source`), else null
  traversal     the metric's "traversal HBM GB/s": the closest-hit kernel of the timed run
  traversal_1m  (N=1) the north star's roofline target: the persistent traversal kernel on the
                ~1M-triangle scene (perf-1M), timed in the same run
  cpu_baseline  the CPU oracle (oracle/, a restatement of the reference's path_mis) timed on
                this host's cores on a bounded sample of the same workload (rank 0, N=1 only)
  denoise       (N=1) Denoiser::denoise on the rendered master block (render.cpp:368-369): the GPU
                SimpleDenoiser with scenes/project/denoiser/denoiser-test.xml's parameters, HIP-event time,
                beside the serial CPU oracle on a crop of the same image
  strong_c4     (every N) the north star's scaling target (BASELINE configs[3]): the fixed C4 image (2048^2,
                mirror + dielectric spheres + area light, path_mis) at --strong-spp spp, split over the ranks by
                32x32 blocks, one nh_render call per rank plus the RCCL reduce inside the timed region, max over
                ranks; the driver's SCALE run gets the strong-scaling curve from this sub-record
  megakernel    (N=1) BASELINE configs[1]'s comparison: C2 through the one-kernel-per-sample path
  denoiser_test (N=1) scenes/project/denoiser/denoiser-test.xml (800x600, checkerboard floor, curvy bowl, two area
                lights) as the reference's report times it (reports/project-report/denoising.html:79-81): 1024 spp
                ground truth ("5 minutes"), 16 spp ("roughly 20 seconds") + SimpleDenoiser ("about one second")
  project_scenes (N=1) the reference's envmap scene (envmap_sphere.xml, 800x800, 128 spp) and its two thin-lens
                scenes (dof-val.xml, table_path_mis.xml) at their own sizes and sample counts
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
from nh_env import parse_hw_queues, raise_hw_queues  # noqa: E402  (loads no library)

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
NODE_BYTES, PRIM_BYTES, RECORD_BYTES = 64, 48, 20
EXTEND_IO_BYTES = 4 + 32 + 16


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=16)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--rounds", type=int, default=16, help="sample rounds per step")
    p.add_argument("--config", default=None, choices=["c1", "c2", "c3", "c4", "c5", "bumpy1m"])
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                   help="weak: N x --rounds rounds per step over each rank's 1/N of the blocks (default); strong: "
                        "a fixed image (C4 2048^2 unless --config) and --rounds x --steps spp split by blocks")
    p.add_argument("--strong-spp", type=int, default=256,
                   help="spp of the strong_c4 sub-record (fixed 2048^2 C4 image split over the ranks; 0 = skip)")
    p.add_argument("--hw-queues", type=int, default=0,
                   help="GPU_MAX_HW_QUEUES for this run (A/B; default: at least 8)")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the N=1 megakernel, denoiser_test and project_scenes sub-records")
    p.add_argument("--traversal-1m-steps", type=int, default=4,
                   help="N=1: also time the perf-1M traversal kernel (0 = skip)")
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--traversal", default="ordered", choices=["ordered", "reference"])
    p.add_argument("--mode", default="wavefront", choices=["megakernel", "wavefront"])
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-denoise", action="store_true", help="skip the denoise record")
    p.add_argument("--no-calibrate", action="store_true")
    p.add_argument("--pools", type=int, default=0,
                   help="wavefront path pools in flight (0: the library default; >1: a chunk's last bounces overlap "
                        "the next chunks)")
    p.add_argument("--roofline-steps", type=int, default=4,
                   help="with --pools > 1: steps of the serialized pass that times the kernels for the roofline")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl = RCCL over xGMI (production); gloo = host-side reduce, for rehearsing the "
                        "multi-process flow with several ranks on one GPU")
    p.add_argument("--dump-framebuffer", default=None,
                   help="rank 0 saves the reduced RGBW framebuffer of the timed steps (.npy) before the roofline pass")
    p.add_argument("--launcher-selftest", action="store_true",
                   help="only rendezvous: every rank all-reduces its rank over gloo and rank 0 prints the world size "
                        "(tests the --gpus N launcher without a GPU)")
    a = p.parse_args()
    a.config_given = a.config is not None
    a.config = a.config or "c2"
    return a


def scene_dims(args):
    w = args.width or {"c4": 2048, "c5": 4096}.get(args.config, 1024)
    return w, args.height or w


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
    """HBM bytes per launch of the roofline kernel from a committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json: FETCH_SIZE x2 + WRITE_SIZE from separate --pmc passes of the same
    bench command), or (None, None) when none exists for this workload. It is read from the file,
    not measured in this run: the PMC passes need rocprofv3 around the process."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    try:
        rec = json.load(open(path)).get(workload_key)
    except (OSError, ValueError):
        return None, None
    if not rec:
        return None, None
    return rec.get("hbm_bytes_per_launch"), f"profiles/pmc_traffic.json[{workload_key}]: {rec.get('source', '')}"


def pmc_record(workload_key):
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        return json.load(open(path)).get(workload_key) or {}
    except (OSError, ValueError):
        return {}


_LIB_SHA = {}


def lib_sha16():
    """The build identity PMC records are checked against: the first 16 hex digits of the SHA-256 of the library
    this process loaded (scripts/pmc_traffic.py records the same for the library its passes loaded)."""
    import nori_hip as nh
    if nh.LIB_PATH not in _LIB_SHA:
        import hashlib
        _LIB_SHA[nh.LIB_PATH] = hashlib.sha256(open(nh.LIB_PATH, "rb").read()).hexdigest()[:16]
    return _LIB_SHA[nh.LIB_PATH]


def stage_work(calib):
    """Traversal work per stage from the calibration launch's in-kernel counters: the tail kernel
    counts into its own slots, so extend / shadow are those kernels' own visits."""
    tq, tn, tp = calib["tail_queries"], calib["tail_nodes_visited"], calib["tail_prims_tested"]
    tsq, tsn, tsp = calib["tail_shadow_queries"], calib["tail_shadow_nodes_visited"], calib["tail_shadow_prims_tested"]
    sq, sn, sp = calib["shadow_queries"] - tsq, calib["shadow_nodes_visited"] - tsn, calib["shadow_prims_tested"] - tsp
    eq = calib["ray_queries"] - calib["shadow_queries"] - (tq - tsq)
    en = calib["nodes_visited"] - calib["shadow_nodes_visited"] - (tn - tsn)
    ep = calib["prims_tested"] - calib["shadow_prims_tested"] - (tp - tsp)
    return {"extend": (eq, en, ep), "shadow": (sq, sn, sp), "tail": (tq, tn, tp)}


def roofline(args, calib, st, W, H, R):
    """Roofline of the dominant kernel (largest summed HIP-event time over the timed kernels).

    Algorithmic bytes per launch = the calibration launch's per-sample bytes x samples per launch,
    divided by the kernel's average launch duration (HIP events on the stream it runs on):
      wf_shade     path-state bytes loaded + stored (counted by construction from the queue counts)
      wf_extend /  BVH nodes x node bytes + primitive tests x 48 B (in-kernel counters) + queue bytes
      wf_shadow    (ray in, hit / occlusion out). Node and primitive reads go to global memory only when
                   the BVH is not staged in LDS; a BVH staged in LDS (the Cornell box, < 1 KB) makes them
                   LDS reads, so `global_gbs` counts the queue bytes alone and `lds_work_gbs` the
                   algorithmic traversal bytes read from LDS (never compared with the HBM peak)
      wf_tail      traversal + shade work of the last few paths, in place
      megakernel   nodes x 64 + prims x 48 + 20 B record per path
    These are algorithmic byte counts; the HBM bytes actually moved come from rocprofv3
    FETCH_SIZE / WRITE_SIZE passes (profiles/pmc_traffic.json) as `traffic` / `traffic_gbs`. `peak` is the
    HBM roofline; `global_gbs` (algorithmic) and `traffic_gbs` (measured) are compared with it."""
    paths = calib["samples"]
    node_b = calib.get("node_bytes") or 64
    lds = bool(calib.get("lds_scene"))
    per_launch = lambda b, launches: b / paths * st["samples"] / max(launches, 1)  # noqa: E731
    stages = {}
    fused = args.mode == "wavefront" and bool(calib.get("fused_bounce"))
    if fused:
        # one wf_bounce kernel per bounce (shade + any-hit + closest hit over the LDS copy of the BVH):
        # its HBM bytes are the path state; the traversal work is LDS reads
        w = stage_work(calib)
        (eq, en, ep), (sq, sn, sp) = w["extend"], w["shadow"]
        trav = (en + sn) * node_b + (ep + sp) * PRIM_BYTES
        stages["bounce"] = {"work_bytes": calib["shade_state_bytes"] + trav, "hbm_bytes": calib["shade_state_bytes"],
                            "queries": eq + sq, "nodes": en + sn, "prims": ep + sp, "ms": "shade"}
        q, n, p = w["tail"]
        trav = n * node_b + p * PRIM_BYTES
        stages["tail"] = {"work_bytes": trav, "hbm_bytes": 0 if lds else trav, "queries": q, "nodes": n, "prims": p}
    elif args.mode == "wavefront" and calib.get("trace_fused"):
        # deep BVHs: one persistent launch per bounce answers both queries (wf_trace_pt2); its time is in the
        # extend slot, and its bytes are both queries' traversal work plus both queues
        w = stage_work(calib)
        (eq, en, ep), (sq, sn, sp) = w["extend"], w["shadow"]
        trav = (en + sn) * node_b + (ep + sp) * PRIM_BYTES
        queue = calib["extend_queue_bytes"] + calib["shadow_queue_bytes"]
        stages["trace"] = {"work_bytes": trav + queue, "hbm_bytes": queue + (0 if lds else trav), "queries": eq + sq,
                           "nodes": en + sn, "prims": ep + sp, "ms": "extend"}
        q, n, p = w["tail"]
        trav = n * node_b + p * PRIM_BYTES
        stages["tail"] = {"work_bytes": trav, "hbm_bytes": 0 if lds else trav, "queries": q, "nodes": n, "prims": p}
        stages["shade"] = {"work_bytes": calib["shade_state_bytes"], "hbm_bytes": calib["shade_state_bytes"]}
    elif args.mode == "wavefront":
        w = stage_work(calib)
        for k in ("extend", "shadow", "tail"):
            q, n, p = w[k]
            trav = n * node_b + p * PRIM_BYTES
            queue = {"extend": calib["extend_queue_bytes"], "shadow": calib["shadow_queue_bytes"], "tail": 0}[k]
            stages[k] = {"work_bytes": trav + queue, "hbm_bytes": queue + (0 if lds else trav),
                         "queries": q, "nodes": n, "prims": p}
        stages["shade"] = {"work_bytes": calib["shade_state_bytes"], "hbm_bytes": calib["shade_state_bytes"]}
    else:
        q, n, p = calib["ray_queries"], calib["nodes_visited"], calib["prims_tested"]
        b = n * 64 + p * PRIM_BYTES + paths * RECORD_BYTES
        stages["path"] = {"work_bytes": b, "hbm_bytes": b, "queries": q, "nodes": n, "prims": p}
    report = {}
    for k, v in stages.items():
        src = v.get("ms", k)  # the fused bounce kernel's time is recorded in the shade slot
        ms, launches = st[f"kernel_ms_{src}"], st[f"launches_{src}"]
        if ms <= 0 or launches == 0:
            continue
        avg = ms / launches
        # global_*: algorithmic bytes the kernel moves through global memory (path state / queues, and the
        # BVH nodes and primitive records unless the BVH is staged in LDS), from counters and queue sizes --
        # not a measurement of HBM traffic (that is roofline.traffic, from PMC counters)
        r = {"ms": round(ms, 3), "launches": launches, "avg_launch_ms": round(avg, 4),
             "global_bytes_per_launch": int(per_launch(v["hbm_bytes"], launches)),
             "global_gbs": round(per_launch(v["hbm_bytes"], launches) / (avg * 1e-3) / 1e9, 1)}
        if v["work_bytes"] != v["hbm_bytes"]:
            r["lds_work_gbs"] = round(per_launch(v["work_bytes"] - v["hbm_bytes"], launches) / (avg * 1e-3) / 1e9, 1)
            r["lds_work_note"] = "algorithmic node/primitive bytes read from the LDS copy of the BVH (not global memory)"
        if "queries" in v and v["queries"]:
            r["nodes_per_query"] = round(v["nodes"] / v["queries"], 3)
            r["prims_per_query"] = round(v["prims"] / v["queries"], 3)
        if r["global_gbs"] > HBM_PEAK_GBS * 1.02:  # a global-memory rate above the HBM peak is an accounting bug
            r["accounting_error"] = "global-memory GB/s above the HBM peak"
        srec = pmc_record(f"{args.config}_{W}x{H}_r{R}_{args.traversal}_{args.mode}/{k}") \
            if int(os.environ.get("WORLD_SIZE", "1")) == 1 else {}
        if srec.get("lib_sha16") != lib_sha16():
            srec = {}  # another build's counters
        if srec.get("hbm_bytes_per_launch"):  # measured HBM bytes of this stage's kernel (committed PMC passes)
            r["measured_hbm_bytes_per_launch"] = srec["hbm_bytes_per_launch"]
            r["measured_hbm_gbs"] = round(srec["hbm_bytes_per_launch"] / (avg * 1e-3) / 1e9, 1)
            r["measured_source"] = f"profiles/pmc_traffic.json[{args.config}_{W}x{H}_r{R}_{args.traversal}_{args.mode}/{k}]"
        report[k] = r
    dom = max(report, key=lambda k: report[k]["ms"])
    wide = node_b in (128, 256)  # deep trees: the persistent 4-wide (8-wide: NH_WIDE8=1) traversal kernels
    ww = node_b // 32
    rr = os.environ.get("NH_RR_AHEAD", "1") != "0"
    kernel = {"shade": "wf_shade",
              "trace": f"wf_trace_pt2 (persistent {ww}-wide closest hit + any hit, one launch per bounce)",
              "extend": f"wf_trace_pt (persistent {ww}-wide closest hit)" if wide else "wf_extend",
              "shadow": f"wf_trace_pt (persistent {ww}-wide any hit)" if wide else "wf_shadow",
              "tail": "wf_tail_rr" if fused and rr else "wf_tail", "path": "nh_path_kernel",
              "bounce": ("wf_bounce_rr (shade body + any-hit + closest-hit + the next vertex's roulette, fused)" if rr
                         else "wf_bounce (shade + any-hit + closest-hit, fused)")}[dom]
    d = report[dom]
    key = f"{args.config}_{W}x{H}_r{R}_{args.traversal}_{args.mode}/{dom}"
    single = int(os.environ.get("WORLD_SIZE", "1")) == 1
    rec = pmc_record(key) if single else {}
    stale = None
    if rec and rec.get("lib_sha16") != lib_sha16():
        # counters of another build (or of another kernel instantiation): not this run's kernel, not reported
        stale = (f"the committed record ({rec.get('kernel', '?')}) is from library build {rec.get('lib_sha16')}, "
                 f"this run loaded {lib_sha16()}: not used")
        rec = {}
    traffic = rec.get("hbm_bytes_per_launch")
    achieved = d["global_gbs"]
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": (f"profiles/pmc_traffic.json[{key}]: {rec.get('source', '')}; kernel "
                               f"{rec.get('kernel')}, library build {rec.get('lib_sha16')}" if traffic else
                               stale or "not collected for this workload (rocprofv3 PMC runs separately)"),
            "lib_sha16": lib_sha16(),
            "kernel": kernel, "avg_launch_ms": d["avg_launch_ms"], "launches": d["launches"],
            "algorithmic_bytes_per_launch": d["global_bytes_per_launch"],
            "bytes_per_sample": round(stages[dom]["hbm_bytes"] / paths, 1), "node_bytes": node_b,
            "lds_scene": lds, "queries_per_sample": round(calib["ray_queries"] / paths, 3),
            "splat_ms_per_launch": round(st["kernel_ms_splat"] / max(st["launches_splat"], 1), 4),
            "stages": report}
    if traffic:
        # measured HBM bytes per launch (PMC, separate passes) over this run's launch time
        roof["traffic_gbs"] = round(traffic / (d["avg_launch_ms"] * 1e-3) / 1e9, 1)
        roof["traffic_frac"] = round(roof["traffic_gbs"] / HBM_PEAK_GBS, 4)
    if rec.get("valu_issue_frac") is not None:
        roof["limiter"] = limiter_record(rec, key, d["avg_launch_ms"], 5 if dom in ("trace", "extend") and wide else 4)
    if calib.get("tail_bounces"):
        # the RR-ahead tail kernel's phases (clock64 in the calibration launch, summed over lanes): where one
        # path-bounce of the specular chains that set the tail's length spends its cycles
        nb = calib["tail_bounces"]
        roof["tail_profile"] = {
            "path_bounces": nb, "longest_chain_bounces": calib["tail_max_bounces"],
            "cycles_per_bounce": {k: round(calib[f"tail_cycles_{k}"] / nb, 1)
                                  for k in ("body", "shadow", "closest", "head")},
            "source": "wf_tail_rr calibration launch (collect_stats), clock64 per phase"}
        nc = calib.get("tail_coop_bounces", 0)
        if nc:
            # bounces the cooperative finish ran (one path per 16-lane group): one bounce's latency on the last chains
            roof["tail_profile"]["coop_bounces"] = nc
            roof["tail_profile"]["coop_cycles_per_bounce"] = {
                k: round(calib[f"tail_coop_cycles_{k}"] / nc, 1) for k in ("body", "shadow", "closest", "head")}
    nbb = calib.get("bounce_bounces", 0)
    if nbb:
        # the RR-ahead bounce kernel's phases in its calibration launch (clock64, summed over lanes; the
        # instrumentation itself adds ~10 % of wave-cycles): where one path-bounce's wave-cycles go
        ph = ("load", "body", "shadow", "closest", "head", "store")
        roof["bounce_profile"] = {
            "path_bounces": nbb,
            "cycles_per_bounce": {k: round(calib[f"bounce_cycles_{k}"] / nbb, 1) for k in ph},
            "source": "wf_bounce_rr calibration launch (collect_stats), clock64 per phase"}
    return roof


VALU_CEILING_FILE = os.path.join(REPO, "profiles", "round4_valu_issue_events.jsonl")
NOMINAL_CLOCK_HZ = 2.4e9  # MI355X peak engine clock (hipDeviceProp_t::clockRate on the box)


def valu_ceiling(waves_per_simd):
    """Measured VALU issue ceiling (tools/valu_issue.hip, scripts/valu_issue.sh; committed events.jsonl): wave64
    instructions per CU-cycle at the nominal clock for independent chains at the given waves/SIMD -- the
    select / compare / integer mix (the path kernels' bookkeeping) and fp32 FMA."""
    try:
        rows = [json.loads(x) for x in open(VALU_CEILING_FILE) if x.startswith("{") and "kind" in x]
    except OSError:
        return None
    # the sweep measures 1, 2, 4 and 8 waves/SIMD: the largest of those not above the kernel's occupancy
    w = max((r["waves_per_simd"] for r in rows if r["waves_per_simd"] <= waves_per_simd), default=None)
    pick = lambda k: next((r["insts_per_cu_cycle_at_peak_clock"] for r in rows  # noqa: E731
                           if r["kind"].startswith(k) and r["waves_per_simd"] == w), None)
    mix, fma = pick("cmp+cndmask"), pick("v_fma_f32")
    return {"mix": mix, "fma32": fma} if mix and fma else None


def limiter_record(rec, key, avg_launch_ms=None, waves_per_simd=4):
    """What bounds the kernel, from the committed PMC passes of the same command: VALU instructions per CU-cycle
    (SQ_INSTS_VALU per launch over this run's launch time at the nominal clock) against the MEASURED issue ceiling
    of the same occupancy (valu_ceiling: round 3 assumed one wave64 instruction per CU-cycle from the quad-cycle
    counter; the microbenchmark shows 1.1-1.4), rocprofv3's VALUBusy and VALUUtilization (active lanes per VALU
    instruction: divergence), and the share of wave-cycles spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES)."""
    out = {"valu_busy_pct": rec.get("valu_busy_pct"), "valu_utilization_pct": rec.get("valu_utilization_pct"),
           "wait_frac": rec.get("wait_frac"), "valu_insts_per_launch": rec.get("valu_insts_per_launch"),
           "source": traffic_source_of(key)}
    ceil = valu_ceiling(waves_per_simd)
    frac = rec.get("valu_issue_frac")
    if ceil and avg_launch_ms and rec.get("valu_insts_per_launch"):
        rate = rec["valu_insts_per_launch"] / (avg_launch_ms * 1e-3 * NOMINAL_CLOCK_HZ * 256)
        frac = rate / ceil["mix"]
        out.update(valu_insts_per_cu_cycle=round(rate, 3), valu_issue_frac=round(frac, 3),
                   valu_ceiling_insts_per_cu_cycle=ceil, valu_ceiling_waves_per_simd=waves_per_simd,
                   valu_ceiling_source="profiles/round4_valu_issue_events.jsonl (tools/valu_issue.hip, the "
                                       "select/compare/integer mix; fp32 FMA quoted beside it)")
    else:
        out["valu_issue_frac"] = frac
    util = rec.get("valu_utilization_pct")
    if util is not None and util < 60:
        out["note"] = (f"divergence-bound: only {util:.0f} % of the lanes are active per VALU instruction, with "
                       f"{frac:.2f} of the measured issue ceiling used and waves waiting "
                       f"{rec.get('wait_frac', 0):.2f} of their cycles -- neither HBM- nor issue-bound")
    elif frac is not None and frac > 0.8:
        out["note"] = "VALU-issue bound: its HBM bytes are the path state only"
    else:
        out["note"] = (f"issue and latency: {frac:.2f} of the measured VALU issue ceiling, waves waiting "
                       f"{rec.get('wait_frac', 0):.2f} of their cycles")
    return out


def traffic_source_of(key):
    return f"profiles/pmc_traffic.json[{key}]"


def traversal_record(roof):
    """The metric's "traversal HBM GB/s": the closest-hit traversal kernel of the timed run (the fused
    bounce kernel when the BVH is traversed inside it): its algorithmic global-memory rate, and for an
    LDS-staged BVH the algorithmic traversal bytes it read from LDS; measured HBM bytes are roofline.traffic."""
    name = next((k for k in ("trace", "extend", "bounce", "path") if k in roof["stages"]), None)
    if name is None:
        return None
    e = roof["stages"][name]
    out = {"kernel": {"trace": "wf_trace_pt2", "extend": "wf_extend", "bounce": "wf_bounce",
                      "path": "nh_path_kernel"}[name],
           "global_gbs": e["global_gbs"], "frac_of_hbm_peak": round(e["global_gbs"] / HBM_PEAK_GBS, 4),
           "avg_launch_ms": e["avg_launch_ms"]}
    if "lds_work_gbs" in e:
        out["lds_work_gbs"] = e["lds_work_gbs"]
        out["note"] = ("BVH staged in LDS: global_gbs is the kernel's global-memory stream (ray/hit queues, or the "
                       "path state of the fused bounce kernel); lds_work_gbs the traversal bytes read from LDS")
    if name == roof_dominant(roof) and roof.get("traffic_gbs"):
        out["measured_hbm_gbs"] = roof["traffic_gbs"]
    return out


def roof_dominant(roof):
    return max(roof["stages"], key=lambda k: roof["stages"][k]["ms"])


def cpu_cores():
    """Host cores this process may run on (affinity mask), and the cgroup CPU quota if one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    return n, quota


def cpu_baseline(scene, budget_s, seed):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import nori_oracle as no
    n_cpu, quota = cpu_cores()
    # every core this process may use: the affinity mask, capped by the cgroup CPU quota (the GPU box
    # grants a 16-core share of a larger host; more threads than the quota only time-slice)
    usable = min(n_cpu, max(1, int(quota + 0.999))) if quota else n_cpu
    threads = int(os.environ.get("NH_CPU_THREADS", "0")) or usable
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
    q = f", cgroup CPU quota {quota:g} cores" if quota else ""
    return {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{rounds} spp of the same {orc.width}x{orc.height} image ({n} samples, {dt:.1f} s), "
                      f"oracle/nori_oracle.cpp restatement of path_mis, {threads} threads = every core this process "
                      f"may use (affinity mask {n_cpu} CPUs{q})"}


def run_workload(nh, args, config, steps, warmup, local, blocks=None, world=1, rank=0, dist=None):
    """Scene setup + calibration + warmup + timed steps (+ serialized roofline pass). Returns a dict."""
    a = argparse.Namespace(**vars(args))
    a.config = config
    if config != args.config:
        a.width = a.height = None
    tmp = tempfile.mkdtemp(prefix="nh_bench_")
    xml, W, H, scene_desc = build_scene(a, tmp)
    scene = nh.Scene(xml)
    t0 = time.perf_counter()
    bvh = nh.Bvh(scene, n_threads=16)
    bvh_s = time.perf_counter() - t0
    ctx = nh.Context(local)
    t0 = time.perf_counter()
    ctx.upload(scene, bvh)
    upload_s = time.perf_counter() - t0
    trav = nh.TRAVERSAL_ORDERED if a.traversal == "ordered" else nh.TRAVERSAL_REFERENCE
    mode = nh.MODE_WAVEFRONT if a.mode == "wavefront" else nh.MODE_MEGAKERNEL
    if args.scaling == "strong":
        R = a.rounds  # every rank renders the whole sample budget of its 1/N of the blocks
    else:
        R = a.rounds * world  # each rank's 1/N of the image for N x --rounds rounds (weak scaling)
    if a.pools:
        os.environ["NH_POOLS"] = str(a.pools)
    calib = None
    if not a.no_calibrate:
        ctx.reset_stats()
        ctx.render(0, R, seed=a.seed, blocks=blocks, traversal=trav, clear=True, stats=True, mode=mode)
        calib = ctx.stats()
    for w in range(warmup):
        ctx.render(R * (steps + w), R * (steps + w + 1), seed=a.seed, blocks=blocks, traversal=trav,
                   clear=(w == 0), mode=mode)
    ctx.synchronize()
    ctx.reset_stats()
    ctx.render(0, 0, seed=a.seed, blocks=blocks, traversal=trav, clear=True)
    ctx.synchronize()
    if dist is not None:
        dist.barrier()
    t_start = time.perf_counter()
    for s in range(steps):
        ctx.render(s * R, (s + 1) * R, seed=a.seed, blocks=blocks, traversal=trav, clear=False, mode=mode)
    reduced = None
    ranks = None
    if dist is not None:
        ctx.synchronize()  # (the reduce waits for every chunk anyway): the render time of this rank alone
        t_render = time.perf_counter() - t_start
        reduced = reduce_framebuffer(ctx, dist, args, local, rank)
    ctx.synchronize()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        ranks = rank_breakdown(dist, args, local, t_render, elapsed - t_render, ctx.stats()["launches_splat"])
        elapsed = max_over_ranks(elapsed, dist, args, local)
    if args.dump_framebuffer and rank == 0:
        np.save(args.dump_framebuffer, reduced if reduced is not None else ctx.framebuffer())
    st = ctx.stats()
    pools = int(st.get("pools_active", 0)) if a.mode == "wavefront" else 0  # path pools of the timed steps
    # chunks of the timed steps and how many of their tails ran decoupled from their path pool (tail slots)
    chunks = {"chunks": int(st["launches_splat"]), "tails_async": int(st["tails_async"])}
    roof_pass = None
    if a.mode == "wavefront" and a.pools != 1 and calib is not None and a.roofline_steps > 0:
        pools_env = os.environ.get("NH_POOLS")
        # Kernels of overlapping pools share the GPU, so their event durations are no kernel roofline:
        # time the kernels in a serialized pass (one pool) over the same workload instead.
        os.environ["NH_POOLS"] = "1"
        ctx.reset_stats()
        base = R * (steps + warmup)
        for s in range(a.roofline_steps):
            ctx.render(base + s * R, base + (s + 1) * R, seed=a.seed, blocks=blocks, traversal=trav, mode=mode)
        ctx.synchronize()
        st = ctx.stats()
        roof_pass = f"serialized pass: {a.roofline_steps} steps with one path pool (kernels alone on the GPU)"
        if pools_env is None:
            del os.environ["NH_POOLS"]
        else:
            os.environ["NH_POOLS"] = pools_env
    # every rank renders its 1/N of the blocks: the whole job is W x H x R samples per step
    samples = W * H * R * steps
    roof = None
    if calib is not None and calib["samples"] > 0:
        roof = roofline(a, calib, st, W, H, R)
        roof["timed"] = roof_pass or "the timed region"
    return {"scene": scene, "W": W, "H": H, "R": R, "desc": scene_desc, "elapsed": elapsed, "samples": samples,
            "roof": roof, "bvh_s": bvh_s, "upload_s": upload_s, "ctx": ctx, "chunks": chunks,
            "pools": pools, "ranks": ranks}


def reduce_framebuffer(ctx, dist, args, local, rank):
    """One sum-reduce of the RGBW framebuffer to rank 0. Returns rank 0's reduced framebuffer for a host-side
    (gloo) reduce, None otherwise (RCCL reduces in place into rank 0's device framebuffer)."""
    import torch
    ptr, n = ctx.framebuffer_device_ptr()  # completes every submitted chunk first
    try:
        if args.dist_backend == "nccl":
            fb = _wrap_device(ptr, n, local)
            dist.reduce(fb, dst=0, op=dist.ReduceOp.SUM)
            torch.cuda.synchronize()
            return None
        host = ctx.framebuffer()
        fb = torch.from_numpy(host.reshape(-1))
        dist.reduce(fb, dst=0, op=dist.ReduceOp.SUM)
    except Exception as e:  # the RCCL (or gloo) error, then a non-zero exit: no retry
        print(f"bench: rank {rank}: framebuffer reduce ({args.dist_backend}) failed: {e!r}", file=sys.stderr,
              flush=True)
        sys.exit(3)
    return host if rank == 0 else None


def rank_breakdown(dist, args, local, render_s, reduce_s, chunks):
    """Per-rank diagnosis of an N-rank timing (verdict r4 item 7): every rank's render time (its nh_render calls
    until its last chunk is done), the framebuffer reduce alone, and its chunk count, gathered to every rank.
    render + reduce = the rank's timed region; the line's time is the max over ranks of that sum."""
    import torch
    dev = f"cuda:{local}" if args.dist_backend == "nccl" else "cpu"
    mine = torch.tensor([render_s, reduce_s, float(chunks)], dtype=torch.float64, device=dev)
    rows = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(rows, mine)
    rows = [r.cpu().tolist() for r in rows]
    render = [r[0] for r in rows]
    reduce = [r[1] for r in rows]
    total = [a + b for a, b in zip(render, reduce)]
    return {"render_s": [round(x, 6) for x in render], "reduce_s": [round(x, 6) for x in reduce],
            "total_s": [round(x, 6) for x in total], "chunks": [int(r[2]) for r in rows],
            "render_s_min": round(min(render), 6), "render_s_max": round(max(render), 6),
            "reduce_s_max": round(max(reduce), 6),
            "render_imbalance": round(max(render) / min(render), 4) if min(render) > 0 else None}


def max_over_ranks(elapsed, dist, args, local):
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64,
                     device=f"cuda:{local}" if args.dist_backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def denoise_record(nh, ctx, scene, no_cpu):
    """SimpleDenoiser (simple.cpp) on the rendered framebuffer, in place, with denoiser-test.xml's parameters
    (sigma_d 6, sigma_vr 1.5, range 7): GPU time from HIP events; the serial CPU oracle on a 128x128 crop."""
    p = nh.simple_denoiser(6.0, 1.5, 7, 1)
    W, H, b = scene.width, scene.height, scene.border
    crop = None
    if not no_cpu:
        fb = ctx.framebuffer()
        crop = np.ascontiguousarray(fb[:128 + 2 * b, :128 + 2 * b])
    ctx.reset_stats()
    t0 = time.perf_counter()
    ctx.denoise(p)
    wall = time.perf_counter() - t0
    st = ctx.stats()
    ms = st["kernel_ms_denoise"]
    out = {"denoiser": "simple (src/denoiser/simple.cpp), sigma_d 6, sigma_vr 1.5, range 7, 1 pass",
           "image": f"{W}x{H}", "ms": round(ms, 3), "wall_ms": round(wall * 1e3, 3), "launches": st["launches_denoise"],
           "mpixels_s": round(W * H / ms / 1e3, 3),
           "order": "serial-order semantics: the reference's in-place row-major sweep with one TBB thread; parity "
                    "with the multi-threaded reference (whose result depends on its row-chunk race) is unpinned"}
    if crop is not None:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import nori_oracle as no
        gpu_crop = ctx.denoise_image(crop, b, p)
        t0 = time.perf_counter()
        ref_crop = no.denoise_simple(crop, b, p)
        dt = time.perf_counter() - t0
        # libm drift (the exp() step, double precision on both sides) would show here
        out["exact_fraction_vs_oracle"] = round(float(np.mean(gpu_crop == ref_crop)), 6)
        out["cpu_baseline"] = {"mpixels_s": round(128 * 128 / dt / 1e6, 4), "cores": 1, "kind": "port",
                               "sample": f"128x128 crop of the same framebuffer ({dt:.2f} s), oracle "
                                         "no_denoise_simple, one thread (the reference's loop order)"}
    return out


def traversal_1m(nh, args, local):
    """perf-1M: the north star's traversal roofline target is set on the BVH-traversal
    kernel of the ~1M-triangle scene at 1 GPU; measured here in the same run (a short bench of it)."""
    a = argparse.Namespace(**vars(args))
    a.dump_framebuffer = None
    r = run_workload(nh, a, "bumpy1m", args.traversal_1m_steps, 1, local)
    roof = r["roof"]
    stage = "trace" if "trace" in roof["stages"] else "extend"
    e = roof["stages"][stage]
    key1m = f"bumpy1m_{r['W']}x{r['H']}_r{r['R']}_{args.traversal}_{args.mode}/{stage}"
    traffic, source = pmc_traffic(key1m)
    rec1m = pmc_record(key1m)
    out = {"workload": r["desc"], "msamples_s": round(r["samples"] / r["elapsed"] / 1e6, 3),
           "kernel": ({"trace": "wf_trace_pt2 (persistent %d-wide closest-hit + any-hit traversal, one launch per bounce)",
                       "extend": "wf_trace_pt (persistent %d-wide closest-hit traversal)"}[stage] % (roof["node_bytes"] // 32)
                      if roof["node_bytes"] in (128, 256) else "wf_extend"),
           "avg_launch_ms": e["avg_launch_ms"], "algorithmic_bytes_per_launch": e["global_bytes_per_launch"],
           "achieved_gbs": e["global_gbs"], "frac": round(e["global_gbs"] / HBM_PEAK_GBS, 4), "target_frac": 0.40,
           "nodes_per_query": e.get("nodes_per_query"), "prims_per_query": e.get("prims_per_query"),
           "node_bytes": roof["node_bytes"],
           "bytes": "algorithmic: nodes x node_bytes + primitive tests x 48 B + the queue bytes (ray in, hit / occlusion "
                    "out) per query",
           "traffic": traffic, "traffic_source": source or "not collected for this workload",
           "traffic_gbs": round(traffic / (e["avg_launch_ms"] * 1e-3) / 1e9, 1) if traffic else None,
           "l2_hit_rate": rec1m.get("l2_hit_rate"),
           "limiter": (limiter_record(rec1m, key1m, e["avg_launch_ms"], 5) if rec1m.get("valu_issue_frac") is not None
                       else None),
           "note": "the ~176 MB tree is resident in the 256 MB MALL: measured HBM traffic (traffic) is well below "
                   "the algorithmic bytes; this kernel is bound by dependent-load latency",
           "steps": args.traversal_1m_steps, "spp": r["R"] * args.traversal_1m_steps, "timed": roof["timed"]}
    r["ctx"].close()
    return out


def strong_c4_record(nh, args, world, rank, local, dist):
    """The north star's >= 6x scaling target on its own configuration (BASELINE configs[3]): the
    fixed C4 image (2048^2 Cornell box, mirror + dielectric spheres, area light, path_mis) at --strong-spp spp,
    32x32 blocks dealt round-robin to the ranks (the reference's fixed sample budget, render.cpp:281-347, split
    by tile). Each rank renders all spp of its blocks in one nh_render call (the library chunks it), then the RCCL
    reduce of the framebuffer to rank 0 -- both inside the timed region; max over ranks. A first identical call
    (untimed) sizes the path pools for the same chunks."""
    a = argparse.Namespace(**vars(args))
    a.config, a.width, a.height = "c4", None, None
    tmp = tempfile.mkdtemp(prefix="nh_strong_")
    xml, W, H, desc = build_scene(a, tmp)
    scene = nh.Scene(xml)
    bvh = nh.Bvh(scene, n_threads=16)
    ctx = nh.Context(local)
    ctx.upload(scene, bvh)
    blocks = nh.tile_shard(W, H, world, rank) if world > 1 else None
    spp = args.strong_spp
    trav = nh.TRAVERSAL_ORDERED if args.traversal == "ordered" else nh.TRAVERSAL_REFERENCE
    ctx.render(spp, 2 * spp, seed=args.seed, blocks=blocks, traversal=trav, clear=True, mode=nh.MODE_WAVEFRONT)
    ctx.render(0, 0, seed=args.seed, blocks=blocks, traversal=trav, clear=True)
    ctx.synchronize()
    ctx.reset_stats()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    ctx.render(0, spp, seed=args.seed, blocks=blocks, traversal=trav, clear=False, mode=nh.MODE_WAVEFRONT)
    ranks = None
    if dist is not None:
        ctx.synchronize()
        t_render = time.perf_counter() - t0
        reduce_framebuffer(ctx, dist, args, local, rank)
    ctx.synchronize()
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    if dist is not None:
        ranks = rank_breakdown(dist, args, local, t_render, elapsed - t_render, st["launches_splat"])
        elapsed = max_over_ranks(elapsed, dist, args, local)
    ctx.close()
    samples = W * H * spp
    return {"workload": f"{desc}, {spp} spp, path_mis (fixed image, BASELINE configs[3])", "n_gpus": world,
            "spp": spp, "samples": samples, "ms": round(elapsed * 1e3, 3),
            "msamples_s": round(samples / elapsed / 1e6, 3), "scaling": "strong",
            "partition": f"32x32 blocks round-robin over {world} rank(s), one nh_render call each"
                         + (f" + {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} reduce" if world > 1 else ""),
            "chunks_rank0": int(st["launches_splat"]), "pools_rank0": int(st.get("pools_active", 0)),
            "ranks": ranks}


def megakernel_record(nh, args, local):
    """BASELINE configs[1] names "megakernel vs wavefront": the same C2 workload through nh_path_kernel (one thread
    per (pixel, round) runs the whole path_mis loop), --rounds rounds per step."""
    a = argparse.Namespace(**vars(args))
    a.mode, a.dump_framebuffer, a.no_calibrate, a.pools = "megakernel", None, True, 0
    r = run_workload(nh, a, "c2", 2, 1, local)
    st = r["ctx"].stats()
    r["ctx"].close()
    return {"workload": f"{r['desc']}, {r['R'] * 2} spp, path_mis", "mode": "megakernel",
            "msamples_s": round(r["samples"] / r["elapsed"] / 1e6, 3),
            "ms_per_step": round(r["elapsed"] / 2 * 1e3, 3),
            "path_kernel_ms_per_launch": round(st["kernel_ms_path"] / max(st["launches_path"], 1), 4)}


def denoiser_test_record(nh, local):
    """scenes/project/denoiser/denoiser-test.xml (tests/golden/textured_scenes.json.gz: 800x600, checkerboard_color
    floor, curvy bowl, two area lights, SimpleDenoiser sigma_d 6 / sigma_vr 1.5 / range 7), timed as the reference's
    report states its numbers (reports/project-report/denoising.html:79-81): the 1024 spp ground truth ("It took 5
    minutes"), the 16 spp input ("roughly 20 seconds") and the denoise ("about one second"). The authors' machine is
    not stated; the published figures are quoted as given."""
    import scenegen
    d = scenegen.materialize(tempfile.mkdtemp(prefix="nh_dn_"))
    scene = nh.Scene(os.path.join(d, "scenes/project/denoiser/denoiser-test.xml"))
    W, H = scene.width, scene.height
    bvh = nh.Bvh(scene, n_threads=16)
    ctx = nh.Context(local)
    ctx.upload(scene, bvh)
    trav, mode = nh.TRAVERSAL_ORDERED, nh.MODE_WAVEFRONT
    ctx.render(0, 1024, seed=1, traversal=trav, clear=True, mode=mode)  # warm: pools sized for the same chunks
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.render(0, 1024, seed=2, traversal=trav, clear=True, mode=mode)
    ctx.synchronize()
    t_gt = time.perf_counter() - t0
    t0 = time.perf_counter()
    ctx.render(0, 16, seed=3, traversal=trav, clear=True, mode=mode)
    ctx.synchronize()
    t16 = time.perf_counter() - t0
    ctx.reset_stats()
    t0 = time.perf_counter()
    ctx.denoise()
    t_dn = time.perf_counter() - t0
    ms_dn = ctx.stats()["kernel_ms_denoise"]
    ctx.close()
    pub_gt, pub_16 = 5 * 60.0, 20.0
    return {"scene": "scenes/project/denoiser/denoiser-test.xml", "image": f"{W}x{H}", "integrator": "path_mis",
            "textures": "checkerboard_color albedo (floor)",
            "groundtruth_1024spp_s": round(t_gt, 4), "groundtruth_msamples_s": round(W * H * 1024 / t_gt / 1e6, 3),
            "input_16spp_s": round(t16, 4), "denoise_s": round(t_dn, 4), "denoise_kernel_ms": round(ms_dn, 3),
            "published": {"groundtruth_1024spp_s": pub_gt, "input_16spp_s": pub_16, "denoise_s": 1.0,
                          "groundtruth_msamples_s": round(W * H * 1024 / pub_gt / 1e6, 3),
                          "source": "reports/project-report/denoising.html:79-81 (Nori CPU path_mis; machine not "
                                    "stated)"},
            "speedup_groundtruth": round(pub_gt / t_gt, 1)}


def project_scenes_record(nh, local):
    """The reference's own project scenes at their own resolution and sample count (tests/golden/project_scenes.json.gz),
    one warm render then one timed render each: the envmap scene (envmap_sphere.xml, the shipped wooden_motel.png,
    800x800, 128 spp) and the two thin-lens scenes (dof-val.xml 800x400 256 spp, table_path_mis.xml 800x600 512 spp:
    lens samples in the serial render order, nh_shade.h lens_uniform)."""
    import scenegen
    d = scenegen.materialize(tempfile.mkdtemp(prefix="nh_proj_"))
    out = {}
    for key, rel in (("envmap_sphere", "scenes/project/envmap/envmap_sphere.xml"),
                     ("dof_val", "scenes/project/dof/dof-val.xml"),
                     ("dof_table", "scenes/project/dof/table_path_mis.xml")):
        scene = nh.Scene(os.path.join(d, rel))
        W, H, spp = scene.width, scene.height, scene.spp
        bvh = nh.Bvh(scene, n_threads=16)
        ctx = nh.Context(local)
        ctx.upload(scene, bvh)
        trav, mode = nh.TRAVERSAL_ORDERED, nh.MODE_WAVEFRONT
        ctx.render(0, spp, seed=1, traversal=trav, clear=True, mode=mode)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.render(0, spp, seed=2, traversal=trav, clear=True, mode=mode)
        ctx.synchronize()
        t = time.perf_counter() - t0
        ctx.close()
        out[key] = {"scene": rel, "image": f"{W}x{H}", "spp": spp, "s": round(t, 4),
                    "msamples_s": round(W * H * spp / t / 1e6, 3)}
    return out


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher around it: start N ranks (one process per GPU) as a
    child torch.distributed.run and exit with its status. Runs before anything touches torch.cuda or the HIP
    library, and starts a child rather than exec'ing."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL between the rank processes
    return subprocess.run(cmd, env=env).returncode


def launcher_selftest(args):
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([float(dist.get_rank())])
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"n_gpus": dist.get_world_size(), "rank_sum": float(t.item()),
                          "gpus_arg": args.gpus}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    args = parse()
    # one hardware queue per path-pool stream: the benchmark's own configuration (the GPU box exports HIP's default
    # of 4, with which two pool streams share a queue and one pool's tail blocks another's bounces: C1 -15 %,
    # profiles/round4_session3_ab.txt). Raised before torch may initialise the HIP runtime in a multi-rank run (the
    # binding's nori_hip.configure_runtime() raises it the same way); the line records the value.
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
        os.environ["NH_KEEP_HW_QUEUES"] = "1"
    else:
        raise_hw_queues()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: using the launcher's world size", file=sys.stderr)
    if args.launcher_selftest:
        return launcher_selftest(args)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        try:
            if args.dist_backend == "nccl":
                torch.cuda.set_device(local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                local = 0  # rehearsal: every rank on GPU 0
                dist.init_process_group("gloo")
        except Exception as e:  # no retry, no re-exec: the run fails with the backend's own error
            print(f"bench: rank {rank}: init_process_group({args.dist_backend}) failed: {e!r}", file=sys.stderr,
                  flush=True)
            sys.exit(3)
    import nori_hip as nh

    if args.scaling == "strong" and args.config == "c2" and not args.config_given:
        args.config = "c4"  # the north star's scaling target: a fixed C4 image split over the ranks
    W, H = scene_dims(args)
    blocks = nh.tile_shard(W, H, world, rank) if world > 1 else None
    r = run_workload(nh, args, args.config, args.steps, args.warmup, local, blocks=blocks, world=world, rank=rank,
                     dist=dist)
    strong = None
    if args.strong_spp > 0 and not (args.scaling == "strong" and args.config == "c4"):
        strong = strong_c4_record(nh, args, world, rank, local, dist)
    if rank == 0:
        W, H, R = r["W"], r["H"], r["R"]
        value = r["samples"] / r["elapsed"] / 1e6
        roof = r["roof"]
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(r["scene"], args.cpu_seconds, args.seed)
        dn = None
        if world == 1 and not args.no_denoise:
            dn = denoise_record(nh, r["ctx"], r["scene"], args.no_cpu)
        t1m = None
        if world == 1 and args.traversal_1m_steps > 0 and args.config != "bumpy1m":
            r["ctx"].close()
            t1m = traversal_1m(nh, args, local)
        mk = dn_scene = proj = None
        if world == 1 and not args.no_extras:
            r["ctx"].close()
            if args.mode == "wavefront":
                mk = megakernel_record(nh, args, local)
            dn_scene = denoiser_test_record(nh, local)
            proj = project_scenes_record(nh, local)
        spp = R * args.steps
        if args.scaling == "strong":
            par = f"tile-shard x{world}, strong scaling: fixed {W}x{H} image, {spp} spp split by blocks"
        else:
            par = f"tile-shard x{world}, weak scaling: each rank {R} rounds per step over its 1/{world} of the blocks"
        line = {
            "metric": "Msamples/sec (whole node) + traversal HBM GB/s, cbox 1024x1024 256spp",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference Cornell box scene files, generated meshes, per-path pcg32 seeds)",
            "config": {"workload": f"{r['desc']}, {spp} spp, path_mis", "config": args.config,
                       "width": W, "height": H, "spp": spp, "rounds_per_step": R,
                       "mode": args.mode, "traversal": args.traversal,
                       "pools": r["pools"] or None,
                       "gpu_max_hw_queues": parse_hw_queues(os.environ.get("GPU_MAX_HW_QUEUES")),
                       "parallelism": (f"{par} + {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} reduce"
                                       if world > 1 else "single GPU"),
                       "bvh_build_s": round(r["bvh_s"], 3), "upload_s": round(r["upload_s"], 3),
                       "timed_chunks": r["chunks"]},
            "ranks": r["ranks"],
            "roofline": roof,
            "traversal": traversal_record(roof) if roof else None,
            "traversal_1m": t1m,
            "cpu_baseline": cpu,
            "denoise": dn,
            "strong_c4": strong,
            "megakernel": mk,
            "denoiser_test": dn_scene,
            "project_scenes": proj,
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
