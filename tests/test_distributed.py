"""Multi-rank tile sharding + framebuffer reduce on CPU (gloo, world sizes 2 and 4).

Each rank renders its round-robin share of 32x32 blocks (nori_hip.tile_shard, as bench.py
does per GPU) into a full-size RGBW framebuffer; a sum-reduce to rank 0 must equal the
single-process render up to fp32 summation order at block borders.
The CPU oracle stands in for the GPU render here; the GPU version of the same check is
tests/test_gpu_parity.py::test_render_deterministic_and_sharded.
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, xml, out_path, port):
    sys.path.insert(0, os.path.join(REPO, "optix-renderer_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import nori_hip as nh
    import nori_oracle as no
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = nh.Scene(xml)
    o = no.OracleScene(s)
    blocks = nh.tile_shard(o.width, o.height, world, rank)
    fb = torch.from_numpy(o.render(0, 4, seed=21, blocks=blocks, threads=2))
    dist.reduce(fb, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(out_path, fb.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tile_shard_reduce(tmp_path, world):
    sys.path.insert(0, os.path.join(REPO, "optix-renderer_amd"))
    import nori_hip as nh
    import nori_oracle as no
    import scenegen
    xml = scenegen.cbox_xml(str(tmp_path), "c1", width=100, height=70)
    shards = [nh.tile_shard(100, 70, world, r) for r in range(world)]
    assert sorted(sum(shards, [])) == list(range(4 * 3)) and all(shards)
    assert sum(len(x) for x in shards) == len(set(sum(shards, [])))
    out = str(tmp_path / "reduced.npy")
    port = 29500 + (os.getpid() + 7 * world) % 1000
    mp.spawn(_worker, args=(world, xml, out, port), nprocs=world, join=True)
    reduced = np.load(out)
    full = no.OracleScene(nh.Scene(xml)).render(0, 4, seed=21, threads=4)
    err = np.sqrt(((reduced.astype(np.float64) - full) ** 2).sum() / (full.astype(np.float64) ** 2).sum())
    assert err < 1e-6, err


def _bench(args, timeout=600):
    import json
    import subprocess
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=REPO)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def check_rank_breakdown(rk, elapsed_s, world=2):
    """The N>1 diagnosis (verdict r4 item 7): per-rank render and reduce times and chunk counts, consistent with
    the line's own time (= the max over ranks of render + reduce)."""
    for key in ("render_s", "reduce_s", "total_s", "chunks"):
        assert len(rk[key]) == world, rk
    assert all(c >= 1 for c in rk["chunks"]) and all(x >= 0 for x in rk["reduce_s"]), rk
    for a, b, t in zip(rk["render_s"], rk["reduce_s"], rk["total_s"]):
        assert abs(a + b - t) < 1e-5, rk
    assert rk["render_s_min"] == min(rk["render_s"]) and rk["render_s_max"] == max(rk["render_s"])
    assert rk["reduce_s_max"] == max(rk["reduce_s"])
    assert abs(max(rk["total_s"]) - elapsed_s) <= 2e-3 * max(1.0, elapsed_s) + 1e-3, (rk, elapsed_s)


def test_bench_gpus_n_launches_n_ranks():
    """`python bench.py --gpus 2` with no launcher around it starts two ranks itself (a child
    torch.distributed.run); here only their rendezvous runs (gloo, no GPU)."""
    line = _bench(["--gpus", "2", "--dist-backend", "gloo", "--launcher-selftest"], timeout=300)
    assert line["n_gpus"] == 2 and line["rank_sum"] == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_bench_hip_ranks_reduce_to_one_rank_render(tmp_path, gpu, world):
    """bench.py --gpus 2 / 8: every rank renders its tile shard with the HIP path (gloo reduce, all on GPU 0: the
    driver's 8-rank launch rehearsed on one card);
    the reduced framebuffer equals one HIP render of the whole image over the same sample range
    (src/utils/render.cpp:281-347 semantics: the samples of a block do not depend on who renders it), up to
    fp32 summation order where block footprints overlap."""
    sys.path.insert(0, os.path.join(REPO, "optix-renderer_amd"))
    import nori_hip as nh
    import scenegen
    out = str(tmp_path / "reduced.npy")
    line = _bench(["--gpus", str(world), "--dist-backend", "gloo", "--config", "c2", "--width", "160", "--height",
                   "96", "--rounds", "2", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-denoise",
                   "--traversal-1m-steps", "0", "--roofline-steps", "0", "--strong-spp", "0", "--no-extras",
                   "--dump-framebuffer", out])
    assert line["n_gpus"] == world and line["value"] > 0
    check_rank_breakdown(line["ranks"], line["ms_per_step"] * line["steps"] / 1e3, world)
    reduced = np.load(out).astype(np.float64)
    xml = scenegen.cbox_xml(str(tmp_path), "c2", width=160, height=96)
    s = nh.Scene(xml)
    ctx = nh.Context(0)
    ctx.upload(s, nh.Bvh(s))
    R = 2 * world  # --rounds x world: each rank's weak-scaling step
    ctx.render(0, 2 * R, seed=1234, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=nh.MODE_WAVEFRONT)
    full = ctx.framebuffer().astype(np.float64)
    ctx.close()
    err = np.sqrt(((reduced - full) ** 2).sum() / (full ** 2).sum())
    assert err < 1e-6, err


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_bench_hip_ranks_strong_scaling_equals_one_rank_render(tmp_path, gpu, world):
    """bench.py --gpus 2 / 4 --scaling strong (every rank a HIP context on GPU 0, gloo reduce): a fixed image (the mirror + dielectric Cornell box, C4's scene at test
    size) whose --rounds x --steps spp are split over the ranks by blocks; the reduced framebuffer equals one HIP
    render of the whole image over the same samples (render.cpp:281-347: the sample budget of a block does not
    depend on the rank that renders it), up to fp32 summation order where block footprints overlap. Also runs the
    strong_c4 sub-record's code path (a small --strong-spp) on both ranks."""
    sys.path.insert(0, os.path.join(REPO, "optix-renderer_amd"))
    import nori_hip as nh
    import scenegen
    out = str(tmp_path / "reduced.npy")
    line = _bench(["--gpus", str(world), "--dist-backend", "gloo", "--scaling", "strong", "--config", "c1", "--width",
                   "160", "--height", "96", "--rounds", "3", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-denoise",
                   "--traversal-1m-steps", "0", "--roofline-steps", "0", "--strong-spp", "2", "--no-extras",
                   "--dump-framebuffer", out])
    assert line["n_gpus"] == world and line["scaling"] == "strong" and line["config"]["spp"] == 6
    sc = line["strong_c4"]
    assert sc["n_gpus"] == world and sc["spp"] == 2 and sc["msamples_s"] > 0
    check_rank_breakdown(line["ranks"], line["ms_per_step"] * line["steps"] / 1e3, world)
    check_rank_breakdown(sc["ranks"], sc["ms"] / 1e3, world)
    reduced = np.load(out).astype(np.float64)
    xml = scenegen.cbox_xml(str(tmp_path), "c1", width=160, height=96)
    s = nh.Scene(xml)
    ctx = nh.Context(0)
    ctx.upload(s, nh.Bvh(s))
    ctx.render(0, 6, seed=1234, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=nh.MODE_WAVEFRONT)
    full = ctx.framebuffer().astype(np.float64)
    ctx.close()
    err = np.sqrt(((reduced - full) ** 2).sum() / (full ** 2).sum())
    assert err < 1e-6, err


_RCCL_ONE_RANK = r'''
import os, sys, types
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["NH_REPO"])
import bench
import nori_hip as nh
import scenegen
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ["NH_PORT"], RANK="0", WORLD_SIZE="1")
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
xml = scenegen.cbox_xml(os.environ["NH_TMP"], "c2", width=96, height=64)
s = nh.Scene(xml)
ctx = nh.Context(0)
ctx.upload(s, nh.Bvh(s))
ctx.render(0, 4, seed=5, clear=True)
before = ctx.framebuffer().copy()
args = types.SimpleNamespace(dist_backend="nccl")
assert bench.reduce_framebuffer(ctx, dist, args, 0, 0) is None  # RCCL: in place on the device framebuffer
after = ctx.framebuffer()
rk = bench.rank_breakdown(dist, args, 0, 0.25, 0.5, 3)
mx = bench.max_over_ranks(1.5, dist, args, 0)
dist.destroy_process_group()
assert np.array_equal(before, after), "a one-rank sum-reduce must leave the framebuffer as it is"
assert rk["total_s"] == [0.75] and rk["chunks"] == [3] and mx == 1.5, (rk, mx)
print("rccl-one-rank ok", float(np.abs(after).sum()))
'''


@pytest.mark.gpu
def test_bench_rccl_collectives_one_rank(tmp_path, gpu):
    """bench.py's RCCL legs on the GPU with a one-rank NCCL (= RCCL) process group: the in-place dist.reduce of the
    wrapped device framebuffer (reduce_framebuffer), the all_gather of the rank breakdown and the all_reduce MAX of
    the step time -- the same calls an N-rank run makes, executed by RCCL on this box's single card."""
    import subprocess
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", NH_REPO=REPO, NH_TMP=str(tmp_path),
               NH_PORT=str(29700 + os.getpid() % 200),
               PYTHONPATH=os.pathsep.join([REPO, os.path.join(REPO, "optix-renderer_amd")]))
    p = subprocess.run([sys.executable, "-c", _RCCL_ONE_RANK], capture_output=True, text=True, timeout=240, env=env,
                       cwd=REPO)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "rccl-one-rank ok" in p.stdout
