"""Multi-rank tile sharding + framebuffer reduce on CPU (gloo, world size 2).

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


def test_tile_shard_reduce_world2(tmp_path):
    sys.path.insert(0, os.path.join(REPO, "optix-renderer_amd"))
    import nori_hip as nh
    import nori_oracle as no
    import scenegen
    xml = scenegen.cbox_xml(str(tmp_path), "c1", width=100, height=70)
    shards = [nh.tile_shard(100, 70, 2, r) for r in range(2)]
    assert sorted(shards[0] + shards[1]) == list(range(4 * 3)) and not set(shards[0]) & set(shards[1])
    out = str(tmp_path / "reduced.npy")
    port = 29500 + os.getpid() % 1000
    mp.spawn(_worker, args=(2, xml, out, port), nprocs=2, join=True)
    reduced = np.load(out)
    full = no.OracleScene(nh.Scene(xml)).render(0, 4, seed=21, threads=4)
    err = np.sqrt(((reduced.astype(np.float64) - full) ** 2).sum() / (full.astype(np.float64) ** 2).sum())
    assert err < 1e-6, err
