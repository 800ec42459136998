"""The pair splat's pixel classes (csrc/nh_splat.hip: tab_body<.., PAIR>, nh_corner_merge_kernel), restated on the CPU.

Every master pixel with at least one covering block must be finished by exactly one writer:
  - one covering block: that block's workgroup (either launch);
  - two side-by-side covering blocks (different colours (bx + by) & 1): the odd block's workgroup;
  - anything else (3-4 blocks, or two diagonal ones): nh_corner_merge_kernel, whose grid covers only the 4x4 squares at
    the interior block corners (32 cx .. 32 cx + 3, 32 cy .. 32 cy + 3 for 1 <= cx < nbx, 1 <= cy < nby).
The last point is the invariant the corner kernel's grid relies on; it is checked here over image sizes with partial
last blocks and over block subsets (multi-GPU tile shards, arbitrary holes). covering_blocks follows the kernel's: a
rendered block (bx, by) covers master columns 32 bx .. 32 bx + sxb + 3 and rows alike (border 2).
"""
import numpy as np
import pytest


def classes(width, height, rendered):
    nbx, nby = (width + 31) // 32, (height + 31) // 32
    mcols, mrows = width + 4, height + 4
    cover = [[[] for _ in range(mcols)] for _ in range(mrows)]
    for bid in rendered:
        by, bx = divmod(bid, nbx)
        sxb, syb = min(32, width - 32 * bx), min(32, height - 32 * by)
        for my in range(32 * by, 32 * by + syb + 4):
            for mx in range(32 * bx, 32 * bx + sxb + 4):
                cover[my][mx].append((bx, by))
    return nbx, nby, cover


def check(width, height, rendered):
    nbx, nby, cover = classes(width, height, rendered)
    corner_px = set()
    for cy in range(1, nby):
        for cx in range(1, nbx):
            for dy in range(4):
                for dx in range(4):
                    corner_px.add((32 * cx + dx, 32 * cy + dy))
    for my, row in enumerate(cover):
        for mx, blocks in enumerate(row):
            if len(blocks) <= 1:
                continue
            par = sum((bx + by) & 1 for bx, by in blocks)
            if len(blocks) == 2 and par == 1:
                (ax, ay), (bx, by) = blocks
                assert abs(ax - bx) + abs(ay - by) == 1, (mx, my, blocks)  # side by side, never diagonal
                continue
            assert (mx, my) in corner_px, (width, height, mx, my, blocks)


@pytest.mark.parametrize("width,height", [(64, 64), (100, 70), (33, 31), (200, 40), (96, 96), (160, 96), (130, 67)])
def test_every_band_pixel_has_one_finisher(width, height):
    nbx, nby = (width + 31) // 32, (height + 31) // 32
    everything = list(range(nbx * nby))
    check(width, height, everything)
    rng = np.random.default_rng(width * 1000 + height)
    for world in (2, 3, 4):  # tile shards (round-robin, as nori_hip.tile_shard) and random subsets
        for r in range(world):
            check(width, height, everything[r::world])
        for _ in range(4):
            keep = [b for b in everything if rng.random() < 0.6]
            check(width, height, keep)
