"""Multi-process row splits on CPU (gloo, world_size 2 and 3): the host logic bench.py uses for
N GPUs — interleaved rows or bands, max/sum over ranks, and the host gather of ARGB rows — with
the CPU oracle standing in for each rank's GPU render (test infrastructure only)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from hippt import distributed as hd
from hippt import scenes

W, H, SPP, DEPTH = 40, 27, 2, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir, split="bands"):
    import pyoracle as po
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ms = po.MeshScene(scenes.cornell34(), W, H)
        if split == "bands":
            y0, y1 = hd.row_band(rank, world, H)
            px, acc, segs, samples = ms.frames(0, SPP, DEPTH, y0=y0, y1=y1, nthreads=1)
            full_px = hd.gather_bands(px, H, dist)
            full_acc = hd.gather_bands(acc, H, dist)
        else:  # interleaved rows rank, rank+N, ...: one oracle row at a time
            parts = [ms.frames(0, SPP, DEPTH, y0=int(y), y1=int(y) + 1, nthreads=1)
                     for y in hd.interleaved_rows(rank, world, H)]
            px = np.concatenate([p[0] for p in parts])
            acc = np.concatenate([p[1] for p in parts])
            segs = sum(p[2] for p in parts)
            full_px = hd.gather_interleaved(px, H, dist)
            full_acc = hd.gather_interleaved(acc, H, dist)
        total_segs = hd.sum_over_ranks(segs, dist)
        slowest = hd.max_over_ranks(float(rank + 1), dist)
        # bench.py's per-rank bookkeeping (kernel ms, wall ms per step) on every rank
        per_rank = hd.gather_floats((rank + 0.5, 2.0 * rank), dist)
        assert per_rank == [[r + 0.5, 2.0 * r] for r in range(world)]
        if rank == 0:
            np.save(os.path.join(out_dir, "px.npy"), full_px)
            np.save(os.path.join(out_dir, "acc.npy"), full_acc)
            np.save(os.path.join(out_dir, "meta.npy"), np.array([total_segs, slowest], np.float64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,split", [(2, "bands"), (3, "bands"), (2, "interleave"), (3, "interleave")])
def test_row_split_gathers_to_single_process_image(tmp_path, world, split):
    import pyoracle as po
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), split), nprocs=world, join=True,
                       start_method="spawn")
    px = np.load(tmp_path / "px.npy")
    acc = np.load(tmp_path / "acc.npy")
    total_segs, slowest = np.load(tmp_path / "meta.npy")
    ref_px, ref_acc, ref_segs, _ = po.MeshScene(scenes.cornell34(), W, H).frames(0, SPP, DEPTH, nthreads=1)
    assert np.array_equal(px, ref_px)
    assert acc.tobytes() == ref_acc.tobytes()
    assert int(total_segs) == ref_segs
    assert slowest == float(world)


def test_row_band_partition_covers_image():
    for world in (1, 2, 3, 4, 8):
        for h in (1, 7, 1080, 2160):
            bands = [hd.row_band(r, world, h) for r in range(world)]
            assert bands[0][0] == 0 and bands[-1][1] == h
            assert all(bands[i][1] == bands[i + 1][0] for i in range(world - 1))
    with pytest.raises(ValueError):
        hd.row_band(2, 2, 10)


def test_interleaved_rows_partition_image():
    for world in (1, 2, 3, 8):
        for h in (1, 7, 1080):
            rows = np.concatenate([hd.interleaved_rows(r, world, h) for r in range(world)])
            assert np.array_equal(np.sort(rows), np.arange(h))


def test_gather_without_process_group_is_identity():
    a = np.arange(12, dtype=np.uint32).reshape(3, 4)
    assert hd.gather_bands(a, 3) is a
    assert hd.max_over_ranks(2.5) == 2.5 and hd.sum_over_ranks(7) == 7
    assert hd.gather_floats((1, 2.5)) == [[1.0, 2.5]]
