"""The group launch's item mapping (hippt_kernels.hip, the CHAIN regen loop): a group
of nb chained batches is one job of nb * total queue positions; position m is 64-item block
m >> 6 = q * nb + b of batch own + b, at position (q << 6) | (m & 63) of that batch's item order.
A restatement of that formula (host-side, no GPU): it must hand out every (batch, position) exactly
once, and a queue's share of the group must cover the same positions of the one-batch order in
every batch, so that each queue walks the one-batch cost order once for the whole group."""
import numpy as np
import pytest


def group_map(m, nb):
    blk = m >> 6
    q = blk // nb
    return blk - q * nb, (q << 6) | (m & 63)


def queue_start(total, g, queues=8):
    return total * g // queues


@pytest.mark.parametrize("nb", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("total", [64 * 45, 64 * 8 * 37, 1920 * 64])
def test_group_positions_are_a_bijection(nb, total):
    assert total % 64 == 0
    m = np.arange(nb * total, dtype=np.int64)
    b, pos = group_map(m, nb)
    assert b.min() == 0 and b.max() == nb - 1 and pos.min() == 0 and pos.max() == total - 1
    flat = b * total + pos
    assert np.array_equal(np.sort(flat), np.arange(nb * total))


@pytest.mark.parametrize("nb", [2, 3, 8])
def test_group_queue_covers_the_one_batch_queue_in_every_batch(nb):
    total = 1920 * 135 * 64  # the 1/8 row share at 64 spp: every queue boundary a multiple of 64
    for g in range(8):
        lo, hi = queue_start(nb * total, g), queue_start(nb * total, g + 1)
        m = np.arange(lo, hi, dtype=np.int64)
        b, pos = group_map(m, nb)
        one_lo, one_hi = queue_start(total, g), queue_start(total, g + 1)
        assert pos.min() == one_lo and pos.max() == one_hi - 1
        for k in range(nb):
            assert np.count_nonzero(b == k) == one_hi - one_lo
