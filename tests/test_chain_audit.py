"""The chained-batch audit's host check (tests/chain_audit.py) on synthetic records: an exact run passes,
and each way a chained run can go wrong (the GPUTEST_r05 failure: a batch's items traced with another
batch's frames; an item traced twice or not at all; a batch combined twice, early or out of order) is
reported.  The GPU fixture runs the same check after every test (tests/test_gpu_parity.py).  No GPU."""
import numpy as np

import chain_audit as ca


def test_hash_sum_matches_a_direct_sum():
    i = np.arange(1000, dtype=np.uint32)
    assert ca.hash_sum(1000) == int(ca.hash32(i ^ np.uint32(0x5BD1E995)).astype(np.uint64).sum())
    assert ca.hash32(np.array([0], np.uint32))[0] == 0
    # the RNG hash of CudaPathTracerKernel.cu:23-30, as the oracle restates it (oracle/pt_oracle.c)
    import pyoracle as po
    for x in (1, 0x5BD1E995, 123456789, 0xFFFFFFFF):
        assert int(ca.hash32(np.array([x], np.uint32))[0]) == po.lib().po_hash32(x)


def test_exact_runs_pass():
    assert ca.check([ca.synthetic_run()]) == []
    assert ca.check([ca.synthetic_run(batches=1, launches=1)]) == []
    assert ca.check([ca.synthetic_run(step=0, trace_epochs=[0, 0, 1, 1, 2], comb_epochs=[1, 1, 2, 3, 3])]) == []


def test_wrong_frames_are_reported():
    hdr, recs = ca.synthetic_run()
    recs[2, 6] = hdr["firstFrame"] + 1  # batch 2's items traced with batch 0's first frame (max)
    bad = ca.check([(hdr, recs)])
    assert any("batch 2/5: traced with first frames" in b for b in bad), bad


def test_missing_or_repeated_items_are_reported():
    hdr, recs = ca.synthetic_run()
    recs[1, 0] -= 1
    assert any("batch 1/5: traced" in b for b in ca.check([(hdr, recs)]))
    hdr, recs = ca.synthetic_run()
    recs[3, 2] ^= 1  # same count, another item set
    assert any("hash differs" in b for b in ca.check([(hdr, recs)]))


def test_bad_combines_are_reported():
    hdr, recs = ca.synthetic_run()
    recs[0, 1] *= 2
    assert any("combined" in b for b in ca.check([(hdr, recs)]))
    hdr, recs = ca.synthetic_run(trace_epochs=[0, 1, 1, 2, 2], comb_epochs=[1, 1, 2, 3, 3])
    assert any("not after the launch that traced it" in b for b in ca.check([(hdr, recs)]))
    hdr, recs = ca.synthetic_run(trace_epochs=[0, 0, 0, 0, 0], comb_epochs=[2, 1, 3, 3, 3])
    assert any("before batch 0" in b for b in ca.check([(hdr, recs)]))
