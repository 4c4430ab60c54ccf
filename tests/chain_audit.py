"""Host check of the chained-batch audit (HIPPT_OPT_CHAIN_AUDIT, include/hippt.h hipptChainAudit): what the
device recorded per batch of each closed run against what the run asked for.  The contract is the
reference's accumulation (CudaPathTracerKernel.cu:157-178): every sample of every frame blended once,
in frame order.  Per batch b of a run: every item traced exactly once (count and a 64-bit sum of a hash
of the item indices), by one launch, with the batch's own first frame (batch 0's first frame + b x
step); every pixel combined exactly once (count and hash sum), by one launch later than the one that
traced the batch, with the same frames; and the combines in batch order (the combining launch never
decreases with b).  Test infrastructure (used by the GPU tests' fixture and tests/test_chain_audit.py).
"""
import functools

import numpy as np

MASK64 = (1 << 64) - 1


def hash32(x: np.ndarray) -> np.ndarray:
    """hippt_trace.h hash32 (CudaPathTracerKernel.cu:23-30) over uint32 arrays."""
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


@functools.lru_cache(maxsize=64)
def hash_sum(n: int) -> int:
    """sum of audit_hash(i) = hash32(i ^ 0x5bd1e995) over i < n, mod 2^64."""
    total = 0
    for a in range(0, n, 1 << 24):
        i = np.arange(a, min(n, a + (1 << 24)), dtype=np.uint32)
        total += int(hash32(i ^ np.uint32(0x5BD1E995)).astype(np.uint64).sum())
    return total & MASK64


def _u64(lo, hi) -> int:
    return int(lo) | (int(hi) << 32)


def _inv(w) -> int:
    return int(np.uint32(~np.uint32(w)))


def check_run(hdr: dict, recs: np.ndarray) -> list:
    """Problems of one run's records (an empty list when the run was exact)."""
    bad = []
    nb = hdr["batches"]
    total, band = hdr["totalItems"], hdr["bandPixels"]
    step = max(hdr["step"], 0)
    if nb <= 0:
        return [f"run {hdr['run']}: no batches"]
    H_items, H_pix = hash_sum(total), hash_sum(band)
    prev_comb = -1
    for b in range(min(nb, len(recs) - 1)):
        r = recs[b]
        tag = f"run {hdr['run']} batch {b}/{nb}"
        f0 = hdr["firstFrame"] + b * step
        if r[0] != total or _u64(r[2], r[3]) != H_items:
            bad.append(f"{tag}: traced {r[0]} of {total} items (hash {'ok' if _u64(r[2], r[3]) == H_items else 'differs'})")
        if r[0]:
            fmax, fmin = int(r[6]) - 1, _inv(r[7])
            if fmin != f0 or fmax != f0:
                bad.append(f"{tag}: traced with first frames {fmin}..{fmax}, expected {f0}")
            emax, emin = int(r[8]) - 1, _inv(r[9])
            if emin != emax:
                bad.append(f"{tag}: traced by launches {emin}..{emax}")
            if emax >= hdr["launches"]:
                bad.append(f"{tag}: traced by launch {emax} of {hdr['launches']}")
        if r[1] != band or _u64(r[4], r[5]) != H_pix:
            bad.append(f"{tag}: combined {r[1]} of {band} pixels (hash {'ok' if _u64(r[4], r[5]) == H_pix else 'differs'})")
        if r[1]:
            cmax, cmin = int(r[10]) - 1, _inv(r[11])
            if cmin != cmax:
                bad.append(f"{tag}: combined by launches {cmin}..{cmax}")
            if r[0] and cmin <= int(r[8]) - 1:
                bad.append(f"{tag}: combined by launch {cmin}, not after the launch that traced it ({int(r[8]) - 1})")
            if cmin < prev_comb:
                bad.append(f"{tag}: combined by launch {cmin} before batch {b - 1} (launch {prev_comb})")
            prev_comb = max(prev_comb, cmax)
            gmax, gmin = int(r[12]) - 1, _inv(r[13])
            if gmin != f0 or gmax != f0:
                bad.append(f"{tag}: combined with first frames {gmin}..{gmax}, expected {f0}")
    extra = nb - (len(recs) - 1)
    if extra > 0:  # the pooled record of the batches past the records
        r = recs[-1]
        if r[0] != total * extra or r[1] != band * extra:
            bad.append(f"run {hdr['run']}: {extra} pooled batches traced {r[0]} / combined {r[1]}")
    elif recs[-1].any():
        bad.append(f"run {hdr['run']}: records past the run's batches")
    return bad


def check(runs: list) -> list:
    out = []
    for hdr, recs in runs:
        out += check_run(hdr, recs)
    return out


def synthetic_run(batches=5, total=64 * 7, band=64 * 7, first=3, step=1, launches=3, trace_epochs=None,
                  comb_epochs=None):
    """Records of an exact run (for the checker's own tests): batch b traced by trace_epochs[b] and
    combined by comb_epochs[b]."""
    trace_epochs = trace_epochs or [min(b, launches - 1) for b in range(batches)]
    comb_epochs = comb_epochs or [launches] * batches
    recs = np.zeros((min(batches, 256) + 1, 16), np.uint32)
    for b in range(min(batches, 256)):
        f0 = first + b * step
        hi, hp = hash_sum(total), hash_sum(band)
        recs[b] = [total, band, hi & 0xFFFFFFFF, hi >> 32, hp & 0xFFFFFFFF, hp >> 32, f0 + 1, ~np.uint32(f0),
                   trace_epochs[b] + 1, ~np.uint32(trace_epochs[b]), comb_epochs[b] + 1, ~np.uint32(comb_epochs[b]),
                   f0 + 1, ~np.uint32(f0), 0, 0]
    hdr = dict(run=1, device=0, firstFrame=first, step=step if batches > 1 else -1, frames=step or 1, bandPixels=band,
               totalItems=total, batches=batches, launches=launches, slots=8, overflow=0)
    return hdr, recs
