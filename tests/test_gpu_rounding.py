"""The kernels' short correctly-rounded sequences (hippt_trace.h sqrt_fix, rcp_nr, rsqrt_rn,
rsqrt_unit_draw) against hipcc's IEEE sqrtf and 1.0f/x on EVERY float bit pattern, on the GPU.

The kernels use them in place of the IEEE expansions (sky gradient RayTracer.h:593-595,
unit_vector of the Lambertian draw :477-484, Metal/Dielectric unit_vector :496-530); the oracle
keeps plain sqrtf / division.  Bit-exact parity of every rendered image rests on these counts
being zero inside each sequence's claimed domain, so the claim is checked exhaustively (2^32
inputs, ~1 s on an MI355X), not sampled.
"""
import ctypes
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "native", "librn_selftest.so")


def test_selftest_library_builds():
    assert os.path.exists(LIB), "build() / make -C tests/native builds it"


@pytest.mark.gpu
def test_fast_sqrt_rcp_exhaustive():
    lib = ctypes.CDLL(LIB)
    counts = (ctypes.c_ulonglong * 4)()
    assert lib.rn_selftest(counts) == 0
    names = ["rsqrt_rn (every x)", "rsqrt_unit_draw (+0, [2^-48, 1))", "sqrt_fix (x >= 2^-104)",
             "rcp_nr (2^-126 <= |x| < 2^126)"]
    assert list(counts) == [0, 0, 0, 0], dict(zip(names, list(counts)))
