"""The queues' item table (qt-raytracer_amd/csrc/item_order.cpp) on the host: a permutation of the
batch's 64-pixel run slots for any band size, frame count and queue count, handed out longest
estimate first within each queue.  (The GPU side, images equal to the oracle's with the order on
and off, is test_gpu_parity.py::test_item_order_does_not_change_results.)"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "qt-raytracer_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_item_table_is_a_sorted_permutation(tmp_path):
    exe = tmp_path / "item_order_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", f"-I{CSRC}", "-I/opt/rocm/include",
                    os.path.join(REPO, "tests", "native", "item_order_check.cpp"),
                    os.path.join(CSRC, "item_order.cpp"), os.path.join(CSRC, "bvh_builder.cpp"),
                    "-o", str(exe)], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_half_planes_round_outward(tmp_path):
    """bvh_builder.cpp half_bvh4 (HIPPT_OPT_BVH_QUANT 3): lo planes round down and hi planes up to
    the adjacent half (checked against all 63,488 finite halves, their float neighbours, 2M random
    floats and values beyond the half range), and the [lo hi] and [hi lo] rows, codes and padding
    sit where the kernel reads them."""
    exe = tmp_path / "half_check"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{CSRC}", os.path.join(REPO, "tests", "native", "half_check.cpp"),
                    os.path.join(CSRC, "bvh_builder.cpp"), "-o", str(exe)], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
