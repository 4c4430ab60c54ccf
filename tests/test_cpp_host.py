"""The C++ host over the C ABI: qt-raytracer_amd/host/HipPathTracer (the CudaPathTracer interface,
src/backends/CudaPathTracer.h:6-23) driven by the hippt_render CLI, as a Qt application would.

GPU tests run the binary as a child process and compare its ARGB output with the oracle.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import pyoracle as po
from hippt import scenes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "qt-raytracer_amd", "hippt_render")


def _run(*args):
    r = subprocess.run([BIN, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_cli_built_and_usage():
    assert os.access(BIN, os.X_OK)
    r = subprocess.run([BIN, "--no-such-flag"], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
def test_cpp_host_legacy_scene_matches_oracle(tmp_path):
    out = tmp_path / "legacy.argb"
    info = _run("--width", 96, "--height", 54, "--spp", 5, "--depth", 8, "--out", out)
    assert info["frames"] == 5
    px = np.fromfile(out, np.uint32).reshape(54, 96)
    ora_px, _ = po.sphere4(96, 54, 0, 5, 8)
    assert np.array_equal(px, ora_px)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [[], ["--per-frame"], ["--present"]])
def test_cpp_host_mesh_file_matches_oracle(tmp_path, mode):
    sc = scenes.cornell34()
    obj = tmp_path / "cornell.obj"
    scenes.write_obj(sc, str(obj), style="quads")
    out = tmp_path / "mesh.argb"
    albedo = ";".join(",".join(f"{c:.9g}" for c in a) for a in sc.albedo)
    info = _run("--mesh", obj, "--albedo", albedo, "--width", 80, "--height", 48, "--spp", 8, "--depth", 8,
                "--out", out, *mode)
    px = np.fromfile(out, np.uint32).reshape(48, 80)
    ora_px, _, segs, samples = po.MeshScene(sc, 80, 48).frames(0, 8, 8)
    assert np.array_equal(px, ora_px)
    assert info["frames"] == 8 and info["pixel_samples"] == samples and info["segments"] == segs


@pytest.mark.gpu
@pytest.mark.parametrize("backend,extra", [("vulkan", []), ("gl", []), ("gl", ["--per-frame"])])
@pytest.mark.parametrize("depth,clamped", [(8, 8), (100, 64), (0, 1)])
def test_cpp_host_vulkan_and_gl_interfaces_match_oracle(tmp_path, backend, extra, depth, clamped):
    """HipVulkanPathTracer (VulkanPathTracer's interface) and HipGpuPathTracer (GpuPathTracer's)
    on the reference kernels' 4-sphere scene: RGBA8 UNORM words equal to the oracle's accumulation
    quantized as the GL / Vulkan image stores it, the bounce count clamped to 1..64 as those
    backends do (GpuPathTracer.cpp:57, VulkanPathTracer.cpp:95), one frame index per sample."""
    out = tmp_path / "frame.rgba"
    info = _run("--backend", backend, "--width", 64, "--height", 40, "--spp", 5, "--depth", depth, "--out", out,
                *extra)
    assert info["backend"] == backend and info["frames"] == 5
    assert info["pixel_format_after"] == 0  # HIPPT_PIXEL_ARGB restored for other callers
    px = np.fromfile(out, np.uint32).reshape(40, 64)
    _, acc = po.sphere4(64, 40, 0, 5, clamped)
    assert np.array_equal(px, po.rgba8(acc))


@pytest.mark.gpu
def test_cpp_host_gl_interface_mesh_scene(tmp_path):
    sc = scenes.cornell34()
    obj = tmp_path / "cornell.obj"
    scenes.write_obj(sc, str(obj), style="quads")
    out = tmp_path / "mesh.rgba"
    albedo = ";".join(",".join(f"{c:.9g}" for c in a) for a in sc.albedo)
    info = _run("--backend", "gl", "--mesh", obj, "--albedo", albedo, "--width", 48, "--height", 32, "--spp", 4,
                "--depth", 8, "--out", out)
    px = np.fromfile(out, np.uint32).reshape(32, 48)
    _, acc, segs, samples = po.MeshScene(sc, 48, 32).frames(0, 4, 8)
    assert np.array_equal(px, po.rgba8(acc))
    assert info["pixel_samples"] == samples and info["segments"] == segs
