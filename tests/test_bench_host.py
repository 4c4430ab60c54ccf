"""bench.py's host logic on CPU (no GPU): BASELINE presets and their workload labels, the CPU
baseline's thread rule and host facts, and that a missing reference harness is reported as
missing (value null + error) instead of silently timing another program."""
import importlib.util
import os
import sys
import types

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _args(bench, argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_default_is_configs1_strong(bench):
    a = _args(bench, [])
    assert (a.scene, a.width, a.height, a.spp, a.depth, a.path_mode) == ("cornell34", 1920, 1080, 64, 8,
                                                                          "megakernel")
    assert a.scaling == "strong" and bench.baseline_config_index(a) == 1


@pytest.mark.parametrize("preset,k,scene,w,h,spp,mode", [
    ("config2", 1, "cornell34", 1920, 1080, 64, "megakernel"),
    ("config3", 2, "blob70k", 1920, 1080, 64, "megakernel"),
    ("config4", 3, "blob70k", 3840, 2160, 256, "megakernel"),
    ("config5", 4, "blob70k", 1920, 1080, 64, "wavefront"),
])
def test_presets_name_their_baseline_config(bench, preset, k, scene, w, h, spp, mode):
    a = _args(bench, ["--preset", preset, "--width", "7"])  # a preset overrides the size flags
    assert (a.scene, a.width, a.height, a.spp, a.depth, a.path_mode) == (scene, w, h, spp, 8, mode)
    assert bench.baseline_config_index(a) == k
    a.spp = 32
    assert bench.baseline_config_index(a) is None


def test_cpu_thread_rule(bench):
    a = _args(bench, [])
    facts = {"nproc": 256, "affinity": 256, "omp_num_threads": 16, "model": "x"}
    assert bench.cpu_threads(a, facts)[0] == 16  # the GPU box: the CPU share, not the whole machine
    facts = {"nproc": 8, "affinity": 8, "omp_num_threads": None, "model": "x"}
    assert bench.cpu_threads(a, facts) == (8, "affinity mask")
    a.cpu_threads = 3
    assert bench.cpu_threads(a, facts) == (3, "--cpu-threads")
    f = bench.host_cpu_facts()
    assert f["nproc"] >= 1 and f["affinity"] >= 1


def test_missing_reference_harness_is_reported_not_substituted(bench, monkeypatch, tmp_path):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    monkeypatch.setattr(pyoracle, "REF_HARNESS", str(tmp_path / "no_such_harness"))
    a = _args(bench, [])
    cb = bench.cpu_baseline(a, types.SimpleNamespace(name="cornell34"))
    assert cb["value"] is None and cb["kind"] == "reference" and "missing" in cb["error"]


def test_reference_harness_parts_cover_the_sample(tmp_path):
    """cpu_baseline's independent_processes: `ref_harness bench ... 1 PART PARTS` renders the sample
    lines k with k % PARTS == PART, so the parts' lines and pixel samples add up to the whole sample."""
    import json
    import subprocess
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    from hippt import scenes
    if not os.path.exists(pyoracle.REF_HARNESS):
        pytest.skip("oracle/_ref/ref_harness not built (needs /root/reference)")
    path = str(tmp_path / "c.scene")
    scenes.write_scene_file(scenes.get_scene("cornell34"), path)

    def run(*extra):
        out = subprocess.run([pyoracle.REF_HARNESS, "bench", path, "64", "37", "3", "1", "2", "1", *extra],
                             capture_output=True, text=True, check=True, timeout=120).stdout
        return json.loads(out.strip().splitlines()[-1])
    whole = run()
    parts = [run(str(k), "3") for k in range(3)]
    assert whole["rows"] == 13 and [p["rows"] for p in parts] == [5, 4, 4]
    assert sum(p["pixel_samples"] for p in parts) == whole["pixel_samples"]


def test_pmc_summary_used_only_for_the_same_run(bench):
    """roofline.traffic comes from a PMC summary only when it describes this
    run — the same image CRC traced by the same libhippt.so (its SHA-256) — and carries bytes per
    step, which the line divides by this run's own kernel time (a profile from a slower box no longer
    distorts the rate); otherwise null, with the reason in roofline.pmc_refused."""
    good = {"source": "profiles/x_pmc.json", "image_crc32": 2540294198, "lib_sha256": "ab" * 32,
            "hbm_bytes_per_step": 123}
    pmc, why = bench.check_pmc(dict(good), 2540294198, "ab" * 32, 1)
    assert pmc and why is None
    pmc, why = bench.check_pmc(dict(good, image_crc32=None), 2540294198, "ab" * 32, 1)
    assert pmc is None and "image_crc32" in why
    pmc, why = bench.check_pmc(dict(good), 1209999578, "ab" * 32, 1)
    assert pmc is None and "CRC" in why
    pmc, why = bench.check_pmc(dict(good), 2540294198, "cd" * 32, 1)
    assert pmc is None and "libhippt.so" in why
    pmc, why = bench.check_pmc(dict(good, hbm_bytes_per_step=None), 2540294198, "ab" * 32, 1)
    assert pmc is None and "per-step" in why
    pmc, why = bench.check_pmc(dict(good), 2540294198, "ab" * 32, 8)
    assert pmc is None and why
    assert bench.check_pmc(None, 1, "x", 1) == (None, None)


def test_pmc_candidates_first_consistent_wins(bench):
    """load_pmc returns every summary of the workload; the first consistent one is used, an older
    summary without a CRC does not hide a newer valid one."""
    old = {"source": "profiles/round3/x_pmc.json", "image_crc32": None}
    new = {"source": "profiles/round5/y_pmc.json", "image_crc32": 1209999578, "lib_sha256": "ef" * 32,
           "hbm_bytes_per_step": 7}
    pmc, why = bench.check_pmc([old, new], 1209999578, "ef" * 32, 1)
    assert pmc is new and why is None
    pmc, why = bench.check_pmc([old], 1209999578, "ef" * 32, 1)
    assert pmc is None and "image_crc32" in why
    assert bench.check_pmc([], 1, "x", 1) == (None, None)


def test_gpus_without_launcher_starts_ranks_or_fails(bench):
    """`bench.py --gpus N` never falls back silently to one GPU.  Without a launcher
    (no WORLD_SIZE) N > 1 becomes a torch.distributed.run child with N ranks on 127.0.0.1 and the
    same arguments; under a launcher WORLD_SIZE must equal --gpus, else a non-zero exit."""
    assert bench.launcher_command(["--steps", "3"], 1, {}) is None
    cmd = bench.launcher_command(["--gpus", "8", "--steps", "3"], 8, {})
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == [os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "3"][-4:]
    assert cmd[-5].endswith("bench.py")
    assert bench.launcher_command(["--gpus", "4"], 4, {"WORLD_SIZE": "4"}) is None
    assert bench.launcher_command([], 1, {"WORLD_SIZE": "1"}) is None
    with pytest.raises(SystemExit) as e:
        bench.launcher_command(["--gpus", "8"], 8, {"WORLD_SIZE": "2"})
    assert e.value.code != 0
    with pytest.raises(SystemExit):
        bench.launcher_command([], 1, {"WORLD_SIZE": "4"})
