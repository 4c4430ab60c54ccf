"""The chained-batch protocol (hippt_trace.h "chained batches", hippt_api.cpp chain_batch)
as a host-compiled model: tests/native/chain_model.cpp drives the product's own integer rules
(qt-raytracer_amd/csrc/hippt_chain_logic.h, the header the gfx950 kernels include) through seeded
adversarial interleavings of host calls and device micro-steps, and checks the reference's contract
for every batch of every run: each work unit traced exactly once with its batch's frames, each batch
combined exactly once, in order, after it is fully traced, from an intact ring slot
(CudaPathTracerKernel.cu:157-178: one sample per frame, blended in frame order).

The round-5 rules are restated in the model (`legacy`): the model reproduces the recorded GPU failure
(GPUTEST_r05: a batch's items traced with another batch's frames), and the fixed rules never fail.
Mutants of the fixed rules (a ring under 2 x cap slots, a launch counting its own waves' batches as
finished) must be caught, so that a green run means the checks can see a broken protocol.  No GPU.
"""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "native", "chain_model.cpp")
HDR = os.path.join(REPO, "qt-raytracer_amd", "csrc")


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("chain_model") / "chain_model")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-I" + HDR, "-o", exe, SRC], check=True)
    return exe


def run(model, *args):
    out = subprocess.run([model, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    line = out.stdout.splitlines()[0]
    counts = dict((k, int(v)) for k, v in re.findall(r"(\S+?)[= ](\d+)", line.split(" ", 2)[2]))
    return counts, out.stdout


def test_directed_r05_interleaving(model):
    """The interleaving VERDICT r5 names, on one block's view: the view refreshed while the run is open
    (batches up to 3 posted, consecutive frames), then refreshed once the host is on a later run, then
    a wave asks for batch 2 <= last.  Round 5's merge traced it with batch 0's frames; the fixed merge
    keeps the frame pattern."""
    out = subprocess.run([model, "directed"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "legacy: last 3 flags 2 took 1 step 0 -> batch 2 traced with batch 0's frames" in out.stdout
    assert "fixed: last 3 flags 7 took 1 step 1 -> frames of batch 2 right" in out.stdout


@pytest.mark.parametrize("seed", [1079, 16413, 18729])
def test_model_reproduces_the_recorded_failure(model, seed):
    """Seeded schedules in which round 5's rules trace a batch's remaining items with the wrong frames
    (a wave hands out its claimed chunk over several refills; the run closes meanwhile and the closed
    view's flags drop the frame pattern; camera_sample then uses step 0 for the whole refill) — the
    fixed rules on the same schedules are exact."""
    legacy, text = run(model, "legacy", 1, seed)
    assert legacy.get("frame", 0) >= 1, text
    fixed, text = run(model, "fixed", 1, seed)
    assert fixed["violations"] == 0, text


def test_fixed_rules_hold_over_many_schedules(model):
    counts, text = run(model, "fixed", 6000, 1)
    assert counts["violations"] == 0, text
    # the schedules reach the hard cases: runs closing under running launches, waves answered from a
    # closed view, and batches taken after it
    assert counts["closed_merges"] > 1000 and counts["closed_answers"] > 1000 and counts["closed_takes"] > 0, text
    assert counts["launches"] > 50000 and counts["batches"] > 100000, text


@pytest.mark.parametrize("mutant,kind", [("small-ring", "slot"), ("own-markers", "untraced")])
def test_model_catches_broken_rules(model, mutant, kind):
    counts, text = run(model, mutant, 500, 1)
    assert counts.get(kind, 0) > 0, text
