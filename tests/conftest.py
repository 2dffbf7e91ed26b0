"""Shared fixtures.  Markers: `gpu` = needs a gfx950 device (run on the MI355X box)."""
import os
import pathlib
import subprocess
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

ORACLE = REPO / "oracle" / "build" / "pafreport_oracle"
GA_ORACLE = REPO / "oracle" / "build" / "gapassem_oracle"
SYNTH = REPO / "synth" / "build" / "pwsynth"
CLI = REPO / "pwasm_amd" / "bin" / "pafreport"
GA_CLI = REPO / "pwasm_amd" / "bin" / "gapassem_consensus"
KAT_DIR = REPO / "tests" / "golden" / "kat"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def built():
    """Make sure the native artefacts exist (builds in-tree with make if needed)."""
    need = [ORACLE, GA_ORACLE, SYNTH, CLI, GA_CLI, REPO / "pwasm_amd" / "lib" / "libpwasm_amd.so"]
    if not all(p.exists() for p in need):
        subprocess.run(["make", "-j8"], cwd=str(REPO), check=True, stdout=subprocess.DEVNULL)
    return True


def run(cmd, cwd=None, timeout=600):
    p = subprocess.run([str(c) for c in cmd], cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=timeout)
    return p.returncode, p.stdout, p.stderr


def synth_paf(tmp, config, seed=None, scale=1.0, extra=()):
    fa, paf = os.path.join(tmp, f"c{config}.fa"), os.path.join(tmp, f"c{config}.paf")
    cmd = [SYNTH, "paf", "--config", config, "--scale", scale, "--fa", fa, "--paf", paf, *extra]
    if seed is not None:
        cmd += ["--seed", seed]
    rc, _, err = run(cmd)
    assert rc == 0, err
    return fa, paf
