"""CLI / run.sh surface (no GPU compute): argument handling and dispatch."""
import os
import subprocess

import pytest

from conftest import ROOT
from mdcommunity_amd import cli


def test_dataset_spec_parsing():
    assert cli._dataset("fao_trade_multiplex:214:3,24") == ("fao_trade_multiplex", 214, (3, 24))


def test_out_of_scope_commands_exit_cleanly():
    assert cli.main(["unit", "train", "--output", "/tmp/x"]) == 2


def test_run_sh_dispatch_without_graphs():
    r = subprocess.run(["bash", os.path.join(ROOT, "run.sh"), "Unknown_dir", "testReal"], capture_output=True, text=True)
    assert r.returncode == 0 and "No training or testing" in r.stdout
    r = subprocess.run(["bash", os.path.join(ROOT, "run.sh")], capture_output=True, text=True)
    assert r.returncode == 2  # default = (unit, train): out of scope


@pytest.mark.gpu
def test_cli_testreal_writes_reference_files(tmp_path):
    golden = os.path.join(ROOT, "tests", "golden")
    real = tmp_path / "data" / "real"
    real.mkdir(parents=True)
    (real / "synth_multiplex.edges").write_text(open(os.path.join(golden, "synth_multiplex.edges")).read())
    out = tmp_path / "out"
    cli.main(["unit", "testReal", "--output", str(out), "--data-root", str(tmp_path / "data"),
              "--model", "./models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt",
              "--dataset", "synth_multiplex:60:1,3"])
    sub = out / "StepRatio_0.0000"
    for fn in ("Soluion_synth_multiplex_13.txt", "NormalizedLMCC_synth_multiplex_13.txt"):
        assert (sub / fn).read_text() == open(os.path.join(golden, "testreal_" + fn)).read()
    assert (sub / "time&audc_synth_multiplex.csv").exists()
